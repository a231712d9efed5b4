// K25 group_reduce: per-group sum / min / max of one column (SQL groupBy().agg(), the per-hospital
// count / avg / max / stddev of ref.py:150-160 and the streaming window counts of ref.py:84-92).
//
// Few groups (hospitals, wards, time buckets) is the hard case for scatter atomics: millions of
// rows hit a few hundred addresses and global f64 atomics serialise in L2 (torch index_add_ took
// ~217 ms for 10M rows into 500 groups, profiles/r2/groupby_kernels.txt). Here every wave owns a
// private copy of the G accumulators in LDS (4 waves x G x 8 B, G <= 2048), so conflicts stay
// inside one wave's LDS instruction. A workgroup reduces a fixed, contiguous row range; at the end
// its four wave copies are combined in wave order and written as one partial row; a second kernel
// reduces the partial rows of each group with a fixed strided assignment + LDS tree. The block
// ranges, the wave copies and both combination trees are fixed by (n, G), so the result does not
// depend on scheduling (the lanes of one LDS atomic instruction are applied in hardware order).
//
// Values: f64 / f32 / i32 / i64 / u8 columns or the row index itself (first / last positions);
// an optional u8 mask skips rows (nulls, NaN). Sums accumulate in f64 (floating) or i64 (integral),
// min / max in the same wide types.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

enum { kSum = 0, kMin = 1, kMax = 2 };
enum { kF64 = 0, kF32 = 1, kI32 = 2, kI64 = 3, kU8 = 4, kRowIndex = 5 };

template <typename T, int OP>
__device__ __forceinline__ void lds_apply(T* p, T v) {
  if constexpr (OP == kSum) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else if constexpr (OP == kMin) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

template <typename T, int OP>
__device__ __forceinline__ T combine(T a, T b) {
  if constexpr (OP == kSum) return a + b;
  else if constexpr (OP == kMin) return b < a ? b : a;
  else return b > a ? b : a;
}

template <typename T, int VT>
__device__ __forceinline__ T load_val(const void* vals, long long r) {  // VT != kRowIndex
  if constexpr (VT == kF64) return (T)static_cast<const double*>(vals)[r];
  else if constexpr (VT == kF32) return (T)static_cast<const float*>(vals)[r];
  else if constexpr (VT == kI32) return (T)static_cast<const int*>(vals)[r];
  else if constexpr (VT == kI64) return (T)static_cast<const long long*>(vals)[r];
  else if constexpr (VT == kU8) return (T)static_cast<const unsigned char*>(vals)[r];
  else return (T)r;
}

// Elements e in [0, n * d): row e / d, column e % d, accumulator slot gid[row] * d + column (d > 1:
// the per-group column sums of a row-major [n, d] matrix, read coalesced). G counts slots (groups * d).
template <typename T, int VT, int OP, bool MULTI>
__global__ __launch_bounds__(kThreads) void group_reduce_kernel(const int* __restrict__ gid, const void* __restrict__ vals,
                                                                const unsigned char* __restrict__ mask, long long n, int d,
                                                                int G, long long rows_per_block, T ident,
                                                                T* __restrict__ partial) {
  extern __shared__ __align__(16) unsigned char smem[];
  T* acc = reinterpret_cast<T*>(smem);  // [kWaves][G]
  for (int i = threadIdx.x; i < kWaves * G; i += kThreads) acc[i] = ident;
  __syncthreads();
  T* mine = acc + (size_t)(threadIdx.x >> 6) * G;
  const long long ne = MULTI ? n * d : n;
  const long long start = (long long)blockIdx.x * rows_per_block;
  const long long end = start + rows_per_block < ne ? start + rows_per_block : ne;
  for (long long e = start + threadIdx.x; e < end; e += kThreads) {
    const long long r = MULTI ? e / d : e;
    if (mask != nullptr && mask[r] == 0) continue;
    const int slot = MULTI ? gid[r] * d + (int)(e - r * d) : gid[r];
    T v;
    if constexpr (VT == kRowIndex) v = (T)r;
    else v = load_val<T, VT>(vals, e);
    lds_apply<T, OP>(mine + slot, v);
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += kThreads) {
    T a = acc[g];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) a = combine<T, OP>(a, acc[w * G + g]);
    partial[(size_t)blockIdx.x * G + g] = a;
  }
}

// One workgroup per group: thread t folds partial rows t, t+256, ... (fixed), then an LDS tree.
template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void group_reduce_final_kernel(const T* __restrict__ partial, long long nb, int G,
                                                                      T ident, T* __restrict__ out) {
  __shared__ T sh[kThreads];
  const int g = blockIdx.x;
  T a = ident;
  for (long long b = threadIdx.x; b < nb; b += kThreads) a = combine<T, OP>(a, partial[(size_t)b * G + g]);
  sh[threadIdx.x] = a;
  __syncthreads();
#pragma unroll
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] = combine<T, OP>(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[g] = sh[0];
}

template <typename T, int VT, int OP>
int launch(const int* gid, const void* vals, const unsigned char* mask, long long n, int d, int G, long long rpb,
           long long nb, T ident, T* scratch, T* out, hipStream_t st) {
  const size_t lds = (size_t)kWaves * G * sizeof(T);
  if (d > 1)
    hipLaunchKernelGGL((group_reduce_kernel<T, VT, OP, true>), dim3((unsigned)nb), dim3(kThreads), lds, st, gid, vals,
                       mask, n, d, G, rpb, ident, scratch);
  else
    hipLaunchKernelGGL((group_reduce_kernel<T, VT, OP, false>), dim3((unsigned)nb), dim3(kThreads), lds, st, gid, vals,
                       mask, n, 1, G, rpb, ident, scratch);
  hipLaunchKernelGGL((group_reduce_final_kernel<T, OP>), dim3((unsigned)G), dim3(kThreads), 0, st, scratch, nb, G,
                     ident, out);
  return cml_status();
}

template <typename T, int OP>
int by_type(int vtype, const int* gid, const void* vals, const unsigned char* mask, long long n, int d, int G,
            long long rpb, long long nb, T ident, T* scratch, T* out, hipStream_t st) {
  switch (vtype) {
    case kF64: return launch<T, kF64, OP>(gid, vals, mask, n, d, G, rpb, nb, ident, scratch, out, st);
    case kF32: return launch<T, kF32, OP>(gid, vals, mask, n, d, G, rpb, nb, ident, scratch, out, st);
    case kI32: return launch<T, kI32, OP>(gid, vals, mask, n, d, G, rpb, nb, ident, scratch, out, st);
    case kI64: return launch<T, kI64, OP>(gid, vals, mask, n, d, G, rpb, nb, ident, scratch, out, st);
    case kU8: return launch<T, kU8, OP>(gid, vals, mask, n, d, G, rpb, nb, ident, scratch, out, st);
    case kRowIndex: return launch<T, kRowIndex, OP>(gid, vals, mask, n, d, G, rpb, nb, ident, scratch, out, st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// Largest group count the LDS-privatised path takes (4 wave copies of G 8-byte accumulators).
CML_API int cml_group_reduce_max_groups() { return 2048; }

// out[g * d + j] = op over rows r with gid[r] == g (and mask[r] != 0) of vals[r * d + j]; acc: 0 = f64,
// 1 = i64. G counts accumulator slots (groups * d); scratch holds nb * G of them; every block covers
// rows_per_block elements and rows_per_block * nb >= n * d.
CML_API int cml_group_reduce(const int* gid, const void* vals, int vtype, const unsigned char* mask, long long n, int d,
                             int G, int op, int acc, long long rows_per_block, long long nb, void* scratch, void* out,
                             void* stream) {
  if (G <= 0 || G > 2048 || d <= 0 || G % d != 0 || nb <= 0 || rows_per_block * nb < n * d)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (acc == 0) {
    double* s = (double*)scratch;
    double* o = (double*)out;
    switch (op) {
      case kSum: return by_type<double, kSum>(vtype, gid, vals, mask, n, d, G, rows_per_block, nb, 0.0, s, o, st);
      case kMin: return by_type<double, kMin>(vtype, gid, vals, mask, n, d, G, rows_per_block, nb, __builtin_inf(), s, o, st);
      case kMax: return by_type<double, kMax>(vtype, gid, vals, mask, n, d, G, rows_per_block, nb, -__builtin_inf(), s, o, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  long long* s = (long long*)scratch;
  long long* o = (long long*)out;
  switch (op) {
    case kSum: return by_type<long long, kSum>(vtype, gid, vals, mask, n, d, G, rows_per_block, nb, 0LL, s, o, st);
    case kMin: return by_type<long long, kMin>(vtype, gid, vals, mask, n, d, G, rows_per_block, nb, (long long)0x7FFFFFFFFFFFFFFFLL, s, o, st);
    case kMax: return by_type<long long, kMax>(vtype, gid, vals, mask, n, d, G, rows_per_block, nb, (long long)(-0x7FFFFFFFFFFFFFFFLL - 1), s, o, st);
    default: return (int)hipErrorInvalidValue;
  }
}
