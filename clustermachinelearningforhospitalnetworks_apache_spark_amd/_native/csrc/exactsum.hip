// Partition-invariant sums (gfx950): the same bits for any split of the rows over ranks.
//
// An f64 all-reduce of per-rank partial sums rounds once per rank, so a fit's scalars (the k-means||
// sampling rate 2k / Σcost, the per-cluster Σ||x||² of the training cost) came out a few ulps apart at
// different rank counts — the strong-scaling curve must fit ONE problem at every N.
// These sums accumulate INTEGERS, which add exactly in any order, and round to f64 once, after the
// int64 all-reduce, in a fixed order:
//
//   every value v (>= 0) is put on the grid 2^g, g = e(bound) - 46, where `bound` is an upper bound of
//   every value on EVERY rank (a device scalar the ranks agree on: e.g. the all-reduced max ||x||²), so
//   q = rint(v / 2^g) < 2^46 — one rounding per value at 2^-47 of the bound (far below what an f64 sum of
//   the values keeps), the same on any rank; q is summed as int64 (per thread in registers for one sum, per
//   label with ONE integer LDS atomic per value — a block sums at most 2^16 values, so its label sums stay below
//   2^62), and each block's sums go to the global accumulators as two 31-bit limbs (integer atomics);
//   fixsum_finalize recombines the (all-reduced) limbs in double-double and scales by 2^g.
#include "common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

// dd (h, l) += v (v exact in f64)
__device__ __forceinline__ void dd_add(double& h, double& l, double v) {
  double s, e;
  two_sum(h, v, s, e);
  l += e;
  two_sum(s, l, h, l);
}

constexpr int kQBits = 46;             // q < 2^46
constexpr long long kBlockValues = 1 << 16;  // at most this many values per block (grid sizing): sums < 2^62

// grid exponent: every value v <= bound·mul·(1 + 2^-10) lies below 2^(g + kQBits)
__device__ __forceinline__ int fix_grid(float bound, float mul) {
  const double m = (double)bound * (double)mul * (1.0 + 1.0 / 1024.0);
  if (!(m > 0.0)) return 0;
  return ilogb(m) + 1 - kQBits;
}

// q = rint(v·2^-g) by a power-of-two multiply (exact) and one rounding conversion; v <= 0 and NaN -> 0
__device__ __forceinline__ long long fix_q(double v, double scale) {
  const double t = v * scale;
  if (!(t > 0.0)) return 0;
  const long long q = __double2ll_rn(t);
  return q > (1LL << kQBits) ? (1LL << kQBits) : q;
}

__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// a block sum s (0 <= s < 2^62) into the two global 31-bit limbs
__device__ __forceinline__ void add_limbs(long long* lo, long long* hi, long long s) {
  if (s == 0) return;
  atomicAdd(reinterpret_cast<unsigned long long*>(lo), (unsigned long long)(s & 0x7fffffffLL));
  atomicAdd(reinterpret_cast<unsigned long long*>(hi), (unsigned long long)(s >> 31));
}

template <typename T, bool VEC4>
__global__ __launch_bounds__(kThreads) void fixsum_kernel(const T* __restrict__ v, long long n,
                                                         const float* __restrict__ bound, float mul,
                                                         long long* __restrict__ limbs) {
  const double scale = ldexp(1.0, -fix_grid(bound[0], mul));
  long long acc = 0;  // < 2^46 per value, at most 4096 values per thread: < 2^58
  const long long stride = (long long)gridDim.x * kThreads;
  long long i = (long long)blockIdx.x * kThreads + threadIdx.x;
  if constexpr (VEC4) {  // 16-byte loads of four f32 values (16-byte aligned vectors)
    const long long n4 = n / 4;
    const float4* v4 = reinterpret_cast<const float4*>(v);
    for (long long j = i; j < n4; j += stride) {
      const float4 w = v4[j];
      acc += fix_q((double)w.x, scale) + fix_q((double)w.y, scale) + fix_q((double)w.z, scale) +
             fix_q((double)w.w, scale);
    }
    if (blockIdx.x == 0 && threadIdx.x < (unsigned)(n - 4 * n4)) acc += fix_q((double)v[4 * n4 + threadIdx.x], scale);
  } else {
    for (long long j = i; j < n; j += stride) acc += fix_q((double)v[j], scale);
  }
  // one atomic pair per BLOCK (the wave-level pairs of a 4096-block grid serialised on the two addresses:
  // 0.42 ms at 100M values instead of the ~0.07 ms the read takes)
  __shared__ long long red[2][kThreads / 64];
  const long long lo = wave_sum_i64(acc & 0x7fffffffLL), hi = wave_sum_i64(acc >> 31);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = lo;
    red[1][threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long L = 0, H = 0;
    for (int w = 0; w < kThreads / 64; ++w) {
      L += red[0][w];
      H += red[1][w];
    }
    if (L) atomicAdd(reinterpret_cast<unsigned long long*>(&limbs[0]), (unsigned long long)L);
    if (H) atomicAdd(reinterpret_cast<unsigned long long*>(&limbs[1]), (unsigned long long)H);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fixsum_label_kernel(const int* __restrict__ lab, const T* __restrict__ v,
                                                               long long n, int k, const float* __restrict__ bound,
                                                               float mul, long long* __restrict__ limbs) {
  extern __shared__ long long acc[];  // [k] label sums of this block (< 2^62: at most kBlockValues values)
  for (int i = threadIdx.x; i < k; i += kThreads) acc[i] = 0;
  __syncthreads();
  const double scale = ldexp(1.0, -fix_grid(bound[0], mul));
  const long long per = (n + gridDim.x - 1) / gridDim.x;  // a contiguous range per block
  const long long b0 = (long long)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  for (long long i = b0 + threadIdx.x; i < b1; i += kThreads) {
    const long long q = fix_q((double)v[i], scale);
    if (q != 0) atomicAdd(reinterpret_cast<unsigned long long*>(&acc[lab[i]]), (unsigned long long)q);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += kThreads) add_limbs(&limbs[i], &limbs[k + i], acc[i]);
}

__global__ __launch_bounds__(kThreads) void fixsum_finalize_kernel(const long long* __restrict__ limbs, int k,
                                                                  const float* __restrict__ bound, float mul,
                                                                  double* __restrict__ out) {
  const int g = fix_grid(bound[0], mul);
  for (int j = blockIdx.x * kThreads + threadIdx.x; j < k; j += gridDim.x * kThreads) {
    const long long lo = limbs[j], hi = limbs[k + j];  // total = hi·2^31 + lo, both in [0, 2^63)
    double h = 0.0, l = 0.0;
    dd_add(h, l, ldexp((double)(hi >> 32), 63));
    dd_add(h, l, ldexp((double)(hi & 0xffffffffLL), 31));
    dd_add(h, l, ldexp((double)(lo >> 32), 32));
    dd_add(h, l, (double)(lo & 0xffffffffLL));
    out[j] = ldexp(h + l, g);
  }
}

inline unsigned grid_for(long long n, long long per, unsigned cap) {
  long long g = (n + per - 1) / per;
  g = g < 1 ? 1 : g;
  return (unsigned)(g > cap ? cap : g);
}

}  // namespace

// limbs: int64 [2k] (k = 1 without labels: [lo, hi]), accumulated into — zeroed by the caller once per sum;
// values v >= 0, f32 (dtype 1) or f64 (dtype 2), v <= bound[0]·mul on every rank (bound: device f32).
// lab (may be null: one sum): int32 in [0, k).
CML_API int cml_fixsum(const void* v, int dtype, const int* lab, long long n, int k, const float* bound, float mul,
                       long long* limbs, void* stream) {
  if (n <= 0) return 0;
  if (k <= 0 || k > 4096 || (lab == nullptr && k != 1) || (dtype != 1 && dtype != 2)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (lab == nullptr) {
    // at most 4096 values per thread (sums < 2^58), ~16 per thread and at most 1024 blocks where the grid allows
    long long g = (n + kThreads * 16LL - 1) / (kThreads * 16LL);
    const long long gmin = (n + kThreads * 4096LL - 1) / (kThreads * 4096LL);
    g = g > 1024 ? 1024 : g;
    g = g < gmin ? gmin : g;
    if (g > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    if (dtype == 1 && (reinterpret_cast<size_t>(v) & 15) == 0)
      hipLaunchKernelGGL((fixsum_kernel<float, true>), dim3((unsigned)g), dim3(kThreads), 0, st, (const float*)v, n,
                         bound, mul, limbs);
    else if (dtype == 1)
      hipLaunchKernelGGL((fixsum_kernel<float, false>), dim3((unsigned)g), dim3(kThreads), 0, st, (const float*)v, n,
                         bound, mul, limbs);
    else
      hipLaunchKernelGGL((fixsum_kernel<double, false>), dim3((unsigned)g), dim3(kThreads), 0, st, (const double*)v, n,
                         bound, mul, limbs);
    return cml_status();
  }
  // at most kBlockValues values per block (its label sums < 2^62), and ~1024 blocks where there are rows for them
  long long g = (n + kBlockValues - 1) / kBlockValues;
  const long long want = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  if (g < want) g = want;
  if (g > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)k * sizeof(long long);
  if (dtype == 1)
    hipLaunchKernelGGL(fixsum_label_kernel<float>, dim3((unsigned)g), dim3(kThreads), lds, st, lab, (const float*)v, n, k,
                       bound, mul, limbs);
  else
    hipLaunchKernelGGL(fixsum_label_kernel<double>, dim3((unsigned)g), dim3(kThreads), lds, st, lab, (const double*)v, n,
                       k, bound, mul, limbs);
  return cml_status();
}

// out: f64 [k] = the (all-reduced) limbs' sums on the grid of bound·mul.
CML_API int cml_fixsum_finalize(const long long* limbs, int k, const float* bound, float mul, double* out,
                                void* stream) {
  if (k <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(fixsum_finalize_kernel, dim3(grid_for(k, kThreads, 64)), dim3(kThreads), 0,
                     (hipStream_t)stream, limbs, k, bound, mul, out);
  return cml_status();
}
