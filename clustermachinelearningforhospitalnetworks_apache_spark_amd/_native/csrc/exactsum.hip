// Partition-invariant sums (gfx950): the same bits for any split of the rows over ranks.
//
// An f64 all-reduce of per-rank partial sums rounds once per rank, so a fit's scalars (the k-means||
// sampling rate 2k / Σcost, the per-cluster Σ||x||² of the training cost) came out a few ulps apart at
// different rank counts — the strong-scaling curve must fit ONE problem at every N.
// These sums accumulate INTEGERS, which add exactly in any order, and round to f64 once, after the
// int64 all-reduce, in a fixed order:
//
//   every value v (>= 0) is put on the grid 2^g, g = e(bound) - 62, where `bound` is an upper bound of
//   every value on EVERY rank (a device scalar the ranks agree on: e.g. the all-reduced max ||x||²), so
//   q = rint(v / 2^g) < 2^62 — one rounding per value at 2^-62 of the bound, the same on any rank;
//   q is split into two 31-bit limbs, summed as int64 (per thread in registers for one sum, per label in
//   LDS with integer atomics, then one global atomic per block and limb); fixsum_finalize recombines the
//   (all-reduced) limbs in double-double and scales by 2^g.
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

// grid exponent: every value v <= bound·mul·(1 + 2^-10) lies below 2^(g + 62)
__device__ __forceinline__ int fix_grid(float bound, float mul) {
  const double m = (double)bound * (double)mul * (1.0 + 1.0 / 1024.0);
  if (!(m > 0.0)) return 0;
  return ilogb(m) + 1 - 62;
}

__device__ __forceinline__ long long fix_q(double v, int g) {
  if (!(v > 0.0)) return 0;  // (negative and NaN values are outside the contract: counted as 0)
  long long q = (long long)rint(ldexp(v, -g));
  return q > (1LL << 62) ? (1LL << 62) : q;
}

__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fixsum_kernel(const T* __restrict__ v, long long n,
                                                         const float* __restrict__ bound, float mul,
                                                         long long* __restrict__ limbs) {
  const int g = fix_grid(bound[0], mul);
  long long lo = 0, hi = 0;  // per thread: at most ~n / (grid·256) values of < 2^31 each
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const long long q = fix_q((double)v[i], g);
    lo += q & 0x7fffffffLL;
    hi += q >> 31;
  }
  lo = wave_sum_i64(lo);
  hi = wave_sum_i64(hi);
  if ((threadIdx.x & 63) == 0) {
    if (lo) atomicAdd(reinterpret_cast<unsigned long long*>(&limbs[0]), (unsigned long long)lo);
    if (hi) atomicAdd(reinterpret_cast<unsigned long long*>(&limbs[1]), (unsigned long long)hi);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fixsum_label_kernel(const int* __restrict__ lab, const T* __restrict__ v,
                                                               long long n, int k, const float* __restrict__ bound,
                                                               float mul, long long* __restrict__ limbs) {
  extern __shared__ long long acc[];  // [2k]: lo limbs, then hi limbs
  for (int i = threadIdx.x; i < 2 * k; i += kThreads) acc[i] = 0;
  __syncthreads();
  const int g = fix_grid(bound[0], mul);
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const long long q = fix_q((double)v[i], g);
    if (q == 0) continue;
    const int j = lab[i];
    atomicAdd(reinterpret_cast<unsigned long long*>(&acc[j]), (unsigned long long)(q & 0x7fffffffLL));
    atomicAdd(reinterpret_cast<unsigned long long*>(&acc[k + j]), (unsigned long long)(q >> 31));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * k; i += kThreads)
    if (acc[i] != 0) atomicAdd(reinterpret_cast<unsigned long long*>(&limbs[i]), (unsigned long long)acc[i]);
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
  if (k <= 0 || k > 4096 || (lab == nullptr && k != 1) || (dtype != 1 && dtype != 2))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(grid_for(n, kThreads * 16LL, 2048)), block(kThreads);
  if (lab == nullptr) {
    if (dtype == 1)
      hipLaunchKernelGGL(fixsum_kernel<float>, grid, block, 0, st, (const float*)v, n, bound, mul, limbs);
    else
      hipLaunchKernelGGL(fixsum_kernel<double>, grid, block, 0, st, (const double*)v, n, bound, mul, limbs);
    return cml_status();
  }
  const size_t lds = (size_t)2 * k * sizeof(long long);
  if (dtype == 1)
    hipLaunchKernelGGL(fixsum_label_kernel<float>, grid, block, lds, st, lab, (const float*)v, n, k, bound, mul,
                       limbs);
  else
    hipLaunchKernelGGL(fixsum_label_kernel<double>, grid, block, lds, st, lab, (const double*)v, n, k, bound, mul,
                       limbs);
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
