// The pruned k-means‖ pass's candidate table in one launch (models/kmeans.py
// _init_candidate_pass_pruned; the k-means‖ rounds of ref.py:147's KMeans.fit): for every existing
// candidate p (row i of P) the distances to the new candidates Y, rounded down to f32 and sorted ascending
// with their indices, and ||p||² rounded up. The pass's classify / near-list kernels read it: a row at
// distance r from p can only move to a y with |p - y| < 2r (a prefix of p's sorted row).
//
// It replaces ~15 eager tensor ops (an f64 GEMM, broadcasts, a batched sort, casts) whose launches sat
// between the round's host read and its passes on the 8-GPU shard (profiles/r4/shard/). Distances come
// from direct differences (no cancellation), so no expansion slack is needed; the outward rounding is.
#include "common.h"

namespace {

constexpr int kTabThreads = 256;
constexpr int kTabMax = 1024;  // new candidates per round (sorted in LDS)

__global__ __launch_bounds__(kTabThreads) void init_table_kernel(const double* __restrict__ P, int mp,
                                                                 const double* __restrict__ Y, int m, int d,
                                                                 float* __restrict__ tab_v, int* __restrict__ tab_j,
                                                                 float* __restrict__ pn32) {
  __shared__ float key[kTabMax];
  __shared__ int id[kTabMax];
  __shared__ double red[kTabThreads];
  const int i = blockIdx.x;
  const double* p = P + (long long)i * d;
  int mm = 1;
  while (mm < m) mm <<= 1;
  for (int j = threadIdx.x; j < mm; j += kTabThreads) {
    float kv = __builtin_huge_valf();
    if (j < m) {
      const double* y = Y + (long long)j * d;
      double a = 0.0;
      for (int t = 0; t < d; ++t) {
        const double e = p[t] - y[t];
        a = __fma_rn(e, e, a);
      }
      const double r = sqrt(a) * (1.0 - 1e-6);
      float f = (float)r;
      if ((double)f > r) f = nextafterf(f, 0.0f);
      kv = f;
    }
    key[j] = kv;
    id[j] = j;
  }
  double pn = 0.0;
  for (int t = threadIdx.x; t < d; t += kTabThreads) pn = __fma_rn(p[t], p[t], pn);
  red[threadIdx.x] = pn;
  __syncthreads();
  // bitonic sort of (key, id) ascending, ties by id
  for (int size = 2; size <= mm; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < mm; t += kTabThreads) {
        const int o = t ^ stride;
        if (o > t) {
          const bool up = (t & size) == 0;
          const float ka = key[t], kb = key[o];
          const int ia = id[t], ib = id[o];
          const bool gt = ka > kb || (ka == kb && ia > ib);
          if (gt == up) {
            key[t] = kb;
            key[o] = ka;
            id[t] = ib;
            id[o] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int j = threadIdx.x; j < m; j += kTabThreads) {
    tab_v[(long long)i * m + j] = key[j];
    tab_j[(long long)i * m + j] = id[j];
  }
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int t = 0; t < kTabThreads; ++t) s += red[t];
    const double u = s * (1.0 + 1e-6);
    float f = (float)u;
    if ((double)f < u) f = nextafterf(f, __builtin_huge_valf());
    pn32[i] = f;
  }
}

// Distinct candidate rows in ascending lexicographic order (models/kmeans.py _init_finish; torch.unique(dim=0)
// with return_inverse replaced: that sorts with a row comparator and runs ~10 small kernels around a host
// read of the count). m is a few thousand at most, so pairwise row comparisons — nearly all decided by the
// first column — are cheap: one block per row.
//   pass 1: dup[i] = some j < i has the same values (==: -0 equals 0, like the comparator's order)
//   pass 2: rank[i] = #{j : !dup[j], row j <lex row i} — equal rows get the same rank, the distinct rows
//           a permutation of 0..u-1 — so inverse = rank, uniq[rank[i]] = row i for !dup[i], u = max rank + 1
__device__ __forceinline__ int lex_cmp(const double* __restrict__ a, const double* __restrict__ b, int d) {
  for (int t = 0; t < d; ++t) {
    if (a[t] < b[t]) return -1;
    if (a[t] > b[t]) return 1;
  }
  return 0;
}

__device__ __forceinline__ int block_sum(int v, int* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = kTabThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const int r = red[0];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kTabThreads) void rows_dup_kernel(const double* __restrict__ P, int m, int d,
                                                               int* __restrict__ dup) {
  __shared__ int red[kTabThreads];
  const int i = blockIdx.x;
  const double* p = P + (long long)i * d;
  int hit = 0;
  for (int j = threadIdx.x; j < i && !hit; j += kTabThreads) hit = lex_cmp(P + (long long)j * d, p, d) == 0;
  const int any = block_sum(hit, red);
  if (threadIdx.x == 0) dup[i] = any > 0;
}

__global__ __launch_bounds__(kTabThreads) void rows_rank_kernel(const double* __restrict__ P, int m, int d,
                                                                const int* __restrict__ dup, long long* __restrict__ inv,
                                                                double* __restrict__ uniq, int* __restrict__ count) {
  __shared__ int red[kTabThreads];
  const int i = blockIdx.x;
  const double* p = P + (long long)i * d;
  int less = 0;
  for (int j = threadIdx.x; j < m; j += kTabThreads)
    if (!dup[j] && lex_cmp(P + (long long)j * d, p, d) < 0) ++less;
  const int r = block_sum(less, red);
  if (threadIdx.x == 0) {
    inv[i] = r;
    if (!dup[i]) atomicMax(count, r + 1);
  }
  if (!dup[i])
    for (int t = threadIdx.x; t < d; t += kTabThreads) uniq[(long long)r * d + t] = p[t];
}

}  // namespace

// P f64 [m, d] (contiguous); dup int32 [m] workspace; inv int64 [m]; uniq f64 [m, d] (first *count rows
// written); count int32 [1], zeroed by the caller.
CML_API int cml_kmeans_unique_rows(const double* P, int m, int d, int* dup, long long* inv, double* uniq, int* count,
                                   void* stream) {
  if (m <= 0) return 0;
  if (d <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_dup_kernel, dim3((unsigned)m), dim3(kTabThreads), 0, (hipStream_t)stream, P, m, d, dup);
  hipLaunchKernelGGL(rows_rank_kernel, dim3((unsigned)m), dim3(kTabThreads), 0, (hipStream_t)stream, P, m, d, dup, inv,
                     uniq, count);
  return cml_status();
}

// P f64 [mp, d], Y f64 [m, d] (m <= 1024); tab_v f32 / tab_j int32 [mp, m]; pn32 f32 [mp].
CML_API int cml_kmeans_init_table(const double* P, int mp, const double* Y, int m, int d, float* tab_v, int* tab_j,
                                  float* pn32, void* stream) {
  if (mp <= 0 || m <= 0) return 0;
  if (d <= 0 || m > kTabMax) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(init_table_kernel, dim3((unsigned)mp), dim3(kTabThreads), 0, (hipStream_t)stream, P, mp, Y, m, d,
                     tab_v, tab_j, pn32);
  return cml_status();
}
