// Latency-lean pieces of the k-means‖ init (models/kmeans.py _init_kmeans_parallel_gpu; the KMeans.fit
// headline of BASELINE.json, and the per-GPU shard of its 8-GPU run). On a 12.5M-row shard the init is a
// few ms of kernels separated by host work: every torch op between two kernels is a launch plus ~20 us of
// host time. These kernels each replace a run of such ops:
//
//   gather_rank_rows  the sampled candidate rows of a round, in row order, widened to f64 straight into the
//                     round's slot of the candidate buffer: a row's position is its rank among the sampled
//                     ids (distinct ids: O(m) comparisons per row, no sort pass), its values the bf16 /
//                     e4m3 row. Replaces torch.sort + an index gather + a dtype cast + a pad copy.
//   seed_table        per distinct init candidate p, its nearest / second-nearest bf16 centre (a, d1, d2)
//                     by direct differences in f64, rounded outward, and ||p||² rounded up: the tables the
//                     first Lloyd step's seeded bounds read (kmeans_seed_bounds_kernel). Replaces an f64
//                     GEMM, a top-k and ~25 elementwise ops.
//   pair_table        init_table's sorted candidate-distance rows with coalesced loads: the new candidates
//                     transposed, four existing candidates per workgroup, a thread per new candidate — the
//                     first version's per-thread row walks read 2-KB strided columns (300 us for 513 x 512
//                     candidates at D = 256).
#include "common.h"

namespace {

constexpr int kGThreads = 256;
constexpr int kGMax = 16384;  // sampled ids one launch ranks (64 KiB of LDS)

// dest[rank(i)] = widen(X[ids[i]]) for i < min(*cnt, cap); rows [m, pad_rows) of dest are zeroed (the
// padded all-gather slot of this rank). ids distinct. X: bf16 (xfp8 = 0) or e4m3 bytes, row pitch ldx BYTES.
__global__ __launch_bounds__(kGThreads) void gather_rank_rows_kernel(const unsigned char* __restrict__ X,
                                                                     long long ldx, int xfp8, int d,
                                                                     const int* __restrict__ ids,
                                                                     const int* __restrict__ cnt, int cap,
                                                                     double* __restrict__ dest, int pad_rows) {
  __shared__ int sid[kGMax];
  const int m = min(*cnt, cap);
  for (int i = threadIdx.x; i < m; i += kGThreads) sid[i] = ids[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = gridDim.x * (kGThreads / 64);
  for (int r = blockIdx.x * (kGThreads / 64) + wave; r < max(m, pad_rows); r += nwaves) {
    double* out;
    if (r < m) {
      const int me = sid[r];
      int less = 0;
      for (int j = lane; j < m; j += 64) less += sid[j] < me;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) less += __shfl_xor(less, o, 64);
      out = dest + (long long)less * d;
      const unsigned char* row = X + (long long)me * ldx;
      for (int t = lane; t < d; t += 64) {
        double v;
        if (xfp8) {
          typedef float f32x2 __attribute__((ext_vector_type(2)));
          const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)row[t], false);
          v = (double)a.x;
        } else {
          v = (double)bf16_to_f32(reinterpret_cast<const u16*>(row)[t]);
        }
        out[t] = v;
      }
    } else {
      out = dest + (long long)r * d;
      for (int t = lane; t < d; t += 64) out[t] = 0.0;
    }
  }
}

// One workgroup per distinct candidate i: top-2 of |U_i - c_j|² over the k bf16 centres (ties: lowest j).
__global__ __launch_bounds__(kGThreads) void seed_table_kernel(const double* __restrict__ U, int m, int d,
                                                               const u16* __restrict__ cb, long long ldc, int k,
                                                               int* __restrict__ a_out, float* __restrict__ d1_out,
                                                               float* __restrict__ d2_out, float* __restrict__ pn_out) {
  extern __shared__ double su[];  // [d]
  __shared__ double bv1[kGThreads / 64], bv2[kGThreads / 64];
  __shared__ int bi1[kGThreads / 64];
  __shared__ double pnw[kGThreads / 64];
  const int i = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double pn = 0.0;
  for (int t = threadIdx.x; t < d; t += kGThreads) {
    const double v = U[(long long)i * d + t];
    su[t] = v;
    pn = __fma_rn(v, v, pn);
  }
  pn = wave_sum_f64(pn);
  if (lane == 0) pnw[wave] = pn;
  __syncthreads();
  // a wave per centre (strided over the waves): lanes over the columns, shuffle sum
  double v1 = __builtin_huge_val(), v2 = __builtin_huge_val();
  int i1 = 0x7fffffff;
  for (int j = wave; j < k; j += kGThreads / 64) {
    double s = 0.0;
    for (int t = lane; t < d; t += 64) {
      const double e = su[t] - (double)bf16_to_f32(cb[(long long)j * ldc + t]);
      s = __fma_rn(e, e, s);
    }
    s = wave_sum_f64(s);
    if (s < v1) { v2 = v1; v1 = s; i1 = j; }  // j ascending per wave: strict < keeps the lowest index
    else if (s < v2) v2 = s;
  }
  if (lane == 0) { bv1[wave] = v1; bv2[wave] = v2; bi1[wave] = i1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t1 = __builtin_huge_val(), t2 = __builtin_huge_val();
    int ti = 0x7fffffff;
    double p = 0.0;
    for (int w = 0; w < kGThreads / 64; ++w) {
      p += pnw[w];
      const double a1 = bv1[w], a2 = bv2[w];
      const int ai = bi1[w];
      if (a1 < t1 || (a1 == t1 && ai < ti)) { t2 = fmin(t1, a2); t1 = a1; ti = ai; }
      else t2 = fmin(t2, a1);
    }
    // direct differences: the f64 fold is within (d + 2)·2^-53 of the exact squared distance; the outward
    // factors keep d1 above and d2 below the real distances by a wide margin, then f32 rounds outward too
    const double u1 = sqrt(t1 * (1.0 + 1e-12)) * (1.0 + 1e-6);
    float f1 = (float)u1;
    if ((double)f1 < u1) f1 = nextafterf(f1, __builtin_huge_valf());
    float f2 = __builtin_huge_valf();
    if (k > 1) {
      const double u2 = sqrt(fmax(t2 * (1.0 - 1e-12), 0.0)) * (1.0 - 1e-6);
      f2 = (float)u2;
      if ((double)f2 > u2) f2 = nextafterf(f2, 0.0f);
    }
    const double up = p * (1.0 + 1e-6);
    float fp = (float)up;
    if ((double)fp < up) fp = nextafterf(fp, __builtin_huge_valf());
    a_out[i] = ti;
    d1_out[i] = f1;
    d2_out[i] = f2;
    pn_out[i] = fp;
  }
}

// init_table with coalesced reads (see the file comment): the new candidates come TRANSPOSED (YT [d][m]),
// thread t owns candidates t, t+256, ... (up to 4), every step c reads one contiguous run YT[c][*] across
// the block and the kPB existing candidates' values from LDS; each (p, y) distance is one serial f64 fold.
constexpr int kTabMax = 1024;
constexpr int kPB = 4;
constexpr int kJPT = kTabMax / kGThreads;
__global__ __launch_bounds__(kGThreads) void pair_table_kernel(const double* __restrict__ P, int mp,
                                                               const double* __restrict__ YT, int m, int d,
                                                               float* __restrict__ tab_v, int* __restrict__ tab_j,
                                                               float* __restrict__ pn32) {
  extern __shared__ double sp[];  // [kPB][d]
  __shared__ float key[kPB][kTabMax];
  __shared__ int id[kPB][kTabMax];
  const int i0 = blockIdx.x * kPB, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int np = min(kPB, mp - i0);
  for (int e = tid; e < kPB * d; e += kGThreads) {
    const int r = e / d, t = e - r * d;
    sp[e] = r < np ? P[(long long)(i0 + r) * d + t] : 0.0;
  }
  __syncthreads();
  double acc[kPB][kJPT];
#pragma unroll
  for (int r = 0; r < kPB; ++r)
#pragma unroll
    for (int q = 0; q < kJPT; ++q) acc[r][q] = 0.0;
#pragma unroll 4
  for (int c = 0; c < d; ++c) {
    double y[kJPT];
#pragma unroll
    for (int q = 0; q < kJPT; ++q) {
      const int j = tid + q * kGThreads;
      y[q] = j < m ? YT[(long long)c * m + j] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < kPB; ++r) {
      const double pv = sp[r * d + c];
#pragma unroll
      for (int q = 0; q < kJPT; ++q) {
        const double e = pv - y[q];
        acc[r][q] = __fma_rn(e, e, acc[r][q]);
      }
    }
  }
  int mm = 1;
  while (mm < m) mm <<= 1;
#pragma unroll
  for (int q = 0; q < kJPT; ++q) {
    const int j = tid + q * kGThreads;
    if (j >= mm) continue;
#pragma unroll
    for (int r = 0; r < kPB; ++r) {
      float kv = __builtin_huge_valf();
      if (j < m) {
        const double rr = sqrt(acc[r][q]) * (1.0 - 1e-6);
        kv = (float)rr;
        if ((double)kv > rr) kv = nextafterf(kv, 0.0f);
      }
      key[r][j] = kv;
      id[r][j] = j;
    }
  }
  __syncthreads();
  // bitonic sort of each row's (key, id) ascending, ties by id
  for (int size = 2; size <= mm; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = tid; e < kPB * mm; e += kGThreads) {
        const int r = e / mm, t = e - r * mm;
        const int o = t ^ stride;
        if (o > t) {
          const bool up = (t & size) == 0;
          const float ka = key[r][t], kb = key[r][o];
          const int ia = id[r][t], ib = id[r][o];
          const bool gt = ka > kb || (ka == kb && ia > ib);
          if (gt == up) {
            key[r][t] = kb;
            key[r][o] = ka;
            id[r][t] = ib;
            id[r][o] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int r = 0; r < np; ++r) {
    for (int j = tid; j < m; j += kGThreads) {
      tab_v[(long long)(i0 + r) * m + j] = key[r][j];
      tab_j[(long long)(i0 + r) * m + j] = id[r][j];
    }
  }
  if (wave < np) {
    double s = 0.0;
    for (int t = lane; t < d; t += 64) s = __fma_rn(sp[wave * d + t], sp[wave * d + t], s);
    s = wave_sum_f64(s);
    if (lane == 0) {
      const double u = s * (1.0 + 1e-6);
      float f = (float)u;
      if ((double)f < u) f = nextafterf(f, __builtin_huge_valf());
      pn32[i0 + wave] = f;
    }
  }
}

}  // namespace

// X row pitch ldx in BYTES; ids int32 [cap] (the first *cnt are the sampled rows); dest f64 [max(m, pad_rows), d].
CML_API int cml_kmeans_gather_rank_rows(const void* X, long long ldx, int xfp8, int d, const int* ids, const int* cnt,
                                        int cap, double* dest, int pad_rows, int grid, void* stream) {
  if (cap < 0 || cap > kGMax || d <= 0 || grid <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rank_rows_kernel, dim3((unsigned)grid), dim3(kGThreads), 0, (hipStream_t)stream,
                     (const unsigned char*)X, ldx, xfp8, d, ids, cnt, cap, dest, pad_rows);
  return cml_status();
}

CML_API int cml_kmeans_gather_rank_max() { return kGMax; }

// U f64 [m, d]; cb bf16 [>= k rows, ldc]; outputs int32 / f32 [m].
CML_API int cml_kmeans_seed_table(const double* U, int m, int d, const void* cb, long long ldc, int k, int* a,
                                  float* d1, float* d2, float* pn, void* stream) {
  if (m <= 0) return 0;
  if (d <= 0 || k <= 0 || (size_t)d * 8 > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(seed_table_kernel, dim3((unsigned)m), dim3(kGThreads), (size_t)d * 8, (hipStream_t)stream, U, m,
                     d, (const u16*)cb, ldc, k, a, d1, d2, pn);
  return cml_status();
}

// P f64 [mp, d], YT f64 [d, m] (the new candidates transposed, m <= 1024); tab_v f32 / tab_j int32 [mp, m];
// pn32 f32 [mp].
CML_API int cml_kmeans_pair_table(const double* P, int mp, const double* YT, int m, int d, float* tab_v, int* tab_j,
                                  float* pn32, void* stream) {
  if (mp <= 0 || m <= 0) return 0;
  if (d <= 0 || m > kTabMax || (size_t)kPB * d * 8 > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pair_table_kernel, dim3((unsigned)((mp + kPB - 1) / kPB)), dim3(kGThreads),
                     (size_t)kPB * d * 8, (hipStream_t)stream, P, mp, YT, m, d, tab_v, tab_j, pn32);
  return cml_status();
}
