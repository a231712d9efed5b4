// K12 — k-means|| initialisation on the device (models/kmeans.py ``init_kmeans_parallel``).
//
// The reference has no KMeans; this is Spark MLlib's default initMode
// ("k-means||", initSteps = 2: mllib/clustering/KMeans.scala initKMeansParallel), re-designed so the
// init of the 100M x 256 headline fit costs a few memory passes instead of ~80 host round trips:
//
//   row pass      one read of X: ||x||² (THE row-norm kernel: cml_row_sqnorm_* run it too, so cached
//                 norms are the same bits whichever path made them), the distance to the first
//                 centre (the first k-means|| cost), max ||x||² (pruning bounds) and the range of
//                 the bf16 exponents (exactness guard of the incremental sums) — fused: the init
//                 used to read X twice for these;
//   sample        u(seed, round, global row) < 2k·cost/Σcost (utils/rng.py counter uniform, the same
//                 splitmix64 as K5), compacted to a row list;
//   merge         cost/nearest-candidate update from one K9r pass over a candidate chunk (strict <:
//                 the earlier candidate keeps ties, i.e. argmin order over the candidate list);
//   local k-means weighted k-means++ seeding + weighted Lloyd (Spark LocalKMeans.kMeansPlusPlus)
//                 on the ~2k·initSteps candidates, as a few small kernels with no host round trip
//                 per pick. Every value is formed in a fixed order with explicitly rounded f64
//                 operations (_rn intrinsics, no contraction), and host/kmeans_local.cpp performs the
//                 same operations in the same order: the CPU session and the GPU pick the same
//                 centres bit for bit.
#include "common.h"

#include <algorithm>
#include <cstdint>

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// u in [0, 1) of counter c under key (utils/rng.py uniform)
__device__ __forceinline__ double cu(unsigned long long c, unsigned long long key) {
  return (double)(splitmix64(c ^ key) >> 11) * (1.0 / 9007199254740992.0);
}

// ----------------------------------------------------------------------------------------- row pass
// A row of NCH 16-byte chunks is read by LPR = NCH / CPL lanes, lane l taking chunks l, l + LPR, ...
// (CPL of them: each load instruction covers LPR·16 contiguous bytes of RPW = 64 / LPR rows). Each lane
// folds its values in chunk order with f32 fma, then a butterfly over the row's lanes: that fold is
// THE definition of the cached ||x||² (cml_row_sqnorm_* run this same kernel). 8 lanes per 512-B row
// (CPL = 4) instead of one lane per chunk keep the shuffle count per byte low; the first version
// (32 lanes per row, 5 butterfly steps for each of the two sums) ran 13 ms for 51 GB, VALU-bound.
// U row groups are in flight per lane. c0 (f32 [Dp], the bf16-rounded first centre) may be null.
// Exponent range of the bf16 magnitudes, branch-free: max of |bits|, min of (|bits| - 1) mod 2^16.
template <int NCH, int CPL, bool F8, int U>
__global__ __launch_bounds__(kThreads) void row_pass_kernel(const unsigned char* __restrict__ X, long long n,
                                                            long long ldb, float* __restrict__ xn_out,
                                                            const float* __restrict__ c0, float c0n,
                                                            float* __restrict__ cost_out, int* __restrict__ near_out,
                                                            unsigned* __restrict__ xn_max,
                                                            int* __restrict__ erange, double* __restrict__ xn64,
                                                            const float* __restrict__ c0n_dev) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  if (c0n_dev != nullptr) c0n = *c0n_dev;  // ||c0||² left on the device by the centre conversion
  constexpr int LPR = NCH / CPL;
  static_assert(LPR >= 1 && LPR <= 64 && NCH % CPL == 0, "row split");
  const bool wide = xn64 != nullptr;
  constexpr int RPW = 64 / LPR;
  constexpr int VPC = F8 ? 16 : 8;  // values per chunk
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, c = lane - sub * LPR;
  const long long w0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  const bool dot = c0 != nullptr;
  // exponent range on packed 16-bit halves (v_pk_max_u16 / v_pk_sub_u16 / v_pk_min_u16: four instructions per
  // pair of values instead of ~eight; the pass is VALU-bound): max |bits|, min (|bits| - 1) mod 2^16
  us2 pmx = {0, 0}, pmn = {0xffff, 0xffff};
  unsigned mxb = 0;
  // this lane's columns of the first centre, in registers for the whole pass (re-reading them from
  // the cache every row tripled the pass's load traffic)
  float cr[CPL][VPC];
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < VPC; ++e) cr[i][e] = dot ? c0[VPC * (c + LPR * i) + e] : 0.f;
  for (long long r0 = w0 * RPW; r0 < n; r0 += nw * RPW * U) {
    uint4 v[U][CPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + (long long)u * nw * RPW + sub;
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        v[u][i] = row < n ? *reinterpret_cast<const uint4*>(X + row * ldb + 16 * (c + LPR * i))
                          : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + (long long)u * nw * RPW + sub;
      float s = 0.f, dt = 0.f;
      double s64 = 0.0;
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const unsigned w[4] = {v[u][i].x, v[u][i].y, v[u][i].z, v[u][i].w};
        float xs[VPC];
        if constexpr (F8) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[q], false);
            const f2 b = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[q], true);
            xs[4 * q] = a.x;
            xs[4 * q + 1] = a.y;
            xs[4 * q + 2] = b.x;
            xs[4 * q + 3] = b.y;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            xs[2 * q] = bf16_to_f32((u16)(w[q] & 0xffffu));
            xs[2 * q + 1] = bf16_to_f32((u16)(w[q] >> 16));
            const us2 m = __builtin_bit_cast(us2, w[q] & 0x7fff7fffu);  // rows past n load zeros
            pmx = __builtin_elementwise_max(pmx, m);
            pmn = __builtin_elementwise_min(pmn, m - us2{1, 1});  // wraps: a zero goes to 0xffff
          }
        }
#pragma unroll
        for (int e = 0; e < VPC; ++e) s = fmaf(xs[e], xs[e], s);
        if (wide) {  // x² of a bf16 / e4m3 value is exact in f64: one f64 fma adds it with the sum's own rounding
#pragma unroll
          for (int e = 0; e < VPC; ++e) {
            const double xd = (double)xs[e];
            s64 = fma(xd, xd, s64);
          }
        }
        if (dot) {
#pragma unroll
          for (int e = 0; e < VPC; ++e) dt = fmaf(xs[e], cr[i][e], dt);
        }
      }
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        if (dot) dt += __shfl_xor(dt, o, 64);
        if (wide) s64 += __shfl_xor(s64, o, 64);
      }
      if (c == 0 && row < n) {
        xn_out[row] = s;
        if (wide) xn64[row] = s64;
        mxb = __float_as_uint(s) > mxb ? __float_as_uint(s) : mxb;
        if (dot) {
          cost_out[row] = fmaxf(fmaf(-2.f, dt, s + c0n), 0.f);
          near_out[row] = 0;
        }
      }
    }
  }
  unsigned umx = pmx[0] > pmx[1] ? pmx[0] : pmx[1], umn = pmn[0] < pmn[1] ? pmn[0] : pmn[1];
  // wave reductions, one atomic per wave (integer min/max: the result does not depend on order)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mxb = max(mxb, (unsigned)__shfl_xor(mxb, o, 64));
    umx = max(umx, (unsigned)__shfl_xor(umx, o, 64));
    umn = min(umn, (unsigned)__shfl_xor(umn, o, 64));
  }
  if (lane == 0) {
    if (xn_max != nullptr) atomicMax(xn_max, mxb);  // non-negative floats order as their bits
    if (erange != nullptr && !F8 && umx != 0u) {
      atomicMin(erange, (int)((umn + 1u) >> 7));
      atomicMax(erange + 1, (int)(umx >> 7));
    }
  }
}

// Exact training cost of an assignment: Σ_i |x_i - c_lab(i)|² with every difference and square in f64
// (the values are bf16 / e4m3 and the centres the bf16 copies the assign compared against, so each
// term is exact up to the f64 sum). The expanded form Σ(Q_j - 2c_j·S_j + n_j|c_j|²) of the pruned step
// cancels catastrophically for data far from the origin (|x|² >> cost); this pass
// reads X once instead, in the row-pass layout (LPR lanes per row, CPL 16-B chunks per lane), and
// leaves fixed-order block partials (deterministic for a given n).
template <int NCH, int CPL, bool F8, int U>
__global__ __launch_bounds__(kThreads) void cost_pass_kernel(const unsigned char* __restrict__ X, long long n,
                                                             long long ldb, const int* __restrict__ lab,
                                                             const u16* __restrict__ cb, long long ldc,
                                                             double* __restrict__ part) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int LPR = NCH / CPL;
  constexpr int RPW = 64 / LPR;
  constexpr int VPC = F8 ? 16 : 8;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, c = lane - sub * LPR;
  const long long w0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  double acc = 0.0;
  for (long long r0 = w0 * RPW; r0 < n; r0 += nw * RPW * U) {
    uint4 v[U][CPL];
    int lb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + (long long)u * nw * RPW + sub;
      lb[u] = row < n ? lab[row] : 0;
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        v[u][i] = row < n ? *reinterpret_cast<const uint4*>(X + row * ldb + 16 * (c + LPR * i))
                          : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + (long long)u * nw * RPW + sub;
      const u16* cr = cb + (long long)lb[u] * ldc;
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const unsigned w[4] = {v[u][i].x, v[u][i].y, v[u][i].z, v[u][i].w};
        float xs[VPC];
        if constexpr (F8) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[q], false);
            const f2 b = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[q], true);
            xs[4 * q] = a.x;
            xs[4 * q + 1] = a.y;
            xs[4 * q + 2] = b.x;
            xs[4 * q + 3] = b.y;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            xs[2 * q] = bf16_to_f32((u16)(w[q] & 0xffffu));
            xs[2 * q + 1] = bf16_to_f32((u16)(w[q] >> 16));
          }
        }
        const int col0 = VPC * (c + LPR * i);
        unsigned cw[VPC / 2];
#pragma unroll
        for (int h = 0; h < VPC / 8; ++h) {
          const uint4 t = row < n ? *reinterpret_cast<const uint4*>(cr + col0 + 8 * h) : make_uint4(0u, 0u, 0u, 0u);
          cw[4 * h] = t.x;
          cw[4 * h + 1] = t.y;
          cw[4 * h + 2] = t.z;
          cw[4 * h + 3] = t.w;
        }
#pragma unroll
        for (int e = 0; e < VPC; ++e) {
          const float cv = bf16_to_f32((u16)((e & 1) ? (cw[e >> 1] >> 16) : (cw[e >> 1] & 0xffffu)));
          const double df = (double)xs[e] - (double)cv;
          s = fma(df, df, s);
        }
      }
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (c == 0 && row < n) acc += s;
    }
  }
  acc = wave_sum_f64(acc);
  __shared__ double ws[kThreads / 64];
  if (lane == 0) ws[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kThreads / 64; ++w) t += ws[w];
    part[blockIdx.x] = t;
  }
}

// cost/nearest from one candidate chunk's K9r pass (best distance + label within the chunk)
__global__ __launch_bounds__(kThreads) void init_merge_kernel(float* __restrict__ cost, int* __restrict__ near,
                                                              const float* __restrict__ best,
                                                              const int* __restrict__ lab, int off, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float b = best[i];
    if (b < cost[i]) {
      cost[i] = b;
      near[i] = lab[i] + off;
    }
  }
}

// rows with u(row id) < scale·cost (Spark: rand < 2·k·cost / Σcost), appended to out (unordered)
__global__ __launch_bounds__(kThreads) void init_sample_kernel(const float* __restrict__ cost,
                                                               const long long* __restrict__ ids, long long n,
                                                               unsigned long long key, double scale,
                                                               int* __restrict__ out, int* __restrict__ count,
                                                               long long cap, const double* __restrict__ scale_dev) {
  // scale_dev (may be null): {Σ cost over every rank, 2k}: the round's rate 2k / Σcost formed on the
  // device (no host read of the all-reduced total); Σcost = 0 draws nothing (inf·0 compares false)
  if (scale_dev != nullptr) scale = scale_dev[1] / scale_dev[0];
  const int lane = threadIdx.x & 63;
  for (long long i0 = (long long)blockIdx.x * blockDim.x; i0 < n; i0 += (long long)gridDim.x * blockDim.x) {
    const long long i = i0 + threadIdx.x;
    bool take = false;
    if (i < n) take = cu((unsigned long long)ids[i], key) < scale * (double)cost[i];
    const unsigned long long bal = __ballot(take);
    if (bal) {
      const int leader = __builtin_ctzll(bal);
      int base = 0;
      if (lane == leader) base = atomicAdd(count, (int)__popcll(bal));
      base = __shfl(base, leader, 64);
      const long long at = base + (long long)__popcll(bal & ((1ull << lane) - 1ull));
      if (take && at < cap) out[at] = (int)i;
    }
  }
}

// ------------------------------------------------------------------------------- local k-means
// dist(p, c) = fold over t of fma(p_t - c_t, p_t - c_t, acc), acc from 0 (host twin: kmeans_local.cpp)
__device__ __forceinline__ double dist_seq(const double* __restrict__ p, const double* c, int d) {
  double acc = 0.0;
  for (int t = 0; t < d; ++t) {
    const double e = __dsub_rn(p[t], c[t]);
    acc = __fma_rn(e, e, acc);
  }
  return acc;
}

constexpr int kBlocks = 256;  // fixed block count of the weighted prefix sums (host twin: the same)

// Weighted k-means++ seeding (Spark LocalKMeans.kMeansPlusPlus): pick 0 ∝ w, pick i ∝ w·d²; the
// cumulative weight is summed in kBlocks contiguous blocks (fixed order), the pick walks it.
// One workgroup of kKppThreads; the points are read transposed (PT[t*m + q]: a wave's reads are
// contiguous), the chosen centre sits in LDS (d doubles). One thread per point and dimension-
// sequential distance folds keep the host twin's order.
constexpr int kKppThreads = 1024;

__global__ __launch_bounds__(kKppThreads) void local_kpp_kernel(const double* __restrict__ P,
                                                                const double* __restrict__ PT,
                                                                const double* __restrict__ D, int m, int d,
                                                                const double* __restrict__ w, int k,
                                                                unsigned long long key, double* __restrict__ C,
                                                                double* __restrict__ CT, double* __restrict__ d2,
                                                                bool lds_pw) {
  extern __shared__ __align__(16) unsigned char smem[];
  double* crow = reinterpret_cast<double*>(smem);
  // with room in LDS the pick weights w·d2 and the distances live there (the serial scans of a pick
  // then read LDS, not L2); same values and order as the global form
  const bool in_lds = lds_pw;
  double* pwl = crow + d;      // [m] pick weights (in_lds)
  double* d2l = pwl + m;       // [m] running distances (in_lds)
  __shared__ double part[kBlocks];
  __shared__ int pick_sh;
  const int tid = threadIdx.x;
  const int L = (m + kBlocks - 1) / kBlocks;
  if (in_lds)
    for (int q = tid; q < m; q += kKppThreads) pwl[q] = w[q];
  __syncthreads();
  for (int i = 0; i < k; ++i) {
    auto pw_at = [&](int q) { return in_lds ? pwl[q] : (i == 0 ? w[q] : __dmul_rn(w[q], d2[q])); };
    if (tid < kBlocks) {
      double s = 0.0;
      const int q1 = min(m, (tid + 1) * L);
      for (int q = tid * L; q < q1; ++q) s = __dadd_rn(s, pw_at(q));
      part[tid] = s;
    }
    __syncthreads();
    if (tid < 64) {
      // wave 0: lane l folds parts 4l..4l+3 in order, an inclusive Hillis-Steele scan over the 64 lane
      // sums (S[l] = S[l - off] + S[l] at off = 1, 2, ..., 32) gives the total and the prefixes; the
      // first lane whose prefix exceeds r walks its 4 parts and then the points of the block
      // (kpp_pick in the host twin: the same operations in the same order)
      const int l = tid;
      double q4 = part[4 * l];
#pragma unroll
      for (int j = 1; j < 4; ++j) q4 = __dadd_rn(q4, part[4 * l + j]);
      double S = q4;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const double o = __shfl_up(S, off, 64);
        if (l >= off) S = __dadd_rn(o, S);
      }
      const double total = __shfl(S, 63, 64);
      const double u = cu((unsigned long long)i, key);
      int pick = -1;
      if (!(total > 0.0)) {
        pick = (int)__dmul_rn(u, (double)m);
        pick = pick < m - 1 ? pick : m - 1;
      } else {
        const double r = __dmul_rn(u, total);
        const unsigned long long over = __ballot(S > r);
        if (over != 0ull) {
          const int ls = __builtin_ctzll(over);
          const double prev = __shfl(S, ls > 0 ? ls - 1 : 0, 64);
          if (l == ls) {
            double cum = ls > 0 ? prev : 0.0;
            int lastb = -1;
            for (int j = 0; j < 4 && pick < 0; ++j) {
              const int b = 4 * l + j;
              const double nxt = __dadd_rn(cum, part[b]);
              if (part[b] > 0.0) lastb = b;
              if (nxt > r) {
                double c2 = cum;
                const int q1 = min(m, (b + 1) * L);
                int lastpos = -1;
                for (int q = b * L; q < q1; ++q) {
                  const double pw = pw_at(q);
                  if (pw > 0.0) lastpos = q;
                  c2 = __dadd_rn(c2, pw);
                  if (c2 > r) { pick = q; break; }
                }
                if (pick < 0) pick = lastpos;
              }
              cum = nxt;
            }
            if (pick < 0 && lastb >= 0) {  // rounding between the lane prefix and the part walk
              const int q1 = min(m, (lastb + 1) * L);
              for (int q = lastb * L; q < q1; ++q)
                if (pw_at(q) > 0.0) pick = q;
            }
          }
          pick = __shfl(pick, ls, 64);
        }
        if (pick < 0 && l == 0) {  // rounding: the last point of positive weight
          for (int q = m - 1; q >= 0 && pick < 0; --q)
            if (pw_at(q) > 0.0) pick = q;
        }
        if (pick < 0) pick = 0;
      }
      if (l == 0) pick_sh = pick;
    }
    __syncthreads();
    const int pk = pick_sh;
    for (int t = tid; t < d; t += kKppThreads) {
      const double v = P[(long long)pk * d + t];
      crow[t] = v;
      C[(long long)i * d + t] = v;
      CT[(long long)t * k + i] = v;
    }
    if (D == nullptr) __syncthreads();  // (crow feeds only the fold below; with D the two row reads overlap)
    if (D != nullptr && in_lds) {
      const double* dr = D + (long long)pk * m;
      for (int q = tid; q < m; q += kKppThreads) {
        const double acc = dr[q];
        const double nd = (i == 0 || acc < d2l[q]) ? acc : d2l[q];
        d2l[q] = nd;
        pwl[q] = __dmul_rn(w[q], nd);
      }
    } else if (D != nullptr) {  // precomputed pairwise distances: the update is one contiguous row read
      const double* dr = D + (long long)pk * m;
      for (int q = tid; q < m; q += kKppThreads) {
        const double acc = dr[q];
        d2[q] = (i == 0 || acc < d2[q]) ? acc : d2[q];
      }
    } else {
      for (int q = tid; q < m; q += kKppThreads) {
        double acc = 0.0;
        for (int t = 0; t < d; ++t) {
          const double e = __dsub_rn(PT[(long long)t * m + q], crow[t]);
          acc = __fma_rn(e, e, acc);
        }
        d2[q] = (i == 0 || acc < d2[q]) ? acc : d2[q];
      }
    }
    __syncthreads();
  }
}

// D[i][q] = dist(P_q, P_i) (the fold of the k-means++ update: e = P_q[t] - P_i[t], acc = fma(e, e,
// acc)) for every candidate pair, 16 x 16 pairs per workgroup with both row blocks staged in LDS
// in 64-dimension slices; each thread folds its pair over the dimensions in order.
constexpr int kPairT = 16, kPairS = 64;
__global__ __launch_bounds__(kThreads) void local_pairdist_kernel(const double* __restrict__ P, int m, int d,
                                                                  double* __restrict__ D) {
  __shared__ double ri[kPairT][kPairS + 1], rq[kPairT][kPairS + 1];
  const int tid = threadIdx.x, ti = tid / kPairT, tq = tid % kPairT;
  const int i0 = blockIdx.y * kPairT, q0 = blockIdx.x * kPairT;
  double acc = 0.0;
  for (int s0 = 0; s0 < d; s0 += kPairS) {
    const int w = min(kPairS, d - s0);
    for (int e = tid; e < kPairT * kPairS; e += kThreads) {
      const int r = e / kPairS, t = e % kPairS;
      ri[r][t] = (i0 + r < m && t < w) ? P[(long long)(i0 + r) * d + s0 + t] : 0.0;
      rq[r][t] = (q0 + r < m && t < w) ? P[(long long)(q0 + r) * d + s0 + t] : 0.0;
    }
    __syncthreads();
    for (int t = 0; t < w; ++t) {
      const double e = __dsub_rn(rq[tq][t], ri[ti][t]);
      acc = __fma_rn(e, e, acc);
    }
    __syncthreads();
  }
  if (i0 + ti < m && q0 + tq < m) D[(long long)(i0 + ti) * m + q0 + tq] = acc;
}

// labels[q] = argmin_j dist(P_q, C_j) (ties: lowest j); *moved = 1 if any label changed.
// One workgroup per point; centres read transposed (CT[t*k + j]) so a wave's reads are contiguous.
__global__ __launch_bounds__(kThreads) void local_assign_kernel(const double* __restrict__ P, int m, int d,
                                                                const double* __restrict__ CT, int k,
                                                                int* __restrict__ labels, int* __restrict__ moved,
                                                                const int* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;  // converged earlier: a queued iteration is a no-op
  extern __shared__ __align__(16) unsigned char smem[];
  double* prow = reinterpret_cast<double*>(smem);
  __shared__ double bd[kThreads];
  __shared__ int bj[kThreads];
  const int q = blockIdx.x, tid = threadIdx.x;
  for (int t = tid; t < d; t += kThreads) prow[t] = P[(long long)q * d + t];
  __syncthreads();
  double best = __builtin_huge_val();
  int bi = 0x7fffffff;
  for (int j = tid; j < k; j += kThreads) {
    double acc = 0.0;
    for (int t = 0; t < d; ++t) {
      const double e = __dsub_rn(prow[t], CT[(long long)t * k + j]);
      acc = __fma_rn(e, e, acc);
    }
    if (acc < best) { best = acc; bi = j; }  // j ascending: strict < keeps the lowest index
  }
  bd[tid] = best;
  bj[tid] = bi;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (tid < o) {
      const double a = bd[tid], b = bd[tid + o];
      const int ia = bj[tid], ib = bj[tid + o];
      if (b < a || (b == a && ib < ia)) { bd[tid] = b; bj[tid] = ib; }
    }
    __syncthreads();
  }
  if (tid == 0 && labels[q] != bj[0]) {
    labels[q] = bj[0];
    *moved = 1;
  }
}

// C_j = Σ_{label q = j, q ascending} w_q·P_q (fma folds) · (1 / Σ w_q); cnt[j] = Σ w_q. One workgroup
// per cluster; spherical: the mean is divided by its norm (sequential fold, correctly rounded sqrt).
__global__ __launch_bounds__(kThreads) void local_update_kernel(const double* __restrict__ P, int m, int d,
                                                                const double* __restrict__ w,
                                                                const int* __restrict__ labels, int k,
                                                                double* __restrict__ C, double* __restrict__ CT,
                                                                double* __restrict__ cnt, int spherical,
                                                                int* __restrict__ flags, int slot) {
  // flags (may be null: unconditional): {stop, moved[2]}. This iteration's assign set moved[slot] if a
  // label changed; none changed -> converged: latch stop (this and every later queued launch is a no-op,
  // as the host loop's break was). Block 0 clears the other slot for the next iteration's assign.
  if (flags != nullptr) {
    if (flags[0] != 0) return;
    if (flags[1 + slot] == 0) {
      if (blockIdx.x == 0 && threadIdx.x == 0) flags[0] = 1;
      return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) flags[2 - slot] = 0;
  }
  extern __shared__ __align__(16) unsigned char smem[];
  int* mem = reinterpret_cast<int*>(smem);                          // [m] members of cluster j, ascending
  double* cvals = reinterpret_cast<double*>(smem + (((size_t)m * 4 + 15) & ~(size_t)15));  // [d]
  __shared__ double inv_sh, nrm_sh;
  __shared__ int wcnt[kThreads / 64], nmem_sh;
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // members in ascending point order (ballot compaction, 256 points per round): the folds below then
  // visit only the cluster's points, in the order the all-points loop did (same bits, ~m/k iterations)
  int nmem = 0;
  for (int q0 = 0; q0 < m; q0 += kThreads) {
    const int q = q0 + tid;
    const bool in = q < m && labels[q] == j;
    const unsigned long long b = __ballot(in);
    if (lane == 0) wcnt[wv] = (int)__popcll(b);
    __syncthreads();
    int off = nmem;
    for (int u = 0; u < wv; ++u) off += wcnt[u];
    if (in) mem[off + (int)__popcll(b & ((1ull << lane) - 1ull))] = q;
    for (int u = 0; u < kThreads / 64; ++u) nmem += wcnt[u];
    __syncthreads();  // wcnt reused by the next round
  }
  if (tid == 0) {
    double c = 0.0;
    for (int u = 0; u < nmem; ++u) c = __dadd_rn(c, w[mem[u]]);
    cnt[j] = c;
    inv_sh = c > 0.0 ? __ddiv_rn(1.0, c) : 0.0;
    nmem_sh = c > 0.0 ? nmem : 0;
  }
  __syncthreads();
  if (nmem_sh == 0) return;  // empty: local_empty_kernel reseeds it
  const double inv = inv_sh;
  for (int t = tid; t < d; t += kThreads) {
    double s = 0.0;
    for (int u = 0; u < nmem; ++u) {
      const int q = mem[u];
      s = __fma_rn(w[q], P[(long long)q * d + t], s);
    }
    cvals[t] = __dmul_rn(s, inv);
  }
  __syncthreads();
  if (spherical) {
    if (tid == 0) {
      double a = 0.0;
      for (int t = 0; t < d; ++t) a = __fma_rn(cvals[t], cvals[t], a);
      const double nr = __dsqrt_rn(a);
      nrm_sh = nr > 1e-300 ? nr : 1e-300;
    }
    __syncthreads();
    for (int t = tid; t < d; t += kThreads) cvals[t] = __ddiv_rn(cvals[t], nrm_sh);
    __syncthreads();
  }
  for (int t = tid; t < d; t += kThreads) {
    C[(long long)j * d + t] = cvals[t];
    CT[(long long)t * k + j] = cvals[t];
  }
}

// Empty clusters (cnt == 0), in index order, take point floor(u·m) of the next counter draw
// (Spark: points(rand.nextInt(points.length))). ctr persists across iterations. One workgroup.
__global__ __launch_bounds__(kThreads) void local_empty_kernel(const double* __restrict__ P, int m, int d,
                                                               const double* __restrict__ cnt, int k,
                                                               unsigned long long key,
                                                               unsigned long long* __restrict__ ctr,
                                                               double* __restrict__ C, double* __restrict__ CT,
                                                               int* __restrict__ picks, const int* __restrict__ stop) {
  if (stop != nullptr && *stop != 0) return;
  // the empty clusters in index order take consecutive counter draws: a ballot scan over 256 clusters at a
  // time gives each its rank (the same draws as one thread walking the clusters, which took ~20 us)
  __shared__ int wcnt[kThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned long long cc0 = *ctr;
  int ne = 0;  // empties so far (uniform)
  for (int j0 = 0; j0 < k; j0 += kThreads) {
    const int j = j0 + tid;
    const bool empty = j < k && !(cnt[j] > 0.0);
    const unsigned long long b = __ballot(empty);
    if (lane == 0) wcnt[wv] = (int)__popcll(b);
    __syncthreads();
    int off = ne;
    for (int w = 0; w < wv; ++w) off += wcnt[w];
    if (empty) {
      const int e = off + (int)__popcll(b & ((1ull << lane) - 1ull));
      int q = (int)__dmul_rn(cu(cc0 + (unsigned long long)e, key), (double)m);
      q = q < m - 1 ? q : m - 1;
      picks[2 * e] = j;
      picks[2 * e + 1] = q;
    }
    for (int w = 0; w < kThreads / 64; ++w) ne += wcnt[w];
    __syncthreads();  // wcnt reused; picks visible to the whole workgroup
  }
  if (tid == 0) *ctr = cc0 + (unsigned long long)ne;
  for (int e = 0; e < ne; ++e) {
    const int j = picks[2 * e], q = picks[2 * e + 1];
    for (int t = tid; t < d; t += kThreads) {
      const double v = P[(long long)q * d + t];
      C[(long long)j * d + t] = v;
      CT[(long long)t * k + j] = v;
    }
  }
}

// Σ x over f32 values in f64 (the k-means|| Σcost): per-block partials over a fixed block-strided
// split, then one thread adds them in block order — deterministic, and no f64 copy of the 100M costs
// (torch.sum(dtype=float64) cast them first: 0.3 ms + 0.16 ms per round).
constexpr int kSumBlocks = 1024;
__global__ __launch_bounds__(kThreads) void sum_f32_f64_kernel(const float* __restrict__ x, long long n,
                                                               double* __restrict__ part) {
  const long long n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (long long)gridDim.x * kThreads) {
    const float4 v = x4[i];
    s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
  }
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)(n - 4 * n4)) s += (double)x[4 * n4 + threadIdx.x];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double ws[kThreads / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kThreads / 64; ++w) t += ws[w];
    part[blockIdx.x] = t;
  }
}

__global__ void sum_partials_kernel(const double* __restrict__ part, int nb, double* __restrict__ out) {
  double t = 0.0;
  for (int b = 0; b < nb; ++b) t += part[b];
  *out = t;
}

inline unsigned grid_for(long long n, long long per) {
  long long g = (n + per - 1) / per;
  g = g < 1 ? 1 : g;
  return (unsigned)(g > 4096 ? 4096 : g);
}

}  // namespace

// X: bf16 [n, ldx elements] (Dp = 16..512) or e4m3fn [n, ldx bytes] (Dp = 64..1024). c0/cost/near may
// be null together (norms only); xn_max (f32 bits, zero-initialised) and erange (int[2], {INT_MAX, -1}
// initialised) may be null; xn64 (f64 [n], may be null) receives the norms summed in f64 (the per-centre
// Σ|x|² of the training cost: the f32 norms lose ~2^-24·|x|², percents of the cost far from the origin).
CML_API int cml_kmeans_row_pass(const void* X, long long n, long long ldx, int Dp, int xfp8, float* xn,
                                const float* c0, float c0n, float* cost, int* near, unsigned* xn_max, int* erange,
                                double* xn64, const float* c0n_dev, void* stream) {
  if (n < 0 || ((c0 == nullptr) != (cost == nullptr)) || ((cost == nullptr) != (near == nullptr)))
    return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned char* x = (const unsigned char*)X;
  constexpr int U = 2;
  const long long rowb = xfp8 ? (long long)Dp : 2LL * Dp;
  if (xfp8 ? (Dp % 64 != 0 || Dp > 1024 || ldx % 16 != 0) : (Dp % 16 != 0 || Dp > 512 || ldx % 8 != 0))
    return (int)hipErrorInvalidValue;
  const long long ldb = xfp8 ? ldx : 2 * ldx;
#define CML_RP(NCH, CPL, F)                                                                                   \
  hipLaunchKernelGGL((row_pass_kernel<NCH, CPL, F, U>), dim3(grid_for(n, 4LL * (64 / ((NCH) / (CPL))) * U)), \
                     dim3(kThreads), 0, st, x, n, ldb, xn, c0, c0n, cost, near, xn_max, erange, xn64, c0n_dev)
  switch ((int)(rowb / 16) * (xfp8 ? -1 : 1)) {
    case 2: CML_RP(2, 2, false); break;        // bf16 Dp = 16
    case 4: CML_RP(4, 4, false); break;        // 32
    case 8: CML_RP(8, 4, false); break;        // 64
    case 16: CML_RP(16, 4, false); break;      // 128
    case 32: CML_RP(32, 4, false); break;      // 256
    case 64: CML_RP(64, 4, false); break;      // 512
    case -4: CML_RP(4, 4, true); break;        // fp8 Dp = 64
    case -8: CML_RP(8, 4, true); break;        // 128
    case -16: CML_RP(16, 4, true); break;      // 256
    case -32: CML_RP(32, 4, true); break;      // 512
    case -64: CML_RP(64, 4, true); break;      // 1024
    default: return (int)hipErrorInvalidValue;
  }
#undef CML_RP
  return cml_status();
}

// out[0] = Σ_i |x_i - cb[lab[i]]|² in f64 (exact terms, fixed-order sum). X as in cml_kmeans_row_pass;
// cb: bf16 [*, ldc elements] with ldc >= Dp (zero beyond the real columns, as X), 16-byte aligned rows;
// lab: int32 [n], every value a valid row of cb; part: cml_kmeans_cost_parts() doubles of scratch.
CML_API int cml_kmeans_cost_parts() { return 4096; }
CML_API int cml_kmeans_cost_pass(const void* X, long long n, long long ldx, int Dp, int xfp8, const int* lab,
                                 const void* cb, long long ldc, double* part, double* out, void* stream) {
  if (n < 0 || ldc < Dp || ldc % 8 != 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return (int)hipMemsetAsync(out, 0, sizeof(double), st);
  const unsigned char* x = (const unsigned char*)X;
  const u16* c = (const u16*)cb;
  constexpr int U = 2;
  const long long rowb = xfp8 ? (long long)Dp : 2LL * Dp;
  if (xfp8 ? (Dp % 64 != 0 || Dp > 1024 || ldx % 16 != 0) : (Dp % 16 != 0 || Dp > 512 || ldx % 8 != 0))
    return (int)hipErrorInvalidValue;
  const long long ldb = xfp8 ? ldx : 2 * ldx;
  unsigned nb = 0;
#define CML_CP(NCH, CPL, F)                                                                                  \
  nb = grid_for(n, 4LL * (64 / ((NCH) / (CPL))) * U);                                                        \
  hipLaunchKernelGGL((cost_pass_kernel<NCH, CPL, F, U>), dim3(nb), dim3(kThreads), 0, st, x, n, ldb, lab, c, \
                     ldc, part)
  switch ((int)(rowb / 16) * (xfp8 ? -1 : 1)) {
    case 2: CML_CP(2, 2, false); break;
    case 4: CML_CP(4, 4, false); break;
    case 8: CML_CP(8, 4, false); break;
    case 16: CML_CP(16, 4, false); break;
    case 32: CML_CP(32, 4, false); break;
    case 64: CML_CP(64, 4, false); break;
    case -4: CML_CP(4, 4, true); break;
    case -8: CML_CP(8, 4, true); break;
    case -16: CML_CP(16, 4, true); break;
    case -32: CML_CP(32, 4, true); break;
    case -64: CML_CP(64, 4, true); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef CML_CP
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(1), 0, st, part, (int)nb, out);
  return cml_status();
}

// out[0] = Σ x[0:n] in f64; part: scratch of cml_sum_f32_f64_parts() doubles. x 16-byte aligned.
CML_API int cml_sum_f32_f64_parts() { return kSumBlocks; }
CML_API int cml_sum_f32_f64(const float* x, long long n, double* part, double* out, void* stream) {
  if (n < 0 || ((uintptr_t)x & 15)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const long long n4 = n / 4;
  const int nb = (int)std::max<long long>(1, std::min<long long>((n4 + kThreads - 1) / kThreads, kSumBlocks));
  hipLaunchKernelGGL(sum_f32_f64_kernel, dim3(nb), dim3(kThreads), 0, st, x, n, part);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(1), 0, st, part, nb, out);
  return cml_status();
}

CML_API int cml_kmeans_init_merge(float* cost, int* near, const float* best, const int* lab, int off, long long n,
                                  void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(init_merge_kernel, dim3(grid_for(n, kThreads * 4LL)), dim3(kThreads), 0, (hipStream_t)stream,
                     cost, near, best, lab, off, n);
  return cml_status();
}

// count must be zeroed by the caller; at most cap rows are written (count holds the total).
CML_API int cml_kmeans_init_sample(const float* cost, const long long* ids, long long n, unsigned long long key,
                                   double scale, int* out, int* count, long long cap, const double* scale_dev,
                                   void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(init_sample_kernel, dim3(grid_for(n, kThreads * 8LL)), dim3(kThreads), 0, (hipStream_t)stream,
                     cost, ids, n, key, scale, out, count, cap, scale_dev);
  return cml_status();
}

// counts[v] += 1 for every v = vals[i] (0 <= v < m): int32 counts (exact in any order), per-block LDS
// histograms for m <= 8192 merged with one integer atomic per bin and block, global atomics above.
__global__ __launch_bounds__(kThreads) void int_hist_kernel(const int* __restrict__ vals, long long n, int m,
                                                            int* __restrict__ counts) {
  extern __shared__ int hist[];
  const bool lds = m <= 8192;
  if (lds) {
    for (int i = threadIdx.x; i < m; i += kThreads) hist[i] = 0;
    __syncthreads();
  }
  // tiles of 16 values per thread: the 16 loads of a tile are issued before its atomics (one memory round
  // trip per tile; a load-then-atomic loop waited for every value in turn: 69 us for 12.5M labels)
  constexpr int U = 16;
  for (long long t0 = (long long)blockIdx.x * kThreads * U; t0 < n; t0 += (long long)gridDim.x * kThreads * U) {
    int v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = t0 + (long long)u * kThreads + threadIdx.x;
      v[u] = i < n ? vals[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v[u] >= 0 && v[u] < m) {
        if (lds) atomicAdd(&hist[v[u]], 1);
        else atomicAdd(&counts[v[u]], 1);
      }
    }
  }
  if (lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += kThreads)
      if (hist[i]) atomicAdd(&counts[i], hist[i]);
  }
}

// counts: int32 [m], zeroed by the caller.
CML_API int cml_int_hist(const int* vals, long long n, int m, int* counts, void* stream) {
  if (n <= 0) return 0;
  if (m <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = m <= 8192 ? (size_t)m * 4 : 0;
  hipLaunchKernelGGL(int_hist_kernel, dim3(grid_for(n, kThreads * 16LL)), dim3(kThreads), lds, (hipStream_t)stream,
                     vals, n, m, counts);
  return cml_status();
}

// Training cost of an assignment from the sums the step already holds (models/kmeans.py _device_cost):
// out = max(0, Σ_j q_j - 2 c_j·(S_j·unit) + n_j |c_j|²), S / n summed over the `rows` message rows (msg [rows,
// ldm]: S at j*d + t, n at k*d + j), c the bf16 centres [k, ldc]. One workgroup per centre forms its term, a
// second launch adds the k terms; fixed reduction orders (the same bits every run). Replaces a dozen eager
// torch reductions at the end of every fit (one workgroup walking the centres one by one took 0.27 ms).
__device__ __forceinline__ double block_sum256(double v, double* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();  // red reused across calls
  if (lane == 0) red[wv] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void kmeans_cost_terms_kernel(const double* __restrict__ q,
                                                                const double* __restrict__ msg, int rows,
                                                                long long ldm, int k, int d, double unit,
                                                                const unsigned short* __restrict__ cb, int ldc,
                                                                double* __restrict__ term) {
  __shared__ double red[4];
  const int j = blockIdx.x;
  double cs = 0.0, cc = 0.0;
  for (int t = threadIdx.x; t < d; t += 256) {
    double s = 0.0;
    for (int r = 0; r < rows; ++r) s += msg[(long long)r * ldm + (long long)j * d + t];
    const double c = (double)__uint_as_float((unsigned)cb[(long long)j * ldc + t] << 16);
    cs += c * (s * unit);
    cc += c * c;
  }
  cs = block_sum256(cs, red);
  cc = block_sum256(cc, red);
  if (threadIdx.x == 0) {
    double n = 0.0;
    for (int r = 0; r < rows; ++r) n += msg[(long long)r * ldm + (long long)k * d + j];
    term[j] = q[j] - 2.0 * cs + n * cc;
  }
}

__global__ __launch_bounds__(256) void kmeans_cost_sum_kernel(const double* __restrict__ term, int k,
                                                              double* __restrict__ out) {
  __shared__ double red[4];
  double v = 0.0;
  for (int j = threadIdx.x; j < k; j += 256) v += term[j];
  v = block_sum256(v, red);
  if (threadIdx.x == 0) out[0] = v > 0.0 ? v : 0.0;
}

// term: f64 [k] scratch.
CML_API int cml_kmeans_cost_combine(const double* q, const double* msg, int rows, long long ldm, int k, int d,
                                    double unit, const void* cb, int ldc, double* term, double* out, void* stream) {
  if (rows <= 0 || k <= 0 || d <= 0 || ldc < d || ldm < (long long)k * d + k) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(kmeans_cost_terms_kernel, dim3(k), dim3(256), 0, st, q, msg, rows, ldm, k, d, unit,
                     (const unsigned short*)cb, ldc, term);
  hipLaunchKernelGGL(kmeans_cost_sum_kernel, dim3(1), dim3(256), 0, st, term, k, out);
  return cml_status();
}

// P: f64 [m, d] candidates, PT: the same transposed [d, m], w: f64 [m]; C: f64 [k, d], CT: f64 [d, k],
// d2: f64 [m] scratch.
// D: f64 [m, m] scratch for the pairwise distances, or null (then each pick folds its distances from PT).
CML_API int cml_local_kpp(const double* P, const double* PT, int m, int d, const double* w, int k,
                          unsigned long long key, double* C, double* CT, double* d2, double* D, void* stream) {
  if (m <= 0 || d <= 0 || k <= 0 || (long long)d * 8 > 64 * 1024) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (D != nullptr) {
    const unsigned g = (unsigned)((m + kPairT - 1) / kPairT);
    hipLaunchKernelGGL(local_pairdist_kernel, dim3(g, g), dim3(kThreads), 0, st, P, m, d, D);
  }
  const size_t big = ((size_t)d + 2 * (size_t)m) * 8;
  const bool lds_pw = D != nullptr && big <= 150 * 1024;
  const size_t lds = lds_pw ? big : (size_t)d * 8;
  if (lds_pw) hipFuncSetAttribute((const void*)local_kpp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(local_kpp_kernel, dim3(1), dim3(kKppThreads), lds, st, P, PT, D, m, d, w, k, key, C, CT, d2,
                     lds_pw);
  return cml_status();
}

// stop / flags (may be null): int[3] {stop, moved[2]} of the host-sync-free loop (local_update_kernel);
// the assign of iteration i is given moved = flags + 1 + (i & 1) and stop = flags.
CML_API int cml_local_assign(const double* P, int m, int d, const double* CT, int k, int* labels, int* moved,
                             const int* stop, void* stream) {
  if (m <= 0 || (long long)d * 8 > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(local_assign_kernel, dim3(m), dim3(kThreads), (size_t)d * 8, (hipStream_t)stream, P, m, d, CT,
                     k, labels, moved, stop);
  return cml_status();
}

CML_API int cml_local_update(const double* P, int m, int d, const double* w, const int* labels, int k, double* C,
                             double* CT, double* cnt, int spherical, int* flags, int slot, void* stream) {
  const size_t lds = (((size_t)m * 4 + 15) & ~(size_t)15) + (size_t)d * 8;
  if (m <= 0 || lds > 150 * 1024 || slot < 0 || slot > 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(local_update_kernel, dim3(k), dim3(kThreads), lds, (hipStream_t)stream, P, m, d, w, labels, k,
                     C, CT, cnt, spherical, flags, slot);
  return cml_status();
}

// picks: int [2k] scratch.
CML_API int cml_local_empty(const double* P, int m, int d, const double* cnt, int k, unsigned long long key,
                            unsigned long long* ctr, double* C, double* CT, int* picks, const int* stop,
                            void* stream) {
  hipLaunchKernelGGL(local_empty_kernel, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, P, m, d, cnt, k, key, ctr,
                     C, CT, picks, stop);
  return cml_status();
}
