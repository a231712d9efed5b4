// Generalised-linear-model and feature-statistics kernels for gfx950 (MI355X).
//
// K7  col_moments     per-feature count / shifted Σ / shifted Σ² in f64 (StandardScaler,
//                     LinearRegression/LogisticRegression standardization, Summarizer)
// K8  scale_apply     (x - μ)·(1/σ) with optional centring, any in/out dtype (bf16/f32/f64)
// K13 logreg_grad     fused binomial logistic pass: margin = x·w + b, p = σ(margin),
//                     ∇w += (p − y)·x, ∇b += p − y, loss += softplus(margin) − y·margin,
//                     X read ONCE per pass (L-BFGS full batch or an SGD mini-batch); the same
//                     pass with loss LS = 1 is the hinge loss of LinearSVC (labels {0,1} -> ±1,
//                     r = −w·y± where 1 − y±·m > 0) and LS = 2 the squared loss ½(m − y)²
// K13b partial_colsum  fixed-order sum of the per-block partials (device-side, capturable)
// K14 sgd_update      momentum SGD step on the device (mini-batch LogisticRegression)
// K15 gram            [X 1 y]ᵀ[X 1 y] upper triangle in f64 (LinearRegression normal equations)
// K24 linear_predict  ŷ = x·w + b (identity) or σ(x·w + b) (logistic)
//
// Layout: X row-major [n, ld] of T ∈ {bf16, f32, f64}. A wave covers RPW rows at once:
// LPR = 64/RPW lanes per row, each lane CPT contiguous columns (one 16-byte load for bf16/f32,
// two 8-byte f64), NCH column chunks of LPR·CPT. Row dot products reduce over the LPR lanes
// of the row group with xor-shuffles; accumulators are per-lane f64 registers; each block
// writes one partial (fixed summation order => deterministic), reduced afterwards.
#include "common.h"

namespace {

constexpr int kGlmThreads = 256;

// OCP e4m3fn storage (SURVEY config 5): decoded with v_cvt_pk_f32_fp8, computed in f32.
typedef unsigned char f8_t;
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ inline float f8_decode(f8_t b) {
  const f32x2_t a = __builtin_amdgcn_cvt_pk_f32_fp8((int)b, false);
  return a.x;
}
template <typename CT>
__device__ inline void f8_decode16(const uint4 w, CT* v) {
  const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2_t a = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], false);
    const f32x2_t b = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], true);
    v[4 * q] = (CT)a.x;
    v[4 * q + 1] = (CT)a.y;
    v[4 * q + 2] = (CT)b.x;
    v[4 * q + 3] = (CT)b.y;
  }
}

template <typename T> struct Elt;
template <> struct Elt<f8_t> {
  static constexpr int CPT = 16;
  __device__ static inline void load(const f8_t* p, double* v) { f8_decode16<double>(*reinterpret_cast<const uint4*>(p), v); }
};
template <> struct Elt<u16> {
  static constexpr int CPT = 8;
  __device__ static inline void load(const u16* p, double* v) {
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = (double)bf16_to_f32((u16)(ws[q] & 0xffffu));
      v[2 * q + 1] = (double)bf16_to_f32((u16)(ws[q] >> 16));
    }
  }
  __device__ static inline void store(u16* p, const double* v) {
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = f32_to_bf16((float)v[j]);
  }
};
template <> struct Elt<float> {
  static constexpr int CPT = 4;
  __device__ static inline void load(const float* p, double* v) {
    const float4 w = *reinterpret_cast<const float4*>(p);
    v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
  }
  __device__ static inline void store(float* p, const double* v) {
    *reinterpret_cast<float4*>(p) = make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
  }
};
template <> struct Elt<double> {
  static constexpr int CPT = 2;
  __device__ static inline void load(const double* p, double* v) {
    const double2 w = *reinterpret_cast<const double2*>(p);
    v[0] = w.x; v[1] = w.y;
  }
  __device__ static inline void store(double* p, const double* v) {
    *reinterpret_cast<double2*>(p) = make_double2(v[0], v[1]);
  }
};


// ---------------------------------------------------------------------------- row streaming
// Streaming kernels below use one layout: a row is split into 16-byte chunks; LPR lanes (power of
// two) share a row and each owns NCH chunks, chunk k of lane li being row chunk k·LPR + li. One
// load instruction therefore covers LPR·16 contiguous bytes of each of 64/LPR rows (>= 128 B per
// row once LPR >= 8: the full-rate shape on MI355X, profiles/README.md). Compute type CT is f32
// for bf16/f32 data (packed FMAs, v_exp_f32) and f64 for f64 data; every accumulation that
// spans rows is f64.
template <typename T> struct CompT { using type = float; };  // bf16, f32, fp8
template <> struct CompT<double> { using type = double; };

template <typename T, typename CT>
__device__ inline void load_chunk_ct(const T* X, long long row, long long ld, int c0, int d, CT* v) {
  constexpr int CPT = Elt<T>::CPT;
  if (c0 + CPT <= d) {
    if constexpr (sizeof(T) == 1) {
      f8_decode16<CT>(*reinterpret_cast<const uint4*>(X + row * ld + c0), v);
    } else if constexpr (sizeof(T) == 2) {
      const uint4 w = *reinterpret_cast<const uint4*>(X + row * ld + c0);
      const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[2 * q] = __uint_as_float(ws[q] << 16);
        v[2 * q + 1] = __uint_as_float(ws[q] & 0xffff0000u);
      }
    } else if constexpr (sizeof(T) == 4) {
      const float4 w = *reinterpret_cast<const float4*>(X + row * ld + c0);
      v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
    } else {
      const double2 w = *reinterpret_cast<const double2*>(X + row * ld + c0);
      v[0] = w.x; v[1] = w.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      CT t = 0;
      if (c0 + j < d) {
        if constexpr (sizeof(T) == 2) t = bf16_to_f32(((const u16*)X)[row * ld + c0 + j]);
        else if constexpr (sizeof(T) == 1) t = (CT)f8_decode(((const f8_t*)X)[row * ld + c0 + j]);
        else t = (CT)X[row * ld + c0 + j];
      }
      v[j] = t;
    }
  }
}

// Raw 16-byte chunks of one row group (zeros for rows past the end; a lane whose chunk starts at
// or beyond d loads nothing). A chunk straddling d is loaded whole — the row pitch is a multiple
// of 16 bytes (ops/glm_ops._prep) so the load stays inside the row — and decode_group zeroes the
// columns >= d, so padding contents (even NaN) never reach a margin.
template <typename T, int NCH>
__device__ inline void load_raw_group(const T* X, long long row, long long ld, int lpr, int li, int d, bool ok,
                                      uint4 (&raw)[NCH]) {
  constexpr int CPT = Elt<T>::CPT;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int c0 = (c * lpr + li) * CPT;
    raw[c] = (ok && c0 < d) ? *reinterpret_cast<const uint4*>(X + row * ld + c0) : make_uint4(0u, 0u, 0u, 0u);
  }
}

// Branch-free form for K13: a row past n loads row n - 1 (the caller gives it weight 0) and a chunk starting at
// or beyond d loads chunk 0 (decode_group zeroes it). Exec-masked loads made the wait-count pass assume the
// worst at every merge: each use of the previous group's label waited for the next group's rows as well.
template <typename T, int NCH>
__device__ inline void load_raw_group_clamped(const T* X, long long row, long long n, long long ld, int lpr, int li,
                                              int d, uint4 (&raw)[NCH]) {
  constexpr int CPT = Elt<T>::CPT;
  const T* xr = X + (row < n ? row : n - 1) * ld;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int c0 = (c * lpr + li) * CPT;
    raw[c] = *reinterpret_cast<const uint4*>(xr + (c0 < d ? c0 : 0));
  }
}

template <typename T, typename CT, int NCH>
__device__ inline void decode_group(const uint4 (&raw)[NCH], int lpr, int li, int d, CT (&v)[NCH][Elt<T>::CPT]) {
  constexpr int CPT = Elt<T>::CPT;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint4 w = raw[c];
    const unsigned ws[4] = {w.x, w.y, w.z, w.w};
    if constexpr (sizeof(T) == 1) {
      f8_decode16<CT>(w, v[c]);
    } else if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[c][2 * q] = __uint_as_float(ws[q] << 16);
        v[c][2 * q + 1] = __uint_as_float(ws[q] & 0xffff0000u);
      }
    } else if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[c][q] = __uint_as_float(ws[q]);
    } else {
      v[c][0] = __hiloint2double((int)ws[1], (int)ws[0]);
      v[c][1] = __hiloint2double((int)ws[3], (int)ws[2]);
    }
    const int c0 = (c * lpr + li) * CPT;
    if (c0 + CPT > d) {
#pragma unroll
      for (int j = 0; j < CPT; ++j)
        if (c0 + j >= d) v[c][j] = 0;
    }
  }
}

// ---------------------------------------------------------------------------- K7 moments
// Row-streaming layout with the next row group's raw chunks prefetched (as K13). t = x − shift is
// formed in CT (exact for bf16/f32/fp8 data: the shift is a data row, so it is representable),
// Σt and Σt² accumulate in f64. Per-wave column sums go through LDS sized at launch.
template <typename T, int NCH, int U = 1>
__global__ __launch_bounds__(kGlmThreads) void col_moments_kernel(const T* __restrict__ X, long long n, long long ld,
                                                                  int d, int lpr, const double* __restrict__ shift,
                                                                  double* __restrict__ out /*[grid][2][d]*/) {
  using CT = typename CompT<T>::type;
  constexpr int CPT = Elt<T>::CPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  double s1[NCH][CPT], s2[NCH][CPT];
  CT sh[NCH][CPT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      s1[c][j] = 0.0;
      s2[c][j] = 0.0;
      const int col = (c * lpr + li) * CPT + j;
      sh[c][j] = col < d ? (CT)shift[col] : (CT)0;
    }
  const long long step = (long long)gridDim.x * nw * rpw;
  long long row0 = ((long long)blockIdx.x * nw + wave) * rpw;
  // the K13 ring: U groups in flight, U + 1 slots, branch-free loads (rows past n re-read row n - 1 and
  // are skipped below)
  constexpr int S = U + 1;
  uint4 raw[S][NCH];
  if (row0 < n) {
#pragma unroll
    for (int q = 0; q < U; ++q) load_raw_group_clamped<T, NCH>(X, row0 + q * step + sub, n, ld, lpr, li, d, raw[q]);
  }
  for (; row0 < n; row0 += S * step) {
#pragma unroll
    for (int q = 0; q < S; ++q) {
      if (row0 + q * step >= n) break;  // wave-uniform
      const bool ok = row0 + q * step + sub < n;
      CT v[NCH][CPT];
      decode_group<T, CT, NCH>(raw[q], lpr, li, d, v);
      load_raw_group_clamped<T, NCH>(X, row0 + (q + U) * step + sub, n, ld, lpr, li, d, raw[(q + U) % S]);
      if (ok) {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < CPT; ++j) {
            const double t = (double)(v[c][j] - sh[c][j]);
            s1[c][j] += t;
            s2[c][j] = fma(t, t, s2[c][j]);
          }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j)
      for (int o = lpr; o < 64; o <<= 1) {  // sum over the wave's row sub-groups
        s1[c][j] += __shfl_xor(s1[c][j], o, 64);
        s2[c][j] += __shfl_xor(s2[c][j], o, 64);
      }
  extern __shared__ double red_dyn[];
  const int rs = 2 * lpr * CPT;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    __syncthreads();
    if (sub == 0) {
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        red_dyn[wave * rs + (li * CPT + j) * 2] = s1[c][j];
        red_dyn[wave * rs + (li * CPT + j) * 2 + 1] = s2[c][j];
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < lpr * CPT; t += blockDim.x) {
      const int col = c * lpr * CPT + t;
      if (col >= d) continue;
      double a = 0.0, b = 0.0;
      for (int w = 0; w < nw; ++w) {
        a += red_dyn[w * rs + t * 2];
        b += red_dyn[w * rs + t * 2 + 1];
      }
      out[((long long)blockIdx.x * 2) * d + col] = a;
      out[((long long)blockIdx.x * 2 + 1) * d + col] = b;
    }
  }
}

// Sum over the lpr lanes of a row group, result in every lane. f32: the within-16-lane steps are
// DPP lane permutes on the VALU (quad swaps, half-row and row mirrors: each pairs a lane with one
// of the other half, which is all a sum needs), only the 16/32 steps cross rows through the LDS
// crossbar — a chain of five ds_bpermute round trips per row group was the latency floor of the
// margin reduction. f64 keeps the shuffle form.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

template <typename CT>
__device__ inline CT group_sum_ct(CT v, int lpr) {
  if constexpr (sizeof(CT) == 4) {
    if (lpr >= 2) v += dpp_f32<0xB1>(v);   // quad_perm(1,0,3,2)
    if (lpr >= 4) v += dpp_f32<0x4E>(v);   // quad_perm(2,3,0,1)
    if (lpr >= 8) v += dpp_f32<0x141>(v);  // row_half_mirror
    if (lpr >= 16) v += dpp_f32<0x140>(v); // row_mirror
    if (lpr >= 32) v += __shfl_xor(v, 16, 64);
    if (lpr >= 64) v += __shfl_xor(v, 32, 64);
    return v;
  } else {
    for (int o = lpr >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
}

// A lane's share of a row dot product. f32: packed FMAs (v_pk_fma_f32) into two independent 2-wide
// partial sums — half the VALU issue of scalar FMAs and no CPT-long dependency chain (fp8 rows give
// a lane 16 columns per chunk; the scalar chain made K13 VALU-latency bound at 4.1 TB/s).
template <typename CT, int NCH, int CPT>
__device__ inline CT dot_ct(const CT (&v)[NCH][CPT], const CT (&w)[NCH][CPT]) {
  if constexpr (sizeof(CT) == 4 && CPT % 4 == 0) {
    f32x2_t ma = {0.f, 0.f}, mb = {0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < CPT; j += 4) {
        ma = __builtin_elementwise_fma(f32x2_t{v[c][j], v[c][j + 1]}, f32x2_t{w[c][j], w[c][j + 1]}, ma);
        mb = __builtin_elementwise_fma(f32x2_t{v[c][j + 2], v[c][j + 3]}, f32x2_t{w[c][j + 2], w[c][j + 3]}, mb);
      }
    return (ma.x + mb.x) + (ma.y + mb.y);
  } else {
    CT m = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < CPT; ++j) m = fma(v[c][j], w[c][j], m);
    return m;
  }
}

// f32 row math on the transcendental unit: v_exp_f32, v_log_f32 (base 2) and v_rcp_f32 (1 ulp). The IEEE
// division and the denormal-safe log expansion were ~16 of the ~130 VALU ops per row group of the fp8 K13
// pass, which issues VALU on ~65% of SIMD cycles (profiles/r6/lr_pmc/).
__device__ inline float sigmoid_ct(float m) { return __builtin_amdgcn_rcpf(1.f + __expf(-m)); }
__device__ inline double sigmoid_ct(double m) {
  const double e = exp(-fabs(m));
  return m >= 0 ? 1.0 / (1.0 + e) : e / (1.0 + e);
}
__device__ inline float softplus_ct(float m) {
  return fmaxf(m, 0.f) + 0.693147180559945f * __builtin_amdgcn_logf(1.f + __expf(-fabsf(m)));  // arg in [1, 2]
}
__device__ inline double softplus_ct(double m) { return fmax(m, 0.0) + log1p(exp(-fabs(m))); }

// ---------------------------------------------------------------------------- K8 scale
// (The K13 branch-free loads measured slower here: bf16 -> e4m3 at 50M x 512 5.32 -> 5.06 TB/s, r6.)
template <typename TI, typename TO, int NCH>
__global__ __launch_bounds__(kGlmThreads) void scale_apply_kernel(const TI* __restrict__ X, long long n, long long ldx,
                                                                  int d, int lpr, const double* __restrict__ mean,
                                                                  const double* __restrict__ inv_std, int with_mean,
                                                                  TO* __restrict__ Y, long long ldy, int dpad) {
  using CT = typename CompT<TO>::type;
  constexpr int CPT = Elt<TI>::CPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  CT mu[NCH][CPT], is[NCH][CPT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int col = (c * lpr + li) * CPT + j;
      mu[c][j] = (col < d && with_mean) ? (CT)mean[col] : (CT)0;
      is[c][j] = col < d ? (CT)inv_std[col] : (CT)0;
    }
  const long long step = (long long)gridDim.x * nw * rpw;
  const bool vec_ok = ((ldy * (long long)sizeof(TO)) % 16 == 0) && ((reinterpret_cast<size_t>(Y) & 15) == 0);
  // f64 input into a narrower output is scaled in f64, then rounded once
  using CD = typename std::conditional<sizeof(TI) == 8, double, CT>::type;
  long long row0 = ((long long)blockIdx.x * nw + wave) * rpw;
  uint4 raw[NCH];
  if (row0 < n) load_raw_group<TI, NCH>(X, row0 + sub, ldx, lpr, li, d, row0 + sub < n, raw);
  for (; row0 < n; row0 += step) {
    const long long row = row0 + sub;
    CD t[NCH][CPT];
    decode_group<TI, CD, NCH>(raw, lpr, li, d, t);
    load_raw_group<TI, NCH>(X, row + step, ldx, lpr, li, d, row + step < n, raw);  // prefetch
    if (row >= n) continue;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int c0 = (c * lpr + li) * CPT;
      if (c0 >= dpad) continue;
      CT v[CPT];
#pragma unroll
      for (int j = 0; j < CPT; ++j) v[j] = (CT)((t[c][j] - (CD)mu[c][j]) * (CD)is[c][j]);
      TO* yp = Y + row * ldy + c0;
      const bool full = vec_ok && c0 + CPT <= dpad;
      if constexpr (sizeof(TO) == 1) {  // OCP e4m3fn output, saturated to +-448, packed 4 per word
        constexpr int NW = (CPT + 3) / 4;
        unsigned w[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) w[q] = 0u;
#pragma unroll
        for (int j = 0; j < CPT; j += 2) {
          const float a0 = fminf(fmaxf((float)v[j], -448.f), 448.f);
          const float a1 = j + 1 < CPT ? fminf(fmaxf((float)v[j + 1], -448.f), 448.f) : 0.f;
          const unsigned pk = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false) & 0xffffu;
          w[j / 4] |= pk << (8 * (j % 4));
        }
        if (full) {
          if constexpr (CPT == 16) *reinterpret_cast<uint4*>(yp) = make_uint4(w[0], w[1], w[2], w[3]);
          else if constexpr (CPT == 8) *reinterpret_cast<uint2*>(yp) = make_uint2(w[0], w[1]);
          else if constexpr (CPT == 4) *reinterpret_cast<unsigned*>(yp) = w[0];
          else *reinterpret_cast<u16*>(yp) = (u16)w[0];
        } else {
          for (int j = 0; c0 + j < dpad && j < CPT; ++j) ((unsigned char*)yp)[j] = (unsigned char)(w[j / 4] >> (8 * (j % 4)));
        }
      } else if (full) {
        if constexpr (sizeof(TO) == 2) {
          unsigned w[(CPT + 1) / 2];
#pragma unroll
          for (int q = 0; q < CPT / 2; ++q)
            w[q] = (unsigned)f32_to_bf16((float)v[2 * q]) | ((unsigned)f32_to_bf16((float)v[2 * q + 1]) << 16);
          if constexpr (CPT == 16) {
            *reinterpret_cast<uint4*>(yp) = make_uint4(w[0], w[1], w[2], w[3]);
            *reinterpret_cast<uint4*>(yp + 8) = make_uint4(w[4], w[5], w[6], w[7]);
          } else if constexpr (CPT == 8) {
            *reinterpret_cast<uint4*>(yp) = make_uint4(w[0], w[1], w[2], w[3]);
          } else if constexpr (CPT == 4) {
            *reinterpret_cast<uint2*>(yp) = make_uint2(w[0], w[1]);
          } else {
            *reinterpret_cast<unsigned*>(yp) = w[0];
          }
        } else {
#pragma unroll
          for (int j = 0; j < CPT; ++j) yp[j] = (TO)v[j];
        }
      } else {
        for (int j = 0; c0 + j < dpad && j < CPT; ++j) {
          if constexpr (sizeof(TO) == 2) ((u16*)yp)[j] = f32_to_bf16((float)v[j]);
          else yp[j] = (TO)v[j];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- K13 logistic gradient
// Per row group: margin m = x·w + b (CT), p = σ(m), r = wt·(p − y); the lane's chunk of r·x goes
// into CT accumulators that are folded into f64 every FLUSH rows; loss and weights in f64.
template <typename T, int NCH, int U, int LS = 0>
__global__ __launch_bounds__(kGlmThreads) void logreg_grad_kernel(
    const T* __restrict__ X, long long n, long long ld, int d, int lpr, const double* __restrict__ y,
    const double* __restrict__ wt, const double* __restrict__ coef /*[d+1], last = intercept*/,
    double* __restrict__ out /*[grid][d + 3]: grad (d), grad_b, loss, weight sum*/,
    const long long* __restrict__ row_base /*optional device row offset: a graph-captured SGD step
                                              reads its mini-batch position at run time*/) {
  using CT = typename CompT<T>::type;
  if (row_base != nullptr) {
    const long long b0 = *row_base;
    X += b0 * ld;
    y += b0;
    if (wt != nullptr) wt += b0;
  }
  constexpr int CPT = Elt<T>::CPT;
  constexpr int FLUSH = 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  CT w[NCH][CPT], g[NCH][CPT];
  double g64[NCH][CPT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int col = (c * lpr + li) * CPT + j;
      w[c][j] = col < d ? (CT)coef[col] : (CT)0;
      g[c][j] = 0;
      g64[c][j] = 0.0;
    }
  const CT b = (CT)coef[d];
  double gb = 0.0, loss = 0.0, wsum = 0.0;
  CT gbc = 0, lossc = 0, wsumc = 0;  // f32 data: per-row scalars in f32, folded into f64 with the gradient
  const long long step = (long long)gridDim.x * nw * rpw;
  // Software pipeline: the raw 16-byte chunks, labels and weights of the wave's next U row groups are in
  // flight while the current one is decoded and reduced. The ring has U + 1 slots and the step loop is
  // unrolled over all of them, so the slot a step refills is never the one it reads: with U slots (the r4
  // form) the refill of the slot being read needed a second register set and a copy on the back edge, and
  // the copy waited for every load in flight, the ring's other groups included. Loads are branch-free
  // (load_raw_group_clamped, labels of rows past n read row n - 1): exec-masked loads made the wait-count
  // pass assume the worst at every merge. A slot costs NCH·4 + 4 VGPRs.
  constexpr int S = U + 1;
  int since = 0;
  long long row0 = ((long long)blockIdx.x * nw + wave) * rpw;
  uint4 raw[S][NCH];
  double yn[S], wn[S];
  const double* wsrc = wt != nullptr ? wt : y;  // no weight column: a valid address, wi = 1 where it is read
#pragma unroll
  for (int q = 0; q < U; ++q) {
    if (n <= 0) break;  // an empty shard reads nothing (row n - 1 does not exist); the partials stay zero
    const long long row = row0 + q * step + sub;
    const long long crow = row < n ? row : n - 1;
    load_raw_group_clamped<T, NCH>(X, row, n, ld, lpr, li, d, raw[q]);
    yn[q] = y[crow];
    wn[q] = wsrc[crow];
  }
  for (; row0 < n; row0 += S * step) {
#pragma unroll
    for (int q = 0; q < S; ++q) {
      if (row0 + q * step >= n) break;  // wave-uniform
      const int ps = (q + U) % S;  // the slot read one step ago
      CT v[NCH][CPT];
      decode_group<T, CT, NCH>(raw[q], lpr, li, d, v);
      {
        const long long nrow = row0 + (q + U) * step + sub;
        const long long crow = nrow < n ? nrow : n - 1;
        load_raw_group_clamped<T, NCH>(X, nrow, n, ld, lpr, li, d, raw[ps]);
        yn[ps] = y[crow];
        wn[ps] = wsrc[crow];
      }
      const double yi = yn[q], wi = row0 + q * step + sub < n ? (wt != nullptr ? wn[q] : 1.0) : 0.0;
      CT m = dot_ct<CT, NCH, CPT>(v, w);
      m = group_sum_ct<CT>(m, lpr) + b;
      CT r;
      CT lrow;
      if constexpr (LS == 0) {  // logistic
        r = (CT)wi * (sigmoid_ct(m) - (CT)yi);
        lrow = softplus_ct(m) - (CT)yi * m;
      } else if constexpr (LS == 1) {  // hinge, labels {0, 1}
        const CT ys = yi > 0.5 ? (CT)1 : (CT)-1;
        const CT t = (CT)1 - ys * m;
        r = t > (CT)0 ? -(CT)wi * ys : (CT)0;
        lrow = t > (CT)0 ? t : (CT)0;
      } else {  // squared
        const CT e = m - (CT)yi;
        r = (CT)wi * e;
        lrow = (CT)0.5 * e * e;
      }
      if constexpr (sizeof(CT) == 4 && CPT % 2 == 0) {
        const f32x2_t r2 = {r, r};
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < CPT; j += 2) {
            const f32x2_t gg = __builtin_elementwise_fma(r2, f32x2_t{v[c][j], v[c][j + 1]},
                                                         f32x2_t{g[c][j], g[c][j + 1]});
            g[c][j] = gg.x;
            g[c][j + 1] = gg.y;
          }
      } else {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < CPT; ++j) g[c][j] = fma(r, v[c][j], g[c][j]);
      }
      // every lane of the row group adds the row's scalars (no li == 0 select: 6 cndmasks); the totals are
      // scaled by 1/lpr at the end, which is exact (power of two, and the lpr copies sum exactly first)
      gbc += r;
      lossc = fma((CT)wi, lrow, lossc);
      wsumc += (CT)wi;
      if constexpr (sizeof(CT) == 4) {
        if (++since >= FLUSH) {
          since = 0;
          gb += (double)gbc;
          loss += (double)lossc;
          wsum += (double)wsumc;
          gbc = lossc = wsumc = 0;
#pragma unroll
          for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int j = 0; j < CPT; ++j) {
              g64[c][j] += (double)g[c][j];
              g[c][j] = 0;
            }
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j) g64[c][j] += (double)g[c][j];
  gb += (double)gbc;
  loss += (double)lossc;
  wsum += (double)wsumc;
  // reduce across row sub-groups, then across waves
  // per-wave rows of lpr·CPT column sums + 3 scalars, sized at launch (logreg_lds_bytes): a fixed
  // fp8-sized buffer (33 KB) would cap residency at 4 blocks per CU for every dtype
  extern __shared__ double red_dyn[];
  const int rs = lpr * CPT + 3;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j)
      for (int o = lpr; o < 64; o <<= 1) g64[c][j] += __shfl_xor(g64[c][j], o, 64);
  for (int o = 1; o < 64; o <<= 1) {
    gb += __shfl_xor(gb, o, 64);
    loss += __shfl_xor(loss, o, 64);
    wsum += __shfl_xor(wsum, o, 64);
  }
  {
    const double il = 1.0 / (double)lpr;
    gb *= il;
    loss *= il;
    wsum *= il;
  }
  double* o_ = out + (long long)blockIdx.x * (d + 3);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    __syncthreads();
    if (sub == 0)
#pragma unroll
      for (int j = 0; j < CPT; ++j) red_dyn[wave * rs + li * CPT + j] = g64[c][j];
    if (lane == 0 && c == 0) {
      red_dyn[wave * rs + rs - 3] = gb;
      red_dyn[wave * rs + rs - 2] = loss;
      red_dyn[wave * rs + rs - 1] = wsum;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < lpr * CPT; t += blockDim.x) {
      const int col = c * lpr * CPT + t;
      if (col >= d) continue;
      double a = 0.0;
      for (int ww = 0; ww < nw; ++ww) a += red_dyn[ww * rs + t];
      o_[col] = a;
    }
    if (c == 0 && threadIdx.x < 3) {
      double a = 0.0;
      for (int ww = 0; ww < nw; ++ww) a += red_dyn[ww * rs + rs - 3 + threadIdx.x];
      o_[d + threadIdx.x] = a;
    }
  }
}

// ---------------------------------------------------------------------------- K13m multinomial gradient
// LogisticRegression family="multinomial" (SURVEY K13 "multinomial C×D variant"): ONE pass over X per
// objective evaluation, no f64 copy of it. Per row group (LPR lanes share a row, each NCH 16-byte chunks of
// CPT columns): the C margins m_c = x·w_c + b_c (lane shares reduced over the row's lanes), the row's
// log-sum-exp, loss += wt·(lse − m_y), r_c = wt·(softmax_c − [c = y]) and ∇w_c += r_c·x. The lane's
// columns of the CP weight rows and CP gradient rows live in VGPRs (CT: f32 for bf16/f32/fp8 rows, f64
// for f64 rows); class slots c >= C are dead (margin -inf, no gradient). Every FLUSH groups the f32
// gradients are summed over the wave's row sub-groups (xor shuffles) and added into the wave's own f64
// image of the C×d gradient in LDS; at the end the block sums its waves' images in wave order into its
// partial [C·d | C | loss | weight] (K13b adds the partials in a fixed order: deterministic).
template <typename T, int NCH, int CP>
__global__ __launch_bounds__(kGlmThreads) void multinomial_grad_kernel(
    const T* __restrict__ X, long long n, long long ld, int d, int lpr, int C, const double* __restrict__ y,
    const double* __restrict__ wt, const double* __restrict__ coef /*[C][d+1], last column = intercepts*/,
    double* __restrict__ out /*[grid][C·d + C + 2]*/) {
  using CT = typename CompT<T>::type;
  constexpr int CPT = Elt<T>::CPT;
  constexpr int FLUSH = 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  const int dpad = lpr * NCH * CPT;
  extern __shared__ double mimg[];  // [nw][CP][dpad] f64 gradient images, then [nw][CP + 2] scalars
  double* img = mimg + (long long)wave * CP * dpad;
  for (int i = lane; i < CP * dpad; i += 64) img[i] = 0.0;
  CT w[CP][NCH][CPT], g[CP][NCH][CPT];
  CT b[CP];
#pragma unroll
  for (int k = 0; k < CP; ++k) {
    b[k] = k < C ? (CT)coef[(long long)k * (d + 1) + d] : (CT)0;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int col = (c * lpr + li) * CPT + j;
        w[k][c][j] = (k < C && col < d) ? (CT)coef[(long long)k * (d + 1) + col] : (CT)0;
        g[k][c][j] = 0;
      }
  }
  double gb[CP];
#pragma unroll
  for (int k = 0; k < CP; ++k) gb[k] = 0.0;
  double loss = 0.0, wsum = 0.0;
  // flush: sub-group sums of the f32 gradients into the wave's f64 image (sub-group 0 writes)
  auto flush = [&]() {
#pragma unroll
    for (int k = 0; k < CP; ++k)
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
          CT v = g[k][c][j];
          for (int o = lpr; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
          if (sub == 0 && k < C) img[k * dpad + (c * lpr + li) * CPT + j] += (double)v;
          g[k][c][j] = 0;
        }
  };
  const long long step = (long long)gridDim.x * nw * rpw;
  int since = 0;
  long long row0 = ((long long)blockIdx.x * nw + wave) * rpw;
  uint4 raw[NCH];
  double yn, wn;
  {
    const long long row = row0 + sub;
    const bool ok = row < n;
    load_raw_group<T, NCH>(X, row, ld, lpr, li, d, ok, raw);
    yn = ok ? y[row] : 0.0;
    wn = ok ? (wt != nullptr ? wt[row] : 1.0) : 0.0;
  }
  for (; row0 < n; row0 += step) {
    CT v[NCH][CPT];
    decode_group<T, CT, NCH>(raw, lpr, li, d, v);
    const double yi = yn, wi = wn;
    {
      const long long row = row0 + step + sub;
      const bool ok = row < n;
      load_raw_group<T, NCH>(X, row, ld, lpr, li, d, ok, raw);
      yn = ok ? y[row] : 0.0;
      wn = ok ? (wt != nullptr ? wt[row] : 1.0) : 0.0;
    }
    CT m[CP];
    CT mx = -__builtin_huge_valf();
#pragma unroll
    for (int k = 0; k < CP; ++k) {
      m[k] = group_sum_ct<CT>(dot_ct<CT, NCH, CPT>(v, w[k]), lpr) + b[k];
      if (k < C) mx = m[k] > mx ? m[k] : mx;
    }
    CT se = 0;
    CT e[CP];
#pragma unroll
    for (int k = 0; k < CP; ++k) {
      if constexpr (sizeof(CT) == 4) e[k] = k < C ? __expf(m[k] - mx) : 0.f;
      else e[k] = k < C ? exp(m[k] - mx) : 0.0;
      se += e[k];
    }
    const int yc = (int)yi;
    const CT inv = (CT)1 / se;
    CT my = 0;
#pragma unroll
    for (int k = 0; k < CP; ++k) {
      my = k == yc ? m[k] : my;
      const CT r = (CT)wi * (e[k] * inv - (k == yc ? (CT)1 : (CT)0));
      if (k < C) {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int j = 0; j < CPT; ++j) g[k][c][j] = fma(r, v[c][j], g[k][c][j]);
        if (li == 0) gb[k] += (double)r;
      }
    }
    if (li == 0) {
      double lse;
      if constexpr (sizeof(CT) == 4) lse = (double)mx + (double)__logf(se);
      else lse = mx + log(se);
      loss += wi * (lse - (double)my);
      wsum += wi;
    }
    if (++since >= FLUSH) {
      since = 0;
      flush();
    }
  }
  flush();
  // wave scalars -> LDS, then the block's partial in wave order
  double* scal = mimg + (long long)nw * CP * dpad;
#pragma unroll
  for (int k = 0; k < CP; ++k) gb[k] = wave_sum_f64(gb[k]);
  loss = wave_sum_f64(loss);
  wsum = wave_sum_f64(wsum);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < CP; ++k) scal[wave * (CP + 2) + k] = gb[k];
    scal[wave * (CP + 2) + CP] = loss;
    scal[wave * (CP + 2) + CP + 1] = wsum;
  }
  __syncthreads();
  const int m_out = C * d + C + 2;
  double* o_ = out + (long long)blockIdx.x * m_out;
  for (int t = threadIdx.x; t < C * d; t += blockDim.x) {
    const int k = t / d, col = t - k * d;
    double a = 0.0;
    for (int ww = 0; ww < nw; ++ww) a += mimg[(long long)ww * CP * dpad + k * dpad + col];
    o_[t] = a;
  }
  for (int t = threadIdx.x; t < C + 2; t += blockDim.x) {
    const int q = t < C ? t : CP + (t - C);
    double a = 0.0;
    for (int ww = 0; ww < nw; ++ww) a += scal[ww * (CP + 2) + q];
    o_[C * d + t] = a;
  }
}

// ---------------------------------------------------------------------------- K13b / K14 SGD step
// K13b partial_colsum: msg[j] = Σ_b part[b][j] over the grid's per-block partials in a fixed order:
// a block owns 16 columns (128-byte row segments) and 64 row slices; slice sums are combined in
// slice order in LDS. Deterministic, no atomics; ~17 blocks for d = 256 — one short latency chain
// per thread (a device-scope fence + arrival-counter two-level version measured 3x slower: the
// release fence writes back L2).
// K14 sgd_update: the mini-batch optimizer step on the device — g = msg/Σw ⊙ gscale (+ L2 on w),
// vel = μ·vel − lr·g, coef += vel, eff = coef ⊙ kscale (the coefficients the next K13 reads),
// loss_acc += loss/Σw, base = (base + batch) mod wrap. With K13 and K13b (plus the RCCL all-reduce
// of msg when there are several ranks) one SGD step is 3 kernels, none of which the host waits on.
constexpr int kColsumCols = 16, kColsumSlices = 64;

__global__ __launch_bounds__(kColsumCols* kColsumSlices) void partial_colsum_kernel(const double* __restrict__ part,
                                                                                   int nb, int m,
                                                                                   double* __restrict__ msg) {
  __shared__ double red[kColsumSlices][kColsumCols + 1];
  const int c = threadIdx.x % kColsumCols, sl = threadIdx.x / kColsumCols;
  const int col = blockIdx.x * kColsumCols + c;
  double a = 0.0;
  if (col < m) {
#pragma unroll 4
    for (int b = sl; b < nb; b += kColsumSlices) a += part[(long long)b * m + col];
  }
  red[sl][c] = a;
  __syncthreads();
  if (sl == 0 && col < m) {
    double t = 0.0;
    for (int q = 0; q < kColsumSlices; ++q) t += red[q][c];
    msg[col] = t;
  }
}

__global__ __launch_bounds__(256) void sgd_update_kernel(const double* __restrict__ msg, int d, double* __restrict__ coef,
                                                         double* __restrict__ vel, double* __restrict__ eff,
                                                         const double* __restrict__ lr, double mom, double l2,
                                                         int fit_intercept, const double* __restrict__ gscale,
                                                         const double* __restrict__ kscale,
                                                         double* __restrict__ loss_acc, long long* __restrict__ base,
                                                         long long batch, long long wrap) {
  const double wsum = fmax(msg[d + 2], 1e-300);
  const double rate = *lr;
  for (int j = threadIdx.x; j <= d; j += blockDim.x) {
    double g = msg[j] / wsum;
    if (gscale != nullptr) g = g * gscale[j];
    if (j < d) {
      if (l2 > 0.0) g = g + l2 * coef[j];
    } else if (!fit_intercept) {
      g = 0.0;
    }
    const double v = vel[j] * mom - g * rate;
    vel[j] = v;
    const double c = coef[j] + v;
    coef[j] = c;
    eff[j] = kscale != nullptr ? c * kscale[j] : c;
  }
  if (threadIdx.x == 0) {
    *loss_acc += msg[d + 1] / wsum;
    *base = (*base + batch) % wrap;
  }
}

// ---------------------------------------------------------------------------- K24 predict
template <typename T, int NCH>
__global__ __launch_bounds__(kGlmThreads) void linear_predict_kernel(const T* __restrict__ X, long long n,
                                                                     long long ld, int d, int lpr,
                                                                     const double* __restrict__ coef, int link,
                                                                     double* __restrict__ out) {
  using CT = typename CompT<T>::type;
  constexpr int CPT = Elt<T>::CPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  CT w[NCH][CPT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int col = (c * lpr + li) * CPT + j;
      w[c][j] = col < d ? (CT)coef[col] : (CT)0;
    }
  const double b = coef[d];
  const long long step = (long long)gridDim.x * nw * rpw;
  long long row0 = ((long long)blockIdx.x * nw + wave) * rpw;
  uint4 raw[NCH];
  if (row0 < n) load_raw_group<T, NCH>(X, row0 + sub, ld, lpr, li, d, row0 + sub < n, raw);
  for (; row0 < n; row0 += step) {
    const long long row = row0 + sub;
    const bool ok = row < n;
    CT v[NCH][CPT];
    decode_group<T, CT, NCH>(raw, lpr, li, d, v);
    load_raw_group<T, NCH>(X, row + step, ld, lpr, li, d, row + step < n, raw);  // prefetch
    const CT m = dot_ct<CT, NCH, CPT>(v, w);
    const double mm = (double)group_sum_ct<CT>(m, lpr) + b;
    if (ok && li == 0) out[row] = link == 1 ? sigmoid_ct(mm) : mm;
  }
}

// ---------------------------------------------------------------------------- K15 gram
// One thread per (i, j) pair of the (d+2)×(d+2) upper triangle over a row block; rows of
// the block are staged through LDS in tiles so X is read once per block from HBM.
template <typename T>
__global__ __launch_bounds__(256) void gram_kernel(const T* __restrict__ X, long long n, long long ld, int d,
                                                   const double* __restrict__ y, const double* __restrict__ wt,
                                                   double* __restrict__ out /*[grid][m*m]*/) {
  constexpr int TILE = 64;
  const int m = d + 2;
  __shared__ double tile[TILE][33];  // supports d <= 30 (m <= 32, one (i,j) pair per thread slot)
  const long long rows_per_block = (n + gridDim.x - 1) / gridDim.x;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  const int npair = m * m;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (long long t0 = r0; t0 < r1; t0 += TILE) {
    __syncthreads();
    for (int e = threadIdx.x; e < TILE * m; e += blockDim.x) {
      const int rr = e / m, cc = e - rr * m;
      const long long row = t0 + rr;
      double v = 0.0;
      if (row < r1) {
        const double sw = wt != nullptr ? sqrt(wt[row]) : 1.0;
        if (cc < d) {
          if constexpr (sizeof(T) == 2) v = (double)bf16_to_f32(((const u16*)X)[row * ld + cc]);
          else if constexpr (sizeof(T) == 1) v = (double)f8_decode(((const f8_t*)X)[row * ld + cc]);
          else v = (double)X[row * ld + cc];
        } else if (cc == d) {
          v = 1.0;
        } else {
          v = y[row];
        }
        v *= sw;
      }
      tile[rr][cc] = v;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = threadIdx.x + q * blockDim.x;
      if (p >= npair) continue;
      const int i = p / m, j = p - i * m;
      if (j < i) continue;
      double s = 0.0;
      for (int rr = 0; rr < TILE; ++rr) s = fma(tile[rr][i], tile[rr][j], s);
      acc[q] += s;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = threadIdx.x + q * blockDim.x;
    if (p < npair) out[(long long)blockIdx.x * npair + p] = acc[q];
  }
}

// Small Gram (m = d + 2 <= 8, e.g. the reference's 4 features): one row per lane, the upper
// triangle of a·aᵀ (a = √w·[x 1 y]) in m(m+1)/2 f64 registers, rows streamed straight from HBM;
// lanes then waves reduced once per block.
template <typename T, int M>
__global__ __launch_bounds__(256) void gram_small_kernel(const T* __restrict__ X, long long n, long long ld, int d,
                                                         const double* __restrict__ y,
                                                         const double* __restrict__ wt,
                                                         double* __restrict__ out /*[grid][M*M]*/) {
  constexpr int NP = M * (M + 1) / 2;
  double acc[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) acc[q] = 0.0;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < n;
       row += (long long)gridDim.x * blockDim.x) {
    double a[M];
    const double sw = wt != nullptr ? sqrt(wt[row]) : 1.0;
#pragma unroll
    for (int j = 0; j < M - 2; ++j) {
      double v;
      if constexpr (sizeof(T) == 2) v = (double)bf16_to_f32(((const u16*)X)[row * ld + j]);
      else if constexpr (sizeof(T) == 1) v = (double)f8_decode(((const f8_t*)X)[row * ld + j]);
      else v = (double)X[row * ld + j];
      a[j] = v * sw;
    }
    a[M - 2] = sw;
    a[M - 1] = y[row] * sw;
    int q = 0;
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = i; j < M; ++j) acc[q++] = fma(a[i], a[j], acc[q]);
  }
  __shared__ double red[256 / 64][NP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const double t = wave_sum_f64(acc[q]);
    if (lane == 0) red[wave][q] = t;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NP; q += blockDim.x) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w][q];
    int i = 0, rem = q;
    while (rem >= M - i) { rem -= M - i; ++i; }
    out[(long long)blockIdx.x * M * M + i * M + (i + rem)] = t;
  }
}

template <typename T>
int launch_gram_small(const void* X, long long n, long long ld, int d, const double* y, const double* wt,
                      double* out, int grid, hipStream_t st) {
  const T* x = (const T*)X;
  switch (d + 2) {
    case 2: hipLaunchKernelGGL((gram_small_kernel<T, 2>), dim3(grid), dim3(256), 0, st, x, n, ld, d, y, wt, out); break;
    case 3: hipLaunchKernelGGL((gram_small_kernel<T, 3>), dim3(grid), dim3(256), 0, st, x, n, ld, d, y, wt, out); break;
    case 4: hipLaunchKernelGGL((gram_small_kernel<T, 4>), dim3(grid), dim3(256), 0, st, x, n, ld, d, y, wt, out); break;
    case 5: hipLaunchKernelGGL((gram_small_kernel<T, 5>), dim3(grid), dim3(256), 0, st, x, n, ld, d, y, wt, out); break;
    case 6: hipLaunchKernelGGL((gram_small_kernel<T, 6>), dim3(grid), dim3(256), 0, st, x, n, ld, d, y, wt, out); break;
    case 7: hipLaunchKernelGGL((gram_small_kernel<T, 7>), dim3(grid), dim3(256), 0, st, x, n, ld, d, y, wt, out); break;
    case 8: hipLaunchKernelGGL((gram_small_kernel<T, 8>), dim3(grid), dim3(256), 0, st, x, n, ld, d, y, wt, out); break;
    default: return (int)hipErrorInvalidValue;
  }
  return cml_status();
}

// Streaming layout choice: ~16 columns per lane, power-of-two lanes per row.
inline int pow2ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}
int g_fp8_nch = 0;  // ablation: chunks per lane of the fp8 (16 values / chunk) streaming layout, 0 = auto

inline bool stream_layout(int d, int cpt, int& lpr, int& nch) {
  const int ch = (d + cpt - 1) / cpt;
  // two 16-B chunks per lane for bf16 and fp8 alike: fp8 x 512 at one chunk per lane kept too few bytes in
  // flight (K13 4.14 -> 5.09 TB/s, K24 5.12 -> 5.80 TB/s at two; four spill: profiles/r4/glm_fp8_layout.log)
  int want = cpt >= 16 ? 2 : (16 / cpt > 0 ? 16 / cpt : 1);
  if (cpt == 16 && g_fp8_nch > 0) want = g_fp8_nch;
  nch = ch < want ? pow2ceil(ch) : want;
  lpr = pow2ceil((ch + nch - 1) / nch);
  if (lpr > 64) {
    lpr = 64;
    nch = pow2ceil((ch + 63) / 64);
  }
  return nch <= 8;
}

int pick_lpr(int d, int cpt, int nch) {
  int need = (d + cpt * nch - 1) / (cpt * nch);
  int l = 1;
  while (l < need) l <<= 1;
  return l > 64 ? 64 : l;
}

int pick_nch(int d, int cpt) {
  const int per = 64 * cpt;
  int nch = (d + per - 1) / per;
  if (nch <= 1) return 1;
  if (nch <= 2) return 2;
  if (nch <= 4) return 4;
  if (nch <= 8) return 8;
  return -1;
}

int grid_for(long long n, int rows_per_block_iter, int cap) {
  long long g = (n + rows_per_block_iter - 1) / rows_per_block_iter;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

}  // namespace

// dtype codes: 0 = bf16, 1 = f32, 2 = f64
#define CML_T_SWITCH(code, BODY)              \
  switch (code) {                             \
    case 0: { using T = u16; BODY; } break;   \
    case 1: { using T = float; BODY; } break; \
    case 2: { using T = double; BODY; } break;\
    case 3: { using T = f8_t; BODY; } break;  \
    default: return (int)hipErrorInvalidValue;\
  }

#define CML_NCH_SWITCH(nch, BODY)                     \
  switch (nch) {                                      \
    case 1: { constexpr int NCH = 1; BODY; } break;   \
    case 2: { constexpr int NCH = 2; BODY; } break;   \
    case 4: { constexpr int NCH = 4; BODY; } break;   \
    case 8: { constexpr int NCH = 8; BODY; } break;   \
    default: return (int)hipErrorInvalidValue;        \
  }

int g_logreg_unroll = 0;  // 0 = auto, else forced prefetch depth U (ablation: cml_glm_set_logreg_unroll)

int logreg_unroll(int nch, int cpt) {
  if (g_logreg_unroll == 1 || g_logreg_unroll == 2 || g_logreg_unroll == 4) return g_logreg_unroll;
  // fp8 rows: two groups ahead (50M x 512: 5.08 -> 5.49 TB/s, profiles/r6/k13_ring/); bf16 / f32 rows: one
  // (U = 2: 6.06 -> 5.91 bf16, 6.01 -> 5.46 f32). The r4 ring of U slots was slower at every U > 1
  // (profiles/logreg_prefetch_depth.log): its back-edge copy waited for the whole ring.
  (void)nch;
  return cpt == 16 ? 2 : 1;
}

#define CML_U_SWITCH(u, BODY)                                          \
  if ((u) == 4) { constexpr int U = 4; BODY; }                         \
  else if ((u) == 2) { constexpr int U = 2; BODY; } else { constexpr int U = 1; BODY; }

size_t moments_lds_bytes(int lpr, int cpt) { return (size_t)(kGlmThreads / 64) * 2 * lpr * cpt * sizeof(double); }
size_t logreg_lds_bytes(int lpr, int cpt) { return (size_t)(kGlmThreads / 64) * (lpr * cpt + 3) * sizeof(double); }

template <typename K>
int resident_blocks(K kernel, size_t lds = 0) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kGlmThreads, lds) != hipSuccess || nb < 1) {
    (void)hipGetLastError();
    nb = 1;
  }
  return nb;
}

CML_API int cml_glm_set_fp8_nch(int v) {
  g_fp8_nch = v;
  return 0;
}

int g_moments_unroll = 0;  // 0 = auto, else forced K7 prefetch depth (1 or 2; ablation)
int moments_unroll(int cpt) {
  if (g_moments_unroll == 1 || g_moments_unroll == 2) return g_moments_unroll;
  // profiles/r6/k13_ring/moments_ring.log (the branch-free ring at 1 / 2 groups in flight): bf16 x 256 6.19 /
  // 6.15 TB/s, e4m3 x 512 5.34 / 5.40, f32 x 256 6.00 / 6.10; the r5 kernel read 5.56 / 5.0-5.3 / 6.07
  return (cpt == 16 || cpt == 4) ? 2 : 1;
}

CML_API int cml_glm_set_moments_unroll(int u) {
  g_moments_unroll = u;
  return 0;
}

CML_API int cml_glm_set_logreg_unroll(int u) {
  g_logreg_unroll = u;
  return 0;
}

// Grid of the grid-stride GLM kernels: one block per block-iteration of rows, capped at what the
// chip holds at once (blocks/CU from the kernel's real VGPR/LDS occupancy × CUs) — a larger
// persistent grid leaves a tail wave of blocks that runs after everything else.
// kind: 0 = K7 moments, 1 = K13 logreg_grad, 2 = K24 linear_predict.
CML_API int cml_glm_grid(long long n, int d, int dtype, int ncu, int kind) {
  const int cpt = dtype == 0 ? 8 : dtype == 1 ? 4 : dtype == 2 ? 2 : 16;
  if (pick_nch(d, cpt) < 0) return -1;  // moments layout limit
  int lpr, nch;
  if (!stream_layout(d, cpt, lpr, nch)) return -1;
  int per_cu = 1;
  CML_T_SWITCH(dtype, {
    if (kind == 0) {
      CML_NCH_SWITCH(nch, {
        if (moments_unroll(Elt<T>::CPT) == 2)
          per_cu = resident_blocks(col_moments_kernel<T, NCH, 2>, moments_lds_bytes(lpr, Elt<T>::CPT));
        else
          per_cu = resident_blocks(col_moments_kernel<T, NCH, 1>, moments_lds_bytes(lpr, Elt<T>::CPT));
      });
    } else if (kind == 1) {
      CML_NCH_SWITCH(nch, {
        CML_U_SWITCH(logreg_unroll(nch, Elt<T>::CPT), { per_cu = resident_blocks(logreg_grad_kernel<T, NCH, U>, logreg_lds_bytes(lpr, Elt<T>::CPT)); });
      });
    } else {
      CML_NCH_SWITCH(nch, { per_cu = resident_blocks(linear_predict_kernel<T, NCH>); });
    }
  });
  const int rows = (kGlmThreads / 64) * (64 / lpr);
  return grid_for(n, rows, per_cu * ncu);
}

CML_API int cml_col_moments(const void* X, long long n, long long ld, int d, int dtype, const double* shift,
                            double* out, int grid, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 3 && d > 512) return (int)hipErrorInvalidValue;  // fp8 wider rows: caller streams bf16 chunks
  CML_T_SWITCH(dtype, {
    int lpr = 0;
    int nch = 0;
    if (!stream_layout(d, Elt<T>::CPT, lpr, nch)) return (int)hipErrorInvalidValue;
    CML_NCH_SWITCH(nch, {
      if (moments_unroll(Elt<T>::CPT) == 2)
        hipLaunchKernelGGL((col_moments_kernel<T, NCH, 2>), dim3(grid), dim3(kGlmThreads),
                           moments_lds_bytes(lpr, Elt<T>::CPT), st, (const T*)X, n, ld, d, lpr, shift, out);
      else
        hipLaunchKernelGGL((col_moments_kernel<T, NCH, 1>), dim3(grid), dim3(kGlmThreads),
                           moments_lds_bytes(lpr, Elt<T>::CPT), st, (const T*)X, n, ld, d, lpr, shift, out);
    });
  });
  return cml_status();
}

CML_API int cml_scale_apply(const void* X, long long n, long long ldx, int d, int in_dtype, const double* mean,
                            const double* inv_std, int with_mean, void* Y, long long ldy, int dpad, int out_dtype,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 0) return 0;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
#define CML_SCALE_LAUNCH(TI, TO)                                                                                  \
  {                                                                                                               \
    int lpr = 0;                                                                                                  \
    int nch = 0;                                                                                                  \
    if (!stream_layout(dpad, Elt<TI>::CPT, lpr, nch)) return (int)hipErrorInvalidValue;                           \
    CML_NCH_SWITCH(nch, {                                                                                         \
      const int grid = grid_for(n, (kGlmThreads / 64) * (64 / lpr),                                              \
                                resident_blocks(scale_apply_kernel<TI, TO, NCH>) * ncu);                           \
      hipLaunchKernelGGL((scale_apply_kernel<TI, TO, NCH>), dim3(grid), dim3(kGlmThreads), 0, st, (const TI*)X, n, \
                         ldx, d, lpr, mean, inv_std, with_mean, (TO*)Y, ldy, dpad);                              \
    });                                                                                                           \
  }
#define CML_SCALE_OUT(TI)                                        \
  switch (out_dtype) {                                           \
    case 0: CML_SCALE_LAUNCH(TI, u16); break;                    \
    case 1: CML_SCALE_LAUNCH(TI, float); break;                  \
    case 2: CML_SCALE_LAUNCH(TI, double); break;                 \
    case 3: CML_SCALE_LAUNCH(TI, f8_t); break;                   \
    default: return (int)hipErrorInvalidValue;                   \
  }
  switch (in_dtype) {
    case 0: CML_SCALE_OUT(u16); break;
    case 1: CML_SCALE_OUT(float); break;
    case 2: CML_SCALE_OUT(double); break;
    case 3: CML_SCALE_OUT(f8_t); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef CML_SCALE_OUT
#undef CML_SCALE_LAUNCH
  return cml_status();
}

CML_API int cml_logreg_grad(const void* X, long long n, long long ld, int d, int dtype, const double* y,
                            const double* wt, const double* coef, double* out, int grid, const long long* row_base,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  CML_T_SWITCH(dtype, {
    int lpr = 0;
    int nch = 0;
    if (!stream_layout(d, Elt<T>::CPT, lpr, nch)) return (int)hipErrorInvalidValue;
    CML_NCH_SWITCH(nch, {
      CML_U_SWITCH(logreg_unroll(nch, Elt<T>::CPT), {
        hipLaunchKernelGGL((logreg_grad_kernel<T, NCH, U>), dim3(grid), dim3(kGlmThreads),
                           logreg_lds_bytes(lpr, Elt<T>::CPT), st, (const T*)X, n, ld,
                           d, lpr, y, wt, coef, out, row_base);
      });
    });
  });
  return cml_status();
}

// K13 with the hinge (LS = 1) or squared (LS = 2) loss, at the logistic form's ring depth.
CML_API int cml_glm_loss_grad(const void* X, long long n, long long ld, int d, int dtype, const double* y,
                              const double* wt, const double* coef, double* out, int grid, int loss, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (loss < 0 || loss > 2) return (int)hipErrorInvalidValue;
  if (loss == 0) return cml_logreg_grad(X, n, ld, d, dtype, y, wt, coef, out, grid, nullptr, stream);
  CML_T_SWITCH(dtype, {
    int lpr = 0;
    int nch = 0;
    if (!stream_layout(d, Elt<T>::CPT, lpr, nch)) return (int)hipErrorInvalidValue;
    CML_NCH_SWITCH(nch, {
      // the logistic form's ring depth (two groups ahead on e4m3 rows); the caller's grid was sized for it
      if (Elt<T>::CPT == 16 && logreg_unroll(nch, Elt<T>::CPT) == 2) {
        if (loss == 1)
          hipLaunchKernelGGL((logreg_grad_kernel<T, NCH, 2, 1>), dim3(grid), dim3(kGlmThreads),
                             logreg_lds_bytes(lpr, Elt<T>::CPT), st, (const T*)X, n, ld, d, lpr, y, wt, coef, out,
                             nullptr);
        else
          hipLaunchKernelGGL((logreg_grad_kernel<T, NCH, 2, 2>), dim3(grid), dim3(kGlmThreads),
                             logreg_lds_bytes(lpr, Elt<T>::CPT), st, (const T*)X, n, ld, d, lpr, y, wt, coef, out,
                             nullptr);
      } else if (loss == 1) {
        hipLaunchKernelGGL((logreg_grad_kernel<T, NCH, 1, 1>), dim3(grid), dim3(kGlmThreads),
                           logreg_lds_bytes(lpr, Elt<T>::CPT), st, (const T*)X, n, ld, d, lpr, y, wt, coef, out,
                           nullptr);
      } else {
        hipLaunchKernelGGL((logreg_grad_kernel<T, NCH, 1, 2>), dim3(grid), dim3(kGlmThreads),
                           logreg_lds_bytes(lpr, Elt<T>::CPT), st, (const T*)X, n, ld, d, lpr, y, wt, coef, out,
                           nullptr);
      }
    });
  });
  return cml_status();
}

// K13m layout: LPR lanes per row (up to 64), NCH chunks; CP class slots. Returns the class-slot count the
// kernel runs for (0: not supported at this width / class count — the caller takes the chunked form).
static int multinomial_layout(int d, int dtype, int C, int& lpr, int& nch) {
  const int cpt = dtype == 0 ? 8 : dtype == 1 ? 4 : dtype == 2 ? 2 : 16;
  const int ch = (d + cpt - 1) / cpt;
  lpr = pow2ceil(ch) < 64 ? pow2ceil(ch) : 64;
  nch = pow2ceil((ch + lpr - 1) / lpr);
  if (nch > 2) return 0;
  const int cp = C <= 4 ? 4 : C <= 8 ? 8 : 0;
  if (cp == 0) return 0;
  const int dpad = lpr * nch * cpt;
  const int vals = cp * nch * cpt * (dtype == 2 ? 2 : 1);  // VGPRs of one class-row set (f64: two each)
  if (vals > 64) return 0;
  if ((long long)(kGlmThreads / 64) * cp * dpad * 8 > 80 * 1024) return 0;
  return cp;
}

CML_API int cml_multinomial_supported(int d, int dtype, int C) {
  int lpr = 0, nch = 0;
  return multinomial_layout(d, dtype, C, lpr, nch);
}

CML_API int cml_multinomial_grid(long long n, int d, int dtype, int C, int ncu) {
  int lpr = 0, nch = 0;
  const int cp = multinomial_layout(d, dtype, C, lpr, nch);
  if (cp == 0) return -1;
  const int rows = (kGlmThreads / 64) * (64 / lpr);
  return grid_for(n, rows, 2 * ncu);
}

CML_API int cml_multinomial_grad(const void* X, long long n, long long ld, int d, int dtype, int C, const double* y,
                                 const double* wt, const double* coef, double* out, int grid, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int lpr = 0, nch = 0;
  const int cp = multinomial_layout(d, dtype, C, lpr, nch);
  if (cp == 0 || grid < 1) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(kGlmThreads / 64) * (cp * lpr * nch * (dtype == 0 ? 8 : dtype == 1 ? 4 : dtype == 2 ? 2 : 16) +
                                                   cp + 2) * sizeof(double);
#define CML_MN(CPV)                                                                                          \
  CML_T_SWITCH(dtype, {                                                                                      \
    if (nch == 1)                                                                                            \
      hipLaunchKernelGGL((multinomial_grad_kernel<T, 1, CPV>), dim3(grid), dim3(kGlmThreads), lds, st,       \
                         (const T*)X, n, ld, d, lpr, C, y, wt, coef, out);                                   \
    else                                                                                                     \
      hipLaunchKernelGGL((multinomial_grad_kernel<T, 2, CPV>), dim3(grid), dim3(kGlmThreads), lds, st,       \
                         (const T*)X, n, ld, d, lpr, C, y, wt, coef, out);                                   \
  })
  if (cp == 4) {
    CML_MN(4);
  } else {
    CML_MN(8);
  }
#undef CML_MN
  return cml_status();
}

CML_API int cml_partial_colsum(const double* part, int nb, int m, double* msg, void* stream) {
  if (nb < 1 || m < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(partial_colsum_kernel, dim3((m + kColsumCols - 1) / kColsumCols), dim3(kColsumCols * kColsumSlices),
                     0, (hipStream_t)stream, part, nb, m, msg);
  return cml_status();
}

CML_API int cml_sgd_update(const double* msg, int d, double* coef, double* vel, double* eff, const double* lr,
                           double mom, double l2, int fit_intercept, const double* gscale, const double* kscale,
                           double* loss_acc, long long* base, long long batch, long long wrap, void* stream) {
  if (d < 1 || batch < 1 || wrap < batch) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sgd_update_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, msg, d, coef, vel, eff, lr, mom,
                     l2, fit_intercept, gscale, kscale, loss_acc, base, batch, wrap);
  return cml_status();
}

CML_API int cml_linear_predict(const void* X, long long n, long long ld, int d, int dtype, const double* coef,
                               int link, double* out, int grid, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  CML_T_SWITCH(dtype, {
    int lpr = 0;
    int nch = 0;
    if (!stream_layout(d, Elt<T>::CPT, lpr, nch)) return (int)hipErrorInvalidValue;
    CML_NCH_SWITCH(nch, {
      hipLaunchKernelGGL((linear_predict_kernel<T, NCH>), dim3(grid), dim3(kGlmThreads), 0, st, (const T*)X, n, ld,
                         d, lpr, coef, link, out);
    });
  });
  return cml_status();
}

CML_API int cml_gram(const void* X, long long n, long long ld, int d, int dtype, const double* y, const double* wt,
                     double* out, int grid, void* stream) {
  if (d > 30) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int m = d + 2;
  if (m <= 8) {
    switch (dtype) {
      case 0: return launch_gram_small<u16>(X, n, ld, d, y, wt, out, grid, st);
      case 1: return launch_gram_small<float>(X, n, ld, d, y, wt, out, grid, st);
      case 2: return launch_gram_small<double>(X, n, ld, d, y, wt, out, grid, st);
      case 3: return launch_gram_small<f8_t>(X, n, ld, d, y, wt, out, grid, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  CML_T_SWITCH(dtype, {
    hipLaunchKernelGGL((gram_kernel<T>), dim3(grid), dim3(256), 0, st, (const T*)X, n, ld, d, y, wt, out);
  });
  return cml_status();
}
