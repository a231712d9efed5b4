// Generalised-linear-model and feature-statistics kernels for gfx950 (MI355X).
//
// K7  col_moments     per-feature count / shifted Σ / shifted Σ² in f64 (StandardScaler,
//                     LinearRegression/LogisticRegression standardization, Summarizer)
// K8  scale_apply     (x - μ)·(1/σ) with optional centring, any in/out dtype (bf16/f32/f64)
// K13 logreg_grad     fused binomial logistic pass: margin = x·w + b, p = σ(margin),
//                     ∇w += (p − y)·x, ∇b += p − y, loss += softplus(margin) − y·margin,
//                     X read ONCE per pass (L-BFGS full batch or an SGD mini-batch)
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

template <typename T> struct Elt;
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

// Load CPT values of row `row` starting at column c0 (zero beyond d; the row stride keeps the
// vector load in bounds because ld is padded to a multiple of CPT).
template <typename T>
__device__ inline void load_chunk(const T* X, long long row, long long ld, int c0, int d, double* v) {
  constexpr int CPT = Elt<T>::CPT;
  if (c0 + CPT <= d) {
    Elt<T>::load(X + row * ld + c0, v);
  } else {
#pragma unroll
    for (int j = 0; j < CPT; ++j) v[j] = 0.0;
    for (int j = 0; c0 + j < d && j < CPT; ++j) {
      if constexpr (sizeof(T) == 2) v[j] = (double)bf16_to_f32(((const u16*)X)[row * ld + c0 + j]);
      else v[j] = (double)X[row * ld + c0 + j];
    }
  }
}

__device__ inline double group_sum(double v, int lpr) {
  for (int o = lpr >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------- K7 moments
template <typename T, int NCH>
__global__ __launch_bounds__(kGlmThreads) void col_moments_kernel(const T* __restrict__ X, long long n, long long ld,
                                                                  int d, int lpr, const double* __restrict__ shift,
                                                                  double* __restrict__ out /*[grid][2][d]*/) {
  constexpr int CPT = Elt<T>::CPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  double s1[NCH][CPT], s2[NCH][CPT], sh[NCH][CPT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      s1[c][j] = 0.0;
      s2[c][j] = 0.0;
      const int col = (c * lpr + li) * CPT + j;
      sh[c][j] = col < d ? shift[col] : 0.0;
    }
  const long long step = (long long)gridDim.x * nw * rpw;
  for (long long row = ((long long)blockIdx.x * nw + wave) * rpw + sub; row < n; row += step) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int c0 = (c * lpr + li) * CPT;
      if (c0 >= d) continue;
      double v[CPT];
      load_chunk<T>(X, row, ld, c0, d, v);
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const double t = v[j] - sh[c][j];
        s1[c][j] += t;
        s2[c][j] = fma(t, t, s2[c][j]);
      }
    }
  }
  // reduce the rpw row groups of the wave and the waves of the block through LDS
  __shared__ double red[kGlmThreads / 64][64 * 8 * 2];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      double a = s1[c][j], b = s2[c][j];
      for (int o = lpr; o < 64; o <<= 1) {  // sum over sub-groups (lanes li, li+lpr, ...)
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
      }
      s1[c][j] = a;
      s2[c][j] = b;
    }
  }
  // lanes 0..lpr-1 of each wave hold the wave totals for their columns
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    __syncthreads();
    if (sub == 0) {
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        red[wave][(li * CPT + j) * 2] = s1[c][j];
        red[wave][(li * CPT + j) * 2 + 1] = s2[c][j];
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < lpr * CPT; t += blockDim.x) {
      const int col = c * lpr * CPT + t;
      if (col >= d) continue;
      double a = 0.0, b = 0.0;
      for (int w = 0; w < nw; ++w) {
        a += red[w][t * 2];
        b += red[w][t * 2 + 1];
      }
      out[((long long)blockIdx.x * 2) * d + col] = a;
      out[((long long)blockIdx.x * 2 + 1) * d + col] = b;
    }
  }
}

// ---------------------------------------------------------------------------- K8 scale
template <typename TI, typename TO>
__global__ void scale_apply_kernel(const TI* __restrict__ X, long long n, long long ldx, int d,
                                   const double* __restrict__ mean, const double* __restrict__ inv_std, int with_mean,
                                   TO* __restrict__ Y, long long ldy, int dpad) {
  const long long total = n * (long long)dpad;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / dpad;
    const int c = (int)(i - r * dpad);
    double v = 0.0;
    if (c < d) {
      double x;
      if constexpr (sizeof(TI) == 2) x = (double)bf16_to_f32(((const u16*)X)[r * ldx + c]);
      else x = (double)X[r * ldx + c];
      v = (with_mean ? x - mean[c] : x) * inv_std[c];
    }
    if constexpr (sizeof(TO) == 2) ((u16*)Y)[r * ldy + c] = f32_to_bf16((float)v);
    else Y[r * ldy + c] = (TO)v;
  }
}

// ---------------------------------------------------------------------------- K13 logistic gradient
template <typename T, int NCH>
__global__ __launch_bounds__(kGlmThreads) void logreg_grad_kernel(
    const T* __restrict__ X, long long n, long long ld, int d, int lpr, const double* __restrict__ y,
    const double* __restrict__ wt, const double* __restrict__ coef /*[d+1], last = intercept*/,
    double* __restrict__ out /*[grid][d + 3]: grad (d), grad_b, loss, weight sum*/) {
  constexpr int CPT = Elt<T>::CPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  double w[NCH][CPT], g[NCH][CPT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int col = (c * lpr + li) * CPT + j;
      w[c][j] = col < d ? coef[col] : 0.0;
      g[c][j] = 0.0;
    }
  const double b = coef[d];
  double gb = 0.0, loss = 0.0, wsum = 0.0;
  const long long step = (long long)gridDim.x * nw * rpw;
  for (long long row0 = ((long long)blockIdx.x * nw + wave) * rpw; row0 < n; row0 += step) {
    const long long row = row0 + sub;
    const bool ok = row < n;
    double v[NCH][CPT];
    double m = 0.0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int c0 = (c * lpr + li) * CPT;
      if (ok && c0 < d) {
        load_chunk<T>(X, row, ld, c0, d, v[c]);
      } else {
#pragma unroll
        for (int j = 0; j < CPT; ++j) v[c][j] = 0.0;
      }
#pragma unroll
      for (int j = 0; j < CPT; ++j) m = fma(v[c][j], w[c][j], m);
    }
    m = group_sum(m, lpr) + b;
    const double yi = ok ? y[row] : 0.0;
    const double wi = ok ? (wt != nullptr ? wt[row] : 1.0) : 0.0;
    // p = sigmoid(m) and softplus(m), numerically stable
    const double e = exp(-fabs(m));
    const double p = m >= 0 ? 1.0 / (1.0 + e) : e / (1.0 + e);
    const double sp = fmax(m, 0.0) + log1p(e);
    const double r = wi * (p - yi);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < CPT; ++j) g[c][j] = fma(r, v[c][j], g[c][j]);
    if (li == 0) {
      gb += r;
      loss += wi * (sp - yi * m);
      wsum += wi;
    }
  }
  // reduce across row sub-groups, then across waves
  __shared__ double red[kGlmThreads / 64][64 * 8 + 3];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CPT; ++j)
      for (int o = lpr; o < 64; o <<= 1) g[c][j] += __shfl_xor(g[c][j], o, 64);
  for (int o = 1; o < 64; o <<= 1) {
    gb += __shfl_xor(gb, o, 64);
    loss += __shfl_xor(loss, o, 64);
    wsum += __shfl_xor(wsum, o, 64);
  }
  double* o_ = out + (long long)blockIdx.x * (d + 3);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    __syncthreads();
    if (sub == 0)
#pragma unroll
      for (int j = 0; j < CPT; ++j) red[wave][li * CPT + j] = g[c][j];
    if (lane == 0 && c == 0) {
      red[wave][64 * 8] = gb;
      red[wave][64 * 8 + 1] = loss;
      red[wave][64 * 8 + 2] = wsum;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < lpr * CPT; t += blockDim.x) {
      const int col = c * lpr * CPT + t;
      if (col >= d) continue;
      double a = 0.0;
      for (int ww = 0; ww < nw; ++ww) a += red[ww][t];
      o_[col] = a;
    }
    if (c == 0 && threadIdx.x < 3) {
      double a = 0.0;
      for (int ww = 0; ww < nw; ++ww) a += red[ww][64 * 8 + threadIdx.x];
      o_[d + threadIdx.x] = a;
    }
  }
}

// ---------------------------------------------------------------------------- K24 predict
template <typename T, int NCH>
__global__ __launch_bounds__(kGlmThreads) void linear_predict_kernel(const T* __restrict__ X, long long n,
                                                                     long long ld, int d, int lpr,
                                                                     const double* __restrict__ coef, int link,
                                                                     double* __restrict__ out) {
  constexpr int CPT = Elt<T>::CPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int rpw = 64 / lpr, sub = lane / lpr, li = lane - sub * lpr;
  const long long step = (long long)gridDim.x * nw * rpw;
  for (long long row0 = ((long long)blockIdx.x * nw + wave) * rpw; row0 < n; row0 += step) {
    const long long row = row0 + sub;
    const bool ok = row < n;
    double m = 0.0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int c0 = (c * lpr + li) * CPT;
      if (ok && c0 < d) {
        double v[CPT];
        load_chunk<T>(X, row, ld, c0, d, v);
#pragma unroll
        for (int j = 0; j < CPT; ++j) m = fma(v[j], c0 + j < d ? coef[c0 + j] : 0.0, m);
      }
    }
    m = group_sum(m, lpr) + coef[d];
    if (ok && li == 0) out[row] = link == 1 ? 1.0 / (1.0 + exp(-m)) : m;
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

CML_API int cml_glm_grid(long long n, int d, int dtype, int cap) {
  const int cpt = dtype == 0 ? 8 : dtype == 1 ? 4 : 2;
  const int nch = pick_nch(d, cpt);
  if (nch < 0) return -1;
  const int lpr = pick_lpr(d, cpt, nch);
  const int rows = (kGlmThreads / 64) * (64 / lpr) * 16;
  return grid_for(n, rows, cap);
}

CML_API int cml_col_moments(const void* X, long long n, long long ld, int d, int dtype, const double* shift,
                            double* out, int grid, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  CML_T_SWITCH(dtype, {
    constexpr int CPT = Elt<T>::CPT;
    const int nch = pick_nch(d, CPT);
    const int lpr = pick_lpr(d, CPT, nch < 0 ? 8 : nch);
    CML_NCH_SWITCH(nch, {
      hipLaunchKernelGGL((col_moments_kernel<T, NCH>), dim3(grid), dim3(kGlmThreads), 0, st, (const T*)X, n, ld, d,
                         lpr, shift, out);
    });
  });
  return cml_status();
}

CML_API int cml_scale_apply(const void* X, long long n, long long ldx, int d, int in_dtype, const double* mean,
                            const double* inv_std, int with_mean, void* Y, long long ldy, int dpad, int out_dtype,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long long total = n * (long long)dpad;
  const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  if (blocks == 0) return 0;
#define CML_SCALE_OUT(TI)                                                                                          \
  switch (out_dtype) {                                                                                             \
    case 0: hipLaunchKernelGGL((scale_apply_kernel<TI, u16>), dim3(blocks), dim3(256), 0, st, (const TI*)X, n, ldx, \
                               d, mean, inv_std, with_mean, (u16*)Y, ldy, dpad); break;                           \
    case 1: hipLaunchKernelGGL((scale_apply_kernel<TI, float>), dim3(blocks), dim3(256), 0, st, (const TI*)X, n,    \
                               ldx, d, mean, inv_std, with_mean, (float*)Y, ldy, dpad); break;                    \
    case 2: hipLaunchKernelGGL((scale_apply_kernel<TI, double>), dim3(blocks), dim3(256), 0, st, (const TI*)X, n,   \
                               ldx, d, mean, inv_std, with_mean, (double*)Y, ldy, dpad); break;                   \
    default: return (int)hipErrorInvalidValue;                                                                     \
  }
  switch (in_dtype) {
    case 0: CML_SCALE_OUT(u16); break;
    case 1: CML_SCALE_OUT(float); break;
    case 2: CML_SCALE_OUT(double); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef CML_SCALE_OUT
  return cml_status();
}

CML_API int cml_logreg_grad(const void* X, long long n, long long ld, int d, int dtype, const double* y,
                            const double* wt, const double* coef, double* out, int grid, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  CML_T_SWITCH(dtype, {
    constexpr int CPT = Elt<T>::CPT;
    const int nch = pick_nch(d, CPT);
    const int lpr = pick_lpr(d, CPT, nch < 0 ? 8 : nch);
    CML_NCH_SWITCH(nch, {
      hipLaunchKernelGGL((logreg_grad_kernel<T, NCH>), dim3(grid), dim3(kGlmThreads), 0, st, (const T*)X, n, ld, d,
                         lpr, y, wt, coef, out);
    });
  });
  return cml_status();
}

CML_API int cml_linear_predict(const void* X, long long n, long long ld, int d, int dtype, const double* coef,
                               int link, double* out, int grid, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  CML_T_SWITCH(dtype, {
    constexpr int CPT = Elt<T>::CPT;
    const int nch = pick_nch(d, CPT);
    const int lpr = pick_lpr(d, CPT, nch < 0 ? 8 : nch);
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
  CML_T_SWITCH(dtype, {
    hipLaunchKernelGGL((gram_kernel<T>), dim3(grid), dim3(256), 0, st, (const T*)X, n, ld, d, y, wt, out);
  });
  return cml_status();
}
