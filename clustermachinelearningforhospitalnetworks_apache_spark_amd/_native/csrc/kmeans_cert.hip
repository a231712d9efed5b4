// Certified pruned Lloyd step on source-precision (f32 / f64) rows — precision "screen" after its
// first, MFMA-screened, assignment (models/kmeans.py LloydEngine._step_screen).
//
// The reference fits f64 feature vectors (ref.py:64-72, ref.py:134-136 -> ref.py:147). The exact
// algorithm assigns every row by the f64 fold of kmeans_exact.hip and sums the rows per cluster; this
// step reproduces it bit for bit while touching only the rows whose label can change:
//
//   cert_stats    drift of every centre (||C_t - C_{t-1}||, rounded up), its top two, and half the
//                 distance to the nearest other centre (rounded down);
//   cert_bounds   per row: u += drift[label], l -= largest other drift (Hamerly); the label is proven
//                 when u < max(l, half-separation[label]) — strictly, in f32 with outward rounding, so
//                 the real distances (hence the f64 folds, ~1e-14 away) order the same way; other rows
//                 are listed (A);
//   cert_tighten  listed rows: u <- the real distance to the label (16 lanes per row); still unproven
//                 rows go to list B, which exact_top2 (kmeans_exact.hip: the exact fold over every
//                 centre, same bits) re-assigns, refreshing u / l and appending the label moves;
//   cert_hist / cert_scan / cert_scatter / cert_delta / cert_apply
//                 the moves' per-cluster deltas (+row into the new cluster, -row out of the old) in
//                 double-double, added to the cluster sums kept as hi + lo: the sums stay exactly the
//                 from-scratch double-double sums (exact_segsum), so the centres are the same bits.
#include "common.h"
#include "exact_util.h"

namespace {

constexpr int kT = 256;

// grid k + 1: block j < k -> s[j] = half the distance from centre j to the nearest other centre (f32,
// rounded down; +inf for k = 1); block k -> drift[j] = ||C_j - Cold_j|| (rounded up) for every j and
// dtop = {largest drift, second largest, index of the largest (as float)}; it also zeroes `zero[nz]`
// (the step's list counters and move histogram).
__global__ __launch_bounds__(kT) void cert_stats_kernel(const double* __restrict__ C, const double* __restrict__ Cold,
                                                        int k, int d, float* __restrict__ s, float* __restrict__ drift,
                                                        float* __restrict__ dtop, int* __restrict__ zero, int nz) {
  __shared__ double red[kT];
  __shared__ int redi[kT];
  const int j = blockIdx.x;
  if (j < k) {
    const double* cj = C + (long long)j * d;
    double m = __builtin_huge_val();
    for (int i = threadIdx.x; i < k; i += kT) {
      if (i == j) continue;
      const double* ci = C + (long long)i * d;
      double a = 0.0;
      for (int t = 0; t < d; ++t) {
        const double e = ci[t] - cj[t];
        a = __fma_rn(e, e, a);
      }
      m = a < m ? a : m;
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = kT / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + w]);
      __syncthreads();
    }
    if (threadIdx.x == 0)
      s[j] = red[0] < __builtin_huge_val() ? f32_dn(0.5 * sqrt(red[0]) * (1.0 - kFoldMargin)) : __builtin_huge_valf();
    return;
  }
  for (int i = threadIdx.x; i < nz; i += kT) zero[i] = 0;
  double b1 = -1.0, b2 = -1.0;
  int i1 = 0;
  for (int i = threadIdx.x; i < k; i += kT) {
    const double* ci = C + (long long)i * d;
    const double* oi = Cold + (long long)i * d;
    double a = 0.0;
    for (int t = 0; t < d; ++t) {
      const double e = ci[t] - oi[t];
      a = __fma_rn(e, e, a);
    }
    const float df = a > 0.0 ? f32_up(sqrt(a) * (1.0 + kFoldMargin)) : 0.0f;
    drift[i] = df;
    const double v = (double)df;
    if (v > b1) {
      b2 = b1;
      b1 = v;
      i1 = i;
    } else if (v > b2) {
      b2 = v;
    }
  }
  // top two over the block: thread-local (b1, i1, b2), merged serially (k is small)
  red[threadIdx.x] = b1;
  redi[threadIdx.x] = i1;
  __shared__ double red2[kT];
  red2[threadIdx.x] = b2;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m1 = -1.0, m2 = -1.0;
    int mi = 0;
    for (int t = 0; t < kT; ++t) {
      const double v1 = red[t], v2 = red2[t];
      if (v1 > m1) {
        m2 = fmax(m1, v2);
        m1 = v1;
        mi = redi[t];
      } else {
        m2 = fmax(m2, v1);
      }
    }
    dtop[0] = (float)fmax(m1, 0.0);
    dtop[1] = (float)fmax(m2, 0.0);
    dtop[2] = (float)mi;
  }
}

// Every row: move the bounds by the drifts, list the rows whose label the bounds no longer prove.
__global__ __launch_bounds__(kT) void cert_bounds_kernel(const int* __restrict__ lab, float* __restrict__ u,
                                                         float* __restrict__ l, const float* __restrict__ drift,
                                                         const float* __restrict__ dtop, const float* __restrict__ s,
                                                         long long n, int* __restrict__ lst, int* __restrict__ count) {
  __shared__ int buf[kBuf];
  __shared__ int nb, base;
  if (threadIdx.x == 0) nb = 0;
  ListBuf lb{buf, &nb, &base};
  const double d1 = (double)dtop[0], d2 = (double)dtop[1];
  const int i1 = (int)dtop[2];
  for (long long r0 = (long long)blockIdx.x * kT; r0 < n; r0 += (long long)gridDim.x * kT) {
    __syncthreads();
    const long long r = r0 + threadIdx.x;
    if (r < n) {
      const int a = lab[r];
      const float uu = f32_up((double)u[r] + (double)drift[a]);
      const float ll = f32_dn((double)l[r] - (a == i1 ? d2 : d1));
      u[r] = uu;
      l[r] = ll;
      if (!(uu < fmaxf(ll, s[a]))) buf[atomicAdd(&nb, 1)] = (int)r;
    }
    list_flush<kT>(lb, lst, count, false);
  }
  list_flush<kT>(lb, lst, count, true);
}

// list_flush that also writes, beside each listed row, its K9r norm and current label (compacted inputs
// of the K9r candidate pass over list B), when xn is given.
__device__ __forceinline__ void list_flush_ext(ListBuf lb, int* lst, int* count, bool force, const float* xn,
                                               float* bxn, const int* lab, int* blab) {
  __syncthreads();
  const int m = *lb.n;
  if (m > 0 && (force || m > kBuf - kT)) {
    if (threadIdx.x == 0) *lb.base = atomicAdd(count, m);
    __syncthreads();
    const int b = *lb.base;
    for (int i = threadIdx.x; i < m; i += kT) {
      const int r = lb.buf[i];
      lst[b + i] = r;
      if (xn != nullptr) {
        bxn[b + i] = xn[r];
        blab[b + i] = lab[r];
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) *lb.n = 0;
  }
  __syncthreads();
}

// Listed rows (A): u <- the real distance to the label (16 lanes per row, any summation order: a bound
// with the fold margin); rows still unproven go to list B.
template <typename T>
__global__ __launch_bounds__(kT) void cert_tighten_kernel(const T* __restrict__ X, long long ldx, int d,
                                                          const double* __restrict__ C, const int* __restrict__ lab,
                                                          float* __restrict__ u, const float* __restrict__ l,
                                                          const float* __restrict__ s, const int* __restrict__ la,
                                                          const int* __restrict__ na, int* __restrict__ lbst,
                                                          int* __restrict__ nbst, const float* __restrict__ xn,
                                                          float* __restrict__ bxn, int* __restrict__ blab) {
  __shared__ int buf[kBuf];
  __shared__ int nb, base;
  if (threadIdx.x == 0) nb = 0;
  ListBuf lbf{buf, &nb, &base};
  const long long cnt = *na;
  const int g = threadIdx.x >> 4, q = threadIdx.x & 15;  // 16 row groups of 16 lanes
  for (long long i0 = (long long)blockIdx.x * 16; i0 < cnt; i0 += (long long)gridDim.x * 16) {
    __syncthreads();
    const long long i = i0 + g;
    const bool live = i < cnt;
    long long r = 0;
    int a = 0;
    double acc = 0.0;
    if (live) {
      r = la[i];
      a = lab[r];
      const T* x = X + r * ldx;
      const double* c = C + (long long)a * d;
      for (int t0 = q; t0 < d; t0 += 16 * 8) {  // 8 loads in flight per lane before the fmas
        double xv[8], cv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int t = t0 + 16 * u;
          xv[u] = t < d ? (double)x[t] : 0.0;
          cv[u] = t < d ? c[t] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double e = xv[u] - cv[u];
          acc = __fma_rn(e, e, acc);
        }
      }
    }
    acc += __shfl_xor(acc, 8, 16);
    acc += __shfl_xor(acc, 4, 16);
    acc += __shfl_xor(acc, 2, 16);
    acc += __shfl_xor(acc, 1, 16);
    if (live && q == 0) {
      const float uu = f32_up(sqrt(acc) * (1.0 + kFoldMargin));
      u[r] = uu;
      if (!(uu < fmaxf(l[r], s[a]))) buf[atomicAdd(&nb, 1)] = (int)r;
    }
    list_flush_ext(lbf, lbst, nbst, false, xn, bxn, lab, blab);
  }
  list_flush_ext(lbf, lbst, nbst, true, xn, bxn, lab, blab);
}

// One block: centres C (f64 [k, d]) -> the split screen's layout cb [kp, ldc] = [c_hi | c_hi | c_lo] in
// ds-wide segments (bf16; padding rows zero), cn = ||c||² (f32; padding rows +inf: they never win) and
// cst = {max ||c_lo||, max ||c||, max ||c - c_hi - c_lo||} (rounded up) — the certificate's constants.
__global__ __launch_bounds__(1024) void split_centres_kernel(const double* __restrict__ C, int k, int kp, int d,
                                                             int ds, u16* __restrict__ cb, long long ldc,
                                                             float* __restrict__ cn, double* __restrict__ cst,
                                                             float* __restrict__ mc) {
  __shared__ double red[4][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double m0 = 0.0, m1 = 0.0, m2 = 0.0, m3 = 0.0;
  for (int j = w; j < kp; j += 16) {
    double a2 = 0.0, c2 = 0.0, r2 = 0.0;
    for (int t = lane; t < ldc; t += 64) {
      u16 hb = 0, lb = 0;
      if (j < k && t < d) {
        const double v = C[(long long)j * d + t];
        hb = f32_to_bf16((float)v);
        const double r1 = v - (double)bf16_to_f32(hb);
        lb = f32_to_bf16((float)r1);
        const double lv = (double)bf16_to_f32(lb);
        const double rc = r1 - lv;
        a2 = __fma_rn(lv, lv, a2);
        c2 = __fma_rn(v, v, c2);
        r2 = __fma_rn(rc, rc, r2);
      }
      if (t < ds) {
        cb[(long long)j * ldc + t] = hb;
        cb[(long long)j * ldc + ds + t] = hb;
        cb[(long long)j * ldc + 2 * ds + t] = lb;
      } else if (t >= 3 * ds) {
        cb[(long long)j * ldc + t] = 0;
      }
    }
    a2 = wave_sum_f64(a2);
    c2 = wave_sum_f64(c2);
    r2 = wave_sum_f64(r2);
    if (lane == 0) cn[j] = j < k ? (float)c2 : __builtin_huge_valf();
    if (j < k) m3 = fmax(m3, (double)(float)c2);
    m0 = fmax(m0, sqrt(a2));
    m1 = fmax(m1, sqrt(c2));
    m2 = fmax(m2, sqrt(r2));
  }
  if (lane == 0) {
    red[0][w] = m0;
    red[1][w] = m1;
    red[2][w] = m2;
    red[3][w] = m3;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double m = 0.0;
    for (int v = 0; v < 16; ++v) m = fmax(m, red[threadIdx.x][v]);
    if (threadIdx.x < 3) cst[threadIdx.x] = m * (1.0 + 1e-9);
    else if (mc != nullptr) mc[0] = (float)m;  // the largest centre norm (K9r's slack term)
  }
}

// List B after the split-screen K9r candidate pass (labels / bf16-model bounds at the real rows): certified
// rows keep the screened label with real-distance bounds (and append a move when it changed); the others
// get their old label back and go to list C for the exact fold (exact_top2, which appends their moves).
__global__ __launch_bounds__(kT) void cert_list_kernel(const int* __restrict__ lst, const int* __restrict__ cnt_dev,
                                                       const int* __restrict__ blab, int* __restrict__ lab,
                                                       float* __restrict__ u, float* __restrict__ l,
                                                       const float* __restrict__ ea, const float* __restrict__ eb,
                                                       const float* __restrict__ en, const double* __restrict__ cst,
                                                       int* __restrict__ lc, int* __restrict__ nc,
                                                       int* __restrict__ mv_row, int* __restrict__ mv_old,
                                                       int* __restrict__ mv_new, int* __restrict__ mv_count) {
  __shared__ int s_w[kT / 64 + 1];
  const long long cnt = *cnt_dev;
  const double c0 = cst[0], c1 = cst[1], c2 = cst[2];
  for (long long i0 = (long long)blockIdx.x * kT; i0 < cnt; i0 += (long long)gridDim.x * kT) {
    const long long i = i0 + threadIdx.x;
    bool bad = false, moved = false;
    int r = 0, old = 0, now = 0;
    if (i < cnt) {
      r = lst[i];
      old = blab[i];
      now = lab[r];
      const double e = 2.0 * ((double)ea[r] * c0 + (double)eb[r] * c1 + 1.01 * (double)en[r] * c2) * (1.0 + 1e-6);
      const double ub = (double)u[r], lbv = (double)l[r];
      const float uu = f32_up(sqrt(ub * ub + e) * (1.0 + kFoldMargin));
      const float ll = f32_dn(sqrt(fmax(lbv * lbv - e, 0.0)) * (1.0 - kFoldMargin));
      bad = !(uu < ll);
      if (bad) {
        lab[r] = old;  // exact_top2 reads the old label to log the move
      } else {
        u[r] = uu;
        l[r] = ll;
        moved = now != old;
      }
    }
    const int pc = block_append<kT>(bad, nc, s_w);
    if (pc >= 0) lc[pc] = r;
    const int pm = block_append<kT>(moved, mv_count, s_w);
    if (pm >= 0) {
      mv_row[pm] = r;
      mv_old[pm] = old;
      mv_new[pm] = now;
    }
  }
}

// Move histogram: bin j = rows moving into cluster j, bin k + j = rows leaving it.
__global__ __launch_bounds__(kT) void cert_hist_kernel(const int* __restrict__ mv_old, const int* __restrict__ mv_new,
                                                       const int* __restrict__ m_dev, int k, int* __restrict__ hist) {
  extern __shared__ int h[];
  for (int b = threadIdx.x; b < 2 * k; b += kT) h[b] = 0;
  __syncthreads();
  const long long m = *m_dev;
  for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < m; i += (long long)gridDim.x * kT) {
    atomicAdd(&h[mv_new[i]], 1);
    atomicAdd(&h[k + mv_old[i]], 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < 2 * k; b += kT)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// One block: seg[0 .. 2k] = exclusive prefix of hist, cursor = seg[0 .. 2k).
__global__ __launch_bounds__(kT) void cert_scan_kernel(const int* __restrict__ hist, int k, int* __restrict__ seg,
                                                       int* __restrict__ cursor) {
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < 2 * k; ++b) {
      seg[b] = acc;
      cursor[b] = acc;
      acc += hist[b];
    }
    seg[2 * k] = acc;
  }
}

// Moves -> rows grouped by bin (order inside a bin is free: the double-double sums do not depend on it).
__global__ __launch_bounds__(kT) void cert_scatter_kernel(const int* __restrict__ mv_row,
                                                          const int* __restrict__ mv_old,
                                                          const int* __restrict__ mv_new, const int* __restrict__ m_dev,
                                                          int k, int* __restrict__ cursor, int* __restrict__ perm) {
  extern __shared__ int sh[];
  int* h = sh;           // [2k] local counts
  int* bs = sh + 2 * k;  // [2k] reserved bases
  const long long m = *m_dev;
  for (long long i0 = (long long)blockIdx.x * kT; i0 < m; i0 += (long long)gridDim.x * kT) {
    for (int b = threadIdx.x; b < 2 * k; b += kT) h[b] = 0;
    __syncthreads();
    const long long i = i0 + threadIdx.x;
    int bn = 0, bo = 0, rn = 0, ro = 0, row = 0;
    if (i < m) {
      row = mv_row[i];
      bn = mv_new[i];
      bo = k + mv_old[i];
      rn = atomicAdd(&h[bn], 1);
      ro = atomicAdd(&h[bo], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < 2 * k; b += kT) bs[b] = h[b] ? atomicAdd(&cursor[b], h[b]) : 0;
    __syncthreads();
    if (i < m) {
      perm[bs[bn] + rn] = row;
      perm[bs[bo] + ro] = row;
    }
    __syncthreads();
  }
}

// grid (k, NS): block (j, s) adds slice s of the rows moving into j and subtracts slice s of the rows
// leaving j, double-double per dimension (4 row lanes x 64 dimensions, lanes combined in order), into
// P_hi / P_lo [NS][k][d].
template <typename T>
__global__ __launch_bounds__(kT) void cert_delta_kernel(const T* __restrict__ X, long long ldx, int d,
                                                        const int* __restrict__ seg, const int* __restrict__ perm,
                                                        int k, double* __restrict__ P_hi, double* __restrict__ P_lo) {
  __shared__ double sh_h[kT], sh_l[kT];
  const int j = blockIdx.x, sl = blockIdx.y, ns = gridDim.y;
  const int lane = threadIdx.x >> 6, col = threadIdx.x & 63;
  const long long p0 = seg[j], p1 = seg[j + 1], q0 = seg[k + j], q1 = seg[k + j + 1];
  const long long np = p1 - p0, nq = q1 - q0;
  const long long pa = p0 + np * sl / ns, pb = p0 + np * (sl + 1) / ns;
  const long long qa = q0 + nq * sl / ns, qb = q0 + nq * (sl + 1) / ns;
  for (int t0 = 0; t0 < d; t0 += 64) {
    const int t = t0 + col;
    double h = 0.0, lo = 0.0;
    if (t < d) {  // 8 rows' loads in flight per lane before their adds (the order of exact adds is free)
      constexpr int B = 8;
      for (long long p0 = pa + lane; p0 < pb; p0 += 4 * B) {
        double v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const long long p = p0 + 4 * u;
          v[u] = p < pb ? (double)X[(long long)perm[p] * ldx + t] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < B; ++u)
          if (p0 + 4 * u < pb) dd_add(h, lo, v[u]);
      }
      for (long long p0 = qa + lane; p0 < qb; p0 += 4 * B) {
        double v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const long long p = p0 + 4 * u;
          v[u] = p < qb ? -(double)X[(long long)perm[p] * ldx + t] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < B; ++u)
          if (p0 + 4 * u < qb) dd_add(h, lo, v[u]);
      }
    }
    sh_h[threadIdx.x] = h;
    sh_l[threadIdx.x] = lo;
    __syncthreads();
    if (lane == 0 && t < d) {
      for (int v = 1; v < 4; ++v) {
        dd_add(h, lo, sh_h[v * 64 + col]);
        lo += sh_l[v * 64 + col];
      }
      dd_norm(h, lo);
      const long long o = ((long long)sl * k + j) * d + t;
      P_hi[o] = h;
      P_lo[o] = lo;
    }
    __syncthreads();
  }
}

// grid k: S_j += the NS partials (slice order), cnt_j += moves in - moves out; with C_next, also the
// one-rank centre update C_next_j = S_j / cnt_j (an empty cluster keeps C_cur_j) and shift2_j.
__global__ __launch_bounds__(kT) void cert_apply_kernel(const double* __restrict__ P_hi,
                                                        const double* __restrict__ P_lo, int ns, int k, int d,
                                                        const int* __restrict__ seg, double* __restrict__ S_hi,
                                                        double* __restrict__ S_lo, int* __restrict__ cnt,
                                                        const double* __restrict__ C_cur, double* __restrict__ C_next,
                                                        double* __restrict__ shift2) {
  __shared__ double red[kT];
  const int j = blockIdx.x;
  const int cj = cnt[j] + (seg[j + 1] - seg[j]) - (seg[k + j + 1] - seg[k + j]);
  double sh = 0.0;
  for (int t = threadIdx.x; t < d; t += kT) {
    const long long o = (long long)j * d + t;
    double h = S_hi[o], lo = S_lo[o];
    for (int s = 0; s < ns; ++s) {
      const long long po = ((long long)s * k + j) * d + t;
      dd_add(h, lo, P_hi[po]);
      lo += P_lo[po];
    }
    dd_norm(h, lo);
    S_hi[o] = h;
    S_lo[o] = lo;
    if (C_next != nullptr) {
      const double c = cj > 0 ? h / (double)cj : C_cur[o];
      C_next[o] = c;
      const double e = c - C_cur[o];
      sh += e * e;
    }
  }
  if (C_next != nullptr && shift2 != nullptr) {
    red[threadIdx.x] = sh;
    __syncthreads();
    for (int w = kT / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) shift2[j] = red[0];
  }
  __syncthreads();
  if (threadIdx.x == 0) cnt[j] = cj;
}

}  // namespace

// C / Cold: f64 [k, d]; s, drift: f32 [k]; dtop: f32 [3]; zero: int [nz] zeroed (may be null).
CML_API int cml_kmeans_cert_stats(const double* C, const double* Cold, int k, int d, float* s, float* drift,
                                  float* dtop, int* zero, int nz, void* stream) {
  if (k <= 0 || d <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(cert_stats_kernel, dim3(k + 1), dim3(kT), 0, (hipStream_t)stream, C, Cold, k, d, s, drift, dtop,
                     zero, zero != nullptr ? nz : 0);
  return cml_status();
}

// lab int [n], u / l f32 [n]; lst int [n], count int [1] (zeroed by cert_stats).
CML_API int cml_kmeans_cert_bounds(const int* lab, float* u, float* l, const float* drift, const float* dtop,
                                   const float* s, long long n, int* lst, int* count, void* stream) {
  if (n <= 0) return 0;
  long long g = (n + kT - 1) / kT;
  g = g > 1024 ? 1024 : g;
  hipLaunchKernelGGL(cert_bounds_kernel, dim3((unsigned)g), dim3(kT), 0, (hipStream_t)stream, lab, u, l, drift, dtop,
                     s, n, lst, count);
  return cml_status();
}

// la / na: list A and its device count; lbst / nbst: list B (capacity n) and its count.
// xn / bxn / blab (all nullable together): the K9r row norms, and the compacted norm and current label of
// every list-B row (beside lbst) for the split-screen candidate pass.
CML_API int cml_kmeans_cert_tighten(const void* X, int xf64, long long n, long long ldx, int d, const double* C,
                                    const int* lab, float* u, const float* l, const float* s, const int* la,
                                    const int* na, int* lbst, int* nbst, const float* xn, float* bxn, int* blab,
                                    void* stream) {
  if (n <= 0) return 0;
  if (d <= 0) return (int)hipErrorInvalidValue;
  long long g = (n + 15) / 16;
  g = g > 1024 ? 1024 : g;
  hipStream_t st = (hipStream_t)stream;
  if (xf64)
    hipLaunchKernelGGL((cert_tighten_kernel<double>), dim3((unsigned)g), dim3(kT), 0, st, (const double*)X, ldx, d, C,
                       lab, u, l, s, la, na, lbst, nbst, xn, bxn, blab);
  else
    hipLaunchKernelGGL((cert_tighten_kernel<float>), dim3((unsigned)g), dim3(kT), 0, st, (const float*)X, ldx, d, C,
                       lab, u, l, s, la, na, lbst, nbst, xn, bxn, blab);
  return cml_status();
}

// Number of row slices of cert_delta (the partial buffers hold ns * k * d doubles each).
CML_API int cml_kmeans_cert_slices(int k) { return k >= 256 ? 4 : (k >= 64 ? 8 : 16); }

// The moves (mv_row / mv_old / mv_new, m_dev entries; capacity n) applied to the double-double sums
// S_hi / S_lo [k, d] and the int counts; hist int [2k] zeroed by cert_stats; seg int [2k + 1],
// cursor int [2k], perm int [2n]; P_hi / P_lo f64 [ns * k * d]. With C_next (one rank): the centre
// update from C_cur and shift2 f64 [k].
CML_API int cml_kmeans_cert_moves(const void* X, int xf64, long long n, long long ldx, int d, int k,
                                  const int* mv_row, const int* mv_old, const int* mv_new, const int* m_dev,
                                  int* hist, int* seg, int* cursor, int* perm, double* P_hi, double* P_lo,
                                  double* S_hi, double* S_lo, int* cnt, const double* C_cur, double* C_next,
                                  double* shift2, void* stream) {
  if (d <= 0 || k <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int ns = cml_kmeans_cert_slices(k);
  if (n > 0) {
    long long g = (n + kT - 1) / kT;
    g = g > 256 ? 256 : g;
    hipLaunchKernelGGL(cert_hist_kernel, dim3((unsigned)g), dim3(kT), (size_t)2 * k * sizeof(int), st, mv_old,
                       mv_new, m_dev, k, hist);
  }
  hipLaunchKernelGGL(cert_scan_kernel, dim3(1), dim3(64), 0, st, hist, k, seg, cursor);
  if (n > 0) {
    long long g = (n + kT - 1) / kT;
    g = g > 512 ? 512 : g;
    hipLaunchKernelGGL(cert_scatter_kernel, dim3((unsigned)g), dim3(kT), (size_t)4 * k * sizeof(int), st, mv_row,
                       mv_old, mv_new, m_dev, k, cursor, perm);
    if (xf64)
      hipLaunchKernelGGL((cert_delta_kernel<double>), dim3(k, ns), dim3(kT), 0, st, (const double*)X, ldx, d, seg,
                         perm, k, P_hi, P_lo);
    else
      hipLaunchKernelGGL((cert_delta_kernel<float>), dim3(k, ns), dim3(kT), 0, st, (const float*)X, ldx, d, seg, perm,
                         k, P_hi, P_lo);
  }
  hipLaunchKernelGGL(cert_apply_kernel, dim3(k), dim3(kT), 0, st, P_hi, P_lo, n > 0 ? ns : 0, k, d, seg, S_hi, S_lo,
                     cnt, C_cur, C_next, shift2);
  return cml_status();
}

// cb bf16 [kp, ldc] (ldc >= 3·ds), cn f32 [kp], cst f64 [3].
CML_API int cml_kmeans_split_centres(const double* C, int k, int kp, int d, int ds, void* cb, long long ldc,
                                     float* cn, double* cst, float* mc, void* stream) {
  if (k <= 0 || kp < k || d <= 0 || ds < d || ldc < 3LL * ds) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(split_centres_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, C, k, kp, d, ds, (u16*)cb, ldc,
                     cn, cst, mc);
  return cml_status();
}

// lst / cnt_dev: list B (after the split K9r candidate pass), blab its old labels; lc / nc: list C.
CML_API int cml_kmeans_cert_list(const int* lst, const int* cnt_dev, long long cap, const int* blab, int* lab, float* u,
                                 float* l, const float* ea, const float* eb, const float* en, const double* cst,
                                 int* lc, int* nc, int* mv_row, int* mv_old, int* mv_new, int* mv_count,
                                 void* stream) {
  if (cap <= 0) return 0;
  long long g = (cap + kT - 1) / kT;
  g = g > 512 ? 512 : g;
  hipLaunchKernelGGL(cert_list_kernel, dim3((unsigned)g), dim3(kT), 0, (hipStream_t)stream, lst, cnt_dev, blab, lab, u,
                     l, ea, eb, en, cst, lc, nc, mv_row, mv_old, mv_new, mv_count);
  return cml_status();
}
