// Source-precision KMeans kernels: the f64 reference algorithm on device-resident f32/f64 features.
//
// The reference's feature vectors are DoubleType/IntegerType columns assembled into f64 vectors
// (ref.py:64-72, ref.py:134-136) and Spark's KMeans works in f64. The bf16 MFMA path rounds rows to
// 8 mantissa bits (a hospital occupancy of 387 becomes 388), so for f32/f64 input the engine runs
// these kernels instead (models/kmeans.py, precision "exact"; cml.ml.kmeans.precision = bf16 opts
// into the fast path):
//
//   exact_assign   label/distance of every row against f64 centres: one thread per row, centres
//                  staged in LDS tiles, distances as a dimension-ordered fold of (x_t - c_t)² in f64,
//                  ties to the lowest centre index;
//   exact_segsum   per-cluster f64 sums of the rows in label-sorted order (a stable sort of the
//                  labels): fixed 1024-position chunks summed sequentially, chunk partials of the
//                  clusters crossing a chunk edge combined in chunk order — deterministic, no atomics.
#include "common.h"
#include "exact_util.h"

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 1024;  // sorted positions per segmented-sum chunk

// idx / n_dev (both null, or both set): assign only the rows idx[0 .. *n_dev) — the rows the bf16
// screen could not certify (precision "screen"); labels / best land at the real rows.
template <typename T, int DREG>
__global__ __launch_bounds__(kThreads) void exact_assign_kernel(const T* __restrict__ X, long long n, long long ldx,
                                                                int d, const double* __restrict__ C, int k, int kt,
                                                                int* __restrict__ labels, double* __restrict__ best,
                                                                int* __restrict__ changed,
                                                                const int* __restrict__ idx,
                                                                const int* __restrict__ n_dev) {
  extern __shared__ __align__(16) unsigned char smem[];
  double* ct = reinterpret_cast<double*>(smem);  // [kt][d]
  const long long t0 = (long long)blockIdx.x * kThreads + threadIdx.x;
  const long long cnt = n_dev != nullptr ? (long long)*n_dev : n;
  if ((long long)blockIdx.x * kThreads >= cnt) return;  // a whole block past the list (block-uniform)
  const bool live = t0 < cnt && t0 < n;
  const long long r = live ? (idx != nullptr ? (long long)idx[t0] : t0) : 0;
  double xr[DREG > 0 ? DREG : 1];
  if constexpr (DREG > 0) {
#pragma unroll
    for (int t = 0; t < DREG; ++t) xr[t] = (live && t < d) ? (double)X[r * ldx + t] : 0.0;
  }
  double bd = __builtin_huge_val();
  int bi = 0;
  for (int c0 = 0; c0 < k; c0 += kt) {
    const int kc = min(kt, k - c0);
    __syncthreads();
    for (int e = threadIdx.x; e < kc * d; e += kThreads) ct[e] = C[(long long)c0 * d + e];
    __syncthreads();
    if (live) {
      for (int j = 0; j < kc; ++j) {
        const double* cj = ct + (long long)j * d;
        double acc = 0.0;
        if constexpr (DREG > 0) {
#pragma unroll
          for (int t = 0; t < DREG; ++t) {
            if (t < d) {
              const double e = xr[t] - cj[t];
              acc = __fma_rn(e, e, acc);
            }
          }
        } else {
          for (int t = 0; t < d; ++t) {
            const double e = (double)X[r * ldx + t] - cj[t];
            acc = __fma_rn(e, e, acc);
          }
        }
        if (acc < bd) {  // centres ascending: strict < keeps the lowest index
          bd = acc;
          bi = c0 + j;
        }
      }
    }
  }
  if (live) {
    if (changed != nullptr && labels[r] != bi) atomicAdd(changed, 1);
    labels[r] = bi;
    best[r] = bd;
  }
}

// Wide rows (d > 16): the same per-centre fold (t ascending, fma from 0.0, strict < over centres in
// index order — the same bits as exact_assign_kernel and the host twin). Dimensions outer, KG centre
// accumulators live in registers: each row is read once per KG centres and every LDS centre value
// (a wave-uniform broadcast) feeds 64 rows' f64 fma — VALU-bound at the f64 rate. The LDS tile is
// zero-padded to a DC multiple of dimensions and a KG multiple of centres (a zero term adds +0.0 to a
// non-negative fold: the same bits). Rows: grid-stride over n or over idx[0 .. *n_dev).
// Optional outputs: ub / lb = f32 bounds (outward-rounded) of the real distance to the label and to
// every other centre (the fold's top-2); mv_* = (row, old label, new label) of the rows whose label
// changed, appended (mv_count) — the certified pruned step's moves (kmeans_cert.hip).
template <typename T, int KG, int DC>
__global__ __launch_bounds__(kThreads) void exact_assign_wide_kernel(
    const T* __restrict__ X, long long n, long long ldx, int d, const double* __restrict__ C, int k, int kt,
    int* __restrict__ labels, double* __restrict__ best, int* __restrict__ changed, const int* __restrict__ idx,
    const int* __restrict__ n_dev, float* __restrict__ ub, float* __restrict__ lb, int* __restrict__ mv_row,
    int* __restrict__ mv_old, int* __restrict__ mv_new, int* __restrict__ mv_count, bool vec) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ int s_w[kThreads / 64 + 1];
  double* ct = reinterpret_cast<double*>(smem);  // [round_up(kt, KG)][dpad]
  const int dpad = (d + DC - 1) / DC * DC;
  const int ktp = (kt + KG - 1) / KG * KG;
  long long cnt = n_dev != nullptr ? (long long)*n_dev : n;
  cnt = cnt < n ? cnt : n;
  const bool single = k <= kt;
  auto load_tile = [&](int c0, int kc) {
    for (int e = threadIdx.x; e < ktp * dpad; e += kThreads) {
      const int j = e / dpad, t = e - j * dpad;
      ct[e] = (j < kc && t < d) ? C[(long long)(c0 + j) * d + t] : 0.0;
    }
  };
  if (single) {
    load_tile(0, k);
    __syncthreads();
  }
  // the block's 256 rows are staged DC dimensions at a time through a transposed LDS tile (coalesced
  // 32-B row segments; a thread-per-row walk of the rows read 64 scattered segments per load and ran a
  // few-centre pass at 0.4 TB/s), each thread folding its own row from it — the same fold order
  __shared__ T xs[DC * (kThreads + 1)];
  __shared__ long long rows_s[kThreads];
  for (long long base = (long long)blockIdx.x * kThreads; base < cnt; base += (long long)gridDim.x * kThreads) {
    const long long t0 = base + threadIdx.x;
    const bool live = t0 < cnt;
    const long long r = live ? (idx != nullptr ? (long long)idx[t0] : t0) : 0;
    __syncthreads();  // rows_s / xs of the previous base are no longer read
    rows_s[threadIdx.x] = live ? r : -1;
    double bd = __builtin_huge_val(), sd = __builtin_huge_val();
    int bi = 0;
    for (int c0 = 0; c0 < k; c0 += kt) {
      const int kc = min(kt, k - c0);
      if (!single) {
        __syncthreads();
        load_tile(c0, kc);
        __syncthreads();
      }
      for (int j0 = 0; j0 < kc; j0 += KG) {
        double acc[KG];
#pragma unroll
        for (int a = 0; a < KG; ++a) acc[a] = 0.0;
        for (int tb = 0; tb < dpad; tb += DC) {
          __syncthreads();
          if (vec && tb + DC <= d) {  // 16-B loads (4 f32 / 2 f64 dimensions of a row each)
            constexpr int V = 16 / sizeof(T);
            for (int e = threadIdx.x; e < kThreads * (DC / V); e += kThreads) {
              const int rr = e / (DC / V), tv = (e - rr * (DC / V)) * V;
              const long long row = rows_s[rr];
              T v[V];
              if (row >= 0) {
                const uint4 q4 = *reinterpret_cast<const uint4*>(X + row * ldx + tb + tv);
                __builtin_memcpy(v, &q4, 16);
              } else {
#pragma unroll
                for (int u = 0; u < V; ++u) v[u] = (T)0;
              }
#pragma unroll
              for (int u = 0; u < V; ++u) xs[(tv + u) * (kThreads + 1) + rr] = v[u];
            }
          } else {
            for (int e = threadIdx.x; e < kThreads * DC; e += kThreads) {
              const int rr = e / DC, tt = e - rr * DC;
              const long long row = rows_s[rr];
              xs[tt * (kThreads + 1) + rr] = (row >= 0 && tb + tt < d) ? X[row * ldx + tb + tt] : (T)0;
            }
          }
          __syncthreads();
          double xv[DC];
#pragma unroll
          for (int u = 0; u < DC; ++u) xv[u] = (double)xs[u * (kThreads + 1) + threadIdx.x];
#pragma unroll
          for (int a = 0; a < KG; ++a) {
            const double* cj = ct + (long long)(j0 + a) * dpad + tb;
#pragma unroll
            for (int u = 0; u < DC; ++u) {
              const double e = xv[u] - cj[u];
              acc[a] = __fma_rn(e, e, acc[a]);
            }
          }
        }
        if (live) {
#pragma unroll
          for (int a = 0; a < KG; ++a) {
            if (j0 + a < kc) {  // centres ascending: strict < keeps the lowest index
              const double v = acc[a];
              if (v < bd) {
                sd = bd;
                bd = v;
                bi = c0 + j0 + a;
              } else if (v < sd) {
                sd = v;
              }
            }
          }
        }
      }
    }
    int old = 0;
    if (live) {
      old = labels[r];
      if (changed != nullptr && old != bi) atomicAdd(changed, 1);
      labels[r] = bi;
      if (best != nullptr) best[r] = bd;
      if (ub != nullptr) {
        ub[r] = f32_up(sqrt(bd) * (1.0 + kFoldMargin));
        lb[r] = k > 1 ? f32_dn(sqrt(sd) * (1.0 - kFoldMargin)) : __builtin_huge_valf();
      }
    }
    if (mv_count != nullptr) {  // block-uniform
      const int pos = block_append<kThreads>(live && old != bi, mv_count, s_w);
      if (pos >= 0) {
        mv_row[pos] = (int)r;
        mv_old[pos] = old;
        mv_new[pos] = bi;
      }
    }
  }
}

// best[r] = the f64 fold Σ_t (x_t - c_lab,t)² of exact_assign_kernel for row r against its label's
// centre only (the same operations in the same order, so the same bits as the full assignment's
// minimum when the label is the argmin): the distances of rows the bf16 screen certified, the lazy cost.
// One thread per row folds from LDS: the block's 256 rows are staged 16 dimensions at a time through a
// transposed LDS tile with coalesced 64-B row segments (a thread-per-row walk of the rows straight from
// HBM read 64 rows x 4 B per load: 0.7 TB/s), and so are the labels' centre columns when the centres fit.
constexpr int kDistCh = 16;
template <typename T>
__global__ __launch_bounds__(kThreads) void exact_dist_kernel(const T* __restrict__ X, long long n, long long ldx,
                                                              int d, const double* __restrict__ C, int kc,
                                                              const int* __restrict__ labels, long long lab_off,
                                                              double* __restrict__ best, bool vec) {
  __shared__ T xs[kDistCh * (kThreads + 1)];
  extern __shared__ __align__(16) unsigned char smem[];
  double* cs = reinterpret_cast<double*>(smem);  // [kc][kDistCh] when kc > 0
  const long long r0 = (long long)blockIdx.x * kThreads;
  const long long r = r0 + threadIdx.x;
  const bool live = r < n;
  const long long j = live ? (long long)labels[r] - lab_off : 0;
  const double* cj = C + j * d;
  double acc = 0.0;
  if (vec && d % kDistCh == 0) {
    // every chunk full: 16-B loads with the next chunk's loads in flight (registers) while the block folds
    // the current one from LDS
    constexpr int V = 16 / sizeof(T);
    constexpr int Q = kDistCh / V;  // 16-B loads per thread per chunk
    uint4 q[Q];
    auto issue = [&](int t0) {
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        const int e = threadIdx.x + i * kThreads;
        const int rr = e / Q, tv = (e - rr * Q) * V;
        const long long row = r0 + rr;
        q[i] = row < n ? *reinterpret_cast<const uint4*>(X + row * ldx + t0 + tv) : uint4{0u, 0u, 0u, 0u};
      }
    };
    issue(0);
    for (int t0 = 0; t0 < d; t0 += kDistCh) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        const int e = threadIdx.x + i * kThreads;
        const int rr = e / Q, tv = (e - rr * Q) * V;
        T v[V];
        __builtin_memcpy(v, &q[i], 16);
#pragma unroll
        for (int u = 0; u < V; ++u) xs[(tv + u) * (kThreads + 1) + rr] = v[u];
      }
      if (kc > 0)
        for (int e = threadIdx.x; e < kc * kDistCh; e += kThreads) {
          const int jj = e / kDistCh, tt = e - jj * kDistCh;
          cs[e] = C[(long long)jj * d + t0 + tt];
        }
      if (t0 + kDistCh < d) issue(t0 + kDistCh);
      __syncthreads();
      if (live) {
        const double* cc = kc > 0 ? cs + j * kDistCh : cj + t0;
#pragma unroll
        for (int tt = 0; tt < kDistCh; ++tt) {
          const double e = (double)xs[tt * (kThreads + 1) + threadIdx.x] - cc[tt];
          acc = __fma_rn(e, e, acc);
        }
      }
    }
    if (live) best[r] = acc;
    return;
  }
  for (int t0 = 0; t0 < d; t0 += kDistCh) {
    const int dc = min(kDistCh, d - t0);
    __syncthreads();
    if (vec && dc == kDistCh) {  // 16-B loads: 4 (f32) / 2 (f64) dimensions of a row per load
      constexpr int V = 16 / sizeof(T);
      for (int e = threadIdx.x; e < kThreads * (kDistCh / V); e += kThreads) {
        const int rr = e / (kDistCh / V), tv = (e - rr * (kDistCh / V)) * V;
        const long long row = r0 + rr;
        T v[V];
        if (row < n) {
          const uint4 q = *reinterpret_cast<const uint4*>(X + row * ldx + t0 + tv);
          __builtin_memcpy(v, &q, 16);
        } else {
#pragma unroll
          for (int u = 0; u < V; ++u) v[u] = (T)0;
        }
#pragma unroll
        for (int u = 0; u < V; ++u) xs[(tv + u) * (kThreads + 1) + rr] = v[u];
      }
    } else {
      for (int e = threadIdx.x; e < kThreads * kDistCh; e += kThreads) {
        const int rr = e / kDistCh, tt = e - rr * kDistCh;
        const long long row = r0 + rr;
        xs[tt * (kThreads + 1) + rr] = (row < n && tt < dc) ? X[row * ldx + t0 + tt] : (T)0;
      }
    }
    if (kc > 0)
      for (int e = threadIdx.x; e < kc * kDistCh; e += kThreads) {
        const int jj = e / kDistCh, tt = e - jj * kDistCh;
        cs[e] = tt < dc ? C[(long long)jj * d + t0 + tt] : 0.0;
      }
    __syncthreads();
    if (live) {
      if (kc > 0) {
        const double* cc = cs + j * kDistCh;
        for (int tt = 0; tt < dc; ++tt) {
          const double e = (double)xs[tt * (kThreads + 1) + threadIdx.x] - cc[tt];
          acc = __fma_rn(e, e, acc);
        }
      } else {
        for (int tt = 0; tt < dc; ++tt) {
          const double e = (double)xs[tt * (kThreads + 1) + threadIdx.x] - cj[t0 + tt];
          acc = __fma_rn(e, e, acc);
        }
      }
    }
  }
  if (live) best[r] = acc;
}

// Source rows -> the bf16 copy the MFMA screen reads (RNE, zero-padded to ldo) and err[r] >= ||x_r -
// bf16(x_r)|| (the f64 norm of the rounding, rounded up to f32): the certificate's per-row slack. One
// wave per row.
template <typename T>
__global__ __launch_bounds__(kThreads) void to_bf16_err_kernel(const T* __restrict__ X, long long n, long long ldx,
                                                               int d, u16* __restrict__ out, long long ldo,
                                                               float* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const long long w0 = ((long long)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * kThreads) >> 6;
  for (long long r = w0; r < n; r += nw) {
    double e2 = 0.0;
    for (int t = lane; t < ldo; t += 64) {
      u16 b = 0;
      if (t < d) {
        const double v = (double)X[r * ldx + t];
        b = f32_to_bf16((float)v);  // f64 -> f32 -> bf16: a double rounding, covered by the exact error below
        const double e = v - (double)bf16_to_f32(b);
        e2 = __fma_rn(e, e, e2);
      }
      out[r * ldo + t] = b;
    }
    e2 = wave_sum_f64(e2);
    if (lane == 0) err[r] = (float)(sqrt(e2) * (1.0 + 1e-6)) + 1e-30f;
  }
}

// Split screen (d <= 170): row r -> [hi | lo | hi] in three ds-wide segments of a zero-padded bf16 row
// (hi = bf16(x), lo = bf16(x - hi)), so that against centres laid out [c_hi | c_hi | c_lo] the MFMA dot is
// hi·c_hi + lo·c_hi + hi·c_lo: x·c to ~2^-16 instead of ~2^-8 (the plain screen left ~24 % of k-means‖
// rows inside the bf16 error band on same-blob candidates). Per row: ea = ||lo||, eb = ||x - hi - lo||,
// en = ||x|| (f32, rounded up) and xn = ||x||² (f32, the K9r row norm).
template <typename T>
__global__ __launch_bounds__(kThreads) void to_bf16_split_kernel(const T* __restrict__ X, long long n, long long ldx,
                                                                 int d, int ds, u16* __restrict__ out, long long ldo,
                                                                 float* __restrict__ ea, float* __restrict__ eb,
                                                                 float* __restrict__ en, float* __restrict__ xn,
                                                                 bool vec) {
  // 16 lanes per row (4 rows per wave); a lane owns 8-dimension groups: one 16-B store per segment
  // (ds and ldo multiples of 8, checked at launch), the three norms reduced over the 16 lanes
  const int lane = threadIdx.x & 63, q = lane & 15;
  const long long g0 = ((long long)blockIdx.x * kThreads + threadIdx.x) >> 4;
  const long long ng = ((long long)gridDim.x * kThreads) >> 4;
  const long long rounds = (n + ng - 1) / ng;  // every lane runs the same number of rounds (shuffles)
  for (long long it = 0; it < rounds; ++it) {
    const long long r = g0 + it * ng;
    const bool live = r < n;
    double a2 = 0.0, b2 = 0.0, n2 = 0.0;
    if (live) {
      uint4* o = reinterpret_cast<uint4*>(out + r * ldo);
      for (int t0 = 8 * q; t0 < ds; t0 += 128) {
        unsigned wh[4] = {0u, 0u, 0u, 0u}, wl[4] = {0u, 0u, 0u, 0u};
        T xv8[8];
        if (vec && t0 + 8 <= d) {  // 16-B loads of the lane's 8 values
#pragma unroll
          for (int h = 0; h < (int)(8 * sizeof(T) / 16); ++h) {
            const uint4 q4 = *reinterpret_cast<const uint4*>(X + r * ldx + t0 + h * (16 / (int)sizeof(T)));
            __builtin_memcpy(&xv8[h * (16 / sizeof(T))], &q4, 16);
          }
        } else {
#pragma unroll
          for (int u = 0; u < 8; ++u) xv8[u] = t0 + u < d ? X[r * ldx + t0 + u] : (T)0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int t = t0 + u;
          if (t < d) {
            const double v = (double)xv8[u];
            const u16 hb = f32_to_bf16((float)v);
            const double r1 = v - (double)bf16_to_f32(hb);
            const u16 lb = f32_to_bf16((float)r1);
            const double lv = (double)bf16_to_f32(lb);
            const double rx = r1 - lv;
            a2 = __fma_rn(lv, lv, a2);
            b2 = __fma_rn(rx, rx, b2);
            n2 = __fma_rn(v, v, n2);
            wh[u >> 1] |= (unsigned)hb << (16 * (u & 1));
            wl[u >> 1] |= (unsigned)lb << (16 * (u & 1));
          }
        }
        const uint4 h4 = {wh[0], wh[1], wh[2], wh[3]}, l4 = {wl[0], wl[1], wl[2], wl[3]};
        o[t0 / 8] = h4;
        o[(ds + t0) / 8] = l4;
        o[(2 * ds + t0) / 8] = h4;
      }
      const uint4 z = {0u, 0u, 0u, 0u};
      for (long long t0 = 3LL * ds + 8 * q; t0 < ldo; t0 += 128) o[t0 / 8] = z;
    }
#pragma unroll
    for (int m = 8; m > 0; m >>= 1) {
      a2 += __shfl_xor(a2, m, 16);
      b2 += __shfl_xor(b2, m, 16);
      n2 += __shfl_xor(n2, m, 16);
    }
    if (live && q == 0) {
      ea[r] = f32_up(sqrt(a2) * (1.0 + 1e-6));
      eb[r] = f32_up(sqrt(b2) * (1.0 + 1e-6) + 1e-300);
      en[r] = f32_up(sqrt(n2) * (1.0 + 1e-6));
      xn[r] = (float)n2;
    }
  }
}

// Split-screen certificate: with cst = {max ||c_lo||, max ||c||, max ||c - c_hi - c_lo||} the squared
// distances of the split model differ from the real ones by at most E = 2(ea·cst0 + eb·cst1 +
// 1.01·en·cst2) per row; the label is certified when sqrt(lb² - E) > sqrt(ub² + E), and u_out / l_out
// get those bounds (rounded outward).
__global__ __launch_bounds__(kThreads) void screen_cert_split_kernel(
    const float* __restrict__ ub, const float* __restrict__ lb, const float* __restrict__ ea,
    const float* __restrict__ eb, const float* __restrict__ en, const double* __restrict__ cst, long long n,
    int* __restrict__ lst, int* __restrict__ count, float* __restrict__ u_out, float* __restrict__ l_out) {
  __shared__ int buf[kBuf];
  __shared__ int nb, base;
  if (threadIdx.x == 0) nb = 0;
  ListBuf lbf{buf, &nb, &base};
  const double c0 = cst[0], c1 = cst[1], c2 = cst[2];
  for (long long i0 = (long long)blockIdx.x * kThreads; i0 < n; i0 += (long long)gridDim.x * kThreads) {
    __syncthreads();
    const long long i = i0 + threadIdx.x;
    bool bad = false;
    if (i < n) {
      const double e = 2.0 * ((double)ea[i] * c0 + (double)eb[i] * c1 + 1.01 * (double)en[i] * c2) * (1.0 + 1e-6);
      const double ubi = (double)ub[i], lbi = (double)lb[i];
      const float uu = f32_up(sqrt(ubi * ubi + e) * (1.0 + kFoldMargin));
      const float ll = f32_dn(sqrt(fmax(lbi * lbi - e, 0.0)) * (1.0 - kFoldMargin));
      bad = !(uu < ll);
      u_out[i] = uu;
      l_out[i] = ll;
      if (bad) buf[atomicAdd(&nb, 1)] = (int)i;
    }
    list_flush<kThreads>(lbf, lst, count, false);
  }
  list_flush<kThreads>(lbf, lst, count, true);
}

// Rows whose bf16-screen label is not certified (kmeans_screen_cert) are appended to lst (count
// zeroed by the caller): certified when lb - ub > 2·(err_r + ecmax), ub / lb the K9r top-2 bounds
// of the bf16 distances (their f32 rounding already inside) and ecmax >= max_j ||c_j - bf16(c_j)||:
// then every other centre is farther than the label's in exact arithmetic too, so the f64 argmin
// is the same label (no tie).
// One reservation per block and 1024-row tile (the list order is free: exact_assign writes every listed
// row at its own position): a per-wave atomic on the single counter serialised ~n/64 atomics in L2 when
// many rows were uncertified (1.6 ms per 10M-row pass; now ~n/1024 of them).
constexpr int kCertQ = 4;  // rows per thread per tile
__global__ __launch_bounds__(kThreads) void screen_cert_kernel(const float* __restrict__ ub,
                                                               const float* __restrict__ lb,
                                                               const float* __restrict__ err,
                                                               const double* __restrict__ ecmax, long long n,
                                                               int* __restrict__ lst, int* __restrict__ count,
                                                               float* __restrict__ u_out, float* __restrict__ l_out) {
  __shared__ int wtot[kThreads / 64][kCertQ];
  __shared__ int base_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double ec = *ecmax;
  constexpr long long kTile = (long long)kThreads * kCertQ;
  for (long long i0 = (long long)blockIdx.x * kTile; i0 < n; i0 += (long long)gridDim.x * kTile) {
    unsigned long long bal[kCertQ];
#pragma unroll
    for (int q = 0; q < kCertQ; ++q) {
      const long long i = i0 + (long long)q * kThreads + threadIdx.x;
      bool bad = false;
      if (i < n) {
        const double ubi = (double)ub[i], lbi = (double)lb[i], e = (double)err[i] + ec;
        bad = !(lbi - ubi > 2.0 * e * (1.0 + 1e-9) + 1e-300);
        if (u_out != nullptr) {  // real-distance bounds of the screened label (overwritten for listed rows)
          u_out[i] = f32_up((ubi + e) * (1.0 + kFoldMargin));
          l_out[i] = f32_dn((lbi - e) * (1.0 - kFoldMargin));
        }
      }
      bal[q] = __ballot(bad);
      if (lane == 0) wtot[w][q] = (int)__popcll(bal[q]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int q = 0; q < kCertQ; ++q)
        for (int v = 0; v < kThreads / 64; ++v) tot += wtot[v][q];
      base_s = tot ? atomicAdd(count, tot) : 0;
    }
    __syncthreads();
    int off = base_s;  // this wave's entries of tile q follow every earlier (q, wave) in (q, wave) order
#pragma unroll
    for (int q = 0; q < kCertQ; ++q) {
      for (int v = 0; v < kThreads / 64; ++v) off += (v < w) ? wtot[v][q] : 0;
      if ((bal[q] >> lane) & 1ull)
        lst[off + __popcll(bal[q] & ((1ull << lane) - 1ull))] = (int)(i0 + (long long)q * kThreads + threadIdx.x);
      for (int v = w; v < kThreads / 64; ++v) off += wtot[v][q];
    }
    __syncthreads();  // wtot / base_s reused by the next tile
  }
}

// seg[c] = first sorted position of cluster c (seg[k] = n); perm[p] = row at sorted position p.
// Chunk ch covers positions [ch*kChunk, ...): clusters strictly inside it are stored complete into
// S / S_lo (normalised double-double); the cluster open at its start goes to slot 2ch, the one open at
// its end (if another) to slot 2ch+1 (hi in slots, lo in slots + 2·nch·d).
template <typename T>
__global__ __launch_bounds__(256) void exact_seg_partial_kernel(const T* __restrict__ X, long long ldx, int d,
                                                               const int* __restrict__ perm,
                                                               const int* __restrict__ seg, int k, long long n,
                                                               double* __restrict__ S, double* __restrict__ S_lo,
                                                               double* __restrict__ slots, int* __restrict__ slot_c) {
  const long long ch = blockIdx.x;
  const long long nch = gridDim.x;
  double* slots_lo = slots + 2 * nch * (long long)d;
  const int col = blockIdx.y * blockDim.x + threadIdx.x;  // one block spans up to 256 columns: whole-row reads
  const long long p0 = ch * kChunk, p1 = min(n, p0 + kChunk);
  int lo_ = 0, hi_ = k;  // seg[lo_] <= p0 < seg[hi_]
  while (hi_ - lo_ > 1) {
    const int mid = (lo_ + hi_) >> 1;
    if (seg[mid] <= p0) lo_ = mid; else hi_ = mid;
  }
  int c = lo_;
  while (seg[c + 1] <= p0) ++c;  // skip empty clusters
  const int ca = c;
  double ah = 0.0, al = 0.0;
  long long next = seg[c + 1];
  auto store = [&](double* dh, double* dl) {
    dd_norm(ah, al);
    *dh = ah;
    *dl = al;
  };
  // PF positions' rows are loaded before any of them is added: the adds' latency chain no longer
  // serialises the gathers
  constexpr int PF = 8;
  for (long long pb = p0; pb < p1; pb += PF) {
    double v[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const long long p = pb + u;
      v[u] = (p < p1 && col < d) ? (double)X[(long long)perm[p] * ldx + col] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const long long p = pb + u;
      if (p >= p1) break;
      while (p >= next) {  // cluster c ended: first one -> slot A, a middle one is complete
        if (col < d) {
          if (c == ca) store(slots + (2 * ch) * (long long)d + col, slots_lo + (2 * ch) * (long long)d + col);
          else store(S + (long long)c * d + col, S_lo + (long long)c * d + col);
        }
        ah = 0.0;
        al = 0.0;
        ++c;
        next = seg[c + 1];
      }
      if (col < d) dd_add(ah, al, v[u]);
    }
  }
  if (col < d) {
    const long long sl = c == ca ? 2 * ch : 2 * ch + 1;
    store(slots + sl * (long long)d + col, slots_lo + sl * (long long)d + col);
  }
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    slot_c[2 * ch] = ca;
    slot_c[2 * ch + 1] = c == ca ? -1 : c;
  }
}

// S[c] for the clusters that touch a chunk edge: the slot partials (double-double) in chunk order.
__global__ __launch_bounds__(kThreads) void exact_seg_fix_kernel(const int* __restrict__ seg, int k, int d,
                                                                 long long nch, double* __restrict__ S,
                                                                 double* __restrict__ S_lo,
                                                                 const double* __restrict__ slots,
                                                                 const int* __restrict__ slot_c) {
  const int c = blockIdx.x;
  const long long s0 = seg[c], s1 = seg[c + 1];
  const double* slots_lo = slots + 2 * nch * (long long)d;
  if (s1 <= s0) {
    for (int t = threadIdx.x; t < d; t += kThreads) {
      S[(long long)c * d + t] = 0.0;
      S_lo[(long long)c * d + t] = 0.0;
    }
    return;
  }
  const long long ch0 = s0 / kChunk, ch1 = (s1 - 1) / kChunk;
  bool edge = false;
  for (long long ch = ch0; ch <= ch1; ++ch) edge |= slot_c[2 * ch] == c || slot_c[2 * ch + 1] == c;
  if (!edge) return;  // complete inside one chunk: stored by the partial kernel
  for (int t = threadIdx.x; t < d; t += kThreads) {
    double h = 0.0, l = 0.0;
    for (long long ch = ch0; ch <= ch1; ++ch) {
      for (int q = 0; q < 2; ++q) {
        if (slot_c[2 * ch + q] == c) {
          dd_add(h, l, slots[(2 * ch + q) * (long long)d + t]);
          l += slots_lo[(2 * ch + q) * (long long)d + t];
        }
      }
    }
    dd_norm(h, l);
    S[(long long)c * d + t] = h;
    S_lo[(long long)c * d + t] = l;
  }
}

// Correctly rounded sum of an f64 vector in two launches: every block folds a contiguous range in
// double-double (threads strided, then the block's partials in thread order), one block folds the block
// partials in block order (the result is exact whenever the inputs' exponents span < ~2^80, and always
// deterministic). The exact paths' trainingCost (kmeans_ops.sum_exact).
constexpr int kSumBlocks = 1024;
__global__ __launch_bounds__(kThreads) void sum_dd_partial_kernel(const double* __restrict__ v, long long n,
                                                                  double* __restrict__ part) {
  __shared__ double sh[kThreads], sl[kThreads];
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long a = (long long)blockIdx.x * per, b = min(n, a + per);
  double h = 0.0, l = 0.0;
  for (long long i = a + threadIdx.x; i < b; i += kThreads) dd_add(h, l, v[i]);
  sh[threadIdx.x] = h;
  sl[threadIdx.x] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    double H = 0.0, L = 0.0;
    for (int t = 0; t < kThreads; ++t) {
      dd_add(H, L, sh[t]);
      L += sl[t];
    }
    dd_norm(H, L);
    part[2 * blockIdx.x] = H;
    part[2 * blockIdx.x + 1] = L;
  }
}

__global__ __launch_bounds__(64) void sum_dd_final_kernel(const double* __restrict__ part, int nb,
                                                          double* __restrict__ out) {
  if (threadIdx.x == 0) {
    double H = 0.0, L = 0.0;
    for (int i = 0; i < nb; ++i) {
      dd_add(H, L, part[2 * i]);
      L += part[2 * i + 1];
    }
    dd_norm(H, L);
    out[0] = H;
  }
}

}  // namespace

// X: f64 (xf64 = 1) or f32 rows [n, ldx elements]; C: f64 [k, d]; labels (int32, read for the change
// count when `changed` is given) and best (f64) [n].
// idx / n_dev: see exact_assign_kernel (n is then the capacity of idx, the grid covers it).
template <typename T, int KG>
static void launch_wide(const T* X, long long n, long long ldx, int d, const double* C, int k, int* labels,
                        double* best, int* changed, const int* idx, const int* n_dev, float* ub, float* lb,
                        int* mv_row, int* mv_old, int* mv_new, int* mv_count, hipStream_t st) {
  constexpr int DC = 8;
  const int dpad = (d + DC - 1) / DC * DC;
  int kt = (8192 / dpad) / KG * KG;  // centres per LDS tile (<= 64 KiB)
  kt = kt < KG ? KG : kt;
  const int kneed = (k + KG - 1) / KG * KG;  // no tile larger than the centres need
  kt = kt < kneed ? kt : kneed;
  const int ktp = kt;
  const size_t lds = (size_t)ktp * dpad * sizeof(double);
  // static LDS (the staged rows, their ids, the append scratch) counts against the same budget
  const size_t stat = (size_t)DC * (kThreads + 1) * sizeof(T) + kThreads * sizeof(long long) + 64;
  if (lds + stat > 65536)
    (void)hipFuncSetAttribute((const void*)exact_assign_wide_kernel<T, KG, DC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  long long blocks = (n + kThreads - 1) / kThreads;
  if (idx != nullptr) blocks = blocks < 4096 ? blocks : 4096;  // grid-stride over the listed rows
  const bool vec = ((uintptr_t)X % 16 == 0) && ((ldx * (long long)sizeof(T)) % 16 == 0);
  hipLaunchKernelGGL((exact_assign_wide_kernel<T, KG, DC>), dim3((unsigned)blocks), dim3(kThreads), lds, st, X, n,
                     ldx, d, C, k, kt, labels, best, changed, idx, n_dev, ub, lb, mv_row, mv_old, mv_new, mv_count,
                     vec);
}

template <typename T>
static void launch_wide_any(const T* X, long long n, long long ldx, int d, const double* C, int k, int* labels,
                            double* best, int* changed, const int* idx, const int* n_dev, float* ub, float* lb,
                            int* mv_row, int* mv_old, int* mv_new, int* mv_count, hipStream_t st) {
  const int dpad = (d + 7) / 8 * 8;
  if (k <= 4 && dpad <= 2048)  // few centres: no zero-padded accumulators
    launch_wide<T, 4>(X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, ub, lb, mv_row, mv_old, mv_new,
                      mv_count, st);
  else if (k <= 8 && dpad <= 1024)
    launch_wide<T, 8>(X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, ub, lb, mv_row, mv_old, mv_new,
                      mv_count, st);
  else if (dpad <= 256 && k > 16)
    launch_wide<T, 32>(X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, ub, lb, mv_row, mv_old, mv_new,
                       mv_count, st);
  else if (dpad <= 512)
    launch_wide<T, 16>(X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, ub, lb, mv_row, mv_old, mv_new,
                       mv_count, st);
  else if (dpad <= 1024)
    launch_wide<T, 8>(X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, ub, lb, mv_row, mv_old, mv_new,
                      mv_count, st);
  else
    launch_wide<T, 1>(X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, ub, lb, mv_row, mv_old, mv_new,
                      mv_count, st);
}

// X: f64 (xf64 = 1) or f32 rows [n, ldx elements]; C: f64 [k, d]; labels (int32, read for the change
// count when `changed` is given) and best (f64) [n].
// idx / n_dev: see exact_assign_kernel (n is then the capacity of idx, the grid covers it).
CML_API int cml_kmeans_exact_assign(const void* X, int xf64, long long n, long long ldx, int d, const double* C,
                                    int k, int* labels, double* best, int* changed, const int* idx, const int* n_dev,
                                    void* stream) {
  if (n <= 0) return 0;
  if (d <= 0 || k <= 0 || ((idx == nullptr) != (n_dev == nullptr))) return (int)hipErrorInvalidValue;
  const int kt = max(1, min(k, 8192 / d));  // centres per LDS tile (<= 64 KiB)
  const size_t lds = (size_t)kt * d * sizeof(double);
  const dim3 g((unsigned)((n + kThreads - 1) / kThreads));
  hipStream_t st = (hipStream_t)stream;
#define CML_EA(T, R)                                                                                        \
  hipLaunchKernelGGL((exact_assign_kernel<T, R>), g, dim3(kThreads), lds, st, (const T*)X, n, ldx, d, C, k, kt, \
                     labels, best, changed, idx, n_dev)
  if (xf64) {
    if (d <= 4) CML_EA(double, 4);
    else if (d <= 16) CML_EA(double, 16);
    else launch_wide_any<double>((const double*)X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, nullptr,
                                 nullptr, nullptr, nullptr, nullptr, nullptr, st);
  } else {
    if (d <= 4) CML_EA(float, 4);
    else if (d <= 16) CML_EA(float, 16);
    else launch_wide_any<float>((const float*)X, n, ldx, d, C, k, labels, best, changed, idx, n_dev, nullptr,
                                nullptr, nullptr, nullptr, nullptr, nullptr, st);
  }
#undef CML_EA
  return cml_status();
}

// The certified step's full re-assignment (any d): the wide fold (same bits as exact_assign) over
// idx[0 .. *n_dev) writing labels, optional best, the f32 top-2 bounds ub / lb and the move list.
CML_API int cml_kmeans_exact_top2(const void* X, int xf64, long long n, long long ldx, int d, const double* C, int k,
                                  int* labels, double* best, const int* idx, const int* n_dev, float* ub, float* lb,
                                  int* mv_row, int* mv_old, int* mv_new, int* mv_count, void* stream) {
  if (n <= 0) return 0;
  if (d <= 0 || k <= 0 || ub == nullptr || lb == nullptr || ((idx == nullptr) != (n_dev == nullptr)) ||
      ((mv_count == nullptr) != (mv_row == nullptr)))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (xf64)
    launch_wide_any<double>((const double*)X, n, ldx, d, C, k, labels, best, nullptr, idx, n_dev, ub, lb, mv_row,
                            mv_old, mv_new, mv_count, st);
  else
    launch_wide_any<float>((const float*)X, n, ldx, d, C, k, labels, best, nullptr, idx, n_dev, ub, lb, mv_row,
                           mv_old, mv_new, mv_count, st);
  return cml_status();
}

// labels[r] - lab_off indexes C (f64 [kc, d]; kc = 0: unknown, the centres are read from global memory).
CML_API int cml_kmeans_exact_dist(const void* X, int xf64, long long n, long long ldx, int d, const double* C, int kc,
                                  const int* labels, long long lab_off, double* best, void* stream) {
  if (n <= 0) return 0;
  if (d <= 0) return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)((n + kThreads - 1) / kThreads));
  hipStream_t st = (hipStream_t)stream;
  if ((size_t)kc * kDistCh * sizeof(double) > 32768) kc = 0;
  const size_t lds = (size_t)kc * kDistCh * sizeof(double);
  const size_t esz = xf64 ? 8 : 4;
  const bool vec = ((uintptr_t)X % 16 == 0) && ((ldx * esz) % 16 == 0);
  if (xf64)
    hipLaunchKernelGGL((exact_dist_kernel<double>), g, dim3(kThreads), lds, st, (const double*)X, n, ldx, d, C, kc,
                       labels, lab_off, best, vec);
  else
    hipLaunchKernelGGL((exact_dist_kernel<float>), g, dim3(kThreads), lds, st, (const float*)X, n, ldx, d, C, kc,
                       labels, lab_off, best, vec);
  return cml_status();
}

// out: bf16 [n, ldo] (ldo >= d, padding zeroed), err: f32 [n].
CML_API int cml_kmeans_to_bf16_err(const void* X, int xf64, long long n, long long ldx, int d, void* out,
                                   long long ldo, float* err, void* stream) {
  if (n <= 0) return 0;
  if (d <= 0 || ldo < d) return (int)hipErrorInvalidValue;
  long long g = (n + 3) / 4;
  g = g > 8192 ? 8192 : g;
  hipStream_t st = (hipStream_t)stream;
  if (xf64)
    hipLaunchKernelGGL((to_bf16_err_kernel<double>), dim3((unsigned)g), dim3(kThreads), 0, st, (const double*)X, n,
                       ldx, d, (u16*)out, ldo, err);
  else
    hipLaunchKernelGGL((to_bf16_err_kernel<float>), dim3((unsigned)g), dim3(kThreads), 0, st, (const float*)X, n,
                       ldx, d, (u16*)out, ldo, err);
  return cml_status();
}

// lst: int [n] (n entries at most), count: int [1] zeroed by the caller; ecmax: f64 device scalar.
// u_out / l_out (nullable, may alias ub / lb): f32 bounds of the real distance to the screened label
// and to every other centre, ub + err + ecmax and lb - err - ecmax rounded outward.
CML_API int cml_kmeans_screen_cert(const float* ub, const float* lb, const float* err, const double* ecmax,
                                   long long n, int* lst, int* count, float* u_out, float* l_out, void* stream) {
  if (n <= 0) return 0;
  long long g = (n + kThreads * kCertQ - 1) / (kThreads * kCertQ);
  g = g > 2048 ? 2048 : (g < 1 ? 1 : g);
  hipLaunchKernelGGL(screen_cert_kernel, dim3((unsigned)g), dim3(kThreads), 0, (hipStream_t)stream, ub, lb, err,
                     ecmax, n, lst, count, u_out, l_out);
  return cml_status();
}

// Slot scratch: slots f64 [4 * nchunks * d] (hi then lo), slot_c int [2 * nchunks], nchunks = ceil(n / 1024).
CML_API long long cml_kmeans_exact_chunks(long long n) { return (n + kChunk - 1) / kChunk; }

// S = the correctly rounded per-cluster sums (double-double accumulation), S_lo = the remainders
// (S + S_lo = the exact sum; the rank fold of a multi-rank fit adds them).
CML_API int cml_kmeans_exact_segsum(const void* X, int xf64, long long ldx, int d, const int* perm, const int* seg,
                                    int k, long long n, double* S, double* S_lo, double* slots, int* slot_c,
                                    void* stream) {
  if (d <= 0 || k <= 0 || S_lo == nullptr) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const long long nch = n > 0 ? (n + kChunk - 1) / kChunk : 0;
  if (n > 0) {
    // threads per block = columns per block: a row's columns in one block (rounded to a wave), so each
    // gathered row is one contiguous read instead of 64-column pieces
    const int bt = d <= 64 ? 64 : (d <= 128 ? 128 : 256);
    const dim3 g((unsigned)nch, (unsigned)((d + bt - 1) / bt));
    if (xf64)
      hipLaunchKernelGGL((exact_seg_partial_kernel<double>), g, dim3(bt), 0, st, (const double*)X, ldx, d, perm, seg,
                         k, n, S, S_lo, slots, slot_c);
    else
      hipLaunchKernelGGL((exact_seg_partial_kernel<float>), g, dim3(bt), 0, st, (const float*)X, ldx, d, perm, seg,
                         k, n, S, S_lo, slots, slot_c);
  }
  hipLaunchKernelGGL(exact_seg_fix_kernel, dim3(k), dim3(kThreads), 0, st, seg, k, d, nch, S, S_lo, slots, slot_c);
  return cml_status();
}

// out: bf16 [n, ldo] with ldo >= 3·ds, ds >= d; ea / eb / en / xn: f32 [n].
CML_API int cml_kmeans_to_bf16_split(const void* X, int xf64, long long n, long long ldx, int d, int ds, void* out,
                                     long long ldo, float* ea, float* eb, float* en, float* xn, void* stream) {
  if (n <= 0) return 0;
  if (d <= 0 || ds < d || ldo < 3LL * ds || (ds % 8) || (ldo % 8)) return (int)hipErrorInvalidValue;
  long long g = (n + 15) / 16;
  g = g > 8192 ? 8192 : g;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = ((uintptr_t)X % 16 == 0) && ((ldx * (xf64 ? 8 : 4)) % 16 == 0);
  if (xf64)
    hipLaunchKernelGGL((to_bf16_split_kernel<double>), dim3((unsigned)g), dim3(kThreads), 0, st, (const double*)X, n,
                       ldx, d, ds, (u16*)out, ldo, ea, eb, en, xn, vec);
  else
    hipLaunchKernelGGL((to_bf16_split_kernel<float>), dim3((unsigned)g), dim3(kThreads), 0, st, (const float*)X, n,
                       ldx, d, ds, (u16*)out, ldo, ea, eb, en, xn, vec);
  return cml_status();
}

// cst: f64 [3] device; lst int [n], count int [1] zeroed by the caller; u_out / l_out f32 [n] (may be ub / lb).
CML_API int cml_kmeans_screen_cert_split(const float* ub, const float* lb, const float* ea, const float* eb,
                                         const float* en, const double* cst, long long n, int* lst, int* count,
                                         float* u_out, float* l_out, void* stream) {
  if (n <= 0) return 0;
  long long g = (n + kThreads - 1) / kThreads;
  g = g > 2048 ? 2048 : g;
  hipLaunchKernelGGL(screen_cert_split_kernel, dim3((unsigned)g), dim3(kThreads), 0, (hipStream_t)stream, ub, lb, ea,
                     eb, en, cst, n, lst, count, u_out, l_out);
  return cml_status();
}

// out: f64 [1]; part: f64 scratch [2 * kSumBlocks].
CML_API int cml_kmeans_sum_dd(const double* v, long long n, double* out, double* part, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  long long nb = (n + kThreads * 16 - 1) / (kThreads * 16);
  nb = nb < 1 ? 1 : (nb > kSumBlocks ? kSumBlocks : nb);
  hipLaunchKernelGGL(sum_dd_partial_kernel, dim3((unsigned)nb), dim3(kThreads), 0, st, v, n, part);
  hipLaunchKernelGGL(sum_dd_final_kernel, dim3(1), dim3(64), 0, st, part, (int)nb, out);
  return cml_status();
}
