// KMeans Lloyd-iteration kernels for gfx950 (MI355X / CDNA4).
//
// Capability parity: the reference has no KMeans; this is the
// north-star workload of BASELINE.json (KMeans fit samples/sec). Kernel IDs
// follow SURVEY.md §2.5: K9 kmeans_assign, K10 kmeans_accumulate, K11 kmeans_update.
//
// K9  kmeans_assign_bf16<DS>: fused distance GEMM + argmin on MFMA.
//     * persistent grid; each workgroup stages a chunk of kc centroids (bf16,
//       XOR-swizzled 16-byte chunks => conflict-free ds_read_b128) plus their
//       squared norms in LDS ONCE and keeps them resident for the whole launch;
//     * each wave owns 32-row tiles of X; the tile is read straight from HBM into
//       VGPRs as the MFMA B operand (lane l: row l&31, k = 16s + 8(l>>5) + j);
//     * v_mfma_f32_32x32x16_bf16 computes C·Xᵀ for 32 centroids × 32 rows, so
//       the accumulator keeps the ROW on the lane and 16 centroids in registers:
//       the argmin over centroids is a per-lane compare chain plus ONE
//       cross-half exchange (lane l <-> l^32) — no LDS round trip, and the N×k
//       distance matrix is never materialised;
//     * score = ||c||² − 2·x·c; d = ||x||² + score (clamped at 0) feeds the cost;
//     * optionally (sort regime) each row also gets its rank among the rows of
//       the same label in this workgroup (LDS int counter) and the workgroup
//       writes its label histogram — the first pass of a counting sort, free.
//     Centroid sets larger than the LDS budget run as several launches over
//     centroid chunks (first/last flags carry the running argmin through HBM).
//
// K10 per-cluster sums, two race-free regimes (no float atomics in LDS: measured on
//     MI355X, ds_add_f32 ran 10-12x slower than plain race-free read-modify-write):
//   A kmeans_accum_priv<CPL,RPW> (small k·D): every (wave, row-group) owns a private
//     k×dw f32 copy in LDS; copies summed once; slabs reduced by kmeans_reduce.
//   B sort regime (large k·D): counting sort of row ids by label
//     (hist+rank from K9 -> kmeans_seg_scan -> kmeans_scatter) then
//     kmeans_segacc<CPL>: every wave streams an equal slice of the sorted order,
//     gathering whole rows (8-16 B per lane, U rows in flight) and keeping the
//     running cluster sum in f64 registers; only at cluster boundaries does it
//     flush (f64 global atomics, ~#waves+k flushes per pass). Work per wave is
//     independent of the label distribution (skew-proof).
//   Both produce ONE f64 message [k·D sums | k counts | cost] — exactly the buffer
//   that is all-reduced over RCCL.
// K11 kmeans_update: new centres (empty clusters keep their old centre, as Spark
//     MLlib does), bf16 copy, norms of the bf16 centres, per-centre squared shift.
#include "common.h"

namespace {

constexpr int kAssignThreads = 512;  // 8 waves: 2 per SIMD
constexpr int kAccumThreads = 1024;  // 16 waves
constexpr int kSegThreads = 256;     // 4 waves

template <int DS>
__device__ __forceinline__ int c_phys(int row, int c16) {
  constexpr int NCH = 2 * DS;
  constexpr int MASK = NCH >= 16 ? 15 : NCH - 1;
  return (c16 & ~MASK) | ((c16 & MASK) ^ (row & MASK));
}

template <int DS>
__global__ __launch_bounds__(kAssignThreads, 2) void kmeans_assign_bf16(
    const u16* __restrict__ X, long long n, long long ldx, const u16* __restrict__ C, long long ldc,
    int kc, int kp, int c_base, const float* __restrict__ cnorm, int* __restrict__ labels,
    float* __restrict__ best_io, int first, int last, double* __restrict__ cost_part,
    int* __restrict__ hist_out, int* __restrict__ rank_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NCH = 2 * DS;
  uint4* cl = reinterpret_cast<uint4*>(smem);
  float* cn = reinterpret_cast<float*>(smem + (size_t)kc * NCH * 16);
  int* hist = reinterpret_cast<int*>(cn + kc);
  double* red = reinterpret_cast<double*>(hist + ((kp + 3) & ~3));

  const int tid = threadIdx.x;
  for (int id = tid; id < kc * NCH; id += blockDim.x) {
    const int row = id / NCH, c16 = id - row * NCH;
    const uint4 v = *reinterpret_cast<const uint4*>(C + (long long)row * ldc + c16 * 8);
    cl[row * NCH + c_phys<DS>(row, c16)] = v;
  }
  for (int i = tid; i < kc; i += blockDim.x) cn[i] = cnorm[i];
  const bool ranking = last && rank_out != nullptr;
  if (ranking)
    for (int i = tid; i < kp; i += blockDim.x) hist[i] = 0;
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const long long ntiles = (n + 31) >> 5;
  const long long tw = (long long)gridDim.x * nwaves;
  double cost = 0.0;

  int aoff[DS];
#pragma unroll
  for (int s = 0; s < DS; ++s) aoff[s] = r * NCH + c_phys<DS>(r, 2 * s + h);

  for (long long tile = (long long)blockIdx.x * nwaves + wave; tile < ntiles; tile += tw) {
    const long long row = tile * 32 + r;
    const bool valid = row < n;
    const u16* xp = X + (valid ? row : 0) * ldx + 8 * h;
    bf16x8 xf[DS];
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      uint4 v = *reinterpret_cast<const uint4*>(xp + 16 * s);
      if (!valid) v = make_uint4(0, 0, 0, 0);
      xf[s] = __builtin_bit_cast(bf16x8, v);
    }
    float best = __builtin_huge_valf();
    int bidx = 0;
    for (int ct = 0; ct < (kc >> 5); ++ct) {
      f32x16 acc = {};
      const uint4* cb = cl + ct * 32 * NCH;
#pragma unroll
      for (int s = 0; s < DS; ++s) {
        const uint4 av = cb[aoff[s]];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av), xf[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = ct * 32 + 8 * g + 4 * h;
        const float4 c4 = *reinterpret_cast<const float4*>(cn + i0);
        const float s0 = fmaf(-2.f, acc[4 * g + 0], c4.x);
        const float s1 = fmaf(-2.f, acc[4 * g + 1], c4.y);
        const float s2 = fmaf(-2.f, acc[4 * g + 2], c4.z);
        const float s3 = fmaf(-2.f, acc[4 * g + 3], c4.w);
        if (s0 < best) { best = s0; bidx = i0 + 0; }
        if (s1 < best) { best = s1; bidx = i0 + 1; }
        if (s2 < best) { best = s2; bidx = i0 + 2; }
        if (s3 < best) { best = s3; bidx = i0 + 3; }
      }
    }
    {
      const float ob = __shfl_xor(best, 32, 64);
      const int oi = __shfl_xor(bidx, 32, 64);
      if (ob < best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    bidx += c_base;
    if (!first && valid) {
      const float pb = best_io[row];
      const int pi = labels[row];
      if (pb <= best) { best = pb; bidx = pi; }  // earlier chunks hold smaller indices
    }
    if (last) {
      float xn = 0.f;
#pragma unroll
      for (int s = 0; s < DS; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)xf[s][j];
          xn = fmaf(f, f, xn);
        }
      }
      xn += __shfl_xor(xn, 32, 64);
      const float d = fmaxf(xn + best, 0.f);
      if (h == 0 && valid) {
        labels[row] = bidx;
        best_io[row] = d;
        cost += (double)d;
        if (ranking) rank_out[row] = atomicAdd(hist + bidx, 1);
      }
    } else if (h == 0 && valid) {
      labels[row] = bidx;
      best_io[row] = best;
    }
  }
  if (last && (cost_part != nullptr || ranking)) {
    cost = wave_sum_f64(cost);
    if (lane == 0) red[wave] = cost;
    __syncthreads();
    if (tid == 0 && cost_part != nullptr) {
      double t = 0.0;
      for (int w = 0; w < nwaves; ++w) t += red[w];
      cost_part[blockIdx.x] = t;
    }
    if (ranking)
      for (int i = tid; i < kp; i += blockDim.x) hist_out[(long long)blockIdx.x * kp + i] = hist[i];
  }
}

template <int CPL>
__device__ __forceinline__ void load_cols(const u16* p, float (&v)[CPL]) {
  if constexpr (CPL == 2) {
    const unsigned w = *reinterpret_cast<const unsigned*>(p);
    v[0] = bf16_to_f32((u16)(w & 0xffffu));
    v[1] = bf16_to_f32((u16)(w >> 16));
  } else if constexpr (CPL == 4) {
    const uint2 w = *reinterpret_cast<const uint2*>(p);
    v[0] = bf16_to_f32((u16)(w.x & 0xffffu));
    v[1] = bf16_to_f32((u16)(w.x >> 16));
    v[2] = bf16_to_f32((u16)(w.y & 0xffffu));
    v[3] = bf16_to_f32((u16)(w.y >> 16));
  } else {
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = bf16_to_f32((u16)(ws[q] & 0xffffu));
      v[2 * q + 1] = bf16_to_f32((u16)(ws[q] >> 16));
    }
  }
}

// K10 regime A (small k·dw): private accumulator copy per (wave, row-group).
template <int CPL, int RPW>
__global__ __launch_bounds__(kAccumThreads) void kmeans_accum_priv(
    const u16* __restrict__ X, long long n, long long ldx, const int* __restrict__ labels, int k, int dw,
    float* __restrict__ slab, int* __restrict__ cslab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = kAccumThreads / 64;
  constexpr int LPR = 64 / RPW;
  constexpr int NC = NW * RPW;
  constexpr int U = 8;
  float* acc = reinterpret_cast<float*>(smem);                      // [NC][k][dw]
  int* cnt = reinterpret_cast<int*>(smem + (size_t)NC * k * dw * 4);  // [NC][k]
  const int tid = threadIdx.x;
  for (int i = tid; i < NC * k * dw; i += blockDim.x) acc[i] = 0.f;
  for (int i = tid; i < NC * k; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane / LPR, li = lane - sub * LPR;
  const int copy = wave * RPW + sub;
  float* wacc = acc + (size_t)copy * k * dw;
  int* wcnt = cnt + copy * k;
  const bool active = CPL * li < dw;
  const long long col0 = (long long)blockIdx.y * dw + CPL * li;
  const bool counter = blockIdx.y == 0 && li == 0;
  const long long step = (long long)gridDim.x * NW * RPW;
  for (long long r0 = ((long long)blockIdx.x * NW + wave) * RPW + sub; r0 < n; r0 += step * U) {
    float v[U][CPL];
    int lab[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + u * step;
      lab[u] = row < n ? labels[row] : -1;
      if (row < n && active) {
        load_cols<CPL>(X + row * ldx + col0, v[u]);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) v[u][j] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int l = lab[u];
      if (l >= 0) {
        if (active) {
          float* p = wacc + (size_t)l * dw + CPL * li;
#pragma unroll
          for (int j = 0; j < CPL; ++j) p[j] += v[u][j];
        }
        if (counter) wcnt[l] += 1;
      }
    }
  }
  __syncthreads();
  float* out = slab + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * (long long)k * dw;
  for (int i = tid; i < k * dw; i += blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < NC; ++c) s += acc[(size_t)c * k * dw + i];
    out[i] = s;
  }
  if (blockIdx.y == 0)
    for (int i = tid; i < k; i += blockDim.x) {
      int s = 0;
      for (int c = 0; c < NC; ++c) s += cnt[c * k + i];
      cslab[(long long)blockIdx.x * k + i] = s;
    }
}

__global__ void kmeans_reduce_kernel(const float* __restrict__ slab, const int* __restrict__ cslab,
                                     const double* __restrict__ cost_part, int gx, int ncost, int k,
                                     int D, int dsl, double* __restrict__ out) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long kd = (long long)k * D;
  if (idx < kd) {
    const int c = (int)(idx / D), d = (int)(idx - (long long)c * D);
    const int sl = d / dsl, dd = d - sl * dsl;
    const float* p = slab + (long long)sl * gx * k * dsl + (long long)c * dsl + dd;
    const long long gs = (long long)k * dsl;
    double s = 0.0;
    for (int g = 0; g < gx; ++g) s += (double)p[g * gs];
    out[idx] = s;
  } else if (idx < kd + k) {
    const int c = (int)(idx - kd);
    long long s = 0;
    for (int g = 0; g < gx; ++g) s += cslab[(long long)g * k + c];
    out[idx] = (double)s;
  } else if (idx == kd + k) {
    double s = 0.0;
    for (int i = 0; i < ncost; ++i) s += cost_part[i];
    out[idx] = s;
  }
}

// Sort regime, pass 2a: tot[c] = Σ_b hist[b][c]   (one block per cluster).
__global__ __launch_bounds__(256) void kmeans_seg_totals(const int* __restrict__ hist, int nblk, int kp,
                                                         long long* __restrict__ tot) {
  __shared__ long long ws[4];
  const int c = blockIdx.x, tid = threadIdx.x;
  long long s = 0;
  for (int b = tid; b < nblk; b += blockDim.x) s += hist[(long long)b * kp + c];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) ws[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) tot[c] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Sort regime, pass 2b (one block per cluster): seg[c] = Σ_{c'<c} tot[c'] (first sorted position of
// cluster c; seg[k] = n), off[c][b] = seg[c] + Σ_{b'<b} hist[b'][c], counts and cost into the message.
__global__ __launch_bounds__(256) void kmeans_seg_offsets(const int* __restrict__ hist, int nblk, int k, int kp,
                                                          const long long* __restrict__ tot,
                                                          const double* __restrict__ cost_part, int ncost, int D,
                                                          int* __restrict__ off, int* __restrict__ seg,
                                                          double* __restrict__ msg) {
  __shared__ long long ws[4];
  __shared__ long long carry;
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long s = 0;
  for (int i = tid; i < c; i += blockDim.x) s += tot[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) ws[wave] = s;
  __syncthreads();
  const long long base = ws[0] + ws[1] + ws[2] + ws[3];
  const long long kd = (long long)k * D;
  if (tid == 0) {
    seg[c] = (int)base;
    msg[kd + c] = (double)tot[c];
    carry = base;
    if (c == k - 1) {
      seg[k] = (int)(base + tot[c]);
      double cs = 0.0;
      for (int i = 0; i < ncost; ++i) cs += cost_part[i];
      msg[kd + k] = cs;
    }
  }
  __syncthreads();
  for (int b0 = 0; b0 < nblk; b0 += blockDim.x) {
    const int b = b0 + tid;
    const long long v = b < nblk ? hist[(long long)b * kp + c] : 0;
    long long incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    __syncthreads();
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    long long pre = carry;
    for (int w = 0; w < wave; ++w) pre += ws[w];
    if (b < nblk) off[(long long)c * nblk + b] = (int)(pre + incl - v);
    __syncthreads();
    if (tid == blockDim.x - 1) carry = pre + incl;
    __syncthreads();
  }
}

// Sort regime, pass 3: perm[off[label][block(row)] + rank[row]] = row.
__global__ void kmeans_scatter(const int* __restrict__ labels, const int* __restrict__ rank, long long n, int nblk,
                               int nwaves, const int* __restrict__ off, int* __restrict__ perm) {
  const long long tw = (long long)nblk * nwaves;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < n;
       row += (long long)gridDim.x * blockDim.x) {
    const long long tile = row >> 5;
    const int blk = (int)((tile % tw) / nwaves);
    const int lab = labels[row];
    perm[off[(long long)lab * nblk + blk] + rank[row]] = (int)row;
  }
}

template <int CPL> struct RawCols;
template <> struct RawCols<2> { using T = unsigned; };
template <> struct RawCols<4> { using T = uint2; };
template <> struct RawCols<8> { using T = uint4; };

template <int CPL>
__device__ __forceinline__ void add_raw(double (&acc)[CPL], const typename RawCols<CPL>::T& w) {
  const unsigned* ws = reinterpret_cast<const unsigned*>(&w);
#pragma unroll
  for (int q = 0; q < CPL / 2; ++q) {
    acc[2 * q] += (double)bf16_to_f32((u16)(ws[q] & 0xffffu));
    acc[2 * q + 1] += (double)bf16_to_f32((u16)(ws[q] >> 16));
  }
}

// Sort regime, pass 4: segmented sum over the label-sorted order. Wave w streams sorted
// positions [w*chunk, (w+1)*chunk): ONE vector load fetches the next U row ids, U whole-row
// gathers (CPL*2 bytes per lane) are in flight, the running sum stays in f64 registers, and
// the wave flushes (f64 global atomic add into the message) only at cluster boundaries and at
// the end of its slice. The common chunk (no boundary inside) takes an unpredicated path.
template <int CPL>
__global__ __launch_bounds__(kSegThreads) void kmeans_segacc(const u16* __restrict__ X, long long n, long long ldx,
                                                             int Dp, int D, const int* __restrict__ perm,
                                                             const int* __restrict__ seg, int k, long long chunk,
                                                             double* __restrict__ msg) {
  using raw_t = typename RawCols<CPL>::T;
  constexpr int U = 16;
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (kSegThreads / 64) + (threadIdx.x >> 6);
  const long long p0 = wave * chunk;
  if (p0 >= n) return;
  const long long p1 = p0 + chunk < n ? p0 + chunk : n;
  int lo = 0, hi = k;  // invariant: seg[lo] <= p0 < seg[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (seg[mid] <= p0) lo = mid; else hi = mid;
  }
  int c = lo;
  long long next = seg[c + 1];
  while (next <= p0) { ++c; next = seg[c + 1]; }  // skip empty clusters
  const int col = CPL * lane;
  const bool active = col < Dp;
  double acc[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) acc[j] = 0.0;
  for (long long p = p0; p < p1; p += U) {
    const int cnt = (int)(p1 - p < U ? p1 - p : U);
    const int pr = lane < cnt ? perm[p + lane] : 0;
    raw_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = __builtin_amdgcn_readlane(pr, u);
      if (u < cnt && active) {
        w[u] = *reinterpret_cast<const raw_t*>(X + row * ldx + col);
      } else {
        w[u] = raw_t{};
      }
    }
    const long long pe = p + cnt;
    if (next >= pe) {
#pragma unroll
      for (int u = 0; u < U; ++u) add_raw<CPL>(acc, w[u]);
    } else {
      long long s0 = p;
      while (true) {
        const long long se = next < pe ? next : pe;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (p + u >= s0 && p + u < se) add_raw<CPL>(acc, w[u]);
        if (se < next) break;  // chunk ends inside cluster c
        if (active) {
#pragma unroll
          for (int j = 0; j < CPL; ++j)
            if (col + j < D) atomicAdd(msg + (long long)c * D + col + j, acc[j]);
        }
#pragma unroll
        for (int j = 0; j < CPL; ++j) acc[j] = 0.0;
        ++c;
        next = seg[c + 1];
        while (next <= se && c < k - 1) { ++c; next = seg[c + 1]; }
        s0 = se;
        if (s0 >= pe) break;
      }
    }
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < CPL; ++j)
      if (col + j < D) atomicAdd(msg + (long long)c * D + col + j, acc[j]);
  }
}

// One workgroup per (padded) centre. Writes bf16 centre row (zero padded), ||c||² of the
// bf16-rounded centre (so scores are consistent with the GEMM operand) and, when
// `bufs` is given, first computes the new centre from nbuf all-reduced messages.
__global__ void kmeans_update_kernel(const double* __restrict__ bufs, int nbuf, long long bstride,
                                     int k, int D, double* __restrict__ cent, u16* __restrict__ cb,
                                     long long ldc, int Dp, float* __restrict__ cnorm,
                                     double* __restrict__ shift2) {
  __shared__ double rn[16], rs[16];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  if (c >= k) {
    for (int d = tid; d < Dp; d += blockDim.x) cb[(long long)c * ldc + d] = 0;
    if (tid == 0) cnorm[c] = __builtin_huge_valf();
    return;
  }
  double cnt = 0.0;
  if (bufs != nullptr)
    for (int b = 0; b < nbuf; ++b) cnt += bufs[b * bstride + (long long)k * D + c];
  double nrm = 0.0, sh = 0.0;
  for (int d = tid; d < Dp; d += blockDim.x) {
    if (d < D) {
      const double old = cent[(long long)c * D + d];
      double nv = old;
      if (bufs != nullptr && cnt > 0.0) {
        double s = 0.0;
        for (int b = 0; b < nbuf; ++b) s += bufs[b * bstride + (long long)c * D + d];
        nv = s / cnt;
      }
      sh += (nv - old) * (nv - old);
      cent[(long long)c * D + d] = nv;
      const u16 q = f32_to_bf16((float)nv);
      cb[(long long)c * ldc + d] = q;
      const double f = (double)bf16_to_f32(q);
      nrm += f * f;
    } else {
      cb[(long long)c * ldc + d] = 0;
    }
  }
  nrm = wave_sum_f64(nrm);
  sh = wave_sum_f64(sh);
  if (lane == 0) { rn[wave] = nrm; rs[wave] = sh; }
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < nw; ++w) { a += rn[w]; b += rs[w]; }
    cnorm[c] = (float)a;
    if (shift2 != nullptr) shift2[c] = b;
  }
}

long long assign_lds_bytes(int kc, int kp, int Dp) {
  return (long long)kc * Dp * 2 + (long long)kc * 4 + (long long)((kp + 3) & ~3) * 4 + 16 * 8;
}

template <int DS>
int launch_assign(const u16* X, long long n, long long ldx, const u16* C, long long ldc, int kc, int kp,
                  int c_base, const float* cnorm, int* labels, float* best, int first, int last,
                  double* cost_part, int* hist, int* rank, int grid, hipStream_t st) {
  const size_t lds = (size_t)assign_lds_bytes(kc, kp, 16 * DS);
  hipFuncSetAttribute((const void*)kmeans_assign_bf16<DS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kmeans_assign_bf16<DS>, dim3(grid), dim3(kAssignThreads), lds, st, X, n, ldx, C, ldc, kc, kp,
                     c_base, cnorm, labels, best, first, last, cost_part, hist, rank);
  return cml_status();
}

long long priv_lds_bytes(int k, int dw, int rpw) {
  const long long NW = kAccumThreads / 64;
  return NW * rpw * k * dw * 4 + NW * rpw * k * 4;
}

template <int CPL, int RPW>
int launch_priv(const u16* X, long long n, long long ldx, const int* labels, int k, int dw, float* slab, int* cslab,
                int gx, int nsl, hipStream_t st) {
  const size_t lds = (size_t)priv_lds_bytes(k, dw, RPW);
  hipFuncSetAttribute((const void*)kmeans_accum_priv<CPL, RPW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((kmeans_accum_priv<CPL, RPW>), dim3(gx, nsl), dim3(kAccumThreads), lds, st, X, n, ldx, labels, k,
                     dw, slab, cslab);
  return cml_status();
}

}  // namespace

CML_API long long cml_kmeans_assign_lds_bytes(int kc, int kp, int Dp) { return assign_lds_bytes(kc, kp, Dp); }
CML_API int cml_kmeans_assign_threads() { return kAssignThreads; }
CML_API int cml_kmeans_accum_threads() { return kAccumThreads; }
CML_API int cml_kmeans_seg_threads() { return kSegThreads; }
CML_API long long cml_kmeans_seg_ints(int k) { return (long long)(k + 1) + ((k + 1) & 1) + 2LL * k + 2; }

// X: bf16 [n, ldx] (Dp = 16*DS used columns, zero padded). C: bf16 [kc, ldc] (kc % 32 == 0).
// hist/rank may be null; when given (last chunk only) hist is [grid][kp] and rank is [n].
CML_API int cml_kmeans_assign_bf16(const void* X, long long n, long long ldx, int Dp, const void* C, long long ldc,
                                   int kc, int kp, int c_base, const float* cnorm, int* labels, float* best,
                                   int first, int last, double* cost_part, int* hist, int* rank, int grid,
                                   void* stream) {
  if (kc % 32 != 0 || Dp % 16 != 0 || ldx % 8 != 0 || ldc % 8 != 0) return (int)hipErrorInvalidValue;
  if ((hist == nullptr) != (rank == nullptr)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  const u16* c = (const u16*)C;
#define CML_ASSIGN(DS) \
  case DS: return launch_assign<DS>(x, n, ldx, c, ldc, kc, kp, c_base, cnorm, labels, best, first, last, cost_part, hist, rank, grid, st)
  switch (Dp / 16) {
    CML_ASSIGN(1); CML_ASSIGN(2); CML_ASSIGN(4); CML_ASSIGN(8); CML_ASSIGN(16); CML_ASSIGN(32);
    default: return (int)hipErrorInvalidValue;
  }
#undef CML_ASSIGN
}

// Regime A. rpw rows per wave-instruction, private copies; dw <= cpl*64/rpw.
CML_API long long cml_kmeans_priv_lds_bytes(int k, int dw, int rpw) { return priv_lds_bytes(k, dw, rpw); }

// Slab layout: slab[nsl][gx][k][dw] f32, cslab[gx][k] int32; nsl*dw >= Dp.
CML_API int cml_kmeans_accum_priv(const void* X, long long n, long long ldx, const int* labels, int k, int dw, int cpl,
                                  int rpw, float* slab, int* cslab, int gx, int nsl, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  if ((cpl != 2 && cpl != 4) || rpw < 1 || dw % cpl != 0 || dw > cpl * 64 / rpw) return (int)hipErrorInvalidValue;
#define CML_PRIV(C, R) if (cpl == C && rpw == R) return launch_priv<C, R>(x, n, ldx, labels, k, dw, slab, cslab, gx, nsl, st)
  CML_PRIV(2, 1); CML_PRIV(2, 2); CML_PRIV(2, 4); CML_PRIV(2, 8); CML_PRIV(2, 16);
  CML_PRIV(4, 1); CML_PRIV(4, 2); CML_PRIV(4, 4); CML_PRIV(4, 8); CML_PRIV(4, 16);
#undef CML_PRIV
  return (int)hipErrorInvalidValue;
}

CML_API int cml_kmeans_reduce(const float* slab, const int* cslab, const double* cost_part, int gx, int ncost, int k,
                              int D, int dsl, double* out, void* stream) {
  const long long total = (long long)k * D + k + 1;
  const int threads = 256;
  const long long blocks = (total + threads - 1) / threads;
  hipLaunchKernelGGL(kmeans_reduce_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, slab, cslab,
                     cost_part, gx, ncost, k, D, dsl, out);
  return cml_status();
}

// Regime B: scan + scatter + segmented accumulate. `nblk`/`nwaves` describe the assign launch
// that produced hist/rank. msg = [k*D sums | k counts | cost]. `seg` must hold k+1 ints plus
// 2k+2 ints of scratch (cml_kmeans_seg_ints).
CML_API int cml_kmeans_sort_accum(const void* X, long long n, long long ldx, int Dp, int D, const int* labels,
                                  const int* rank, const int* hist, int nblk, int nwaves, int k, int kp,
                                  const double* cost_part, int ncost, int* off, int* seg, int* perm, int cpl,
                                  int seg_grid, double* msg, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  long long* tot = reinterpret_cast<long long*>(seg + k + 1 + ((k + 1) & 1));  // scratch after seg (8-B aligned)
  hipMemsetAsync(msg, 0, sizeof(double) * (size_t)k * D, st);
  hipLaunchKernelGGL(kmeans_seg_totals, dim3(k), dim3(256), 0, st, hist, nblk, kp, tot);
  hipLaunchKernelGGL(kmeans_seg_offsets, dim3(k), dim3(256), 0, st, hist, nblk, k, kp, tot, cost_part, ncost, D, off,
                     seg, msg);
  int e = cml_status();
  if (e) return e;
  if (n == 0) return 0;
  const long long sblocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
  hipLaunchKernelGGL(kmeans_scatter, dim3((unsigned)sblocks), dim3(256), 0, st, labels, rank, n, nblk, nwaves, off,
                     perm);
  e = cml_status();
  if (e) return e;
  const long long waves = (long long)seg_grid * (kSegThreads / 64);
  const long long chunk = (n + waves - 1) / waves;
  const u16* x = (const u16*)X;
  if (cpl == 2)
    hipLaunchKernelGGL(kmeans_segacc<2>, dim3(seg_grid), dim3(kSegThreads), 0, st, x, n, ldx, Dp, D, perm, seg, k,
                       chunk, msg);
  else if (cpl == 4)
    hipLaunchKernelGGL(kmeans_segacc<4>, dim3(seg_grid), dim3(kSegThreads), 0, st, x, n, ldx, Dp, D, perm, seg, k,
                       chunk, msg);
  else if (cpl == 8)
    hipLaunchKernelGGL(kmeans_segacc<8>, dim3(seg_grid), dim3(kSegThreads), 0, st, x, n, ldx, Dp, D, perm, seg, k,
                       chunk, msg);
  else
    return (int)hipErrorInvalidValue;
  return cml_status();
}

CML_API int cml_kmeans_update(const double* bufs, int nbuf, long long bstride, int k, int D, double* cent, void* cb,
                              long long ldc, int Dp, int Kp, float* cnorm, double* shift2, void* stream) {
  hipLaunchKernelGGL(kmeans_update_kernel, dim3(Kp), dim3(256), 0, (hipStream_t)stream, bufs, nbuf, bstride, k, D,
                     cent, (u16*)cb, ldc, Dp, cnorm, shift2);
  return cml_status();
}
