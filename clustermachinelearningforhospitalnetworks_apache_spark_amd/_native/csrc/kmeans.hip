// KMeans Lloyd-iteration kernels for gfx950 (MI355X / CDNA4).
//
// Capability parity: the reference has no KMeans; this is the
// north-star workload of BASELINE.json (KMeans fit samples/sec). Kernel IDs
// follow SURVEY.md §2.5: K9 kmeans_assign, K10 kmeans_accumulate (+reduce),
// K11 kmeans_update.
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
//     * score = ||c||² − 2·x·c; d = ||x||² + score (clamped at 0) feeds the cost.
//     Centroid sets larger than the LDS budget run as several launches over
//     centroid chunks (first/last flags carry the running argmin through HBM).
// K10 kmeans_accum_bf16<LPR>: per-cluster partial sums with LDS-privatised f32
//     accumulators (k × DSL per workgroup, D split over grid.y), conflict-free
//     ds_add_f32 (element order rotated for the upper 16 lanes of each half),
//     counts in LDS ints; one slab store per workgroup, no global atomics, so
//     the final reduction order is fixed (deterministic).
// K10b kmeans_reduce: fixed-order f64 reduction of the slabs into ONE contiguous
//     f64 message [k·D sums | k counts | cost] — exactly the buffer that is
//     all-reduced over RCCL.
// K11 kmeans_update / kmeans_pack: new centres (empty clusters keep their old
//     centre, as Spark MLlib does), bf16 copy, norms, per-centre squared shift.
#include "common.h"

namespace {

constexpr int kAssignThreads = 512;  // 8 waves: 2 per SIMD
constexpr int kAccumThreads = 1024;  // 16 waves: memory-latency hiding at 1 WG/CU

template <int DS>
__device__ __forceinline__ int c_phys(int row, int c16) {
  constexpr int NCH = 2 * DS;
  constexpr int MASK = NCH >= 16 ? 15 : NCH - 1;
  return (c16 & ~MASK) | ((c16 & MASK) ^ (row & MASK));
}

template <int DS>
__global__ __launch_bounds__(kAssignThreads, 2) void kmeans_assign_bf16(
    const u16* __restrict__ X, long long n, long long ldx, const u16* __restrict__ C, long long ldc,
    int kc, int c_base, const float* __restrict__ cnorm, int* __restrict__ labels,
    float* __restrict__ best_io, int first, int last, double* __restrict__ cost_part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NCH = 2 * DS;
  uint4* cl = reinterpret_cast<uint4*>(smem);
  float* cn = reinterpret_cast<float*>(smem + (size_t)kc * NCH * 16);
  double* red = reinterpret_cast<double*>(smem + (size_t)kc * NCH * 16 + (size_t)kc * 4);

  const int tid = threadIdx.x;
  for (int id = tid; id < kc * NCH; id += blockDim.x) {
    const int row = id / NCH, c16 = id - row * NCH;
    const uint4 v = *reinterpret_cast<const uint4*>(C + (long long)row * ldc + c16 * 8);
    cl[row * NCH + c_phys<DS>(row, c16)] = v;
  }
  for (int i = tid; i < kc; i += blockDim.x) cn[i] = cnorm[i];
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
      }
    } else if (h == 0 && valid) {
      labels[row] = bidx;
      best_io[row] = best;
    }
  }
  if (last && cost_part != nullptr) {
    cost = wave_sum_f64(cost);
    if (lane == 0) red[wave] = cost;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int w = 0; w < nwaves; ++w) t += red[w];
      cost_part[blockIdx.x] = t;
    }
  }
}

template <int LPR>
__global__ __launch_bounds__(kAccumThreads) void kmeans_accum_bf16(
    const u16* __restrict__ X, long long n, long long ldx, const int* __restrict__ labels, int k,
    float* __restrict__ slab, int* __restrict__ cslab) {
  constexpr int DSL = 2 * LPR;
  constexpr int RPW = 64 / LPR;
  constexpr int U = 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* acc = reinterpret_cast<float*>(smem);
  int* cnt = reinterpret_cast<int*>(smem + (size_t)k * DSL * 4);
  const int tid = threadIdx.x;
  for (int i = tid; i < k * DSL; i += blockDim.x) acc[i] = 0.f;
  for (int i = tid; i < k; i += blockDim.x) cnt[i] = 0;
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int sub = lane / LPR, li = lane - sub * LPR;
  const int rot = (lane >> 4) & 1;
  const long long col0 = (long long)blockIdx.y * DSL + 2 * li;
  const bool counter = (blockIdx.y == 0) && (li == 0);
  const long long step = (long long)gridDim.x * nw * RPW;
  for (long long base = ((long long)blockIdx.x * nw + wave) * RPW + sub; base < n; base += step * U) {
    unsigned v[U];
    int lab[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = base + u * step;
      const bool ok = row < n;
      v[u] = ok ? *reinterpret_cast<const unsigned*>(X + row * ldx + col0) : 0u;
      lab[u] = ok ? labels[row] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (lab[u] >= 0) {
        const float a = bf16_to_f32((u16)(v[u] & 0xffffu));
        const float b = bf16_to_f32((u16)(v[u] >> 16));
        float* p = acc + lab[u] * DSL + 2 * li;
        atomicAdd(p + rot, rot ? b : a);
        atomicAdd(p + 1 - rot, rot ? a : b);
        if (counter) atomicAdd(cnt + lab[u], 1);
      }
    }
  }
  __syncthreads();
  float* out = slab + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * (long long)k * DSL;
  for (int i = tid; i < k * DSL; i += blockDim.x) out[i] = acc[i];
  if (blockIdx.y == 0)
    for (int i = tid; i < k; i += blockDim.x) cslab[(long long)blockIdx.x * k + i] = cnt[i];
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

template <int DS>
int launch_assign(const u16* X, long long n, long long ldx, const u16* C, long long ldc, int kc,
                  int c_base, const float* cnorm, int* labels, float* best, int first, int last,
                  double* cost_part, int grid, hipStream_t st) {
  const size_t lds = (size_t)kc * 2 * DS * 16 + (size_t)kc * 4 + 16 * sizeof(double);
  hipFuncSetAttribute((const void*)kmeans_assign_bf16<DS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  hipLaunchKernelGGL(kmeans_assign_bf16<DS>, dim3(grid), dim3(kAssignThreads), lds, st, X, n, ldx, C,
                     ldc, kc, c_base, cnorm, labels, best, first, last, cost_part);
  return cml_status();
}

template <int LPR>
int launch_accum(const u16* X, long long n, long long ldx, const int* labels, int k, float* slab,
                 int* cslab, int gx, int nsl, hipStream_t st) {
  const size_t lds = (size_t)k * 2 * LPR * 4 + (size_t)k * 4;
  hipFuncSetAttribute((const void*)kmeans_accum_bf16<LPR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  hipLaunchKernelGGL(kmeans_accum_bf16<LPR>, dim3(gx, nsl), dim3(kAccumThreads), lds, st, X, n, ldx,
                     labels, k, slab, cslab);
  return cml_status();
}

}  // namespace

// Bytes of dynamic LDS the assign kernel needs for a chunk of kc centres at padded width Dp.
CML_API long long cml_kmeans_assign_lds_bytes(int kc, int Dp) {
  return (long long)kc * Dp * 2 + (long long)kc * 4 + 16 * 8;
}
CML_API int cml_kmeans_assign_threads() { return kAssignThreads; }
CML_API int cml_kmeans_accum_threads() { return kAccumThreads; }

// X: bf16 [n, ldx] (Dp = 16*DS used columns, zero padded). C: bf16 [kc, ldc] (kc % 32 == 0).
CML_API int cml_kmeans_assign_bf16(const void* X, long long n, long long ldx, int Dp, const void* C,
                                   long long ldc, int kc, int c_base, const float* cnorm, int* labels,
                                   float* best, int first, int last, double* cost_part, int grid,
                                   void* stream) {
  if (kc % 32 != 0 || Dp % 16 != 0 || ldx % 8 != 0 || ldc % 8 != 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  const u16* c = (const u16*)C;
  switch (Dp / 16) {
    case 1: return launch_assign<1>(x, n, ldx, c, ldc, kc, c_base, cnorm, labels, best, first, last, cost_part, grid, st);
    case 2: return launch_assign<2>(x, n, ldx, c, ldc, kc, c_base, cnorm, labels, best, first, last, cost_part, grid, st);
    case 4: return launch_assign<4>(x, n, ldx, c, ldc, kc, c_base, cnorm, labels, best, first, last, cost_part, grid, st);
    case 8: return launch_assign<8>(x, n, ldx, c, ldc, kc, c_base, cnorm, labels, best, first, last, cost_part, grid, st);
    case 16: return launch_assign<16>(x, n, ldx, c, ldc, kc, c_base, cnorm, labels, best, first, last, cost_part, grid, st);
    case 32: return launch_assign<32>(x, n, ldx, c, ldc, kc, c_base, cnorm, labels, best, first, last, cost_part, grid, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// Slab layout: slab[nsl][gx][k][dsl] f32, cslab[gx][k] int32. dsl = 2*lpr, nsl*dsl >= Dp.
CML_API int cml_kmeans_accum_bf16(const void* X, long long n, long long ldx, const int* labels, int k,
                                  int lpr, float* slab, int* cslab, int gx, int nsl, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  switch (lpr) {
    case 1: return launch_accum<1>(x, n, ldx, labels, k, slab, cslab, gx, nsl, st);
    case 2: return launch_accum<2>(x, n, ldx, labels, k, slab, cslab, gx, nsl, st);
    case 4: return launch_accum<4>(x, n, ldx, labels, k, slab, cslab, gx, nsl, st);
    case 8: return launch_accum<8>(x, n, ldx, labels, k, slab, cslab, gx, nsl, st);
    case 16: return launch_accum<16>(x, n, ldx, labels, k, slab, cslab, gx, nsl, st);
    case 32: return launch_accum<32>(x, n, ldx, labels, k, slab, cslab, gx, nsl, st);
    case 64: return launch_accum<64>(x, n, ldx, labels, k, slab, cslab, gx, nsl, st);
    default: return (int)hipErrorInvalidValue;
  }
}

CML_API int cml_kmeans_reduce(const float* slab, const int* cslab, const double* cost_part, int gx,
                              int ncost, int k, int D, int dsl, double* out, void* stream) {
  const long long total = (long long)k * D + k + 1;
  const int threads = 256;
  const long long blocks = (total + threads - 1) / threads;
  hipLaunchKernelGGL(kmeans_reduce_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream,
                     slab, cslab, cost_part, gx, ncost, k, D, dsl, out);
  return cml_status();
}

CML_API int cml_kmeans_update(const double* bufs, int nbuf, long long bstride, int k, int D,
                              double* cent, void* cb, long long ldc, int Dp, int Kp, float* cnorm,
                              double* shift2, void* stream) {
  hipLaunchKernelGGL(kmeans_update_kernel, dim3(Kp), dim3(256), 0, (hipStream_t)stream, bufs, nbuf,
                     bstride, k, D, cent, (u16*)cb, ldc, Dp, cnorm, shift2);
  return cml_status();
}
