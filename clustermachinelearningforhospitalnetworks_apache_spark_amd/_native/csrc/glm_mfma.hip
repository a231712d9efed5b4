// K13m on MFMA: the multinomial logistic loss and C×d gradient for up to 64 classes (gfx950).
//
// The VALU form (glm.hip multinomial_grad_kernel) keeps a lane's columns of every class row in VGPRs, which
// caps it at 8 classes. Past that the work per row — 2·C·d multiply-adds for the margins, 2·C·d for the
// gradient — is matrix work: this kernel runs both products on v_mfma_f32_32x32x2_f32 (exact f32 products
// of the bf16 rows and f32 weights / residuals, f32 accumulation: the VALU kernel's arithmetic), with X read
// from HBM once per launch:
//
//   per wave, per 32-row tile (rows staged in LDS, pitch dpad + 2 elements: the margin reads of 32 rows at one
//   column are conflict-free):
//     M[row][class] = b[class] + Σ_k X[row][k]·W[class][k]        A = X (lane: row l&31, k = 2s + l>>5),
//                                                                 B = Wᵀ (LDS, [k][class]: one f32 per lane)
//     softmax over the classes of each row (the classes of a row sit on the 32 lanes of a half, its rows on
//     the 16 accumulator registers): max / Σexp by xor shuffles, r = w·(p − [class = y]), loss += w·lse − w·m_y
//     G[class][feature] += Σ_rows r·X                             A = Rᵀ: register s of the M tile IS the A
//                                                                 operand of step s (row ρ(s, h) on lane half h),
//                                                                 B = X[ρ(s, h)][32t + l&31] from LDS
//   at the end the f32 G accumulators (AGPRs) are added, wave by wave in a fixed order, into the block's f64
//   partial — the layout K13b (partial_colsum) sums in a fixed order: the result is bitwise repeatable. The grid
//   is sized so a wave accumulates at most kWaveTiles tiles (16K rows) in f32 (an in-loop f64 flush of the
//   accumulators doubled the register demand and spilled).
//
// Class tiles CT = 1 (C <= 32) or 2 (C <= 64); feature tiles FT = dpad / 32 (dpad <= 256). A launch accumulates
// FTG of the FT gradient feature tiles (from ft0): C <= 32 takes every tile in one launch (<= 128 f32
// accumulators per lane); C > 32 with dpad > 128 runs as two launches (FTG = FT / 2: more accumulators spilled),
// each recomputing the margins from every feature (X re-read from HBM).
// Rows: bf16 with d % 8 == 0 (16-byte chunks), any row stride ld % 8 == 0.
#include "common.h"

namespace {

constexpr int kMnThreads = 256;  // 4 waves, each on its own 32-row tiles
constexpr int kWaveTiles = 512;  // f32 gradient accumulation over at most 16K rows per wave (grid sizing)

typedef float f32x16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

template <int CT, int FT, int FTG>
__global__ __launch_bounds__(kMnThreads) void multinomial_mfma_kernel(
    const u16* __restrict__ X, long long n, long long ld, int d, int C, const double* __restrict__ y,
    const double* __restrict__ wt, const double* __restrict__ coef /*[C][d+1]*/, double* __restrict__ out, int ft0,
    int scalars) {
  constexpr int CP = 32 * CT;
  constexpr int DP = 32 * FT;            // padded width
  constexpr int XP = DP + 2;             // X tile pitch (elements): conflict-free column reads
  constexpr int NCHUNK = DP / 8;         // 16-byte chunks per row
  constexpr int LCH = 32 * NCHUNK / 64;  // chunks per lane per tile
  extern __shared__ __align__(16) unsigned char smem[];
  float* wT = reinterpret_cast<float*>(smem);                       // [DP][CP] weights, transposed
  u16* xs_all = reinterpret_cast<u16*>(smem + (size_t)DP * CP * 4);  // [4 waves][32][XP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, c31 = lane & 31;
  u16* xs = xs_all + (size_t)wave * 32 * XP;
  // block partial, padded: [CP·DP gradient (class-major, DP columns) | C bias | loss | weight]
  const int m_out = CP * DP + C + 2;
  double* part = out + (long long)blockIdx.x * m_out;
  for (int i = tid; i < DP * CP; i += kMnThreads) {
    const int k = i / CP, c = i - k * CP;
    wT[i] = (c < C && k < d) ? (float)coef[(long long)c * (d + 1) + k] : 0.f;
  }
  for (int i = tid; i < CP * 32 * FTG; i += kMnThreads) {  // this launch's gradient columns
    const int c = i / (32 * FTG), f = i - c * (32 * FTG);
    part[c * DP + 32 * ft0 + f] = 0.0;
  }
  if (scalars)
    for (int i = tid; i < C + 2; i += kMnThreads) part[CP * DP + i] = 0.0;
  __syncthreads();
  float bias[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int c = 32 * ct + c31;
    bias[ct] = c < C ? (float)coef[(long long)c * (d + 1) + d] : -__builtin_huge_valf();
  }
  f32x16v G[CT][FTG];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int t = 0; t < FTG; ++t) G[ct][t] = (f32x16v)0.f;
  double gb[CT], loss = 0.0, wsum = 0.0;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) gb[ct] = 0.0;

  const long long ntiles = (n + 31) / 32;
  const long long ngroups = (ntiles + 3) / 4;
  uint4 xr[LCH];
  auto load_tile = [&](long long tile) {
#pragma unroll
    for (int i = 0; i < LCH; ++i) {
      const int q = lane + 64 * i, r = q / NCHUNK, ch = q - r * NCHUNK;
      const long long row = tile * 32 + r;
      if (row < n && ch * 8 < d)
        xr[i] = *reinterpret_cast<const uint4*>(X + row * ld + ch * 8);
      else
        xr[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  const u16* xrow = xs + c31 * XP + h;              // margin reads: row l&31, columns 2s + h
  const u16* xg = xs + 4 * h * XP + 32 * ft0 + c31;  // gradient reads: rows ρ(reg, h), column 32(ft0 + t) + l&31
  const float* wrow = wT + h * CP + c31;             // Wᵀ[2s + h][32ct + l&31]

  long long g = blockIdx.x;
  if (g < ngroups) load_tile(4 * g + wave);
  for (; g < ngroups; g += gridDim.x) {
    const long long tile = 4 * g + wave;
    // this tile's rows -> LDS (4 dwords per chunk: pitch XP keeps 4-byte alignment only)
#pragma unroll
    for (int i = 0; i < LCH; ++i) {
      const int q = lane + 64 * i, r = q / NCHUNK, ch = q - r * NCHUNK;
      unsigned* dst = reinterpret_cast<unsigned*>(xs + r * XP + ch * 8);
      dst[0] = xr[i].x;
      dst[1] = xr[i].y;
      dst[2] = xr[i].z;
      dst[3] = xr[i].w;
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (g + gridDim.x < ngroups) load_tile(4 * (g + gridDim.x) + wave);  // prefetch the next tile
    // margins: M = b + X·Wᵀ (rows on the registers, classes on the lanes)
    f32x16v M[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) M[ct] = (f32x16v)bias[ct];
#pragma unroll 4
    for (int s = 0; s < DP / 2; ++s) {
      const float a = bf16_to_f32(xrow[2 * s]);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        M[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, wrow[2 * s * CP + 32 * ct], M[ct], 0, 0, 0);
    }
    // softmax, loss, residuals (in place of the margins)
    const long long row0 = tile * 32;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const long long row = row0 + acc_row(reg, h);
      const bool ok = row < n;
      const double yv = ok ? y[row] : 0.0;
      const double wv = ok ? (wt != nullptr ? wt[row] : 1.0) : 0.0;
      const int yc = (int)yv;
      float mx = M[0][reg];
#pragma unroll
      for (int ct = 1; ct < CT; ++ct) mx = fmaxf(mx, M[ct][reg]);
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 32));
      float e[CT], se = 0.f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        e[ct] = (32 * ct + c31 < C) ? __expf(M[ct][reg] - mx) : 0.f;
        se += e[ct];
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) se += __shfl_xor(se, o, 32);
      float my = M[0][reg];
#pragma unroll
      for (int ct = 1; ct < CT; ++ct) my = (yc >> 5) == ct ? M[ct][reg] : my;
      my = __shfl(my, yc & 31, 32);
      const float inv = 1.f / se;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int c = 32 * ct + c31;
        const float r = (float)wv * (e[ct] * inv - (c == yc ? 1.f : 0.f));
        M[ct][reg] = c < C ? r : 0.f;
      }
      if (c31 == 0 && ok) {
        loss += wv * (((double)mx + (double)__logf(se)) - (double)my);
        wsum += wv;
      }
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float s = 0.f;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) s += M[ct][reg];
      gb[ct] += (double)s;
    }
    // gradient: G += Rᵀ·X over the tile's rows (register reg of R = rows ρ(reg, h)); four registers per group,
    // a scheduling barrier between groups bounds the hoisted LDS reads; one lane-variant base (xg) and
    // compile-time offsets (ds_read_u16 immediates)
#pragma unroll
    for (int rg = 0; rg < 16; rg += 4) {
#pragma unroll
      for (int reg = rg; reg < rg + 4; ++reg) {
#pragma unroll
        for (int t = 0; t < FTG; ++t) {
          const float b = bf16_to_f32(xg[((reg & 3) + 8 * (reg >> 2)) * XP + 32 * t]);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
            G[ct][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(M[ct][reg], b, G[ct][t], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tile's LDS reads done before it is rewritten
    __builtin_amdgcn_wave_barrier();
  }
  // G (f32) -> the block's f64 partial, waves in order (padded slots: no per-element conditions)
  double* pg = part + 4 * h * DP + 32 * ft0 + c31;  // this lane's base: class 4h, feature 32·ft0 + l&31
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {  // (not unrolled, one feature tile at a time: an unrolled flush spilled)
    if (wave == w) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < FTG; ++t) {
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) pg[(32 * ct + acc_row(reg, 0)) * DP + 32 * t] += (double)G[ct][t][reg];
          __builtin_amdgcn_sched_barrier(0);
        }
    }
    __syncthreads();
  }
  if (!scalars) return;
  // bias gradients (lanes l and l + 32 hold one class), loss and weight: waves in order
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) gb[ct] += __shfl_xor(gb[ct], 32, 64);
  loss = wave_sum_f64(loss);
  wsum = wave_sum_f64(wsum);
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
      if (h == 0) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int c = 32 * ct + c31;
          if (c < C) part[CP * DP + c] += gb[ct];
        }
      }
      if (lane == 0) {
        part[CP * DP + C] += loss;
        part[CP * DP + C + 1] += wsum;
      }
    }
    __syncthreads();
  }
}

template <int CT, int FT>
size_t mn_lds() {
  return (size_t)32 * FT * 32 * CT * 4 + (size_t)4 * 32 * (32 * FT + 2) * 2;
}

}  // namespace

// Supported: bf16 rows (dtype 0), d % 8 == 0, d <= 256, C <= 64 (the caller keeps the VALU kernel for C <= 8).
// Returns the class-slot count CP (32 / 64) or 0.
CML_API int cml_multinomial_mfma_supported(int d, int dtype, int C) {
  if (dtype != 0 || d < 8 || d % 8 != 0 || d > 256 || C < 2 || C > 64) return 0;
  return C <= 32 ? 32 : 64;
}

// Block count: enough blocks that a wave accumulates at most kWaveTiles 32-row tiles, at least one per CU.
CML_API int cml_multinomial_mfma_grid(long long n, int ncu) {
  const long long tiles = (n + 31) / 32;
  long long g = (tiles + 4LL * kWaveTiles - 1) / (4LL * kWaveTiles);
  if (g < ncu) g = ncu;
  const long long groups = (tiles + 3) / 4;
  if (g > groups) g = groups;
  return (int)(g < 1 ? 1 : g);
}

// Padded width DP the partials use: 32·ceil(d / 32), for C > 32 and d > 128 rounded up to 192 / 256.
CML_API int cml_multinomial_mfma_dpad(int d, int C) {
  int ft = (d + 31) / 32;
  if (C > 32 && ft > 4) ft = ft <= 6 ? 6 : 8;
  return 32 * ft;
}

// out: [grid][CP·DP + C + 2] f64 block partials, CP = cml_multinomial_mfma_supported(...), DP = _dpad(d, C)
// (K13b: cml_partial_colsum, then the host keeps [:C, :d] of the gradient); X 16-byte aligned, ld % 8 == 0.
CML_API int cml_multinomial_mfma_grad(const void* X, long long n, long long ld, int d, int C, const double* y,
                                      const double* wt, const double* coef, double* out, int grid, void* stream) {
  if (cml_multinomial_mfma_supported(d, 0, C) == 0 || grid < 1 || n < 1 || ld % 8 != 0 ||
      (reinterpret_cast<size_t>(X) & 15) != 0)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  int ft = (d + 31) / 32;
  const int ct = C <= 32 ? 1 : 2;
  if (ct == 2 && ft > 4) ft = ft <= 6 ? 6 : 8;  // padded to two launches of FT / 2 gradient tiles
  const u16* x = (const u16*)X;
#define CML_MNM(CTV, FTV, FTGV)                                                                                 \
  if (ct == CTV && ft == FTV) {                                                                                 \
    const size_t lds = mn_lds<CTV, FTV>();                                                                      \
    hipFuncSetAttribute((const void*)multinomial_mfma_kernel<CTV, FTV, FTGV>,                                   \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                                 \
    for (int f0 = 0; f0 < FTV; f0 += FTGV)                                                                      \
      hipLaunchKernelGGL((multinomial_mfma_kernel<CTV, FTV, FTGV>), dim3(grid), dim3(kMnThreads), lds, st, x, n, \
                         ld, d, C, y, wt, coef, out, f0, f0 == 0 ? 1 : 0);                                    \
    return cml_status();                                                                                        \
  }
  CML_MNM(1, 1, 1) CML_MNM(1, 2, 2) CML_MNM(1, 3, 3) CML_MNM(1, 4, 4) CML_MNM(1, 5, 5) CML_MNM(1, 6, 6)
  CML_MNM(1, 7, 7) CML_MNM(1, 8, 8)
  CML_MNM(2, 1, 1) CML_MNM(2, 2, 2) CML_MNM(2, 3, 3) CML_MNM(2, 4, 4) CML_MNM(2, 6, 3) CML_MNM(2, 8, 4)
#undef CML_MNM
  return (int)hipErrorInvalidValue;
}
