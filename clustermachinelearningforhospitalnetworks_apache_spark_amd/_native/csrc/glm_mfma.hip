// K13m on MFMA: the multinomial logistic loss and C×d gradient for up to 64 classes (gfx950), and K13t, the
// multinomial model's transform. Kernels, in file order:
//   multinomial_mfma_kernel   f32 MFMAs (the first form; cml_multinomial_mfma_set_mode(1): A/B and precision
//                             reference)
//   multinomial_bf16_kernel   bf16 MFMAs on each f32 operand split into three bf16 terms, 32-class tiles of
//                             v_mfma_f32_32x32x16_bf16, the data row on the lane: the default for 17..64 classes
//   multinomial_c16_kernel    the same on a 16-class tile of v_mfma_f32_16x16x32_bf16: the default for C <= 16
//   multinomial_predict_kernel  K13t: f64 margins + softmax probabilities on v_mfma_f64_16x16x4_f64
// Measurements: profiles/r6/README.md §4, §7.
//
// The VALU form (glm.hip multinomial_grad_kernel) keeps a lane's columns of every class row in VGPRs, which
// caps it at 8 classes. Past that the work per row — 2·C·d multiply-adds for the margins, 2·C·d for the
// gradient — is matrix work: the first kernel below runs both products on v_mfma_f32_32x32x2_f32 (exact f32 products
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

// The same pass on bf16 MFMAs (v_mfma_f32_32x32x16_bf16, 16 times the f32 form's rate): every f32 operand
// is split into three bf16 terms (hi = bf16(v), mid = bf16(v - hi), lo = bf16(v - hi - mid): hi + mid + lo
// carries 24 bits, the f32 value to 2^-24), so each product is three MFMAs against the exact bf16 rows and the
// result keeps the f32 form's precision. Orientation (what makes it cheap besides the MFMA rate):
//   margins  Mᵀ = W·Xᵀ (A = W rows, B = X rows): the tile is [class][data row] with the DATA ROW on the lane,
//            so the softmax over classes is in-register (a lane's 16 classes, one exchange with lane ^ 32) —
//            the [row][class] tile of the f32 form needs 11 cross-lane steps per register; y and the weight
//            are one load per lane per tile, not one per register
//   gradient G = R·X over the tile's rows: the residual tile goes through a per-wave LDS image
//            [row][class] (three bf16 planes, 8-byte writes of 4 classes) and both operands come back with
//            ds_read_b64_tr_b16 (transposed reads): A = R [class][k = row], B = X [k = row][feature]
//   bias gradient Σ_rows R: per-lane f32 sums per register (f32 over the wave's tiles, as the gradient
//            accumulators are), reduced over the lanes once at the end
// X tiles live in a per-wave image of [DP/128][32 rows][256 B] with XOR-swizzled 16-byte chunks (conflict-free
// for the row reads of the margins and the transposed reads of the gradient).
__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)v[j];
    const float r1 = v[j] - (float)h;
    const __bf16 m = (__bf16)r1;
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)(r1 - (float)m);
  }
}

// byte offset of 16-byte chunk ch (8 features) of tile row `row` in a wave's X image
__device__ __forceinline__ int ximg_off(int row, int ch) {
  return ((ch >> 4) << 13) + (row << 8) + (((ch & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}
// element offset of 4-class chunk cc of tile row `row` in a residual plane [32 rows][32 classes] (64-B rows)
__device__ __forceinline__ int rimg_off(int row, int cc) { return (row << 5) + ((cc ^ ((row >> 1) & 7)) << 2); }

typedef short v4s __attribute__((ext_vector_type(4)));
struct v4s2 {
  v4s a, b;
};
__device__ __forceinline__ v4s tr_read(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}
__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* p0, const unsigned char* p1) {
  return __builtin_bit_cast(bf16x8, v4s2{tr_read(p0), tr_read(p1)});
}
__device__ __forceinline__ unsigned pack_bf16(__bf16 a, __bf16 b) {
  return (unsigned)__builtin_bit_cast(u16, a) | ((unsigned)__builtin_bit_cast(u16, b) << 16);
}

// e4m3 rows (F8): a 16-byte load holds 16 values; they are widened exactly to bf16 (two image chunks) when the tile
// is staged, so the MFMA passes and the image layout are the bf16 ones and HBM reads half the bytes
template <bool F8>
struct XLoad {
  static constexpr int VPL = F8 ? 16 : 8;  // values per 16-byte load
  static constexpr int ES = F8 ? 1 : 2;    // bytes per value
};
__device__ __forceinline__ void widen_e4m3(const uint4 q, uint4& lo, uint4& hi) {
  const unsigned w[4] = {q.x, q.y, q.z, q.w};
  unsigned o[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[2 * j] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[j], 1.0f, false));
    o[2 * j + 1] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[j], 1.0f, true));
  }
  lo = make_uint4(o[0], o[1], o[2], o[3]);
  hi = make_uint4(o[4], o[5], o[6], o[7]);
}

template <int CT, int FT, int FTG, bool PRESPLIT, bool F8 = false>
__global__ __launch_bounds__(kMnThreads) void multinomial_bf16_kernel(
    const void* __restrict__ Xv, long long n, long long ld, int d, int C, const double* __restrict__ y,
    const double* __restrict__ wt, const double* __restrict__ coef /*[C][d+1]*/, double* __restrict__ out, int ft0,
    int scalars) {
  constexpr int CP = 32 * CT;
  constexpr int DP = 32 * FT;
  constexpr int WP = DP + 4;  // f32 W pitch (floats)
  constexpr int BP = DP + 8;  // split-W pitch (bf16 elements, PRESPLIT)
  constexpr size_t WBYTES = PRESPLIT ? (size_t)3 * CP * BP * 2 : (size_t)CP * WP * 4;
  constexpr int XIMG = ((DP + 127) / 128) * 8192;  // bytes per wave
  constexpr int RPLANE = 32 * 32;                  // elements per residual plane
  constexpr int LCHUNK = DP / XLoad<F8>::VPL;  // 16-byte loads per row
  constexpr int LCH = 32 * LCHUNK / 64;        // loads per lane per tile
  const unsigned char* X = reinterpret_cast<const unsigned char*>(Xv);
  constexpr int ES = XLoad<F8>::ES;
  extern __shared__ __align__(16) unsigned char smem[];
  float* wf = reinterpret_cast<float*>(smem);      // [CP][WP] f32 weights, or
  __bf16* wb = reinterpret_cast<__bf16*>(smem);    // PRESPLIT: [3][CP][BP] hi, mid, lo
  float* bias_l = reinterpret_cast<float*>(smem + WBYTES);  // [CP], -inf on padded classes
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, c31 = lane & 31;
  unsigned char* xim = smem + WBYTES + CP * 4 + (size_t)wave * XIMG;
  __bf16* rim = reinterpret_cast<__bf16*>(smem + WBYTES + CP * 4 + 4 * (size_t)XIMG) + (size_t)wave * 3 * RPLANE;
  const int m_out = CP * DP + C + 2;
  double* part = out + (long long)blockIdx.x * m_out;
  if constexpr (PRESPLIT) {
    for (int i = tid; i < CP * BP; i += kMnThreads) {
      const int c = i / BP, k = i - c * BP;
      const float w = (c < C && k < d) ? (float)coef[(long long)c * (d + 1) + k] : 0.f;
      const __bf16 hi = (__bf16)w;
      const float r1 = w - (float)hi;
      const __bf16 mid = (__bf16)r1;
      wb[i] = hi;
      wb[CP * BP + i] = mid;
      wb[2 * CP * BP + i] = (__bf16)(r1 - (float)mid);
    }
  } else {
    for (int i = tid; i < CP * WP; i += kMnThreads) {
      const int c = i / WP, k = i - c * WP;
      wf[i] = (c < C && k < d) ? (float)coef[(long long)c * (d + 1) + k] : 0.f;
    }
  }
  for (int c = tid; c < CP; c += kMnThreads) bias_l[c] = c < C ? (float)coef[(long long)c * (d + 1) + d] : -__builtin_huge_valf();
  for (int i = tid; i < CP * 32 * FTG; i += kMnThreads) {
    const int c = i / (32 * FTG), f = i - c * (32 * FTG);
    part[c * DP + 32 * ft0 + f] = 0.0;
  }
  if (scalars)
    for (int i = tid; i < C + 2; i += kMnThreads) part[CP * DP + i] = 0.0;
  __syncthreads();
  f32x16v G[CT][FTG];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int t = 0; t < FTG; ++t) G[ct][t] = (f32x16v)0.f;
  float gbr[CT][16];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) gbr[ct][r] = 0.f;
  double gb[CT], loss = 0.0, wsum = 0.0;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) gb[ct] = 0.0;
  // bias-gradient partials over the lanes (rows): lane c31 < 16 keeps register c31's class
  auto flush_gb = [&]() {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float pick = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = gbr[ct][r];
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 32);
        pick = (r == (c31 & 15)) ? v : pick;
        gbr[ct][r] = 0.f;
      }
      gb[ct] += (double)pick;
    }
  };

  const long long ntiles = (n + 31) / 32;
  const long long ngroups = (ntiles + 3) / 4;
  uint4 xr[LCH];
  double ynext = 0.0, wnext = 0.0;  // the next tile's label and weight of this lane's row, loaded with its X
  auto load_tile = [&](long long tile) {
    const long long yrow = tile * 32 + c31;
    ynext = yrow < n ? y[yrow] : 0.0;
    wnext = yrow < n ? (wt != nullptr ? wt[yrow] : 1.0) : 0.0;
    if (tile * 32 + 32 <= n && d == DP) {  // a whole tile of full rows (all but the last tile): no per-load tests
      const unsigned char* base = X + tile * 32 * ld * ES;
#pragma unroll
      for (int i = 0; i < LCH; ++i) {
        const int q = lane + 64 * i, r = q / LCHUNK, ch = q - r * LCHUNK;
        xr[i] = *reinterpret_cast<const uint4*>(base + (r * ld + ch * XLoad<F8>::VPL) * ES);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LCH; ++i) {
      const int q = lane + 64 * i, r = q / LCHUNK, ch = q - r * LCHUNK;
      const long long row = tile * 32 + r;
      if (row < n && ch * XLoad<F8>::VPL < d)
        xr[i] = *reinterpret_cast<const uint4*>(X + (row * ld + ch * XLoad<F8>::VPL) * ES);
      else
        xr[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  };

  long long g = blockIdx.x;
  if (g < ngroups) load_tile(4 * g + wave);
  for (; g < ngroups; g += gridDim.x) {
    const long long tile = 4 * g + wave;
    const int ln = lane;
    const int lc = ln & 31, lh = ln >> 5;
    const float* wr = wf + lc * WP + 8 * lh;  // W[32ct + l&31][16s + 8h + j]
    const __bf16* wbr = wb + lc * BP + 8 * lh;
    // transposed-read lane roles: group G = lane >> 4 reads rows R0 + q, 4 columns from 4p (T10 addressing)
    const int trg = ln >> 4, trq = (ln >> 2) & 3, trp = ln & 3;
#pragma unroll
    for (int i = 0; i < LCH; ++i) {
      const int q = ln + 64 * i, r = q / LCHUNK, ch = q - r * LCHUNK;
      if constexpr (F8) {
        uint4 lo, hi;
        widen_e4m3(xr[i], lo, hi);
        *reinterpret_cast<uint4*>(xim + ximg_off(r, 2 * ch)) = lo;
        *reinterpret_cast<uint4*>(xim + ximg_off(r, 2 * ch + 1)) = hi;
      } else {
        *reinterpret_cast<uint4*>(xim + ximg_off(r, ch)) = xr[i];
      }
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const double yv = ynext, wv = wnext;
    if (g + gridDim.x < ngroups) load_tile(4 * (g + gridDim.x) + wave);
    // margins Mᵀ[class][row] = bias + W·Xᵀ
    f32x16v M[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 b = *reinterpret_cast<const float4*>(bias_l + 32 * ct + 8 * g4 + 4 * h);
        M[ct][4 * g4 + 0] = b.x;
        M[ct][4 * g4 + 1] = b.y;
        M[ct][4 * g4 + 2] = b.z;
        M[ct][4 * g4 + 3] = b.w;
      }
    if constexpr (PRESPLIT) {
      // software-pipelined: the LDS reads of step s + 2 go out before the MFMAs of step s (pinned with
      // sched_group_barrier: left alone, the scheduler issued each read one MFMA ahead and waited on it)
      constexpr int S = DP / 16, PD = 2, NR = 1 + 3 * CT;
      uint4 buf[PD + 1][NR];
      auto fetch = [&](int s, uint4(&b)[NR]) {
        b[0] = *reinterpret_cast<const uint4*>(xim + ximg_off(lc, 2 * s + lh));
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const __bf16* q = wbr + 32 * ct * BP + 16 * s;
          b[1 + 3 * ct] = *reinterpret_cast<const uint4*>(q);
          b[2 + 3 * ct] = *reinterpret_cast<const uint4*>(q + CP * BP);
          b[3 + 3 * ct] = *reinterpret_cast<const uint4*>(q + 2 * CP * BP);
        }
      };
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < PD && s < S; ++s) fetch(s, buf[s]);
      __builtin_amdgcn_sched_group_barrier(0x100, NR * (S < PD ? S : PD), 0);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s + PD < S) fetch(s + PD, buf[(s + PD) % (PD + 1)]);
        const uint4(&b)[NR] = buf[s % (PD + 1)];
        const bf16x8 xb = __builtin_bit_cast(bf16x8, b[0]);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          M[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, b[1 + 3 * ct]), xb, M[ct], 0, 0, 0);
          M[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, b[2 + 3 * ct]), xb, M[ct], 0, 0, 0);
          M[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, b[3 + 3 * ct]), xb, M[ct], 0, 0, 0);
        }
        if (s + PD < S) __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * CT, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        const bf16x8 xb = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(xim + ximg_off(lc, 2 * s + lh)));
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          bf16x8 bh, bm, bl;
          const float4 w0 = *reinterpret_cast<const float4*>(wr + 32 * ct * WP + 16 * s);
          const float4 w1 = *reinterpret_cast<const float4*>(wr + 32 * ct * WP + 16 * s + 4);
          const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
          split3(wv, bh, bm, bl);
          M[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, xb, M[ct], 0, 0, 0);
          M[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bm, xb, M[ct], 0, 0, 0);
          M[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl, xb, M[ct], 0, 0, 0);
        }
      }
    }
    // softmax over the classes of this lane's row (registers of both lane halves)
    const bool ok = tile * 32 + c31 < n;
    const int yc = (int)yv;
    float mx = M[0][0];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, M[ct][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float se = 0.f, my = 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = 32 * ct + acc_row(r, h);
        my += c == yc ? M[ct][r] : 0.f;
        const float e = __expf(M[ct][r] - mx);  // padded classes: margin -inf (bias), e = 0
        M[ct][r] = e;
        se += e;
      }
    se += __shfl_xor(se, 32, 64);
    my += __shfl_xor(my, 32, 64);
    const float inv = 1.f / se, wf32 = (float)wv;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = 32 * ct + acc_row(r, h);
        const float rr = wf32 * (M[ct][r] * inv - (c == yc ? 1.f : 0.f));
        M[ct][r] = rr;
        gbr[ct][r] += rr;
      }
    if (h == 0 && ok) {
      loss += wv * (((double)mx + (double)__logf(se)) - (double)my);
      wsum += wv;
    }
    // gradient: G[ct][t] += R[class][rows] · X[rows][features], one class tile at a time through the image
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {  // registers 4g4 .. 4g4+3: classes 8g4 + 4h + 0..3 of row c31
        const float rv[4] = {M[ct][4 * g4], M[ct][4 * g4 + 1], M[ct][4 * g4 + 2], M[ct][4 * g4 + 3]};
        __bf16 hi[4], mi[4], lo[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hi[j] = (__bf16)rv[j];
          const float r1 = rv[j] - (float)hi[j];
          mi[j] = (__bf16)r1;
          lo[j] = (__bf16)(r1 - (float)mi[j]);
        }
        const int o = rimg_off(lc, 2 * g4 + lh);
        *reinterpret_cast<uint2*>(rim + o) = make_uint2(pack_bf16(hi[0], hi[1]), pack_bf16(hi[2], hi[3]));
        *reinterpret_cast<uint2*>(rim + RPLANE + o) = make_uint2(pack_bf16(mi[0], mi[1]), pack_bf16(mi[2], mi[3]));
        *reinterpret_cast<uint2*>(rim + 2 * RPLANE + o) =
            make_uint2(pack_bf16(lo[0], lo[1]), pack_bf16(lo[2], lo[3]));
      }
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r0 = 16 * s + 8 * (trg >> 1) + trq;  // + 4 for the second read
        const unsigned char* ra = reinterpret_cast<const unsigned char*>(rim);
        const int oa0 = 2 * rimg_off(r0, 4 * (trg & 1) + trp), oa1 = 2 * rimg_off(r0 + 4, 4 * (trg & 1) + trp);
        const bf16x8 ah = tr_frag(ra + oa0, ra + oa1);
        const bf16x8 am = tr_frag(ra + 2 * RPLANE + oa0, ra + 2 * RPLANE + oa1);
        const bf16x8 al = tr_frag(ra + 4 * RPLANE + oa0, ra + 4 * RPLANE + oa1);
#pragma unroll
        for (int t = 0; t < FTG; ++t) {
          const int ch = 4 * (ft0 + t) + 2 * (trg & 1) + (trp >> 1);
          const bf16x8 bx = tr_frag(xim + ximg_off(r0, ch) + 8 * (trp & 1), xim + ximg_off(r0 + 4, ch) + 8 * (trp & 1));
          G[ct][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bx, G[ct][t], 0, 0, 0);
          G[ct][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bx, G[ct][t], 0, 0, 0);
          G[ct][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bx, G[ct][t], 0, 0, 0);
        }
      }
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  }
  flush_gb();
  double* pg = part + 4 * h * DP + 32 * ft0 + c31;
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
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
  loss = wave_sum_f64(loss);
  wsum = wave_sum_f64(wsum);
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
      if (c31 < 16) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int c = 32 * ct + acc_row(c31, h);
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

// C <= 16: a 16-class tile on v_mfma_f32_16x16x32_bf16 (16 cycles, half the work of a 32x32x16 MFMA): the
// 32-class tile above spends half its MFMAs on padded classes there. Same algorithm and bf16 x3 split; the
// shapes (lane l: A[i = l&15][k = 8(l>>4) + j], B[k = 8(l>>4) + j][col l&15], C/D col = l&15, row = 4(l>>4) + reg):
//   margins  Mᵀ[16 classes][16 rows] per 16-row half u of the 32-row tile: A = W (presplit planes), B = X rows
//            (one 16-byte read); a lane holds 4 classes of ONE row: the softmax is 4 registers plus two
//            exchanges (lanes l ^ 16, l ^ 32)
//   gradient G[16 classes][16 features] per feature tile t, k = the tile's 32 rows: A = R through the per-wave
//            [row][class] image (ds_read_b64_tr_b16, 32-byte rows), B = X via transposed reads of the X image
// byte offset of 16-byte chunk ch of tile row `row` in the X image of multinomial_c16_kernel: the chunk XOR is
// f(row) = 2·b0 ^ 4·b1 ^ 8·b2 ^ 9·b3 of the row's low bits (found by exhaustive search over linear swizzles:
// conflict-free for both the 16x16x32 row reads of the margins — 16 rows, two column halves — and the
// transposed gradient reads; ximg_off's XOR leaves the row reads 2-way)
__device__ __forceinline__ int ximg16_off(int row, int ch) {
  const int f = ((row & 7) << 1) ^ (((row >> 3) & 1) * 9);
  return ((ch >> 4) << 13) + (row << 8) + (((ch & 15) ^ f) << 4);
}
// element offset of row r of a residual plane of multinomial_c16_kernel
__device__ __forceinline__ int rimg16_off(int r) { return r * 16 + (r >> 3) * 64; }

template <int FT, int CTN, bool F8 = false>
__global__ __launch_bounds__(kMnThreads) void multinomial_c16_kernel(
    const void* __restrict__ Xv, long long n, long long ld, int d, int C, const double* __restrict__ y,
    const double* __restrict__ wt, const double* __restrict__ coef /*[C][d+1]*/, double* __restrict__ out) {
  constexpr int CP = 16 * CTN;  // CTN class tiles of 16
  constexpr int DP = 32 * FT;
  constexpr int BP = DP + 16;  // split-W pitch (bf16 elements): rows 8 dwords apart mod 64, so the row reads
                               // of a 16-lane group (rows r, column half g4) fall on distinct banks
  constexpr size_t WBYTES = (size_t)3 * CP * BP * 2;
  constexpr int XIMG = ((DP + 127) / 128) * 8192;  // bytes per wave
  // residual plane (one class tile at a time): [32 rows][16 classes] bf16, 32-byte rows, 64 elements (128 B) of
  // padding after every 8 rows: the two 16-lane groups of a transposed read (rows 8 apart) then take different
  // bank halves
  constexpr int RPLANE = 4 * (8 * 16 + 64);
  constexpr int LCHUNK = DP / XLoad<F8>::VPL;  // 16-byte loads per row
  constexpr int LCH = 32 * LCHUNK / 64;        // loads per lane per tile
  const unsigned char* X = reinterpret_cast<const unsigned char*>(Xv);
  constexpr int ES = XLoad<F8>::ES;
  constexpr int NT = DP / 16;                      // 16-feature gradient tiles
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* wb = reinterpret_cast<__bf16*>(smem);                  // [3][CP][BP] hi, mid, lo
  float* bias_l = reinterpret_cast<float*>(smem + WBYTES);       // [CP], -inf on padded classes
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r16 = lane & 15, g4 = lane >> 4;
  unsigned char* xim = smem + WBYTES + CP * 4 + (size_t)wave * XIMG;
  __bf16* rim = reinterpret_cast<__bf16*>(smem + WBYTES + CP * 4 + 4 * (size_t)XIMG) + (size_t)wave * 3 * RPLANE;
  double* part = out + (long long)blockIdx.x * (CP * DP + C + 2);
  for (int i = tid; i < CP * BP; i += kMnThreads) {
    const int c = i / BP, k = i - c * BP;
    const float w = (c < C && k < d) ? (float)coef[(long long)c * (d + 1) + k] : 0.f;
    const __bf16 hi = (__bf16)w;
    const float r1 = w - (float)hi;
    const __bf16 mid = (__bf16)r1;
    wb[i] = hi;
    wb[CP * BP + i] = mid;
    wb[2 * CP * BP + i] = (__bf16)(r1 - (float)mid);
  }
  for (int c = tid; c < CP; c += kMnThreads) bias_l[c] = c < C ? (float)coef[(long long)c * (d + 1) + d] : -__builtin_huge_valf();
  for (int i = tid; i < CP * DP + C + 2; i += kMnThreads) part[i] = 0.0;
  __syncthreads();
  f32x4 G[CTN][NT];
#pragma unroll
  for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
    for (int t = 0; t < NT; ++t) G[ct][t] = (f32x4)0.f;
  float gbr[CTN][4];
#pragma unroll
  for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) gbr[ct][r] = 0.f;
  double loss = 0.0, wsum = 0.0;

  const long long ntiles = (n + 31) / 32;
  const long long ngroups = (ntiles + 3) / 4;
  uint4 xr[LCH];
  double ynext[2] = {0.0, 0.0}, wnext[2] = {0.0, 0.0};  // the next tile's labels / weights of rows 16u + r16
  auto load_tile = [&](long long tile) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long long yrow = tile * 32 + 16 * u + r16;
      ynext[u] = yrow < n ? y[yrow] : 0.0;
      wnext[u] = yrow < n ? (wt != nullptr ? wt[yrow] : 1.0) : 0.0;
    }
    if (tile * 32 + 32 <= n && d == DP) {
      const unsigned char* base = X + tile * 32 * ld * ES;
#pragma unroll
      for (int i = 0; i < LCH; ++i) {
        const int q = lane + 64 * i, r = q / LCHUNK, ch = q - r * LCHUNK;
        xr[i] = *reinterpret_cast<const uint4*>(base + (r * ld + ch * XLoad<F8>::VPL) * ES);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LCH; ++i) {
      const int q = lane + 64 * i, r = q / LCHUNK, ch = q - r * LCHUNK;
      const long long row = tile * 32 + r;
      if (row < n && ch * XLoad<F8>::VPL < d)
        xr[i] = *reinterpret_cast<const uint4*>(X + (row * ld + ch * XLoad<F8>::VPL) * ES);
      else
        xr[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  const __bf16* wa = wb + r16 * BP + 8 * g4;        // W[16 ct + r16][32s + 8 g4 + j] at + 16 ct BP
  const int trq = (lane >> 2) & 3, trp = lane & 3;  // transposed reads: lane 4q + p of its 16-lane group

  long long g = blockIdx.x;
  if (g < ngroups) load_tile(4 * g + wave);
  for (; g < ngroups; g += gridDim.x) {
    const long long tile = 4 * g + wave;
#pragma unroll
    for (int i = 0; i < LCH; ++i) {
      const int q = lane + 64 * i, r = q / LCHUNK, ch = q - r * LCHUNK;
      if constexpr (F8) {
        uint4 lo, hi;
        widen_e4m3(xr[i], lo, hi);
        *reinterpret_cast<uint4*>(xim + ximg16_off(r, 2 * ch)) = lo;
        *reinterpret_cast<uint4*>(xim + ximg16_off(r, 2 * ch + 1)) = hi;
      } else {
        *reinterpret_cast<uint4*>(xim + ximg16_off(r, ch)) = xr[i];
      }
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const double yv[2] = {ynext[0], ynext[1]}, wv[2] = {wnext[0], wnext[1]};
    if (g + gridDim.x < ngroups) load_tile(4 * (g + gridDim.x) + wave);
    // margins Mᵀ[class 16 ct + 4 g4 + reg][row 16u + r16] = bias + W·Xᵀ
    f32x4 M[CTN][2];
#pragma unroll
    for (int ct = 0; ct < CTN; ++ct) {
      const float4 b = *reinterpret_cast<const float4*>(bias_l + 16 * ct + 4 * g4);
      M[ct][0] = f32x4{b.x, b.y, b.z, b.w};
      M[ct][1] = M[ct][0];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < DP / 32; ++s) {
      bf16x8 xb[2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
        xb[u] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(xim + ximg16_off(16 * u + r16, 4 * s + g4)));
#pragma unroll
      for (int ct = 0; ct < CTN; ++ct) {
        const __bf16* wc = wa + 16 * ct * BP + 32 * s;
        const bf16x8 ah = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(wc));
        const bf16x8 am = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(wc + CP * BP));
        const bf16x8 al = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(wc + 2 * CP * BP));
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          M[ct][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xb[u], M[ct][u], 0, 0, 0);
          M[ct][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, xb[u], M[ct][u], 0, 0, 0);
          M[ct][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, xb[u], M[ct][u], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // softmax over the CP classes of row 16u + r16 (4·CTN registers x lanes r16, r16 + 16, + 32, + 48); the
    // residuals replace the margins in M
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool ok = tile * 32 + 16 * u + r16 < n;
      const int yc = (int)yv[u];
      float mx = M[0][u][0];
#pragma unroll
      for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, M[ct][u][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float se = 0.f, my = 0.f;
#pragma unroll
      for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          my += (16 * ct + 4 * g4 + r == yc) ? M[ct][u][r] : 0.f;
          const float e = __expf(M[ct][u][r] - mx);  // padded classes: margin -inf (bias), e = 0
          M[ct][u][r] = e;
          se += e;
        }
      se += __shfl_xor(se, 16, 64);
      se += __shfl_xor(se, 32, 64);
      my += __shfl_xor(my, 16, 64);
      my += __shfl_xor(my, 32, 64);
      const float inv = 1.f / se, wf32 = (float)wv[u];
#pragma unroll
      for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float rr = wf32 * (M[ct][u][r] * inv - (16 * ct + 4 * g4 + r == yc ? 1.f : 0.f));
          M[ct][u][r] = rr;
          gbr[ct][r] += rr;
        }
      if (g4 == 0 && ok) {
        loss += wv[u] * (((double)mx + (double)__logf(se)) - (double)my);
        wsum += wv[u];
      }
    }
    // gradient, one class tile at a time through the residual image: G[ct][t] += R[class][rows 0..31] ·
    // X[rows][features 16t ..]; group g4 of a transposed read takes rows 8 g4 + 4 rd + q
    const int r0 = 8 * g4 + trq;
#pragma unroll
    for (int ct = 0; ct < CTN; ++ct) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // residual rows 16u + r16, classes 4 g4 .. 4 g4 + 3 -> the three planes
        __bf16 hi[4], mi[4], lo[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hi[j] = (__bf16)M[ct][u][j];
          const float r1 = M[ct][u][j] - (float)hi[j];
          mi[j] = (__bf16)r1;
          lo[j] = (__bf16)(r1 - (float)mi[j]);
        }
        const int o = rimg16_off(16 * u + r16) + 4 * g4;
        *reinterpret_cast<uint2*>(rim + o) = make_uint2(pack_bf16(hi[0], hi[1]), pack_bf16(hi[2], hi[3]));
        *reinterpret_cast<uint2*>(rim + RPLANE + o) = make_uint2(pack_bf16(mi[0], mi[1]), pack_bf16(mi[2], mi[3]));
        *reinterpret_cast<uint2*>(rim + 2 * RPLANE + o) =
            make_uint2(pack_bf16(lo[0], lo[1]), pack_bf16(lo[2], lo[3]));
      }
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const unsigned char* ra = reinterpret_cast<const unsigned char*>(rim);
      const int oa0 = 2 * (rimg16_off(r0) + 4 * trp), oa1 = 2 * (rimg16_off(r0 + 4) + 4 * trp);
      const bf16x8 ah = tr_frag(ra + oa0, ra + oa1);
      const bf16x8 am = tr_frag(ra + 2 * RPLANE + oa0, ra + 2 * RPLANE + oa1);
      const bf16x8 al = tr_frag(ra + 4 * RPLANE + oa0, ra + 4 * RPLANE + oa1);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int ch = 2 * t + (trp >> 1);
        const bf16x8 bx = tr_frag(xim + ximg16_off(r0, ch) + 8 * (trp & 1), xim + ximg16_off(r0 + 4, ch) + 8 * (trp & 1));
        G[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bx, G[ct][t], 0, 0, 0);
        G[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bx, G[ct][t], 0, 0, 0);
        G[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bx, G[ct][t], 0, 0, 0);
      }
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  }
  // bias gradient: each register's class summed over the 16 rows of the lane group
#pragma unroll
  for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) gbr[ct][r] += __shfl_xor(gbr[ct][r], o, 64);
  loss = wave_sum_f64(loss);
  wsum = wave_sum_f64(wsum);
  double* pg = part + (4 * g4) * DP + r16;
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) pg[(16 * ct + r) * DP + 16 * t] += (double)G[ct][t][r];
          __builtin_amdgcn_sched_barrier(0);
        }
      if (r16 == 0)
#pragma unroll
        for (int ct = 0; ct < CTN; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (16 * ct + 4 * g4 + r < C) part[CP * DP + 16 * ct + 4 * g4 + r] += (double)gbr[ct][r];
      if (lane == 0) {
        part[CP * DP + C] += loss;
        part[CP * DP + C + 1] += wsum;
      }
    }
    __syncthreads();
  }
}

template <int FT, int CTN>
constexpr size_t mnc16_lds() {
  return (size_t)3 * 16 * CTN * (32 * FT + 16) * 2 + 16 * CTN * 4 + (size_t)4 * ((32 * FT + 127) / 128) * 8192 +
         (size_t)4 * 3 * (4 * (8 * 16 + 64)) * 2;
}

template <int CT, int FT, bool PRESPLIT>
constexpr size_t mn16_lds() {
  return (PRESPLIT ? (size_t)3 * 32 * CT * (32 * FT + 8) * 2 : (size_t)32 * CT * (32 * FT + 4) * 4) + 32 * CT * 4 +
         (size_t)4 * ((32 * FT + 127) / 128) * 8192 + (size_t)4 * 3 * 32 * 32 * 2;
}
constexpr size_t kLdsMax = 160 * 1024;

template <int CT, int FT>
size_t mn_lds() {
  return (size_t)32 * FT * 32 * CT * 4 + (size_t)4 * 32 * (32 * FT + 2) * 2;
}

}  // namespace

int g_mn_f32 = 0;      // 1: the f32-MFMA form (A/B and precision reference)
int g_mn_nosplit = 0;  // 1: split W on the fly also where the three bf16 planes fit in LDS (A/B)
int g_mn_no16 = 0;     // 1: C <= 16 on the 32-class tile too (A/B of multinomial_c16_kernel)
// mode: 0 = bf16 three-term MFMAs (default; C <= 16 on the 16-class tile), 1 = f32 MFMAs, 2 = bf16 with W split
// on the fly, 3 = mode 0 on 32-class tiles for every C; -1 = query
CML_API int cml_multinomial_mfma_set_mode(int mode) {
  const int prev = g_mn_f32 ? 1 : (g_mn_nosplit ? 2 : (g_mn_no16 ? 3 : 0));
  if (mode >= 0) {
    g_mn_f32 = mode == 1;
    g_mn_nosplit = mode == 2;
    g_mn_no16 = mode == 3;
  }
  return prev;
}

// Supported: bf16 rows (dtype 0), d % 8 == 0, d <= 256, C <= 64 (the caller keeps the VALU kernel for C <= 8).
// Returns the class-slot count CP (32 / 64) or 0.
CML_API int cml_multinomial_mfma_supported(int d, int dtype, int C) {
  // bf16 rows (dtype 0, d % 8 == 0) or e4m3 rows (dtype 3, d % 16 == 0: whole 16-byte loads, widened to bf16 when
  // staged; not on the f32-MFMA form)
  if (d < 8 || d > 256 || C < 2 || C > 64) return 0;
  if (!(dtype == 0 && d % 8 == 0) && !(dtype == 3 && d % 16 == 0 && !g_mn_f32)) return 0;
  // multinomial_c16_kernel for C <= 16. Two 16-class tiles (CTN = 2) for 17..32 classes measured slower than the
  // 32-class tile: 14.45 vs 13.71 ms at C = 32 over 100M x 256 (profiles/r6/README.md)
  if (C <= 16 && !g_mn_f32 && !g_mn_nosplit && !g_mn_no16) return 16;
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
  if (C <= 32) return 32 * ft;  // (both tile forms)
  if (C > 32 && ft > 4) ft = ft <= 6 ? 6 : 8;
  return 32 * ft;
}

// out: [grid][CP·DP + C + 2] f64 block partials, CP = cml_multinomial_mfma_supported(...), DP = _dpad(d, C)
// (K13b: cml_partial_colsum, then the host keeps [:C, :d] of the gradient); X 16-byte aligned, ld % 8 == 0.
CML_API int cml_multinomial_mfma_grad(const void* X, long long n, long long ld, int d, int dtype, int C,
                                      const double* y, const double* wt, const double* coef, double* out, int grid,
                                      void* stream) {
  const int lq = dtype == 3 ? 16 : 8;  // values per 16-byte load: the row pitch is a whole number of them
  if (cml_multinomial_mfma_supported(d, dtype, C) == 0 || grid < 1 || n < 1 || ld % lq != 0 || ld < d ||
      (reinterpret_cast<size_t>(X) & 15) != 0)
    return (int)hipErrorInvalidValue;
  const bool f8 = dtype == 3;
  hipStream_t st = (hipStream_t)stream;
  int ft = (d + 31) / 32;
  if (cml_multinomial_mfma_supported(d, dtype, C) == 16) {  // multinomial_c16_kernel
    const int ctn = 1;
#define CML_MNC_L(FTV, CTNV, F8V)                                                                              \
  {                                                                                                            \
    constexpr size_t lds = mnc16_lds<FTV, CTNV>();                                                             \
    hipFuncSetAttribute((const void*)multinomial_c16_kernel<FTV, CTNV, F8V>,                                   \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                                 \
    hipLaunchKernelGGL((multinomial_c16_kernel<FTV, CTNV, F8V>), dim3(grid), dim3(kMnThreads), lds, st, X, n,   \
                       ld, d, C, y, wt, coef, out);                                                            \
    return cml_status();                                                                                       \
  }
#define CML_MNC(FTV, CTNV)                                                                                     \
    if (ft == FTV && ctn == CTNV) {                                                                            \
      if (f8) CML_MNC_L(FTV, CTNV, true) else CML_MNC_L(FTV, CTNV, false)                                      \
    }
    CML_MNC(1, 1) CML_MNC(2, 1) CML_MNC(3, 1) CML_MNC(4, 1) CML_MNC(5, 1) CML_MNC(6, 1) CML_MNC(7, 1) CML_MNC(8, 1)
#undef CML_MNC
#undef CML_MNC_L
    return (int)hipErrorInvalidValue;
  }
  const int ct = C <= 32 ? 1 : 2;
  if (ct == 2 && ft > 4) ft = ft <= 6 ? 6 : 8;  // padded to two launches of FT / 2 gradient tiles
  const u16* x = (const u16*)X;
#define CML_MNM(CTV, FTV, FTGV)                                                                                 \
  if (ct == CTV && ft == FTV) {                                                                                 \
    if (g_mn_f32) {                                                                                             \
      const size_t lds = mn_lds<CTV, FTV>();                                                                    \
      hipFuncSetAttribute((const void*)multinomial_mfma_kernel<CTV, FTV, FTGV>,                                 \
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                               \
      for (int f0 = 0; f0 < FTV; f0 += FTGV)                                                                    \
        hipLaunchKernelGGL((multinomial_mfma_kernel<CTV, FTV, FTGV>), dim3(grid), dim3(kMnThreads), lds, st, x,  \
                           n, ld, d, C, y, wt, coef, out, f0, f0 == 0 ? 1 : 0);                               \
    } else {                                                                                                    \
      constexpr bool PS = mn16_lds<CTV, FTV, true>() <= kLdsMax;                                                \
      if (f8) {  /* e4m3 rows: the default split only */                                                        \
        const size_t lds = mn16_lds<CTV, FTV, PS>();                                                            \
        hipFuncSetAttribute((const void*)multinomial_bf16_kernel<CTV, FTV, FTGV, PS, true>,                     \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                             \
        for (int f0 = 0; f0 < FTV; f0 += FTGV)                                                                  \
          hipLaunchKernelGGL((multinomial_bf16_kernel<CTV, FTV, FTGV, PS, true>), dim3(grid), dim3(kMnThreads),  \
                             lds, st, X, n, ld, d, C, y, wt, coef, out, f0, f0 == 0 ? 1 : 0);                 \
      } else if (PS && !g_mn_nosplit) {                                                                         \
        const size_t lds = mn16_lds<CTV, FTV, PS>();                                                            \
        hipFuncSetAttribute((const void*)multinomial_bf16_kernel<CTV, FTV, FTGV, PS>,                           \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                             \
        for (int f0 = 0; f0 < FTV; f0 += FTGV)                                                                  \
          hipLaunchKernelGGL((multinomial_bf16_kernel<CTV, FTV, FTGV, PS>), dim3(grid), dim3(kMnThreads), lds,   \
                             st, x, n, ld, d, C, y, wt, coef, out, f0, f0 == 0 ? 1 : 0);                      \
      } else {                                                                                                  \
        const size_t lds = mn16_lds<CTV, FTV, false>();                                                         \
        hipFuncSetAttribute((const void*)multinomial_bf16_kernel<CTV, FTV, FTGV, false>,                        \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                             \
        for (int f0 = 0; f0 < FTV; f0 += FTGV)                                                                  \
          hipLaunchKernelGGL((multinomial_bf16_kernel<CTV, FTV, FTGV, false>), dim3(grid), dim3(kMnThreads),     \
                             lds, st, x, n, ld, d, C, y, wt, coef, out, f0, f0 == 0 ? 1 : 0);                 \
      }                                                                                                         \
    }                                                                                                           \
    return cml_status();                                                                                        \
  }
  CML_MNM(1, 1, 1) CML_MNM(1, 2, 2) CML_MNM(1, 3, 3) CML_MNM(1, 4, 4) CML_MNM(1, 5, 5) CML_MNM(1, 6, 6)
  CML_MNM(1, 7, 7) CML_MNM(1, 8, 8)
  CML_MNM(2, 1, 1) CML_MNM(2, 2, 2) CML_MNM(2, 3, 3) CML_MNM(2, 4, 4) CML_MNM(2, 6, 3) CML_MNM(2, 8, 4)
#undef CML_MNM
  return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------------------------
// K13t: multinomial LogisticRegressionModel.transform — raw margins X·Wᵀ + b and the softmax probabilities, in
// f64 as Spark computes them (LogisticRegressionModel.predictRaw / raw2probabilityInPlace), one pass over X.
// The products run on v_mfma_f64_16x16x4_f64 (f64 accumulation; the bf16 / f32 rows convert exactly), 16 rows
// per wave tile: lane l holds A = X[row l&15][k = l>>4] and B = W[k = l>>4][class l&15]; the k index of step s
// of lane quarter kq is feature kq·K4 + s, so every lane walks a contiguous run of its row (K4 = DP/4 values,
// loaded once into registers). Results: col = class (lane&15), row = (lane>>4) + 4·reg. The softmax over a
// row's classes is a 16-lane reduction per register. W (f64, padded to 16-class blocks) lives in LDS.
namespace {

constexpr int kPtThreads = 256;
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <typename T, int K4, int CB>
__global__ __launch_bounds__(kPtThreads) void multinomial_predict_kernel(const T* __restrict__ X, long long n,
                                                                        long long ld, int d, int C,
                                                                        const double* __restrict__ coef,
                                                                        double* __restrict__ raw,
                                                                        double* __restrict__ prob) {
  constexpr int DP = 4 * K4;
  constexpr int CP = 16 * CB;
  constexpr int LDW = DP + 1;  // f64 pitch: the 16 classes of a read on distinct banks
  extern __shared__ __align__(16) unsigned char smem[];
  double* w = reinterpret_cast<double*>(smem);  // [CP][LDW]
  double* bias = w + CP * LDW;                  // [CP]
  for (int i = threadIdx.x; i < CP * LDW; i += kPtThreads) {
    const int c = i / LDW, k = i - c * LDW;
    w[i] = (c < C && k < d) ? coef[(long long)c * (d + 1) + k] : 0.0;
  }
  for (int c = threadIdx.x; c < CP; c += kPtThreads) bias[c] = c < C ? coef[(long long)c * (d + 1) + d] : 0.0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r16 = lane & 15, kq = lane >> 4;
  const long long ntiles = (n + 15) / 16;
  const double* wl = w + r16 * LDW + kq * K4;
  // the next tile's row segment is in flight (raw 16-byte loads) while this one is multiplied
  constexpr int NQ = K4 * (int)sizeof(T) / 16;  // 16-byte loads per lane per tile
  constexpr int EQ = 16 / (int)sizeof(T);       // values per load
  uint4 xq[NQ];
  auto load = [&](long long tile) {
    const long long row = tile * 16 + r16;
    const T* xr = X + row * ld + kq * K4;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      // rows 16-byte aligned with a 16-byte multiple pitch (the caller's _prep): a load that starts below d
      // stays inside the row's pitch
      const bool ok = row < n && kq * K4 + EQ * q < d;
      xq[q] = ok ? *reinterpret_cast<const uint4*>(xr + EQ * q) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  long long tile = (long long)blockIdx.x * 4 + wave;
  if (tile < ntiles) load(tile);
  for (; tile < ntiles; tile += (long long)gridDim.x * 4) {
    float xv[K4];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const unsigned wv[4] = {xq[q].x, xq[q].y, xq[q].z, xq[q].w};
#pragma unroll
      for (int e = 0; e < EQ; ++e) {
        float v;
        if constexpr (sizeof(T) == 2)
          v = __uint_as_float((e & 1) ? (wv[e >> 1] & 0xffff0000u) : (wv[e >> 1] << 16));
        else
          v = __uint_as_float(wv[e]);
        xv[EQ * q + e] = kq * K4 + EQ * q + e < d ? v : 0.f;  // the row's pad columns
      }
    }
    if (tile + (long long)gridDim.x * 4 < ntiles) load(tile + (long long)gridDim.x * 4);
    f64x4 D[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) D[cb] = (f64x4)0.0;
    // fully unrolled (xv stays in registers), in blocks of 8 steps fenced by sched_barrier so that the W reads
    // are not all hoisted to the top (K4·CB f64 values: spilled)
#pragma unroll
    for (int s0 = 0; s0 < K4; s0 += 8) {
#pragma unroll
      for (int s = s0; s < s0 + 8; ++s) {
        const double a = (double)xv[s];
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
          D[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, wl[16 * cb * LDW + s], D[cb], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // raw = D + b; softmax over the classes of each row: register reg holds row (lane>>4) + 4·reg
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const long long orow = tile * 16 + kq + 4 * reg;
      double v[CB], mx = -__builtin_huge_val();
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const int c = 16 * cb + r16;
        v[cb] = D[cb][reg] + bias[c];
        if (c < C) mx = fmax(mx, v[cb]);
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 16));
      double e[CB], se = 0.0;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        e[cb] = (16 * cb + r16 < C) ? exp(v[cb] - mx) : 0.0;
        se += e[cb];
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) se += __shfl_xor(se, o, 16);
      if (orow < n) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          const int c = 16 * cb + r16;
          if (c < C) {
            raw[orow * C + c] = v[cb];
            prob[orow * C + c] = e[cb] / se;
          }
        }
      }
    }
  }
}

}  // namespace

// K13t support: bf16 (0) or f32 (1) rows, d <= 256, C <= 64 and W in LDS. Returns the LDS bytes, 0 = unsupported.
CML_API long long cml_multinomial_predict_lds(int d, int dtype, int C) {
  if ((dtype != 0 && dtype != 1) || d < 1 || d > 256 || C < 1 || C > 64) return 0;
  const int k4 = ((d + 31) / 32) * 8, cp = 16 * ((C + 15) / 16);
  const long long lds = (long long)cp * (4 * k4 + 1) * 8 + cp * 8;
  return lds <= 160 * 1024 ? lds : 0;
}

// raw, prob: f64 [n, C] row-major; coef [C][d+1] f64 (last column the intercepts).
CML_API int cml_multinomial_predict(const void* X, long long n, long long ld, int d, int dtype, int C,
                                    const double* coef, double* raw, double* prob, int ncu, void* stream) {
  const long long lds = cml_multinomial_predict_lds(d, dtype, C);
  if (lds == 0) return (int)hipErrorInvalidValue;
  if (n <= 0) return 0;
  // the 16-byte row loads: a 16-byte aligned base and a 16-byte multiple pitch (glm_ops._prep), ld >= d
  const long long esz = dtype == 0 ? 2 : 4;
  if ((reinterpret_cast<size_t>(X) & 15) != 0 || (ld * esz) % 16 != 0 || ld < d) return (int)hipErrorInvalidValue;
  const int k4 = ((d + 31) / 32) * 8, cb = (C + 15) / 16;
  const long long tiles = (n + 15) / 16;
  const int per_cu = (int)((160 * 1024) / lds) > 0 ? (int)((160 * 1024) / lds) : 1;
  long long grid = (tiles + 3) / 4;
  const long long cap = (long long)(ncu > 0 ? ncu : 256) * (per_cu < 4 ? per_cu : 4);
  grid = grid < cap ? grid : cap;
  hipStream_t st = (hipStream_t)stream;
#define CML_MNP(TT, K4V, CBV)                                                                                  \
  if (k4 == K4V && cb == CBV) {                                                                                \
    hipFuncSetAttribute((const void*)multinomial_predict_kernel<TT, K4V, CBV>,                                \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                                \
    hipLaunchKernelGGL((multinomial_predict_kernel<TT, K4V, CBV>), dim3((unsigned)grid), dim3(kPtThreads),      \
                       (size_t)lds, st, (const TT*)X, n, ld, d, C, coef, raw, prob);                           \
    return cml_status();                                                                                       \
  }
#define CML_MNP_K(TT, K4V) CML_MNP(TT, K4V, 1) CML_MNP(TT, K4V, 2) CML_MNP(TT, K4V, 3) CML_MNP(TT, K4V, 4)
#define CML_MNP_T(TT)                                                                                          \
  CML_MNP_K(TT, 8) CML_MNP_K(TT, 16) CML_MNP_K(TT, 24) CML_MNP_K(TT, 32) CML_MNP_K(TT, 40) CML_MNP_K(TT, 48)   \
  CML_MNP_K(TT, 56) CML_MNP_K(TT, 64)
  if (dtype == 0) {
    CML_MNP_T(__bf16)
  } else {
    CML_MNP_T(float)
  }
#undef CML_MNP_T
#undef CML_MNP_K
#undef CML_MNP
  return (int)hipErrorInvalidValue;
}
