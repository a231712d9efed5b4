// MX-scaled fp8 MFMA support for the fp8 KMeans passes (kmeans_rr.h compute_mx, SURVEY config 5).
//
// v_mfma_scale_f32_16x16x128_f8f6f4 runs e4m3 x e4m3 products at twice the bf16 MFMA rate, with one E8M0
// scale per 32-element block of each operand row. The fp8 K9r pass feeds the e4m3 rows to it directly and
// splits each bf16 centre value into two e4m3 terms under their own block scales (hi + lo); this file keeps
// the centres of the fp8 engines on the grid where that split is exact (kmeans_mx_snap_kernel) and holds a
// one-instruction probe that pins the operand / scale layout (tests/test_kmeans_mx_gpu.py).
#include "common.h"

typedef int v8i __attribute__((ext_vector_type(8)));

// e4m3fn byte of a finite f32 (|v| <= 448): the hardware round-to-nearest-even conversion.
__device__ __forceinline__ unsigned e4m3_of(float v) {
  return (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xffu;
}
__device__ __forceinline__ float f32_of_e4m3(unsigned b) { return __builtin_amdgcn_cvt_f32_fp8((int)b, 0); }

// One 64-lane wave: out[i][j] = sum_k A[i][k]·B[j][k]·2^(sa-127)·2^(sb-127) over one 16x16x128 MX MFMA
// with per-lane scales sa[lane], sb[lane] (lane l: row l & 15, k block l >> 4). Layout probe for tests.
__global__ __launch_bounds__(64) void mx_probe_kernel(const unsigned char* __restrict__ A,
                                                      const unsigned char* __restrict__ B,
                                                      const int* __restrict__ sa, const int* __restrict__ sb,
                                                      float* __restrict__ out) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  const v8i a = *reinterpret_cast<const v8i*>(A + r * 128 + 32 * g);
  const v8i b = *reinterpret_cast<const v8i*>(B + r * 128 + 32 * g);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[l], 0, sb[l]);
#pragma unroll
  for (int i = 0; i < 4; ++i) out[(4 * g + i) * 16 + r] = c[i];
}

CML_API int cml_mx_probe(const void* A, const void* B, const int* sa, const int* sb, float* out, void* stream) {
  hipLaunchKernelGGL(mx_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const unsigned char*)A,
                     (const unsigned char*)B, sa, sb, out);
  return cml_status();
}

// Scale exponent s with m·2^s in [128, 256) (every block value then fits e4m3's 448), clamped to the
// E8M0 range of the scale 2^-s (kmeans_rr.h mx_shift: the same rule).
__device__ __forceinline__ int block_shift(float m) {
  if (!(m > 0.f)) return 0;
  int e;
  (void)frexpf(m, &e);  // m in [2^(e-1), 2^e)
  int s = 8 - e;
  s = s < -120 ? -120 : (s > 120 ? 120 : s);
  return s;
}

// Centres onto the MX grid, in place: every 32-element block of a bf16 centre row becomes hi·2^-s + lo·2^-t
// (the split the MX assign makes of -2·c, scaled by -1/2: the same blocks, shifts one lower), so that split
// is exact and the MX pass computes the bf16 pass's products. A value loses bits only when it sits ~2^-14
// or further below its block's largest; the result is a bf16 value again (at most 8 significant bits).
// Snapping a snapped row changes nothing. A wave per centre, a lane per block (Dp / 32 <= 64). Also
// rewrites the derived values of the row: cnorm = |c|² (f32 of the f64 sum), and when given cn64 (f64)
// and drift = |c - cb_old| rounded up (kmeans_update_pdev_kernel's outputs).
__global__ __launch_bounds__(256) void kmeans_mx_snap_kernel(u16* __restrict__ cb, long long ldc, int kc, int Dp,
                                                             float* __restrict__ cnorm, double* __restrict__ cn64,
                                                             const u16* __restrict__ cb_old,
                                                             float* __restrict__ drift) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 4 + wave;
  if (c >= kc) return;
  u16* row = cb + (long long)c * ldc;
  double nrm = 0.0, dr = 0.0;
  for (int q = lane; q < Dp / 32; q += 64) {
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = bf16_to_f32(row[32 * q + j]);
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) m = fmaxf(m, fabsf(v[j]));
    const int s = block_shift(m);
    float hv[32];
    float mr = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      hv[j] = ldexpf(f32_of_e4m3(e4m3_of(ldexpf(v[j], s))), -s);
      mr = fmaxf(mr, fabsf(v[j] - hv[j]));
    }
    const int t = block_shift(mr);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const float lo = ldexpf(f32_of_e4m3(e4m3_of(ldexpf(v[j] - hv[j], t))), -t);
      const u16 b = f32_to_bf16(hv[j] + lo);  // exact: hi + lo has at most 8 significant bits
      row[32 * q + j] = b;
      const double f = (double)bf16_to_f32(b);
      nrm += f * f;
      if (cb_old != nullptr) {
        const double e = f - (double)bf16_to_f32(cb_old[(long long)c * ldc + 32 * q + j]);
        dr += e * e;
      }
    }
  }
  nrm = wave_sum_f64(nrm);
  dr = wave_sum_f64(dr);
  if (lane == 0) {
    cnorm[c] = (float)nrm;
    if (cn64 != nullptr) cn64[c] = nrm;
    if (drift != nullptr) drift[c] = (float)(sqrt(dr) * (1.0 + 1e-6));
  }
}

CML_API int cml_kmeans_mx_snap(void* cb, long long ldc, int kc, int Dp, float* cnorm, double* cn64,
                               const void* cb_old, float* drift, void* stream) {
  if (Dp <= 0 || Dp % 32 != 0 || Dp / 32 > 64 || kc < 0 || ldc < Dp || (drift != nullptr) != (cb_old != nullptr))
    return (int)hipErrorInvalidValue;
  if (kc == 0) return 0;
  hipLaunchKernelGGL(kmeans_mx_snap_kernel, dim3((kc + 3) / 4), dim3(256), 0, (hipStream_t)stream, (u16*)cb, ldc, kc,
                     Dp, cnorm, cn64, (const u16*)cb_old, drift);
  return cml_status();
}
