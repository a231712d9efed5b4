// MX-scaled fp8 operands of the K9r screen pass (kmeans_rr.h MODE 3, SURVEY config 5: fp8 rows).
//
// v_mfma_scale_f32_16x16x128_f8f6f4 runs e4m3 x e4m3 products at twice the bf16 MFMA rate, with one
// E8M0 scale per 32-element block of each operand row. The fp8 K9r pass widened every X fragment to bf16
// in every compute wave (v_cvt_scalef32_pk_bf16_fp8, 8 per 16 bytes) and was bound by that vector work;
// the screen pass feeds the e4m3 bytes straight to the MX MFMA instead and represents each bf16 centre
// value -2·c as hi + lo, two e4m3 values under their own block scales:
//
//   hi = e4m3(v · 2^s),  lo = e4m3((v - hi·2^-s) · 2^t),  ~c = -(hi·2^-s + lo·2^-t) / 2
//
// Two MX MFMAs per 128 k (hi, lo) cost what the four bf16 MFMAs of that k range cost, with no
// conversion. ~c equals the bf16 centre except where a value sits far below its block's largest (e4m3
// subnormals drop its low bits); this pass also returns e_j = |~c_j - cb_j| (rounded up) and |~c_j|²,
// and the screen certifies a row's label only when its top-2 gap exceeds what e and the
// f32 rounding of both passes can move (kmeans_rr.h, MODE 3). Rows it cannot certify are re-assigned by
// the bf16 pass, so labels and sums are those of the bf16 path.
//
// Lane layout (the K9r fp8 k order): lane (r, g) of MX block b holds the 16-B chunks 8b + g and 8b + 4 + g
// of row r — the two 16-B units the compute wave reads for that block. The instruction's k order is the
// same (bytes 0-15 of lane group g are k 16g + j, bytes 16-31 are k 64 + 16g + j), and its scale block q
// (scale from lane group q) is k [32q, 32q + 32): chunks 8b + 2q, 8b + 2q + 1 — measured on MI355X
// (scripts/r5/mx_probe_diag3.py; tests/test_kmeans_mx_gpu.py pins it).
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
// E8M0 range of the scale 2^-s.
__device__ __forceinline__ int block_shift(float m) {
  if (!(m > 0.f)) return 0;
  int e;
  (void)frexpf(m, &e);  // m in [2^(e-1), 2^e)
  int s = 8 - e;
  s = s < -120 ? -120 : (s > 120 ? 120 : s);
  return s;
}

// A wave per centre (4 per workgroup). cb: bf16 [kc, ldc]; Dp % 128 == 0; mx_c: bytes
// [kp][Dp/128][lane group 4][hi 32 | lo 32]; mx_s: int32 [kp][Dp/128][scale block 4] = hi scale | lo scale
// << 8 (E8M0); cn_t: f32
// [kp] |~c|² (+inf past kc); e_c: f32 [kp] |~c - cb| rounded up (0 past kc). gate (nullable): run only
// when gate[0] == 1 (the pruned step's full-pass flag).
__global__ __launch_bounds__(256) void kmeans_mx_centres_kernel(const u16* __restrict__ cb, long long ldc, int kc,
                                                                int kp, int Dp, unsigned char* __restrict__ mx_c,
                                                                int* __restrict__ mx_s, float* __restrict__ cn_t,
                                                                float* __restrict__ e_c, const int* __restrict__ gate) {
  if (gate != nullptr && gate[0] != 1) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nb = Dp / 128, nblk = nb * 4;  // 32-element blocks per centre
  const int c = blockIdx.x * 4 + wave;
  if (c >= kp) return;
  {
    double err = 0.0, nrm = 0.0;
    for (int q = lane; q < nblk; q += 64) {
      const int b = q >> 2, sq = q & 3;  // MX block, scale block: k = 128b + 32sq + j
      float v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const int k = 128 * b + 32 * sq + j;
        v[j] = c < kc ? -2.f * bf16_to_f32(cb[(long long)c * ldc + k]) : 0.f;
      }
      float m = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) m = fmaxf(m, fabsf(v[j]));
      const int s = block_shift(m);
      unsigned hb[32];
      float r[32];
      float mr = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        hb[j] = e4m3_of(ldexpf(v[j], s));
        r[j] = v[j] - ldexpf(f32_of_e4m3(hb[j]), -s);  // exact: both are short dyadic values
        mr = fmaxf(mr, fabsf(r[j]));
      }
      const int t = block_shift(mr);
      unsigned wh[8] = {0, 0, 0, 0, 0, 0, 0, 0}, wl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const unsigned lb = e4m3_of(ldexpf(r[j], t));
        const double ct = (double)ldexpf(f32_of_e4m3(hb[j]), -s) + (double)ldexpf(f32_of_e4m3(lb), -t);
        const double dlt = ct - (double)v[j];
        err += dlt * dlt;
        nrm += ct * ct;
        wh[j >> 2] |= hb[j] << (8 * (j & 3));
        wl[j >> 2] |= lb << (8 * (j & 3));
      }
      // chunk i = 2sq + u of the block sits in lane group i & 3, half i >> 2 (bytes 16·(i >> 2) of its 32)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = 2 * sq + u;
        unsigned char* dst = mx_c + ((long long)(c * nb + b) * 4 + (i & 3)) * 64 + 16 * (i >> 2);
        *reinterpret_cast<uint4*>(dst) = make_uint4(wh[4 * u], wh[4 * u + 1], wh[4 * u + 2], wh[4 * u + 3]);
        *reinterpret_cast<uint4*>(dst + 32) = make_uint4(wl[4 * u], wl[4 * u + 1], wl[4 * u + 2], wl[4 * u + 3]);
      }
      mx_s[(long long)c * nblk + q] = (127 - s) | ((127 - t) << 8);  // lane group sq provides block sq's scale
    }
    err = wave_sum_f64(err);
    nrm = wave_sum_f64(nrm);
    // ~c = -(hi + lo) / 2: |~c - cb| = sqrt(err) / 2, |~c|² = nrm / 4 (rounded up: the screen's slack)
    if (lane == 0) {
      cn_t[c] = c < kc ? (float)(0.25 * nrm) : __builtin_huge_valf();
      e_c[c] = c < kc ? (float)(0.5 * sqrt(err) * (1.0 + 1e-6)) + 1e-30f : 0.f;
    }
  }
}

CML_API int cml_kmeans_mx_centres(const void* cb, long long ldc, int kc, int kp, int Dp, void* mx_c, int* mx_s,
                                  float* cn_t, float* e_c, const int* gate, void* stream) {
  if (Dp <= 0 || Dp % 128 != 0 || Dp / 32 > 64 || kc > kp || kc <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_mx_centres_kernel, dim3((kp + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const u16*)cb,
                     ldc, kc, kp, Dp, (unsigned char*)mx_c, mx_s, cn_t, e_c, gate);
  return cml_status();
}
