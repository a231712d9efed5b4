// Synthetic feature rows keyed by their GLOBAL row index (gfx950).
//
// The benchmarks' datasets (BASELINE.json configs 2-5: Gaussian blobs, Gaussian features with
// logistic labels) must be one fixed table however it is partitioned: the reference's data
// parallelism is Spark row partitions of ONE table (ref.py:57, ref.py:139), so the 1/2/4/8-GPU
// scaling curve has to fit the same rows at every N. Every value here is a pure function of
// (key, global row, column): rank r generating rows [r0, r0 + n) writes exactly those rows of the
// one-rank table, bit for bit, whatever the rank count.
//
//   label(row)     = hi32(splitmix64(row ^ key_label)) * kt >> 32         (uniform in [0, kt))
//   noise(row, j)  = Box-Muller of splitmix64((row * d + j) ^ key)        (N(0, 1), f32 math)
//                    or 4·u - 2 with u from the same hash                 (mode 1: U(-2, 2))
//   out[row, j]    = centres[label(row), j] + noise(row, j)               (centres optional)
//
// One thread writes 8 consecutive columns of a row (a 16-byte bf16 store or two f32x4 stores);
// pure ALU + streaming stores, no LDS. Columns d <= j < ldo are written as zeros (padded layouts).
#include "common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float noise_value(unsigned long long h, int mode) {
  // 24-bit uniforms: u1 in (0, 1] (log finite), u2 in [0, 1)
  const float u1 = ((float)(unsigned)(h >> 40) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = (float)(unsigned)(h & 0xFFFFFFull) * (1.0f / 16777216.0f);
  if (mode == 1) return 4.0f * u2 - 2.0f;
  return sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795864f * u2);
}

template <int OUT>  // 0: bf16 (u16 bits), 1: f32
__global__ __launch_bounds__(kThreads) void synth_rows_kernel(long long row0, long long n, int d, long long ldo,
                                                              const float* __restrict__ centres, int kt,
                                                              unsigned long long key, unsigned long long key_label,
                                                              int mode, void* __restrict__ out,
                                                              int* __restrict__ labels) {
  const int groups = (int)((ldo + 7) / 8);
  const long long total = n * groups;
  for (long long t = (long long)blockIdx.x * kThreads + threadIdx.x; t < total; t += (long long)gridDim.x * kThreads) {
    const long long i = t / groups;
    const int j0 = (int)(t - i * groups) * 8;
    const unsigned long long row = (unsigned long long)(row0 + i);
    int lab = 0;
    if (centres != nullptr || labels != nullptr)
      lab = (int)(((mix64(row ^ key_label) >> 32) * (unsigned long long)kt) >> 32);
    if (labels != nullptr && j0 == 0) labels[i] = lab;
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = j0 + q;
      float z = 0.0f;
      if (j < d) {
        z = noise_value(mix64((row * (unsigned long long)d + (unsigned long long)j) ^ key), mode);
        if (centres != nullptr) z += centres[(long long)lab * d + j];
      }
      v[q] = z;
    }
    if (OUT == 0) {
      u16* o = (u16*)out + i * ldo + j0;
      if (j0 + 8 <= ldo && (ldo & 7) == 0) {
        uint4 w;
        w.x = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
        w.y = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
        w.z = (unsigned)f32_to_bf16(v[4]) | ((unsigned)f32_to_bf16(v[5]) << 16);
        w.w = (unsigned)f32_to_bf16(v[6]) | ((unsigned)f32_to_bf16(v[7]) << 16);
        *reinterpret_cast<uint4*>(o) = w;
      } else {
        for (int q = 0; q < 8 && j0 + q < ldo; ++q) o[q] = f32_to_bf16(v[q]);
      }
    } else {
      float* o = (float*)out + i * ldo + j0;
      if (j0 + 8 <= ldo && (ldo & 3) == 0) {
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        for (int q = 0; q < 8 && j0 + q < ldo; ++q) o[q] = v[q];
      }
    }
  }
}

}  // namespace

// out: [n, ldo] bf16 (out_dtype 0) or f32 (1), 16-byte aligned; centres: [kt, d] f32 or null;
// labels: [n] int32 or null. Rows are global rows row0 .. row0 + n - 1.
CML_API int cml_synth_rows(long long row0, long long n, int d, long long ldo, const float* centres, int kt,
                           unsigned long long key, unsigned long long key_label, int mode, void* out, int out_dtype,
                           int* labels, void* stream) {
  if (n <= 0) return 0;
  if (d <= 0 || ldo < d || (centres != nullptr && kt <= 0) || (labels != nullptr && kt <= 0) || mode < 0 ||
      mode > 1 || (reinterpret_cast<size_t>(out) & 15) != 0)
    return (int)hipErrorInvalidValue;
  const long long total = n * ((ldo + 7) / 8);
  long long g = (total + kThreads - 1) / kThreads;
  if (g > 256LL * 1024) g = 256LL * 1024;  // grid-stride beyond ~1000 waves per CU
  hipStream_t st = (hipStream_t)stream;
  if (out_dtype == 0)
    hipLaunchKernelGGL(synth_rows_kernel<0>, dim3((unsigned)g), dim3(kThreads), 0, st, row0, n, d, ldo, centres, kt,
                       key, key_label, mode, out, labels);
  else if (out_dtype == 1)
    hipLaunchKernelGGL(synth_rows_kernel<1>, dim3((unsigned)g), dim3(kThreads), 0, st, row0, n, d, ldo, centres, kt,
                       key, key_label, mode, out, labels);
  else
    return (int)hipErrorInvalidValue;
  return cml_status();
}
