// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of the engine.
//
// Conventions used by every kernel in this directory:
//   * wavefront = 64 lanes, workgroups are multiples of 64 threads;
//   * feature matrices are row-major with a padded leading dimension `ld`
//     (elements), 16-byte aligned rows, zero-filled padding columns;
//   * bf16 values travel as raw uint16 bit patterns (no host-side bf16 type);
//   * every extern "C" launcher takes the HIP stream as `void*` and returns the
//     hipError_t of the launch (0 = success) so the Python layer can raise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CML_API extern "C" __attribute__((visibility("default")))

__device__ __forceinline__ float bf16_to_f32(u16 v) { return __uint_as_float(((unsigned)v) << 16); }

// Round-to-nearest-even f32 -> bf16 keeping NaN a NaN (plain cast lowers to v_cvt_pk_bf16_f32).
__device__ __forceinline__ u16 f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(u16, b);
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Host-side launch status helper.
static inline int cml_status() { return (int)hipGetLastError(); }
