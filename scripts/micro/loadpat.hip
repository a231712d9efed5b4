// Global-load pattern microbenchmark: bytes/s for a wave reading a 32-row x 512-B tile with
// different lane->address mappings (rows per instruction x contiguous bytes per row).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// RPI rows per instruction, each row gets 64/RPI lanes x 16 B = 1024/RPI contiguous bytes.
template <int RPI>
__global__ __launch_bounds__(256) void kload(const unsigned char* __restrict__ X, long long ntiles, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const long long w0 = (blockIdx.x * 256LL + threadIdx.x) >> 6;
  const long long nw = (gridDim.x * 256LL) >> 6;
  constexpr int LPR = 64 / RPI;           // lanes per row
  constexpr int NI = 16;                  // instructions per 16 KB tile
  const int r = lane % RPI, c = lane / RPI;
  u32x4 acc = {0, 0, 0, 0};
  for (long long t = w0; t < ntiles; t += nw) {
    const unsigned char* base = X + t * 16384;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      // instruction i covers rows [ (i*RPI) % 32 ...], column block ((i*RPI)/32)
      const int rowblk = (i * RPI) % 32, colblk = (i * RPI) / 32;
      const int row = rowblk + r;
      const int col = (colblk * LPR + c) * 16;
      acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + row * 512 + col));
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

template <int RPI>
float run(const unsigned char* X, long long ntiles, unsigned* out, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  kload<RPI><<<grid, 256>>>(X, ntiles, out);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) kload<RPI><<<grid, 256>>>(X, ntiles, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const long long bytes = 10LL << 30;
  const long long ntiles = bytes / 16384;
  unsigned char* X; unsigned* out;
  if (hipMalloc(&X, bytes) != hipSuccess) return 1;
  hipMalloc(&out, 4);
  hipMemset(X, 1, bytes);
  for (int grid : {1024, 2048, 4096, 8192}) {
    printf("grid %d: rpi32 %.1f  rpi16 %.1f  rpi8 %.1f  rpi4 %.1f  rpi2 %.1f GB/s\n", grid,
           bytes / 1e6 / run<32>(X, ntiles, out, grid), bytes / 1e6 / run<16>(X, ntiles, out, grid),
           bytes / 1e6 / run<8>(X, ntiles, out, grid), bytes / 1e6 / run<4>(X, ntiles, out, grid),
           bytes / 1e6 / run<2>(X, ntiles, out, grid));
  }
  hipFree(X);
  return 0;
}
