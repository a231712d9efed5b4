// Shared helpers of the source-precision KMeans kernels (kmeans_exact.hip, kmeans_cert.hip).
#pragma once
#include "common.h"

// Double-double accumulation: hi + lo holds a running sum of f32/f64 values exactly while the values'
// binary exponents span less than ~2^80 (f32 rows: any practical data), so the rounded total
// fl(hi + lo) is the correctly rounded exact sum whatever the order of the additions — the host twin,
// the device chunks, the certified step's incremental deltas and the rank fold all give the same bits.
__device__ __forceinline__ void dd_add(double& hi, double& lo, double v) {
  const double s = hi + v;
  const double bb = s - hi;
  lo += (hi - (s - bb)) + (v - bb);
  hi = s;
}
__device__ __forceinline__ void dd_norm(double& hi, double& lo) {
  const double s = hi + lo;
  const double bb = s - hi;
  lo = (hi - (s - bb)) + (lo - bb);
  hi = s;
}

// Directed f64 -> f32 rounding (the certified pruned step's bounds stay conservative in f32).
__device__ __forceinline__ float f32_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, __builtin_huge_valf());
  return f;
}
__device__ __forceinline__ float f32_dn(double v) {
  if (!(v > 0.0)) return 0.0f;
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, 0.0f);
  return f;
}
// a fold of d f64 products differs from the real squared distance by far less than this (relative)
constexpr double kFoldMargin = 1e-10;

// Block-aggregated append to a device list: every thread of the block calls it (flag may be false);
// returns the list position of this thread's entry (-1 without one). One global atomic per call and
// block (a per-wave or per-row atomic on one counter serialises in L2 when many rows append).
// s_w: __shared__ int [NT / 64 + 1].
template <int NT>
__device__ __forceinline__ int block_append(bool flag, int* count, int* s_w) {
  constexpr int nw = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(flag);
  if (lane == 0) s_w[w] = (int)__popcll(bal);
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int v = 0; v < nw; ++v) {
      const int c = s_w[v];
      s_w[v] = tot;
      tot += c;
    }
    s_w[nw] = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  const int pos = flag ? s_w[nw] + s_w[w] + (int)__popcll(bal & ((1ull << lane) - 1ull)) : -1;
  __syncthreads();  // s_w is reused by the next call
  return pos;
}

// LDS-buffered list append for kernels whose rows append sparsely: entries gather in an LDS buffer
// (LDS atomics; the order inside a block is free) and reach the global list in one reservation per
// flush. Call list_flush(..., false) after each block-uniform step (it flushes when fewer than NT slots
// are left) and list_flush(..., true) at the end.
constexpr int kBuf = 2048;
struct ListBuf {
  int* buf;
  int* n;
  int* base;
};

template <int NT>
__device__ __forceinline__ void list_flush(ListBuf lb, int* lst, int* count, bool force) {
  __syncthreads();
  const int m = *lb.n;
  if (m > 0 && (force || m > kBuf - NT)) {
    if (threadIdx.x == 0) *lb.base = atomicAdd(count, m);
    __syncthreads();
    const int b = *lb.base;
    for (int i = threadIdx.x; i < m; i += NT) lst[b + i] = lb.buf[i];
    __syncthreads();
    if (threadIdx.x == 0) *lb.n = 0;
  }
  __syncthreads();
}
