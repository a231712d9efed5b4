// Columnar-frame kernels for gfx950: the memory-bound glue between the
// reference's DataFrame steps and the estimators. Every kernel streams its inputs once.
//
// K2  assemble_pack   typed columns (+ validity bytes, + vector columns) -> row-major [n, ld]
//                     f64/f32/bf16 feature matrix and a per-row "invalid" byte (null or NaN) —
//                     VectorAssembler (ref.py:134-136) with handleInvalid error/skip/keep.
// K3  compact         bool mask -> ascending int64 indices of the set rows (count, block scan,
//                     scatter) — filter / na.drop / BETWEEN (ref.py:123-128) and the splits.
// K5  split_buckets   counter hash (splitmix64) of (seed, stream, global row id) -> split index
//                     by cumulative weights; GPU-count invariant (ref.py:139, ref.py:180).
// K22 poisson1        Poisson(1) bagging counts by CDF inversion of the same counter uniform
//                     (RandomForest bootstrap, ref.py:155-158, ref.py:187-190).
// K6  binarize        y = x > thr ? 1 : 0 (ref.py:176-177 `when(col > 5.0, 1).otherwise(0)`).
// K23 reg_metrics     fused weighted SSE / SAE / Σy / Σy² / Σŷ / Σŷ² / Σw partials (RMSE, MSE, MAE,
//                     R², explained variance: ref.py:160-169); cls_confusion: weighted confusion
//                     matrix (accuracy, F1, precision, recall: ref.py:192-198).
// K4  col_absmax / quant_fp8   per-feature amax and x·scale -> OCP e4m3fn bytes.
//
// The uniform/Poisson kernels reproduce utils/rng.py bit for bit (same uint64 arithmetic, the
// CDF thresholds are computed on the host once), so CPU and GPU runs make identical decisions.
#include "common.h"

#include <type_traits>

namespace {

constexpr int kThreads = 256;
constexpr int kCompactItems = 16;                       // per thread
constexpr int kCompactTile = kThreads * kCompactItems;  // rows per compaction block

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ double counter_uniform(long long row, unsigned long long key) {
  const unsigned long long h = splitmix64((unsigned long long)row ^ key);
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

// ------------------------------------------------------------------------------------- K5 / K22
struct Cum {
  double c[17];  // c[0] = 0 ... c[nb] (>= 1)
  int nb;
};

__global__ __launch_bounds__(kThreads) void split_buckets_kernel(const long long* __restrict__ rows, long long n,
                                                                 unsigned long long key, Cum cum,
                                                                 signed char* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const double u = counter_uniform(rows[i], key);
    int b = -1;
    for (int j = 0; j < cum.nb; ++j)
      if (b < 0 && u >= cum.c[j] && u < cum.c[j + 1]) b = j;
    out[i] = (signed char)b;
  }
}

struct PoissonCdf {
  double t[17];  // t[k-1] = P(X <= k-1); count = #{k : u >= t[k-1]}
  int kmax;
};

__global__ __launch_bounds__(kThreads) void poisson1_kernel(const long long* __restrict__ rows, long long n,
                                                            unsigned long long key, PoissonCdf cdf,
                                                            int* __restrict__ out_i32, float* __restrict__ out_f32) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const double u = counter_uniform(rows[i], key);
    int c = 0;
    for (int k = 0; k < cdf.kmax; ++k) c += u >= cdf.t[k] ? 1 : 0;
    if (out_i32 != nullptr) out_i32[i] = c;
    if (out_f32 != nullptr) out_f32[i] = (float)c;
  }
}

__global__ __launch_bounds__(kThreads) void uniform_kernel(const long long* __restrict__ rows, long long n,
                                                           unsigned long long key, double* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads)
    out[i] = counter_uniform(rows[i], key);
}

// --------------------------------------------------------------------------------------------- K3
__device__ __forceinline__ int block_exclusive_scan(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  int wbase = 0, tot = 0;
#pragma unroll
  for (int j = 0; j < kThreads / 64; ++j) {
    const int s = sh[j];
    if (j < w) wbase += s;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return wbase + incl - v;
}

// 16 mask bytes of the thread's 16 consecutive rows as a bit set (one 16-byte load when the tile is
// whole and aligned, byte loads for the tail)
__device__ __forceinline__ unsigned mask_bits16(const unsigned char* __restrict__ mask, long long base, long long n) {
  unsigned bits = 0;
  if (base + kCompactItems <= n && (reinterpret_cast<size_t>(mask + base) & 15) == 0) {
    const uint4 w = *reinterpret_cast<const uint4*>(mask + base);
    const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b) bits |= ((ws[q] >> (8 * b)) & 0xffu) ? (1u << (4 * q + b)) : 0u;
  } else {
#pragma unroll
    for (int j = 0; j < kCompactItems; ++j) bits |= (base + j < n && mask[base + j]) ? (1u << j) : 0u;
  }
  return bits;
}

__global__ __launch_bounds__(kThreads) void compact_count_kernel(const unsigned char* __restrict__ mask, long long n,
                                                                 long long* __restrict__ bcount) {
  __shared__ int sh[kThreads / 64];
  const long long base = (long long)blockIdx.x * kCompactTile + (long long)threadIdx.x * kCompactItems;
  const int c = __popc(mask_bits16(mask, base, n));
  int total;
  block_exclusive_scan(c, sh, total);
  if (threadIdx.x == 0) bcount[blockIdx.x] = total;
}

// one block: in-place exclusive scan of the block counts, total -> count_out
__global__ __launch_bounds__(kThreads) void compact_scan_kernel(long long* __restrict__ bcount, long long nb,
                                                                long long* __restrict__ count_out) {
  __shared__ int sh[kThreads / 64];
  long long carry = 0;
  for (long long b0 = 0; b0 < nb; b0 += kThreads) {
    const long long i = b0 + threadIdx.x;
    const int v = i < nb ? (int)bcount[i] : 0;  // per-block counts <= kCompactTile
    int total;
    const int ex = block_exclusive_scan(v, sh, total);
    if (i < nb) bcount[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) *count_out = carry;
}

// The tile's kept indices are placed in LDS at their scanned positions, then copied out by the whole
// block with consecutive 8-byte stores (coalesced) instead of per-thread runs.
__global__ __launch_bounds__(kThreads) void compact_scatter_kernel(const unsigned char* __restrict__ mask, long long n,
                                                                   const long long* __restrict__ boff,
                                                                   long long* __restrict__ idx) {
  __shared__ int sh[kThreads / 64];
  __shared__ long long buf[kCompactTile];
  const long long tile0 = (long long)blockIdx.x * kCompactTile;
  const long long base = tile0 + (long long)threadIdx.x * kCompactItems;
  const unsigned bits = mask_bits16(mask, base, n);
  int total;
  int pos = block_exclusive_scan(__popc(bits), sh, total);
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j)
    if (bits & (1u << j)) buf[pos++] = base + j;
  __syncthreads();
  const long long o = boff[blockIdx.x];
  for (int i = threadIdx.x; i < total; i += kThreads) idx[o + i] = buf[i];
}

// --------------------------------------------------------------------------------------------- K2
// Source column types.
enum SrcType : int { kF64 = 0, kF32 = 1, kI32 = 2, kI64 = 3, kU8 = 4, kI16 = 5, kBF16 = 6, kI8 = 7 };

struct AsmCol {
  const void* ptr;
  const unsigned char* valid;  // null = all valid
  long long ld;                // elements between rows (vector columns), 1 for scalars
  int type;
  int width;                   // 1 for scalars
  int out_off;
  int pad;
};

__device__ __forceinline__ double load_as_f64(const void* p, int type, long long i) {
  switch (type) {
    case kF64: return reinterpret_cast<const double*>(p)[i];
    case kF32: return (double)reinterpret_cast<const float*>(p)[i];
    case kI32: return (double)reinterpret_cast<const int*>(p)[i];
    case kI64: return (double)reinterpret_cast<const long long*>(p)[i];
    case kU8: return (double)reinterpret_cast<const unsigned char*>(p)[i];
    case kI16: return (double)reinterpret_cast<const short*>(p)[i];
    case kBF16: return (double)bf16_to_f32(reinterpret_cast<const u16*>(p)[i]);
    default: return (double)reinterpret_cast<const signed char*>(p)[i];
  }
}

// f64 -> bf16 as torch's .to(bfloat16) does it: through f32 (two round-to-nearest-even steps).
__device__ __forceinline__ u16 f64_to_bf16(double v) { return f32_to_bf16((float)v); }

template <int OUT>  // 0 f64, 1 f32, 2 bf16
__global__ __launch_bounds__(kThreads) void assemble_kernel(const AsmCol* __restrict__ cols, int ncols, long long n,
                                                            void* __restrict__ out, long long ldo, int dout,
                                                            unsigned char* __restrict__ invalid, int nan_keep) {
  for (long long r = (long long)blockIdx.x * kThreads + threadIdx.x; r < n; r += (long long)gridDim.x * kThreads) {
    bool bad = false;
    for (int c = 0; c < ncols; ++c) {
      const AsmCol col = cols[c];
      const bool ok = col.valid == nullptr || col.valid[r] != 0;
      for (int j = 0; j < col.width; ++j) {
        double v = ok ? load_as_f64(col.ptr, col.type, r * col.ld + j) : __builtin_nan("");
        bad |= !ok || v != v;
        if (!nan_keep && v != v) v = 0.0;
        const long long o = r * ldo + col.out_off + j;
        if constexpr (OUT == 0) reinterpret_cast<double*>(out)[o] = v;
        else if constexpr (OUT == 1) reinterpret_cast<float*>(out)[o] = (float)v;
        else reinterpret_cast<u16*>(out)[o] = f64_to_bf16(v);
      }
    }
    for (long long o = r * ldo + dout; o < r * ldo + ldo; ++o) {  // zero the padding columns
      if constexpr (OUT == 0) reinterpret_cast<double*>(out)[o] = 0.0;
      else if constexpr (OUT == 1) reinterpret_cast<float*>(out)[o] = 0.f;
      else reinterpret_cast<u16*>(out)[o] = 0;
    }
    if (invalid != nullptr) invalid[r] = bad ? 1 : 0;
  }
}

// Scalar-columns fast path (every column width 1, at most 16 of them, row width ldo <= 16): the
// column table is staged in LDS once per block, each thread builds its whole output row in registers
// (the per-column loads of a wave are coalesced) and writes it with 16-byte stores.
constexpr int kAsmMax = 16;

template <int OUT, int MAXC>
__global__ __launch_bounds__(kThreads) void assemble_scalar_kernel(const AsmCol* __restrict__ cols, int ncols,
                                                                   long long n, void* __restrict__ out, long long ldo,
                                                                   unsigned char* __restrict__ invalid, int nan_keep) {
  // RPT rows per thread per pass (rows r, r + 256, ...): their loads are all issued before the first
  // store, so a wave keeps RPT x ncols loads in flight (Little's law at ~2 us HBM latency).
  constexpr int RPT = 4;
  __shared__ AsmCol sc[MAXC];
  if (threadIdx.x < ncols) sc[threadIdx.x] = cols[threadIdx.x];
  __syncthreads();
  using OT = typename std::conditional<OUT == 0, double, typename std::conditional<OUT == 1, float, u16>::type>::type;
  constexpr int PER16 = 16 / (int)sizeof(OT);
  const bool vec = (ldo % PER16) == 0 && (reinterpret_cast<size_t>(out) & 15) == 0;
  const long long step = (long long)gridDim.x * kThreads * RPT;
  for (long long r0 = (long long)blockIdx.x * kThreads * RPT + threadIdx.x; r0 < n; r0 += step) {
    double v[RPT][MAXC];
    bool bad[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) bad[q] = false;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < ncols) {
        const AsmCol& col = sc[c];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
          const long long r = r0 + (long long)q * kThreads;
          const bool inr = r < n;
          const bool ok = col.valid == nullptr || (inr && col.valid[r] != 0);
          double x = (ok && inr) ? load_as_f64(col.ptr, col.type, r) : __builtin_nan("");
          bad[q] |= !ok || x != x;
          if (!nan_keep && x != x) x = 0.0;
          v[q][c] = x;
        }
      } else {
#pragma unroll
        for (int q = 0; q < RPT; ++q) v[q][c] = 0.0;
      }
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const long long r = r0 + (long long)q * kThreads;
      if (r >= n) break;
      OT row[MAXC];
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if constexpr (OUT == 0) row[c] = v[q][c];
        else if constexpr (OUT == 1) row[c] = (float)v[q][c];
        else row[c] = f64_to_bf16(v[q][c]);
      }
      OT* o = reinterpret_cast<OT*>(out) + r * ldo;
      if (vec) {
#pragma unroll
        for (int k = 0; k < MAXC / PER16; ++k) {
          if (k * PER16 < ldo) {
            uint4 w;
            __builtin_memcpy(&w, &row[k * PER16], 16);
            *reinterpret_cast<uint4*>(o + k * PER16) = w;
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < MAXC; ++c)
          if (c < ldo) o[c] = row[c];
      }
      if (invalid != nullptr) invalid[r] = bad[q] ? 1 : 0;
    }
  }
}

// --------------------------------------------------------------------------------------------- K6
__global__ __launch_bounds__(kThreads) void binarize_kernel(const void* __restrict__ x, int type, long long n,
                                                            double thr, double* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads)
    out[i] = load_as_f64(x, type, i) > thr ? 1.0 : 0.0;
}

// -------------------------------------------------------------------------------------------- K23
// partial[b][0..6] = Σw, Σw e², Σw |e|, Σw y, Σw y², Σw p, Σw p²   (e = y - p)
__global__ __launch_bounds__(kThreads) void reg_metrics_kernel(const double* __restrict__ y, const double* __restrict__ p,
                                                               const double* __restrict__ w, long long n,
                                                               double* __restrict__ partial) {
  __shared__ double sh[7][kThreads / 64];
  double s[7] = {0, 0, 0, 0, 0, 0, 0};
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kThreads) {
    const double wi = w != nullptr ? w[i] : 1.0;
    const double yi = y[i], pi = p[i], e = yi - pi;
    s[0] += wi;
    s[1] += wi * e * e;
    s[2] += wi * fabs(e);
    s[3] += wi * yi;
    s[4] += wi * yi * yi;
    s[5] += wi * pi;
    s[6] += wi * pi * pi;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    const double t = wave_sum_f64(s[q]);
    if (lane == 0) sh[q][wv] = t;
  }
  __syncthreads();
  if (threadIdx.x < 7) {
    double t = 0.0;
    for (int j = 0; j < kThreads / 64; ++j) t += sh[threadIdx.x][j];
    partial[(long long)blockIdx.x * 7 + threadIdx.x] = t;
  }
}

// partial[b][C*C]: weighted confusion counts cm[label][pred], labels/preds in [0, C).
// Deterministic (no float atomics): a wave takes 64 rows at a time and folds them cell by cell — the
// first pending lane's cell, the masked weights of every lane holding that cell summed by a fixed
// butterfly, added by that lane into the wave's private LDS histogram — so each cell's partial is a
// fixed-order sum for a given n and grid; the block then adds its waves' histograms in wave order.
// (Binary labels: at most 4 distinct cells per 64 rows, so ~4 butterflies per 64 rows.)
__global__ __launch_bounds__(kThreads) void cls_confusion_kernel(const long long* __restrict__ y,
                                                                 const long long* __restrict__ p,
                                                                 const double* __restrict__ w, long long n, int C,
                                                                 double* __restrict__ partial) {
  extern __shared__ double cm[];  // [kThreads / 64][C * C]
  const int CC = C * C, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int kWaves = kThreads / 64;
  for (int i = threadIdx.x; i < kWaves * CC; i += kThreads) cm[i] = 0.0;
  __syncthreads();
  double* mine = cm + wv * CC;
  for (long long base = ((long long)blockIdx.x * kWaves + wv) * 64; base < n; base += (long long)gridDim.x * kThreads) {
    const long long i = base + lane;
    int cell = -1;
    double wi = 0.0;
    if (i < n) {
      const long long a = y[i], b = p[i];
      if (a >= 0 && a < C && b >= 0 && b < C) {
        cell = (int)(a * C + b);
        wi = w != nullptr ? w[i] : 1.0;
      }
    }
    unsigned long long pending = __ballot(cell >= 0);
    while (pending) {
      const int leader = __builtin_ctzll(pending);
      const int lc = __shfl(cell, leader, 64);
      const bool same = cell == lc;
      const double v = wave_sum_f64(same ? wi : 0.0);
      if (lane == leader) mine[lc] += v;
      pending &= ~__ballot(same);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < CC; c += kThreads) {
    double t = 0.0;
    for (int q = 0; q < kWaves; ++q) t += cm[q * CC + c];
    partial[(long long)blockIdx.x * CC + c] = t;
  }
}

// --------------------------------------------------------------------------------------------- K4
// per-block partial column amax: partial[b][j] = max |x[r, j]| over the block's rows.
template <typename T>
__device__ __forceinline__ float ld_f32(const T* p, long long i);
template <>
__device__ __forceinline__ float ld_f32<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld_f32<u16>(const u16* p, long long i) { return bf16_to_f32(p[i]); }

template <typename T>
__global__ __launch_bounds__(kThreads) void col_absmax_kernel(const T* __restrict__ x, long long n, int d, long long ldx,
                                                              int rows_per_block, float* __restrict__ partial) {
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  for (int j = threadIdx.x; j < d; j += kThreads) {
    float m = 0.f;
    for (long long r = r0; r < r1; ++r) m = fmaxf(m, fabsf(ld_f32<T>(x, r * ldx + j)));
    partial[(long long)blockIdx.x * d + j] = m;
  }
}

// 16-byte fast path: a row is cpr = d / E chunks of E = 16 / sizeof(T) values; thread t of the block
// takes chunk t % cpr of rows t / cpr + k * (kThreads / cpr) (1 KiB per wave instruction), keeps E
// running maxima and the block folds its row groups through LDS at the end.
template <typename T>
__global__ __launch_bounds__(kThreads) void col_absmax16_kernel(const T* __restrict__ x, long long n, int d,
                                                                long long ldx, int rows_per_block,
                                                                float* __restrict__ partial) {
  constexpr int E = 16 / (int)sizeof(T);
  __shared__ float sh[2048];  // (kThreads / cpr) x d floats = 8 KiB
  const int cpr = d / E;
  const int rpi = kThreads / cpr;
  const int t = threadIdx.x, ch = t % cpr, rg = t / cpr;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  float m[E];
#pragma unroll
  for (int e = 0; e < E; ++e) m[e] = 0.f;
  if (rg < rpi) {
    for (long long r = r0 + rg; r < r1; r += rpi) {
      const uint4 w = *reinterpret_cast<const uint4*>(x + r * ldx + ch * E);
      const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float v;
        if constexpr (sizeof(T) == 2) v = bf16_to_f32((u16)((ws[e >> 1] >> (16 * (e & 1))) & 0xffffu));
        else v = __uint_as_float(ws[e]);
        m[e] = fmaxf(m[e], fabsf(v));
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) sh[rg * d + ch * E + e] = m[e];
  }
  __syncthreads();
  for (int j = t; j < d; j += kThreads) {
    float v = 0.f;
    for (int q = 0; q < rpi; ++q) v = fmaxf(v, sh[q * d + j]);
    partial[(long long)blockIdx.x * d + j] = v;
  }
}

// 8 values per thread -> one 8-byte store of e4m3fn bytes (rows of d = ldo values, d % 8 == 0,
// cpr = d / 8 a power of two: row and chunk by shift / mask, no 64-bit division per element).
template <typename T>
__global__ __launch_bounds__(kThreads) void quant_fp8_v8_kernel(const T* __restrict__ x, long long n, int d,
                                                                long long ldx, const float* __restrict__ scale,
                                                                unsigned char* __restrict__ out, int cpr_shift) {
  const long long total = n << cpr_shift;
  const long long cmask = (1LL << cpr_shift) - 1;
  for (long long t = (long long)blockIdx.x * kThreads + threadIdx.x; t < total; t += (long long)gridDim.x * kThreads) {
    const long long r = t >> cpr_shift;
    const int j = (int)(t & cmask) * 8;
    float v[8];
    if constexpr (sizeof(T) == 2) {
      const uint4 w = *reinterpret_cast<const uint4*>(x + r * ldx + j);
      const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = bf16_to_f32((u16)((ws[e >> 1] >> (16 * (e & 1))) & 0xffffu));
    } else {
      const float4 a = *reinterpret_cast<const float4*>(x + r * ldx + j);
      const float4 b = *reinterpret_cast<const float4*>(x + r * ldx + j + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    const float4 s0 = *reinterpret_cast<const float4*>(scale + j);
    const float4 s1 = *reinterpret_cast<const float4*>(scale + j + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    unsigned lo = 0, hi = 0;
    lo = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[0] * sc[0], v[1] * sc[1], (int)lo, false);
    lo = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[2] * sc[2], v[3] * sc[3], (int)lo, true);
    hi = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[4] * sc[4], v[5] * sc[5], (int)hi, false);
    hi = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[6] * sc[6], v[7] * sc[7], (int)hi, true);
    *reinterpret_cast<uint2*>(out + r * (long long)d + j) = make_uint2(lo, hi);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void quant_fp8_kernel(const T* __restrict__ x, long long n, int d, long long ldx,
                                                             const float* __restrict__ scale,
                                                             unsigned char* __restrict__ out, long long ldo) {
  // two values per thread -> one packed v_cvt_pk_fp8_f32 (OCP e4m3fn on gfx950, saturating)
  const long long pairs_per_row = (ldo + 1) / 2;
  const long long total = n * pairs_per_row;
  for (long long t = (long long)blockIdx.x * kThreads + threadIdx.x; t < total; t += (long long)gridDim.x * kThreads) {
    const long long r = t / pairs_per_row;
    const int j = (int)(t - r * pairs_per_row) * 2;
    const float a = j < d ? ld_f32<T>(x, r * ldx + j) * scale[j] : 0.f;
    const float b = j + 1 < d ? ld_f32<T>(x, r * ldx + j + 1) * scale[j + 1] : 0.f;
    const int packed = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    out[r * ldo + j] = (unsigned char)(packed & 0xff);
    if (j + 1 < ldo) out[r * ldo + j + 1] = (unsigned char)((packed >> 8) & 0xff);
  }
}

// ----------------------------------------------------------------------------- invalid check
// Any NaN among the first d columns of a row-major bf16 / f32 / f64 matrix: 16-byte loads, NaN
// test on the raw bits, one flag per block (VectorAssembler handleInvalid="error" on a vector
// input that is used in place).
template <int ESZ>
__global__ __launch_bounds__(kThreads) void has_nan_kernel(const unsigned char* __restrict__ x, long long n, int d,
                                                           long long ld_bytes, int* __restrict__ flag) {
  const int per = 16 / ESZ;
  const int chunks = (d + per - 1) / per;
  const long long total = n * chunks;
  int found = 0;
  for (long long t = (long long)blockIdx.x * kThreads + threadIdx.x; t < total; t += (long long)gridDim.x * kThreads) {
    const long long r = t / chunks;
    const int c = (int)(t - r * chunks);
    const uint4 v = *reinterpret_cast<const uint4*>(x + r * ld_bytes + 16LL * c);
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
    const int valid = d - c * per < per ? d - c * per : per;
    if constexpr (ESZ == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const unsigned h = (w[e >> 1] >> (16 * (e & 1))) & 0xffffu;
        found |= (e < valid) & ((h & 0x7fffu) > 0x7f80u);
      }
    } else if constexpr (ESZ == 4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) found |= (e < valid) & ((w[e] & 0x7fffffffu) > 0x7f800000u);
    } else {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const unsigned long long b = ((unsigned long long)w[2 * e + 1] << 32) | w[2 * e];
        found |= (e < valid) & ((b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull);
      }
    }
  }
  if (__any(found) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

inline unsigned grid_for(long long n, long long per = kThreads) {
  long long g = (n + per - 1) / per;
  if (g < 1) g = 1;
  if (g > 256LL * 32) g = 256LL * 32;
  return (unsigned)g;
}

}  // namespace

// ---------------------------------------------------------------------------------------- exports

CML_API int cml_split_buckets(const long long* rows, long long n, unsigned long long key, const double* cum, int nb,
                              signed char* out, void* stream) {
  if (nb < 1 || nb > 16) return (int)hipErrorInvalidValue;
  Cum c{};
  for (int i = 0; i <= nb; ++i) c.c[i] = cum[i];
  c.nb = nb;
  if (n > 0)
    hipLaunchKernelGGL(split_buckets_kernel, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, rows, n, key,
                       c, out);
  return cml_status();
}

CML_API int cml_poisson1(const long long* rows, long long n, unsigned long long key, const double* thresholds,
                         int kmax, int* out_i32, float* out_f32, void* stream) {
  if (kmax < 1 || kmax > 17) return (int)hipErrorInvalidValue;
  PoissonCdf c{};
  for (int i = 0; i < kmax; ++i) c.t[i] = thresholds[i];
  c.kmax = kmax;
  if (n > 0)
    hipLaunchKernelGGL(poisson1_kernel, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, rows, n, key, c,
                       out_i32, out_f32);
  return cml_status();
}

CML_API int cml_counter_uniform(const long long* rows, long long n, unsigned long long key, double* out,
                                void* stream) {
  if (n > 0)
    hipLaunchKernelGGL(uniform_kernel, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, rows, n, key, out);
  return cml_status();
}

CML_API long long cml_compact_blocks(long long n) { return (n + kCompactTile - 1) / kCompactTile; }

// idx must hold n entries (worst case); bscratch cml_compact_blocks(n) int64; count_out one int64 (device).
CML_API int cml_compact(const unsigned char* mask, long long n, long long* idx, long long* bscratch,
                        long long* count_out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long long nb = (n + kCompactTile - 1) / kCompactTile;
  if (nb > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  if (n <= 0) {
    hipMemsetAsync(count_out, 0, sizeof(long long), st);
    return cml_status();
  }
  hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)nb), dim3(kThreads), 0, st, mask, n, bscratch);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(kThreads), 0, st, bscratch, nb, count_out);
  hipLaunchKernelGGL(compact_scatter_kernel, dim3((unsigned)nb), dim3(kThreads), 0, st, mask, n, bscratch, idx);
  return cml_status();
}

// the smallest row capacity (4, 8 or 16 values) that holds both the columns and the output width
template <int OUT>
int launch_asm_scalar(const AsmCol* c, int ncols, long long n, void* out, long long ldo, unsigned char* invalid,
                      int nan_keep, hipStream_t st) {
  const long long need = ncols > ldo ? ncols : ldo;
  const dim3 grid(grid_for(n, 4LL * kThreads)), block(kThreads);
  if (need <= 4)
    hipLaunchKernelGGL((assemble_scalar_kernel<OUT, 4>), grid, block, 0, st, c, ncols, n, out, ldo, invalid, nan_keep);
  else if (need <= 8)
    hipLaunchKernelGGL((assemble_scalar_kernel<OUT, 8>), grid, block, 0, st, c, ncols, n, out, ldo, invalid, nan_keep);
  else
    hipLaunchKernelGGL((assemble_scalar_kernel<OUT, 16>), grid, block, 0, st, c, ncols, n, out, ldo, invalid,
                       nan_keep);
  return cml_status();
}

// cols: device array of AsmCol (see struct layout: ptr, valid, ld, type, width, out_off, pad).
CML_API int cml_assemble(const void* cols, int ncols, long long n, void* out, int out_dtype, long long ldo, int dout,
                         unsigned char* invalid, int nan_keep, int scalar_only, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const AsmCol* c = (const AsmCol*)cols;
  if (n <= 0) return 0;
  if (scalar_only && ncols <= kAsmMax && ldo <= kAsmMax) {
    switch (out_dtype) {
      case 0: return launch_asm_scalar<0>(c, ncols, n, out, ldo, invalid, nan_keep, st);
      case 1: return launch_asm_scalar<1>(c, ncols, n, out, ldo, invalid, nan_keep, st);
      case 2: return launch_asm_scalar<2>(c, ncols, n, out, ldo, invalid, nan_keep, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  switch (out_dtype) {
    case 0: hipLaunchKernelGGL(assemble_kernel<0>, dim3(grid_for(n)), dim3(kThreads), 0, st, c, ncols, n, out, ldo, dout, invalid, nan_keep); break;
    case 1: hipLaunchKernelGGL(assemble_kernel<1>, dim3(grid_for(n)), dim3(kThreads), 0, st, c, ncols, n, out, ldo, dout, invalid, nan_keep); break;
    case 2: hipLaunchKernelGGL(assemble_kernel<2>, dim3(grid_for(n)), dim3(kThreads), 0, st, c, ncols, n, out, ldo, dout, invalid, nan_keep); break;
    default: return (int)hipErrorInvalidValue;
  }
  return cml_status();
}

CML_API int cml_assemble_col_bytes() { return (int)sizeof(AsmCol); }

CML_API int cml_binarize(const void* x, int type, long long n, double thr, double* out, void* stream) {
  if (n > 0)
    hipLaunchKernelGGL(binarize_kernel, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, x, type, n, thr,
                       out);
  return cml_status();
}

CML_API int cml_metric_grid(long long n) { return (int)grid_for(n, 4LL * kThreads); }

CML_API int cml_reg_metrics(const double* y, const double* p, const double* w, long long n, double* partial, int grid,
                            void* stream) {
  hipLaunchKernelGGL(reg_metrics_kernel, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, y, p, w, n, partial);
  return cml_status();
}

CML_API int cml_cls_confusion(const long long* y, const long long* p, const double* w, long long n, int C,
                              double* partial, int grid, void* stream) {
  if (C < 1 || C > 64) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(kThreads / 64) * C * C * sizeof(double);  // <= 128 KiB (C = 64)
  if (lds > 64 * 1024)
    hipFuncSetAttribute((const void*)cls_confusion_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(cls_confusion_kernel, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, y, p, w, n, C,
                     partial);
  return cml_status();
}

CML_API int cml_col_absmax(const void* x, int dtype, long long n, int d, long long ldx, int rows_per_block,
                           float* partial, void* stream) {
  const long long nb = (n + rows_per_block - 1) / rows_per_block;
  if (nb <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int E = dtype == 0 ? 8 : 4;
  const bool fast = (dtype == 0 || dtype == 1) && d % E == 0 && ldx % E == 0 && d / E <= kThreads && d <= 2048 &&
                    (reinterpret_cast<size_t>(x) & 15) == 0;
  if (fast) {
    if (dtype == 1)
      hipLaunchKernelGGL(col_absmax16_kernel<float>, dim3((unsigned)nb), dim3(kThreads), 0, st, (const float*)x, n, d,
                         ldx, rows_per_block, partial);
    else
      hipLaunchKernelGGL(col_absmax16_kernel<u16>, dim3((unsigned)nb), dim3(kThreads), 0, st, (const u16*)x, n, d,
                         ldx, rows_per_block, partial);
    return cml_status();
  }
  if (dtype == 1)
    hipLaunchKernelGGL(col_absmax_kernel<float>, dim3((unsigned)nb), dim3(kThreads), 0, st, (const float*)x, n, d,
                       ldx, rows_per_block, partial);
  else if (dtype == 0)
    hipLaunchKernelGGL(col_absmax_kernel<u16>, dim3((unsigned)nb), dim3(kThreads), 0, st, (const u16*)x, n, d, ldx,
                       rows_per_block, partial);
  else
    return (int)hipErrorInvalidValue;
  return cml_status();
}

CML_API int cml_quant_fp8(const void* x, int dtype, long long n, int d, long long ldx, const float* scale,
                          unsigned char* out, long long ldo, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int cpr = d / 8;
  const bool pow2 = cpr > 0 && (cpr & (cpr - 1)) == 0;
  const int align = dtype == 0 ? 8 : 4;
  if (ldo == d && d % 8 == 0 && pow2 && ldx % align == 0 && (reinterpret_cast<size_t>(x) & 15) == 0 &&
      (reinterpret_cast<size_t>(scale) & 15) == 0 && (reinterpret_cast<size_t>(out) & 7) == 0 &&
      (dtype == 0 || dtype == 1)) {
    const int sh = __builtin_ctz((unsigned)cpr);
    const long long chunks = n * cpr;
    if (dtype == 1)
      hipLaunchKernelGGL(quant_fp8_v8_kernel<float>, dim3(grid_for(chunks)), dim3(kThreads), 0, st, (const float*)x,
                         n, d, ldx, scale, out, sh);
    else
      hipLaunchKernelGGL(quant_fp8_v8_kernel<u16>, dim3(grid_for(chunks)), dim3(kThreads), 0, st, (const u16*)x, n,
                         d, ldx, scale, out, sh);
    return cml_status();
  }
  const long long total = n * ((ldo + 1) / 2);
  if (dtype == 1)
    hipLaunchKernelGGL(quant_fp8_kernel<float>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const float*)x, n, d,
                       ldx, scale, out, ldo);
  else if (dtype == 0)
    hipLaunchKernelGGL(quant_fp8_kernel<u16>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const u16*)x, n, d, ldx,
                       scale, out, ldo);
  else
    return (int)hipErrorInvalidValue;
  return cml_status();
}

// flag (device int, zeroed by the caller) |= any NaN in x[:, :d]; esize 2 (bf16), 4 (f32), 8 (f64).
CML_API int cml_has_nan(const void* x, long long n, int d, long long ld_bytes, int esize, int* flag, void* stream) {
  if (n <= 0 || d <= 0) return 0;
  if (ld_bytes % 16 != 0 || (reinterpret_cast<size_t>(x) & 15) != 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const long long total = n * ((d * esize + 15) / 16);
  const unsigned char* p = (const unsigned char*)x;
  switch (esize) {
    case 2: hipLaunchKernelGGL(has_nan_kernel<2>, dim3(grid_for(total)), dim3(kThreads), 0, st, p, n, d, ld_bytes, flag); break;
    case 4: hipLaunchKernelGGL(has_nan_kernel<4>, dim3(grid_for(total)), dim3(kThreads), 0, st, p, n, d, ld_bytes, flag); break;
    case 8: hipLaunchKernelGGL(has_nan_kernel<8>, dim3(grid_for(total)), dim3(kThreads), 0, st, p, n, d, ld_bytes, flag); break;
    default: return (int)hipErrorInvalidValue;
  }
  return cml_status();
}
