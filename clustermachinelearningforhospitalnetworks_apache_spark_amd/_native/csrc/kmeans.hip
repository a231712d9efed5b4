// KMeans Lloyd-iteration kernels for gfx950 (MI355X / CDNA4).
//
// Capability parity: the reference has no KMeans; this is the
// north-star workload of BASELINE.json (KMeans fit samples/sec). Kernel IDs
// follow SURVEY.md §2.5: K9 kmeans_assign, K10 kmeans_accumulate, K11 kmeans_update.
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
//     * score = ||c||² − 2·x·c; d = ||x||² + score (clamped at 0) feeds the cost;
//     * optionally (sort regime) each row also gets its rank among the rows of
//       the same label in this workgroup (LDS int counter) and the workgroup
//       writes its label histogram — the first pass of a counting sort, free.
//     Centroid sets larger than the LDS budget run as several launches over
//     centroid chunks (first/last flags carry the running argmin through HBM).
//
// K10 per-cluster sums, two race-free regimes (no float atomics in LDS: measured on
//     MI355X, ds_add_f32 ran 10-12x slower than plain race-free read-modify-write):
//   A kmeans_accum_priv<CPL,RPW> (small k·D): every (wave, row-group) owns a private
//     k×dw f32 copy in LDS; copies summed once; slabs reduced by kmeans_reduce.
//   B sort regime (large k·D): counting sort of row ids by label
//     (hist+rank from K9 -> kmeans_seg_scan -> kmeans_scatter) then
//     kmeans_segacc<CPL>: every wave streams an equal slice of the sorted order,
//     gathering whole rows (8-16 B per lane, U rows in flight) and keeping the
//     running cluster sum in f64 registers; only at cluster boundaries does it
//     flush (f64 global atomics, ~#waves+k flushes per pass). Work per wave is
//     independent of the label distribution (skew-proof).
//   Both produce ONE f64 message [k·D sums | k counts | cost] — exactly the buffer
//   that is all-reduced over RCCL.
// K11 kmeans_update: new centres (empty clusters keep their old centre, as Spark
//     MLlib does), bf16 copy, norms of the bf16 centres, per-centre squared shift.
#include <algorithm>

#include "common.h"

namespace {

constexpr int kAccumThreads = 1024;  // 16 waves
constexpr int kSegThreads = 256;     // 4 waves

// ---------------------------------------------------------------------------------------------
// K9 on v_mfma_f32_16x16x32_bf16. Operand layout (wave64): lane l holds A row (l&15) /
// B column (l&15), k = 8(l>>4) + j; the 16x16 f32 result puts column (l&15) on the lane and
// rows 4(l>>4)+i, i<4, in its 4 registers. X is the B operand (row of X on the lane), the
// -2-scaled centres the A operand. Why 16x16x32 and not 32x32x16: the B operand of a 32-wide
// MFMA forces every global load to touch 32 rows x 32 B (measured 3.5 TB/s ceiling on MI355X),
// the 16-wide one 16 rows x 64 B (6.0 TB/s) — the assign pass is HBM-bound, so the load shape
// decides. It also runs ~1.1x the FLOP/s of the 32-wide form.
// ---------------------------------------------------------------------------------------------
template <int DP>
struct AssignShape {
  static constexpr int NCH = DP / 8;                 // 16-byte chunks per row
  static constexpr int KS = DP >= 32 ? DP / 32 : 1;  // MFMA k-steps per 16x16 block
};

// X fragments of one 16-row sub-tile: lane (row l&15, group g=l>>4) reads chunk 4s+g of its row,
// so each load instruction covers 16 rows x 64 contiguous bytes.
// F8 (OCP e4m3fn storage, half the bytes): one 16-byte load per lane covers TWO k-steps — step
// 2t+h of lane (r,g) holds k = 64t + 16g + 8h + j — still 16 rows x 64 B per instruction; the
// fp8 -> bf16 conversion is exact (e4m3 values are a subset of bf16) and runs once per X tile,
// which is then reused against every centre tile. The centre fragments use the same k order.
template <bool HI>
__device__ __forceinline__ unsigned f8x2_to_bf16x2(unsigned w) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, HI);
  return (__float_as_uint(v.x) >> 16) | (__float_as_uint(v.y) & 0xffff0000u);
}

template <int DP, bool F8>
__device__ __forceinline__ void load_x16(const void* __restrict__ Xv, long long n, long long ldx, long long row0,
                                         int r, int g, bf16x8 (&xf)[AssignShape<DP>::KS]) {
  constexpr int KS = AssignShape<DP>::KS;
  const long long row = row0 + r;
  const bool valid = row < n;
  if constexpr (F8) {
    static_assert(DP >= 64, "fp8 rows are padded to >= 64 features");
    const unsigned char* xp = reinterpret_cast<const unsigned char*>(Xv) + (valid ? row : 0) * ldx;
#pragma unroll
    for (int t = 0; t < KS / 2; ++t) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (valid) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(xp + 64 * t + 16 * g));
      const u32x4 lo = {f8x2_to_bf16x2<false>(v.x), f8x2_to_bf16x2<true>(v.x), f8x2_to_bf16x2<false>(v.y),
                        f8x2_to_bf16x2<true>(v.y)};
      const u32x4 hi = {f8x2_to_bf16x2<false>(v.z), f8x2_to_bf16x2<true>(v.z), f8x2_to_bf16x2<false>(v.w),
                        f8x2_to_bf16x2<true>(v.w)};
      xf[2 * t] = __builtin_bit_cast(bf16x8, lo);
      xf[2 * t + 1] = __builtin_bit_cast(bf16x8, hi);
    }
  } else {
    constexpr int NCH = AssignShape<DP>::NCH;
    const u16* xp = reinterpret_cast<const u16*>(Xv) + (valid ? row : 0) * ldx;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int q = 4 * s + g;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (q < NCH && valid) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(xp + 8 * q));
      xf[s] = __builtin_bit_cast(bf16x8, v);
    }
  }
}

// first k of the 8 a lane of group g holds at MFMA step s (X and centre fragments agree)
template <bool F8>
__device__ __forceinline__ int frag_k0(int s, int g) {
  return F8 ? 64 * (s >> 1) + 16 * g + 8 * (s & 1) : 32 * s + 8 * g;
}

template <int DP, int RT>
struct XTile {
  bf16x8 f[RT][AssignShape<DP>::KS];
};

template <int DP, int RT, bool F8>
__device__ __forceinline__ void load_xtile(const void* __restrict__ X, long long n, long long ldx, long long tile,
                                           int r, int g, XTile<DP, RT>& xt) {
#pragma unroll
  for (int t = 0; t < RT; ++t) load_x16<DP, F8>(X, n, ldx, tile * (16 * RT) + 16 * t, r, g, xt.f[t]);
}

// Centres live in LDS in FRAGMENT order: fragment (ct, s) is 64 lanes x 16 B contiguous, lane l
// holding -2·c[16ct + (l&15)][k = 32s + 8(l>>4) .. +8) (zero past Dp). A lane's read address is
// therefore lane·16 + (ct·KS + s)·1 KiB: conflict-free for ds_read_b128 (16 distinct 16-B bank
// slots per lane group), the s part folds into the instruction's immediate offset and the ct
// part is one add per centre tile — no per-read address arithmetic.
struct AssignCtx {
  const unsigned char* frag;  // this lane's byte address of fragment (0, 0)
  const float* cn;            // ||c||² of the chunk's centres
  int nct;                    // 16-centre tiles
  int cmask;                  // low key bits holding the tile index
};

template <int DP>
__device__ __forceinline__ uint4 frag_at(const AssignCtx& cx, int ct, int s) {
  ct = ct < cx.nct ? ct : cx.nct - 1;  // ring run-ahead past the last tile: harmless re-read
  return *reinterpret_cast<const uint4*>(cx.frag + ((ct * AssignShape<DP>::KS + s) << 10));
}

// Running minimum per (sub-tile, accumulator slot) as ONE signed int key: the f32 distance bits
// with the low `cmask` bits replaced by the centre-tile index. Distances are >= 0 up to rounding;
// a rounding-negative one keys below every positive distance (it IS the near-zero minimum), and
// non-negative f32 order equals int order, so v_and_or + v_min_i32 (2 VALU) replace a compare
// and two selects. The tile index in the low bits makes ties resolve to the earliest tile; the
// truncation costs 2^-(23-bits) relative precision (bits = log2 #tiles, 4 for k = 256).
template <int RT>
__device__ __forceinline__ void slot_update(const f32x4 (&acc)[RT], int t, int i, int ct, int cmask,
                                            int (&key)[RT][4]) {
  const int k = (__float_as_int(acc[t][i]) & ~cmask) | ct;
  key[t][i] = k < key[t][i] ? k : key[t][i];
}

// PACK4: the 4 slots of sub-tile t hold the SAME X row against centres 4g+i, so they merge into
// ONE key per row whose low bits carry (tile, i): 4 v_and_or + 2 v_min3_i32 per 4 distances
// instead of 4 + 4 (and 4x fewer key registers). Two more mantissa bits are truncated
// (2^-17 relative for k = 256).
template <int RT>
__device__ __forceinline__ void group_update(const f32x4 (&acc)[RT], int t, int ct4, int cmask, int (&key)[RT][4]) {
  const int k0 = (__float_as_int(acc[t][0]) & ~cmask) | ct4;
  const int k1 = (__float_as_int(acc[t][1]) & ~cmask) | (ct4 + 1);
  const int k2 = (__float_as_int(acc[t][2]) & ~cmask) | (ct4 + 2);
  const int k3 = (__float_as_int(acc[t][3]) & ~cmask) | (ct4 + 3);
  int m = key[t][0];
  m = min(m, min(k0, k1));
  m = min(m, min(k2, k3));
  key[t][0] = m;
}

template <int RT, bool PACK4>
__device__ __forceinline__ void tile_update_all(const f32x4 (&acc)[RT], int ct, int cmask, int (&key)[RT][4]) {
  if constexpr (PACK4) {
#pragma unroll
    for (int t = 0; t < RT; ++t) group_update<RT>(acc, t, ct << 2, cmask, key);
  } else {
#pragma unroll
    for (int q = 0; q < RT * 4; ++q) slot_update<RT>(acc, q >> 2, q & 3, ct, cmask, key);
  }
}

// MFMA chain of centre tile `ct` for all RT sub-tiles into `acc` (each A fragment feeds RT
// MFMAs), with the slot updates of the previous tile's accumulators interleaved. The first k-step
// of every sub-tile takes its C operand from ONE register set, cinit = ||c||² + moff, where moff
// is the largest ||x||² among the lane's RT rows: the accumulators end as the squared distance
// plus the row's offset moff − ||x||² >= 0 (the packed-key minimum needs non-negative values; the
// epilogue subtracts it). Seeding each sub-tile with its own ||x||² cost RT·4 VALU per centre tile
// in an issue stream where MFMAs leave ~8 of every 16 cycles for everything else.
// Precision: a row's candidates carry the offset moff − ||x||², so their f32 rounding is on the
// scale of the tile's largest norm instead of the row's own. That only matters for rows sharing
// a 64-row tile with an outlier ~100x their norm; bf16 quantisation of x (2^-8 relative in x·c)
// is the larger error below that.
// SHARED = false keeps the per-sub-tile seeding (c4 + ||x||² of each row) — the A/B reference of
// kmeans_ops.set_assign_variant(6); in one process it measured 2.77 vs 2.71 ms full and 2.15 vs
// 2.07 ms compute-only (profiles/assign_shared_seed_ab_20Mx256.log).
template <int DP, int RT, int RING, bool PREV, bool SHARED, bool PACK4>
__device__ __forceinline__ void chain(const AssignCtx& cx, const XTile<DP, RT>& xt, float moff,
                                      const float (&xn)[RT], int ct, int g, f32x4 (&acc)[RT],
                                      const f32x4 (&prev)[RT], uint4 (&ring)[RING], int (&key)[RT][4]) {
  constexpr int KS = AssignShape<DP>::KS;
  constexpr int NSLOT = RT * 4;
  const float4 c4 = *reinterpret_cast<const float4*>(cx.cn + ct * 16 + 4 * g);
  const f32x4 cinit = {c4.x + moff, c4.y + moff, c4.z + moff, c4.w + moff};
  if constexpr (!SHARED) {
#pragma unroll
    for (int t = 0; t < RT; ++t) acc[t] = f32x4{c4.x + xn[t], c4.y + xn[t], c4.z + xn[t], c4.w + xn[t]};
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const uint4 a = ring[s % RING];
    ring[s % RING] = frag_at<DP>(cx, ct + (s + RING) / KS, (s + RING) % KS);
#pragma unroll
    for (int t = 0; t < RT; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), xt.f[t][s],
                                                       (SHARED && s == 0) ? cinit : acc[t], 0, 0, 0);
    if constexpr (PREV && PACK4) {
#pragma unroll
      for (int t = (s * RT) / KS; t < ((s + 1) * RT) / KS; ++t) group_update<RT>(prev, t, (ct - 1) << 2, cx.cmask, key);
    } else if constexpr (PREV) {
#pragma unroll
      for (int q = (s * NSLOT) / KS; q < ((s + 1) * NSLOT) / KS; ++q)
        slot_update<RT>(prev, q >> 2, q & 3, ct - 1, cx.cmask, key);
    }
  }
}

// Incremental sums (Lloyd step on label changes only): the single-launch assign appends every row
// whose label differs from the one it held before this step to its WORKGROUP's list
// (rows/old[b * pcap ...], one LDS counter per workgroup, one LDS atomic per wave batch; a single
// global counter serialised ~8M atomics per pass when many labels moved). wg_count[b] receives the
// list length; a list longer than pcap sets *overflow (the step then re-accumulates in full).
struct DeltaOut {
  int* rows;
  int* old;
  int* wg_count;
  int* overflow;
  int pcap;
  int* lds_count;  // set in the kernel
};

template <int DP, int RT, int RINGMAX, bool SHARED, bool PACK4>
__device__ __forceinline__ void assign_tile(const AssignCtx& cx, const XTile<DP, RT>& xt, long long tile,
                                            long long n, int r, int g, int c_base, const float* __restrict__ xnorm,
                                            int* __restrict__ labels, float* __restrict__ best_io, int first,
                                            int last, bool ranking, int* hist, int* __restrict__ rank_out,
                                            const DeltaOut& dout, double& cost) {
  constexpr int KS = AssignShape<DP>::KS;
  constexpr int RING = KS < RINGMAX ? KS : RINGMAX;
  float xn[RT];
  float moff = 0.f;  // largest ||x||² of this lane's rows (see chain)
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const long long row = tile * (16 * RT) + 16 * t + r;
    xn[t] = row < n ? xnorm[row] : 0.f;
    moff = fmaxf(moff, xn[t]);
  }
  int key[RT][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) key[t][i] = 0x7fffffff;
  uint4 ring[RING];
#pragma unroll
  for (int q = 0; q < RING; ++q) ring[q] = frag_at<DP>(cx, q / KS, q % KS);
  f32x4 acc0[RT], acc1[RT];
  const int nct = cx.nct;
  chain<DP, RT, RING, false, SHARED, PACK4>(cx, xt, moff, xn, 0, g, acc0, acc1, ring, key);
  int ct = 1;
  for (; ct + 1 < nct; ct += 2) {
    chain<DP, RT, RING, true, SHARED, PACK4>(cx, xt, moff, xn, ct, g, acc1, acc0, ring, key);
    chain<DP, RT, RING, true, SHARED, PACK4>(cx, xt, moff, xn, ct + 1, g, acc0, acc1, ring, key);
  }
  if (ct < nct) {
    chain<DP, RT, RING, true, SHARED, PACK4>(cx, xt, moff, xn, ct, g, acc1, acc0, ring, key);
    tile_update_all<RT, PACK4>(acc1, ct, cx.cmask, key);
  } else {
    tile_update_all<RT, PACK4>(acc0, ct - 1, cx.cmask, key);
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    // slot (t,i) holding tile c is centre 16c + 4g + i
    float best = __int_as_float(key[t][0] & ~cx.cmask);
    int bidx;
    if constexpr (PACK4) {
      const int tag = key[t][0] & cx.cmask;  // (tile << 2) | i: centre 16 tile + 4g + i
      bidx = (tag >> 2) * 16 + 4 * g + (tag & 3);
    } else {
      bidx = (key[t][0] & cx.cmask) * 16 + 4 * g;
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        const float v = __int_as_float(key[t][i] & ~cx.cmask);
        const int idx = (key[t][i] & cx.cmask) * 16 + 4 * g + i;
        if (v < best || (v == best && idx < bidx)) { best = v; bidx = idx; }
      }
    }
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bidx, o, 64);
      if (ob < best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    bidx += c_base;
    if constexpr (SHARED) best = best - moff + xn[t];  // remove the row offset: squared distance
    const long long row = tile * (16 * RT) + 16 * t + r;
    const bool mine = g == 0 && row < n;
    if (!first && mine) {
      const float pb = best_io[row];
      const int pi = labels[row];
      if (pb <= best) { best = pb; bidx = pi; }  // earlier chunks hold smaller indices
    }
    if (dout.rows != nullptr) {  // incremental sums: log rows whose label changed (single-launch assign)
      const int prev = mine ? labels[row] : bidx;
      const bool ch = mine && prev != bidx;
      const unsigned long long bal = __ballot(ch);
      if (bal != 0ull) {
        const int lane = r + 16 * g;
        const int leader = __builtin_ctzll(bal);
        int base = 0;
        if (lane == leader) base = atomicAdd(dout.lds_count, (int)__popcll(bal));
        base = __shfl(base, leader, 64);
        const int at = base + (int)__popcll(bal & ((1ull << lane) - 1ull));
        if (ch && at < dout.pcap) {
          const long long o = (long long)blockIdx.x * dout.pcap + at;
          dout.rows[o] = (int)row;
          dout.old[o] = prev;
        }
      }
    }
    if (mine) {
      labels[row] = bidx;
      if (last) {
        const float d = fmaxf(best, 0.f);
        if (best_io != nullptr) best_io[row] = d;
        cost += (double)d;
        if (ranking) rank_out[row] = atomicAdd(hist + bidx, 1);
      } else {
        best_io[row] = best;
      }
    }
  }
}

// NT threads; each wave owns super-tiles of RT x 16 rows. PF: the next super-tile's rows are in
// flight while this one computes (double-buffered X registers).
template <int DP, int RT, int NT, bool PF, int RINGMAX, bool F8, bool SHARED = true, bool PACK4 = false>
__global__ __launch_bounds__(NT, 1) void kmeans_assign_bf16(
    const void* __restrict__ X, long long n, long long ldx, const u16* __restrict__ C, long long ldc,
    int kc, int kp, int c_base, const float* __restrict__ cnorm, const float* __restrict__ xnorm,
    int* __restrict__ labels, float* __restrict__ best_io, int first, int last, double* __restrict__ cost_part,
    int* __restrict__ hist_out, int* __restrict__ rank_out, DeltaOut dout, int sched) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NCH = AssignShape<DP>::NCH;
  constexpr int KS = AssignShape<DP>::KS;
  const int nct = kc >> 4;
  uint4* fr = reinterpret_cast<uint4*>(smem);
  float* cn = reinterpret_cast<float*>(smem + (size_t)nct * KS * 1024);
  int* hist = reinterpret_cast<int*>(cn + kc);
  double* red = reinterpret_cast<double*>(hist + ((kp + 3) & ~3));
  dout.lds_count = reinterpret_cast<int*>(red + 16);

  const int tid = threadIdx.x;
  for (int id = tid; id < nct * KS * 64; id += NT) {
    const int l = id & 63, f = id >> 6;  // fragment f = ct*KS + s
    const int ct = f / KS, st = f - ct * KS;
    const int c = ct * 16 + (l & 15), k0 = frag_k0<F8>(st, l >> 4);
    unsigned o[4] = {0u, 0u, 0u, 0u};
    if (k0 < 8 * NCH) {
      const uint4 v = *reinterpret_cast<const uint4*>(C + (long long)c * ldc + k0);
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // x -2, exact: bf16 -> f32 -> bf16 round trip of a power-of-two scale
        const float lo = -2.f * bf16_to_f32((u16)(w[e] & 0xffffu));
        const float hi = -2.f * bf16_to_f32((u16)(w[e] >> 16));
        o[e] = (unsigned)f32_to_bf16(lo) | ((unsigned)f32_to_bf16(hi) << 16);
      }
    }
    fr[id] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  for (int i = tid; i < kc; i += NT) cn[i] = cnorm[i];
  const bool ranking = last && rank_out != nullptr;
  if (ranking)
    for (int i = tid; i < kp; i += NT) hist[i] = 0;
  if (tid == 0) *dout.lds_count = 0;
  __syncthreads();

  constexpr int nwaves = NT / 64;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  constexpr int ROWS = 16 * RT;
  const long long ntiles = (n + ROWS - 1) / ROWS;
  const long long tw = (long long)gridDim.x * nwaves;
  double cost = 0.0;

  AssignCtx cx;
  cx.frag = smem + lane * 16;
  cx.cn = cn;
  cx.nct = nct;
  int bits = 1;
  while ((1 << bits) < nct) ++bits;
  if (PACK4) bits += 2;
  cx.cmask = (1 << bits) - 1;

  long long tile = (long long)blockIdx.x * nwaves + wave;
  // SIMD partners (waves w and w + 4) run the same program: desynchronise them so one streams its
  // next X tile while the other computes (sched bit 0: static priority for the second half, bit 1:
  // the second half starts ~sched>>2 x 512 cycles late).
  if (wave >= nwaves / 2) {
    if (sched & 1) __builtin_amdgcn_s_setprio(1);
    if (sched & 2)
      for (int i = 0; i < (sched >> 2); ++i) __builtin_amdgcn_s_sleep(8);
  }
  if constexpr (PF) {
    XTile<DP, RT> xa, xb;
    if (tile < ntiles) load_xtile<DP, RT, F8>(X, n, ldx, tile, r, g, xa);
    for (; tile < ntiles; tile += 2 * tw) {
      const long long t1 = tile + tw;
      if (t1 < ntiles) load_xtile<DP, RT, F8>(X, n, ldx, t1, r, g, xb);
      assign_tile<DP, RT, RINGMAX, SHARED, PACK4>(cx, xa, tile, n, r, g, c_base, xnorm, labels, best_io, first, last, ranking, hist,
                          rank_out, dout, cost);
      if (t1 >= ntiles) break;
      if (t1 + tw < ntiles) load_xtile<DP, RT, F8>(X, n, ldx, t1 + tw, r, g, xa);
      assign_tile<DP, RT, RINGMAX, SHARED, PACK4>(cx, xb, t1, n, r, g, c_base, xnorm, labels, best_io, first, last, ranking, hist,
                          rank_out, dout, cost);
    }
  } else {
    for (; tile < ntiles; tile += tw) {
      XTile<DP, RT> xt;
      load_xtile<DP, RT, F8>(X, n, ldx, tile, r, g, xt);
      assign_tile<DP, RT, RINGMAX, SHARED, PACK4>(cx, xt, tile, n, r, g, c_base, xnorm, labels, best_io, first, last, ranking, hist,
                          rank_out, dout, cost);
    }
  }
  if (last && (cost_part != nullptr || ranking)) {
    cost = wave_sum_f64(cost);
    if (lane == 0) red[wave] = cost;
    __syncthreads();
    if (tid == 0 && cost_part != nullptr) {
      double t = 0.0;
      for (int w = 0; w < nwaves; ++w) t += red[w];
      cost_part[blockIdx.x] = t;
    }
    if (ranking)
      for (int i = tid; i < kp; i += NT) hist_out[(long long)blockIdx.x * kp + i] = hist[i];
    if (dout.rows != nullptr && tid == 0) {
      const int c = *dout.lds_count;
      dout.wg_count[blockIdx.x] = c < dout.pcap ? c : dout.pcap;
      if (c > dout.pcap) *dout.overflow = 1;
    }
  }
}

}  // namespace

#include "kmeans_rr.h"

namespace {

template <int CPL>
__device__ __forceinline__ void load_cols(const u16* p, float (&v)[CPL]) {
  if constexpr (CPL == 2) {
    const unsigned w = *reinterpret_cast<const unsigned*>(p);
    v[0] = bf16_to_f32((u16)(w & 0xffffu));
    v[1] = bf16_to_f32((u16)(w >> 16));
  } else if constexpr (CPL == 4) {
    const uint2 w = *reinterpret_cast<const uint2*>(p);
    v[0] = bf16_to_f32((u16)(w.x & 0xffffu));
    v[1] = bf16_to_f32((u16)(w.x >> 16));
    v[2] = bf16_to_f32((u16)(w.y & 0xffffu));
    v[3] = bf16_to_f32((u16)(w.y >> 16));
  } else {
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = bf16_to_f32((u16)(ws[q] & 0xffffu));
      v[2 * q + 1] = bf16_to_f32((u16)(ws[q] >> 16));
    }
  }
}

// K10 regime A (small k·dw): private accumulator copy per (wave, row-group).
template <int CPL, int RPW>
__global__ __launch_bounds__(kAccumThreads) void kmeans_accum_priv(
    const u16* __restrict__ X, long long n, long long ldx, const int* __restrict__ labels, int k, int dw,
    float* __restrict__ slab, int* __restrict__ cslab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = kAccumThreads / 64;
  constexpr int LPR = 64 / RPW;
  constexpr int NC = NW * RPW;
  constexpr int U = 8;
  float* acc = reinterpret_cast<float*>(smem);                      // [NC][k][dw]
  int* cnt = reinterpret_cast<int*>(smem + (size_t)NC * k * dw * 4);  // [NC][k]
  const int tid = threadIdx.x;
  for (int i = tid; i < NC * k * dw; i += blockDim.x) acc[i] = 0.f;
  for (int i = tid; i < NC * k; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane / LPR, li = lane - sub * LPR;
  const int copy = wave * RPW + sub;
  float* wacc = acc + (size_t)copy * k * dw;
  int* wcnt = cnt + copy * k;
  const bool active = CPL * li < dw;
  const long long col0 = (long long)blockIdx.y * dw + CPL * li;
  const bool counter = blockIdx.y == 0 && li == 0;
  const long long step = (long long)gridDim.x * NW * RPW;
  for (long long r0 = ((long long)blockIdx.x * NW + wave) * RPW + sub; r0 < n; r0 += step * U) {
    float v[U][CPL];
    int lab[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + u * step;
      lab[u] = row < n ? labels[row] : -1;
      if (row < n && active) {
        load_cols<CPL>(X + row * ldx + col0, v[u]);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) v[u][j] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int l = lab[u];
      if (l >= 0) {
        if (active) {
          float* p = wacc + (size_t)l * dw + CPL * li;
#pragma unroll
          for (int j = 0; j < CPL; ++j) p[j] += v[u][j];
        }
        if (counter) wcnt[l] += 1;
      }
    }
  }
  __syncthreads();
  float* out = slab + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * (long long)k * dw;
  for (int i = tid; i < k * dw; i += blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < NC; ++c) s += acc[(size_t)c * k * dw + i];
    out[i] = s;
  }
  if (blockIdx.y == 0)
    for (int i = tid; i < k; i += blockDim.x) {
      int s = 0;
      for (int c = 0; c < NC; ++c) s += cnt[c * k + i];
      cslab[(long long)blockIdx.x * k + i] = s;
    }
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

// Sort regime, pass 2a: tot[c] = Σ_b hist[b][c]   (one block per cluster).
__global__ __launch_bounds__(256) void kmeans_seg_totals(const int* __restrict__ hist, int nblk, int kp,
                                                         long long* __restrict__ tot, const int* __restrict__ gate,
                                                         int want) {
  if (gate != nullptr && gate[0] != want) return;  // step-mode gate (incremental sums)
  __shared__ long long ws[4];
  const int c = blockIdx.x, tid = threadIdx.x;
  long long s = 0;
  for (int b = tid; b < nblk; b += blockDim.x) s += hist[(long long)b * kp + c];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) ws[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) tot[c] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Sort regime, pass 2b (one block per cluster): seg[c] = Σ_{c'<c} tot[c'] (first sorted position of
// cluster c; seg[k] = n), off[c][b] = seg[c] + Σ_{b'<b} hist[b'][c], counts and cost into the message.
__global__ __launch_bounds__(256) void kmeans_seg_offsets(const int* __restrict__ hist, int nblk, int k, int kp,
                                                          const long long* __restrict__ tot,
                                                          const double* __restrict__ cost_part, int ncost, int D,
                                                          int* __restrict__ off, int* __restrict__ seg,
                                                          double* __restrict__ msg, const int* __restrict__ gate,
                                                          int want) {
  if (gate != nullptr && gate[0] != want) return;  // step-mode gate (incremental sums)
  __shared__ long long ws[4];
  __shared__ long long carry;
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long s = 0;
  for (int i = tid; i < c; i += blockDim.x) s += tot[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) ws[wave] = s;
  __syncthreads();
  const long long base = ws[0] + ws[1] + ws[2] + ws[3];
  const long long kd = (long long)k * D;
  if (tid == 0) {
    seg[c] = (int)base;
    msg[kd + c] = (double)tot[c];
    carry = base;
    if (c == k - 1) {
      seg[k] = (int)(base + tot[c]);
      double cs = 0.0;
      for (int i = 0; i < ncost; ++i) cs += cost_part[i];
      msg[kd + k] = cs;
    }
  }
  __syncthreads();
  for (int b0 = 0; b0 < nblk; b0 += blockDim.x) {
    const int b = b0 + tid;
    const long long v = b < nblk ? hist[(long long)b * kp + c] : 0;
    long long incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    __syncthreads();
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    long long pre = carry;
    for (int w = 0; w < wave; ++w) pre += ws[w];
    if (b < nblk) off[(long long)c * nblk + b] = (int)(pre + incl - v);
    __syncthreads();
    if (tid == blockDim.x - 1) carry = pre + incl;
    __syncthreads();
  }
}

// Sort regime, pass 3: perm[off[label][block(row)] + rank[row]] = row.
// One workgroup per assign workgroup b: it walks exactly the rows b ranked (groups of
// nwaves*tile_rows consecutive rows every nblk*nwaves tiles), so the block index needs no
// per-row 64-bit division, and b's k offsets sit in LDS instead of being gathered per row.
// Every thread keeps kScatterU of b's rounds' loads in flight (one dependent load pair per thread
// left the pass latency-bound). All of b's rows stay on ONE workgroup: its (b, label) output runs
// are then written from one CU / L2 only — splitting a run over workgroups on several XCDs made
// the partial-line writes 1.4x slower.
constexpr int kScatterThreads = 512;
constexpr int kScatterU = 4;
__global__ __launch_bounds__(kScatterThreads) void kmeans_scatter(const int* __restrict__ labels,
                                                                  const int* __restrict__ rank, long long n, int nblk,
                                                                  int nwaves, int tile_rows, int k,
                                                                  const int* __restrict__ off, int* __restrict__ perm,
                                                                  const int* __restrict__ gate, int want) {
  extern __shared__ int soff[];
  if (gate != nullptr && gate[0] != want) return;  // step-mode gate (incremental sums)
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < k; c += blockDim.x) soff[c] = off[(long long)c * nblk + b];
  __syncthreads();
  const long long grp = (long long)nwaves * tile_rows;  // rows b owns per round
  const long long stride = grp * nblk;                  // rows between two of b's rounds
  // every thread of the block works: `per` of b's rounds side by side (K9r's rounds are one 64-row
  // tile, so a one-round-at-a-time walk left 448 of the 512 threads idle and the pass latency-bound)
  const int per = (long long)blockDim.x >= grp ? (int)(blockDim.x / grp) : 1;
  const int ro = per > 1 ? (int)(threadIdx.x / grp) : 0;
  if (ro >= per) return;
  const long long o0 = per > 1 ? (long long)threadIdx.x - ro * grp : (long long)threadIdx.x;
  const long long ostep = per > 1 ? grp : (long long)blockDim.x;
  for (long long q0 = ro; (long long)b * grp + q0 * stride < n; q0 += (long long)per * kScatterU) {
    for (long long o = o0; o < grp; o += ostep) {
      int lab[kScatterU], rk[kScatterU];
      long long rows[kScatterU];
#pragma unroll
      for (int u = 0; u < kScatterU; ++u) {
        rows[u] = (long long)b * grp + (q0 + (long long)u * per) * stride + o;
        lab[u] = rows[u] < n ? labels[rows[u]] : -1;
        rk[u] = rows[u] < n ? rank[rows[u]] : 0;
      }
#pragma unroll
      for (int u = 0; u < kScatterU; ++u)
        if (lab[u] >= 0) {
          const long long pos = (long long)soff[lab[u]] + rk[u];
          if (pos < n) perm[pos] = (int)rows[u];  // ranks from this step's assign: always
        }
    }
  }
}

template <int CPL> struct RawCols;
template <> struct RawCols<2> { using T = unsigned; };
template <> struct RawCols<4> { using T = uint2; };
template <> struct RawCols<8> { using T = uint4; };

template <int CPL>
__device__ __forceinline__ void add_raw(double (&acc)[CPL], const typename RawCols<CPL>::T& w) {
  const unsigned* ws = reinterpret_cast<const unsigned*>(&w);
#pragma unroll
  for (int q = 0; q < CPL / 2; ++q) {
    acc[2 * q] += (double)bf16_to_f32((u16)(ws[q] & 0xffffu));
    acc[2 * q + 1] += (double)bf16_to_f32((u16)(ws[q] >> 16));
  }
}

// The same on the sum grid: every value scaled by qs = 2^S and rounded to an integer (exact in f64),
// so the f64 sums are exact integers whatever the data's exponent span (models/kmeans.py _sum_grid).
// qsf = qs as an f32 normal (0 when qs is outside f32's normal range): a bf16 value times a power of
// two is then exact in f32 (|x·qs| <= 2^(53 - log2 n) by the grid's choice, far inside the range; a
// result below the normal range rounds to 0 either way), and rintf rounds it half-to-even as rint
// does, so the f32 form gives the same integers at full-rate f32 instead of f64 mul + round.
template <int CPL>
__device__ __forceinline__ void add_raw_q(double (&acc)[CPL], const typename RawCols<CPL>::T& w, double qs,
                                          float qsf) {
  const unsigned* ws = reinterpret_cast<const unsigned*>(&w);
  if (qsf != 0.f) {
#pragma unroll
    for (int q = 0; q < CPL / 2; ++q) {
      acc[2 * q] += (double)rintf(bf16_to_f32((u16)(ws[q] & 0xffffu)) * qsf);
      acc[2 * q + 1] += (double)rintf(bf16_to_f32((u16)(ws[q] >> 16)) * qsf);
    }
  } else {
#pragma unroll
    for (int q = 0; q < CPL / 2; ++q) {
      acc[2 * q] += rint((double)bf16_to_f32((u16)(ws[q] & 0xffffu)) * qs);
      acc[2 * q + 1] += rint((double)bf16_to_f32((u16)(ws[q] >> 16)) * qs);
    }
  }
}

__device__ __forceinline__ float grid_scale_f32(double qs) {
  return (qs >= 0x1p-126 && qs <= 0x1p126) ? (float)qs : 0.f;
}

// OCP e4m3fn rows: CPL bytes per lane.
template <int CPL> struct RawCols8;
template <> struct RawCols8<4> { using T = unsigned; };
template <> struct RawCols8<8> { using T = uint2; };
template <> struct RawCols8<16> { using T = uint4; };

template <int CPL>
__device__ __forceinline__ void add_raw8(double (&acc)[CPL], const typename RawCols8<CPL>::T& w) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const unsigned* ws = reinterpret_cast<const unsigned*>(&w);
#pragma unroll
  for (int q = 0; q < CPL / 4; ++q) {
    const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], false);
    const f2 b = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], true);
    acc[4 * q] += (double)a.x;
    acc[4 * q + 1] += (double)a.y;
    acc[4 * q + 2] += (double)b.x;
    acc[4 * q + 3] += (double)b.y;
  }
}

template <int CPL>
__device__ __forceinline__ void add_raw8_f32(float (&acc)[CPL], const typename RawCols8<CPL>::T& w) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const unsigned* ws = reinterpret_cast<const unsigned*>(&w);
#pragma unroll
  for (int q = 0; q < CPL / 4; ++q) {
    const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], false);
    const f2 b = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], true);
    acc[4 * q] += a.x;
    acc[4 * q + 1] += a.y;
    acc[4 * q + 2] += b.x;
    acc[4 * q + 3] += b.y;
  }
}

template <int CPL, bool F8> struct SegRaw { using T = typename RawCols<CPL>::T; };
template <int CPL> struct SegRaw<CPL, true> { using T = typename RawCols8<CPL>::T; };

// Σ (x_j - c_j)² over this lane's CPL columns of a raw row (bf16 or e4m3 bytes), f32.
template <int CPL, bool F8>
__device__ __forceinline__ float sqdist_raw(const typename SegRaw<CPL, F8>::T& w, const float (&cv)[CPL]) {
  const unsigned* ws = reinterpret_cast<const unsigned*>(&w);
  float s = 0.f;
  if constexpr (F8) {
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int q = 0; q < CPL / 4; ++q) {
      const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], false);
      const f2 b = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[q], true);
      const float e0 = a.x - cv[4 * q], e1 = a.y - cv[4 * q + 1], e2 = b.x - cv[4 * q + 2], e3 = b.y - cv[4 * q + 3];
      s = fmaf(e0, e0, s);
      s = fmaf(e1, e1, s);
      s = fmaf(e2, e2, s);
      s = fmaf(e3, e3, s);
    }
  } else {
#pragma unroll
    for (int q = 0; q < CPL / 2; ++q) {
      const float e0 = bf16_to_f32((u16)(ws[q] & 0xffffu)) - cv[2 * q];
      const float e1 = bf16_to_f32((u16)(ws[q] >> 16)) - cv[2 * q + 1];
      s = fmaf(e0, e0, s);
      s = fmaf(e1, e1, s);
    }
  }
  return s;
}

// Wave total of v by DPP (quad swaps, half-row and row mirrors, row broadcasts 15 / 31): six vector
// adds and no LDS traffic; the total is read from lane 63 into a scalar register.
__device__ __forceinline__ float wave_total_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));   // quad [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));   // quad [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xf, 0xf, false));  // row_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false));  // row_bcast15
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false));  // row_bcast31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Row totals of a batch of 16 rows by a transposing butterfly: s[u] is this lane's partial of row u.
// Each xor level halves the values a lane carries (it keeps one half of the rows and adds its
// partner's partials of them), so 8 + 4 + 2 + 1 shuffles and two quad DPP steps leave row
// 8·b5 + 4·b4 + 2·b3 + b2 (bits of the lane id) summed over the wave, and lane u < 16 reads row u
// from lane 4u: 18 cross-lane ops for 16 rows instead of 16 wave totals of 6 DPP steps each.
__device__ __forceinline__ float batch16_totals(const float (&s)[16]) {
  const int lane = threadIdx.x & 63;
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8, h2 = lane & 4;
  float a[8], b[4], c[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (h5 ? s[8 + i] : s[i]) + __shfl_xor(h5 ? s[i] : s[8 + i], 32, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) b[i] = (h4 ? a[4 + i] : a[i]) + __shfl_xor(h4 ? a[i] : a[4 + i], 16, 64);
#pragma unroll
  for (int i = 0; i < 2; ++i) c[i] = (h3 ? b[2 + i] : b[i]) + __shfl_xor(h3 ? b[i] : b[2 + i], 8, 64);
  float v = (h2 ? c[1] : c[0]) + __shfl_xor(h2 ? c[0] : c[1], 4, 64);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));  // quad [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));  // quad [2,3,0,1]
  return __shfl(v, 4 * (lane & 15), 64);
}

// Optional side output of the segmented accumulate (UB): ub[row] = an upper bound of |x - c_label|
// over the bf16 centres `cb` (row stride ldc) the labels were assigned against — the exact-pruning
// upper bound of every row, formed while the rows stream through (models/kmeans.py _step_seeded).
struct SegUB {
  const u16* cb;
  long long ldc;
  float* ub;
  double qs;             // sum grid scale (0: plain f64 sums of the raw values)
  const float* cu = nullptr;  // offset-form bounds: ub - cu[label] is stored (kmeans_prune.hip)
};

// Sort regime, pass 4: segmented sum over the label-sorted order. Wave w streams sorted
// positions [w*chunk, (w+1)*chunk): ONE vector load fetches the next U row ids, U whole-row
// gathers (CPL*2 bytes per lane) are in flight, the running sum stays in f64 registers, and
// the wave flushes only at cluster boundaries and at the end of its slice. The common chunk
// (no boundary inside) takes an unpredicated path.
// Deterministic, atomic-free flushes: a cluster that starts and ends inside the slice belongs
// to this wave alone and is STORED into the message; the slice's first cluster (may have begun
// in earlier slices) goes to slot A[w], its last (may continue in later slices) to slot B[w];
// kmeans_seg_fixup adds the slots in ascending wave order. The result is bitwise identical
// run to run (SURVEY.md §5.2 deterministic-reduction mode, here the only mode).
// Positions per wave slice: an even split, but at least 128 (a short delta list — the incremental
// steps' moved rows — then occupies few waves, so a cluster spans few slices and the fixup stays short).
__device__ __forceinline__ long long seg_chunk(long long filled, long long waves) {
  const long long c = (filled + waves - 1) / waves;
  return c > 128 ? c : 128;
}

template <int CPL, bool F8, bool UB = false, bool Q = false>
__global__ __launch_bounds__(kSegThreads, (CPL <= 4 ? 4 : 1)) void kmeans_segacc(const void* __restrict__ X, long long n, long long ldx,
                                                             int Dp, int D, const int* __restrict__ perm,
                                                             const int* __restrict__ seg, int k,
                                                             double* __restrict__ msg, double* __restrict__ slots,
                                                             int* __restrict__ slot_c, const int* __restrict__ gate,
                                                             int want, SegUB sub) {
  using raw_t = typename SegRaw<CPL, F8>::T;
  constexpr int U = 16;
  if (gate != nullptr && gate[0] != want) return;  // step-mode gate (incremental sums)
  const unsigned char* xb = reinterpret_cast<const unsigned char*>(X);
  constexpr int ESZ = F8 ? 1 : 2;  // bytes per element
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (kSegThreads / 64) + (threadIdx.x >> 6);
  // slices follow the positions actually filled (seg[k], on the device): a delta list is bounded by
  // 2·cap on the host but usually holds far fewer entries, which must still spread over every wave
  n = n < (long long)seg[k] ? n : (long long)seg[k];
  const long long chunk = seg_chunk(n, (long long)gridDim.x * (kSegThreads / 64));
  const long long p0 = wave * chunk;
  if (p0 >= n) {
    if (lane == 0) {
      slot_c[2 * wave] = -1;
      slot_c[2 * wave + 1] = -1;
    }
    return;
  }
  double* slotA = slots + (2 * wave) * (long long)D;
  double* slotB = slotA + D;
  int nflush = 0;
  const long long p1 = p0 + chunk < n ? p0 + chunk : n;
  int lo = 0, hi = k;  // invariant: seg[lo] <= p0 < seg[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (seg[mid] <= p0) lo = mid; else hi = mid;
  }
  int c = lo;
  long long next = seg[c + 1];
  while (next <= p0) { ++c; next = seg[c + 1]; }  // skip empty clusters
  const int col = CPL * lane;
  const bool active = col < Dp;
  double acc[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) acc[j] = 0.0;
  float cv[CPL];  // UB: this lane's columns of centre c
  auto load_cv = [&](int cc) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) cv[j] = active ? bf16_to_f32(sub.cb[(long long)cc * sub.ldc + col + j]) : 0.f;
  };
  if constexpr (UB) load_cv(c);
  const float qsf = grid_scale_f32(sub.qs);
  // f32 sum of <= 512 rounded squares of exact differences: relative error < 2^-14; rounded up
  auto ub_of = [](float s) { return sqrtf(s * (1.0f + 1.0f / 8192.0f)) * (1.0f + 1e-6f); };
  // offset form: ub - cu[label], rounded up
  auto ub_store = [&](float u, int cc) {
    if (sub.cu == nullptr) return u;
    const float cu = sub.cu[cc];
    return (u - cu) + 1e-6f * (u + cu);
  };
  // the next batch's row ids are loaded one batch ahead: the row gathers then wait for one memory
  // round trip per batch instead of two dependent ones (the pass was latency-bound at 3.7 TB/s)
  int pr_next = (lane < U && p0 + lane < p1) ? perm[p0 + lane] : 0;
  for (long long p = p0; p < p1; p += U) {
    const int cnt = (int)(p1 - p < U ? p1 - p : U);
    const int pr = pr_next;
    pr_next = (lane < U && p + U + lane < p1) ? perm[p + U + lane] : 0;
    float mine = 0.f;  // UB: squared distance of the batch's row `lane`
    raw_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = __builtin_amdgcn_readlane(pr, u);
      if (u < cnt && active) {
        w[u] = *reinterpret_cast<const raw_t*>(xb + (row * ldx + col) * ESZ);
      } else {
        w[u] = raw_t{};
      }
    }
    const long long pe = p + cnt;
    if (next >= pe) {
      if constexpr (UB) {
        static_assert(U == 16, "batch16_totals");
        if constexpr (CPL <= 8) {
          float sq[U];
#pragma unroll
          for (int u = 0; u < U; ++u) sq[u] = sqdist_raw<CPL, F8>(w[u], cv);
          mine = batch16_totals(sq);
        } else {  // 16 B per lane per row: the 16 partials would not fit beside the batch
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const float t = wave_total_dpp(sqdist_raw<CPL, F8>(w[u], cv));
            mine = lane == u ? t : mine;
          }
        }
        if (lane < cnt) sub.ub[pr] = ub_store(ub_of(mine), c);
      }
      if constexpr (F8) {
        // e4m3 values are multiples of 2^-9 below 2^9: 16 of them sum EXACTLY in f32, so the rows
        // are added in f32 and folded into f64 once per batch (half the f64 adds and conversions)
        float part[CPL];
#pragma unroll
        for (int j = 0; j < CPL; ++j) part[j] = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) add_raw8_f32<CPL>(part, w[u]);
#pragma unroll
        for (int j = 0; j < CPL; ++j) acc[j] += (double)part[j];
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr (Q) add_raw_q<CPL>(acc, w[u], sub.qs, qsf);
          else add_raw<CPL>(acc, w[u]);
        }
      }
    } else {
      // a cluster boundary inside this batch (~k + #waves batches per pass): walk its rows one at a
      // time, re-reading each (cache hits) instead of keeping the batch's registers live — the
      // unrolled predicated form doubled the kernel's VGPRs and halved its occupancy
      int rc = c;  // UB: the cluster of the batch's row `lane`
#pragma unroll 1
      for (int u = 0; u < cnt; ++u) {
        const long long pos = p + u;
        while (pos >= next) {  // cluster c ended before pos
          double* dst = nflush == 0 ? slotA : msg + (long long)c * D;  // later clusters are ours alone
          if (active) {
#pragma unroll
            for (int j = 0; j < CPL; ++j)
              if (col + j < D) dst[col + j] = acc[j];
          }
          if (nflush == 0 && lane == 0) slot_c[2 * wave] = c;
          ++nflush;
#pragma unroll
          for (int j = 0; j < CPL; ++j) acc[j] = 0.0;
          ++c;
          next = seg[c + 1];
          while (next <= pos && c < k - 1) { ++c; next = seg[c + 1]; }
          if constexpr (UB) load_cv(c);
        }
        const long long row = __builtin_amdgcn_readlane(pr, u);
        raw_t v = raw_t{};
        if (active) v = *reinterpret_cast<const raw_t*>(xb + (row * ldx + col) * ESZ);
        if constexpr (UB) {
          const float t = wave_total_dpp(sqdist_raw<CPL, F8>(v, cv));
          mine = lane == u ? t : mine;
          rc = lane == u ? c : rc;
        }
        if constexpr (F8) add_raw8<CPL>(acc, v);
        else if constexpr (Q) add_raw_q<CPL>(acc, v, sub.qs, qsf);
        else add_raw<CPL>(acc, v);
      }
      if constexpr (UB) {
        if (lane < cnt) sub.ub[pr] = ub_store(ub_of(mine), rc);
      }
    }
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < CPL; ++j)
      if (col + j < D) slotB[col + j] = acc[j];
  }
  if (lane == 0) {
    if (nflush == 0) slot_c[2 * wave] = -1;
    slot_c[2 * wave + 1] = c;
  }
}

// ---------------------------------------------------------------------------------------------------
// Pruned k-means|| candidate pass (models/kmeans.py _init_candidate_pass_pruned). A row x whose
// nearest candidate so far is p at distance r (cost, plus the slack of the pass that measured it) can
// only move to a new candidate y with |p - y| < 2r (else |x - y| >= |p - y| - r >= r). tab_v[p] holds
// the distances from p to the m new candidates sorted ascending (rounded down), tab_j their indices:
// L(x) = #{y : tab_v[p][y] < 2r} new candidates are relevant. L = 0: nothing to do; L <= lmax: the
// few distances are computed here (one wave per row, DPP sums); otherwise the row goes to the K9r
// candidate pass (list B).
__device__ __forceinline__ float init_reach(float cost, float xn, float pn, float tau) {
  return 2.0f * sqrtf(fmaxf(cost, 0.f) + tau * (xn + pn)) * (1.0f + 2e-6f);
}

// Each block classifies a contiguous chunk of kClsRows rows (kClsPer per thread) and reserves its
// list slots with ONE atomic per list: per-wave atomics on two counters serialised at the L2 and cost
// ~30 ms for 100M rows (1.6M waves).
constexpr int kClsPer = 16;
constexpr int kClsRows = 256 * kClsPer;

__global__ __launch_bounds__(256) void init_classify_kernel(const float* __restrict__ cost,
                                                            const int* __restrict__ near, const float* __restrict__ xn,
                                                            const float* __restrict__ pn,
                                                            const float* __restrict__ tab_v, int m, float tau,
                                                            long long n, int lmax, int* __restrict__ list_a,
                                                            int* __restrict__ cnt_a, int* __restrict__ list_b,
                                                            int* __restrict__ cnt_b) {
  __shared__ int wa[4], wb[4], base[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (long long c0 = (long long)blockIdx.x * kClsRows; c0 < n; c0 += (long long)gridDim.x * kClsRows) {
    unsigned cls = 0;  // 2 bits per row: 0 skip, 1 list A, 2 list B
#pragma unroll
    for (int q = 0; q < kClsPer; ++q) {
      const long long i = c0 + (long long)q * 256 + threadIdx.x;
      unsigned k = 0;
      if (i < n) {  // the sorted row only needs two probes: L == 0 iff v[0] >= t, L <= lmax iff v[lmax] >= t
        const int p = near[i];
        const float t = init_reach(cost[i], xn[i], pn[p], tau);
        const float* v = tab_v + (long long)p * m;
        const float v0 = v[0], vl = lmax < m ? v[lmax] : __builtin_huge_valf();
        k = v0 >= t ? 0u : (vl >= t ? 1u : 2u);
      }
      cls |= k << (2 * q);
    }
    int na = 0, nb = 0;
#pragma unroll
    for (int q = 0; q < kClsPer; ++q) {
      const unsigned c = (cls >> (2 * q)) & 3u;
      na += (int)__popcll(__ballot(c == 1));
      nb += (int)__popcll(__ballot(c == 2));
    }
    if (lane == 0) {
      wa[wv] = na;
      wb[wv] = nb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int ta = wa[0] + wa[1] + wa[2] + wa[3], tb = wb[0] + wb[1] + wb[2] + wb[3];
      base[0] = ta ? atomicAdd(cnt_a, ta) : 0;
      base[1] = tb ? atomicAdd(cnt_b, tb) : 0;
    }
    __syncthreads();
    int pa = base[0], pb = base[1];
    for (int w = 0; w < wv; ++w) {
      pa += wa[w];
      pb += wb[w];
    }
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int q = 0; q < kClsPer; ++q) {
      const unsigned c = (cls >> (2 * q)) & 3u;
      const unsigned long long ba = __ballot(c == 1), bb = __ballot(c == 2);
      const long long i = c0 + (long long)q * 256 + threadIdx.x;
      if (c == 1) {  // list A entry: the row with its nearest candidate, reach and cost (int4; re-read: cache hits)
        const int p = near[i];
        const float cst = cost[i];
        reinterpret_cast<int4*>(list_a)[pa + (int)__popcll(ba & below)] =
            make_int4((int)i, p, __float_as_int(init_reach(cst, xn[i], pn[p], tau)), __float_as_int(cst));
      }
      if (c == 2) list_b[pb + (int)__popcll(bb & below)] = (int)i;
      pa += (int)__popcll(ba);
      pb += (int)__popcll(bb);
    }
    __syncthreads();  // wa/wb/base reused by the next chunk
  }
}

// List A: 16 lanes per row (NCOL = Dp/16 columns each, one 16-lane DPP row), 4 rows per wave step.
// Each lane group takes one list entry (row, nearest candidate p, reach t, cost: written by the
// classify kernel, so no per-row lookups) and keeps the nearest of its relevant new candidates (a
// prefix of p's sorted table row, at most LMAX). Lane sl of a group loads entry sl of the table row
// with the X slice; a ballot gives every group's relevant count; candidate l's index comes from lane
// g*16 + l by ds_bpermute, and the Y slices of 2 candidates are loaded together — the pass was
// latency-bound on dependent loads (list -> row state -> table -> each candidate), now a row costs
// three memory round trips for up to 2 relevant candidates. Batches of 4 held 74 VGPRs (6 waves per SIMD);
// batches of 2 hold 56 (8 waves), and the extra waves hide more than the extra round trips cost (same-box
// A/B, profiles/r5/ab_near_list: 10.67 -> 10.14 ms for the headline's two launches).
// Strict improvement over the current cost moves the row; ties among the new candidates go to the
// lowest index (K9r's argmin rule). A 16-lane sum is 4 DPP steps (no row broadcasts), and the f32
// math is on packed pairs, so a (row, candidate) pair costs ~a dozen vector instructions.
template <int NCOL, bool F8, int LMAX>
__global__ __launch_bounds__(256) void init_near_list_kernel(const void* __restrict__ X, long long ldx, int Dp,
                                                             float* __restrict__ cost, int* __restrict__ near,
                                                             const float* __restrict__ tab_v,
                                                             const int* __restrict__ tab_j, int m,
                                                             const u16* __restrict__ Y, int off,
                                                             const int4* __restrict__ list, const int* __restrict__ cnt) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int XB = F8 ? NCOL : 2 * NCOL;  // bytes of this lane's X slice
  constexpr int YQ = (2 * NCOL) / 16;       // uint4s of this lane's Y slice
  constexpr int CB = 2;                     // candidates loaded together
  static_assert(XB % 16 == 0 && (2 * NCOL) % 16 == 0, "16-B slices");
  static_assert(LMAX <= 16 && LMAX % CB == 0, "one table entry per lane of a 16-lane group");
  const unsigned char* xb = reinterpret_cast<const unsigned char*>(X);
  const int lane = threadIdx.x & 63, g = lane >> 4, sl = lane & 15;
  const long long nwaves = (long long)gridDim.x * (blockDim.x / 64);
  const long long total = *cnt;
  const int lm = LMAX < m ? LMAX : m;
  for (long long base = ((long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * 4; base < total;
       base += nwaves * 4) {
    const long long idx = base + g;
    const bool act = idx < total;
    const int4 e = list[act ? idx : base];
    const int row = e.x, p = e.y;
    const float t = __int_as_float(e.z), cr = __int_as_float(e.w);
    const bool own = sl < lm;
    const float vv = own ? tab_v[(long long)p * m + sl] : __builtin_huge_valf();
    const int jj = own ? tab_j[(long long)p * m + sl] : 0;
    f2 xf[NCOL / 2];  // this lane's columns as f32 pairs, in column order
    {
      const uint4* src =
          reinterpret_cast<const uint4*>(xb + (long long)row * ldx * (F8 ? 1 : 2) + (long long)sl * XB);
#pragma unroll
      for (int b = 0; b < XB / 16; ++b) {
        const uint4 q4 = src[b];
        const unsigned ws[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          if constexpr (F8) {
            xf[8 * b + 2 * e4] = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[e4], false);
            xf[8 * b + 2 * e4 + 1] = __builtin_amdgcn_cvt_pk_f32_fp8((int)ws[e4], true);
          } else {
            xf[4 * b + e4] = f2{__uint_as_float(ws[e4] << 16), __uint_as_float(ws[e4] & 0xffff0000u)};
          }
        }
      }
    }
    // relevant candidates of each group: a prefix of its sorted row (v ascending), so a popcount
    const unsigned long long relb = __ballot(act && vv < t);
    const int L = __popcll((relb >> (16 * g)) & 0xffffull);
    int lw = 0;  // the wave's longest list (uniform)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = __popcll((relb >> (16 * q)) & 0xffffull);
      lw = c > lw ? c : lw;
    }
    float best = cr;
    int bj = -1;
#pragma unroll 1
    for (int l0 = 0; l0 < lw; l0 += CB) {
      uint4 yq[CB][YQ];
      int jc[CB];
#pragma unroll
      for (int q = 0; q < CB; ++q) {
        jc[q] = __shfl(jj, 16 * g + l0 + q, 64);
        if (l0 + q < lw) {
          const uint4* ysrc = reinterpret_cast<const uint4*>(Y + (long long)jc[q] * Dp + (long long)sl * NCOL);
#pragma unroll
          for (int b = 0; b < YQ; ++b) yq[q][b] = ysrc[b];
        }
      }
#pragma unroll
      for (int q = 0; q < CB; ++q) {
        if (l0 + q < lw) {
          f2 acc2 = f2{0.f, 0.f};
#pragma unroll
          for (int b = 0; b < YQ; ++b) {
            const unsigned ys[4] = {yq[q][b].x, yq[q][b].y, yq[q][b].z, yq[q][b].w};
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
              const f2 dv = xf[4 * b + e4] - f2{__uint_as_float(ys[e4] << 16), __uint_as_float(ys[e4] & 0xffff0000u)};
              acc2 = dv * dv + acc2;
            }
          }
          float d = acc2.x + acc2.y;  // 16-lane sum: quad swaps, half-row mirror, row mirror
          d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0xB1, 0xf, 0xf, false));
          d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x4E, 0xf, 0xf, false));
          d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x141, 0xf, 0xf, false));
          d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x140, 0xf, 0xf, false));
          if (l0 + q < L && (d < best || (d == best && bj >= 0 && jc[q] < bj))) {
            best = d;
            bj = jc[q];
          }
        }
      }
    }
    if (act && sl == 0 && bj >= 0) {
      cost[row] = best;
      near[row] = off + bj;
    }
  }
}

// List B after a K9r candidate pass over a chunk of the new candidates (labels relative to the chunk).
__global__ __launch_bounds__(256) void init_merge_list_kernel(float* __restrict__ cost, int* __restrict__ near,
                                                              const float* __restrict__ best,
                                                              const int* __restrict__ lab, int off,
                                                              const int* __restrict__ list,
                                                              const int* __restrict__ cnt) {
  const long long total = *cnt;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int row = list[i];
    const float b = best[row];
    if (b < cost[row]) {
      cost[row] = b;
      near[row] = lab[row] + off;
    }
  }
}

// Σ over the slices overlapping segment c, in ascending slice order, of their head (A) / tail (B) partials
// for c, column d (what kmeans_segacc left in the slots for segments that cross a wave slice).
__device__ __forceinline__ double seg_fix(const int* __restrict__ seg, int k, int D, long long n, long long nwaves,
                                          const double* __restrict__ slots, const int* __restrict__ slot_c, int c,
                                          int d) {
  const long long s0 = seg[c], s1 = seg[c + 1];
  if (s1 <= s0) return 0.0;
  const long long chunk = seg_chunk(n < (long long)seg[k] ? n : (long long)seg[k], nwaves);  // as kmeans_segacc
  const long long w0 = s0 / chunk;
  long long w1 = (s1 - 1) / chunk;
  if (w1 >= nwaves) w1 = nwaves - 1;
  double t = 0.0;
  // 8 slices per round, loads issued together (a cluster can span thousands of slices); the last round is
  // predicated rather than walked one slice at a time (a segment typically spans ~8 slices: the walk paid one
  // memory round trip per slice). The sums are exact (grid integers / bf16 values in f64), so the grouping of
  // the additions does not change them.
  for (long long w = w0; w <= w1; w += 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const long long ww = w + q;
      v[q] = 0.0;
      if (ww <= w1) {
        const int ca = slot_c[2 * ww], cb = slot_c[2 * ww + 1];
        const double a = slots[(2 * ww) * (long long)D + d], b = slots[(2 * ww + 1) * (long long)D + d];
        v[q] = ca == c ? a : 0.0;
        v[q] = cb == c ? v[q] + b : v[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) t += v[q];
  }
  return t;
}

// msg[c] += seg_fix(c) for every column. One workgroup per cluster.
__global__ __launch_bounds__(256) void kmeans_seg_fixup(const int* __restrict__ seg, int k, int D, long long n,
                                                        long long nwaves, const double* __restrict__ slots,
                                                        const int* __restrict__ slot_c, double* __restrict__ msg,
                                                        const int* __restrict__ gate, int want) {
  if (gate != nullptr && gate[0] != want) return;  // step-mode gate (incremental sums)
  const int c = blockIdx.x;
  if (seg[c + 1] <= seg[c]) return;
  for (int d = threadIdx.x; d < D; d += blockDim.x) msg[(long long)c * D + d] += seg_fix(seg, k, D, n, nwaves, slots, slot_c, c, d);
}

// One workgroup per (padded) centre. Writes bf16 centre row (zero padded), ||c||² of the
// bf16-rounded centre (so scores are consistent with the GEMM operand) and, when
// `bufs` is given, first computes the new centre from nbuf all-reduced messages.
__global__ void kmeans_update_kernel(const double* __restrict__ bufs, int nbuf, long long bstride,
                                     int k, int D, double* __restrict__ cent, u16* __restrict__ cb,
                                     long long ldc, int Dp, float* __restrict__ cnorm,
                                     double* __restrict__ shift2, double unit) {
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
        nv = (s * unit) / cnt;  // unit: the sum grid step (a power of two: exact), 1 for plain sums
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

__global__ void zero_f64_gated(double* __restrict__ p, long long n, const int* __restrict__ gate, int want) {
  if (gate != nullptr && gate[0] != want) return;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = 0.0;
}

// ---------------------------------------------------------------------------------------------
// Incremental sums. Lloyd's new per-cluster sums equal the previous ones plus the rows that moved
// in minus the rows that moved out, so once labels settle (measured on the bench data: 0.03-0.4 %
// of rows change per iteration) the accumulate only has to touch the changed rows instead of
// re-reading all of X. The state `acc` = [k·D sums | k counts | cost] of the CURRENT labels lives
// across steps; the message that is all-reduced is a copy of it.
//   gate kernel : mode[0] = 1 (full accumulate into acc) if forced or more than cap rows changed,
//                 else 0; mode[1] = #changed rows; resets the change counter and the delta histogram.
//   delta path  : counting sort of the 2m entries (+row under its new label, -row under its old
//                 label, key = label or k + label) -> the same segmented f64 sums as the full path
//                 over 2k segments -> acc[c] += S[c] - S[k + c], counts likewise.
// Every value is a bf16/fp8 row summed in f64: those sums are exact while they stay inside f64's
// 53-bit window, so the incremental result equals the full recompute (and, like the full path, does
// not depend on the order rows are added in) — tests/test_kmeans_kernels_gpu.py checks it bitwise.
// ---------------------------------------------------------------------------------------------
constexpr int kDeltaThreads = 256;

__global__ __launch_bounds__(256) void kmeans_delta_gate(const int* __restrict__ wg_count, int nblk, int cap,
                                                         int* __restrict__ overflow, int* __restrict__ force,
                                                         int* __restrict__ mode, int k, int* __restrict__ dh) {
  __shared__ long long part[4];
  long long m = 0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) m += wg_count[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = part[0] + part[1] + part[2] + part[3];
    const int full = (*force != 0 || *overflow != 0 || m > (long long)cap) ? 1 : 0;
    mode[0] = full;
    mode[1] = full ? 0 : (int)m;
    *overflow = 0;
    *force = 0;
  }
  for (int i = threadIdx.x; i < 2 * k; i += blockDim.x) dh[i] = 0;
}

// One delta workgroup per assign workgroup b: its change list is rows/old[b*pcap, + wg_count[b]).
// Histogram of the 2m delta entries by key, block-aggregated in LDS. The launch also clears the delta sums
// (dsum, 2k·D doubles: the segmented pass stores or adds into them) and the per-key scatter counters — the
// separate zeroing and scan launches of each delta step are gone (kmeans_delta_scatter forms the segment
// offsets itself).
__global__ __launch_bounds__(kDeltaThreads) void kmeans_delta_hist(const int* __restrict__ rows,
                                                                   const int* __restrict__ old,
                                                                   const int* __restrict__ labels,
                                                                   const int* __restrict__ wg_count, int pcap,
                                                                   const int* __restrict__ mode, int k,
                                                                   int* __restrict__ dh, double* __restrict__ dsum,
                                                                   long long nsum, int* __restrict__ cursor) {
  if (mode[0] != 0) return;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nsum; i += (long long)gridDim.x * blockDim.x)
    dsum[i] = 0.0;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < 2 * k; i += blockDim.x) cursor[i] = 0;
  extern __shared__ int lh[];
  for (int i = threadIdx.x; i < 2 * k; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  const long long i0 = (long long)blockIdx.x * pcap, i1 = i0 + wg_count[blockIdx.x];
  for (long long i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    atomicAdd(lh + labels[rows[i]], 1);
    atomicAdd(lh + k + old[i], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * k; i += blockDim.x)
    if (lh[i]) atomicAdd(dh + i, lh[i]);
}

// perm[seg[key] + cursor[key]++] = row for both entries of every changed row (block reserves per-key ranges).
// Every workgroup forms the segment offsets seg (exclusive prefix of the 2k key counts dh) in LDS itself —
// one scan per workgroup instead of a one-workgroup scan launch between the histogram and this pass — and
// workgroup 0 publishes them for the segmented sums and the apply; cursor (zeroed by kmeans_delta_hist)
// counts each key's reserved entries.
__global__ __launch_bounds__(kDeltaThreads) void kmeans_delta_scatter(const int* __restrict__ rows,
                                                                      const int* __restrict__ old,
                                                                      const int* __restrict__ labels,
                                                                      const int* __restrict__ wg_count, int pcap,
                                                                      const int* __restrict__ mode, int k,
                                                                      int* __restrict__ cursor,
                                                                      int* __restrict__ perm,
                                                                      const int* __restrict__ dh,
                                                                      int* __restrict__ seg) {
  if (mode[0] != 0) return;
  extern __shared__ int lh[];  // [2k] counts, then bases; [2k + 1] segment offsets
  const int nk = 2 * k;
  int* segl = lh + nk;
  __shared__ int wtot[kDeltaThreads / 64];
  {
    // exclusive scan of dh: thread t owns keys [t·per, (t+1)·per), a wave scan of the thread sums, then
    // the wave totals (the same integer offsets as a serial scan)
    const int per = (nk + kDeltaThreads - 1) / kDeltaThreads, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    int sum = 0;
    for (int j = t * per; j < (t + 1) * per && j < nk; ++j) sum += dh[j];
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wtot[wv] = incl;
    for (int i = t; i < nk; i += kDeltaThreads) lh[i] = 0;
    __syncthreads();
    int acc = incl - sum;
    for (int w = 0; w < wv; ++w) acc += wtot[w];
    for (int j = t * per; j < (t + 1) * per && j < nk; ++j) {
      segl[j] = acc;
      acc += dh[j];
    }
    if (t == kDeltaThreads - 1) segl[nk] = acc;
    __syncthreads();
    if (blockIdx.x == 0)
      for (int j = t; j <= nk; j += kDeltaThreads) seg[j] = segl[j];
  }
  const long long i0 = (long long)blockIdx.x * pcap, i1 = i0 + wg_count[blockIdx.x];
  for (long long i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    atomicAdd(lh + labels[rows[i]], 1);
    atomicAdd(lh + k + old[i], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * k; i += blockDim.x) lh[i] = lh[i] ? segl[i] + atomicAdd(cursor + i, lh[i]) : 0;
  __syncthreads();
  for (long long i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int row = rows[i];
    perm[atomicAdd(lh + labels[row], 1)] = row;
    perm[atomicAdd(lh + k + old[i], 1)] = row;
  }
}

// acc[c] += S[c] - S[k+c] (sums), counts from the segment sizes, cost from the assign partials;
// on full steps only the cost. Then msg = acc (the buffer that is all-reduced).
// With slots (the delta path): the segmented pass left its cross-slice partials there instead of adding them
// into dsum (no seg_fixup launch): each element adds its two segments' partials here, the same additions.
__global__ void kmeans_delta_apply(double* __restrict__ acc, const double* __restrict__ dsum,
                                   const int* __restrict__ seg, const int* __restrict__ mode, int k, int D,
                                   const double* __restrict__ cost_part, int ncost, double* __restrict__ msg,
                                   const double* __restrict__ slots, const int* __restrict__ slot_c, long long nseg,
                                   long long nwaves) {
  const long long kd = (long long)k * D;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool delta = mode[0] == 0;
  if (idx < kd) {
    double v = acc[idx];
    if (delta) {
      double a = dsum[idx], b = dsum[kd + idx];
      if (slots != nullptr) {
        const int c = (int)(idx / D), d = (int)(idx - (long long)c * D);
        a += seg_fix(seg, 2 * k, D, nseg, nwaves, slots, slot_c, c, d);
        b += seg_fix(seg, 2 * k, D, nseg, nwaves, slots, slot_c, k + c, d);
      }
      v += a - b;
      acc[idx] = v;
    }
    msg[idx] = v;
  } else if (idx < kd + k) {
    const int c = (int)(idx - kd);
    double v = acc[idx];
    if (delta) {
      v += (double)((seg[c + 1] - seg[c]) - (seg[k + c + 1] - seg[k + c]));
      acc[idx] = v;
    }
    msg[idx] = v;
  } else if (idx == kd + k) {
    double cs = 0.0;
    for (int i = 0; i < ncost; ++i) cs += cost_part[i];
    acc[idx] = cs;
    msg[idx] = cs;
  }
}

long long assign_lds_bytes(int kc, int kp, int Dp) {
  const long long ks = Dp >= 32 ? Dp / 32 : 1;
  return (long long)(kc / 16) * ks * 1024 + (long long)kc * 4 + (long long)((kp + 3) & ~3) * 4 + 16 * 8 + 16;
}

// Assign launch shape (measured on MI355X, see profiles/): RT 16-row sub-tiles per wave share
// each centre fragment; 512 threads = two waves per SIMD. Large rows (Dp >= 256) are MFMA-heavy
// per byte: RT 4 halves the LDS fragment traffic and amortises the per-tile epilogue (no X
// double buffer fits next to it; the partner wave hides the loads). Small rows are bytes-heavy:
// RT 1 with the next tile's X in flight and more waves per CU.
// Variant (tuning/experiments): 0 auto, 1 = RT 2 + X double buffer, 2 = RT 1, 3 = RT 4.
int g_assign_variant = 0;
int g_assign_sched = 0;
// K9r (kmeans_rr.h, register-resident centres + LDS-DMA X ring) on variant 8, and by default
// (variant 0) wherever rr::plan_ct accepts the shape while this is set (CML_KMEANS_RR=0 turns it off).
// Measured (profiles/r2_assign_rr.md): 100M x 256, k = 256: 12.2 vs 13.2 ms; 10M x 128, k = 64: 0.457 vs
// 0.509 ms.
int g_rr_default = 1;
int g_rr_dbg = 0;  // K9r ablation bits (kmeans_rr.h), 0 in production  // kmeans_assign_bf16 `sched` (partner-wave desynchronisation), tuning knob
inline int assign_threads(int /*DS*/) {
  return g_assign_variant == 4 ? 768 : (g_assign_variant == 5 ? 1024 : 512);
}

template <int DP, bool F8>
const void* assign_kernel_ptr() {
  constexpr bool PF = AssignShape<DP>::KS <= 8;
  constexpr int RT_BIG = DP >= 512 ? 2 : 4;
  switch (g_assign_variant) {
    case 1: return (const void*)kmeans_assign_bf16<DP, 2, 512, PF, 4, F8>;
    case 2: return (const void*)kmeans_assign_bf16<DP, 1, 512, PF, 4, F8>;
    case 3: return (const void*)kmeans_assign_bf16<DP, RT_BIG, 512, false, 2, F8>;
    case 4: return (const void*)kmeans_assign_bf16<DP, 2, 768, false, 4, F8>;
    case 5: return (const void*)kmeans_assign_bf16<DP, 1, 1024, PF, 4, F8>;
    case 6:  // the default launch with per-sub-tile accumulator seeding (A/B reference of SHARED)
      if constexpr (DP >= 256)
        return (const void*)kmeans_assign_bf16<DP, RT_BIG, 512, false, DP >= 512 ? 4 : 2, F8, false>;
      else
        return (const void*)kmeans_assign_bf16<DP, 1, 512, PF, 4, F8, false>;
    case 7:  // the default launch with the PACK4 per-row key (4 slots merged by v_min3)
      if constexpr (DP >= 256)
        return (const void*)kmeans_assign_bf16<DP, RT_BIG, 512, false, DP >= 512 ? 4 : 2, F8, true, true>;
      else
        return (const void*)kmeans_assign_bf16<DP, 1, 512, PF, 4, F8, true, true>;
    default:
      if constexpr (DP >= 256) return (const void*)kmeans_assign_bf16<DP, RT_BIG, 512, false, DP >= 512 ? 4 : 2, F8>;
      else return (const void*)kmeans_assign_bf16<DP, 1, 512, PF, 4, F8>;
  }
}

// Rows per wave tile of the launch assign_kernel_ptr<DP> selects (the sort regime's scatter
// recovers a row's workgroup from it).
inline int assign_tile_rows(int Dp) {
  switch (g_assign_variant) {
    case 1: return 32;
    case 2: return 16;
    case 3: return Dp >= 512 ? 32 : 64;
    case 4: return 32;
    case 5: return 16;
    case 6: return Dp >= 512 ? 32 : (Dp >= 256 ? 64 : 16);
    case 7: return Dp >= 512 ? 32 : (Dp >= 256 ? 64 : 16);
    default: return Dp >= 512 ? 32 : (Dp >= 256 ? 64 : 16);
  }
}

template <int DP, bool F8>
int assign_occupancy(int kc, int kp) {
  const size_t lds = (size_t)assign_lds_bytes(kc, kp, DP);
  const void* fn = assign_kernel_ptr<DP, F8>();
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int nb = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, assign_threads(0), lds);
  return nb;
}

template <int DP, bool F8>
int launch_assign(const void* X, long long n, long long ldx, const u16* C, long long ldc, int kc, int kp,
                  int c_base, const float* cnorm, const float* xnorm, int* labels, float* best, int first, int last,
                  double* cost_part, int* hist, int* rank, DeltaOut dout, int grid, hipStream_t st) {
  const size_t lds = (size_t)assign_lds_bytes(kc, kp, DP);
  const void* fn = assign_kernel_ptr<DP, F8>();
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  void* args[] = {(void*)&X, (void*)&n, (void*)&ldx, (void*)&C, (void*)&ldc, (void*)&kc, (void*)&kp,
                  (void*)&c_base, (void*)&cnorm, (void*)&xnorm, (void*)&labels, (void*)&best, (void*)&first,
                  (void*)&last, (void*)&cost_part, (void*)&hist, (void*)&rank, (void*)&dout,
                  (void*)&g_assign_sched};
  const hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(assign_threads(0)), args, lds, st);
  if (e != hipSuccess) return (int)e;
  return cml_status();
}

long long priv_lds_bytes(int k, int dw, int rpw) {
  const long long NW = kAccumThreads / 64;
  return NW * rpw * k * dw * 4 + NW * rpw * k * 4;
}

template <int CPL, int RPW>
int launch_priv(const u16* X, long long n, long long ldx, const int* labels, int k, int dw, float* slab, int* cslab,
                int gx, int nsl, hipStream_t st) {
  const size_t lds = (size_t)priv_lds_bytes(k, dw, RPW);
  hipFuncSetAttribute((const void*)kmeans_accum_priv<CPL, RPW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((kmeans_accum_priv<CPL, RPW>), dim3(gx, nsl), dim3(kAccumThreads), lds, st, X, n, ldx, labels, k,
                     dw, slab, cslab);
  return cml_status();
}

// Segmented f64 sums over a sorted position list (kmeans_segacc + kmeans_seg_fixup); n is an upper
// bound of the filled positions (the kernels clamp to seg[k]).
int launch_segsum(const void* X, long long n, long long ldx, int Dp, int D, const int* perm, const int* seg, int k,
                  int cpl, int seg_grid, double* msg, double* slots, int* slot_c, int xfp8, const int* gate, int want,
                  hipStream_t st, SegUB sub = SegUB{nullptr, 0, nullptr, 0.0}, bool fixup = true) {
  const long long waves = (long long)seg_grid * (kSegThreads / 64);
#define CML_SEG_L(C, F, U, Q)                                                                                       \
  hipLaunchKernelGGL((kmeans_segacc<C, F, U, Q>), dim3(seg_grid), dim3(kSegThreads), 0, st, X, n, ldx, Dp, D, perm, \
                     seg, k, msg, slots, slot_c, gate, want, sub)
#define CML_SEG(C, F)                                                  \
  if (sub.ub != nullptr) {                                             \
    if (!F && sub.qs != 0.0) CML_SEG_L(C, F, true, !F);               \
    else CML_SEG_L(C, F, true, false);                                 \
  } else {                                                             \
    if (!F && sub.qs != 0.0) CML_SEG_L(C, F, false, !F);              \
    else CML_SEG_L(C, F, false, false);                                \
  }
  if (xfp8) {
    if (cpl == 4) CML_SEG(4, true)
    else if (cpl == 8) CML_SEG(8, true)
    else if (cpl == 16) CML_SEG(16, true)
    else return (int)hipErrorInvalidValue;
  } else if (cpl == 2) CML_SEG(2, false)
  else if (cpl == 4) CML_SEG(4, false)
  else if (cpl == 8) CML_SEG(8, false)
  else return (int)hipErrorInvalidValue;
#undef CML_SEG
#undef CML_SEG_L
  const int e = cml_status();
  if (e || !fixup) return e;
  hipLaunchKernelGGL(kmeans_seg_fixup, dim3(k), dim3(256), 0, st, seg, k, D, n, waves, slots, slot_c, msg, gate,
                     want);
  return cml_status();
}

}  // namespace

CML_API long long cml_kmeans_assign_lds_bytes(int kc, int kp, int Dp) { return assign_lds_bytes(kc, kp, Dp); }
CML_API int cml_kmeans_assign_threads(int Dp) { return assign_threads(Dp / 16); }
// Resident workgroups per CU of the assign kernel for this shape (persistent-grid sizing).
CML_API int cml_kmeans_assign_occupancy(int Dp, int kc, int kp, int xfp8) {
  if (xfp8) {
    switch (Dp) {
      case 64: return assign_occupancy<64, true>(kc, kp);
      case 128: return assign_occupancy<128, true>(kc, kp);
      case 256: return assign_occupancy<256, true>(kc, kp);
      case 512: return assign_occupancy<512, true>(kc, kp);
      default: return 0;
    }
  }
  switch (Dp / 16) {
    case 1: return assign_occupancy<16, false>(kc, kp);
    case 2: return assign_occupancy<32, false>(kc, kp);
    case 4: return assign_occupancy<64, false>(kc, kp);
    case 8: return assign_occupancy<128, false>(kc, kp);
    case 16: return assign_occupancy<256, false>(kc, kp);
    case 32: return assign_occupancy<512, false>(kc, kp);
    default: return 0;
  }
}
CML_API int cml_kmeans_set_assign_sched(int v) {
  if (v < 0) return (int)hipErrorInvalidValue;
  g_assign_sched = v;
  return 0;
}
// K9r plan for (Dp, kc): returns the centre tiles per compute wave (0: K9r not used — variant, fp8 rows
// or shape), out[0] = LDS bytes, out[1] = rows per tile (= rows per workgroup round), out[2] = threads.
CML_API int cml_kmeans_assign_rr_plan(int Dp, int kc, int kp, int xfp8, long long* out) {
  if (kc != kp) return 0;
  if (!(g_assign_variant == 8 || (g_assign_variant == 0 && g_rr_default))) return 0;
  const int ct = rr::plan_ct(Dp, kc, xfp8 != 0);
  if (ct == 0) return 0;
  const long long lds = rr::lds_for(Dp, kp, xfp8 != 0);
  if (lds <= 0 || lds > 160 * 1024) return 0;
  out[0] = lds;
  out[1] = rr::tile_rows(Dp, xfp8 != 0);
  out[2] = rr::kThreads;
  return ct;
}
CML_API int cml_kmeans_set_rr_debug(int bits) {
  g_rr_dbg = bits;
  return 0;
}
CML_API int cml_kmeans_set_rr_m32(int on) {
  rr::g_m32 = on ? 1 : 0;
  return 0;
}
// MX arithmetic of the fp8 K9r passes (kmeans_rr.h compute_mx): on by default; returns the previous setting.
CML_API int cml_kmeans_set_fp8_mx(int on) {
  const int prev = rr::g_mx;
  if (on >= 0) rr::g_mx = on ? 1 : 0;
  return prev;
}
CML_API int cml_kmeans_set_rr_default(int on) {
  g_rr_default = on ? 1 : 0;
  return 0;
}
// Rows per wave tile of the K9 launch the current variant selects (sort-regime scatter geometry).
CML_API int cml_kmeans_assign_tile_rows(int Dp) { return assign_tile_rows(Dp); }
CML_API int cml_kmeans_set_assign_variant(int v) {
  if (v < 0 || v > 8) return (int)hipErrorInvalidValue;
  g_assign_variant = v;
  return 0;
}
CML_API int cml_kmeans_accum_threads() { return kAccumThreads; }
CML_API int cml_kmeans_seg_threads() { return kSegThreads; }
CML_API long long cml_kmeans_seg_ints(int k) { return (long long)(k + 1) + ((k + 1) & 1) + 2LL * k + 2; }

// X: bf16 [n, ldx] (Dp = 16*DS used columns, zero padded), or with xfp8 OCP e4m3fn bytes [n, ldx]
// (Dp in {64,...,512}, ldx bytes, 16-B aligned rows). C: bf16 [kc, ldc] (kc % 16 == 0).
// hist/rank may be null; when given (last chunk only) hist is [grid][kp] and rank is [n].
// xnorm (f32 [n], cml_row_sqnorm_*) is required: it seeds the MFMA accumulators.
// best may be null on a single-chunk (first && last) launch: only labels/cost are produced.
CML_API int cml_kmeans_assign_bf16(const void* X, long long n, long long ldx, int Dp, const void* C, long long ldc,
                                   int kc, int kp, int c_base, const float* cnorm, const float* xnorm, int* labels,
                                   float* best, int first, int last, double* cost_part, int* hist, int* rank,
                                   int grid, int xfp8, int* chg_rows, int* chg_old, int* chg_wg_count,
                                   int* chg_overflow, int chg_pcap, int rr_ct,
                                   void* stream) {
  if (kc % 16 != 0 || Dp % 16 != 0 || ldc % 8 != 0) return (int)hipErrorInvalidValue;
  if (chg_rows != nullptr && (!(first && last) || chg_old == nullptr || chg_wg_count == nullptr ||
                              chg_overflow == nullptr || chg_pcap < 0 || hist == nullptr || cost_part == nullptr))
    return (int)hipErrorInvalidValue;  // label changes: single-launch assign with the ranking epilogue
  const DeltaOut dout{chg_rows, chg_old, chg_wg_count, chg_overflow, chg_pcap, nullptr};
  if (xfp8 ? (ldx % 16 != 0) : (ldx % 8 != 0)) return (int)hipErrorInvalidValue;
  if ((hist == nullptr) != (rank == nullptr)) return (int)hipErrorInvalidValue;
  if (best == nullptr && !(first && last)) return (int)hipErrorInvalidValue;
  if (xnorm == nullptr) return (int)hipErrorInvalidValue;  // ||x||² seeds the accumulators
  hipStream_t st = (hipStream_t)stream;
  const u16* c = (const u16*)C;
  if (rr_ct > 0) {  // K9r: single launch over every centre
    if (!(first && last) || kc != kp || rr::plan_ct(Dp, kc, xfp8 != 0) != rr_ct) return (int)hipErrorInvalidValue;
    return rr::dispatch(0, Dp, rr_ct, xfp8 != 0, X, n, ldx, c, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part,
                        hist, rank, dout, rr::Ext{}, grid, g_rr_dbg, st);
  }
  if (xfp8) {
    switch (Dp) {
#define CML_ASSIGN8(DP)                                                                                          \
  case DP:                                                                                                       \
    return launch_assign<DP, true>(X, n, ldx, c, ldc, kc, kp, c_base, cnorm, xnorm, labels, best, first, last,  \
                                   cost_part, hist, rank, dout, grid, st)
      CML_ASSIGN8(64); CML_ASSIGN8(128); CML_ASSIGN8(256); CML_ASSIGN8(512);
#undef CML_ASSIGN8
      default: return (int)hipErrorInvalidValue;
    }
  }
#define CML_ASSIGN(DS, DP)                                                                                       \
  case DS:                                                                                                       \
    return launch_assign<DP, false>(X, n, ldx, c, ldc, kc, kp, c_base, cnorm, xnorm, labels, best, first, last, \
                                    cost_part, hist, rank, dout, grid, st)
  switch (Dp / 16) {
    CML_ASSIGN(1, 16); CML_ASSIGN(2, 32); CML_ASSIGN(4, 64); CML_ASSIGN(8, 128); CML_ASSIGN(16, 256);
    CML_ASSIGN(32, 512);
    default: return (int)hipErrorInvalidValue;
  }
#undef CML_ASSIGN
}

// K9r with the pruned-step extensions (kmeans_rr.h modes): mode 1 = every row + top-2 bounds
// (ub/lb), mode 2 = the positions of a candidate list (idx, compacted xn/lab, count on the device)
// + top-2 bounds. gate/want: the launch returns at once unless *gate == want (null: always runs).
// hist/rank (counting-sort ranks) and the change log as for cml_kmeans_assign_bf16; mode 2 takes no
// hist/rank. n is the row count (mode 1) or the capacity the grid is sized for (mode 2).
CML_API int cml_kmeans_assign_rr_ext(int mode, const void* X, long long n, long long ldx, int Dp, const void* C,
                                     long long ldc, int kc, int kp, const float* cnorm, const float* xnorm,
                                     int* labels, double* cost_part, int* hist, int* rank, int grid, int xfp8,
                                     int* chg_rows, int* chg_old, int* chg_wg_count, int* chg_overflow, int chg_pcap,
                                     int rr_ct, const int* idx, const int* n_dev, const int* lab_in, float* ub,
                                     float* lb, const float* mc, float tau, const int* gate, int want, float* best,
                                     const float* cum, int k_cum, float* mcost, int* mnear, int moff,
                                     void* stream) {
  if (mode < 1 || mode > 2 || kc != kp || kc % 16 != 0 || ldc % 8 != 0) return (int)hipErrorInvalidValue;
  if ((mcost == nullptr) != (mnear == nullptr) || (mcost != nullptr && mode != 2)) return (int)hipErrorInvalidValue;
  if (xfp8 ? (ldx % 16 != 0) : (ldx % 8 != 0)) return (int)hipErrorInvalidValue;
  if (rr_ct <= 0 || rr::plan_ct(Dp, kc, xfp8 != 0) != rr_ct) return (int)hipErrorInvalidValue;
  if (xnorm == nullptr || ub == nullptr || lb == nullptr || mc == nullptr) return (int)hipErrorInvalidValue;
  if ((hist == nullptr) != (rank == nullptr)) return (int)hipErrorInvalidValue;
  if (mode == 2 && (idx == nullptr || n_dev == nullptr || lab_in == nullptr || hist != nullptr))
    return (int)hipErrorInvalidValue;
  if (chg_rows != nullptr && (chg_old == nullptr || chg_wg_count == nullptr || chg_overflow == nullptr || chg_pcap < 0))
    return (int)hipErrorInvalidValue;
  const long long lds = rr::lds_for(Dp, kp, xfp8 != 0, mode);
  if (lds <= 0 || lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const DeltaOut dout{chg_rows, chg_old, chg_wg_count, chg_overflow, chg_pcap, nullptr};
  const rr::Ext ext{idx,  n_dev, lab_in, ub,    lb,    mc,   tau, gate, want, cum, cum != nullptr ? cum + k_cum : nullptr,
                    mcost, mnear, moff};
  return rr::dispatch(mode, Dp, rr_ct, xfp8 != 0, X, n, ldx, (const u16*)C, ldc, kc, kp, cnorm, xnorm, labels,
                      best, cost_part, hist, rank, dout, ext, grid, g_rr_dbg, (hipStream_t)stream);
}

// ||x||² of the device matrix: the row pass of kmeans_init.hip (norms only), the one definition of
// the cached norms.
extern "C" int cml_kmeans_row_pass(const void* X, long long n, long long ldx, int Dp, int xfp8, float* xn,
                                   const float* c0, float c0n, float* cost, int* near, unsigned* xn_max,
                                   int* erange, double* xn64, const float* c0n_dev, void* stream);

CML_API int cml_row_sqnorm_fp8(const void* X, long long n, long long ldx, int Dp, float* out, void* stream) {
  return cml_kmeans_row_pass(X, n, ldx, Dp, 1, out, nullptr, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr, stream);
}

CML_API int cml_row_sqnorm_bf16(const void* X, long long n, long long ldx, int Dp, float* out, void* stream) {
  return cml_kmeans_row_pass(X, n, ldx, Dp, 0, out, nullptr, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr, stream);
}

// Regime A. rpw rows per wave-instruction, private copies; dw <= cpl*64/rpw.
CML_API long long cml_kmeans_priv_lds_bytes(int k, int dw, int rpw) { return priv_lds_bytes(k, dw, rpw); }

// Slab layout: slab[nsl][gx][k][dw] f32, cslab[gx][k] int32; nsl*dw >= Dp.
CML_API int cml_kmeans_accum_priv(const void* X, long long n, long long ldx, const int* labels, int k, int dw, int cpl,
                                  int rpw, float* slab, int* cslab, int gx, int nsl, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  if ((cpl != 2 && cpl != 4) || rpw < 1 || dw % cpl != 0 || dw > cpl * 64 / rpw) return (int)hipErrorInvalidValue;
#define CML_PRIV(C, R) if (cpl == C && rpw == R) return launch_priv<C, R>(x, n, ldx, labels, k, dw, slab, cslab, gx, nsl, st)
  CML_PRIV(2, 1); CML_PRIV(2, 2); CML_PRIV(2, 4); CML_PRIV(2, 8); CML_PRIV(2, 16);
  CML_PRIV(4, 1); CML_PRIV(4, 2); CML_PRIV(4, 4); CML_PRIV(4, 8); CML_PRIV(4, 16);
#undef CML_PRIV
  return (int)hipErrorInvalidValue;
}

CML_API int cml_kmeans_reduce(const float* slab, const int* cslab, const double* cost_part, int gx, int ncost, int k,
                              int D, int dsl, double* out, void* stream) {
  const long long total = (long long)k * D + k + 1;
  const int threads = 256;
  const long long blocks = (total + threads - 1) / threads;
  hipLaunchKernelGGL(kmeans_reduce_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, slab, cslab,
                     cost_part, gx, ncost, k, D, dsl, out);
  return cml_status();
}

// Regime B: scan + scatter + segmented accumulate. `nblk`/`round_rows` describe the assign launch
// that produced hist/rank (workgroup b ranked rows [b·round_rows + i·nblk·round_rows, +round_rows)). msg = [k*D sums | k counts | cost]. `seg` must hold k+1 ints plus
// 2k+2 ints of scratch (cml_kmeans_seg_ints).
static int sort_accum(const void* X, long long n, long long ldx, int Dp, int D, const int* labels, const int* rank,
                      const int* hist, int nblk, int round_rows, int k, int kp, const double* cost_part, int ncost,
                      int* off, int* seg, int* perm, int cpl, int seg_grid, double* msg, double* slots, int* slot_c,
                      int xfp8, const int* gate, void* stream, SegUB sub);
// qscale: the sum grid (0 = plain f64 sums); see add_raw_q.
CML_API int cml_kmeans_sort_accum(const void* X, long long n, long long ldx, int Dp, int D, const int* labels,
                                  const int* rank, const int* hist, int nblk, int round_rows, int k, int kp,
                                  const double* cost_part, int ncost, int* off, int* seg, int* perm, int cpl,
                                  int seg_grid, double* msg, double* slots, int* slot_c, int xfp8, const int* gate,
                                  double qscale, void* stream) {
  return sort_accum(X, n, ldx, Dp, D, labels, rank, hist, nblk, round_rows, k, kp, cost_part, ncost, off, seg, perm,
                    cpl, seg_grid, msg, slots, slot_c, xfp8, gate, stream, SegUB{nullptr, 0, nullptr, qscale});
}
// The same, also writing ub[row] >= |x_row - cb[label]| (bf16 centres, row stride ldc) for every row.
CML_API int cml_kmeans_sort_accum_ub(const void* X, long long n, long long ldx, int Dp, int D, const int* labels,
                                     const int* rank, const int* hist, int nblk, int round_rows, int k, int kp,
                                     const double* cost_part, int ncost, int* off, int* seg, int* perm, int cpl,
                                     int seg_grid, double* msg, double* slots, int* slot_c, int xfp8, const int* gate,
                                     const void* cb, long long ldc, float* ub, double qscale, const float* cu,
                                     void* stream) {
  if (cb == nullptr || ub == nullptr || ldc < Dp) return (int)hipErrorInvalidValue;
  return sort_accum(X, n, ldx, Dp, D, labels, rank, hist, nblk, round_rows, k, kp, cost_part, ncost, off, seg, perm,
                    cpl, seg_grid, msg, slots, slot_c, xfp8, gate, stream, SegUB{(const u16*)cb, ldc, ub, qscale, cu});
}
static int sort_accum(const void* X, long long n, long long ldx, int Dp, int D, const int* labels, const int* rank,
                      const int* hist, int nblk, int round_rows, int k, int kp, const double* cost_part, int ncost,
                      int* off, int* seg, int* perm, int cpl, int seg_grid, double* msg, double* slots, int* slot_c,
                      int xfp8, const int* gate, void* stream, SegUB sub) {
  hipStream_t st = (hipStream_t)stream;
  long long* tot = reinterpret_cast<long long*>(seg + k + 1 + ((k + 1) & 1));  // scratch after seg (8-B aligned)
  const int want = 1;  // gated launches run on full-accumulate steps only
  if (gate == nullptr) {
    hipMemsetAsync(msg, 0, sizeof(double) * (size_t)k * D, st);
  } else {
    hipLaunchKernelGGL(zero_f64_gated, dim3(256), dim3(256), 0, st, msg, (long long)k * D, gate, want);
  }
  hipLaunchKernelGGL(kmeans_seg_totals, dim3(k), dim3(256), 0, st, hist, nblk, kp, tot, gate, want);
  hipLaunchKernelGGL(kmeans_seg_offsets, dim3(k), dim3(256), 0, st, hist, nblk, k, kp, tot, cost_part, ncost, D, off,
                     seg, msg, gate, want);
  int e = cml_status();
  if (e) return e;
  if (n == 0) return 0;
  hipLaunchKernelGGL(kmeans_scatter, dim3(nblk), dim3(kScatterThreads), sizeof(int) * (size_t)k, st,
                     labels, rank, n,
                     nblk, 1, round_rows, k, off, perm, gate, want);
  e = cml_status();
  if (e) return e;
  return launch_segsum(X, n, ldx, Dp, D, perm, seg, k, cpl, seg_grid, msg, slots, slot_c, xfp8, gate, want, st, sub);
}

// ---- incremental sums (see kmeans_delta_gate). Per step, after the single-launch assign that
// logged label changes: cml_kmeans_delta_gate, then cml_kmeans_sort_accum(gate = mode, msg = acc),
// then cml_kmeans_delta_accum (which also publishes msg = acc).
CML_API int cml_kmeans_delta_gate(const int* chg_wg_count, int nblk, int cap, int* chg_overflow, int* force, int* mode,
                                  int k, int* dh, void* stream) {
  hipLaunchKernelGGL(kmeans_delta_gate, dim3(1), dim3(256), 0, (hipStream_t)stream, chg_wg_count, nblk, cap,
                     chg_overflow, force, mode, k, dh);
  return cml_status();
}

int g_delta_fused_fixup = 1;  // cml_kmeans_set_delta_fused_fixup (A/B knob)
CML_API int cml_kmeans_set_delta_fused_fixup(int on) {
  const int prev = g_delta_fused_fixup;
  if (on >= 0) g_delta_fused_fixup = on;
  return prev;
}

// dseg: 2k+1 ints, cursor: 2k ints, dperm: 2*cap ints, dsum: 2k*D doubles; slots/slot_c sized for
// seg_grid (cml_kmeans_seg_slot_*); acc/msg: k*D + k + 1 doubles.
CML_API int cml_kmeans_delta_accum(const void* X, long long ldx, int Dp, int D, const int* labels, const int* chg_rows,
                                   const int* chg_old, const int* chg_wg_count, int nblk, int pcap, int cap,
                                   const int* mode, int k, int* dh, int* dseg,
                                   int* cursor, int* dperm, int cpl, int seg_grid, double* dsum, double* slots,
                                   int* slot_c, double* acc, const double* cost_part, int ncost, double* msg, int xfp8,
                                   double qscale, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t lh = sizeof(int) * 2 * (size_t)k;
  hipLaunchKernelGGL(kmeans_delta_hist, dim3(nblk), dim3(kDeltaThreads), lh, st, chg_rows, chg_old, labels,
                     chg_wg_count, pcap, mode, k, dh, dsum, 2LL * k * D, cursor);
  hipLaunchKernelGGL(kmeans_delta_scatter, dim3(nblk), dim3(kDeltaThreads), lh + sizeof(int) * (2 * (size_t)k + 1), st,
                     chg_rows, chg_old, labels, chg_wg_count, pcap, mode, k, cursor, dperm, dh, dseg);
  int e = cml_status();
  if (e) return e;
  // the cross-slice partials: added by the apply (per element, seg_fix) instead of a fixup launch (one
  // workgroup per key); CML_DELTA_FUSED_FIXUP=0 keeps the launch (A/B: profiles/r5/README.md)
  const bool fused = g_delta_fused_fixup != 0;
  if (cap > 0) {
    e = launch_segsum(X, 2LL * cap, ldx, Dp, D, dperm, dseg, 2 * k, cpl, seg_grid, dsum, slots, slot_c, xfp8, mode, 0,
                      st, SegUB{nullptr, 0, nullptr, qscale}, !fused);
    if (e) return e;
  }
  const long long total = (long long)k * D + k + 1;
  const long long waves = (long long)seg_grid * (kSegThreads / 64);
  hipLaunchKernelGGL(kmeans_delta_apply, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, acc, dsum, dseg,
                     mode, k, D, cost_part, ncost, msg, (cap > 0 && fused) ? slots : nullptr, slot_c, 2LL * cap, waves);
  return cml_status();
}

// Doubles / ints of the deterministic slot scratch for a sort-regime launch of seg_grid blocks.
CML_API long long cml_kmeans_seg_slot_doubles(int seg_grid, int D) {
  return 2LL * seg_grid * (kSegThreads / 64) * D;
}
CML_API long long cml_kmeans_seg_slot_ints(int seg_grid) { return 2LL * seg_grid * (kSegThreads / 64); }

CML_API int cml_kmeans_update(const double* bufs, int nbuf, long long bstride, int k, int D, double* cent, void* cb,
                              long long ldc, int Dp, int Kp, float* cnorm, double* shift2, double unit,
                              void* stream) {
  hipLaunchKernelGGL(kmeans_update_kernel, dim3(Kp), dim3(256), 0, (hipStream_t)stream, bufs, nbuf, bstride, k, D,
                     cent, (u16*)cb, ldc, Dp, cnorm, shift2, unit);
  return cml_status();
}

// Pruned k-means|| candidate pass: classification (list A / list B, counters zeroed by the caller).
CML_API int cml_kmeans_init_classify(const float* cost, const int* near, const float* xn, const float* pn,
                                     const float* tab_v, int m, float tau, long long n, int lmax, int* list_a,
                                     int* cnt_a, int* list_b, int* cnt_b, void* stream) {
  if (n <= 0) return 0;
  if (m <= 0) return (int)hipErrorInvalidValue;
  const long long blocks = std::min<long long>((n + kClsRows - 1) / kClsRows, 4096);
  hipLaunchKernelGGL(init_classify_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, cost, near, xn,
                     pn, tab_v, m, tau, n, lmax, list_a, cnt_a, list_b, cnt_b);
  return cml_status();
}

// List A distances. X: bf16 rows (ldx elements) or e4m3 bytes (ldx bytes); Y: bf16 [m, Dp] new
// candidates; list: the classify kernel's int4 entries (xn, pn and tau are folded into them and are
// not read); n_cap: an upper bound of *cnt (sizes the grid).
constexpr int kInitLmax = 8;  // models/kmeans.py _INIT_LMAX
CML_API int cml_kmeans_init_lmax() { return kInitLmax; }
CML_API int cml_kmeans_init_near_list(const void* X, long long ldx, int Dp, int xfp8, float* cost, int* near,
                                      const float* xn, const float* pn, const float* tab_v, const int* tab_j, int m,
                                      const void* Y, int off, float tau, const int* list, const int* cnt,
                                      long long n_cap, void* stream) {
  if (n_cap <= 0) return 0;
  const int ncol = Dp / 16;
  const long long blocks = std::max<long long>(1, std::min<long long>((n_cap + 15) / 16, 8192));
  hipStream_t st = (hipStream_t)stream;
#define CML_NL(C, F)                                                                                                \
  hipLaunchKernelGGL((init_near_list_kernel<C, F, kInitLmax>), dim3((unsigned)blocks), dim3(256), 0, st, X, ldx, Dp, \
                     cost, near, tab_v, tab_j, m, (const u16*)Y, off, reinterpret_cast<const int4*>(list), cnt)
  if (xfp8) {
    if (ncol == 16) CML_NL(16, true);
    else if (ncol == 32) CML_NL(32, true);
    else return (int)hipErrorInvalidValue;
  } else if (ncol == 8) CML_NL(8, false);
  else if (ncol == 16) CML_NL(16, false);
  else if (ncol == 32) CML_NL(32, false);
  else return (int)hipErrorInvalidValue;
#undef CML_NL
  return cml_status();
}

CML_API int cml_kmeans_init_merge_list(float* cost, int* near, const float* best, const int* lab, int off,
                                       const int* list, const int* cnt, long long n_cap, void* stream) {
  if (n_cap <= 0) return 0;
  const long long blocks = std::max<long long>(1, std::min<long long>((n_cap + 255) / 256, 4096));
  hipLaunchKernelGGL(init_merge_list_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, cost, near,
                     best, lab, off, list, cnt);
  return cml_status();
}
