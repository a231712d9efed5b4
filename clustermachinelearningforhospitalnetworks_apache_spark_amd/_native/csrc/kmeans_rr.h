// K9r — KMeans assign with REGISTER-resident centres and an LDS-DMA ring of X tiles (gfx950).
//
// Included by kmeans.hip (uses its DeltaOut). Why a second assign design: K9 (kmeans_assign_bf16)
// keeps the centres in LDS and streams X into VGPRs, so every wave must hold a whole 64-row X tile
// (128 VGPRs) and cannot double-buffer it: X loads stall the wave, and the pass ends up neither at
// the HBM roofline (5.3 TB/s alone) nor at the MFMA one (1.3 PF/s alone) — 13.2 ms for 100M x 256,
// k = 256 against ~9.5 ms for either bound. Here the roles swap:
//
//   * the k centres are split over the 4 COMPUTE waves (one per SIMD): wave w keeps centres
//     [w·kc/4, (w+1)·kc/4) as MFMA A fragments in VGPRs for the whole launch (k = 256, D = 256:
//     64 centres x 256 x bf16 = 128 VGPRs per lane), pre-scaled by -2;
//   * X streams through an NS-slot LDS ring of 32-KiB tiles filled by LDS-DMA
//     (global_load_lds_dwordx4) issued by 2 DMA waves that do nothing else, so the loads never stall
//     a computing wave and ~96 KiB per CU stay in flight;
//   * every compute wave reads each X tile from LDS (B operand of v_mfma_f32_16x16x32_bf16, one
//     ds_read_b128 per 16 rows x 32 k) against its own centres; its per-row minimum key over its
//     centres goes to an exchange buffer;
//   * 2 FINALIZE waves take the minimum over the 4 compute waves one tile later and run the
//     epilogue K9 runs inline (labels, cost, label-change lists, counting-sort ranks).
//
// Modes (template MODE):
//   0  the plain assign above;
//   1  + TOP-2: compute waves keep the two smallest keys per row, the finalize waves merge them and
//        write the exact-pruning bounds of every row (models/kmeans.py pruned step):
//        ub = sqrt(best + tau·(|x|²+max|c|²)) rounded up, lb = sqrt(second - tau·(...)) rounded down.
//        The second-best distance is what the Hamerly lower bound needs, so a full step leaves valid
//        bounds behind with no extra pass (it replaced a [n, k] GEMM + row-min over every row);
//   2  TOP-2 over a CANDIDATE list: position p of the launch is row idx[p]; the position count is
//        read on the device (*n_dev), so the pruned step needs no host synchronisation. X rows are
//        fetched through the index (the DMA waves read each tile's indices with scalar loads, which
//        do not count against the vmcnt that paces the LDS-DMA ring); norms/labels/indices of the
//        positions are compacted arrays (written by the bounds pass) that ride the trailer ring.
//        Outputs (labels, bounds, change log) go to the real rows.
// Any mode can be gated by a device flag (*gate == want, else every workgroup returns at once), so
// a step can enqueue both the full and the candidate launch and let the device pick one.
//
// Tile rows are stored in LDS row-major with the 16-byte chunks of row R permuted (chunk c at
// position c ^ (R & 15)): one DMA instruction then reads 1 KiB of whole rows from HBM (2 rows of
// 512 B at D = 256: full-line reads), and the B-fragment reads — 16 rows at the same chunk — hit 16
// distinct bank slots (conflict-free ds_read_b128; the permutation is applied to the DMA SOURCE
// address, the LDS destination of an LDS-DMA being lane-linear).
//
// Synchronisation: one workgroup barrier per tile. Tile j is computed from slot j % NS while the DMA
// waves keep tiles j+1 .. j+NS-1 in flight (counted vmcnt, never 0 in steady state) and the
// finalize waves finish tile j-1. A slot is refilled only after the barrier that ends the tile
// reading it; keys are double-buffered; norms/labels of a tile ride in a trailer ring of NS+1
// entries, so the finalize waves can read tile j-1's trailer while tile j+NS-1's lands.
// Every wave executes the same number of barriers (prologue, one per tile, epilogue) whatever its
// role or tile count, and the loop bound is the block's tile count, so the grid always drains.
//
// Precision: accumulators start at ||c||² + ||x||² (this lane's own row), so they end as the exact
// f32 squared distance; the key truncates log2(CT)+2 low mantissa bits for the (tile, slot) tag
// (2^-19 relative at k = 256), ties resolve to the lowest centre index.
#pragma once

namespace rr {

constexpr int kThreads = 512;   // waves 0-3 compute, 4-5 LDS-DMA, 6-7 finalize
constexpr int kCompute = 4;

// Extra inputs/outputs of modes 1 and 2 and of the device gate.
struct Ext {
  const int* idx;     // MODE 2: real row of every position (compacted, >= roundup(n, TR) readable entries)
  const int* n_dev;   // MODE 2: number of positions
  const int* lab_in;  // MODE 2: labels of the positions (compacted)
  float* ub;          // MODE >= 1: upper bound of |x - c_label| per row
  float* lb;          // MODE >= 1: lower bound of the distance to every other centre per row
  const float* mc;    // MODE >= 1: max ||c||² (device scalar)
  float tau;          // MODE >= 1: error allowance relative to ||x||² + max||c||²
  const int* gate;    // launch runs only when gate == nullptr || *gate == want
  int want;
  // offset-form bounds (kmeans_prune.hip): stored ub - cu[label] (rounded up) and lb + cl[label]
  // (rounded down) against the per-centre cumulative drifts; null: absolute bounds
  const float* cu = nullptr;
  const float* cl = nullptr;
  // k-means|| candidate merge (MODE 2): a row whose distance to its nearest centre of this launch is
  // strictly below mcost[row] takes it (mcost = dist, mnear = label + moff) — the init's merge kernel
  // folded into the epilogue
  float* mcost = nullptr;
  int* mnear = nullptr;
  int moff = 0;
};

__host__ __device__ constexpr int cn_slots(int kp) { return ((kp + 3) & ~3) > 256 ? ((kp + 3) & ~3) : 256; }

template <int DP, bool F8 = false, int MODE = 0, bool M32 = false>
struct Geo {
  static constexpr int KS = DP / 32;            // MFMA k-steps per row
  static constexpr int ROWB = F8 ? DP : DP * 2; // bytes per row (bf16, or OCP e4m3fn bytes)
  static constexpr int TR = 32768 / ROWB;       // rows per tile (32 KiB of X)
  static constexpr int NSUB = TR / 16;          // 16-row MFMA sub-tiles per tile
  static constexpr int SLOT = TR * ROWB;        // 32 KiB
  static constexpr int PIECES = SLOT / 1024;    // 1-KiB DMA pieces per tile (32)
  static constexpr int RPP = 1024 / ROWB;       // rows per piece
  static constexpr int LPR = ROWB / 16;         // lanes (16-B chunks) per row in a piece
  static constexpr int TRAIL_Q = TR >= 64 ? TR / 64 : 1;  // dword DMA instructions per trailer array
  static constexpr int NARR = MODE == 2 ? 3 : 2;          // trailer arrays: norms, labels (, rows)
  // DMA instructions per tile: wave 0 carries the norms, wave 1 the labels (and rows)
  static constexpr int CNT0 = PIECES / 2 + TRAIL_Q;
  static constexpr int CNT1 = PIECES / 2 + (NARR - 1) * TRAIL_Q;
  static constexpr int TRB = TR * 4 * NARR;     // trailer entry bytes
  static constexpr int NK = MODE >= 1 ? 2 : 1;  // keys per (row, wave, lane group)
  // key entries per row: (compute wave, lane group) = 4 x 4 for the 16x16 MFMA tiles, 4 x 2 (lane
  // halves) for the 32x32 ones
  static constexpr int NQ = M32 ? 8 : 16;
  static constexpr int STRIDE = NQ * NK + 1;    // dwords per row of the key exchange (+1: conflict-free writes)
  static constexpr int RED = TR * STRIDE * 4;
  // M32: the finalize waves run two tiles behind the compute waves (the last sub-tile's keys of tile j
  // are formed during tile j+1), so keys are triple-buffered and the trailer ring is one entry deeper;
  // the centre norms sit in LDS (kp floats) instead of registers
  static constexpr int LAG = M32 ? 2 : 1;
  static constexpr int NKB = LAG + 1;           // key exchange buffers
  static constexpr long long fixed_bytes(int ns, int kp) {
    // (M32) the centre norms cover every centre slot a compute wave reads (4 waves x 64), padded with +inf
    const long long kp4 = (kp + 3) & ~3;
    return (long long)(ns + LAG) * TRB + (long long)NKB * RED + 4LL * kp4 + (M32 ? 4LL * cn_slots(kp) : 0LL) + 64;
  }
  // ring depth: 4 slots where LDS allows, 3 for the 128-row tiles of the top-2 modes
  static constexpr int NS = (4LL * SLOT + fixed_bytes(4, 1024)) <= 160 * 1024 ? 4 : 3;
  static constexpr int NTR = NS + LAG;          // trailer ring entries
};

// LDS layout (bytes): [X ring NS*SLOT | trailers NTR*TRB | keys NKB*RED | hist kp ints | (M32) centre
// norms kp floats | misc 64 B]
template <int DP, bool F8 = false, int MODE = 0, bool M32 = false>
__host__ __device__ constexpr long long lds_bytes(int kp) {
  using G = Geo<DP, F8, MODE, M32>;
  return (long long)G::NS * G::SLOT + G::fixed_bytes(G::NS, kp);
}

// s_waitcnt with only vmcnt = N (expcnt, lgkmcnt at their maxima: not waited for). gfx9 encoding.
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Workgroup barrier that neither drains vmcnt (in-flight LDS-DMA survives it) nor lets the compiler
// move memory accesses across it.
__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

typedef const __attribute__((address_space(4))) int* cidx_t;  // constant address space: scalar loads

// median of three (one v_med3_i32): with a <= c it is the second smallest of {a, b, c}
__device__ __forceinline__ int med3(int a, int b, int c) {
  const int lo = a < b ? a : b, hi = a < b ? b : a;
  const int m = hi < c ? hi : c;
  return lo > m ? lo : m;
}

// ldx in BYTES; rows are 16-B aligned. Positions past n load row n-1 (discarded).
template <int DP, bool F8, int MODE, bool M32>
__device__ __forceinline__ void issue_tile(const unsigned char* __restrict__ X, long long ldx, long long n,
                                           const float* __restrict__ xnorm, const int* __restrict__ labels,
                                           const int* __restrict__ idx, long long tile, int slot, int tr, int dw,
                                           int lane, unsigned char* smem) {
  using G = Geo<DP, F8, MODE, M32>;
  const long long row0 = tile * G::TR;
  unsigned char* sdst = smem + slot * G::SLOT;
  if constexpr (MODE == 2) {
    // this wave's TR/2 positions start at row0 + dw*TR/2: their rows come in as uniform scalar loads
    // (the index buffer is padded to whole tiles, entries past n are stale but valid rows), in
    // batches of 16 with the next batch's loads in flight while the current one's pieces issue
    // (a whole tile's 64 indices at once ran out of SGPRs and fell back to vector loads, whose
    // vmcnt wait would drain the ring)
    constexpr int NR = G::TR / 2;
    constexpr int BAT = NR < 16 ? NR : 16;
    constexpr int NBAT = NR / BAT;
    constexpr int PPB = BAT / G::RPP;  // pieces per batch
    const cidx_t ci = (cidx_t)(idx + row0 + dw * NR);
    const int sub = lane / G::LPR;  // row within the piece
    int cur[BAT];
#pragma unroll
    for (int i = 0; i < BAT; ++i) cur[i] = ci[i];
#pragma unroll
    for (int b = 0; b < NBAT; ++b) {
      int nxt[BAT];
      if (b + 1 < NBAT) {
#pragma unroll
        for (int i = 0; i < BAT; ++i) nxt[i] = ci[(b + 1) * BAT + i];
      }
#pragma unroll
      for (int qq = 0; qq < PPB; ++qq) {
        const int q = b * PPB + qq;
        const int p = dw * (G::PIECES / 2) + q;
        const int R = p * G::RPP + sub;
        int grow = cur[qq * G::RPP];
#pragma unroll
        for (int s = 1; s < G::RPP; ++s) grow = sub == s ? cur[qq * G::RPP + s] : grow;
        const int pos = lane % G::LPR;
        const int gch = pos ^ (R & 15);
        glds16(X + (long long)grow * ldx + 16 * gch, sdst + p * 1024);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (b + 1 < NBAT) {
#pragma unroll
        for (int i = 0; i < BAT; ++i) cur[i] = nxt[i];
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < G::PIECES / 2; ++q) {
      const int p = dw * (G::PIECES / 2) + q;
      const int R = p * G::RPP + lane / G::LPR;  // row within the tile
      const int pos = lane % G::LPR;             // LDS chunk position in the row
      const int gch = pos ^ (R & 15);            // global chunk stored there
      long long grow = row0 + R;
      grow = grow < n ? grow : n - 1;            // rows past n: any valid row (discarded)
      glds16(X + grow * ldx + 16 * gch, sdst + p * 1024);
    }
  }
  unsigned char* tbase = smem + G::NS * G::SLOT + tr * G::TRB;
#pragma unroll
  for (int q = 0; q < G::TRAIL_Q; ++q) {
    const int R = q * 64 + lane;
    long long grow = row0 + R;
    grow = grow < n ? grow : n - 1;
    if (R < G::TR) {
      if (dw == 0) {
        glds4(xnorm + grow, tbase + q * 256);
      } else {
        glds4(labels + grow, tbase + G::TR * 4 + q * 256);
        if constexpr (MODE == 2) glds4(idx + grow, tbase + G::TR * 8 + q * 256);
      }
    }
  }
}

// Compute waves on 32x32 MFMA tiles (v_mfma_f32_32x32x16_bf16), CT even: wave w holds centres
// [w·16CT, (w+1)·16CT) as NT = CT/2 A tiles of 32 centres; a 32-row sub-tile of X is the B operand
// (lane: row l&31, k half l>>5), so every output lane holds ONE X row against 16 centres per tile.
// Why: with 16x16 tiles the key epilogue (and-or tag, min3, med3) and the accumulator seeding filled
// every vector-issue slot the 16-cycle MFMAs leave (2-3 vector instructions per MFMA, ISA count of
// the steady loop), so the pass ran at ~60 % of MFMA peak even without HBM traffic; a 32x32x16 MFMA
// holds vector issue for 8 of its 32 cycles, so the same epilogue per output fits beside it.
// Accumulators start at ||c||² (read from LDS into the free buffer during the previous sub-tile's
// second half); ||x||² (one value per lane) is added when the keys are formed, in the first half of
// the NEXT sub-tile's k-steps — across tiles too, so tile j's last keys land during tile j+1 and the
// finalize waves run two tiles behind (Geo::LAG). Tags: a·16 + reg (increasing with the centre index
// for a lane, ties to the lowest centre); the finalize decodes centre = w·16CT + 32a + (reg&3) +
// 8(reg>>2) + 4h.
template <int DP, int CT, bool F8, int MODE>
__device__ __forceinline__ void compute_m32(const u16* __restrict__ C, long long ldc, int kc, long long nt,
                                            int wave, int lane, unsigned char* smem, const float* cnl, int dbg) {
  using G = Geo<DP, F8, MODE, true>;
  constexpr int NT = CT / 2;            // 32-centre A tiles per wave
  constexpr int KS2 = DP / 16;          // 32x32x16 k-steps per row
  constexpr int SPU = F8 ? 2 : 1;       // k-steps per 16-B LDS read unit
  constexpr int UPS = KS2 / SPU;        // read units per sub-tile
  constexpr int NSUB = G::TR / 32;      // 32-row sub-tiles per tile (even)
  constexpr int NU = NSUB * UPS;
  constexpr int NE = NT * 16;           // key elements per lane per sub-tile
  constexpr int HALF = KS2 / 2 < NE / 2 ? KS2 / 2 : NE / 2;  // keys are formed in the first HALF k-steps
  constexpr int EPS = NE / HALF;        // key elements per k-step (even)
  constexpr int TAGB = 4 + (NT > 1);
  constexpr int TAGM = (1 << TAGB) - 1;
  constexpr bool TOP2 = MODE >= 1;
  constexpr int PF = 2;
  static_assert(NSUB % 2 == 0 && NE % HALF == 0 && EPS % 2 == 0, "M32 geometry");
  unsigned char* trail = smem + G::NS * G::SLOT;
  int* red = reinterpret_cast<int*>(trail + G::NTR * G::TRB);
  const int r = lane & 31, hh = lane >> 5;
  const int cw0 = wave * (CT * 16);
  bf16x8 creg[NT][KS2];
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int c = cw0 + 32 * a + r;
#pragma unroll
    for (int s = 0; s < KS2; ++s) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      // bf16: step s, lane half h holds k = 16s + 8h + j; fp8: the 16-B unit v = s/2 of lane half h
      // holds k = 32v + 16h + (0..15), its low / high 8 are steps 2v / 2v+1
      const int k0 = F8 ? 32 * (s >> 1) + 16 * hh + 8 * (s & 1) : 16 * s + 8 * hh;
      if (c < kc) v = *reinterpret_cast<const uint4*>(C + (long long)c * ldc + k0);
      const unsigned w4[4] = {v.x, v.y, v.z, v.w};
      unsigned o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // x -2, exact
        const float lo = -2.f * bf16_to_f32((u16)(w4[e] & 0xffffu));
        const float hi = -2.f * bf16_to_f32((u16)(w4[e] >> 16));
        o[e] = (unsigned)f32_to_bf16(lo) | ((unsigned)f32_to_bf16(hi) << 16);
      }
      creg[a][s] = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
    }
  }
  __builtin_amdgcn_s_setprio(1);
  // B fragment of unit v, sub-tile t: row 32t + r, 16-B chunk 2v + h stored at (2v + h) ^ (r & 15)
  int boff[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) boff[m] = r * G::ROWB + (((2 * m + hh) ^ (r & 15)) << 4);
  const float* cnp = cnl + cw0 + 4 * hh;
  auto load_cn = [&](f32x16(&dst)[NT]) {
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(cnp + 32 * a + 8 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[a][4 * q + i] = v[i];
      }
  };
  f32x16 acc[2][NT];
  wait_lgkm0();
  barrier();  // B(-1): first tile landed, centre norms in LDS
  load_cn(acc[0]);
  int key = 0x7fffffff, key2 = 0x7fffffff;
  // forms key elements [e0, e1) of the pending sub-tile (accumulators pa, row norm xv)
  auto keys = [&](const f32x16(&pa)[NT], float xv, int e0, int e1) {
#pragma unroll
    for (int e = e0; e < e1; e += 2) {
      const int a = e >> 4, i = e & 15;
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      const f32x2 v = f32x2{pa[a][i], pa[a][i + 1]} + f32x2{xv, xv};  // one v_pk_add_f32
      const int k0 = (__float_as_int(v[0]) & ~TAGM) | (a << 4 | i);
      const int k1 = (__float_as_int(v[1]) & ~TAGM) | (a << 4 | (i + 1));
      if constexpr (TOP2) {
        key2 = med3(key, k0, key2);
        key = k0 < key ? k0 : key;
        key2 = med3(key, k1, key2);
        key = k1 < key ? k1 : key;
      } else {
        const int m = k0 < k1 ? k0 : k1;
        key = m < key ? m : key;
      }
    }
  };
  auto put_keys = [&](int* kred, int row) {
    kred[row * G::STRIDE + wave * 2 + hh] = key;
    if constexpr (TOP2) kred[row * G::STRIDE + 8 + wave * 2 + hh] = key2;
    key = 0x7fffffff;
    key2 = 0x7fffffff;
  };
  for (long long j = 0; j < nt; ++j) {
    if (dbg & 2) {
      wait_lgkm0();
      barrier();
      continue;
    }
    const unsigned char* xs = smem + (int)(j % G::NS) * G::SLOT;
    const float* tn = reinterpret_cast<const float*>(trail + (int)(j % G::NTR) * G::TRB);
    const float* tnp = reinterpret_cast<const float*>(trail + (int)((j + G::NTR - 1) % G::NTR) * G::TRB);
    int* kr = red + (int)(j % G::NKB) * G::TR * G::STRIDE;
    int* krp = red + (int)((j + G::NKB - 1) % G::NKB) * G::TR * G::STRIDE;
    auto xaddr = [&](int u) {
      const int t = u / UPS, v = u % UPS;
      return xs + 32 * t * G::ROWB + 256 * (v >> 3) + boff[v & 7];
    };
    uint4 xr[PF + 1];
#pragma unroll
    for (int u = 0; u < PF && u < NU; ++u) xr[u] = *reinterpret_cast<const uint4*>(xaddr(u));
    // the pending sub-tile at t = 0 is the previous tile's last one (none before the first tile)
    float xpend = j > 0 ? tnp[32 * (NSUB - 1) + r] : 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int t = u / UPS, v = u % UPS, cur = t & 1, prv = cur ^ 1;
      if (u + PF < NU) xr[(u + PF) % (PF + 1)] = *reinterpret_cast<const uint4*>(xaddr(u + PF));
      if (v == 0 && t > 0) xpend = tn[32 * (t - 1) + r];
      bf16x8 xb[SPU];
      if constexpr (F8) {
        const uint4 w = xr[u % (PF + 1)];
        const unsigned ws[4] = {w.x, w.y, w.z, w.w};
        unsigned o[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          o[2 * q] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(ws[q], 1.0f, false));
          o[2 * q + 1] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(ws[q], 1.0f, true));
        }
        xb[0] = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
        xb[SPU - 1] = __builtin_bit_cast(bf16x8, make_uint4(o[4], o[5], o[6], o[7]));
      } else {
        xb[0] = __builtin_bit_cast(bf16x8, xr[u % (PF + 1)]);
      }
#pragma unroll
      for (int h = 0; h < SPU; ++h) {
        const int s = v * SPU + h;
#pragma unroll
        for (int a = 0; a < NT; ++a)
          acc[cur][a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(creg[a][s], xb[h], acc[cur][a], 0, 0, 0);
        const bool pending = t > 0 || j > 0;
        if (s < HALF) {
          if (pending) keys(acc[prv], xpend, s * EPS, (s + 1) * EPS);
          if (s == HALF - 1 && pending) {
            if (t > 0) put_keys(kr, 32 * (t - 1) + r);
            else put_keys(krp, 32 * (NSUB - 1) + r);
          }
        } else if (s == HALF) {
          load_cn(acc[prv]);  // seeds of the next sub-tile (its accumulators are free now)
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_lgkm0();
    barrier();  // B(j)
  }
  if (nt > 0 && !(dbg & 2)) {  // keys of the very last sub-tile (accumulator parity (NSUB-1)&1 = 1)
    const float* tn = reinterpret_cast<const float*>(trail + (int)((nt - 1) % G::NTR) * G::TRB);
    keys(acc[1], tn[32 * (NSUB - 1) + r], 0, NE);
    put_keys(red + (int)((nt - 1) % G::NKB) * G::TR * G::STRIDE, 32 * (NSUB - 1) + r);
  }
  wait_lgkm0();
  barrier();  // B(nt)
}

// MX compute waves (fp8 rows): the e4m3 X bytes go straight into v_mfma_scale_f32_16x16x128_f8f6f4 as the
// B operand (no widening), against an exact two-term e4m3 split of the bf16 centres held in VGPRs:
//
//   v = -2·c (bf16),  hi = e4m3(v·2^s),  lo = e4m3((v - hi·2^-s)·2^t),  v = hi·2^-s + lo·2^-t
//
// with E8M0 block scales 2^-s, 2^-t per 32 k (the block's largest value scaled into [128, 256)). The split is
// exact for centres on the MX grid, which the fp8 engines keep theirs on (kmeans_mx.hip mx_snap after every
// centre update: a bf16 value far below its block's largest loses the bits e4m3 subnormals cannot hold), so
// the products are those of the bf16 pass; per 128 k two MX MFMAs (hi, lo) at twice the bf16 rate — the
// MFMA time of the bf16 pass with none of its v_cvt_scalef32_pk_bf16_fp8 widening of every X fragment in
// every compute wave, which bound that pass (19.6 ms at 125M x 512, k = 128).
// Layout (measured, scripts/mx_probe_layout.py, pinned by tests/test_kmeans_mx_gpu.py): bytes 0-15 of lane
// (r, g) are k 16g + j, bytes 16-31 are k 64 + 16g + j, and lane group q supplies the scale of k [32q, 32q+32).
// Lane (r, g) of block b therefore reads the 16-B units 2b and 2b + 1 of the K9r fp8 order (chunks 8b + g
// and 8b + 4 + g of row r); its split partner for both halves' scale blocks is lane (r, g ^ 1).
// Accumulators start at |c|² + |x|²; keys and the exchange are those of the 16x16 bf16 path.
typedef int mx_v8i __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned mx_e4m3(float v) {
  return (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xffu;
}
__device__ __forceinline__ float mx_f32(unsigned b) { return __builtin_amdgcn_cvt_f32_fp8((int)b, 0); }
// s with m·2^s in [128, 256): every value of the block fits e4m3 (max 448); E8M0 range clamp
__device__ __forceinline__ int mx_shift(float m) {
  if (!(m > 0.f)) return 0;
  int e;
  (void)frexpf(m, &e);
  const int s = 8 - e;
  return s < -120 ? -120 : (s > 120 ? 120 : s);
}

// One half of a lane's MX operand: the 16 bf16 values of one 16-B chunk (4 dwords) as -2·c, split into
// packed hi / lo e4m3 bytes; the block scales are shared with the partner lane (lane ^ 16, the other half
// of the 32-element block). Returns the E8M0 pair (hi | lo << 8) of this half's block.
__device__ __forceinline__ int mx_split_half(const uint4 w0, const uint4 w1, unsigned (&wh)[4], unsigned (&wl)[4]) {
  const unsigned ws[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
  float v[16];
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[2 * e] = -2.f * __uint_as_float(ws[e] << 16);
    v[2 * e + 1] = -2.f * __uint_as_float(ws[e] & 0xffff0000u);
    m = fmaxf(m, fmaxf(fabsf(v[2 * e]), fabsf(v[2 * e + 1])));
  }
  const int s = mx_shift(fmaxf(m, __shfl_xor(m, 16, 64)));
  // two values per v_cvt_pk_fp8_f32 into one half of the dword: the bytes are packed as they are made (the
  // empty asm keeps each packed dword opaque: otherwise the compiler carried every byte in its own VGPR up
  // to the MFMA operand and spilled)
  float mr = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * q], s), ldexpf(v[4 * q + 1], s), 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * q + 2], s), ldexpf(v[4 * q + 3], s), w, true);
    asm volatile("" : "+v"(w));
    wh[q] = (unsigned)w;
    // the residuals, in place
    v[4 * q] -= ldexpf(__builtin_amdgcn_cvt_f32_fp8(w, 0), -s);
    v[4 * q + 1] -= ldexpf(__builtin_amdgcn_cvt_f32_fp8(w, 1), -s);
    v[4 * q + 2] -= ldexpf(__builtin_amdgcn_cvt_f32_fp8(w, 2), -s);
    v[4 * q + 3] -= ldexpf(__builtin_amdgcn_cvt_f32_fp8(w, 3), -s);
    mr = fmaxf(fmaxf(mr, fmaxf(fabsf(v[4 * q]), fabsf(v[4 * q + 1]))), fmaxf(fabsf(v[4 * q + 2]), fabsf(v[4 * q + 3])));
  }
  const int t = mx_shift(fmaxf(mr, __shfl_xor(mr, 16, 64)));
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * q], t), ldexpf(v[4 * q + 1], t), 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * q + 2], t), ldexpf(v[4 * q + 3], t), w, true);
    asm volatile("" : "+v"(w));
    wl[q] = (unsigned)w;
  }
  return (127 - s) | ((127 - t) << 8);
}

template <int DP, int CT, int MODE>
__device__ __forceinline__ void compute_mx(const u16* __restrict__ C, long long ldc, const float* __restrict__ cnorm,
                                           int kc, long long nt, int wave, int lane, unsigned char* smem, int dbg) {
  using G = Geo<DP, true, MODE, false>;
  constexpr int NB = DP / 128;          // MX k-blocks per row
  constexpr int UPS = 2 * NB;           // 16-B read units per 16-row sub-tile
  constexpr int NU = G::NSUB * UPS;
  constexpr int TAGB = 2 + (CT > 1) + (CT > 2) + (CT > 4);
  constexpr int TAGM = (1 << TAGB) - 1;
  constexpr bool TOP2 = MODE >= 1;
  constexpr int PF = 4;                 // units read ahead (two blocks)
  constexpr int RING = PF + 2;          // a block's first unit stays live while its second lands
  static_assert(DP % 128 == 0, "MX blocks");
  unsigned char* trail = smem + G::NS * G::SLOT;
  int* red = reinterpret_cast<int*>(trail + G::NTR * G::TRB);
  const int r = lane & 15, g = lane >> 4;
  const int cw0 = wave * CT * 16;
  mx_v8i chi[CT][NB], clo[CT][NB];
  int csc[CT][NB];
  f32x4 c4[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int c = cw0 + ct * 16 + r;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      // half h: chunk 8b + 4h + g; half h of lanes g and g ^ 1 form scale block 2h + (g >> 1)
      unsigned wh[2][4], wl[2][4];
      int sc2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint4 w0 = make_uint4(0u, 0u, 0u, 0u), w1 = make_uint4(0u, 0u, 0u, 0u);
        if (c < kc) {
          const uint4* src = reinterpret_cast<const uint4*>(C + (long long)c * ldc + 16 * (8 * b + 4 * h + g));
          w0 = src[0];
          w1 = src[1];
        }
        sc2[h] = mx_split_half(w0, w1, wh[h], wl[h]);
        __builtin_amdgcn_sched_barrier(0);
      }
      chi[ct][b] = mx_v8i{(int)wh[0][0], (int)wh[0][1], (int)wh[0][2], (int)wh[0][3],
                          (int)wh[1][0], (int)wh[1][1], (int)wh[1][2], (int)wh[1][3]};
      clo[ct][b] = mx_v8i{(int)wl[0][0], (int)wl[0][1], (int)wl[0][2], (int)wl[0][3],
                          (int)wl[1][0], (int)wl[1][1], (int)wl[1][2], (int)wl[1][3]};
      // lane group g supplies the scale of block g = 2h + (g' >> 1): half g >> 1 of lane group 2(g & 1)
      const int src = r + 16 * (2 * (g & 1));
      const int s0 = __shfl(sc2[0], src, 64);
      const int s1 = __shfl(sc2[1], src, 64);
      csc[ct][b] = (g >> 1) ? s1 : s0;
      // one block at a time: left free, the scheduler hoisted every block's loads and split temporaries
      // ahead and spilled (the operands alone take 128 VGPRs at CT = 2, D = 512)
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c2 = cw0 + ct * 16 + 4 * g + i;
      c4[ct][i] = c2 < kc ? cnorm[c2] : __builtin_huge_valf();
    }
  }
  __builtin_amdgcn_s_setprio(1);
  int boff[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) boff[b] = r * G::ROWB + (((4 * b + g) ^ r) << 4);
  barrier();  // B(-1): first tile landed
  for (long long j = 0; j < nt; ++j) {
    if (dbg & 2) {
      wait_lgkm0();
      barrier();
      continue;
    }
    const unsigned char* xs = smem + (int)(j % G::NS) * G::SLOT;
    const float* tn = reinterpret_cast<const float*>(trail + (int)(j % G::NTR) * G::TRB);
    int* kred = red + (int)(j & 1) * G::TR * G::STRIDE;
    float xnv[G::NSUB];
#pragma unroll
    for (int t = 0; t < G::NSUB; ++t) xnv[t] = tn[16 * t + r];
    auto xaddr = [&](int u) {  // unit v of sub-tile t: chunk 4v + g of row 16t + r
      const int t = u / UPS, v = u % UPS;
      return xs + 16 * t * G::ROWB + 256 * (v >> 2) + boff[v & 3];
    };
    uint4 xr[RING];
#pragma unroll
    for (int u = 0; u < PF && u < NU; ++u) xr[u] = *reinterpret_cast<const uint4*>(xaddr(u));
    f32x4 acc[2][CT];
    int key[2] = {0x7fffffff, 0x7fffffff};
    int key2[2] = {0x7fffffff, 0x7fffffff};
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int t = u / UPS, v = u % UPS, cur = t & 1, prv = cur ^ 1;
      if (u + PF < NU) xr[(u + PF) % RING] = *reinterpret_cast<const uint4*>(xaddr(u + PF));
      if (v & 1) {
        const int s = v >> 1;  // MX block
        const uint4 a0 = xr[(u - 1) % RING], a1 = xr[u % RING];
        const mx_v8i xb = mx_v8i{(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
        if (s == 0) {
          key[cur] = 0x7fffffff;
          if constexpr (TOP2) key2[cur] = 0x7fffffff;
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const f32x4 a = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              chi[ct][s], xb, s == 0 ? (c4[ct] + xnv[t]) : acc[cur][ct], 0, 0, 0, csc[ct][s], 0, 127);
          acc[cur][ct] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(clo[ct][s], xb, a, 0, 0, 1, csc[ct][s], 0, 127);
        }
        if (t > 0) {  // keys of the previous sub-tile, spread over this one's blocks
#pragma unroll
          for (int e = (s * CT * 4) / NB; e < ((s + 1) * CT * 4) / NB; ++e) {
            const int ct = e >> 2, i = e & 3;
            const int kv = (__float_as_int(acc[prv][ct][i]) & ~TAGM) | (ct << 2 | i);
            if constexpr (TOP2) key2[prv] = med3(key[prv], kv, key2[prv]);
            key[prv] = kv < key[prv] ? kv : key[prv];
          }
          if (s == NB - 1) {
            kred[(16 * (t - 1) + r) * G::STRIDE + wave * 4 + g] = key[prv];
            if constexpr (TOP2) kred[(16 * (t - 1) + r) * G::STRIDE + 16 + wave * 4 + g] = key2[prv];
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    {
      constexpr int t = G::NSUB - 1, cur = t & 1;
#pragma unroll
      for (int e = 0; e < CT * 4; ++e) {
        const int ct = e >> 2, i = e & 3;
        const int kv = (__float_as_int(acc[cur][ct][i]) & ~TAGM) | (ct << 2 | i);
        if constexpr (TOP2) key2[cur] = med3(key[cur], kv, key2[cur]);
        key[cur] = kv < key[cur] ? kv : key[cur];
      }
      kred[(16 * t + r) * G::STRIDE + wave * 4 + g] = key[cur];
      if constexpr (TOP2) kred[(16 * t + r) * G::STRIDE + 16 + wave * 4 + g] = key2[cur];
    }
    wait_lgkm0();
    barrier();  // B(j)
  }
}

// F8: X rows are OCP e4m3fn bytes (SURVEY config 5). They travel through the ring as bytes (half the
// HBM and LDS traffic) and every compute wave widens its fragments with v_cvt_scalef32_pk_bf16_fp8
// (exact: e4m3 values are a subset of bf16); one 16-B read then covers TWO k-steps, step 2v+h of lane
// (r, g) holding k = 64v + 16g + 8h + j, and the centre fragments follow the same k order.
template <int DP, int CT, bool F8, int MODE, bool M32, bool MX = false>
__global__ __launch_bounds__(kThreads, 1) void kmeans_assign_rr(
    const unsigned char* __restrict__ X, long long n, long long ldx, const u16* __restrict__ C, long long ldc, int kc,
    int kp, const float* __restrict__ cnorm, const float* __restrict__ xnorm, int* __restrict__ labels,
    float* __restrict__ best_out, double* __restrict__ cost_part, int* __restrict__ hist_out,
    int* __restrict__ rank_out, DeltaOut dout, Ext ext, int dbg) {
  // dbg (ablation only, 0 in production): bit 0 DMA waves issue nothing, bit 1 compute waves skip
  // their MFMAs/keys, bit 2 finalize waves skip the epilogue
  using G = Geo<DP, F8, MODE, M32>;
  constexpr int KS = G::KS;
  constexpr int NS = G::NS;
  constexpr int CPW = CT * 16;  // centres per compute wave
  constexpr int TAGB = 2 + (CT > 1) + (CT > 2) + (CT > 4);
  constexpr int TAGM = (1 << TAGB) - 1;
  constexpr bool TOP2 = MODE >= 1;
  if (ext.gate != nullptr && *ext.gate != ext.want) return;  // uniform: before any barrier
  if constexpr (MODE == 2) n = *ext.n_dev;
  const int* lab_src = MODE == 2 ? ext.lab_in : labels;  // trailer source of the previous labels
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* trail = smem + NS * G::SLOT;
  int* red = reinterpret_cast<int*>(trail + G::NTR * G::TRB);
  int* hist = red + G::NKB * G::TR * G::STRIDE;
  float* cnl = reinterpret_cast<float*>(hist + ((kp + 3) & ~3));  // M32: centre norms [cn_slots(kp)]
  int* misc = M32 ? reinterpret_cast<int*>(cnl + cn_slots(kp)) : hist + ((kp + 3) & ~3);
  // misc: [0] change counter, [2..5] two f64 cost partials
  double* cost_sh = reinterpret_cast<double*>(misc + 2);

  // the role index is wave-uniform: readfirstlane lets the compiler branch on it with scalar
  // instructions and keep addresses derived from it (the MODE 2 index loads) in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long ntiles = (n + G::TR - 1) / G::TR;
  const long long nt = ntiles > blockIdx.x ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const bool ranking = rank_out != nullptr;
  auto tile_of = [&](long long j) { return (long long)blockIdx.x + j * gridDim.x; };

  if (wave < kCompute) {
   if constexpr (MX) {
    compute_mx<DP, CT, MODE>(C, ldc, cnorm, kc, nt, wave, lane, smem, dbg);
   } else if constexpr (M32) {
    for (int i = tid; i < cn_slots(kp); i += kCompute * 64) cnl[i] = i < kc ? cnorm[i] : __builtin_huge_valf();
    compute_m32<DP, CT, F8, MODE>(C, ldc, kc, nt, wave, lane, smem, cnl, dbg);
   } else {
    // ------------------------------------------------------------------ compute waves
    const int r = lane & 15, g = lane >> 4;
    const int cw0 = wave * CPW;
    bf16x8 creg[CT][KS];
    f32x4 c4[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int c = cw0 + ct * 16 + r;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        const int k0 = F8 ? 64 * (s >> 1) + 16 * g + 8 * (s & 1) : 32 * s + 8 * g;
        if (c < kc) v = *reinterpret_cast<const uint4*>(C + (long long)c * ldc + k0);
        const unsigned w4[4] = {v.x, v.y, v.z, v.w};
        unsigned o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // x -2, exact (power-of-two scale of a bf16 value)
          const float lo = -2.f * bf16_to_f32((u16)(w4[e] & 0xffffu));
          const float hi = -2.f * bf16_to_f32((u16)(w4[e] >> 16));
          o[e] = (unsigned)f32_to_bf16(lo) | ((unsigned)f32_to_bf16(hi) << 16);
        }
        creg[ct][s] = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c2 = cw0 + ct * 16 + 4 * g + i;
        c4[ct][i] = c2 < kc ? cnorm[c2] : __builtin_huge_valf();
      }
    }
    __builtin_amdgcn_s_setprio(1);
    // per-lane byte offset of B fragment (sub-tile 0, k-step s): row r, chunk (4s + g) ^ r
    int boff[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) boff[b] = r * G::ROWB + (((4 * b + g) ^ r) << 4);
    barrier();  // B(-1): first tile landed
    for (long long j = 0; j < nt; ++j) {
      if (dbg & 2) {
        wait_lgkm0();
        barrier();
        continue;
      }
      const unsigned char* xs = smem + (int)(j % NS) * G::SLOT;
      const float* tn = reinterpret_cast<const float*>(trail + (int)(j % G::NTR) * G::TRB);
      int* kred = red + (int)(j & 1) * G::TR * G::STRIDE;
      // The tile is one flat, fully unrolled sequence of NSUB*KS steps (sub-tile t, k-step s). The B
      // fragment of step u+PF is read while step u's MFMAs issue (a scheduling barrier per step pins
      // it: left alone, the scheduler issued each read one step ahead, 4 MFMAs = 64 cycles, under the
      // LDS latency), and the previous sub-tile's key updates ride in the VALU gaps.
      constexpr int SPU = F8 ? 2 : 1;      // k-steps per 16-B LDS read unit
      constexpr int UPS = KS / SPU;        // read units per sub-tile
      constexpr int NU = G::NSUB * UPS;
      constexpr int PF = 3;
      float xnv[G::NSUB];
#pragma unroll
      for (int t = 0; t < G::NSUB; ++t) xnv[t] = tn[16 * t + r];
      auto xaddr = [&](int u) {
        const int t = u / UPS, v = u % UPS;
        return xs + 16 * t * G::ROWB + 256 * (v >> 2) + boff[v & 3];
      };
      uint4 xr[PF + 1];
#pragma unroll
      for (int u = 0; u < PF && u < NU; ++u) xr[u] = *reinterpret_cast<const uint4*>(xaddr(u));
      f32x4 acc[2][CT];
      int key[2] = {0x7fffffff, 0x7fffffff};
      int key2[2] = {0x7fffffff, 0x7fffffff};  // TOP2: second smallest key
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int t = u / UPS, v = u % UPS, cur = t & 1, prv = cur ^ 1;
        if (u + PF < NU) xr[(u + PF) % (PF + 1)] = *reinterpret_cast<const uint4*>(xaddr(u + PF));
        bf16x8 xb[SPU];
        if constexpr (F8) {
          const uint4 w = xr[u % (PF + 1)];
          const unsigned ws[4] = {w.x, w.y, w.z, w.w};
          unsigned o[8];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o[2 * q] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(ws[q], 1.0f, false));
            o[2 * q + 1] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(ws[q], 1.0f, true));
          }
          xb[0] = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
          xb[SPU - 1] = __builtin_bit_cast(bf16x8, make_uint4(o[4], o[5], o[6], o[7]));
        } else {
          xb[0] = __builtin_bit_cast(bf16x8, xr[u % (PF + 1)]);
        }
#pragma unroll
        for (int h = 0; h < SPU; ++h) {
          const int s = v * SPU + h;
          if (s == 0) {
            key[cur] = 0x7fffffff;
            if constexpr (TOP2) key2[cur] = 0x7fffffff;
          }
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
            acc[cur][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                creg[ct][s], xb[h], s == 0 ? (c4[ct] + xnv[t]) : acc[cur][ct], 0, 0, 0);
          if (t > 0) {  // keys of the previous sub-tile, spread over this one's k-steps
#pragma unroll
            for (int e = (s * CT * 4) / KS; e < ((s + 1) * CT * 4) / KS; ++e) {
              const int ct = e >> 2, i = e & 3;
              const int kv = (__float_as_int(acc[prv][ct][i]) & ~TAGM) | (ct << 2 | i);
              if constexpr (TOP2) key2[prv] = med3(key[prv], kv, key2[prv]);  // key <= key2: new second
              key[prv] = kv < key[prv] ? kv : key[prv];
            }
            if (s == KS - 1) {
              kred[(16 * (t - 1) + r) * G::STRIDE + wave * 4 + g] = key[prv];
              if constexpr (TOP2) kred[(16 * (t - 1) + r) * G::STRIDE + 16 + wave * 4 + g] = key2[prv];
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep every unit's read PF units ahead of its use
      }
      {
        constexpr int t = G::NSUB - 1, cur = t & 1;
#pragma unroll
        for (int e = 0; e < CT * 4; ++e) {
          const int ct = e >> 2, i = e & 3;
          const int kv = (__float_as_int(acc[cur][ct][i]) & ~TAGM) | (ct << 2 | i);
          if constexpr (TOP2) key2[cur] = med3(key[cur], kv, key2[cur]);
          key[cur] = kv < key[cur] ? kv : key[cur];
        }
        kred[(16 * t + r) * G::STRIDE + wave * 4 + g] = key[cur];
        if constexpr (TOP2) kred[(16 * t + r) * G::STRIDE + 16 + wave * 4 + g] = key2[cur];
      }
      wait_lgkm0();
      barrier();  // B(j)
    }
   }
  } else if (wave < kCompute + 2) {
    // ------------------------------------------------------------------ LDS-DMA waves
    const int dw = wave - kCompute;
    for (long long j = 0; j < NS - 1 && j < nt && !(dbg & 1); ++j)
      issue_tile<DP, F8, MODE, M32>(X, ldx, n, xnorm, lab_src, ext.idx, tile_of(j), (int)j, (int)j, dw, lane, smem);
    if (nt >= NS - 1) {
      if (dw == 0) wait_vm<(NS - 2) * G::CNT0>();
      else wait_vm<(NS - 2) * G::CNT1>();
    } else {
      wait_vm<0>();
    }
    barrier();  // B(-1)
    for (long long j = 0; j < nt; ++j) {
      const long long jn = j + NS - 1;
      if (jn < nt && !(dbg & 1)) {
        issue_tile<DP, F8, MODE, M32>(X, ldx, n, xnorm, lab_src, ext.idx, tile_of(jn), (int)(jn % NS),
                                      (int)(jn % G::NTR), dw, lane, smem);
        // tile j+1 has landed; j+2 .. j+NS-1 stay in flight
        if (dw == 0) wait_vm<(NS - 2) * G::CNT0>();
        else wait_vm<(NS - 2) * G::CNT1>();
      } else {
        wait_vm<0>();
      }
      barrier();  // B(j)
    }
    if constexpr (M32) barrier();  // B(nt)
  } else {
    // ------------------------------------------------------------------ finalize waves
    const int fw = wave - kCompute - 2;
    constexpr int RPF = G::TR / 2;  // rows per finalize wave
    if (fw == 0) {
      for (int i = lane; i < kp; i += 64) hist[i] = 0;
      if (lane == 0) misc[0] = 0;
    }
    double cost = 0.0;
    float mcv = 0.f;
    if constexpr (TOP2) mcv = *ext.mc;
    // LPR_F lanes per row, each taking 16 / LPR_F of the 16 (wave, lane-group) keys; keys are loaded
    // in one batch and reduced branch-free on a 64-bit (value, centre index) composite
    constexpr int LPR_F = 64 / RPF;
    constexpr int QPL = G::NQ / LPR_F;
    const int rl = lane % RPF, part = lane / RPF;
    auto finalize = [&](long long j) {
      const int* kr = red + (int)(j % G::NKB) * G::TR * G::STRIDE;
      const unsigned char* te = trail + (int)(j % G::NTR) * G::TRB;
      const int R = fw * RPF + rl;
      const long long pos = tile_of(j) * G::TR + R;
      int kv[QPL], kv2[QPL];
#pragma unroll
      for (int q = 0; q < QPL; ++q) {
        kv[q] = kr[R * G::STRIDE + part * QPL + q];
        if constexpr (TOP2) kv2[q] = kr[R * G::STRIDE + G::NQ + part * QPL + q];
      }
      const int old = reinterpret_cast<const int*>(te + G::TR * 4)[R];
      long long row = pos;
      if constexpr (MODE == 2) row = reinterpret_cast<const int*>(te + G::TR * 8)[R];
      unsigned long long best = ~0ull;
      unsigned sec = ~0u;  // TOP2: second smallest value, order-preserving unsigned form
#pragma unroll
      for (int q = 0; q < QPL; ++q) {
        const int qq = part * QPL + q;
        unsigned idx;
        if constexpr (M32) {  // qq = w*2 + h, tag = a*16 + reg: centre w*CPW + 32a + (reg&3) + 8(reg>>2) + 4h
          const int tag = kv[q] & ((1 << (4 + (CT > 2))) - 1);
          const int rg = tag & 15;
          idx = (unsigned)((qq >> 1) * CPW + 32 * (tag >> 4) + (rg & 3) + 8 * (rg >> 2) + 4 * (qq & 1));
        } else {  // qq = w*4 + g: centres w*CPW + ct*16 + 4g + i
          const int tag = kv[q] & TAGM;
          idx = (unsigned)((qq >> 2) * CPW + (qq & 3) * 4 + (tag >> 2) * 16 + (tag & 3));
        }
        const int tagm = M32 ? ((1 << (4 + (CT > 2))) - 1) : TAGM;
        const unsigned u1 = (unsigned)(kv[q] & ~tagm) ^ 0x80000000u;
        const unsigned long long c = ((unsigned long long)u1 << 32) | idx;
        if constexpr (TOP2) {
          // second of the union = min(larger of the two firsts, smaller of the two seconds)
          const unsigned u2 = (unsigned)(kv2[q] & ~tagm) ^ 0x80000000u;
          const unsigned bv = (unsigned)(best >> 32);
          const unsigned mx = u1 > bv ? u1 : bv;
          const unsigned s2 = u2 < sec ? u2 : sec;
          sec = mx < s2 ? mx : s2;
        }
        best = c < best ? c : best;
      }
#pragma unroll
      for (int o = RPF; o < 64; o <<= 1) {
        const unsigned long long ob = __shfl_xor(best, o, 64);
        if constexpr (TOP2) {
          const unsigned os = __shfl_xor(sec, o, 64);
          const unsigned bv = (unsigned)(best >> 32), obv = (unsigned)(ob >> 32);
          const unsigned mx = obv > bv ? obv : bv;
          const unsigned s2 = os < sec ? os : sec;
          sec = mx < s2 ? mx : s2;
        }
        best = ob < best ? ob : best;
      }
      const int bi = (int)(best & 0xffffffffu);
      const float dist = fmaxf(__int_as_float((int)((unsigned)(best >> 32) ^ 0x80000000u)), 0.f);
      const bool mine = part == 0 && pos < n;
      const bool ch = mine && old != bi;
      if (dout.rows != nullptr) {
        const unsigned long long bal = __ballot(ch);
        if (bal != 0ull) {
          const int leader = __builtin_ctzll(bal);
          int base = 0;
          if (lane == leader) base = atomicAdd(misc, (int)__popcll(bal));
          base = __shfl(base, leader, 64);
          const int at = base + (int)__popcll(bal & ((1ull << lane) - 1ull));
          if (ch && at < dout.pcap) {
            const long long o = (long long)blockIdx.x * dout.pcap + at;
            dout.rows[o] = (int)row;
            dout.old[o] = old;
          }
        }
      }
      if (ch) labels[row] = bi;
      if (mine) {
        cost += (double)dist;
        if (best_out != nullptr) best_out[row] = dist;
        if constexpr (MODE == 2) {
          if (ext.mcost != nullptr && dist < ext.mcost[row]) {
            ext.mcost[row] = dist;
            ext.mnear[row] = bi + ext.moff;
          }
        }
        if (ranking) rank_out[row] = atomicAdd(hist + bi, 1);
        if constexpr (TOP2) {
          const float xn = reinterpret_cast<const float*>(te)[R];
          const float slack = ext.tau * (xn + mcv);
          const float sd = __int_as_float((int)(sec ^ 0x80000000u));
          float u = sqrtf(dist + slack) * (1.0f + 1e-6f);
          float w = sqrtf(fmaxf(sd - slack, 0.f)) * (1.0f - 1e-6f);
          if (ext.cu != nullptr) {
            const float cu = ext.cu[bi], cl = ext.cl[bi];
            u = (u - cu) + 1e-6f * (u + cu);
            w = (w + cl) - 1e-6f * (w + cl);
          }
          ext.ub[row] = u;
          ext.lb[row] = w;
        }
      }
    };
    wait_lgkm0();
    barrier();  // B(-1)
    constexpr int LAG = G::LAG;  // tile j's keys are complete at B(j + LAG - 1)
    for (long long j = 0; j < nt; ++j) {
      if (j >= LAG && !(dbg & 4)) finalize(j - LAG);
      wait_lgkm0();
      barrier();  // B(j)
    }
    if constexpr (LAG == 2) {
      if (nt >= 2 && !(dbg & 4)) finalize(nt - 2);
      wait_lgkm0();
      barrier();  // B(nt)
    }
    if (nt > 0 && !(dbg & 4)) finalize(nt - 1);
    cost = wave_sum_f64(cost);
    if (lane == 0) cost_sh[fw] = cost;
    wait_lgkm0();
  }
  __syncthreads();  // epilogue: every wave, all DMA drained
  if (tid == 0) {
    if (cost_part != nullptr) cost_part[blockIdx.x] = cost_sh[0] + cost_sh[1];
    if (dout.rows != nullptr) {
      const int c = misc[0];
      dout.wg_count[blockIdx.x] = c < dout.pcap ? c : dout.pcap;
      if (c > dout.pcap) *dout.overflow = 1;
    }
  }
  if (ranking)
    for (int i = tid; i < kp; i += kThreads) hist_out[(long long)blockIdx.x * kp + i] = hist[i];
}

// Centre tiles per compute wave for kc centres (kc <= 64·CT), or 0 when K9r does not apply
// (D outside {128, 256, 512} — {256, 512} for fp8 rows —, or the centres do not fit 128 VGPRs per lane).
// CT = 3 and 5 exist for bf16 Dp <= 256 (CT = 5 holds 160 VGPRs of centres at Dp = 256): a 320-centre
// chunk is one pass where 256 + 64 took two (k-means|| candidate rounds of 2k = 512-640 centres).
inline int plan_ct(int Dp, int kc, bool f8 = false) {
  if (Dp != 128 && Dp != 256 && Dp != 512) return 0;
  if (f8 && Dp < 256) return 0;
  const int ct = (kc + 63) / 64;
  if (ct > 5) return 0;  // CT = 8 spills at 256 VGPRs
  const int c = ct <= 2 ? (ct < 1 ? 1 : ct) : (Dp <= 256 ? ct : 4);
  if (ct > 4 && (Dp > 256 || f8)) return 0;  // fp8 CT = 5 spills (the widening needs registers)
  if (c * (Dp / 32) > 40) return 0;
  return c;
}

inline int tile_rows(int Dp, bool f8 = false) { return Dp > 0 ? 32768 / ((f8 ? 1 : 2) * Dp) : 0; }

// 32x32 MFMA compute waves (compute_m32) for even CT where a tile holds an even number of 32-row
// sub-tiles (not bf16 D = 512), selected by cml_kmeans_set_rr_m32(1) / CML_KMEANS_RR_M32=1. Off by
// default: measured on MI355X (profiles/r3/k9r_m32_vs_m16.txt) the 16x16 form is faster — 2.45 vs
// 2.71 ms for 20M x 256, k = 256 — because the pass is bound by the MFMA pipe under the power-limited
// clock (MFMA-only ablation 1.86 ms either way), not by vector issue slots.
inline int g_m32 = 0;
inline bool use_m32(int Dp, int ct, bool f8) {
  const int tr = tile_rows(Dp, f8);
  return g_m32 && (ct == 2 || ct == 4) && tr >= 64 && (tr / 32) % 2 == 0;
}

template <int MODE, bool M32>
inline long long lds_for_mode(int Dp, int kp, bool f8) {
  if (f8) {
    switch (Dp) {
      case 256: return lds_bytes<256, true, MODE, M32>(kp);
      case 512: return lds_bytes<512, true, MODE, M32>(kp);
      default: return 0;
    }
  }
  switch (Dp) {
    case 128: return lds_bytes<128, false, MODE, M32>(kp);
    case 256: return lds_bytes<256, false, MODE, M32>(kp);
    case 512: return lds_bytes<512, false, MODE, M32>(kp);
    default: return 0;
  }
}

inline long long lds_for(int Dp, int kp, bool f8 = false, int mode = 0) {
  const bool m32 = use_m32(Dp, plan_ct(Dp, kp, f8), f8);
  switch (mode * 2 + (m32 ? 1 : 0)) {
    case 0: return lds_for_mode<0, false>(Dp, kp, f8);
    case 1: return lds_for_mode<0, true>(Dp, kp, f8);
    case 2: return lds_for_mode<1, false>(Dp, kp, f8);
    case 3: return lds_for_mode<1, true>(Dp, kp, f8);
    case 4: return lds_for_mode<2, false>(Dp, kp, f8);
    case 5: return lds_for_mode<2, true>(Dp, kp, f8);
    default: return 0;
  }
}

// MX arithmetic for fp8 rows (compute_mx), on unless cml_kmeans_set_fp8_mx(0) / CML_KMEANS_FP8_MX=0 (the
// widening bf16 pass: A/B). The fp8 engines snap their centres to the MX grid while it is on.
inline int g_mx = 1;
inline bool use_mx(int Dp, bool f8, bool m32) { return f8 && g_mx && !m32 && Dp % 128 == 0; }

// X: bf16 rows (ldx elements) or, with f8, e4m3fn rows (ldx bytes).
template <int DP, int CT, bool F8, int MODE, bool M32, bool MX = false>
int launch(const void* X, long long n, long long ldx, const u16* C, long long ldc, int kc, int kp, const float* cnorm,
           const float* xnorm, int* labels, float* best, double* cost_part, int* hist, int* rank, DeltaOut dout,
           Ext ext, int grid, int dbg, hipStream_t st) {
  const size_t lds = (size_t)lds_bytes<DP, F8, MODE, M32>(kp);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const void* fn = (const void*)kmeans_assign_rr<DP, CT, F8, MODE, M32, MX>;
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const long long ldb = F8 ? ldx : 2 * ldx;
  hipLaunchKernelGGL((kmeans_assign_rr<DP, CT, F8, MODE, M32, MX>), dim3(grid), dim3(kThreads), lds, st,
                     (const unsigned char*)X, n, ldb, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part, hist,
                     rank, dout, ext, dbg);
  return cml_status();
}

template <int MODE>
inline int dispatch_mode(int Dp, int ct, bool f8, const void* X, long long n, long long ldx, const u16* C,
                         long long ldc, int kc, int kp, const float* cnorm, const float* xnorm, int* labels,
                         float* best, double* cost_part, int* hist, int* rank, DeltaOut dout, Ext ext, int grid,
                         int dbg, hipStream_t st) {
  const bool m32 = use_m32(Dp, ct, f8);
  if (use_mx(Dp, f8, m32)) {
#define CML_RX(D, T)                                                                                                \
  if (Dp == D && ct == T)                                                                                           \
  return launch<D, T, true, MODE, false, true>(X, n, ldx, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part,   \
                                               hist, rank, dout, ext, grid, dbg, st)
    CML_RX(256, 1); CML_RX(256, 2); CML_RX(256, 3); CML_RX(256, 4);
    CML_RX(512, 1); CML_RX(512, 2);
#undef CML_RX
    return (int)hipErrorInvalidValue;
  }
#define CML_RR(D, T, F, M)                                                                                          \
  if (Dp == D && ct == T && f8 == F && m32 == M)                                                                    \
  return launch<D, T, F, MODE, M>(X, n, ldx, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part, hist, rank,    \
                                  dout, ext, grid, dbg, st)
  CML_RR(128, 1, false, false); CML_RR(128, 2, false, false); CML_RR(128, 3, false, false);
  CML_RR(128, 4, false, false); CML_RR(128, 5, false, false);
  CML_RR(256, 1, false, false); CML_RR(256, 2, false, false); CML_RR(256, 3, false, false);
  CML_RR(256, 4, false, false); CML_RR(256, 5, false, false);
  CML_RR(512, 1, false, false); CML_RR(512, 2, false, false);
  CML_RR(256, 1, true, false); CML_RR(256, 2, true, false); CML_RR(256, 3, true, false); CML_RR(256, 4, true, false);
  CML_RR(512, 1, true, false); CML_RR(512, 2, true, false);
  CML_RR(128, 2, false, true); CML_RR(128, 4, false, true);
  CML_RR(256, 2, false, true); CML_RR(256, 4, false, true);
  CML_RR(256, 2, true, true); CML_RR(256, 4, true, true);
  CML_RR(512, 2, true, true);
#undef CML_RR
  return (int)hipErrorInvalidValue;
}

inline int dispatch(int mode, int Dp, int ct, bool f8, const void* X, long long n, long long ldx, const u16* C,
                    long long ldc, int kc, int kp, const float* cnorm, const float* xnorm, int* labels, float* best,
                    double* cost_part, int* hist, int* rank, DeltaOut dout, Ext ext, int grid, int dbg,
                    hipStream_t st) {
  switch (mode) {
    case 0: return dispatch_mode<0>(Dp, ct, f8, X, n, ldx, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part,
                                    hist, rank, dout, ext, grid, dbg, st);
    case 1: return dispatch_mode<1>(Dp, ct, f8, X, n, ldx, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part,
                                    hist, rank, dout, ext, grid, dbg, st);
    case 2: return dispatch_mode<2>(Dp, ct, f8, X, n, ldx, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part,
                                    hist, rank, dout, ext, grid, dbg, st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace rr
