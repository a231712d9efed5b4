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
//   * X streams through a 4-slot LDS ring of 32-KiB tiles filled by LDS-DMA
//     (global_load_lds_dwordx4) issued by 2 DMA waves that do nothing else, so the loads never stall
//     a computing wave and ~96 KiB per CU stay in flight;
//   * every compute wave reads each X tile from LDS (B operand of v_mfma_f32_16x16x32_bf16, one
//     ds_read_b128 per 16 rows x 32 k) against its own centres; its per-row minimum key over its
//     centres goes to an exchange buffer;
//   * 2 FINALIZE waves take the minimum over the 4 compute waves one tile later and run the
//     epilogue K9 runs inline (labels, cost, label-change lists, counting-sort ranks).
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
constexpr int kRedStride = 17;  // dwords per row of the key exchange: 16 keys + 1 pad (conflict-free writes)
constexpr int kNS = 4;          // X ring slots

template <int DP, bool F8 = false>
struct Geo {
  static constexpr int KS = DP / 32;            // MFMA k-steps per row
  static constexpr int ROWB = F8 ? DP : DP * 2; // bytes per row (bf16, or OCP e4m3fn bytes)
  static constexpr int TR = 32768 / ROWB;       // rows per tile (32 KiB of X)
  static constexpr int NSUB = TR / 16;          // 16-row MFMA sub-tiles per tile
  static constexpr int SLOT = TR * ROWB;        // 32 KiB
  static constexpr int NTR = kNS + 1;           // trailer ring entries
  static constexpr int PIECES = SLOT / 1024;    // 1-KiB DMA pieces per tile (32)
  static constexpr int LPR = ROWB / 16;         // lanes (16-B chunks) per row in a piece
  static constexpr int TRAIL_Q = TR >= 64 ? TR / 64 : 1;  // dword DMA instructions per trailer array
  static constexpr int CNT = PIECES / 2 + TRAIL_Q;        // DMA instructions per DMA wave per tile
  static constexpr int TRB = TR * 8;            // trailer entry bytes (norms f32 + labels i32)
  static constexpr int RED = TR * kRedStride * 4;
};

// LDS layout (bytes): [X ring NS*SLOT | trailers NTR*TRB | keys 2*RED | hist kp ints | misc 64 B]
template <int DP, bool F8 = false>
__host__ __device__ constexpr long long lds_bytes(int kp) {
  using G = Geo<DP, F8>;
  return (long long)kNS * G::SLOT + (long long)G::NTR * G::TRB + 2LL * G::RED + 4LL * ((kp + 3) & ~3) + 64;
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

// ldx in BYTES; rows are 16-B aligned.
template <int DP, bool F8>
__device__ __forceinline__ void issue_tile(const unsigned char* __restrict__ X, long long ldx, long long n,
                                           const float* __restrict__ xnorm, const int* __restrict__ labels,
                                           long long tile, int slot, int tr, int dw, int lane,
                                           unsigned char* smem) {
  using G = Geo<DP, F8>;
  const long long row0 = tile * G::TR;
  unsigned char* sdst = smem + slot * G::SLOT;
#pragma unroll
  for (int q = 0; q < G::PIECES / 2; ++q) {
    const int p = dw * (G::PIECES / 2) + q;
    const int R = p * (1024 / G::ROWB) + lane / G::LPR;  // row within the tile
    const int pos = lane % G::LPR;                       // LDS chunk position in the row
    const int gch = pos ^ (R & 15);                      // global chunk stored there
    long long grow = row0 + R;
    grow = grow < n ? grow : n - 1;                      // rows past n: any valid row (discarded)
    glds16(X + grow * ldx + 16 * gch, sdst + p * 1024);
  }
  unsigned char* tdst = smem + kNS * G::SLOT + tr * G::TRB + (dw ? G::TR * 4 : 0);
#pragma unroll
  for (int q = 0; q < G::TRAIL_Q; ++q) {
    const int R = q * 64 + lane;
    long long grow = row0 + R;
    grow = grow < n ? grow : n - 1;
    if (R < G::TR) {
      if (dw == 0) glds4(xnorm + grow, tdst + q * 256);
      else glds4(labels + grow, tdst + q * 256);
    }
  }
}

// F8: X rows are OCP e4m3fn bytes (SURVEY config 5). They travel through the ring as bytes (half the
// HBM and LDS traffic) and every compute wave widens its fragments with v_cvt_scalef32_pk_bf16_fp8
// (exact: e4m3 values are a subset of bf16); one 16-B read then covers TWO k-steps, step 2v+h of lane
// (r, g) holding k = 64v + 16g + 8h + j, and the centre fragments follow the same k order.
template <int DP, int CT, bool F8>
__global__ __launch_bounds__(kThreads, 1) void kmeans_assign_rr(
    const unsigned char* __restrict__ X, long long n, long long ldx, const u16* __restrict__ C, long long ldc, int kc,
    int kp, const float* __restrict__ cnorm, const float* __restrict__ xnorm, int* __restrict__ labels,
    float* __restrict__ best_out, double* __restrict__ cost_part, int* __restrict__ hist_out,
    int* __restrict__ rank_out, DeltaOut dout, int dbg) {
  // dbg (ablation only, 0 in production): bit 0 DMA waves issue nothing, bit 1 compute waves skip
  // their MFMAs/keys, bit 2 finalize waves skip the epilogue
  using G = Geo<DP, F8>;
  constexpr int KS = G::KS;
  constexpr int CPW = CT * 16;  // centres per compute wave
  constexpr int TAGB = 2 + (CT > 1) + (CT > 2) + (CT > 4);
  constexpr int TAGM = (1 << TAGB) - 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* trail = smem + kNS * G::SLOT;
  int* red = reinterpret_cast<int*>(trail + G::NTR * G::TRB);
  int* hist = red + 2 * G::TR * kRedStride;
  int* misc = hist + ((kp + 3) & ~3);  // [0] change counter, [2..5] two f64 cost partials
  double* cost_sh = reinterpret_cast<double*>(misc + 2);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long ntiles = (n + G::TR - 1) / G::TR;
  const long long nt = ntiles > blockIdx.x ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const bool ranking = rank_out != nullptr;
  auto tile_of = [&](long long j) { return (long long)blockIdx.x + j * gridDim.x; };

  if (wave < kCompute) {
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
      const unsigned char* xs = smem + (int)(j % kNS) * G::SLOT;
      const float* tn = reinterpret_cast<const float*>(trail + (int)(j % G::NTR) * G::TRB);
      int* kred = red + (int)(j & 1) * G::TR * kRedStride;
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
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int t = u / UPS, v = u % UPS, cur = t & 1, prv = cur ^ 1;
        if (u + PF < NU) xr[(u + PF) % (PF + 1)] = *reinterpret_cast<const uint4*>(xaddr(u + PF));
        bf16x8 xb[SPU];
        if constexpr (F8) {
          typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
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
          if (s == 0) key[cur] = 0x7fffffff;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
            acc[cur][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                creg[ct][s], xb[h], s == 0 ? (c4[ct] + xnv[t]) : acc[cur][ct], 0, 0, 0);
          if (t > 0) {  // keys of the previous sub-tile, spread over this one's k-steps
#pragma unroll
            for (int e = (s * CT * 4) / KS; e < ((s + 1) * CT * 4) / KS; ++e) {
              const int ct = e >> 2, i = e & 3;
              const int kv = (__float_as_int(acc[prv][ct][i]) & ~TAGM) | (ct << 2 | i);
              key[prv] = kv < key[prv] ? kv : key[prv];
            }
            if (s == KS - 1) kred[(16 * (t - 1) + r) * kRedStride + wave * 4 + g] = key[prv];
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
          key[cur] = kv < key[cur] ? kv : key[cur];
        }
        kred[(16 * t + r) * kRedStride + wave * 4 + g] = key[cur];
      }
      wait_lgkm0();
      barrier();  // B(j)
    }
  } else if (wave < kCompute + 2) {
    // ------------------------------------------------------------------ LDS-DMA waves
    const int dw = wave - kCompute;
    for (long long j = 0; j < kNS - 1 && j < nt && !(dbg & 1); ++j)
      issue_tile<DP, F8>(X, ldx, n, xnorm, labels, tile_of(j), (int)j, (int)j, dw, lane, smem);
    if (nt >= kNS - 1) wait_vm<(kNS - 2) * G::CNT>();
    else wait_vm<0>();
    barrier();  // B(-1)
    for (long long j = 0; j < nt; ++j) {
      const long long jn = j + kNS - 1;
      if (jn < nt && !(dbg & 1)) {
        issue_tile<DP, F8>(X, ldx, n, xnorm, labels, tile_of(jn), (int)(jn % kNS), (int)(jn % G::NTR), dw, lane,
                       smem);
        wait_vm<(kNS - 2) * G::CNT>();  // tile j+1 has landed; j+2 .. j+NS-1 stay in flight
      } else {
        wait_vm<0>();
      }
      barrier();  // B(j)
    }
  } else {
    // ------------------------------------------------------------------ finalize waves
    const int fw = wave - kCompute - 2;
    constexpr int RPF = G::TR / 2;  // rows per finalize wave
    if (fw == 0) {
      for (int i = lane; i < kp; i += 64) hist[i] = 0;
      if (lane == 0) misc[0] = 0;
    }
    double cost = 0.0;
    // LPR_F lanes per row, each taking 16 / LPR_F of the 16 (wave, lane-group) keys; keys are loaded
    // in one batch and reduced branch-free on a 64-bit (value, centre index) composite
    constexpr int LPR_F = 64 / RPF;
    constexpr int QPL = 16 / LPR_F;
    const int rl = lane % RPF, part = lane / RPF;
    auto finalize = [&](long long j) {
      const int* kr = red + (int)(j & 1) * G::TR * kRedStride;
      const unsigned char* te = trail + (int)(j % G::NTR) * G::TRB;
      const int R = fw * RPF + rl;
      const long long row = tile_of(j) * G::TR + R;
      int kv[QPL];
#pragma unroll
      for (int q = 0; q < QPL; ++q) kv[q] = kr[R * kRedStride + part * QPL + q];
      const int old = reinterpret_cast<const int*>(te + G::TR * 4)[R];
      unsigned long long best = ~0ull;
#pragma unroll
      for (int q = 0; q < QPL; ++q) {  // qq = w*4 + g: centres w*CPW + ct*16 + 4g + i
        const int qq = part * QPL + q;
        const int tag = kv[q] & TAGM;
        const unsigned idx = (unsigned)((qq >> 2) * CPW + (qq & 3) * 4 + (tag >> 2) * 16 + (tag & 3));
        const unsigned long long c = ((unsigned long long)((unsigned)(kv[q] & ~TAGM) ^ 0x80000000u) << 32) | idx;
        best = c < best ? c : best;
      }
#pragma unroll
      for (int o = RPF; o < 64; o <<= 1) {
        const unsigned long long ob = __shfl_xor(best, o, 64);
        best = ob < best ? ob : best;
      }
      const int bi = (int)(best & 0xffffffffu);
      const float dist = fmaxf(__int_as_float((int)((unsigned)(best >> 32) ^ 0x80000000u)), 0.f);
      const bool mine = part == 0 && row < n;
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
        if (ranking) rank_out[row] = atomicAdd(hist + bi, 1);
      }
    };
    wait_lgkm0();
    barrier();  // B(-1)
    for (long long j = 0; j < nt; ++j) {
      if (j > 0 && !(dbg & 4)) finalize(j - 1);
      wait_lgkm0();
      barrier();  // B(j)
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
inline int plan_ct(int Dp, int kc, bool f8 = false) {
  if (Dp != 128 && Dp != 256 && Dp != 512) return 0;
  if (f8 && Dp < 256) return 0;
  const int ct = (kc + 63) / 64;
  if (ct > 4) return 0;  // CT = 8 spills at 256 VGPRs
  const int c = ct <= 1 ? 1 : (ct <= 2 ? 2 : 4);
  if (c * (Dp / 32) > 32) return 0;
  return c;
}

inline long long lds_for(int Dp, int kp, bool f8 = false) {
  if (f8) {
    switch (Dp) {
      case 256: return lds_bytes<256, true>(kp);
      case 512: return lds_bytes<512, true>(kp);
      default: return 0;
    }
  }
  switch (Dp) {
    case 128: return lds_bytes<128>(kp);
    case 256: return lds_bytes<256>(kp);
    case 512: return lds_bytes<512>(kp);
    default: return 0;
  }
}

inline int tile_rows(int Dp, bool f8 = false) { return Dp > 0 ? 32768 / ((f8 ? 1 : 2) * Dp) : 0; }

// X: bf16 rows (ldx elements) or, with f8, e4m3fn rows (ldx bytes).
template <int DP, int CT, bool F8>
int launch(const void* X, long long n, long long ldx, const u16* C, long long ldc, int kc, int kp, const float* cnorm,
           const float* xnorm, int* labels, float* best, double* cost_part, int* hist, int* rank, DeltaOut dout,
           int grid, int dbg, hipStream_t st) {
  const size_t lds = (size_t)lds_bytes<DP, F8>(kp);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const void* fn = (const void*)kmeans_assign_rr<DP, CT, F8>;
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const long long ldb = F8 ? ldx : 2 * ldx;
  hipLaunchKernelGGL((kmeans_assign_rr<DP, CT, F8>), dim3(grid), dim3(kThreads), lds, st,
                     (const unsigned char*)X, n, ldb, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part, hist,
                     rank, dout, dbg);
  return cml_status();
}

inline int dispatch(int Dp, int ct, bool f8, const void* X, long long n, long long ldx, const u16* C, long long ldc,
                    int kc, int kp, const float* cnorm, const float* xnorm, int* labels, float* best,
                    double* cost_part, int* hist, int* rank, DeltaOut dout, int grid, int dbg, hipStream_t st) {
#define CML_RR(D, T, F)                                                                                             \
  if (Dp == D && ct == T && f8 == F)                                                                                \
  return launch<D, T, F>(X, n, ldx, C, ldc, kc, kp, cnorm, xnorm, labels, best, cost_part, hist, rank, dout, grid, \
                         dbg, st)
  CML_RR(128, 1, false); CML_RR(128, 2, false); CML_RR(128, 4, false);
  CML_RR(256, 1, false); CML_RR(256, 2, false); CML_RR(256, 4, false);
  CML_RR(512, 1, false); CML_RR(512, 2, false);
  CML_RR(256, 1, true); CML_RR(256, 2, true); CML_RR(256, 4, true);
  CML_RR(512, 1, true); CML_RR(512, 2, true);
#undef CML_RR
  return (int)hipErrorInvalidValue;
}

}  // namespace rr
