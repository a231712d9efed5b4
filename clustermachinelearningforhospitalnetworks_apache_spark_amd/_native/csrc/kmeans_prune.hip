// K9p: bounds pass of the exact pruned Lloyd step (models/kmeans.py ``LloydEngine(prune=True)``).
//
// Spark's EuclideanDistanceMeasure.findClosest (mllib/clustering/DistanceMeasure.scala) skips a
// centre when the triangle inequality proves it cannot be the closest one (centre-to-centre
// distances precomputed once per iteration). This is the same idea carried across iterations
// (Hamerly's upper bound + half the distance to the nearest other centre):
//
//   ub[i] >= ||x_i - c_{a(i)}||  (a(i) = current label), lb[i] <= min_{j != a(i)} ||x_i - c_j||,
//   kept per row in HBM (8 B / row);
//   after a centre update:  ub[i] += drift[a(i)], lb[i] -= max_{j != a(i)} drift[j]
//   (drift[j] = ||c_j_new - c_j_old||; ub rounded up, lb rounded down);
//   the label provably stays if ub[i] <= thr[a(i)] (thr[j] = half the distance from c_j to its
//   nearest other centre less a slack) or ub[i] <= lb[i] - c2 / lb[i]. Both slacks keep the
//   squared-distance gap above twice the f32 error of the full assign's MFMA distance, so the full
//   assign would pick the same centre. Such rows are not read at all; every other row is appended
//   to `cand` and re-assigned against all centres by K9 on a gathered copy.
//
// One pass reads 12 B and writes 8 B per row (100M rows: 2 GB, ~0.35 ms at HBM speed) instead of
// the 51 GB X stream of the full assign. Rows are read 4 per lane with 16-byte loads; each block
// compacts its candidates through one LDS scan and one global atomic (the candidate ORDER depends
// on block scheduling, the candidate SET does not; everything downstream is per-row or an exact
// f64 sum, so results do not depend on it).
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kIters = 4;  // 4 x 4 rows per lane: 4096 rows per block (8192 for the bounds pass)
// The bounds pass runs 512-thread workgroups: each takes one slot of the candidate list with a device-scope
// atomic on ONE counter (and one completion atomic for the folded gate), and those same-address atomics
// serialise at the L2 — with 256-thread workgroups (4096 rows each) they bounded the pass at ~2-3 TB/s.
// 1024-thread workgroups went the other way: at 78 VGPRs (6 waves per SIMD) only one fits a CU, so 100M rows
// ran in three rounds of 256 blocks with a ragged tail; 512 threads fit three per CU (same-box A/B,
// profiles/r5/ab_bounds_wg: 346 -> 300 us per 100M-row pass, headline fit -0.7 ms, 12.5M-row shard unchanged).
constexpr int kBoundsThreads = 512;

// Offset form (cum != null): the stored values are us = ub - cu[a] and ls = lb + cl[a] against the
// per-centre cumulative drifts cu[j] = Σ drift_j and cl[j] = Σ (largest drift of a centre other than
// j), both rounded up as they accumulate (kmeans_centre_stats2_kernel). The effective bounds are
// us + cu[a] (rounded up) and ls - cl[a] (rounded down), so a row whose label holds is only READ — the
// pass drops its 8 B/row of bound writes — and the writers (K9r epilogue, the seeded accumulate) store
// the offsets of the bounds they compute.
__device__ __forceinline__ bool bound_lazy(int a, float us, float ls, const float* cu, const float* cl,
                                           const float* st, float c2) {
  const float ca = cu[a], la = cl[a];
  const float u = (us + ca) + 1e-6f * (fabsf(us) + ca);                     // rounded up (inf stays inf)
  const float w = fmaxf((ls - la) - 1e-6f * (fabsf(ls) + la), 0.f);        // rounded down
  const float lt = w > 0.f ? (w - c2 / w) * (1.0f - 1e-6f) : -1.f;
  return u <= st[a] || u <= lt;
}

// Moves one row's bounds to the new centres; true when they still prove its label.
__device__ __forceinline__ bool bound_step(int a, float& u, float& w, const float* sd, const float* st, float dm1,
                                           float dm2, int jm, float c2) {
  u = (u + sd[a]) * (1.0f + 2.4e-7f);                           // rounded up (inf stays inf)
  w = fmaxf((w - (a == jm ? dm2 : dm1)) * (1.0f - 2.4e-7f), 0.f);  // rounded down
  const float lt = w > 0.f ? (w - c2 / w) * (1.0f - 1e-6f) : -1.f;
  return u <= st[a] || u <= lt;
}

// The pruned step's gate (kmeans_prune_gate_kernel's body): one thread.
__device__ __forceinline__ void prune_gate_body(int* __restrict__ count, long long cap, const int* __restrict__ flags,
                                                int* __restrict__ mode, int* __restrict__ backoff, int nback,
                                                int* __restrict__ mode_host = nullptr) {
  if (flags[1] != 0) {
    mode[0] = 0;
    mode[1] = 0;
    *count = 0;
    return;
  }
  // the count is only ever changed by device-scope atomics: read it the same way (no stale cached copy)
  const int c = __hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (backoff != nullptr && flags[0] == 0 && (long long)c > cap) *backoff = nback;
  const int full = (flags[0] != 0 || (long long)c > cap) ? 1 : 0;
  mode[0] = full;
  mode[1] = full ? 0 : c;
  // mode_host: pinned host memory the host reads without a synchronisation (a lagged hint of the regime:
  // models/kmeans.py _pdev_pre enqueues the full-accumulate launches while full passes are being picked)
  if (mode_host != nullptr) mode_host[0] = full;
}

// Gate folded into the bounds pass (one launch less per step): with gmode != null the workgroup that
// finishes last (device-scope counter gdone) runs the gate on the final count; a skipped pass (force /
// done) runs it in workgroup 0 at once.
struct GateArgs {
  int* mode;
  long long cap;
  int* backoff;
  int nback;
  int* done;
  int* mode_host = nullptr;
};

__global__ __launch_bounds__(kBoundsThreads) void kmeans_prune_bounds_kernel(const int* __restrict__ lab,
                                                                       float* __restrict__ ub,
                                                                       float* __restrict__ lb,
                                                                       const float* __restrict__ drift,
                                                                       const float* __restrict__ dmax,
                                                                       const float* __restrict__ thr,
                                                                       const float* __restrict__ c2p, int k,
                                                                       long long n, int* __restrict__ cand,
                                                                       int* __restrict__ count,
                                                                       const float* __restrict__ xn,
                                                                       int* __restrict__ cand_lab,
                                                                       float* __restrict__ cand_xn,
                                                                       const int* __restrict__ skip,
                                                                       long long cap, const float* __restrict__ cum,
                                                                       GateArgs gate) {
  // skip = the step's flags {force, done}: bounds invalid this step (full pass instead), or the fit has
  // converged and the step is a frozen no-op (kmeans_prune_gate_kernel)
  if (skip != nullptr && (skip[0] != 0 || skip[1] != 0)) {
    if (gate.mode != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
      prune_gate_body(count, gate.cap, skip, gate.mode, gate.backoff, gate.nback, gate.mode_host);
    return;
  }
  extern __shared__ __align__(16) unsigned char smem[];
  const float c2 = *c2p;
  float* sd = reinterpret_cast<float*>(smem);  // [k] drift
  float* st = sd + k;                          // [k] threshold
  float* scu = st + k;                         // [k] cumulative drifts (offset form)
  float* scl = scu + k;                        // [k]
  __shared__ int wsum[kBoundsThreads / 64];
  __shared__ int base;
  const bool lazy = cum != nullptr;
  for (int i = threadIdx.x; i < k; i += kBoundsThreads) {
    sd[i] = drift[i];
    st[i] = thr[i];
    if (lazy) {
      scu[i] = cum[i];
      scl[i] = cum[k + i];
    }
  }
  __syncthreads();
  // largest drift, second largest, index of the largest: the lower bound moves by the largest drift
  // of any OTHER centre
  const float dm1 = dmax[0], dm2 = dmax[1];
  const int jm = (int)dmax[2];
  const long long blk0 = (long long)blockIdx.x * kBoundsThreads * kIters * 4;
  unsigned mask = 0;  // bit it*4+j: row blk0 + (it*kBoundsThreads + tid)*4 + j is a candidate
  if (lazy) {
    // read-only: rows whose label holds keep their stored offsets. All kIters groups' loads are issued
    // before any test (48 B in flight per lane; one group at a time ran the pass at 3.3 TB/s)
    int4 L[kIters];
    float4 U[kIters], W[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const long long r0 = blk0 + ((long long)it * kBoundsThreads + threadIdx.x) * 4;
      if (r0 + 3 < n) {
        L[it] = *reinterpret_cast<const int4*>(lab + r0);
        U[it] = *reinterpret_cast<const float4*>(ub + r0);
        W[it] = *reinterpret_cast<const float4*>(lb + r0);
      }
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const long long r0 = blk0 + ((long long)it * kBoundsThreads + threadIdx.x) * 4;
      if (r0 >= n) break;
      if (r0 + 3 < n) {
        const int ls[4] = {L[it].x, L[it].y, L[it].z, L[it].w};
        const float us[4] = {U[it].x, U[it].y, U[it].z, U[it].w};
        const float ws[4] = {W[it].x, W[it].y, W[it].z, W[it].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (!bound_lazy(ls[j], us[j], ws[j], scu, scl, st, c2)) mask |= 1u << (it * 4 + j);
      } else {
        for (int j = 0; j < 4 && r0 + j < n; ++j)
          if (!bound_lazy(lab[r0 + j], ub[r0 + j], lb[r0 + j], scu, scl, st, c2)) mask |= 1u << (it * 4 + j);
      }
    }
  }
#pragma unroll
  for (int it = 0; it < kIters && !lazy; ++it) {
    const long long r0 = blk0 + ((long long)it * kBoundsThreads + threadIdx.x) * 4;
    if (r0 >= n) break;
    if (r0 + 3 < n) {
      const int4 l = *reinterpret_cast<const int4*>(lab + r0);
      const float4 u = *reinterpret_cast<const float4*>(ub + r0);
      const float4 w = *reinterpret_cast<const float4*>(lb + r0);
      const int ls[4] = {l.x, l.y, l.z, l.w};
      float us[4] = {u.x, u.y, u.z, u.w};
      float ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (!bound_step(ls[j], us[j], ws[j], sd, st, dm1, dm2, jm, c2)) mask |= 1u << (it * 4 + j);
      *reinterpret_cast<float4*>(ub + r0) = make_float4(us[0], us[1], us[2], us[3]);
      *reinterpret_cast<float4*>(lb + r0) = make_float4(ws[0], ws[1], ws[2], ws[3]);
    } else {
      for (int j = 0; j < 4 && r0 + j < n; ++j) {
        float u = ub[r0 + j], w = lb[r0 + j];
        if (!bound_step(lab[r0 + j], u, w, sd, st, dm1, dm2, jm, c2)) mask |= 1u << (it * 4 + j);
        ub[r0 + j] = u;
        lb[r0 + j] = w;
      }
    }
  }
  // block-wide exclusive scan of the per-lane candidate counts
  const int mine = __popc(mask);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kBoundsThreads / 64; ++w) t += wsum[w];
    base = t ? atomicAdd(count, t) : 0;
  }
  __syncthreads();
  int off = base + incl - mine;
  for (int w = 0; w < wave; ++w) off += wsum[w];
  while (mask) {
    const int b = __ffs(mask) - 1;
    mask &= mask - 1;
    const int row = (int)(blk0 + ((long long)(b >> 2) * kBoundsThreads + threadIdx.x) * 4 + (b & 3));
    if (off >= cap) break;  // list full: *count still gets every candidate (the step then runs in full)
    cand[off] = row;
    if (cand_lab != nullptr) {  // compacted label / norm of the candidate (trailer of the K9r mode-2 pass)
      cand_lab[off] = lab[row];
      cand_xn[off] = xn[row];
    }
    ++off;
  }
  if (gate.mode != nullptr) {
    // no fence: the gate reads only the count, which every block changed by an atomic whose result it
    // waited for (base above) before this completion atomic — device-scope atomics in issue order
    if (threadIdx.x == 0 && atomicAdd(gate.done, 1) == (int)gridDim.x - 1) {
      prune_gate_body(count, gate.cap, skip, gate.mode, gate.backoff, gate.nback, gate.mode_host);
      __hip_atomic_store(gate.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Pruned-step mode: full pass (1) when the bounds are invalid (flags[0], force) or more than cap rows
// are candidates, else the candidate pass (0); mode[1] keeps the candidate count. flags[1] (done) set by
// kmeans_converge_latch_kernel once every centre moved <= tol: the step is frozen — candidate pass over
// 0 rows, so no label changes, the sums and therefore the centres stay bit for bit — which lets the host
// enqueue steps ahead and read the convergence flag lagged (no per-step host sync). One thread.
__global__ void kmeans_prune_gate_kernel(int* __restrict__ count, long long cap, const int* __restrict__ flags,
                                         int* __restrict__ mode, int* __restrict__ backoff, int nback) {
  if (flags[1] != 0) {
    mode[0] = 0;
    mode[1] = 0;
    *count = 0;
    return;
  }
  // bounds that stopped pruning (more than cap candidates) stay off for the next nback steps: those go
  // straight to the full pass, which skips the bounds pass and its compaction (kmeans_centre_stats2)
  if (backoff != nullptr && flags[0] == 0 && (long long)*count > cap) *backoff = nback;
  const int full = (flags[0] != 0 || (long long)*count > cap) ? 1 : 0;
  mode[0] = full;
  mode[1] = full ? 0 : *count;  // re-assigned rows of a candidate pass (stats; count is reset later)
}

// done |= (every shift2[j] <= lim): Spark's convergence rule (all centres moved at most tol), decided
// on the device and latched. One workgroup.
__global__ __launch_bounds__(256) void kmeans_converge_latch_kernel(const double* __restrict__ shift2, int k,
                                                                     double lim, int* __restrict__ flags) {
  __shared__ int any_moved;
  if (threadIdx.x == 0) any_moved = 0;
  __syncthreads();
  int moved = 0;
  for (int j = threadIdx.x; j < k; j += 256) moved |= !(shift2[j] <= lim);  // NaN counts as moved
  if (moved) any_moved = 1;
  __syncthreads();
  if (threadIdx.x == 0 && !any_moved) flags[1] = 1;
}

// dst <- src (n 32-bit words) unless flags[1] (done) is set: the centres of the last live step's
// assignment survive the frozen steps (training cost); dst_always (may be null) <- src every step (the
// pruned step's cb_old: one launch for both copies).
__global__ __launch_bounds__(256) void kmeans_cond_copy_kernel(unsigned* __restrict__ dst,
                                                               const unsigned* __restrict__ src, long long n,
                                                               const int* __restrict__ flags,
                                                               unsigned* __restrict__ dst_always) {
  const bool live = flags[1] == 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const unsigned v = src[i];
    if (dst_always != nullptr) dst_always[i] = v;
    if (live) dst[i] = v;
  }
}

// Centre statistics of the pruned step, part 1 (one workgroup per centre j, over the bf16 centres
// the assign compares against, in f64): ||c_j||², drift_j = |c_j - old_j| rounded up, and
// half_j = half the distance from c_j to its nearest other centre.
__global__ __launch_bounds__(256) void kmeans_centre_stats_kernel(const u16* __restrict__ cb,
                                                                  const u16* __restrict__ cb_old, long long ldc, int k,
                                                                  int d, double* __restrict__ cn,
                                                                  float* __restrict__ drift,
                                                                  double* __restrict__ half) {
  extern __shared__ __align__(16) unsigned char smem[];
  double* cj = reinterpret_cast<double*>(smem);  // [d]
  __shared__ double red[256];
  __shared__ double red2[256];
  const int j = blockIdx.x, tid = threadIdx.x;
  double nrm = 0.0, dr = 0.0;
  for (int t = tid; t < d; t += 256) {
    const double v = (double)bf16_to_f32(cb[(long long)j * ldc + t]);
    cj[t] = v;
    nrm += v * v;
    if (cb_old != nullptr) {
      const double o = v - (double)bf16_to_f32(cb_old[(long long)j * ldc + t]);
      dr += o * o;
    }
  }
  red[tid] = nrm;
  red2[tid] = dr;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[tid] += red[tid + o];
      red2[tid] += red2[tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    cn[j] = red[0];
    if (cb_old != nullptr) drift[j] = (float)(sqrt(red2[0]) * (1.0 + 1e-6));
  }
  __syncthreads();
  // nearest other centre: thread t walks centres t, t+256, ... (each distance summed over d in f64)
  double best = __builtin_huge_val();
  for (int i = tid; i < k; i += 256) {
    if (i == j) continue;
    double s = 0.0;
    for (int t = 0; t < d; ++t) {
      const double e = (double)bf16_to_f32(cb[(long long)i * ldc + t]) - cj[t];
      s += e * e;
    }
    best = s < best ? s : best;
  }
  red[tid] = best;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = red[tid + o] < red[tid] ? red[tid + o] : red[tid];
    __syncthreads();
  }
  if (tid == 0) half[j] = 0.5 * sqrt(red[0]);
}

// Part 2 (one workgroup): mc = max ||c||², c2 = 2·tau·(mx + mc), thr_j = (half_j - tau·(mx + mc) /
// (2 half_j))·(1 - 1e-6) (or -inf / +inf), dmax = {largest drift, second largest, its index};
// resets the candidate count and the force flag for the next step.
__global__ __launch_bounds__(256) void kmeans_centre_stats2_kernel(const double* __restrict__ cn,
                                                                   const double* __restrict__ half,
                                                                   const float* __restrict__ drift, int k,
                                                                   const float* __restrict__ mx, float tau,
                                                                   int have_drift, float* __restrict__ thr,
                                                                   float* __restrict__ dmax, float* __restrict__ mc,
                                                                   float* __restrict__ c2, int* __restrict__ count,
                                                                   int* __restrict__ force, float* __restrict__ cum,
                                                                   int* __restrict__ backoff) {
  __shared__ double smax[256];
  __shared__ float sdm[3];
  __shared__ float d1[256], d2[256];
  __shared__ int i1[256];
  // the first 256 threads of the workgroup do the work (callers run 256 or more threads; all reach the barriers)
  const int tid = threadIdx.x;
  const bool act = tid < 256;
  double m = 0.0;
  float a = -1.f, b = -1.f;
  int ia = 0;
  for (int j = tid; act && j < k; j += 256) {
    m = cn[j] > m ? cn[j] : m;
    if (have_drift) {
      const float v = drift[j];
      if (v > a) { b = a; a = v; ia = j; }
      else if (v > b) { b = v; }
    }
  }
  if (act) {
    smax[tid] = m;
    d1[tid] = a;
    d2[tid] = b;
    i1[tid] = ia;
  }
  __syncthreads();
  if (tid == 0) {
    double mm = 0.0;
    float ta = -1.f, tb = -1.f;
    int ti = 0;
    for (int t = 0; t < 256; ++t) {
      mm = smax[t] > mm ? smax[t] : mm;
      // merge (d1[t], d2[t]) into (ta, tb): lowest index wins ties of the largest drift
      if (d1[t] > ta) { tb = ta > d2[t] ? ta : d2[t]; ta = d1[t]; ti = i1[t]; }
      else { const float c = d1[t]; tb = c > tb ? c : tb; }
    }
    smax[0] = mm;
    const float mcf = (float)mm;
    *mc = mcf;
    *c2 = (float)(2.0 * (double)tau * ((double)*mx + mm));
    if (have_drift) {
      dmax[0] = ta < 0.f ? 0.f : ta;
      dmax[1] = tb < 0.f ? 0.f : tb;
      dmax[2] = (float)ti;
    }
    sdm[0] = ta < 0.f ? 0.f : ta;
    sdm[1] = tb < 0.f ? 0.f : tb;
    sdm[2] = (float)ti;
    *count = 0;
    // a backed-off pruned step forces the next one full (its bounds pass is skipped)
    const int bo = backoff != nullptr ? *backoff : 0;
    *force = bo > 0 ? 1 : 0;
    if (bo > 0) *backoff = bo - 1;
  }
  __syncthreads();
  const double sl = (double)tau * ((double)*mx + smax[0]);
  for (int j = tid; act && j < k; j += 256) {
    float t;
    if (k == 1) t = __builtin_huge_valf();
    else if (half[j] > 0.0) t = (float)((half[j] - sl / (2.0 * half[j])) * (1.0 - 1e-6));
    else t = -__builtin_huge_valf();
    thr[j] = t;
    if (have_drift && cum != nullptr) {  // cumulative drifts of the offset-form bounds, rounded up
      cum[j] = (cum[j] + drift[j]) * (1.0f + 2.4e-7f);
      cum[k + j] = (cum[k + j] + (j == (int)sdm[2] ? sdm[1] : sdm[0])) * (1.0f + 2.4e-7f);
    }
  }
}

// Lower bounds of the candidate rows from their GEMM block dist[r][j] = |c_j|² - 2 x_r·c_j (f32, k
// columns): lb[r] = sqrt(max(min_{j != lab[r]} dist[r][j] + xn[r] - tau·(xn[r] + mc), 0)) rounded down.
// 16 lanes per row read its k floats as 16-byte loads (one contiguous 1 KiB row at k = 256), then a
// 4-step xor-shuffle min; one launch replaces the mask / row-min / bound elementwise passes.
__global__ __launch_bounds__(kThreads) void kmeans_prune_lower_kernel(const float* __restrict__ dist, int k,
                                                                      const int* __restrict__ lab,
                                                                      const float* __restrict__ xn, float mc,
                                                                      float tau, long long m,
                                                                      float* __restrict__ lb) {
  const long long r = (long long)blockIdx.x * (kThreads / 16) + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  float best = __builtin_huge_valf();
  const int a = r < m ? lab[r] : -1;
  if (r < m) {
    const float4* row = reinterpret_cast<const float4*>(dist + r * (long long)k);
    for (int c4 = sub; c4 < (k >> 2); c4 += 16) {
      const float4 v = row[c4];
      const int c = c4 << 2;
      best = fminf(best, c + 0 == a ? best : v.x);
      best = fminf(best, c + 1 == a ? best : v.y);
      best = fminf(best, c + 2 == a ? best : v.z);
      best = fminf(best, c + 3 == a ? best : v.w);
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) best = fminf(best, __shfl_xor(best, o, 64));
  if (r < m && sub == 0) {
    const float x = xn[r];
    const float sec = best + x - tau * (x + mc);
    lb[r] = sqrtf(fmaxf(sec, 0.f)) * (1.0f - 1e-6f);
  }
}


// Bounds of the first Lloyd step seeded by the k-means|| init (models/kmeans.py _seed_from_init):
// row x's nearest init candidate p = qmap[nearest[x]] lies within r = sqrt(cost + slack) of x, and p's
// nearest / second-nearest centres are a(p) at d1(p) / d2(p) (exact f64 over the bf16 operands, rounded
// outward), so |x - c_a| <= r + d1 and |x - c_j| >= d2 - r for every other j: label a(p), ub, lb.
__global__ __launch_bounds__(256) void kmeans_seed_bounds_kernel(
    const int* __restrict__ nearest, const float* __restrict__ cost, const float* __restrict__ xn,
    const int* __restrict__ qmap, const int* __restrict__ a, const float* __restrict__ d1,
    const float* __restrict__ d2, const float* __restrict__ pn, float tau, long long n, int* __restrict__ labels,
    float* __restrict__ ub, float* __restrict__ lb) {
  const long long row = (long long)blockIdx.x * 256 + threadIdx.x;
  if (row >= n) return;
  const int q = qmap[nearest[row]];
  const float r = sqrtf(fmaxf(cost[row], 0.f) + tau * (xn[row] + pn[q])) * (1.0f + 1e-6f);
  labels[row] = a[q];
  ub[row] = (r + d1[q]) * (1.0f + 1e-6f);
  lb[row] = fmaxf(d2[q] - r, 0.f) * (1.0f - 1e-6f);
}

// Counting-sort ranks of the current labels in the K9r workgroup geometry (row -> workgroup
// (row / tr) % grid), for a full accumulate after a step that ran only the candidate pass:
// hist[b][label] and rank[row] = the row's position among its workgroup's rows of that label.
// 1024 threads = 1024 / tr of the workgroup's tiles per sweep (tr <= 1024 rows per tile).
__global__ __launch_bounds__(1024) void kmeans_label_hist_kernel(const int* __restrict__ labels, long long n, int tr,
                                                                 int kp, int* __restrict__ hist,
                                                                 int* __restrict__ rank, const int* __restrict__ gate,
                                                                 int want) {
  if (gate != nullptr && gate[0] != want) return;  // the pass the gate picked made hist/rank itself
  extern __shared__ int h[];
  for (int i = threadIdx.x; i < kp; i += 1024) h[i] = 0;
  __syncthreads();
  const int per = 1024 / tr, t = threadIdx.x / tr, i = threadIdx.x % tr;
  for (long long j0 = 0; ((long long)blockIdx.x + j0 * gridDim.x) * tr < n; j0 += per) {
    const long long row = ((long long)blockIdx.x + (j0 + t) * gridDim.x) * tr + i;
    if (t < per && row < n) rank[row] = atomicAdd(&h[labels[row]], 1);
  }
  __syncthreads();
  for (int i2 = threadIdx.x; i2 < kp; i2 += 1024) hist[(long long)blockIdx.x * kp + i2] = h[i2];
}

// ---------------------------------------------------------------------------------------------
// Fused tail of the device pruned step (fewer launches per Lloyd step: each launch costs ~4-5 us on the
// shard of an 8-GPU run, where a whole step is ~0.3 ms).
//
// kmeans_update_pdev_kernel: K11 (kmeans_update_kernel: new centre = Σx·unit / count, empty clusters keep
// theirs, bf16 copy, ||cb||²) plus what the pruned step needs from the old and new bf16 centres in the same
// pass — cb_old <- old cb (always), cb_cost <- old cb unless the fit is frozen (flags[1]; the centres of the
// last live assignment, for the training cost), cn64 = ||cb_new||² in f64 and drift = |cb_new - cb_old|
// rounded up. Replaces cond_copy + K11 + the norm/drift half of centre_stats.
__global__ void kmeans_update_pdev_kernel(const double* __restrict__ bufs, int nbuf, long long bstride, int k, int D,
                                          double* __restrict__ cent, u16* __restrict__ cb, long long ldc, int Dp,
                                          float* __restrict__ cnorm, double* __restrict__ shift2, double unit,
                                          u16* __restrict__ cb_old, u16* __restrict__ cb_cost,
                                          const int* __restrict__ flags, double* __restrict__ cn64,
                                          float* __restrict__ drift) {
  __shared__ double rn[16], rs[16], rd[16];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const bool live = flags[1] == 0;
  if (c >= k) {
    for (int d = tid; d < Dp; d += blockDim.x) {
      const u16 o = cb[(long long)c * ldc + d];
      cb_old[(long long)c * ldc + d] = o;
      if (live) cb_cost[(long long)c * ldc + d] = o;
      cb[(long long)c * ldc + d] = 0;
    }
    if (tid == 0) cnorm[c] = __builtin_huge_valf();
    return;
  }
  double cnt = 0.0;
  for (int b = 0; b < nbuf; ++b) cnt += bufs[b * bstride + (long long)k * D + c];
  double nrm = 0.0, sh = 0.0, dr = 0.0;
  for (int d = tid; d < Dp; d += blockDim.x) {
    const u16 o = cb[(long long)c * ldc + d];
    cb_old[(long long)c * ldc + d] = o;
    if (live) cb_cost[(long long)c * ldc + d] = o;
    if (d < D) {
      const double old = cent[(long long)c * D + d];
      double nv = old;
      if (cnt > 0.0) {
        double s = 0.0;
        for (int b = 0; b < nbuf; ++b) s += bufs[b * bstride + (long long)c * D + d];
        nv = (s * unit) / cnt;
      }
      sh += (nv - old) * (nv - old);
      cent[(long long)c * D + d] = nv;
      const u16 q = f32_to_bf16((float)nv);
      cb[(long long)c * ldc + d] = q;
      const double f = (double)bf16_to_f32(q);
      nrm += f * f;
      const double e = f - (double)bf16_to_f32(o);
      dr += e * e;
    } else {
      cb[(long long)c * ldc + d] = 0;
    }
  }
  nrm = wave_sum_f64(nrm);
  sh = wave_sum_f64(sh);
  dr = wave_sum_f64(dr);
  if (lane == 0) { rn[wave] = nrm; rs[wave] = sh; rd[wave] = dr; }
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, b = 0.0, e = 0.0;
    for (int w = 0; w < nw; ++w) { a += rn[w]; b += rs[w]; e += rd[w]; }
    cnorm[c] = (float)a;
    if (shift2 != nullptr) shift2[c] = b;
    cn64[c] = a;
    drift[c] = (float)(sqrt(e) * (1.0 + 1e-6));
  }
}

// Centre statistics of the pruned step in one launch: one workgroup per centre j computes half_j (half the
// distance from c_j to its nearest other centre, as kmeans_centre_stats_kernel); the workgroup that
// finishes last (device-scope counter) runs the single-workgroup part (kmeans_centre_stats2_kernel's work:
// mc, c2, thr, dmax, the cumulative drifts, the count / force / backoff resets) and re-arms the counter.
// decay: half_j is not recomputed this step but lowered to a bound of the new centres' one — the distance
// from c_j to any c_i shrinks by at most drift_j + drift_i, so half_j' >= half_j - (drift_j + max_{i!=j}
// drift_i) / 2 (rounded down). A smaller half only makes the thresholds more conservative.
__device__ void centre_stats2_body(const double* __restrict__ cn, double* __restrict__ half,
                                   const float* __restrict__ drift, int k, const float* __restrict__ mx, float tau,
                                   int have_drift, float* __restrict__ thr, float* __restrict__ dmax,
                                   float* __restrict__ mc, float* __restrict__ c2, int* __restrict__ count,
                                   int* __restrict__ force, float* __restrict__ cum, int* __restrict__ backoff,
                                   int decay = 0) {
  __shared__ double smax[256];
  __shared__ float sdm[3];
  __shared__ float d1[256], d2[256];
  __shared__ int i1[256];
  // the first 256 threads of the workgroup do the work (callers run 256 or more threads; all reach the barriers)
  const int tid = threadIdx.x;
  const bool act = tid < 256;
  double m = 0.0;
  float a = -1.f, b = -1.f;
  int ia = 0;
  for (int j = tid; act && j < k; j += 256) {
    m = cn[j] > m ? cn[j] : m;
    if (have_drift) {
      const float v = drift[j];
      if (v > a) { b = a; a = v; ia = j; }
      else if (v > b) { b = v; }
    }
  }
  // max norm and top-2 drifts (+ index of the largest, lowest index on ties) by wave butterflies, then the four
  // wave results (a thread-0 loop over 256 partials was most of this single-workgroup launch)
  auto merge = [](float& pa, float& pb, int& pi, float qa, float qb, int qi) {
    if (qa > pa || (qa == pa && qi < pi)) {
      pb = qb > pa ? qb : pa;
      pa = qa;
      pi = qi;
    } else {
      pb = pb > qa ? pb : qa;
    }
  };
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double om = __shfl_xor(m, o, 64);
    const float oa = __shfl_xor(a, o, 64), ob = __shfl_xor(b, o, 64);
    const int oi = __shfl_xor(ia, o, 64);
    m = om > m ? om : m;
    merge(a, b, ia, oa, ob, oi);
  }
  if (act && (tid & 63) == 0) {
    smax[tid >> 6] = m;
    d1[tid >> 6] = a;
    d2[tid >> 6] = b;
    i1[tid >> 6] = ia;
  }
  __syncthreads();
  if (tid == 0) {
    double mm = smax[0];
    float ta = d1[0], tb = d2[0];
    int ti = i1[0];
    for (int t = 1; t < 4; ++t) {
      mm = smax[t] > mm ? smax[t] : mm;
      merge(ta, tb, ti, d1[t], d2[t], i1[t]);
    }
    smax[0] = mm;
    *mc = (float)mm;
    *c2 = (float)(2.0 * (double)tau * ((double)*mx + mm));
    if (have_drift) {
      dmax[0] = ta < 0.f ? 0.f : ta;
      dmax[1] = tb < 0.f ? 0.f : tb;
      dmax[2] = (float)ti;
    }
    sdm[0] = ta < 0.f ? 0.f : ta;
    sdm[1] = tb < 0.f ? 0.f : tb;
    sdm[2] = (float)ti;
    *count = 0;
    const int bo = backoff != nullptr ? *backoff : 0;
    *force = bo > 0 ? 1 : 0;
    if (bo > 0) *backoff = bo - 1;
  }
  __syncthreads();
  const double sl = (double)tau * ((double)*mx + smax[0]);
  for (int j = tid; act && j < k; j += 256) {
    float t;
    double hj = half[j];
    if (decay && have_drift) {
      const double other = j == (int)sdm[2] ? (double)sdm[1] : (double)sdm[0];
      hj = fmax(0.0, hj - 0.5 * ((double)drift[j] + other)) * (1.0 - 1e-12);
      half[j] = hj;
    }
    if (k == 1) t = __builtin_huge_valf();
    else if (hj > 0.0) t = (float)((hj - sl / (2.0 * hj)) * (1.0 - 1e-6));
    else t = -__builtin_huge_valf();
    thr[j] = t;
    if (have_drift && cum != nullptr) {
      cum[j] = (cum[j] + drift[j]) * (1.0f + 2.4e-7f);
      cum[k + j] = (cum[k + j] + (j == (int)sdm[2] ? sdm[1] : sdm[0])) * (1.0f + 2.4e-7f);
    }
  }
}

constexpr int kHalfThreads = 1024;

__global__ __launch_bounds__(kHalfThreads) void kmeans_centre_half_stats_kernel(
    const u16* __restrict__ cb, long long ldc, int k, int d, const double* __restrict__ cn,
    double* __restrict__ half, const float* __restrict__ drift, const float* __restrict__ mx, float tau,
    float* __restrict__ thr, float* __restrict__ dmax, float* __restrict__ mc, float* __restrict__ c2,
    int* __restrict__ count, int* __restrict__ force, float* __restrict__ cum, int* __restrict__ backoff,
    int* __restrict__ done_ctr) {
  extern __shared__ __align__(16) unsigned char smem[];
  float* cj = reinterpret_cast<float*>(smem);  // [d] (d a multiple of 8: the padded bf16 rows)
  __shared__ float red[kHalfThreads / 64];
  __shared__ int last;
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int t = tid; t < d; t += kHalfThreads) cj[t] = bf16_to_f32(cb[(long long)j * ldc + t]);
  __syncthreads();
  // f32 direct differences (each difference of two bf16 values is exact in f32); the sum of d rounded
  // squares is within d·2^-24 of the real one, so the result is scaled down by 1 - 4e-5 (d <= 2048) —
  // half_j stays below half the real distance, as the pruning threshold needs.
  // L lanes (a power of two) share a row, each reading 16-B chunks c ≡ sub (mod L): coalesced row reads,
  // 64/L rows per wave instruction, two row groups in flight per lane, then an xor-shuffle sum.
  const int nch = d >> 3;
  int L = 1;
  while (2 * L <= nch && 2 * L <= 64) L *= 2;
  const int rp = 64 / L, sub = lane & (L - 1), rw = lane / L;
  const int step = (kHalfThreads / 64) * rp;  // rows per block pass
  float best = __builtin_huge_valf();
  for (int i0 = wave * rp + rw; i0 < k; i0 += 2 * step) {
    float s[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + u * step;
      float s0 = 0.f, s1 = 0.f;
      if (i < k) {
        const uint4* row = reinterpret_cast<const uint4*>(cb + (long long)i * ldc);
        for (int c = sub; c < nch; c += L) {
          const uint4 w = row[c];
          const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float e0 = __uint_as_float(ws[q] << 16) - cj[8 * c + 2 * q];
            const float e1 = __uint_as_float(ws[q] & 0xffff0000u) - cj[8 * c + 2 * q + 1];
            s0 = fmaf(e0, e0, s0);
            s1 = fmaf(e1, e1, s1);
          }
        }
      }
      s[u] = s0 + s1;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      if (o < L) {
        s[0] += __shfl_xor(s[0], o, 64);
        s[1] += __shfl_xor(s[1], o, 64);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + u * step;
      if (i < k && i != j) best = s[u] < best ? s[u] : best;
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float v = __shfl_xor(best, o, 64);
    best = v < best ? v : best;
  }
  if (lane == 0) red[wave] = best;
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kHalfThreads / 64; ++w) red[0] = red[w] < red[0] ? red[w] : red[0];
  }
  if (tid == 0) {
    half[j] = 0.5 * sqrt((double)red[0] * (1.0 - 4e-5));
    __threadfence();  // half[j] visible device-wide before this block counts itself done
    last = atomicAdd(done_ctr, 1) == k - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();  // acquire side: every other block's half[] is visible
  centre_stats2_body(cn, half, drift, k, mx, tau, 1, thr, dmax, mc, c2, count, force, cum, backoff);
  // re-armed for the next step (stream order: nothing else reads it now)
  if (tid == 0) __hip_atomic_store(done_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

CML_API int cml_kmeans_prune_lower(const float* dist, int k, const int* lab, const float* xn, float mc, float tau,
                                   long long m, float* lb, void* stream) {
  if (k <= 0 || (k & 3) || ((uintptr_t)dist & 15) || m < 0) return (int)hipErrorInvalidValue;
  if (m == 0) return 0;
  const long long rows_per_block = kThreads / 16;
  hipLaunchKernelGGL(kmeans_prune_lower_kernel, dim3((unsigned)((m + rows_per_block - 1) / rows_per_block)),
                     dim3(kThreads), 0, (hipStream_t)stream, dist, k, lab, xn, mc, tau, m, lb);
  return cml_status();
}

// Moves every row's bounds by the centre drifts; rows whose bounds no longer prove the label are
// appended to cand (at most cap entries are written), their number added to *count (zeroed by the
// caller). dmax = {largest drift,
// second largest, index of the largest}. lab / ub / lb 16-byte aligned, k <= 8192.
CML_API int cml_kmeans_prune_bounds_gated(const int* lab, float* ub, float* lb, const float* drift, const float* dmax,
                                          const float* thr, const float* c2, int k, long long n, int* cand, int* count,
                                          const float* xn, int* cand_lab, float* cand_xn, const int* skip,
                                          long long cap, const float* cum, int* mode, long long gate_cap, int* backoff,
                                          int nback, int* done, int* mode_host, void* stream);
CML_API int cml_kmeans_prune_bounds(const int* lab, float* ub, float* lb, const float* drift, const float* dmax,
                                    const float* thr, const float* c2, int k, long long n, int* cand, int* count,
                                    const float* xn, int* cand_lab, float* cand_xn, const int* skip,
                                    long long cap, const float* cum, void* stream) {
  return cml_kmeans_prune_bounds_gated(lab, ub, lb, drift, dmax, thr, c2, k, n, cand, count, xn, cand_lab, cand_xn,
                                       skip, cap, cum, nullptr, 0, nullptr, 0, nullptr, nullptr, stream);
}

// The bounds pass with the step gate folded in (mode / gate_cap / backoff / nback as kmeans_prune_gate; done:
// int32 [1] zero before the first launch, left zero). With n == 0 the gate still runs (one workgroup).
CML_API int cml_kmeans_prune_bounds_gated(const int* lab, float* ub, float* lb, const float* drift, const float* dmax,
                                          const float* thr, const float* c2, int k, long long n, int* cand, int* count,
                                          const float* xn, int* cand_lab, float* cand_xn, const int* skip,
                                          long long cap, const float* cum, int* mode, long long gate_cap, int* backoff,
                                          int nback, int* done, int* mode_host, void* stream) {
  if (mode != nullptr && (skip == nullptr || done == nullptr)) return (int)hipErrorInvalidValue;
  if ((cand_lab == nullptr) != (cand_xn == nullptr) || (cand_lab != nullptr && xn == nullptr))
    return (int)hipErrorInvalidValue;
  if (cum != nullptr && k > 4096) return (int)hipErrorInvalidValue;  // 4k floats of LDS
  if (k <= 0 || k > 8192 || n < 0 || n >= (1LL << 31) || ((uintptr_t)lab & 15) || ((uintptr_t)ub & 15) ||
      ((uintptr_t)lb & 15))
    return (int)hipErrorInvalidValue;
  if (n == 0) {
    if (mode == nullptr) return 0;
    hipLaunchKernelGGL(kmeans_prune_gate_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, count, gate_cap, skip, mode,
                       backoff, nback);
    return cml_status();
  }
  const long long per = (long long)kBoundsThreads * kIters * 4;
  const unsigned grid = (unsigned)((n + per - 1) / per);
  const GateArgs g{mode, gate_cap, backoff, nback, done, mode_host};
  hipLaunchKernelGGL(kmeans_prune_bounds_kernel, dim3(grid), dim3(kBoundsThreads),
                     (size_t)(cum != nullptr ? 4 : 2) * k * sizeof(float), (hipStream_t)stream, lab, ub, lb, drift,
                     dmax, thr, c2, k, n, cand, count, xn, cand_lab, cand_xn, skip, cap, cum, g);
  return cml_status();
}

// flags: int[2] {force, done} (see kmeans_prune_gate_kernel).
// backoff (nullable, int [1]): see kmeans_prune_gate_kernel.
CML_API int cml_kmeans_prune_gate(int* count, long long cap, const int* flags, int* mode, int* backoff, int nback,
                                  void* stream) {
  hipLaunchKernelGGL(kmeans_prune_gate_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, count, cap, flags, mode,
                     backoff, nback);
  return cml_status();
}

CML_API int cml_kmeans_converge_latch(const double* shift2, int k, double lim, int* flags, void* stream) {
  if (k <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_converge_latch_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, shift2, k, lim, flags);
  return cml_status();
}

// n_bytes a multiple of 4, both pointers 4-byte aligned.
CML_API int cml_kmeans_cond_copy(void* dst, const void* src, long long n_bytes, const int* flags, void* dst_always,
                                  void* stream) {
  if (n_bytes % 4 != 0 || ((uintptr_t)dst & 3) || ((uintptr_t)src & 3) || ((uintptr_t)dst_always & 3))
    return (int)hipErrorInvalidValue;
  const long long n = n_bytes / 4;
  if (n == 0) return 0;
  long long g = (n + 255) / 256;
  g = g > 1024 ? 1024 : g;
  hipLaunchKernelGGL(kmeans_cond_copy_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, (unsigned*)dst,
                     (const unsigned*)src, n, flags, (unsigned*)dst_always);
  return cml_status();
}

// cb / cb_old: bf16 centres [>= k rows, ldc]; cb_old may be null (no drift: the bounds start over).
// mx: device scalar max ||x||² (all ranks). Outputs: cn (f64 [k]), half (f64 [k] scratch), drift/thr
// (f32 [k]), dmax (f32 [3]), mc / c2 (f32 scalars); count and force are reset to 0.
CML_API int cml_kmeans_centre_stats(const void* cb, const void* cb_old, long long ldc, int k, int d, const float* mx,
                                    float tau, double* cn, double* half, float* drift, float* thr, float* dmax,
                                    float* mc, float* c2, int* count, int* force, float* cum, int* backoff,
                                    void* stream) {
  if (k <= 0 || d <= 0 || d > 8192) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(kmeans_centre_stats_kernel, dim3(k), dim3(256), (size_t)d * sizeof(double), st,
                     (const u16*)cb, (const u16*)cb_old, ldc, k, d, cn, drift, half);
  hipLaunchKernelGGL(kmeans_centre_stats2_kernel, dim3(1), dim3(256), 0, st, cn, half, drift, k, mx, tau,
                     cb_old != nullptr ? 1 : 0, thr, dmax, mc, c2, count, force, cum, backoff);
  return cml_status();
}

// The centre statistics of a pruned step that keeps last step's half distances, lowered by the drifts
// (centre_stats2_body decay): one workgroup instead of the k-workgroup nearest-centre pass. drift / cn as
// kmeans_update_pdev_kernel leaves them.
__global__ __launch_bounds__(256) void kmeans_centre_decay_stats_kernel(
    const double* __restrict__ cn, double* __restrict__ half, const float* __restrict__ drift, int k,
    const float* __restrict__ mx, float tau, float* __restrict__ thr, float* __restrict__ dmax, float* __restrict__ mc,
    float* __restrict__ c2, int* __restrict__ count, int* __restrict__ force, float* __restrict__ cum,
    int* __restrict__ backoff) {
  centre_stats2_body(cn, half, drift, k, mx, tau, 1, thr, dmax, mc, c2, count, force, cum, backoff, 1);
}

CML_API int cml_kmeans_centre_decay_stats(const double* cn, double* half, const float* drift, int k, const float* mx,
                                          float tau, float* thr, float* dmax, float* mc, float* c2, int* count,
                                          int* force, float* cum, int* backoff, void* stream) {
  if (k <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_centre_decay_stats_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, cn, half, drift, k,
                     mx, tau, thr, dmax, mc, c2, count, force, cum, backoff);
  return cml_status();
}

CML_API int cml_kmeans_seed_bounds(const int* nearest, const float* cost, const float* xn, const int* qmap,
                                   const int* a, const float* d1, const float* d2, const float* pn, float tau,
                                   long long n, int* labels, float* ub, float* lb, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(kmeans_seed_bounds_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     nearest, cost, xn, qmap, a, d1, d2, pn, tau, n, labels, ub, lb);
  return cml_status();
}

// gate (may be null): run only when gate[0] == want (the pruned-step mode flags).
CML_API int cml_kmeans_label_hist(const int* labels, long long n, int tr, int grid, int kp, int* hist, int* rank,
                                  const int* gate, int want, void* stream) {
  if (tr <= 0 || tr > 1024 || grid <= 0 || kp <= 0 || (size_t)kp * 4 > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_label_hist_kernel, dim3(grid), dim3(1024), (size_t)kp * 4, (hipStream_t)stream, labels,
                     n, tr, kp, hist, rank, gate, want);
  return cml_status();
}

// Fused pruned-step tail (see kmeans_update_pdev_kernel / kmeans_centre_half_stats_kernel). bufs: the
// all-reduced [k·D sums | k counts | cost] rows (nbuf of them); cb / cb_old / cb_cost bf16 [Kp, ldc];
// flags int32 [2]; cn64 f64 [k]; drift f32 [k].
CML_API int cml_kmeans_update_pdev(const double* bufs, int nbuf, long long bstride, int k, int D, double* cent,
                                   void* cb, long long ldc, int Dp, int Kp, float* cnorm, double* shift2, double unit,
                                   void* cb_old, void* cb_cost, const int* flags, double* cn64, float* drift,
                                   void* stream) {
  if (bufs == nullptr || nbuf < 1 || k <= 0 || Kp < k) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_update_pdev_kernel, dim3(Kp), dim3(256), 0, (hipStream_t)stream, bufs, nbuf, bstride, k,
                     D, cent, (u16*)cb, ldc, Dp, cnorm, shift2, unit, (u16*)cb_old, (u16*)cb_cost, flags, cn64, drift);
  return cml_status();
}

// done_ctr: int32 [1], zero before the first launch (each launch leaves it zero).
CML_API int cml_kmeans_centre_half_stats(const void* cb, long long ldc, int k, int d, const double* cn, double* half,
                                         const float* drift, const float* mx, float tau, float* thr, float* dmax,
                                         float* mc, float* c2, int* count, int* force, float* cum, int* backoff,
                                         int* done_ctr, void* stream) {
  if (k <= 0 || d <= 0 || d > 2048 || (d & 7) || (ldc & 7) || ((uintptr_t)cb & 15)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_centre_half_stats_kernel, dim3(k), dim3(kHalfThreads), (size_t)d * sizeof(float),
                     (hipStream_t)stream, (const u16*)cb, ldc, k, d, cn, half, drift, mx, tau, thr, dmax, mc, c2,
                     count, force, cum, backoff, done_ctr);
  return cml_status();
}
