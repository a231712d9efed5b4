// Decision-tree / random-forest kernels for gfx950 (K16-K21 in SURVEY.md §2.5).
//
// Capability parity: DecisionTree{Regressor,Classifier} and RandomForest{Regressor,
// Classifier} of the reference (ref.py:150-158, ref.py:182-190), trained level-wise like
// Spark MLlib: binned features, one histogram pass per tree level for ALL trees of the
// forest at once ("ensemble packing"), splits chosen on the host from the all-reduced
// histograms, rows routed to children on the device.
//
// K17 tree_binize  value -> bin: #thresholds < value (binary search, thresholds in LDS);
//                  uint8 codes up to 256 bins, uint16 above
// K18 tree_hist    hist[t][node][f][bin][s] += w_t(row)·stat_s(row) for rows whose node
//                  at this level is `node`; LDS-privatised per workgroup (one tree ×
//                  feature chunk per workgroup), 64-bit fixed point (order-independent,
//                  exact), flushed once with integer global adds.
// K20 tree_route   node_of[t][row] <- left/right child after the level's splits
// K21 tree_predict per-row traversal of every tree, forest mean (regression) or summed
//                  normalised class distributions (classification)
// K21b forest_vote class distribution + thresholded argmax of a classifier transform
#include "common.h"

namespace {

// Bin codes are uint8 while nbins <= 256 (Spark's default maxBins = 32) and uint16 above it, so
// maxBins > 256 never wraps. Thresholds sit in LDS when d * max_splits doubles fit 64 KiB; wider
// tables (d = 512 features, large maxBins) are read from global memory (L2-resident, read-only).
template <typename BinT, bool kLds>
__global__ void tree_binize_kernel(const double* __restrict__ X, long long n, long long ld, int d,
                                   const double* __restrict__ thr, int max_splits, const int* __restrict__ nsplit,
                                   BinT* __restrict__ bins) {
  extern __shared__ double sthr[];
  if (kLds) {
    for (int i = threadIdx.x; i < d * max_splits; i += blockDim.x) sthr[i] = thr[i];
    __syncthreads();
  }
  const double* tab = kLds ? sthr : thr;
  const long long total = n * (long long)d;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / d;
    const int f = (int)(i - r * d);
    const double v = X[r * ld + f];
    const double* t = tab + (long long)f * max_splits;
    int lo = 0, hi = nsplit[f];  // first index with t[idx] >= v
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (t[mid] < v) lo = mid + 1; else hi = mid;
    }
    bins[r * d + f] = (BinT)lo;
  }
}

// grid: (row blocks, trees, feature chunks x node chunks). LDS: nc * fc * nbins * S int64.
// Statistics accumulate as 64-bit FIXED POINT (value * 2^e_s, e_s chosen on the host from the
// global n, max weight and max |y| so no sum can overflow): integer adds are associative, so the
// histogram — and every split chosen from it — is bit-identical whatever the row order, the number
// of workgroups or the number of GPUs, with f64-class precision (Spark aggregates these in f64;
// f32 partials lost ~1e-7 of Σy² and made splits world-size dependent).
// A level whose (node, feature) histograms exceed the LDS budget is split into node chunks
// (blockIdx.z = node chunk * fchunks + feature chunk; each chunk re-reads the row stream); one
// whose single (node, feature) histogram is larger than LDS (nbins * S > 12288) adds straight into
// the global histogram (kDirect, integer atomics: still exact and order-independent).
template <typename BinT, bool kDirect>
__global__ __launch_bounds__(256) void tree_hist_kernel(const BinT* __restrict__ bins, long long n, int d,
                                                        int nbins, const int* __restrict__ node_of,
                                                        const float* __restrict__ wt, const double* __restrict__ y,
                                                        const int* __restrict__ cls, int S, int nodes, int fc,
                                                        int nc, int fchunks, double sc0, double sc1, double sc2,
                                                        unsigned long long* __restrict__ out) {
  extern __shared__ unsigned long long h[];
  const int t = blockIdx.y;
  const int f0 = (blockIdx.z % fchunks) * fc;
  const int n0 = (blockIdx.z / fchunks) * nc;
  const int fcount = min(fc, d - f0);
  const int ncount = min(nc, nodes - n0);
  const int hsize = nc * fc * nbins * S;
  if (!kDirect) {
    for (int i = threadIdx.x; i < hsize; i += blockDim.x) h[i] = 0ull;
    __syncthreads();
  }
  const int* nd = node_of + (long long)t * n;
  const float* w = wt != nullptr ? wt + (long long)t * n : nullptr;
  for (long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long long)gridDim.x * blockDim.x) {
    const int node = nd[r] - n0;
    if (node < 0 || node >= ncount) continue;
    const double wr = w != nullptr ? (double)w[r] : 1.0;
    if (wr == 0.0) continue;
    unsigned long long q0 = (unsigned long long)llrint(wr * sc0), q1 = 0ull, q2 = 0ull;
    int c = -1;
    if (cls == nullptr) {
      const double yv = y[r];
      q1 = (unsigned long long)llrint(wr * yv * sc1);
      q2 = (unsigned long long)llrint(wr * yv * yv * sc2);
    } else {
      c = cls[r];
    }
    const BinT* br = bins + r * d + f0;
    for (int f = 0; f < fcount; ++f) {
      unsigned long long* cell =
          kDirect ? out + ((((long long)t * nodes + n0 + node) * d + f0 + f) * nbins + br[f]) * S
                  : h + ((node * fc + f) * nbins + br[f]) * S;
      if (cls == nullptr) {
        atomicAdd(cell + 0, q0);
        atomicAdd(cell + 1, q1);
        atomicAdd(cell + 2, q2);
      } else {
        atomicAdd(cell + c, q0);
      }
    }
  }
  if (kDirect) return;
  __syncthreads();
  for (int i = threadIdx.x; i < hsize; i += blockDim.x) {
    const unsigned long long v = h[i];
    if (v == 0ull) continue;
    const int s = i % S;
    const int rest = i / S;
    const int b = rest % nbins;
    const int rest2 = rest / nbins;
    const int f = rest2 % fc;
    const int node = rest2 / fc;
    if (f >= fcount || node >= ncount) continue;
    atomicAdd(out + ((((long long)t * nodes + n0 + node) * d + f0 + f) * nbins + b) * S + s, v);
  }
}

// K19 best split, one workgroup per (tree, node) of the level, on the all-reduced fixed-point
// histogram (exact int64 prefix sums over bins, converted to f64 per candidate). Spark's
// binsToBestSplit takes the first maximum gain in (feature, bin) order among candidates whose two
// children reach the minimum weight and whose gain reaches minInfoGain. Small nodes often have
// EXACT ties (two features separating the same rows), which rounding then breaks arbitrarily, so
// the rule here is order-independent: G = max gain, then the first (feature, bin) whose gain is
// within kTreeTieRel·|G| of G (two block reductions) — CPU, GPU and any world size pick the same
// split. out row: [gain, feature, bin, total S, left S, right S]; gain = -inf and feature = -1 when
// no valid split exists. Only (f, b) with mask[f] and b < nsplit[f] are candidates. S <= kTreeSMax.
constexpr int kTreeSMax = 16;
constexpr double kTreeTieRel = 1e-12;

__device__ double impurity_dev(const double* st, int S, int kind) {
  if (kind == 0) {
    const double w = st[0];
    if (w <= 0.0) return 0.0;
    const double m = st[1] / w;
    const double v = st[2] / w - m * m;
    return v > 0.0 ? v : 0.0;
  }
  double tot = 0.0;
  for (int c = 0; c < S; ++c) tot += st[c];
  if (tot <= 0.0) return 0.0;
  double r = kind == 1 ? 1.0 : 0.0;
  for (int c = 0; c < S; ++c) {
    const double p = st[c] / tot;
    if (kind == 1) r -= p * p;
    else if (p > 0.0) r -= p * log2(p);
  }
  return r;
}

__device__ __forceinline__ double count_dev(const double* st, int S, int kind) {
  if (kind == 0) return st[0];
  double t = 0.0;
  for (int c = 0; c < S; ++c) t += st[c];
  return t;
}

__global__ __launch_bounds__(256) void tree_best_split_kernel(const long long* __restrict__ hist, int d, int nbins,
                                                              int S, const double* __restrict__ scale, int kind,
                                                              const unsigned char* __restrict__ mask,
                                                              const int* __restrict__ nsplit, double min_inst,
                                                              double min_wfrac, double min_gain,
                                                              double* __restrict__ out) {
  __shared__ long long tot_i[kTreeSMax];
  __shared__ double bg[256];
  __shared__ int bi[256];
  const int tn = blockIdx.x;  // tree * nodes + node
  const long long* h = hist + (long long)tn * d * nbins * S;
  const int tid = threadIdx.x;
  if (tid < S) {
    long long t = 0;
    for (int b = 0; b < nbins; ++b) t += h[(long long)b * S + tid];  // feature 0 covers every row once
    tot_i[tid] = t;
  }
  __syncthreads();
  double sc[kTreeSMax], tot[kTreeSMax];
  for (int c = 0; c < S; ++c) {
    sc[c] = scale[kind == 0 ? c : 0];
    tot[c] = (double)tot_i[c] / sc[c];
  }
  const double wtot = count_dev(tot, S, kind);
  const double imp = impurity_dev(tot, S, kind);
  const double min_w = fmax(min_inst, min_wfrac * wtot);
  // pass 0: G = the maximum valid gain; pass 1: first (f, b) whose gain is within the tie tolerance
  double G = -__builtin_huge_val();
  int bidx = 0x7fffffff;
  for (int pass = 0; pass < 2; ++pass) {
    const double thr = pass == 0 ? 0.0 : G - kTreeTieRel * fabs(G);
    double best = -__builtin_huge_val();
    bidx = 0x7fffffff;
    for (int f = tid; f < d; f += blockDim.x) {
      if (!mask[(long long)tn * d + f]) continue;
      const int ns = nsplit[f];
      const long long* hf = h + (long long)f * nbins * S;
      long long cum[kTreeSMax];
      for (int c = 0; c < S; ++c) cum[c] = 0;
      for (int b = 0; b < ns; ++b) {
        double ls[kTreeSMax], rs[kTreeSMax];
        for (int c = 0; c < S; ++c) {
          cum[c] += hf[(long long)b * S + c];
          ls[c] = (double)cum[c] / sc[c];
          rs[c] = (double)(tot_i[c] - cum[c]) / sc[c];
        }
        const double wl = count_dev(ls, S, kind), wr = count_dev(rs, S, kind);
        if (wl < min_w || wr < min_w || wl <= 0.0 || wr <= 0.0) continue;
        const double gain = imp - (wl / wtot) * impurity_dev(ls, S, kind) - (wr / wtot) * impurity_dev(rs, S, kind);
        if (gain < min_gain) continue;
        if (pass == 0) {
          best = gain > best ? gain : best;
        } else if (gain >= thr && f * nbins + b < bidx) {
          bidx = f * nbins + b;
          best = gain;
        }
      }
    }
    bg[tid] = best;
    bi[tid] = bidx;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (tid < o) {
        if (pass == 0) {
          bg[tid] = bg[tid + o] > bg[tid] ? bg[tid + o] : bg[tid];
        } else if (bi[tid + o] < bi[tid]) {
          bg[tid] = bg[tid + o];
          bi[tid] = bi[tid + o];
        }
      }
      __syncthreads();
    }
    if (pass == 0) {
      G = bg[0];
      __syncthreads();
      if (!(G > -__builtin_huge_val())) break;  // no valid candidate (uniform)
    }
  }
  if (tid == 0) {
    double* o = out + (long long)tn * (3 + 3 * S);
    const bool valid = G > -__builtin_huge_val() && bi[0] != 0x7fffffff;
    const int f = valid ? bi[0] / nbins : -1, b = valid ? bi[0] % nbins : -1;
    o[0] = valid ? bg[0] : -__builtin_huge_val();
    o[1] = (double)f;
    o[2] = (double)b;
    long long cum[kTreeSMax];
    for (int c = 0; c < S; ++c) cum[c] = 0;
    if (valid)
      for (int bb = 0; bb <= b; ++bb)
        for (int c = 0; c < S; ++c) cum[c] += h[((long long)f * nbins + bb) * S + c];
    for (int c = 0; c < S; ++c) {
      o[3 + c] = tot[c];
      o[3 + S + c] = (double)cum[c] / sc[c];
      o[3 + 2 * S + c] = (double)(tot_i[c] - cum[c]) / sc[c];
    }
  }
}

// split_feat/split_bin/left_id/right_id: [T][nodes]; split_feat < 0 => node is a leaf (row retires).
template <typename BinT>
__global__ void tree_route_kernel(const BinT* __restrict__ bins, long long n, int d, int T, int nodes,
                                  int* __restrict__ node_of, const int* __restrict__ split_feat,
                                  const int* __restrict__ split_bin, const int* __restrict__ left_id,
                                  const int* __restrict__ right_id) {
  const long long total = n * (long long)T;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / n);
    const long long r = i - (long long)t * n;
    const int node = node_of[i];
    if (node < 0) continue;
    const int k = t * nodes + node;
    const int f = split_feat[k];
    if (f < 0) {
      node_of[i] = -1;
      continue;
    }
    node_of[i] = (int)bins[r * d + f] <= split_bin[k] ? left_id[k] : right_id[k];
  }
}

// Flattened forest: per node feature (-1 leaf), threshold, left, right (absolute indices),
// leaf value offset into `leaf` (S values). tree_root[t] = index of tree t's root.
__global__ void tree_predict_kernel(const double* __restrict__ X, long long n, long long ld, int T,
                                    const int* __restrict__ root, const int* __restrict__ feat,
                                    const double* __restrict__ thr, const int* __restrict__ left,
                                    const int* __restrict__ right, const double* __restrict__ leaf, int S,
                                    double div, double* __restrict__ out /*[n][S]*/) {
  for (long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long long)gridDim.x * blockDim.x) {
    double acc[16];
    for (int s = 0; s < S; ++s) acc[s] = 0.0;
    for (int t = 0; t < T; ++t) {
      int k = root[t];
      while (feat[k] >= 0) k = X[r * ld + feat[k]] <= thr[k] ? left[k] : right[k];
      for (int s = 0; s < S; ++s) acc[s] += leaf[(long long)k * S + s];
    }
    // the forest mean as a true division (correctly rounded, like the host's tensor division)
    for (int s = 0; s < S; ++s) out[r * S + s] = div == 1.0 ? acc[s] : acc[s] / div;
  }
}

// K21b forest vote: per row, the class distribution raw/sum(raw) (uniform 1/S when the sum is not
// positive) and the prediction argmax(prob / thresholds) (first maximum). Replaces five tensor ops of
// the transform (row sum, clamp, divide, select, argmax), each a separate launch and, on a session's
// first tree transform, a separate first-use code-object load.
__global__ void forest_vote_kernel(const double* __restrict__ raw, long long n, int S,
                                   const double* __restrict__ thr /* [S] or null */, double* __restrict__ prob,
                                   double* __restrict__ pred) {
  for (long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long long)gridDim.x * blockDim.x) {
    const double* v = raw + r * S;
    double sum = 0.0;
    for (int s = 0; s < S; ++s) sum += v[s];
    int best = 0;
    double bv = 0.0;
    for (int s = 0; s < S; ++s) {
      const double p = sum > 0.0 ? v[s] / sum : 1.0 / (double)S;
      prob[r * S + s] = p;
      const double q = thr ? p / fmax(thr[s], 1e-300) : p;
      if (s == 0 || q > bv) {
        bv = q;
        best = s;
      }
    }
    pred[r] = (double)best;
  }
}

int blocks_for(long long work, int threads, int cap) {
  long long b = (work + threads - 1) / threads;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

}  // namespace

// bin_bytes: 1 (uint8 codes, nbins <= 256) or 2 (uint16 codes, nbins <= 65536).
CML_API int cml_tree_binize(const double* X, long long n, long long ld, int d, const double* thr, int max_splits,
                            const int* nsplit, void* bins, int bin_bytes, void* stream) {
  if (bin_bytes != 1 && bin_bytes != 2) return (int)hipErrorInvalidValue;
  if (bin_bytes == 1 && max_splits > 255) return (int)hipErrorInvalidValue;
  const size_t lds = sizeof(double) * (size_t)d * max_splits;
  const bool use_lds = lds <= 64 * 1024;
  const dim3 grid(blocks_for(n * d, 256, 4096));
  hipStream_t s = (hipStream_t)stream;
  if (bin_bytes == 1) {
    if (use_lds)
      hipLaunchKernelGGL((tree_binize_kernel<unsigned char, true>), grid, dim3(256), lds, s, X, n, ld, d, thr,
                         max_splits, nsplit, (unsigned char*)bins);
    else
      hipLaunchKernelGGL((tree_binize_kernel<unsigned char, false>), grid, dim3(256), 0, s, X, n, ld, d, thr,
                         max_splits, nsplit, (unsigned char*)bins);
  } else {
    if (use_lds)
      hipLaunchKernelGGL((tree_binize_kernel<unsigned short, true>), grid, dim3(256), lds, s, X, n, ld, d, thr,
                         max_splits, nsplit, (unsigned short*)bins);
    else
      hipLaunchKernelGGL((tree_binize_kernel<unsigned short, false>), grid, dim3(256), 0, s, X, n, ld, d, thr,
                         max_splits, nsplit, (unsigned short*)bins);
  }
  return cml_status();
}

namespace {
template <typename BinT>
void launch_hist(const BinT* bins, long long n, int d, int nbins, const int* node_of, int T, const float* wt,
                 const double* y, const int* cls, int S, int nodes, const double* scales, unsigned long long* out,
                 int row_blocks, hipStream_t stream) {
  constexpr long long kBudget = 96 * 1024;
  const long long per_cell = (long long)nbins * S * 8;  // one (node, feature) histogram
  if (per_cell > kBudget) {
    hipLaunchKernelGGL((tree_hist_kernel<BinT, true>), dim3(row_blocks, T, 1), dim3(256), 0, stream, bins, n, d,
                       nbins, node_of, wt, y, cls, S, nodes, d, nodes, 1, scales[0], scales[1], scales[2], out);
    return;
  }
  int fc, nc;
  if ((long long)nodes * per_cell <= kBudget) {
    nc = nodes;
    fc = (int)(kBudget / ((long long)nodes * per_cell));
    if (fc > d) fc = d;
  } else {
    fc = 1;
    nc = (int)(kBudget / per_cell);
  }
  const int fchunks = (d + fc - 1) / fc;
  const int nchunks = (nodes + nc - 1) / nc;
  const size_t lds = (size_t)per_cell * fc * nc;
  hipFuncSetAttribute((const void*)tree_hist_kernel<BinT, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  hipLaunchKernelGGL((tree_hist_kernel<BinT, false>), dim3(row_blocks, T, fchunks * nchunks), dim3(256), lds, stream,
                     bins, n, d, nbins, node_of, wt, y, cls, S, nodes, fc, nc, fchunks, scales[0], scales[1],
                     scales[2], out);
}
}  // namespace

// out must be zeroed; bin_bytes as for cml_tree_binize.
CML_API int cml_tree_hist(const void* bins, long long n, int d, int nbins, const int* node_of, int T,
                          const float* wt, const double* y, const int* cls, int S, int nodes, const double* scales,
                          unsigned long long* out, int row_blocks, int bin_bytes, void* stream) {
  if (nodes < 1 || d < 1 || nbins < 1 || S < 1) return (int)hipErrorInvalidValue;
  if (bin_bytes == 1)
    launch_hist((const unsigned char*)bins, n, d, nbins, node_of, T, wt, y, cls, S, nodes, scales, out, row_blocks,
                (hipStream_t)stream);
  else if (bin_bytes == 2)
    launch_hist((const unsigned short*)bins, n, d, nbins, node_of, T, wt, y, cls, S, nodes, scales, out, row_blocks,
                (hipStream_t)stream);
  else
    return (int)hipErrorInvalidValue;
  return cml_status();
}

// K19: out [T*nodes][3 + 3S] (see tree_best_split_kernel). kind 0 variance, 1 gini, 2 entropy.
CML_API int cml_tree_best_split(const long long* hist, int tn, int d, int nbins, int S, const double* scale, int kind,
                                const unsigned char* mask, const int* nsplit, double min_inst, double min_wfrac,
                                double min_gain, double* out, void* stream) {
  if (S < 1 || S > kTreeSMax || tn < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tree_best_split_kernel, dim3(tn), dim3(256), 0, (hipStream_t)stream, hist, d, nbins, S, scale,
                     kind, mask, nsplit, min_inst, min_wfrac, min_gain, out);
  return cml_status();
}

CML_API int cml_tree_route(const void* bins, long long n, int d, int T, int nodes, int* node_of,
                           const int* split_feat, const int* split_bin, const int* left_id, const int* right_id,
                           int bin_bytes, void* stream) {
  const dim3 grid(blocks_for(n * T, 256, 8192));
  if (bin_bytes == 1)
    hipLaunchKernelGGL(tree_route_kernel<unsigned char>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const unsigned char*)bins, n, d, T, nodes, node_of, split_feat, split_bin, left_id, right_id);
  else if (bin_bytes == 2)
    hipLaunchKernelGGL(tree_route_kernel<unsigned short>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const unsigned short*)bins, n, d, T, nodes, node_of, split_feat, split_bin, left_id, right_id);
  else
    return (int)hipErrorInvalidValue;
  return cml_status();
}

CML_API int cml_tree_predict(const double* X, long long n, long long ld, int T, const int* root, const int* feat,
                             const double* thr, const int* left, const int* right, const double* leaf, int S,
                             double div, double* out, void* stream) {
  if (S > 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tree_predict_kernel, dim3(blocks_for(n, 256, 8192)), dim3(256), 0, (hipStream_t)stream, X, n, ld,
                     T, root, feat, thr, left, right, leaf, S, div, out);
  return cml_status();
}

CML_API int cml_forest_vote(const double* raw, long long n, int S, const double* thr, double* prob, double* pred,
                            void* stream) {
  if (S < 1 || S > 16) return (int)hipErrorInvalidValue;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(forest_vote_kernel, dim3(blocks_for(n, 256, 8192)), dim3(256), 0, (hipStream_t)stream, raw, n, S,
                     thr, prob, pred);
  return cml_status();
}
