// Decision-tree / random-forest kernels for gfx950 (K16-K21 in SURVEY.md §2.5).
//
// Capability parity: DecisionTree{Regressor,Classifier} and RandomForest{Regressor,
// Classifier} of the reference (ref.py:150-158, ref.py:182-190), trained level-wise like
// Spark MLlib: binned features, one histogram pass per tree level for ALL trees of the
// forest at once ("ensemble packing"), splits chosen on the host from the all-reduced
// histograms, rows routed to children on the device.
//
// K17 tree_binize  value -> bin: #thresholds < value (binary search, thresholds in LDS)
// K18 tree_hist    hist[t][node][f][bin][s] += w_t(row)·stat_s(row) for rows whose node
//                  at this level is `node`; LDS-privatised per workgroup (one tree ×
//                  feature chunk per workgroup), 64-bit fixed point (order-independent,
//                  exact), flushed once with integer global adds.
// K20 tree_route   node_of[t][row] <- left/right child after the level's splits
// K21 tree_predict per-row traversal of every tree (arrays in LDS), forest mean
//                  (regression) or summed normalised class distributions (classification)
#include "common.h"

namespace {

__global__ void tree_binize_kernel(const double* __restrict__ X, long long n, long long ld, int d,
                                   const double* __restrict__ thr, int max_splits, const int* __restrict__ nsplit,
                                   unsigned char* __restrict__ bins) {
  extern __shared__ double sthr[];
  for (int i = threadIdx.x; i < d * max_splits; i += blockDim.x) sthr[i] = thr[i];
  __syncthreads();
  const long long total = n * (long long)d;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / d;
    const int f = (int)(i - r * d);
    const double v = X[r * ld + f];
    const double* t = sthr + f * max_splits;
    int lo = 0, hi = nsplit[f];  // first index with t[idx] >= v
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (t[mid] < v) lo = mid + 1; else hi = mid;
    }
    bins[r * d + f] = (unsigned char)lo;
  }
}

// grid: (row blocks, trees, feature chunks). LDS: nodes * fc * nbins * S int64.
// Statistics accumulate as 64-bit FIXED POINT (value * 2^e_s, e_s chosen on the host from the
// global n, max weight and max |y| so no sum can overflow): integer adds are associative, so the
// histogram — and every split chosen from it — is bit-identical whatever the row order, the number
// of workgroups or the number of GPUs, with f64-class precision (Spark aggregates these in f64;
// f32 partials lost ~1e-7 of Σy² and made splits world-size dependent).
__global__ __launch_bounds__(256) void tree_hist_kernel(const unsigned char* __restrict__ bins, long long n, int d,
                                                        int nbins, const int* __restrict__ node_of,
                                                        const float* __restrict__ wt, const double* __restrict__ y,
                                                        const int* __restrict__ cls, int S, int nodes, int fc,
                                                        double sc0, double sc1, double sc2,
                                                        unsigned long long* __restrict__ out) {
  extern __shared__ unsigned long long h[];
  const int t = blockIdx.y;
  const int f0 = blockIdx.z * fc;
  const int fcount = min(fc, d - f0);
  const int hsize = nodes * fc * nbins * S;
  for (int i = threadIdx.x; i < hsize; i += blockDim.x) h[i] = 0ull;
  __syncthreads();
  const int* nd = node_of + (long long)t * n;
  const float* w = wt != nullptr ? wt + (long long)t * n : nullptr;
  for (long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long long)gridDim.x * blockDim.x) {
    const int node = nd[r];
    if (node < 0) continue;
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
    const unsigned char* br = bins + r * d + f0;
    for (int f = 0; f < fcount; ++f) {
      unsigned long long* cell = h + ((node * fc + f) * nbins + br[f]) * S;
      if (cls == nullptr) {
        atomicAdd(cell + 0, q0);
        atomicAdd(cell + 1, q1);
        atomicAdd(cell + 2, q2);
      } else {
        atomicAdd(cell + c, q0);
      }
    }
  }
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
    if (f >= fcount) continue;
    atomicAdd(out + ((((long long)t * nodes + node) * d + f0 + f) * nbins + b) * S + s, v);
  }
}

// split_feat/split_bin/left_id/right_id: [T][nodes]; split_feat < 0 => node is a leaf (row retires).
__global__ void tree_route_kernel(const unsigned char* __restrict__ bins, long long n, int d, int T, int nodes,
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
    node_of[i] = bins[r * d + f] <= split_bin[k] ? left_id[k] : right_id[k];
  }
}

// Flattened forest: per node feature (-1 leaf), threshold, left, right (absolute indices),
// leaf value offset into `leaf` (S values). tree_root[t] = index of tree t's root.
__global__ void tree_predict_kernel(const double* __restrict__ X, long long n, long long ld, int T,
                                    const int* __restrict__ root, const int* __restrict__ feat,
                                    const double* __restrict__ thr, const int* __restrict__ left,
                                    const int* __restrict__ right, const double* __restrict__ leaf, int S,
                                    double* __restrict__ out /*[n][S]*/) {
  for (long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long long)gridDim.x * blockDim.x) {
    double acc[16];
    for (int s = 0; s < S; ++s) acc[s] = 0.0;
    for (int t = 0; t < T; ++t) {
      int k = root[t];
      while (feat[k] >= 0) k = X[r * ld + feat[k]] <= thr[k] ? left[k] : right[k];
      for (int s = 0; s < S; ++s) acc[s] += leaf[(long long)k * S + s];
    }
    for (int s = 0; s < S; ++s) out[r * S + s] = acc[s];
  }
}

int blocks_for(long long work, int threads, int cap) {
  long long b = (work + threads - 1) / threads;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

}  // namespace

CML_API int cml_tree_binize(const double* X, long long n, long long ld, int d, const double* thr, int max_splits,
                            const int* nsplit, unsigned char* bins, void* stream) {
  const size_t lds = sizeof(double) * (size_t)d * max_splits;
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tree_binize_kernel, dim3(blocks_for(n * d, 256, 4096)), dim3(256), lds, (hipStream_t)stream, X,
                     n, ld, d, thr, max_splits, nsplit, bins);
  return cml_status();
}

// Returns the feature chunk used (features per workgroup) so the host can size nothing; out must be zeroed.
CML_API int cml_tree_hist(const unsigned char* bins, long long n, int d, int nbins, const int* node_of, int T,
                          const float* wt, const double* y, const int* cls, int S, int nodes, const double* scales,
                          unsigned long long* out, int row_blocks, void* stream) {
  const long long per_feat = (long long)nodes * nbins * S * 8;
  int fc = (int)((96 * 1024) / (per_feat > 0 ? per_feat : 1));
  if (fc < 1) return (int)hipErrorInvalidValue;
  if (fc > d) fc = d;
  const int fchunks = (d + fc - 1) / fc;
  const size_t lds = (size_t)per_feat * fc;
  hipFuncSetAttribute((const void*)tree_hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(tree_hist_kernel, dim3(row_blocks, T, fchunks), dim3(256), lds, (hipStream_t)stream, bins, n, d,
                     nbins, node_of, wt, y, cls, S, nodes, fc, scales[0], scales[1], scales[2], out);
  return cml_status();
}

CML_API int cml_tree_route(const unsigned char* bins, long long n, int d, int T, int nodes, int* node_of,
                           const int* split_feat, const int* split_bin, const int* left_id, const int* right_id,
                           void* stream) {
  hipLaunchKernelGGL(tree_route_kernel, dim3(blocks_for(n * T, 256, 8192)), dim3(256), 0, (hipStream_t)stream, bins,
                     n, d, T, nodes, node_of, split_feat, split_bin, left_id, right_id);
  return cml_status();
}

CML_API int cml_tree_predict(const double* X, long long n, long long ld, int T, const int* root, const int* feat,
                             const double* thr, const int* left, const int* right, const double* leaf, int S,
                             double* out, void* stream) {
  if (S > 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tree_predict_kernel, dim3(blocks_for(n, 256, 8192)), dim3(256), 0, (hipStream_t)stream, X, n, ld,
                     T, root, feat, thr, left, right, leaf, S, out);
  return cml_status();
}
