// Host twin of the local k-means kernels of csrc/kmeans_init.hip (weighted k-means++ seeding +
// weighted Lloyd on the k-means|| candidates, Spark LocalKMeans.kMeansPlusPlus semantics).
//
// The CPU session (local[n]) and the GPU must start Lloyd from the same centres, so every value is
// formed here with the operations, in the order, the device kernels use: distances as a fold of
// fma(p_t - c_t, p_t - c_t, acc) over t; the cumulative pick weight summed in kBlocks contiguous
// blocks; weighted sums as fma folds in point order; a division for 1 / Σw then a product; IEEE
// correctly-rounded operations everywhere (this file is built with -ffp-contract=off, and std::fma /
// std::sqrt are correctly rounded), so both produce the same bits.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#define CML_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kBlocks = 256;

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

inline double cu(uint64_t c, uint64_t key) {
  return (double)(splitmix64(c ^ key) >> 11) * (1.0 / 9007199254740992.0);
}

inline double dist_seq(const double* p, const double* c, int d) {
  double acc = 0.0;
  for (int t = 0; t < d; ++t) {
    const double e = p[t] - c[t];
    acc = std::fma(e, e, acc);
  }
  return acc;
}

void kpp(const double* P, int m, int d, const double* w, int k, uint64_t key, double* C, double* d2) {
  const int L = (m + kBlocks - 1) / kBlocks;
  std::vector<double> part(kBlocks);
  for (int i = 0; i < k; ++i) {
    auto pw = [&](int q) { return i == 0 ? w[q] : w[q] * d2[q]; };
    for (int b = 0; b < kBlocks; ++b) {
      double s = 0.0;
      const int q1 = std::min(m, (b + 1) * L);
      for (int q = b * L; q < q1; ++q) s = s + pw(q);
      part[b] = s;
    }
    // lane sums of 4 parts, inclusive Hillis-Steele scan over the 64 lanes (the device's wave 0)
    double S[64], T[64];
    for (int l = 0; l < 64; ++l) {
      double q4 = part[4 * l];
      for (int j = 1; j < 4; ++j) q4 = q4 + part[4 * l + j];
      S[l] = q4;
    }
    for (int off = 1; off < 64; off <<= 1) {
      for (int l = 0; l < 64; ++l) T[l] = l >= off ? S[l - off] + S[l] : S[l];
      std::memcpy(S, T, sizeof(S));
    }
    const double total = S[63];
    const double u = cu((uint64_t)i, key);
    int pick = -1;
    if (!(total > 0.0)) {
      pick = (int)(u * (double)m);
      pick = pick < m - 1 ? pick : m - 1;
    } else {
      const double r = u * total;
      int ls = -1;
      for (int l = 0; l < 64 && ls < 0; ++l)
        if (S[l] > r) ls = l;
      if (ls >= 0) {
        double cum = ls > 0 ? S[ls - 1] : 0.0;
        int lastb = -1;
        for (int j = 0; j < 4 && pick < 0; ++j) {
          const int b = 4 * ls + j;
          const double nxt = cum + part[b];
          if (part[b] > 0.0) lastb = b;
          if (nxt > r) {
            double c2 = cum;
            const int q1 = std::min(m, (b + 1) * L);
            int lastpos = -1;
            for (int q = b * L; q < q1; ++q) {
              const double p = pw(q);
              if (p > 0.0) lastpos = q;
              c2 = c2 + p;
              if (c2 > r) { pick = q; break; }
            }
            if (pick < 0) pick = lastpos;
          }
          cum = nxt;
        }
        if (pick < 0 && lastb >= 0) {
          const int q1 = std::min(m, (lastb + 1) * L);
          for (int q = lastb * L; q < q1; ++q)
            if (pw(q) > 0.0) pick = q;
        }
      }
      if (pick < 0)
        for (int q = m - 1; q >= 0 && pick < 0; --q)
          if (pw(q) > 0.0) pick = q;
      if (pick < 0) pick = 0;
    }
    std::memcpy(C + (size_t)i * d, P + (size_t)pick * d, sizeof(double) * (size_t)d);
    for (int q = 0; q < m; ++q) {
      const double dd = dist_seq(P + (size_t)q * d, C + (size_t)i * d, d);
      d2[q] = (i == 0 || dd < d2[q]) ? dd : d2[q];
    }
  }
}

}  // namespace

// Weighted k-means++ + up to max_iter weighted Lloyd iterations; C: f64 [k, d] out. Returns the
// number of Lloyd assignments run.
CML_HOST_API int cml_local_kmeans_host(const double* P, int m, int d, const double* w, int k, uint64_t key_pp,
                                       uint64_t key_empty, int max_iter, int spherical, double* C) {
  if (m <= 0 || d <= 0 || k <= 0) return -1;
  std::vector<double> d2(m);
  kpp(P, m, d, w, k, key_pp, C, d2.data());
  std::vector<int> lab(m, -1);
  std::vector<double> cnt(k), cvals(d);
  uint64_t ctr = 0;
  int it = 0;
  for (; it < max_iter; ++it) {
    bool moved = false;
    for (int q = 0; q < m; ++q) {
      double best = HUGE_VAL;
      int bi = 0x7fffffff;
      for (int j = 0; j < k; ++j) {
        const double a = dist_seq(P + (size_t)q * d, C + (size_t)j * d, d);
        if (a < best) { best = a; bi = j; }
      }
      if (lab[q] != bi) { lab[q] = bi; moved = true; }
    }
    if (!moved) break;
    for (int j = 0; j < k; ++j) {
      double c = 0.0;
      for (int q = 0; q < m; ++q)
        if (lab[q] == j) c = c + w[q];
      cnt[j] = c;
      if (!(c > 0.0)) continue;
      const double inv = 1.0 / c;
      for (int t = 0; t < d; ++t) {
        double s = 0.0;
        for (int q = 0; q < m; ++q)
          if (lab[q] == j) s = std::fma(w[q], P[(size_t)q * d + t], s);
        cvals[t] = s * inv;
      }
      if (spherical) {
        double a = 0.0;
        for (int t = 0; t < d; ++t) a = std::fma(cvals[t], cvals[t], a);
        double nr = std::sqrt(a);
        nr = nr > 1e-300 ? nr : 1e-300;
        for (int t = 0; t < d; ++t) cvals[t] = cvals[t] / nr;
      }
      std::memcpy(C + (size_t)j * d, cvals.data(), sizeof(double) * (size_t)d);
    }
    for (int j = 0; j < k; ++j) {
      if (!(cnt[j] > 0.0)) {
        int q = (int)(cu(ctr++, key_empty) * (double)m);
        q = q < m - 1 ? q : m - 1;
        std::memcpy(C + (size_t)j * d, P + (size_t)q * d, sizeof(double) * (size_t)d);
      }
    }
  }
  return it;
}

// ---- host twins of csrc/kmeans_exact.hip (the CPU session's KMeans assignment and sums) ----------
// exact_assign: dimension-ordered fold of fma(x_t - c_t, x_t - c_t, acc), ties to the lowest index —
// the device kernel's arithmetic, so CPU and GPU sessions label rows identically. Rows are split over
// `threads` std::threads (each row's result does not depend on the split).
CML_HOST_API int cml_exact_assign_host(const double* X, long long n, long long ldx, int d, const double* C, int k,
                                       long long* labels, double* best, int threads) {
  if (n < 0 || d <= 0 || k <= 0) return -1;
  auto work = [&](long long r0, long long r1) {
    for (long long r = r0; r < r1; ++r) {
      const double* x = X + r * ldx;
      double bd = HUGE_VAL;
      int bi = 0;
      for (int j = 0; j < k; ++j) {
        const double* c = C + (long long)j * d;
        double acc = 0.0;
        for (int t = 0; t < d; ++t) {
          const double e = x[t] - c[t];
          acc = std::fma(e, e, acc);
        }
        if (acc < bd) { bd = acc; bi = j; }
      }
      labels[r] = bi;
      best[r] = bd;
    }
  };
  threads = std::max(1, std::min(threads, (int)std::max(1LL, n / 4096)));
  std::vector<std::thread> ts;
  const long long per = (n + threads - 1) / threads;
  for (int i = 1; i < threads; ++i) ts.emplace_back(work, std::min(n, i * per), std::min(n, (i + 1) * per));
  work(0, std::min(n, per));
  for (auto& t : ts) t.join();
  return 0;
}

// exact_sums: the correctly rounded per-cluster sums (S) and their remainders (S_lo, nullable) by
// double-double accumulation — the device kernel's result (csrc/kmeans_exact.hip): hi + lo holds the
// running sum exactly while the values' exponents span less than ~2^80, so the order of the additions
// (row order here, sorted chunks there) does not change the rounded total.
static inline void dd_add_h(double& hi, double& lo, double v) {
  const double s = hi + v;
  const double bb = s - hi;
  lo += (hi - (s - bb)) + (v - bb);
  hi = s;
}
static inline void dd_norm_h(double& hi, double& lo) {
  const double s = hi + lo;
  const double bb = s - hi;
  lo = (hi - (s - bb)) + (lo - bb);
  hi = s;
}

CML_HOST_API int cml_exact_sums_host(const double* X, long long n, long long ldx, int d, const long long* labels,
                                     int k, double* S, double* counts, double* S_lo) {
  if (n < 0 || d <= 0 || k <= 0) return -1;
  std::vector<double> lo((size_t)k * d, 0.0);
  std::vector<long long> cnt(k, 0);
  for (long long i = 0; i < (long long)k * d; ++i) S[i] = 0.0;
  for (long long r = 0; r < n; ++r) {
    const long long c = labels[r];
    if (c < 0 || c >= k) return -2;
    ++cnt[c];
    const double* x = X + r * ldx;
    double* s = S + c * d;
    double* l = lo.data() + c * d;
    for (int t = 0; t < d; ++t) dd_add_h(s[t], l[t], x[t]);
  }
  for (long long i = 0; i < (long long)k * d; ++i) {
    dd_norm_h(S[i], lo[i]);
    if (S_lo != nullptr) S_lo[i] = lo[i];
  }
  for (int c = 0; c < k; ++c) counts[c] = (double)cnt[c];
  return 0;
}
