// Host-side CSV tokenizer / typed parser (K1 in SURVEY.md §2.5).
//
// Replaces Spark's per-row CSV parsing on executors for the streaming file source and
// spark.read.csv (ref.py:75-78).  Two passes over an in-memory file image:
//   1. cml_csv_index   — find record starts (RFC-4180 quoting: separators and newlines inside
//                        "..." do not split, "" is an escaped quote), optional header skip;
//   2. cml_csv_parse   — split each record into fields and convert them straight into typed,
//                        column-major output buffers (int32/int64/float64/float32/bool/
//                        timestamp-µs/date-days) plus a validity byte per cell; string cells
//                        are returned as (offset, length, needs-unquote) triples into the
//                        image.  Records are distributed over std::threads in contiguous
//                        blocks, so the output is identical for any thread count.
// PERMISSIVE semantics like Spark: empty or unparseable cells become null, short records pad
// with nulls, extra fields are ignored.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#define CML_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

enum ColType : int { kString = 0, kInt32 = 1, kInt64 = 2, kFloat64 = 3, kTimestamp = 4, kBool = 5, kFloat32 = 6, kDate = 7 };

inline long long days_from_civil(long long y, unsigned m, unsigned d) {
  y -= m <= 2;
  const long long era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = static_cast<unsigned>(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + static_cast<long long>(doe) - 719468;
}

inline bool parse_uint(const char*& p, const char* e, int ndig_min, int ndig_max, long long& out) {
  long long v = 0;
  int n = 0;
  while (p < e && n < ndig_max && *p >= '0' && *p <= '9') {
    v = v * 10 + (*p - '0');
    ++p;
    ++n;
  }
  out = v;
  return n >= ndig_min;
}

// "YYYY-MM-DD[( |T)HH:MM[:SS[.ffffff]]][Z]" -> microseconds since epoch (UTC)
bool parse_timestamp(const char* p, const char* e, long long& us, bool date_only) {
  long long y, mo, d, hh = 0, mm = 0, ss = 0, frac = 0;
  if (!parse_uint(p, e, 4, 4, y) || p >= e || *p++ != '-') return false;
  if (!parse_uint(p, e, 1, 2, mo) || p >= e || *p++ != '-') return false;
  if (!parse_uint(p, e, 1, 2, d)) return false;
  if (p < e && (*p == ' ' || *p == 'T')) {
    ++p;
    if (!parse_uint(p, e, 1, 2, hh) || p >= e || *p++ != ':') return false;
    if (!parse_uint(p, e, 1, 2, mm)) return false;
    if (p < e && *p == ':') {
      ++p;
      if (!parse_uint(p, e, 1, 2, ss)) return false;
      if (p < e && *p == '.') {
        ++p;
        int n = 0;
        while (p < e && *p >= '0' && *p <= '9') {
          if (n < 6) { frac = frac * 10 + (*p - '0'); ++n; }
          ++p;
        }
        while (n < 6) { frac *= 10; ++n; }
      }
    }
  }
  if (p < e && *p == 'Z') ++p;
  while (p < e && (*p == ' ' || *p == '\r')) ++p;
  if (p != e) return false;
  if (mo < 1 || mo > 12 || d < 1 || d > 31 || hh > 23 || mm > 59 || ss > 60) return false;
  const long long days = days_from_civil(y, (unsigned)mo, (unsigned)d);
  us = date_only ? days : ((days * 86400 + hh * 3600 + mm * 60 + ss) * 1000000LL + frac);
  return true;
}

// Decimal integer without a copy: [+-]digits. False on anything else or overflow of 18+ digits.
inline bool fast_int(const char* b, const char* e, long long& out) {
  bool neg = false;
  if (b < e && (*b == '-' || *b == '+')) { neg = *b == '-'; ++b; }
  if (b == e || e - b > 18) return false;
  long long v = 0;
  for (; b < e; ++b) {
    const unsigned d = (unsigned)(*b - '0');
    if (d > 9) return false;
    v = v * 10 + d;
  }
  out = neg ? -v : v;
  return true;
}

// Clinger's fast path: [+-]digits[.digits][(e|E)[+-]digits] with at most 19 significant digits whose
// value fits 2^53 and a decimal exponent in [-22, 22] is exactly one correctly rounded multiply or
// divide by an exact power of ten. Anything else returns false (the caller uses strtod).
inline bool fast_double(const char* b, const char* e, double& out) {
  static const double kPow10[] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  bool neg = false;
  if (b < e && (*b == '-' || *b == '+')) { neg = *b == '-'; ++b; }
  unsigned long long m = 0;
  int nd = 0, ex = 0;
  bool any = false;
  for (; b < e && (unsigned)(*b - '0') <= 9; ++b) {
    any = true;
    if (nd < 19) { m = m * 10 + (unsigned)(*b - '0'); if (m) ++nd; }
    else ++ex;
  }
  if (b < e && *b == '.') {
    ++b;
    for (; b < e && (unsigned)(*b - '0') <= 9; ++b) {
      any = true;
      if (nd < 19) { m = m * 10 + (unsigned)(*b - '0'); if (m) ++nd; --ex; }
    }
  }
  if (!any) return false;
  if (b < e && (*b == 'e' || *b == 'E')) {
    ++b;
    bool eneg = false;
    if (b < e && (*b == '-' || *b == '+')) { eneg = *b == '-'; ++b; }
    if (b == e) return false;
    int x = 0;
    for (; b < e && (unsigned)(*b - '0') <= 9; ++b) { if (x < 10000) x = x * 10 + (*b - '0'); }
    ex += eneg ? -x : x;
  }
  if (b != e) return false;
  if (m > (1ULL << 53) || ex < -22 || ex > 22) return false;
  double v = (double)m;
  v = ex < 0 ? v / kPow10[-ex] : v * kPow10[ex];
  out = neg ? -v : v;
  return true;
}

inline void trim(const char*& b, const char*& e) {
  while (b < e && (*b == ' ' || *b == '\t')) ++b;
  while (e > b && (e[-1] == ' ' || e[-1] == '\t' || e[-1] == '\r')) --e;
}

struct Outputs {
  int ncols;
  const int* types;
  void** data;               // per column: typed array [nrows] (strings: int64 triples [nrows*3])
  unsigned char** valid;     // per column: [nrows]
};

void store_cell(const Outputs& o, int c, long long r, const char* b, const char* e, bool quoted, bool has_esc) {
  unsigned char* v = o.valid[c];
  if (o.types[c] != kString) trim(b, e);
  if (b == e && (!quoted || o.types[c] != kString)) {  // "" is an empty string, but a null number
    v[r] = 0;
    if (o.types[c] == kString) {
      long long* t = static_cast<long long*>(o.data[c]) + 3 * r;
      t[0] = 0; t[1] = 0; t[2] = 0;
    }
    return;
  }
  char buf[96];
  switch (o.types[c]) {
    case kString: {
      long long* t = static_cast<long long*>(o.data[c]) + 3 * r;
      t[0] = (long long)(intptr_t)b;  // absolute pointer; converted to an offset by the caller
      t[1] = (long long)(e - b);
      t[2] = has_esc ? 1 : 0;
      v[r] = 1;
      return;
    }
    case kInt32:
    case kInt64: {
      long long fi;
      if (fast_int(b, e, fi)) {
        if (o.types[c] == kInt32) {
          if (fi < INT32_MIN || fi > INT32_MAX) { v[r] = 0; return; }
          static_cast<int32_t*>(o.data[c])[r] = (int32_t)fi;
        } else {
          static_cast<int64_t*>(o.data[c])[r] = fi;
        }
        v[r] = 1;
        return;
      }
      const size_t n = std::min<size_t>(e - b, sizeof(buf) - 1);
      memcpy(buf, b, n);
      buf[n] = 0;
      char* end = nullptr;
      errno = 0;
      long long x = strtoll(buf, &end, 10);
      bool ok = end == buf + n && errno == 0;
      if (!ok) {  // accept "3.0"-style integers like Spark's permissive cast? no: Spark nulls them
        v[r] = 0;
        return;
      }
      if (o.types[c] == kInt32) {
        if (x < INT32_MIN || x > INT32_MAX) { v[r] = 0; return; }
        static_cast<int32_t*>(o.data[c])[r] = (int32_t)x;
      } else {
        static_cast<int64_t*>(o.data[c])[r] = x;
      }
      v[r] = 1;
      return;
    }
    case kFloat64:
    case kFloat32: {
      double fx;
      if (fast_double(b, e, fx)) {
        if (o.types[c] == kFloat64) static_cast<double*>(o.data[c])[r] = fx;
        else static_cast<float*>(o.data[c])[r] = (float)fx;
        v[r] = 1;
        return;
      }
      const size_t n = std::min<size_t>(e - b, sizeof(buf) - 1);
      memcpy(buf, b, n);
      buf[n] = 0;
      char* end = nullptr;
      double x = strtod(buf, &end);
      if (end != buf + n) { v[r] = 0; return; }
      if (o.types[c] == kFloat64) static_cast<double*>(o.data[c])[r] = x;
      else static_cast<float*>(o.data[c])[r] = (float)x;
      v[r] = 1;
      return;
    }
    case kBool: {
      const size_t n = e - b;
      bool val;
      if (n == 4 && strncasecmp(b, "true", 4) == 0) val = true;
      else if (n == 5 && strncasecmp(b, "false", 5) == 0) val = false;
      else { v[r] = 0; return; }
      static_cast<unsigned char*>(o.data[c])[r] = val;
      v[r] = 1;
      return;
    }
    case kTimestamp:
    case kDate: {
      long long us = 0;
      const bool date_only = o.types[c] == kDate;
      if (!parse_timestamp(b, e, us, date_only)) { v[r] = 0; return; }
      if (date_only) static_cast<int32_t*>(o.data[c])[r] = (int32_t)us;
      else static_cast<int64_t*>(o.data[c])[r] = us;
      v[r] = 1;
      return;
    }
    default:
      v[r] = 0;
  }
}

void parse_record(const char* p, const char* end, char sep, char quote, const Outputs& o, long long r) {
  int c = 0;
  while (c < o.ncols) {
    const char* fb;
    const char* fe;
    bool quoted = false, esc = false;
    if (p < end && *p == quote) {
      quoted = true;
      ++p;
      fb = p;
      while (p < end) {
        if (*p == quote) {
          if (p + 1 < end && p[1] == quote) { esc = true; p += 2; continue; }
          break;
        }
        ++p;
      }
      fe = p;
      if (p < end) ++p;  // closing quote
      while (p < end && *p != sep && *p != '\n') ++p;
    } else {
      fb = p;
      while (p < end && *p != sep && *p != '\n') ++p;
      fe = p;
    }
    store_cell(o, c, r, fb, fe, quoted, esc);
    ++c;
    if (p < end && *p == sep) {
      ++p;
      continue;
    }
    break;  // end of record
  }
  for (; c < o.ncols; ++c) store_cell(o, c, r, p, p, false, false);  // short record: nulls
}

}  // namespace

// Record starts of `buf`: returns the number of records (after skipping `skip_header` records),
// writes at most `cap` starts (pass cap = 0 to only count). Blank lines are skipped.
CML_HOST_API long long cml_csv_index(const char* buf, long long len, char quote, int skip_header, long long* starts,
                                     long long cap) {
  long long n = 0;
  long long i = 0;
  int skipped = 0;
  while (i < len) {
    const long long s = i;
    bool inq = false;
    while (i < len) {
      const char ch = buf[i];
      if (ch == quote) inq = !inq;
      else if (ch == '\n' && !inq) break;
      ++i;
    }
    long long e = i;
    if (i < len) ++i;  // consume '\n'
    while (e > s && (buf[e - 1] == '\r' || buf[e - 1] == ' ')) --e;
    if (e == s) continue;  // blank line
    if (skipped < skip_header) { ++skipped; continue; }
    if (n < cap && starts) starts[n] = s;
    ++n;
  }
  return n;
}

// Multithreaded record index. Phase 1: each thread counts the quote characters of its byte range;
// the prefix parity gives the quoting state at every range start. Phase 2: each thread lists the
// record starts (first byte after an unquoted newline) of its range. The header / blank-line rules
// of cml_csv_index then run over the merged list. `starts` needs room for (#newlines + 1) entries.
CML_HOST_API long long cml_csv_index_mt(const char* buf, long long len, char quote, int skip_header,
                                        long long* starts, long long cap, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (len < (1LL << 20)) nthreads = 1;
  const long long per = (len + nthreads - 1) / nthreads;
  std::vector<long long> nq(nthreads, 0);
  std::vector<std::vector<long long>> brk(nthreads);
  auto count_q = [&](int t) {
    const long long a = t * per, b = std::min(len, a + per);
    long long q = 0;
    for (long long i = a; i < b; ++i) q += buf[i] == quote;
    nq[t] = q;
  };
  auto scan = [&](int t, bool inq) {
    const long long a = t * per, b = std::min(len, a + per);
    std::vector<long long>& out = brk[t];
    out.reserve((size_t)((b - a) / 32 + 16));
    if (nq[t] == 0 && !inq) {  // no quotes in this range: memchr over the newlines
      const char* p = buf + a;
      const char* end = buf + b;
      while (p < end) {
        const void* hit = std::memchr(p, '\n', (size_t)(end - p));
        if (hit == nullptr) break;
        const char* q = static_cast<const char*>(hit);
        out.push_back(q - buf);
        p = q + 1;
      }
      return;
    }
    for (long long i = a; i < b; ++i) {
      const char ch = buf[i];
      if (ch == quote) inq = !inq;
      else if (ch == '\n' && !inq) out.push_back(i);
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(count_q, t);
    count_q(0);
    for (auto& x : th) x.join();
  }
  {
    std::vector<std::thread> th;
    long long q = 0;
    std::vector<bool> state(nthreads);
    for (int t = 0; t < nthreads; ++t) { state[t] = (q & 1) != 0; q += nq[t]; }
    for (int t = 1; t < nthreads; ++t) th.emplace_back(scan, t, (bool)state[t]);
    scan(0, false);
    for (auto& x : th) x.join();
  }
  // records: [prev newline + 1, newline) in order; trailing record without a newline
  long long n = 0, s = 0;
  int skipped = 0;
  auto emit = [&](long long a, long long e) {
    long long ee = e;
    while (ee > a && (buf[ee - 1] == '\r' || buf[ee - 1] == ' ')) --ee;
    if (ee == a) return;
    if (skipped < skip_header) { ++skipped; return; }
    if (n < cap && starts) starts[n] = a;
    ++n;
  };
  for (int t = 0; t < nthreads; ++t)
    for (long long nl : brk[t]) { emit(s, nl); s = nl + 1; }
  if (s < len) emit(s, len);
  return n;
}

// Parse `nrows` records starting at byte offsets `starts` into column buffers. String cells are
// written as (byte offset into buf, byte length, needs-unquote) triples. Returns 0 on success.
CML_HOST_API int cml_csv_parse(const char* buf, long long len, const long long* starts, long long nrows, int ncols,
                               char sep, char quote, const int* types, void** data, unsigned char** valid,
                               int nthreads) {
  Outputs o{ncols, types, data, valid};
  if (nthreads < 1) nthreads = 1;
  const long long per = (nrows + nthreads - 1) / nthreads;
  auto work = [&](long long r0, long long r1) {
    for (long long r = r0; r < r1; ++r) {
      const char* p = buf + starts[r];
      const char* e = r + 1 < nrows ? buf + starts[r + 1] : buf + len;
      // the record ends at the first unquoted newline; parse_record stops there itself
      parse_record(p, e, sep, quote, o, r);
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    const long long r0 = t * per, r1 = std::min(nrows, r0 + per);
    if (r0 >= r1) break;
    if (t == nthreads - 1 || r1 == nrows) { work(r0, r1); break; }
    th.emplace_back(work, r0, r1);
  }
  for (auto& x : th) x.join();
  // convert string pointers to offsets
  for (int c = 0; c < ncols; ++c) {
    if (types[c] != kString) continue;
    long long* t = static_cast<long long*>(data[c]);
    for (long long r = 0; r < nrows; ++r)
      if (valid[c][r]) t[3 * r] -= (long long)(intptr_t)buf;
  }
  return 0;
}

// Days-from-civil exposed for the Python side (tests / scalar conversions).
CML_HOST_API long long cml_days_from_civil(long long y, int m, int d) { return days_from_civil(y, (unsigned)m, (unsigned)d); }

// Arrow-layout materialisation of a parsed string column: trip = n x (offset, len, needs_unquote)
// from cml_csv_parse, valid = n bytes. First call with data == nullptr returns the byte total
// (after "" -> " unescaping); second call fills offsets[n+1] (int64) and data.
CML_HOST_API long long cml_csv_gather_strings(const char* buf, const long long* trip, const unsigned char* valid,
                                              long long n, char quote, long long* offsets, char* data) {
  long long pos = 0;
  for (long long r = 0; r < n; ++r) {
    if (offsets != nullptr) offsets[r] = pos;
    if (!valid[r]) continue;
    const char* s = buf + trip[3 * r];
    const long long len = trip[3 * r + 1];
    if (!trip[3 * r + 2]) {
      if (data != nullptr) std::memcpy(data + pos, s, (size_t)len);
      pos += len;
    } else {
      for (long long i = 0; i < len; ++i) {
        if (s[i] == quote && i + 1 < len && s[i + 1] == quote) ++i;  // "" -> "
        if (data != nullptr) data[pos] = s[i];
        ++pos;
      }
    }
  }
  if (offsets != nullptr) offsets[n] = pos;
  return pos;
}

// ------------------------------------------------------------------------------------------ dictionary
// Dictionary encoding of a parsed string column (strings are dictionary-encoded). Each thread
// hashes a contiguous block of rows into a local dictionary (first-appearance order); the blocks'
// dictionaries are merged in block order, so code c is the c-th distinct string in row order for any
// thread count, and local codes are remapped in parallel. Nulls get code -1.
namespace {
struct DictResult {
  std::vector<int> codes;
  std::vector<std::vector<std::string>> owned;  // per-thread unescaped strings ("" -> "), never moved
  std::vector<std::string_view> values;    // global dictionary in code order
};
}  // namespace

CML_HOST_API void* cml_dict_build(const char* buf, const long long* trip, const unsigned char* valid, long long n,
                                  char quote, int nthreads) {
  auto* res = new DictResult();
  res->codes.assign((size_t)n, -1);
  if (nthreads < 1) nthreads = 1;
  if (n < 65536) nthreads = 1;
  const long long per = (n + nthreads - 1) / nthreads;
  std::vector<std::vector<std::string_view>> ldict(nthreads);
  res->owned.resize((size_t)nthreads);
  auto& lowned = res->owned;
  auto work = [&](int t) {
    const long long r0 = t * per, r1 = std::min(n, r0 + per);
    std::unordered_map<std::string_view, int> m;
    m.reserve(1024);
    std::vector<std::string>& own = lowned[t];
    // reserve so that string_views into `own` stay valid while it grows
    long long nesc = 0;
    for (long long r = r0; r < r1; ++r) nesc += valid[r] && trip[3 * r + 2];
    own.reserve((size_t)nesc);
    for (long long r = r0; r < r1; ++r) {
      if (!valid[r]) continue;
      const char* p = buf + trip[3 * r];
      const long long len = trip[3 * r + 1];
      std::string_view key(p, (size_t)len);
      if (trip[3 * r + 2]) {
        std::string u;
        u.reserve((size_t)len);
        for (long long i = 0; i < len; ++i) {
          if (p[i] == quote && i + 1 < len && p[i + 1] == quote) ++i;
          u.push_back(p[i]);
        }
        own.push_back(std::move(u));
        key = std::string_view(own.back());
      }
      auto it = m.find(key);
      int code;
      if (it == m.end()) {
        code = (int)ldict[t].size();
        ldict[t].push_back(key);
        m.emplace(key, code);
      } else {
        code = it->second;
      }
      res->codes[(size_t)r] = code;
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
  }
  std::unordered_map<std::string_view, int> g;
  std::vector<std::vector<int>> remap(nthreads);
  for (int t = 0; t < nthreads; ++t) {
    remap[t].resize(ldict[t].size());
    for (size_t i = 0; i < ldict[t].size(); ++i) {
      auto it = g.find(ldict[t][i]);
      if (it == g.end()) {
        const int c = (int)res->values.size();
        res->values.push_back(ldict[t][i]);
        g.emplace(ldict[t][i], c);
        remap[t][i] = c;
      } else {
        remap[t][i] = it->second;
      }
    }
  }
  {
    auto fix = [&](int t) {
      const long long r0 = t * per, r1 = std::min(n, r0 + per);
      for (long long r = r0; r < r1; ++r) {
        int& c = res->codes[(size_t)r];
        if (c >= 0) c = remap[t][(size_t)c];
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(fix, t);
    fix(0);
    for (auto& x : th) x.join();
  }
  return res;
}

// dictionary size: entries and total bytes
CML_HOST_API void cml_dict_size(void* h, long long* count, long long* bytes) {
  auto* res = static_cast<DictResult*>(h);
  long long b = 0;
  for (auto& v : res->values) b += (long long)v.size();
  *count = (long long)res->values.size();
  *bytes = b;
}

// codes [n] (int32), dictionary as Arrow large-string offsets [count+1] + data
CML_HOST_API void cml_dict_fill(void* h, int* codes, long long* offsets, char* data) {
  auto* res = static_cast<DictResult*>(h);
  std::memcpy(codes, res->codes.data(), res->codes.size() * sizeof(int));
  long long pos = 0;
  for (size_t c = 0; c < res->values.size(); ++c) {
    offsets[c] = pos;
    std::memcpy(data + pos, res->values[c].data(), res->values[c].size());
    pos += (long long)res->values[c].size();
  }
  offsets[res->values.size()] = pos;
}

CML_HOST_API void cml_dict_free(void* h) { delete static_cast<DictResult*>(h); }
