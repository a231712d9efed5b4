// Host AddressSanitizer / UBSan harness for the native CSV tokenizer + parser (SURVEY.md §5.2:
// sanitizers run on host code only). Randomised RFC-4180 inputs: quoted fields with embedded
// separators / quotes / newlines, unterminated quotes, empty and over-long fields, ragged rows,
// CRLF, header or not; every column type; 1 and 4 parser threads.
//   g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -pthread csv_fuzz.cpp -o csv_fuzz
#include "../../clustermachinelearningforhospitalnetworks_apache_spark_amd/_native/host/csv.cpp"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

extern "C" long long cml_csv_index(const char*, long long, char, int, long long*, long long);
extern "C" int cml_csv_parse(const char*, long long, const long long*, long long, int, char, char, const int*, void**,
                             unsigned char**, int);
extern "C" long long cml_csv_gather_strings(const char*, const long long*, const unsigned char*, long long, char,
                                            long long*, char*);

static std::string field(std::mt19937& g) {
  static const char* pieces[] = {"", "1", "-42", "3.25", "1e308", "nan", "true", "false", "2025-03-31 22:00:00",
                                 "2025-03-31", "abc", "\"q,uo\"\"ted\"", "\"multi\nline\"", "\"unterminated",
                                 "99999999999999999999", "  7 ", "\"\"", "x\"y", "1.5e-3", "T"};
  std::string s = pieces[g() % (sizeof(pieces) / sizeof(pieces[0]))];
  if (g() % 17 == 0) s += std::string(g() % 300, 'z');
  return s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  std::mt19937 g(12345);
  long long total_rows = 0;
  for (int it = 0; it < iters; ++it) {
    const int ncols = 1 + g() % 8;
    const int nrows = g() % 40;
    std::string buf;
    const bool header = g() % 2;
    if (header) {
      for (int c = 0; c < ncols; ++c) buf += (c ? "," : "") + std::string("c") + std::to_string(c);
      buf += "\n";
    }
    for (int r = 0; r < nrows; ++r) {
      const int nf = ncols + (g() % 5 == 0 ? (int)(g() % 3) - 1 : 0);  // ragged rows
      for (int c = 0; c < nf; ++c) buf += (c ? "," : "") + field(g);
      buf += (g() % 4 == 0) ? "\r\n" : "\n";
    }
    if (g() % 3 == 0 && !buf.empty()) buf.pop_back();  // no trailing newline
    std::vector<long long> starts(buf.size() + 2);
    const long long n = cml_csv_index(buf.data(), (long long)buf.size(), '"', header ? 1 : 0, starts.data(),
                                      (long long)starts.size());
    if (n < 0) continue;
    std::vector<int> types(ncols);
    std::vector<std::vector<unsigned char>> store(ncols);
    std::vector<std::vector<unsigned char>> valid(ncols, std::vector<unsigned char>(n + 1));
    std::vector<void*> data(ncols);
    std::vector<unsigned char*> vptr(ncols);
    for (int c = 0; c < ncols; ++c) {
      types[c] = g() % 8;
      store[c].resize((size_t)(n + 1) * 24);  // widest slot: string triple (3 x int64)
      data[c] = store[c].data();
      vptr[c] = valid[c].data();
    }
    const int rc = cml_csv_parse(buf.data(), (long long)buf.size(), starts.data(), n, ncols, ',', '"', types.data(),
                                 data.data(), vptr.data(), 1 + (int)(g() % 4));
    if (rc != 0) continue;
    for (int c = 0; c < ncols; ++c) {
      if (types[c] != 0) continue;
      const long long* trip = reinterpret_cast<const long long*>(store[c].data());
      const long long bytes = cml_csv_gather_strings(buf.data(), trip, vptr[c], n, '"', nullptr, nullptr);
      std::vector<long long> offs(n + 1);
      std::vector<char> chars((size_t)bytes + 1);
      cml_csv_gather_strings(buf.data(), trip, vptr[c], n, '"', offs.data(), chars.data());
      if (offs[n] != bytes) return 2;
    }
    total_rows += n;
  }
  std::printf("csv_fuzz ok: %d inputs, %lld rows parsed\n", iters, total_rows);
  return 0;
}
