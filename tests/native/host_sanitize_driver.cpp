// Sanitizer driver for the host runtime library ("ASan-enabled
// build for host code").  Built by tests/test_host_sanitizers.py together with
// ops/csrc/host/fedmx_host.cpp under -fsanitize=address,undefined and run as a
// plain executable (no Python, no GPU): the CSV reader is exercised on
// awkward inputs (CRLF, blank lines, missing final newline, NaN/inf, '+'
// signs, short rows, the multi-threaded chunking path) and the exact AUC on
// ties and degenerate label sets.  Any sanitizer report aborts with a nonzero
// exit code; wrong values exit with 1 and a message.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" {
int fedmx_csv_shape(const char* path, int64_t* rows, int64_t* cols);
int64_t fedmx_csv_parse(const char* path, double* out, int64_t rows, int64_t cols, int nthreads);
double fedmx_roc_auc(const double* score, const int64_t* label, int64_t n);
}

static int failures = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

static std::string write_file(const std::string& dir, const char* name, const std::string& body) {
  std::string p = dir + "/" + name;
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) { std::perror("fopen"); std::exit(2); }
  std::fwrite(body.data(), 1, body.size(), f);
  std::fclose(f);
  return p;
}

static void csv_small(const std::string& dir) {
  // CRLF, a blank line, a whitespace-only line, '+' sign, nan/inf, no final newline
  std::string p = write_file(dir, "small.csv", "1,2,3\r\n\n  \t\r\n+4.5,-0.25,nan\r\n1e-3,inf,-inf");
  int64_t r = 0, c = 0;
  CHECK(fedmx_csv_shape(p.c_str(), &r, &c) == 0);
  CHECK(r == 3 && c == 3);
  std::vector<double> out(static_cast<size_t>(r * c));
  CHECK(fedmx_csv_parse(p.c_str(), out.data(), r, c, 4) == 3);
  CHECK(out[0] == 1 && out[1] == 2 && out[2] == 3);
  CHECK(out[3] == 4.5 && out[4] == -0.25 && std::isnan(out[5]));
  CHECK(out[6] == 1e-3 && std::isinf(out[7]) && out[7] > 0 && std::isinf(out[8]) && out[8] < 0);
  // row count mismatch and a short row are reported, not overrun
  CHECK(fedmx_csv_parse(p.c_str(), out.data(), 2, c, 1) == -2);
  std::string q = write_file(dir, "short.csv", "1,2,3\n4,5\n");
  CHECK(fedmx_csv_parse(q.c_str(), out.data(), 2, 3, 1) < 0);
  // empty and missing files
  std::string e = write_file(dir, "empty.csv", "");
  CHECK(fedmx_csv_shape(e.c_str(), &r, &c) == 0 && r == 0);
  CHECK(fedmx_csv_shape((dir + "/does_not_exist.csv").c_str(), &r, &c) < 0);
}

static void csv_threaded(const std::string& dir) {
  // > 2048 rows so the reader takes the multi-threaded path; odd row count
  // and uneven chunk boundaries
  const int rows = 5003, cols = 115;
  std::string body;
  body.reserve(static_cast<size_t>(rows) * cols * 12);
  char buf[64];
  for (int i = 0; i < rows; ++i) {
    for (int j = 0; j < cols; ++j) {
      std::snprintf(buf, sizeof buf, "%.17g", (i * 131 + j * 7) * 0.001 - 3.0);
      body += buf;
      body += (j + 1 < cols) ? "," : (i % 3 ? "\n" : "\r\n");
    }
    if (i % 997 == 0) body += "\n";  // interleaved blank lines
  }
  std::string p = write_file(dir, "big.csv", body);
  int64_t r = 0, c = 0;
  CHECK(fedmx_csv_shape(p.c_str(), &r, &c) == 0);
  CHECK(r == rows && c == cols);
  std::vector<double> out(static_cast<size_t>(r * c));
  for (int nt : {1, 3, 8, 200}) {
    CHECK(fedmx_csv_parse(p.c_str(), out.data(), r, c, nt) == rows);
    bool ok = true;
    for (int i = 0; i < rows && ok; i += 17)
      for (int j = 0; j < cols; ++j)
        if (out[static_cast<size_t>(i) * cols + j] != (i * 131 + j * 7) * 0.001 - 3.0) { ok = false; break; }
    CHECK(ok);
  }
}

static void auc_cases() {
  // all tied -> 0.5; perfect separation -> 1; reversed -> 0; one class -> NaN
  std::vector<double> s = {0.5, 0.5, 0.5, 0.5};
  std::vector<int64_t> l = {0, 1, 0, 1};
  CHECK(std::fabs(fedmx_roc_auc(s.data(), l.data(), 4) - 0.5) < 1e-15);
  s = {0.1, 0.2, 0.8, 0.9};
  l = {0, 0, 1, 1};
  CHECK(fedmx_roc_auc(s.data(), l.data(), 4) == 1.0);
  l = {1, 1, 0, 0};
  CHECK(fedmx_roc_auc(s.data(), l.data(), 4) == 0.0);
  l = {1, 1, 1, 1};
  CHECK(std::isnan(fedmx_roc_auc(s.data(), l.data(), 4)));
  CHECK(std::isnan(fedmx_roc_auc(s.data(), l.data(), 0)));
  s = {0.1, NAN, 0.8, 0.9};
  l = {0, 0, 1, 1};
  CHECK(std::isnan(fedmx_roc_auc(s.data(), l.data(), 4)));
  // partial ties: pos {0.3, 0.5}, neg {0.3, 0.1}: pairs (0.3>0.1)=1,(0.3=0.3)=.5,(0.5>*)=2 -> 3.5/4
  s = {0.3, 0.5, 0.3, 0.1};
  l = {1, 1, 0, 0};
  CHECK(std::fabs(fedmx_roc_auc(s.data(), l.data(), 4) - 0.875) < 1e-15);
  // larger random set against the O(n^2) pair count
  const int n = 3001;
  std::vector<double> rs(n);
  std::vector<int64_t> rl(n);
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    rs[i] = static_cast<double>(x % 97) / 97.0;  // many ties
    rl[i] = (x >> 20) % 3 == 0;
  }
  double wins = 0, np = 0, nn = 0;
  for (int i = 0; i < n; ++i) {
    if (!rl[i]) { nn += 1; continue; }
    np += 1;
    for (int j = 0; j < n; ++j)
      if (!rl[j]) wins += rs[i] > rs[j] ? 1.0 : (rs[i] == rs[j] ? 0.5 : 0.0);
  }
  CHECK(std::fabs(fedmx_roc_auc(rs.data(), rl.data(), n) - wins / (np * nn)) < 1e-12);
}

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: %s <scratch dir>\n", argv[0]); return 2; }
  const std::string dir = argv[1];
  csv_small(dir);
  csv_threaded(dir);
  auc_cases();
  if (failures) { std::fprintf(stderr, "%d check(s) failed\n", failures); return 1; }
  std::printf("host sanitizer driver: all checks passed\n");
  return 0;
}
