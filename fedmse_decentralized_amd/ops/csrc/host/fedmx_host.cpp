// fedmx host runtime library (C++17, no GPU dependency).
//
// * Multi-threaded headerless numeric CSV reader.  The reference reads every
//   client split with pandas (`load_data`, src/DataLoader/dataloader.py:22-30)
//   and re-parses all CSVs for every sweep combination (~6.3 s per combo for
//   10 Kitsune clients).  Here a file is mmap'ed, split into
//   line-aligned chunks and parsed with std::from_chars (correctly rounded)
//   on a thread pool, straight into a caller-provided float64 buffer.
// * Exact tie-aware ROC-AUC on the host (Mann-Whitney with mid-ranks), the
//   oracle for the device AUC kernel and the fallback for very large sets.
//
// C ABI; loaded with ctypes from fedmse_decentralized_amd/ops/_host.py.

#include <algorithm>
#include <charconv>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <numeric>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    size = static_cast<size_t>(st.st_size);
    if (size == 0) return true;
    void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (p == MAP_FAILED) return false;
    data = static_cast<const char*>(p);
    madvise(p, size, MADV_SEQUENTIAL);
    return true;
  }
  ~MappedFile() {
    if (data) munmap(const_cast<char*>(data), size);
    if (fd >= 0) ::close(fd);
  }
};

inline bool is_blank_line(const char* b, const char* e) {
  for (const char* p = b; p < e; ++p)
    if (*p != ' ' && *p != '\r' && *p != '\t') return false;
  return true;
}

// Parse one line into `out` (cols values). Returns number parsed or -1.
int parse_line(const char* b, const char* e, double* out, int cols) {
  int c = 0;
  const char* p = b;
  while (p < e && c < cols) {
    while (p < e && (*p == ' ' || *p == '\t')) ++p;
    const char* q = p;
    while (q < e && *q != ',' && *q != '\r') ++q;
    // from_chars does not accept a leading '+'
    const char* s = p;
    if (s < q && *s == '+') ++s;
    double v = 0.0;
    if (s == q) {
      v = __builtin_nan("");  // empty field -> NaN (pandas behaviour)
    } else {
      auto r = std::from_chars(s, q, v);
      if (r.ec != std::errc()) {
        // accept "nan"/"inf" spellings that from_chars rejects in some libstdc++
        std::string tok(s, q);
        char* endp = nullptr;
        v = std::strtod(tok.c_str(), &endp);
        if (endp == tok.c_str()) return -1;
      }
    }
    out[c++] = v;
    p = q;
    if (p < e && *p == ',') ++p;
    while (p < e && *p == '\r') ++p;
  }
  return c;
}

}  // namespace

extern "C" {

// Count data rows and columns (columns of the first non-blank line).
int fedmx_csv_shape(const char* path, int64_t* rows, int64_t* cols) {
  MappedFile f;
  if (!f.open(path)) return -1;
  int64_t r = 0, c = 0;
  const char* p = f.data;
  const char* end = f.data + f.size;
  while (p < end) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', end - p));
    const char* le = nl ? nl : end;
    if (!is_blank_line(p, le)) {
      if (r == 0) {
        c = 1;
        for (const char* q = p; q < le; ++q) c += (*q == ',');
      }
      ++r;
    }
    p = nl ? nl + 1 : end;
  }
  *rows = r;
  *cols = c;
  return 0;
}

// Parse into out[rows*cols] (row-major float64). Returns rows parsed or <0.
int64_t fedmx_csv_parse(const char* path, double* out, int64_t rows, int64_t cols, int nthreads) {
  MappedFile f;
  if (!f.open(path)) return -1;
  // index line starts
  std::vector<const char*> starts;
  starts.reserve(static_cast<size_t>(rows) + 1);
  const char* p = f.data;
  const char* end = f.data + f.size;
  while (p < end) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', end - p));
    const char* le = nl ? nl : end;
    if (!is_blank_line(p, le)) starts.push_back(p);
    p = nl ? nl + 1 : end;
  }
  const int64_t n = static_cast<int64_t>(starts.size());
  if (n != rows) return -2;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  std::vector<int> status(nthreads, 0);
  auto work = [&](int t) {
    int64_t a = n * t / nthreads, b = n * (t + 1) / nthreads;
    for (int64_t i = a; i < b; ++i) {
      const char* s = starts[i];
      const char* nl = static_cast<const char*>(memchr(s, '\n', end - s));
      const char* le = nl ? nl : end;
      int got = parse_line(s, le, out + i * cols, static_cast<int>(cols));
      if (got != cols) { status[t] = -3; return; }
    }
  };
  if (n < 2048) { nthreads = 1; status.assign(1, 0); }
  if (nthreads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  for (int s : status) if (s != 0) return s;
  return n;
}

// Exact ROC-AUC (sklearn roc_curve+auc semantics: positives = label!=0,
// ties count 1/2).  Returns NaN if a class is empty or a score is NaN (sklearn
// rejects NaN input; a NaN would also break the sort's strict weak ordering).
double fedmx_roc_auc(const double* score, const int64_t* label, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    if (score[i] != score[i]) return __builtin_nan("");
  std::vector<int64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return score[a] < score[b]; });
  double npos = 0, nneg = 0, rank_sum_pos = 0;
  int64_t i = 0;
  while (i < n) {
    int64_t j = i;
    while (j + 1 < n && score[idx[j + 1]] == score[idx[i]]) ++j;
    double mid = 0.5 * (static_cast<double>(i + 1) + static_cast<double>(j + 1));
    for (int64_t k = i; k <= j; ++k) {
      if (label[idx[k]] != 0) { npos += 1; rank_sum_pos += mid; } else { nneg += 1; }
    }
    i = j + 1;
  }
  if (npos == 0 || nneg == 0) return __builtin_nan("");
  return (rank_sum_pos - npos * (npos + 1) / 2.0) / (npos * nneg);
}

int fedmx_host_abi_version() { return 1; }

}  // extern "C"
