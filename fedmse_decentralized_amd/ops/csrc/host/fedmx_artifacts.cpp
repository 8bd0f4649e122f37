// Batched per-round checkpoint artefact writer (C++17, no GPU dependency).
//
// Every round the reference rewrites, for each trained client, its
// best-validation `model.cpt` (legacy torch serialisation, written by
// `save_model`, src/Trainer/client_trainer.py:337-350) and its
// `training_tracking.pkl` (pickle protocol 4 of [(train_loss, valid_loss)],
// :416/:419).  In Python that is ~70-150 us of GIL-holding work per client
// (gather of the canonical parameters, template patch, pickle, two writes),
// which made the background writer the bound of large federations (64
// clients: 4.8 ms of writer time per round).  Here ONE call renders and
// writes every client of a round on a few threads, without the GIL:
//
//   * model.cpt: the byte template of the legacy format (produced once by
//     torch.save itself, io/checkpoint.py:_CptTemplate) with the canonical
//     parameters gathered from the padded host snapshot row and patched into
//     the storage regions.  The file has a fixed size, so it stays mapped
//     (MAP_SHARED, fedmx_map_file): the template bytes are written once when
//     the mapping is made and a round only copies the 27 KB of parameters
//     into the page cache — no system call per file and round.
//   * training_tracking.pkl: the exact bytes pickle.dumps(list_of_tuples,
//     protocol=4) produces (PROTO 4, FRAME when the body is >= 4 bytes,
//     EMPTY_LIST MEMOIZE, MARK ... APPENDS (or APPEND for one element),
//     BINFLOAT x2 TUPLE2 MEMOIZE per epoch, STOP); tested byte-for-byte
//     against Python's pickle (tests/test_files.py).
//
// A file shrinks (ftruncate) only when its new content is shorter than what
// it held, so a steady-state rewrite is a single pwrite.
//
// C ABI; loaded with ctypes from fedmse_decentralized_amd/ops/_host.py.

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <immintrin.h>
#include <mutex>
#include <string>
#include <unordered_map>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

inline void put_be_f64(std::vector<uint8_t>& b, double v) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  for (int i = 7; i >= 0; --i) b.push_back(static_cast<uint8_t>(u >> (8 * i)));
}

inline void put_le_u64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = static_cast<uint8_t>(v >> (8 * i));
}

// pickle.dumps([(a0, b0), (a1, b1), ...], protocol=4) for n <= 1000 (one
// APPENDS batch, one frame).  Returns false for larger n (caller falls back).
bool pickle_tracking(const double* t, int n, std::vector<uint8_t>& out) {
  if (n < 0 || n > 1000) return false;
  std::vector<uint8_t> body;
  body.reserve(4 + 20 * static_cast<size_t>(n));
  body.push_back(']');   // EMPTY_LIST
  body.push_back(0x94);  // MEMOIZE
  if (n >= 2) body.push_back('(');  // MARK
  for (int i = 0; i < n; ++i) {
    body.push_back('G');
    put_be_f64(body, t[2 * i]);
    body.push_back('G');
    put_be_f64(body, t[2 * i + 1]);
    body.push_back(0x86);  // TUPLE2
    body.push_back(0x94);  // MEMOIZE
  }
  if (n >= 2) body.push_back('e');       // APPENDS
  else if (n == 1) body.push_back('a');  // APPEND
  body.push_back('.');                   // STOP
  out.clear();
  out.push_back(0x80);  // PROTO
  out.push_back(4);
  if (body.size() >= 4) {   // pickle's framer skips frames shorter than 4 bytes
    uint8_t hdr[9];
    hdr[0] = 0x95;  // FRAME
    put_le_u64(hdr + 1, body.size());
    out.insert(out.end(), hdr, hdr + 9);
  }
  out.insert(out.end(), body.begin(), body.end());
  return true;
}

// First content of a new (empty) file through a temporary shared mapping:
// on the GPU hosts' filesystem the first write(2) into a new file costs
// ~2.8 ms (block allocation on the caller's thread) while a mapping's dirty
// pages are allocated by the kernel's writeback (~0.09 ms for a new 28 KB
// model.cpt, scripts/first_write_probe.py).
int write_new_mapped(int fd, const uint8_t* p, size_t n) {
  if (ftruncate(fd, static_cast<off_t>(n)) != 0) return -errno;
  void* m = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) return -errno;
  std::memcpy(m, p, n);
  munmap(m, n);
  return 0;
}

int write_all(int fd, const uint8_t* p, size_t n, int64_t* size_io) {
  if (*size_io == 0 && n > 0) {
    const int rc = write_new_mapped(fd, p, n);
    if (rc == 0) {
      *size_io = static_cast<int64_t>(n);
      return 0;
    }
  }
  size_t off = 0;
  while (off < n) {
    const ssize_t w = pwrite(fd, p + off, n - off, static_cast<off_t>(off));
    if (w < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    off += static_cast<size_t>(w);
  }
  if (*size_io > static_cast<int64_t>(n)) {
    if (ftruncate(fd, static_cast<off_t>(n)) != 0) return -errno;
  }
  *size_io = static_cast<int64_t>(n);
  return 0;
}

}  // namespace

extern "C" {

// Bytes of pickle.dumps(tracking, protocol=4) into out (capacity cap);
// returns the length, -1 if unsupported, -2 if cap is too small.
int64_t fedmx_pickle_tracking(const double* t, int32_t n, uint8_t* out, int64_t cap) {
  std::vector<uint8_t> b;
  if (!pickle_tracking(t, n, b)) return -1;
  if (static_cast<int64_t>(b.size()) > cap) return -2;
  std::memcpy(out, b.data(), b.size());
  return static_cast<int64_t>(b.size());
}

// Shared writable mapping of an open file, resized to exactly `size` bytes
// (nullptr on failure).
void* fedmx_map_file(int32_t fd, int64_t size) {
  if (size <= 0 || ftruncate(fd, static_cast<off_t>(size)) != 0) return nullptr;
  void* p = mmap(nullptr, static_cast<size_t>(size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  return p == MAP_FAILED ? nullptr : p;
}

int32_t fedmx_unmap_file(void* p, int64_t size) {
  return munmap(p, static_cast<size_t>(size)) == 0 ? 0 : -errno;
}

// One round's artefacts for n_jobs clients.
//   snap [*, snap_stride] f32 host snapshot; canon_idx[n_canon] gathers the
//   canonical parameter vector out of a padded row; tpl/regions: the legacy
//   model.cpt template and its (byte pos, count, canonical offset) triples.
//   Job j: snapshot row rows[j]; when improved[j], the parameters are patched
//   into the mapped model.cpt at cpt_dst[j] (template bytes already there);
//   tracking trk[j*trk_stride*2 ...] of trk_len[j] epochs into fd_trk[j].
//   size_trk: current tracking file sizes (in/out).
// Returns 0, or the first negative errno / -1 (tracking too long) per job in
// status[j] and the count of failed jobs as the (negative) return value.
int32_t fedmx_write_artifacts(const float* snap, int64_t snap_stride, const int32_t* canon_idx, int32_t n_canon,
                              const uint8_t* tpl, int64_t tpl_len, const int64_t* regions, int32_t n_regions,
                              int32_t n_jobs, const int32_t* rows, const int32_t* improved, const int64_t* cpt_dst,
                              const int32_t* fd_trk, int64_t* size_trk, const double* trk,
                              const int32_t* trk_len, int32_t trk_stride, int32_t* status, int32_t n_threads) {
  if (n_jobs <= 0) return 0;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > n_jobs) n_threads = n_jobs;
  (void)tpl;
  (void)tpl_len;
  auto work = [&](int j0, int j1) {
    std::vector<float> canon(static_cast<size_t>(n_canon));
    std::vector<uint8_t> pk;
    for (int j = j0; j < j1; ++j) {
      int st = 0;
      if (improved[j]) {
        uint8_t* dst = reinterpret_cast<uint8_t*>(cpt_dst[j]);
        const float* row = snap + static_cast<int64_t>(rows[j]) * snap_stride;
        for (int i = 0; i < n_canon; ++i) canon[i] = row[canon_idx[i]];
        for (int r = 0; r < n_regions; ++r) {
          const int64_t pos = regions[3 * r], cnt = regions[3 * r + 1], off = regions[3 * r + 2];
          std::memcpy(dst + pos, canon.data() + off, static_cast<size_t>(cnt) * 4);
        }
      }
      if (st == 0) {
        if (!pickle_tracking(trk + static_cast<int64_t>(j) * trk_stride * 2, trk_len[j], pk))
          st = -1;
        else
          st = write_all(fd_trk[j], pk.data(), pk.size(), &size_trk[j]);
      }
      status[j] = st;
    }
  };
  if (n_threads == 1) {
    work(0, n_jobs);
  } else {
    std::vector<std::thread> th;
    const int per = (n_jobs + n_threads - 1) / n_threads;
    for (int t = 0; t < n_threads; ++t) {
      const int j0 = t * per, j1 = std::min(n_jobs, j0 + per);
      if (j0 < j1) th.emplace_back(work, j0, j1);
    }
    for (auto& x : th) x.join();
  }
  int32_t bad = 0;
  for (int j = 0; j < n_jobs; ++j) bad += status[j] != 0;
  return -bad;
}

// ---------------------------------------------------------------------------
// Asynchronous native writer thread.  The device-resident round protocol
// collects round r's results while the GPU already runs r+1 / r+2; handing
// the checkpoint writes to a Python thread made them wait for the GIL behind
// the enqueueing main thread (64 clients: ~5 ms of GIL waits per round for
// ~0.2 ms of work).  Here a submit copies the job's small arrays and returns
// a ticket; a C++ thread patches the mapped model.cpt files and writes the
// tracking pickles; fedmx_writer_wait(ticket) blocks (GIL released by
// ctypes) until that job is done — the snapshot slot it reads may then be
// reused.
namespace {

struct WJob {
  const float* snap;
  int64_t stride;
  std::vector<int32_t> rows, improved, trk_len;
  std::vector<std::string> cpt_path, trk_path;
  std::vector<double> trk;
  int32_t trk_stride;
  int64_t ticket;
};

// mkdir -p of the directory holding `path` (a client's save directory)
bool make_parents(const std::string& path) {
  const size_t slash = path.rfind('/');
  if (slash == std::string::npos || slash == 0) return false;
  std::string dir = path.substr(0, slash);
  for (size_t i = 1; i <= dir.size(); ++i) {
    if (i == dir.size() || dir[i] == '/') {
      const std::string part = dir.substr(0, i);
      if (mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
  }
  return true;
}

struct FileEnt {
  int fd = -1;
  uint8_t* map = nullptr;   // model.cpt: shared mapping of the whole file
  int64_t size = -1;        // tracking: current file size (-1: unknown)
};

struct Writer {
  std::vector<int32_t> canon_idx;
  std::vector<int64_t> regions;
  std::vector<uint8_t> tpl;   // legacy model.cpt template
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::deque<WJob> q;
  int64_t next_ticket = 0, done_ticket = 0;
  int32_t first_error = 0;
  bool stop = false, release = false;
  std::unordered_map<std::string, FileEnt> files;   // writer thread only
  std::thread th;
  // writer-thread clock, ns: [open/create, first map of model.cpt, parameter
  // patch, tracking pickle + write, jobs, files opened]
  std::atomic<int64_t> stat[6] = {};

  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  FileEnt* open_file(const std::string& path, int32_t& err) {
    FileEnt& e = files[path];
    if (e.fd < 0) {
      const int64_t t0 = now_ns();
      e.fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0644);
      if (e.fd < 0 && errno == ENOENT && make_parents(path))
        e.fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0644);
      if (e.fd < 0 && errno == EMFILE) {
        // descriptor limit: release every cached file, then retry
        files.erase(path);
        close_all();
        FileEnt& f = files[path];
        f.fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0644);
        if (f.fd < 0) {
          if (!err) err = -errno;
          files.erase(path);
          return nullptr;
        }
        stat[0] += now_ns() - t0;
        stat[5] += 1;
        return &f;
      }
      if (e.fd < 0) {
        if (!err) err = -errno;
        files.erase(path);
        return nullptr;
      }
      stat[0] += now_ns() - t0;
      stat[5] += 1;
    }
    return &e;
  }

  void close_all() {
    for (auto& kv : files) {
      if (kv.second.map) munmap(kv.second.map, tpl.size());
      if (kv.second.fd >= 0) ::close(kv.second.fd);
    }
    files.clear();
  }

  void run() {
    std::vector<float> canon(canon_idx.size());
    std::vector<uint8_t> pk;
    for (;;) {
      WJob job;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_job.wait(lk, [&] { return stop || release || !q.empty(); });
        if (q.empty()) {
          if (release) {
            // every queued job is written: drop descriptors / mappings
            close_all();
            release = false;
            cv_done.notify_all();
            continue;
          }
          close_all();
          return;
        }
        job = std::move(q.front());
        q.pop_front();
      }
      int32_t err = 0;
      const int n = static_cast<int>(job.rows.size());
      const int nreg = static_cast<int>(regions.size() / 3);
      for (int j = 0; j < n; ++j) {
        if (job.improved[j]) {
          FileEnt* e = open_file(job.cpt_path[j], err);
          if (e && !e->map) {
            const int64_t t0 = now_ns();
            // first use: the file becomes the template, kept mapped
            if (ftruncate(e->fd, static_cast<off_t>(tpl.size())) == 0) {
              void* m = mmap(nullptr, tpl.size(), PROT_READ | PROT_WRITE, MAP_SHARED, e->fd, 0);
              if (m != MAP_FAILED) {
                e->map = static_cast<uint8_t*>(m);
                std::memcpy(e->map, tpl.data(), tpl.size());
              }
            }
            if (!e->map && !err) err = -EIO;
            stat[1] += now_ns() - t0;
          }
          if (e && e->map) {
            const int64_t t0 = now_ns();
            const float* row = job.snap + static_cast<int64_t>(job.rows[j]) * job.stride;
            for (size_t i = 0; i < canon.size(); ++i) canon[i] = row[canon_idx[i]];
            for (int r = 0; r < nreg; ++r)
              std::memcpy(e->map + regions[3 * r], canon.data() + regions[3 * r + 2],
                          static_cast<size_t>(regions[3 * r + 1]) * 4);
            stat[2] += now_ns() - t0;
          }
        }
        const int64_t t1 = now_ns();
        if (!pickle_tracking(job.trk.data() + static_cast<int64_t>(j) * job.trk_stride * 2, job.trk_len[j], pk)) {
          if (!err) err = -1;
          continue;
        }
        FileEnt* e = open_file(job.trk_path[j], err);
        if (!e) continue;
        if (e->size < 0) {
          struct stat st;
          e->size = fstat(e->fd, &st) == 0 ? static_cast<int64_t>(st.st_size) : 0;
        }
        const int rc = write_all(e->fd, pk.data(), pk.size(), &e->size);
        if (rc && !err) err = rc;
        stat[3] += now_ns() - t1;
      }
      stat[4] += 1;
      {
        std::lock_guard<std::mutex> lk(mu);
        if (err && !first_error) first_error = err;
        done_ticket = job.ticket;
      }
      cv_done.notify_all();
    }
  }
};

}  // namespace

void* fedmx_writer_create(const int32_t* canon_idx, int32_t n_canon, const int64_t* regions, int32_t n_regions,
                          const uint8_t* tpl, int64_t tpl_len) {
  Writer* w = new Writer();
  w->canon_idx.assign(canon_idx, canon_idx + n_canon);
  w->regions.assign(regions, regions + 3 * static_cast<int64_t>(n_regions));
  w->tpl.assign(tpl, tpl + tpl_len);
  w->th = std::thread([w] { w->run(); });
  return w;
}

// Queue one round's checkpoint job; returns its ticket (> 0).  Paths are
// NUL-separated in `paths` (2n entries: model.cpt, tracking, per client);
// the writer thread opens / creates / maps the files itself, so the caller
// never waits on the filesystem.
int64_t fedmx_writer_submit(void* handle, const float* snap, int64_t stride, int32_t n, const int32_t* rows,
                            const int32_t* improved, const char* paths, int64_t paths_len, const double* trk,
                            const int32_t* trk_len, int32_t trk_stride) {
  Writer* w = static_cast<Writer*>(handle);
  WJob job;
  job.snap = snap;
  job.stride = stride;
  job.rows.assign(rows, rows + n);
  job.improved.assign(improved, improved + n);
  job.trk_len.assign(trk_len, trk_len + n);
  job.trk.assign(trk, trk + static_cast<int64_t>(n) * trk_stride * 2);
  job.trk_stride = trk_stride;
  job.cpt_path.reserve(n);
  job.trk_path.reserve(n);
  const char* p = paths;
  const char* end = paths + paths_len;
  for (int j = 0; j < 2 * n && p < end; ++j) {
    const size_t len = strnlen(p, static_cast<size_t>(end - p));
    (j % 2 == 0 ? job.cpt_path : job.trk_path).emplace_back(p, len);
    p += len + 1;
  }
  if (static_cast<int>(job.trk_path.size()) != n) return -1;
  int64_t t;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    t = job.ticket = ++w->next_ticket;
    w->q.push_back(std::move(job));
  }
  w->cv_job.notify_one();
  return t;
}

// Block until job `ticket` (and every earlier one) is written; ticket <= 0:
// every submitted job.  Returns the first write error seen so far (0: none).
int32_t fedmx_writer_wait(void* handle, int64_t ticket) {
  Writer* w = static_cast<Writer*>(handle);
  std::unique_lock<std::mutex> lk(w->mu);
  const int64_t t = ticket > 0 ? ticket : w->next_ticket;
  w->cv_done.wait(lk, [&] { return w->done_ticket >= t; });
  return w->first_error;
}

// Every queued job written, then the writer thread closes its descriptors and
// mappings (end of a sweep combination).  Returns the first write error.
int32_t fedmx_writer_flush(void* handle) {
  Writer* w = static_cast<Writer*>(handle);
  std::unique_lock<std::mutex> lk(w->mu);
  const int64_t t = w->next_ticket;
  w->cv_done.wait(lk, [&] { return w->done_ticket >= t; });
  w->release = true;
  w->cv_job.notify_one();
  w->cv_done.wait(lk, [&] { return !w->release; });
  return w->first_error;
}

// Full store fence: the host's write-combined stores into fine-grained
// device memory (the descriptor ring, ops/_hiprt.py) are globally visible
// before the kernel launch that reads them is submitted.
void fedmx_store_fence() {
  _mm_sfence();   // drains the write-combining buffers
  std::atomic_thread_fence(std::memory_order_seq_cst);
}

// Writer-thread clock: out[0..5] = ms opening / creating files, ms first
// mapping model.cpt files, ms patching parameters, ms pickling + writing
// tracking (includes its opens), jobs done, files opened.
void fedmx_writer_stats(void* handle, double* out) {
  Writer* w = static_cast<Writer*>(handle);
  for (int i = 0; i < 4; ++i) out[i] = 1e-6 * static_cast<double>(w->stat[i].load());
  out[4] = static_cast<double>(w->stat[4].load());
  out[5] = static_cast<double>(w->stat[5].load());
}

void fedmx_writer_destroy(void* handle) {
  Writer* w = static_cast<Writer*>(handle);
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->stop = true;
  }
  w->cv_job.notify_all();
  w->th.join();
  delete w;
}

}  // extern "C"
