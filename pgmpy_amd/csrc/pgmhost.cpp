// pgmhost.cpp — host-side ingestion helpers of the public DataFrame API (no GPU work).
//
// predict / predict_probability on a pandas Categorical frame (DiscreteBayesianNetwork.py:731-989)
// must find every NaN cell of every column (a NaN changes the row's evidence pattern) and map the
// plan's columns from category codes to state codes.  A munin frame of 100 k rows is 1,038 int8 columns
// (104 MB) to scan and 7 columns to map.  r05 scanned with threads spawned per call and mapped with
// np.take on the Python thread (0.72 + 0.30 ms of a 1.6 ms call, profiles/r06c/).  Here both run on one
// persistent pool of host threads, and the scan is a job the caller feeds column by column while it
// walks the frame in Python (pgm_host_scan_begin / _push / _end), so the walk and the scan overlap.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "pgm_internal.h"
#include "pgmhip.h"

namespace {

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return pgmi_fail(code, buf);
}

// A fixed pool of worker threads, started on first use and kept for the life of the process (workers
// block on a condition variable between tasks; spawning 16 threads per call cost ~0.1 ms).
class Pool {
 public:
  // min(16, hardware threads) workers whatever the first caller asks for (16: the host share of one GPU
  // on the MI355X boxes); a job's `threads` only caps how many tasks it has in flight
  static Pool &get(int) {
    static Pool *p = new Pool((int)std::max(1u, std::min(16u, std::thread::hardware_concurrency())));  // never destroyed
    return *p;
  }
  int size() const { return (int)workers_.size(); }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
    for (auto &t : workers_) t.detach();
  }
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> workers_;
};

// a counter of outstanding tasks that a caller waits on (held by shared_ptr in every task, so the last
// task's done() never touches a latch the waiter has already freed)
struct Latch {
  std::mutex mu;
  std::condition_variable cv;
  int64_t pending = 0;
  void add(int64_t k) {
    std::lock_guard<std::mutex> lk(mu);
    pending += k;
  }
  void done() {
    std::lock_guard<std::mutex> lk(mu);
    if (--pending == 0) cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return pending == 0; });
  }
};

// any byte of c[0, n) negative (an int8 category code of -1 = NaN): 8-byte words ORed, the sign bits tested
bool any_negative(const int8_t *c, int64_t n) {
  const int64_t words = n / 8;
  uint64_t acc = 0;
  for (int64_t w = 0; w < words; ++w) {
    uint64_t x;
    memcpy(&x, c + 8 * w, 8);
    acc |= x;
  }
  bool neg = (acc & 0x8080808080808080ull) != 0;
  for (int64_t i = words * 8; i < n && !neg; ++i) neg = c[i] < 0;
  return neg;
}

struct ScanState {
  int64_t n = 0;
  std::vector<const int8_t *> cols;  // capacity reserved up front: pushes never reallocate
  std::vector<uint8_t> flag;
  Latch latch;
};

struct ScanJob {
  std::shared_ptr<ScanState> st;  // shared with the job's tasks
  int threads = 1;
};

constexpr int32_t kScanTask = 16;  // columns per pool task

}  // namespace

extern "C" {

int pgm_host_scan_begin(int64_t n, int32_t capacity, int32_t threads, void **job) {
  if (!job || n < 0 || capacity < 0) return fail(PGM_EINVAL, "host_scan_begin: bad argument");
  *job = nullptr;
  ScanJob *j = new (std::nothrow) ScanJob;
  if (!j) return fail(PGM_ENOMEM, "host_scan_begin: out of host memory");
  try {
    j->st = std::make_shared<ScanState>();
    j->st->cols.reserve((size_t)capacity);
    j->st->flag.assign((size_t)capacity, 0);
  } catch (...) {
    delete j;
    return fail(PGM_ENOMEM, "host_scan_begin: out of host memory");
  }
  j->st->n = n;
  j->threads = std::max(1, std::min(16, (int)threads));
  Pool::get(j->threads);
  *job = j;
  return PGM_OK;
}

int pgm_host_scan_push(void *job, const int8_t *const *cols, int32_t count) {
  ScanJob *j = (ScanJob *)job;
  if (!j || count < 0 || (count > 0 && !cols)) return fail(PGM_EINVAL, "host_scan_push: bad argument");
  ScanState &S = *j->st;
  if (S.cols.size() + (size_t)count > S.cols.capacity())
    return fail(PGM_EINVAL, "host_scan_push: %zu columns > the capacity of %zu", S.cols.size() + (size_t)count,
                S.cols.capacity());
  for (int32_t i = 0; i < count; ++i)
    if (!cols[i] && S.n > 0) return fail(PGM_EINVAL, "host_scan_push: column %d is null", i);
  const size_t base = S.cols.size();
  S.cols.insert(S.cols.end(), cols, cols + count);
  if (S.n == 0) return PGM_OK;
  Pool &p = Pool::get(j->threads);
  for (int32_t c0 = 0; c0 < count; c0 += kScanTask) {
    const size_t lo = base + (size_t)c0, hi = base + (size_t)std::min(count, c0 + kScanTask);
    S.latch.add(1);
    std::shared_ptr<ScanState> sp = j->st;
    p.submit([sp, lo, hi] {
      for (size_t c = lo; c < hi; ++c) sp->flag[c] = any_negative(sp->cols[c], sp->n) ? 1 : 0;
      sp->latch.done();
    });
  }
  return PGM_OK;
}

int pgm_host_scan_end(void *job, uint8_t *out, int32_t *n_cols) {
  ScanJob *j = (ScanJob *)job;
  if (!j) return fail(PGM_EINVAL, "host_scan_end: null job");
  ScanState &S = *j->st;
  S.latch.wait();
  if (n_cols) *n_cols = (int32_t)S.cols.size();
  if (out && !S.cols.empty()) memcpy(out, S.flag.data(), S.cols.size());
  delete j;
  return PGM_OK;
}

int pgm_host_lut_map_u8(const int8_t *const *src, const uint8_t *const *luts, int32_t n_cols, int64_t n, uint8_t *dst,
                        int64_t ld, int32_t threads) {
  if (n_cols < 0 || n < 0 || ld < n || (n_cols > 0 && (!src || !luts || !dst)))
    return fail(PGM_EINVAL, "host_lut_map_u8: bad argument");
  for (int32_t j = 0; j < n_cols; ++j)
    if (!src[j] && n > 0) return fail(PGM_EINVAL, "host_lut_map_u8: column %d is null", j);
  if (n == 0 || n_cols == 0) return PGM_OK;
  // tasks of >= 64 KiB of one column each
  const int64_t chunk = std::max<int64_t>(1 << 16, (n + 3) / 4);
  auto latch = std::make_shared<Latch>();
  Pool &p = Pool::get(std::max(1, std::min(16, (int)threads)));
  for (int32_t j = 0; j < n_cols; ++j) {
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
      const int64_t r1 = std::min(n, r0 + chunk);
      const int8_t *s = src[j];
      const uint8_t *lut = luts[j];
      uint8_t *d = dst + (int64_t)j * ld;
      latch->add(1);
      p.submit([s, lut, d, r0, r1, latch] {
        if (lut) {
          for (int64_t i = r0; i < r1; ++i) d[i] = lut[(uint8_t)s[i]];
        } else {  // identity: category codes ARE state codes (-1, a NaN, reads as 255 = unobserved)
          memcpy(d + r0, s + r0, (size_t)(r1 - r0));
        }
        latch->done();
      });
    }
  }
  latch->wait();
  return PGM_OK;
}

int pgm_host_any_negative_i8(const int8_t *const *cols, int32_t n_cols, int64_t n, uint8_t *out, int32_t threads) {
  if (n_cols < 0 || n < 0 || (n_cols > 0 && (!cols || !out))) return fail(PGM_EINVAL, "host_any_negative_i8: bad argument");
  void *job = nullptr;
  int rc = pgm_host_scan_begin(n, n_cols, threads, &job);
  if (rc != PGM_OK) return rc;
  rc = pgm_host_scan_push(job, cols, n_cols);
  const int rc2 = pgm_host_scan_end(job, rc == PGM_OK ? out : nullptr, nullptr);
  return rc != PGM_OK ? rc : rc2;
}

}  // extern "C"
