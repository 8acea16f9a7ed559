// pgmdq.cpp — direct AQL dispatch of prepared row-plan launches on a user-mode HSA queue.
//
// A bound launch of the plan-specialised row kernel (pgm_rows_plan_bind) is one fixed kernel with
// a fixed argument segment.  Through HIP every launch of it still costs the runtime's generic path
// (~4.5 us of host time on the MI355X boxes, more than the 100k-row kernel itself).  Here the
// launch is what CDNA executes natively: one 64-byte kernel-dispatch packet written into an HSA
// user-mode queue of the GPU agent and a doorbell write.  The code object is the same hipRTC
// output HIP loaded (pgmi_rows_bound_jit), loaded a second time into an HSA executable; the
// argument segment lives in device memory, written once at bind time.
//
// Ordering contract (include/pgmhip.h, pgm_dq_*): pgm_dq_bind_rows drains the device (HIP work that
// produced the inputs is complete); packets on the queue run in order (barrier bit set: each
// dispatch waits for the previous one, as kernels on one HIP stream do) — except inside a group
// (pgm_dq_launch_group: launches with pairwise distinct outputs, e.g. independent row batches):
// its first packet carries the barrier bit, the others do not, so the CP starts each member's
// workgroups while the previous member drains (the per-dispatch launch and drain latency of a
// 100k-row batch is longer than its HBM time); inputs may change only
// between pgm_dq_sync and the next launch (the first dispatch after a sync acquires at system
// scope); pgm_dq_sync issues a system-scope release barrier and waits for it, after which HIP
// streams may consume the outputs.  Every packet completes an interrupt-free signal from a ring,
// so waits and kernel timestamps (queue profiling on) need no extra packets.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "pgm_internal.h"
#include "pgmhip.h"

namespace {

constexpr uint64_t kRing = 256;           // completion signals in flight at most
constexpr double kWaitLimitS = 20.0;      // a dispatch that takes longer is reported as hung

struct DirectQueue {
  int device = -1;
  hsa_agent_t agent{};
  hsa_profile_t profile = HSA_PROFILE_BASE;
  hsa_queue_t *q = nullptr;
  std::vector<hsa_signal_t> ring;
  std::vector<uint8_t> armed;  // per ring slot: the dispatch that last used it carried its signal
  uint64_t issued = 0;  // dispatches written so far
  uint64_t freq = 1;    // HSA system timestamp frequency (Hz)
  // fences: the first dispatch after bind/sync acquires at system scope (inputs written by HIP are
  // visible); later ones acquire at acq_scope (none by default: they read the same, unchanged
  // inputs); a dispatch releases at agent scope unless its kernel stores write-through (then
  // none: its output lines are past the L2 when it completes); pgm_dq_sync ends with one
  // system-scope release barrier packet.  PGM_DQ_ACQ / PGM_DQ_REL override (A/B knobs).
  uint16_t acq_scope = HSA_FENCE_SCOPE_NONE;
  uint16_t fresh_acq_scope = HSA_FENCE_SCOPE_SYSTEM;
  bool fresh = true;          // next dispatch is the first since bind/sync
  bool need_release = false;  // dispatches since the last system-scope release
  uint64_t last_kernel = 0;   // index of the last kernel dispatch (timer end)
  uint64_t group_first = 0;   // first dispatch of the last group (its members may finish in any order)
  std::mutex mu;
  std::atomic<int> queue_error{0};
  // timer: the GPU span from the first dispatch after pgm_dq_timer_start to the last one issued
  bool timing = false;
  bool have_start = false;
  uint64_t t_first = 0;
  uint64_t start_ticks = 0;
  uint64_t disp_ticks = 0, disp_n = 0;  // last span: sum of per-dispatch (end - start), dispatches summed
  bool hsa_up = false;
  bool profiling = true;
};

struct DirectBound {
  DirectQueue *dq = nullptr;
  hsa_code_object_reader_t reader{};
  hsa_executable_t exec{};
  uint64_t kernel_object = 0;
  uint32_t group_bytes = 0, private_bytes = 0;
  uint16_t rel_scope = HSA_FENCE_SCOPE_AGENT;
  void *kernarg = nullptr;  // device memory
  unsigned blocks = 0, wg = 0;
};

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return pgmi_fail(code, buf);
}

const char *hsa_msg(hsa_status_t st) {
  const char *s = nullptr;
  if (hsa_status_string(st, &s) != HSA_STATUS_SUCCESS || !s) return "unknown HSA status";
  return s;
}

#define HSA_TRY(expr)                                                              \
  do {                                                                             \
    const hsa_status_t st_ = (expr);                                               \
    if (st_ != HSA_STATUS_SUCCESS && st_ != HSA_STATUS_INFO_BREAK)                  \
      return fail(PGM_EDEVICE, "%s: %s", #expr, hsa_msg(st_));                       \
  } while (0)

struct AgentMatch {
  uint32_t bdf_hi;  // (bus << 5) | device
  uint32_t domain;
  bool found = false;
  hsa_agent_t agent{};
};

hsa_status_t match_agent(hsa_agent_t a, void *data) {
  AgentMatch *m = (AgentMatch *)data;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  if ((bdf >> 3) == m->bdf_hi && dom == m->domain) {
    m->agent = a;
    m->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

void queue_error_cb(hsa_status_t status, hsa_queue_t *, void *data) {
  DirectQueue *dq = (DirectQueue *)data;
  dq->queue_error.store((int)status);
  fprintf(stderr, "pgmhip: direct queue error: %s\n", hsa_msg(status));
}

// spin until the signal reaches 0 (active wait: the dispatches are microseconds long)
int wait_zero(DirectQueue *dq, hsa_signal_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  // poll the value (no interrupt-driven wait: the ring signals carry no event, see pgm_dq_create)
  for (uint32_t spin = 0; hsa_signal_load_scacquire(s) != 0; ++spin) {
    if (spin < 4096) continue;
    spin = 0;
    if (dq->queue_error.load()) return fail(PGM_EDEVICE, "direct queue: queue error %d", dq->queue_error.load());
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt > kWaitLimitS) return fail(PGM_EDEVICE, "direct queue: a dispatch did not complete within %.0f s", kWaitLimitS);
  }
  return PGM_OK;
}

// the gfx950 code object inside a clang offload bundle, or the object itself when it is a bare ELF
bool code_object_of(const char *p, size_t n, const char **out, size_t *out_n) {
  if (n >= 4 && memcmp(p, "\x7f" "ELF", 4) == 0) {
    *out = p;
    *out_n = n;
    return true;
  }
  static const char kMagic[] = "__CLANG_OFFLOAD_BUNDLE__";
  const size_t ml = sizeof kMagic - 1;
  if (n < ml + 8 || memcmp(p, kMagic, ml) != 0) return false;
  uint64_t count;
  memcpy(&count, p + ml, 8);
  size_t at = ml + 8;
  for (uint64_t i = 0; i < count; ++i) {
    if (at + 24 > n) return false;
    uint64_t off, size, idlen;
    memcpy(&off, p + at, 8);
    memcpy(&size, p + at + 8, 8);
    memcpy(&idlen, p + at + 16, 8);
    at += 24;
    if (at + idlen > n) return false;
    const std::string id(p + at, idlen);
    at += idlen;
    if (id.find("gfx950") != std::string::npos && off + size <= n && size > 0) {
      *out = p + off;
      *out_n = size;
      return true;
    }
  }
  return false;
}

}  // namespace

extern "C" {

int pgm_dq_create(int hip_device, void **out) {
  if (!out) return fail(PGM_EINVAL, "dq_create: null output pointer");
  *out = nullptr;
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, hip_device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, hip_device) != hipSuccess) {
    (void)hipGetLastError();
    return fail(PGM_EDEVICE, "dq_create: no HIP device %d", hip_device);
  }
  if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, hip_device) != hipSuccess) {
    (void)hipGetLastError();
    dom = 0;
  }
  DirectQueue *dq = new (std::nothrow) DirectQueue;
  if (!dq) return fail(PGM_ENOMEM, "dq_create: out of host memory");
  dq->device = hip_device;
  auto bail = [&](int rc) {
    if (dq->q) (void)hsa_queue_destroy(dq->q);
    for (hsa_signal_t s : dq->ring) (void)hsa_signal_destroy(s);
    if (dq->hsa_up) (void)hsa_shut_down();
    delete dq;
    return rc;
  };
  if (hsa_init() != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "dq_create: hsa_init failed"));
  dq->hsa_up = true;
  AgentMatch m;
  m.bdf_hi = ((uint32_t)bus << 5) | (uint32_t)dev;
  m.domain = (uint32_t)dom;
  (void)hsa_iterate_agents(match_agent, &m);
  if (!m.found) return bail(fail(PGM_EDEVICE, "dq_create: no HSA GPU agent at PCI %04x:%02x:%02x", dom, bus, dev));
  dq->agent = m.agent;
  (void)hsa_agent_get_info(dq->agent, HSA_AGENT_INFO_PROFILE, &dq->profile);
  uint32_t qmax = 0;
  (void)hsa_agent_get_info(dq->agent, HSA_AGENT_INFO_QUEUE_MAX_SIZE, &qmax);
  const uint32_t qsize = std::min<uint32_t>(4096, qmax ? qmax : 4096);
  hsa_status_t st = hsa_queue_create(dq->agent, qsize, HSA_QUEUE_TYPE_SINGLE, queue_error_cb, dq, UINT32_MAX,
                                     UINT32_MAX, &dq->q);
  if (st != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "dq_create: hsa_queue_create: %s", hsa_msg(st)));
  // dispatch timestamps for pgm_dq_timer_* (A/B knob PGM_DQ_PROFILE=0: off, the timer then reports 0)
  const char *pe = getenv("PGM_DQ_PROFILE");
  dq->profiling = !(pe && strcmp(pe, "0") == 0);
  st = dq->profiling ? hsa_amd_profiling_set_profiler_enabled(dq->q, 1) : HSA_STATUS_SUCCESS;
  if (st != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "dq_create: queue profiling: %s", hsa_msg(st)));
  (void)hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &dq->freq);
  if (!dq->freq) dq->freq = 1;
  dq->ring.reserve(kRing);
  dq->armed.assign(kRing, 0);
  // completion signals without an interrupt event (HSA_AMD_SIGNAL_AMD_GPU_ONLY): the CP only writes
  // the value (and the profiling timestamps); the host polls it (an interrupt signal: +0.5 us per
  // dispatch, profiles/r02e_store_release_ab.json)
  for (uint64_t i = 0; i < kRing; ++i) {
    hsa_signal_t s;
    st = hsa_amd_signal_create(0, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &s);
    if (st != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "dq_create: hsa_signal_create: %s", hsa_msg(st)));
    dq->ring.push_back(s);
  }
  *out = dq;
  return PGM_OK;
}

// the next ring signal (armed to 1) and queue slot; recycles the signal of dispatch n - kRing (chains
// reserve their slots in pgm_dq_run_chain)
static int next_slot(DirectQueue *dq, hsa_signal_t *sig, void **slot, uint64_t *qidx) {
  if (dq->queue_error.load()) return fail(PGM_EDEVICE, "direct queue: queue error %d", dq->queue_error.load());
  const uint64_t n = dq->issued;
  hsa_signal_t s = dq->ring[n % kRing];
  if (n >= kRing) {  // its dispatch must be complete (and, when it opened the timed span, its start kept)
    const int rc = wait_zero(dq, s);
    if (rc != PGM_OK) return rc;
    if (dq->profiling && dq->timing && !dq->have_start && n - kRing == dq->t_first) {
      hsa_amd_profiling_dispatch_time_t t;
      HSA_TRY(hsa_amd_profiling_get_dispatch_time(dq->agent, s, &t));
      dq->start_ticks = t.start;
      dq->have_start = true;
    }
  }
  hsa_signal_store_relaxed(s, 1);
  dq->armed[n % kRing] = 1;
  hsa_queue_t *q = dq->q;
  const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
  const auto t0 = std::chrono::steady_clock::now();
  while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kWaitLimitS)
      return fail(PGM_EDEVICE, "direct queue: full for %.0f s", kWaitLimitS);
  }
  *sig = s;
  *slot = (char *)q->base_address + (idx & (q->size - 1)) * 64;
  *qidx = idx;
  return PGM_OK;
}

static uint32_t header_word(uint16_t type, uint16_t acq, uint16_t rel, uint16_t setup, bool barrier = true) {
  const uint16_t h = (uint16_t)((type << HSA_PACKET_HEADER_TYPE) | ((barrier ? 1u : 0u) << HSA_PACKET_HEADER_BARRIER) |
                                (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  return (uint32_t)h | ((uint32_t)setup << 16);
}

static void publish(DirectQueue *dq, void *slot, uint32_t header, uint64_t idx) {
  __atomic_store_n((uint32_t *)slot, header, __ATOMIC_RELEASE);
  hsa_signal_store_screlease(dq->q->doorbell_signal, (hsa_signal_value_t)idx);
  dq->issued += 1;
}

// wait for every dispatch from the last group's first member on (members without the barrier bit
// may complete out of order; everything before the group completed before it started)
static int wait_tail(DirectQueue *dq) {
  const uint64_t from = std::max(dq->group_first, dq->issued >= kRing ? dq->issued - kRing : 0);
  for (uint64_t i = from; i < dq->issued; ++i) {
    if (!dq->armed[i % kRing]) continue;  // an inner chain packet: no signal (its chain's last one covers it)
    const int rc = wait_zero(dq, dq->ring[i % kRing]);
    if (rc != PGM_OK) return rc;
  }
  return PGM_OK;
}

// append the system-scope release barrier packet if a dispatch since the last one needs it (caller
// holds dq->mu); the next dispatch acquires at system scope
static int release_locked(DirectQueue *dq) {
  if (dq->issued == 0) return PGM_OK;
  if (dq->need_release) {
    hsa_signal_t sig;
    void *slot;
    uint64_t idx;
    const int rc = next_slot(dq, &sig, &slot, &idx);
    if (rc != PGM_OK) return rc;
    hsa_barrier_and_packet_t *b = (hsa_barrier_and_packet_t *)slot;
    b->reserved0 = 0;
    b->reserved1 = 0;
    for (int i = 0; i < 5; ++i) b->dep_signal[i].handle = 0;
    b->reserved2 = 0;
    b->completion_signal = sig;
    publish(dq, slot, header_word(HSA_PACKET_TYPE_BARRIER_AND, HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_SYSTEM, 0), idx);
    dq->need_release = false;
  }
  dq->fresh = true;
  return PGM_OK;
}

extern "C" int pgm_dq_release(void *handle) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq) return fail(PGM_EINVAL, "dq_release: null handle");
  std::lock_guard<std::mutex> lk(dq->mu);
  return release_locked(dq);
}

extern "C" int pgm_dq_sync(void *handle) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq) return fail(PGM_EINVAL, "dq_sync: null handle");
  std::lock_guard<std::mutex> lk(dq->mu);
  if (dq->issued == 0) return PGM_OK;
  const int rc = release_locked(dq);  // one barrier packet makes every dispatch's writes visible system-wide
  return rc != PGM_OK ? rc : wait_tail(dq);
}

int pgm_dq_wait(void *handle) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq) return fail(PGM_EINVAL, "dq_wait: null handle");
  std::lock_guard<std::mutex> lk(dq->mu);
  return dq->issued ? wait_tail(dq) : PGM_OK;
}

int pgm_dq_destroy(void *handle) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq) return PGM_OK;
  const int rc = pgm_dq_sync(dq);
  if (dq->q) (void)hsa_queue_destroy(dq->q);
  for (hsa_signal_t s : dq->ring) (void)hsa_signal_destroy(s);
  if (dq->hsa_up) (void)hsa_shut_down();
  delete dq;
  return rc;
}

// load a launch's code object into an HSA executable of the queue's agent, find its kernel, and write
// its explicit arguments into a device-memory kernarg segment (drains the device first: inputs HIP
// produced are complete)
static int bind_launch(DirectQueue *dq, const pgmi_jit_launch &L, const char *what, void **out) {
  if (L.blocks == 0 || L.wg == 0) return fail(PGM_EINVAL, "%s: empty launch", what);
  if ((uint64_t)L.blocks * L.wg > UINT32_MAX || L.wg > 1024)
    return fail(PGM_EINVAL, "%s: grid of %u x %u work-items does not fit a dispatch packet", what, L.blocks, L.wg);
  const char *co = nullptr;
  size_t co_n = 0;
  if (!code_object_of((const char *)L.code, L.code_size, &co, &co_n))
    return fail(PGM_EDEVICE, "%s: no gfx950 code object in the compiled kernel", what);
  DirectBound *db = new (std::nothrow) DirectBound;
  if (!db) return fail(PGM_ENOMEM, "%s: out of host memory", what);
  db->dq = dq;
  db->blocks = L.blocks;
  db->wg = L.wg;
  db->rel_scope = (uint16_t)(L.write_through ? HSA_FENCE_SCOPE_NONE : HSA_FENCE_SCOPE_AGENT);
  bool reader = false, exec = false;
  auto bail = [&](int rc2) {
    if (exec) (void)hsa_executable_destroy(db->exec);
    if (reader) (void)hsa_code_object_reader_destroy(db->reader);
    if (db->kernarg) (void)hipFree(db->kernarg);
    delete db;
    return rc2;
  };
  hsa_status_t st = hsa_code_object_reader_create_from_memory(co, co_n, &db->reader);
  if (st != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "%s: code object reader: %s", what, hsa_msg(st)));
  reader = true;
  st = hsa_executable_create_alt(dq->profile, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &db->exec);
  if (st != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "%s: executable: %s", what, hsa_msg(st)));
  exec = true;
  st = hsa_executable_load_agent_code_object(db->exec, dq->agent, db->reader, nullptr, nullptr);
  if (st == HSA_STATUS_SUCCESS) st = hsa_executable_freeze(db->exec, nullptr);
  if (st != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "%s: load code object: %s", what, hsa_msg(st)));
  hsa_executable_symbol_t sym;
  const std::string kd = std::string(L.kernel) + ".kd";
  st = hsa_executable_get_symbol_by_name(db->exec, kd.c_str(), &dq->agent, &sym);
  if (st != HSA_STATUS_SUCCESS) st = hsa_executable_get_symbol_by_name(db->exec, L.kernel, &dq->agent, &sym);
  if (st != HSA_STATUS_SUCCESS) return bail(fail(PGM_EDEVICE, "%s: kernel %s not found: %s", what, L.kernel, hsa_msg(st)));
  uint32_t ka_size = 0;
  (void)hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &db->kernel_object);
  (void)hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &db->group_bytes);
  (void)hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &db->private_bytes);
  (void)hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &ka_size);
  if (!db->kernel_object) return bail(fail(PGM_EDEVICE, "%s: null kernel object", what));
  if (ka_size > L.args_size + 64)  // the kernel reads implicit arguments this path does not provide
    return bail(fail(PGM_EDEVICE, "%s: kernarg segment %u B > %zu B of explicit arguments", what, ka_size,
                     L.args_size));
  const size_t bytes = std::max<size_t>(256, (std::max<size_t>(ka_size, L.args_size) + 63) & ~(size_t)63);
  hipError_t e = hipMalloc(&db->kernarg, bytes);
  if (e == hipSuccess) e = hipMemset(db->kernarg, 0, bytes);
  if (e == hipSuccess) e = hipMemcpy(db->kernarg, L.args, L.args_size, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipDeviceSynchronize();  // inputs produced on HIP streams are complete
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return bail(fail(PGM_EDEVICE, "%s: kernarg setup: %s", what, hipGetErrorString(e)));
  }
  *out = db;
  return PGM_OK;
}

int pgm_dq_bind_rows(void *handle, void *bound, void **out) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq || !bound || !out) return fail(PGM_EINVAL, "dq_bind_rows: null argument");
  *out = nullptr;
  pgmi_jit_launch L;
  const int rc = pgmi_rows_bound_jit(bound, &L);
  return rc != PGM_OK ? rc : bind_launch(dq, L, "dq_bind_rows", out);
}

int pgm_dq_bind_pm(void *handle, void *bound, void **out) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq || !bound || !out) return fail(PGM_EINVAL, "dq_bind_pm: null argument");
  *out = nullptr;
  pgmi_jit_launch L;
  const int rc = pgmi_pm_bound_jit(bound, &L);
  return rc != PGM_OK ? rc : bind_launch(dq, L, "dq_bind_pm", out);
}

// one kernel-dispatch packet of a bound launch (caller holds dq->mu)
static int dispatch(DirectBound *db, bool barrier, bool sys_release = false) {
  DirectQueue *dq = db->dq;
  if (dq->fresh) {
    // the first dispatch after bind/sync: HIP work issued since (a copy or kernel writing the inputs)
    // must be complete before the packet's system-scope acquire; the queue does not order against
    // HIP streams, so drain the device here (once per sync, never inside a stream of dispatches)
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return fail(PGM_EDEVICE, "dq_launch: synchronising HIP work before the first dispatch: %s", hipGetErrorString(e));
    }
  }
  hsa_signal_t sig;
  void *slot;
  uint64_t idx;
  const int rc = next_slot(dq, &sig, &slot, &idx);
  if (rc != PGM_OK) return rc;
  hsa_kernel_dispatch_packet_t *pkt = (hsa_kernel_dispatch_packet_t *)slot;
  pkt->workgroup_size_x = (uint16_t)db->wg;
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->reserved0 = 0;
  pkt->grid_size_x = db->blocks * db->wg;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = db->private_bytes;
  pkt->group_segment_size = db->group_bytes;
  pkt->kernel_object = db->kernel_object;
  pkt->kernarg_address = db->kernarg;
  pkt->reserved2 = 0;
  pkt->completion_signal = sig;
  const uint16_t acq = dq->fresh ? dq->fresh_acq_scope : dq->acq_scope;
  const uint16_t rel = sys_release ? (uint16_t)HSA_FENCE_SCOPE_SYSTEM : db->rel_scope;
  dq->fresh = false;
  dq->need_release = sys_release ? false : (dq->need_release || db->rel_scope != HSA_FENCE_SCOPE_SYSTEM);
  dq->last_kernel = dq->issued;
  if (barrier) dq->group_first = dq->issued;
  publish(dq, slot, header_word(HSA_PACKET_TYPE_KERNEL_DISPATCH, acq, rel,
                                (uint16_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS), barrier), idx);
  return PGM_OK;
}

int pgm_dq_launch(void *dbound) {
  DirectBound *db = (DirectBound *)dbound;
  if (!db) return fail(PGM_EINVAL, "dq_launch: null handle");
  std::lock_guard<std::mutex> lk(db->dq->mu);
  return dispatch(db, true);
}

int pgm_dq_launch_release(void *dbound) {
  DirectBound *db = (DirectBound *)dbound;
  if (!db) return fail(PGM_EINVAL, "dq_launch_release: null handle");
  std::lock_guard<std::mutex> lk(db->dq->mu);
  const int rc = dispatch(db, true, true);
  if (rc == PGM_OK) db->dq->fresh = true;  // as after pgm_dq_sync: the next dispatch acquires at system scope
  return rc;
}

int pgm_dq_launch_group(void *const *dbounds, int32_t n) {
  if (!dbounds || n <= 0) return fail(PGM_EINVAL, "dq_launch_group: empty group");
  if (n > (int32_t)(kRing / 2)) return fail(PGM_EINVAL, "dq_launch_group: %d launches > %d per group", n, (int)(kRing / 2));
  DirectQueue *dq = nullptr;
  for (int32_t i = 0; i < n; ++i) {
    const DirectBound *db = (const DirectBound *)dbounds[i];
    if (!db) return fail(PGM_EINVAL, "dq_launch_group: null handle at %d", i);
    if (dq && db->dq != dq) return fail(PGM_EINVAL, "dq_launch_group: launches bound to different queues");
    dq = db->dq;
    for (int32_t j = 0; j < i; ++j)
      if (dbounds[j] == dbounds[i]) return fail(PGM_EINVAL, "dq_launch_group: launch %d repeats launch %d", i, j);
  }
  std::lock_guard<std::mutex> lk(dq->mu);
  for (int32_t i = 0; i < n; ++i) {
    const int rc = dispatch((DirectBound *)dbounds[i], i == 0);
    if (rc != PGM_OK) return rc;
  }
  return PGM_OK;
}

uint16_t env_scope(const char *name) {
  const char *v = getenv(name);
  if (!v || !*v) return HSA_FENCE_SCOPE_AGENT;
  return v[0] == '0' ? (uint16_t)HSA_FENCE_SCOPE_NONE : v[0] == '2' ? (uint16_t)HSA_FENCE_SCOPE_SYSTEM : (uint16_t)HSA_FENCE_SCOPE_AGENT;
}

// A/B knob (timing only): fence scope of a chain's inner packets (0 none, 1 agent = default)
uint16_t chain_scope(const char *name) {
  static const uint16_t acq = env_scope("PGM_DQ_CHAIN_ACQ"), rel = env_scope("PGM_DQ_CHAIN_REL");
  return name[13] == 'A' ? acq : rel;
}

// a dependent chain (a compiled program's steps): every packet waits for the ones before it (barrier bit;
// not on a packet flagged independent of its predecessor — the parts of one split level — except the
// last, which always waits, so its completion signal and system-scope release cover the whole chain) and
// fences at agent scope, so each reads what the earlier ones wrote; the last releases at system scope
// (outputs the host reads in mapped memory; inputs it writes there are coherent host memory, read
// uncached).  The packets are written together and the doorbell rung once; no HIP drain (the caller's
// contract: HIP work that produced the inputs completed before).  Waits for the chain's last packet
// outside the queue lock, so other threads' chains queue behind it meanwhile.
//
// Everything that can fail is checked before the first slot is reserved (queue error, the timer, the
// ring signal of the last packet, room for all n packets), so a failure never leaves reserved slots
// without a valid header in front of the packet processor.
int pgm_dq_run_chain(void *const *dbounds, const uint8_t *independent, int32_t n) {
  if (!dbounds || n <= 0) return fail(PGM_EINVAL, "dq_run_chain: empty chain");
  if (n > (int32_t)(kRing / 2)) return fail(PGM_EINVAL, "dq_run_chain: %d launches > %d per chain", n, (int)(kRing / 2));
  DirectQueue *dq = nullptr;
  for (int32_t i = 0; i < n; ++i) {
    const DirectBound *db = (const DirectBound *)dbounds[i];
    if (!db) return fail(PGM_EINVAL, "dq_run_chain: null handle at %d", i);
    if (dq && db->dq != dq) return fail(PGM_EINVAL, "dq_run_chain: launches bound to different queues");
    dq = db->dq;
  }
  hsa_signal_t last{};
  {
    std::lock_guard<std::mutex> lk(dq->mu);
    if (dq->queue_error.load()) return fail(PGM_EDEVICE, "direct queue: queue error %d", dq->queue_error.load());
    // only the last packet carries a completion signal, so a timer span (dispatch timestamps per ring
    // signal) cannot cover a chain: refuse rather than report stale timestamps
    if (dq->timing) return fail(PGM_EINVAL, "dq_run_chain: a pgm_dq_timer span is open on this queue");
    const uint64_t first = dq->issued, last_n = first + (uint64_t)n - 1;
    // the last packet's ring signal: its previous use (dispatch last_n - kRing) must have completed
    last = dq->ring[last_n % kRing];
    if (last_n >= kRing) {
      const int rc = wait_zero(dq, last);
      if (rc != PGM_OK) return rc;
    }
    // room for all n packets before any is reserved
    hsa_queue_t *q = dq->q;
    const auto t0 = std::chrono::steady_clock::now();
    while (hsa_queue_load_write_index_relaxed(q) + (uint64_t)n - hsa_queue_load_read_index_scacquire(q) > q->size) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kWaitLimitS)
        return fail(PGM_EDEVICE, "direct queue: no room for a %d-packet chain for %.0f s", n, kWaitLimitS);
    }
    hsa_signal_store_relaxed(last, 1);
    // one reservation of n slots (single-producer queue: the caller holds dq->mu)
    const uint64_t idx0 = hsa_queue_add_write_index_relaxed(q, (uint64_t)n);
    for (int32_t i = 0; i < n; ++i) {
      const DirectBound *db = (const DirectBound *)dbounds[i];
      const uint64_t idx = idx0 + (uint64_t)i;
      void *slot = (char *)q->base_address + (idx & (q->size - 1)) * 64;
      // only the last packet signals its completion: a signal on every packet lengthened each dependent
      // launch by ~1 us (C2, 20 launches: 0.123 vs 0.104 ms/query, profiles/r05t/); the queue's read
      // index guards the slots of the others
      const bool is_last = i == n - 1;
      hsa_kernel_dispatch_packet_t *pkt = (hsa_kernel_dispatch_packet_t *)slot;
      pkt->workgroup_size_x = (uint16_t)db->wg;
      pkt->workgroup_size_y = 1;
      pkt->workgroup_size_z = 1;
      pkt->reserved0 = 0;
      pkt->grid_size_x = db->blocks * db->wg;
      pkt->grid_size_y = 1;
      pkt->grid_size_z = 1;
      pkt->private_segment_size = db->private_bytes;
      pkt->group_segment_size = db->group_bytes;
      pkt->kernel_object = db->kernel_object;
      pkt->kernarg_address = db->kernarg;
      pkt->reserved2 = 0;
      pkt->completion_signal.handle = is_last ? last.handle : 0;
      // every packet acquires at agent scope, the first one too: the inputs the host writes between chains live
      // in coherent (fine-grained) host memory the kernels read uncached, so no system-scope acquire (which
      // also dropped the CPT tables from L2 each query) is needed — C2 0.106 -> 0.103 ms, C1 0.043 -> 0.040
      // (profiles/r05an/); the last packet still releases at system scope for the host's reads
      const uint16_t acq = i == 0 ? (uint16_t)HSA_FENCE_SCOPE_AGENT : chain_scope("PGM_DQ_CHAIN_ACQ");
      const uint16_t rel = is_last ? (uint16_t)HSA_FENCE_SCOPE_SYSTEM : chain_scope("PGM_DQ_CHAIN_REL");
      const bool barrier = i == 0 || is_last || !independent || !independent[i];
      __atomic_store_n((uint32_t *)slot,
                       header_word(HSA_PACKET_TYPE_KERNEL_DISPATCH, acq, rel,
                                   (uint16_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS), barrier),
                       __ATOMIC_RELEASE);
      dq->armed[(first + (uint64_t)i) % kRing] = is_last ? 1 : 0;
      // the doorbell never covers the end of the ring: ring it on the last slot before the wrap as
      // well.  A profiler's intercept queue (rocprofv3 --kernel-trace) hands the packets one doorbell
      // covers to its interceptor as ONE contiguous array starting at the first new slot; a run that
      // wraps is read past the end of the ring.  r06a's trace of C2 (20 packets per chain on a
      // 4,096-slot queue) died with SIGSEGV at the page after the proxy ring, in the HSA runtime called
      // from this doorbell store, on the 205th chain — the first whose slots wrap (slots 4,080..4,099);
      // producers that ring once per packet (HIP, pgm_dq_launch) never hand it a wrapping run.
      if (!is_last && ((idx + 1) & (q->size - 1)) == 0)
        hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
    }
    dq->group_first = first;
    dq->last_kernel = last_n;
    dq->issued = last_n + 1;
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(idx0 + (uint64_t)n - 1));
    dq->need_release = false;  // the last packet released at system scope
    dq->fresh = true;
  }
  return wait_zero(dq, last);
}

int pgm_dq_profiling(void *handle, int32_t on) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq) return fail(PGM_EINVAL, "dq_profiling: null handle");
  std::lock_guard<std::mutex> lk(dq->mu);
  HSA_TRY(hsa_amd_profiling_set_profiler_enabled(dq->q, on ? 1 : 0));
  dq->profiling = on != 0;
  return PGM_OK;
}

int pgm_dq_timer_start(void *handle) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq) return fail(PGM_EINVAL, "dq_timer_start: null handle");
  std::lock_guard<std::mutex> lk(dq->mu);
  dq->timing = true;
  dq->have_start = false;
  dq->t_first = dq->issued;
  return PGM_OK;
}

int pgm_dq_timer_stop_ms(void *handle, float *ms) {
  if (!ms) return fail(PGM_EINVAL, "dq_timer_stop: null argument");
  *ms = 0.f;
  uint64_t t0 = 0, t1 = 0, f = 1;
  const int rc = pgm_dq_timer_stop_ticks(handle, &t0, &t1, &f);
  if (rc == PGM_OK && t1 > t0) *ms = (float)((double)(t1 - t0) * 1e3 / (double)f);
  return rc;
}

int pgm_dq_timer_stop_ticks(void *handle, uint64_t *start, uint64_t *end, uint64_t *freq) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq || !start || !end || !freq) return fail(PGM_EINVAL, "dq_timer_stop: null argument");
  *start = *end = 0;
  *freq = dq->freq;
  std::lock_guard<std::mutex> lk(dq->mu);
  if (!dq->timing) return fail(PGM_EINVAL, "dq_timer_stop: timer not started");
  dq->timing = false;
  if (dq->issued == dq->t_first) return PGM_OK;  // nothing dispatched in the span
  int rc = wait_tail(dq);
  if (rc != PGM_OK || !dq->profiling) return rc;
  // the span ends with the latest end among the last group's members (up to the last kernel)
  hsa_amd_profiling_dispatch_time_t te{};
  const uint64_t from = std::max(std::max(dq->group_first, dq->t_first), dq->issued >= kRing ? dq->issued - kRing + 1 : 0);
  for (uint64_t i = from; i <= dq->last_kernel; ++i) {
    if (!dq->armed[i % kRing]) continue;
    hsa_amd_profiling_dispatch_time_t t;
    HSA_TRY(hsa_amd_profiling_get_dispatch_time(dq->agent, dq->ring[i % kRing], &t));
    te.end = std::max(te.end, t.end);
  }
  // per-dispatch durations (what a kernel trace reports per launch) of the span's dispatches still in
  // the signal ring
  dq->disp_ticks = dq->disp_n = 0;
  const uint64_t lo = std::max(dq->t_first, dq->issued >= kRing ? dq->issued - kRing : 0);
  for (uint64_t i = lo; i <= dq->last_kernel && i < dq->issued; ++i) {
    if (!dq->armed[i % kRing]) continue;
    hsa_amd_profiling_dispatch_time_t t;
    HSA_TRY(hsa_amd_profiling_get_dispatch_time(dq->agent, dq->ring[i % kRing], &t));
    if (t.end > t.start) {
      dq->disp_ticks += t.end - t.start;
      ++dq->disp_n;
    }
  }
  if (!dq->have_start) {
    hsa_amd_profiling_dispatch_time_t ts;
    HSA_TRY(hsa_amd_profiling_get_dispatch_time(dq->agent, dq->ring[dq->t_first % kRing], &ts));
    dq->start_ticks = ts.start;
  }
  *start = dq->start_ticks;
  *end = te.end > dq->start_ticks ? te.end : dq->start_ticks;
  return PGM_OK;
}

int pgm_dq_timer_dispatch_stats(void *handle, uint64_t *sum_ticks, uint64_t *count) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq || !sum_ticks || !count) return fail(PGM_EINVAL, "dq_timer_dispatch_stats: null argument");
  std::lock_guard<std::mutex> lk(dq->mu);
  *sum_ticks = dq->disp_ticks;
  *count = dq->disp_n;
  return PGM_OK;
}

// after a timer stop: each timed dispatch's own (start, end) in HSA system ticks, in issue order — the
// dispatches of the span still in the signal ring (the C3 line commits them so its span-based frac can
// be recomputed from the raw timestamps, tools/c3_span_check.py)
int pgm_dq_timer_dispatch_times(void *handle, uint64_t *start, uint64_t *end, int32_t cap, int32_t *count) {
  DirectQueue *dq = (DirectQueue *)handle;
  if (!dq || !count || (cap > 0 && (!start || !end))) return fail(PGM_EINVAL, "dq_timer_dispatch_times: null argument");
  *count = 0;
  std::lock_guard<std::mutex> lk(dq->mu);
  if (dq->timing) return fail(PGM_EINVAL, "dq_timer_dispatch_times: timer still running");
  if (!dq->profiling || dq->issued == dq->t_first) return PGM_OK;
  const uint64_t lo = std::max(dq->t_first, dq->issued >= kRing ? dq->issued - kRing : 0);
  int32_t k = 0;
  for (uint64_t i = lo; i <= dq->last_kernel && i < dq->issued && k < cap; ++i) {
    if (!dq->armed[i % kRing]) continue;
    hsa_amd_profiling_dispatch_time_t t;
    HSA_TRY(hsa_amd_profiling_get_dispatch_time(dq->agent, dq->ring[i % kRing], &t));
    start[k] = t.start;
    end[k] = t.end;
    ++k;
  }
  *count = k;
  return PGM_OK;
}

int pgm_dq_bound_destroy(void *dbound) {
  DirectBound *db = (DirectBound *)dbound;
  if (!db) return PGM_OK;
  const int rc = pgm_dq_sync(db->dq);  // no dispatch of this kernel may still be in flight
  (void)hsa_executable_destroy(db->exec);
  (void)hsa_code_object_reader_destroy(db->reader);
  if (db->kernarg) (void)hipFree(db->kernarg);
  delete db;
  return rc;
}

}  // extern "C"
