// pgmpm.cpp — plan-specialised batched-BP steps (host code; the kernels it generates are compiled for
// gfx950 with hipRTC at run time): the fused product + marginal, n-ary products, separator marginals
// and two-marginal passes of a batched calibration (pgmpy ExactInference.py:770-805), merged per
// dependency level into one launch, plus the on-disk code-object cache shared with the specialised
// row kernels of pgmhip.hip.  C-ABI: include/pgmhip.h (pgm_product_n_marginal_bind, pgm_pm_*).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <functional>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "pgm_internal.h"
#include "pgmhip.h"

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) {                                                                   \
      (void)hipGetLastError();                                                                \
      return pgmi_failf(e_ == hipErrorOutOfMemory ? PGM_ENOMEM : PGM_EDEVICE, "%s: %s", #expr, \
                        hipGetErrorString(e_));                                               \
    }                                                                                         \
  } while (0)

static inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

static std::mutex g_rtc_mu;  // PGM_RTC_SERIAL=1: one hipRTC compile at a time

// ----------------------------------------------------------------------------- code-object cache
// On-disk cache of specialised code objects: directory PGM_KERNEL_CACHE (default
// $XDG_CACHE_HOME/pgmpy_amd or ~/.cache/pgmpy_amd; "0" disables), one file per source hash holding
// the full source (compared on load, so a hash collision only misses) and the gfx950 code object.
static std::string rtc_cache_dir() {
  static const std::string dir = [] {
    const char *e = getenv("PGM_KERNEL_CACHE");
    if (e) return std::string(strcmp(e, "0") == 0 ? "" : e);
    const char *x = getenv("XDG_CACHE_HOME");
    if (x && *x) return std::string(x) + "/pgmpy_amd";
    const char *h = getenv("HOME");
    return h && *h ? std::string(h) + "/.cache/pgmpy_amd" : std::string();
  }();
  return dir;
}

static const char *const kRtcOpts[] = {"--offload-arch=gfx950", "-O3"};

// what else decides the code object besides the source: the hipRTC (compiler) version, the target
// and the options; folded into the cache key so an upgraded compiler never reuses an old object
static const std::string &rtc_toolchain_tag() {
  static const std::string tag = [] {
    int major = 0, minor = 0;
    if (hiprtcVersion(&major, &minor) != HIPRTC_SUCCESS) major = minor = -1;
    std::string t = "hiprtc " + std::to_string(major) + "." + std::to_string(minor);
    for (const char *o : kRtcOpts) t += std::string(" ") + o;
    return t;
  }();
  return tag;
}

static std::string rtc_cache_path(const std::string &src) {
  const std::string dir = rtc_cache_dir();
  if (dir.empty()) return dir;
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the source, the toolchain tag and the ABI version
  for (unsigned char c : src) h = (h ^ c) * 1099511628211ull;
  for (unsigned char c : rtc_toolchain_tag()) h = (h ^ c) * 1099511628211ull;
  h = (h ^ (uint64_t)pgm_version()) * 1099511628211ull;
  char name[64];
  snprintf(name, sizeof name, "/k%016llx.co", (unsigned long long)h);
  return dir + name;
}

static bool rtc_cache_load(const std::string &path, const std::string &src, std::vector<char> &code) {
  if (path.empty()) return false;
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) return false;
  uint64_t n = 0, m = 0;
  bool ok = fread(&n, 8, 1, f) == 1 && n == src.size();
  std::string s2;
  if (ok) {
    s2.resize(n);
    ok = fread(&s2[0], 1, n, f) == n && s2 == src && fread(&m, 8, 1, f) == 1 && m > 0 && m < (1ull << 30);
  }
  if (ok) {
    code.resize(m);
    ok = fread(code.data(), 1, m, f) == m;
  }
  fclose(f);
  return ok;
}

static void rtc_cache_store(const std::string &path, const std::string &src, const std::vector<char> &code) {
  if (path.empty()) return;
  const std::string dir = path.substr(0, path.rfind('/'));
  // mkdir -p: create each component
  for (size_t i = 1; i <= dir.size(); ++i)
    if (i == dir.size() || dir[i] == '/') (void)mkdir(dir.substr(0, i).c_str(), 0755);
  const std::string tmp = path + ".tmp." + std::to_string((long long)getpid());
  FILE *f = fopen(tmp.c_str(), "wb");
  if (!f) return;
  const uint64_t n = src.size(), m = code.size();
  const bool ok = fwrite(&n, 8, 1, f) == 1 && fwrite(src.data(), 1, n, f) == n && fwrite(&m, 8, 1, f) == 1 &&
                  fwrite(code.data(), 1, m, f) == m;
  if (fclose(f) == 0 && ok) (void)rename(tmp.c_str(), path.c_str());
  else (void)remove(tmp.c_str());
}

// gfx950 code object of a specialised kernel source: the disk cache, else hipRTC (then cached)
bool pgmi_rtc_code(const std::string &src, const char *what, std::vector<char> &code) {
  const std::string path = rtc_cache_path(src);
  // the stored header holds the toolchain tag and the source; both must match on load
  const std::string keyed = rtc_toolchain_tag() + "\n" + src;
  if (rtc_cache_load(path, keyed, code)) return true;
  // hipRTC programs compile concurrently from several threads (pgm_pm_prepare); PGM_RTC_SERIAL=1
  // serialises every compile
  static const bool serial = getenv("PGM_RTC_SERIAL") && atoi(getenv("PGM_RTC_SERIAL")) != 0;
  std::unique_lock<std::mutex> lk(g_rtc_mu, std::defer_lock);
  if (serial) lk.lock();
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "pgm_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return false;
  if (hiprtcCompileProgram(prog, (int)(sizeof kRtcOpts / sizeof kRtcOpts[0]), (const char **)kRtcOpts) != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    fprintf(stderr, "pgmhip: %s did not compile (generic kernel used):\n%s\n", what, log.c_str());
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t sz = 0;
  hiprtcGetCodeSize(prog, &sz);
  code.resize(sz);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  rtc_cache_store(path, keyed, code);
  return true;
}


// ----------------------------------------------------------------------------- specialised product+marginal
// The fused batched-BP step (k_productn_marg_jx) with its plan baked in as literals: outer digits
// decoded with constant divisors, the reduced entries walked as nested loops with literal bounds and
// strides (inner ones unrolled, so several entries' operand loads are in flight together), operands
// that lack the row axis read at wave-uniform addresses (scalar loads), one 1-D grid with an optional
// XCD-grouped block order.  Compiled once per shape (hipRTC, cached by source), bound to its
// pointers, launched by pgm_pm_bound_run (capturable in a HIP graph).
// two marginals of one product in a single pass (no product stored): block = one state of the dims
// both keep (K) x a row chunk; the dims only one of them keeps (U = R1 + R2) are unrolled at
// generation time with one register accumulator per R1 / R2 state; dims neither keeps (Z) are runtime
// inner loops.  Batched-BP distribute: a parent's sigma' for two child scopes from its operands.
struct PMMulti {
  int n_ops = 0;
  int kind[MOPS] = {}, vec[MOPS] = {};
  int nK = 0, nU = 0, nZ = 0;
  unsigned kcard[KMAX] = {}, ucard[KMAX] = {}, zcard[KMAX] = {};
  int64_t ks[MOPS][KMAX] = {}, k1[KMAX] = {}, k2[KMAX] = {};
  int64_t us[MOPS][KMAX] = {}, u1[KMAX] = {}, u2[KMAX] = {};
  int64_t zs[MOPS][KMAX] = {};
  uint32_t n_outer = 0, NP = 0;
  unsigned n1 = 1, n2 = 1;  // accumulators (R1 / R2 states)
};

struct PMSpec {  // one fused step's specialisation
  int multi = 0;  // 1: PMMulti body (two marginals), else the ProdMK body
  PMMulti mm;
  ProdMK k;
  int red = PGM_RED_SUM, XI = 1, unroll = 8;
  bool store = true, xcd = false, nt = false;
  bool has_m = true;  // false: the product alone (pgm_product_n_bind), no marginal
  unsigned gx = 1;
  uint64_t total = 0;  // blocks
  // marginal-only passes: a kept dim no row operand carries (only row-less operands such as psi vary along
  // it), walked inside the block — its T states share the loaded row-operand values (-1: none)
  int tdim = -1;
  unsigned T = 1;
};

// a bound launch: one step, or several independent steps merged into one kernel (pgm_pm_merge:
// body i runs on blocks [start_i, start_i + total_i), starts padded to multiples of 8 so each body's
// XCD grouping holds)
struct PMBound {
  hipFunction_t fn = nullptr;  // compiled lazily: pgm_pm_prepare (in parallel) or the first run
  std::string src;
  unsigned blocks = 0;
  std::vector<PMSpec> specs;
  std::vector<const double *> ptrs;  // per body: its n_ops operands, then C, M
  unsigned threads = 256;  // workitems per workgroup (a specialised contraction chain: 1,024)
  // a contraction batch over the kernel-argument budget: its pointers in device memory, ptrs = {table}
  void *table = nullptr;
  PMBound() = default;
  PMBound(const PMBound &) = delete;
  PMBound &operator=(const PMBound &) = delete;
  ~PMBound() {
    if (table) (void)hipFree(table);
  }
};

static int pm_knob(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}

// Decode order of a step's kept outer dims, fastest first (the last one is the slowest: with the XCD
// grouping each XCD takes a contiguous range of it).  The kept dim carried by the most row-operand bytes
// becomes the slowest, so each XCD reads a disjoint slice of every operand that carries it (instead of
// all 8 re-reading an operand that lacks the belief's slowest dim), and the other dims vary fastest in
// order of the bytes that carry them (least first), so consecutive blocks re-read the same operand
// entries while they are in the XCD's L2 (C4 pathfinder, 4,000 rows: fetch 7.75 -> 6.32 GB per sweep,
// 1.04x the steps' own reads; r03's belief order and r04's partition-only and reversed forms measured
// slower, profiles/r04c/).  cards[q], bytes_of(q) = row-operand bytes that vary along kept dim q.
template <class BytesOf>
static std::vector<int> pm_kept_order(int kx, const unsigned *cards, BytesOf bytes_of) {
  std::vector<int> ord;
  for (int qi = 0; qi < kx; ++qi) ord.push_back(kx - 1 - qi);
  if (kx < 2) return ord;
  int p = -1;
  double best = -1.0;
  for (int q = 0; q < kx; ++q) {
    if (cards[q] < 2) continue;
    const double b = bytes_of(q);
    if (b > best || (b == best && p >= 0 && cards[q] > cards[p])) best = b, p = q;
  }
  if (p < 0) return ord;
  ord.erase(std::find(ord.begin(), ord.end(), p));
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return bytes_of(a) < bytes_of(b); });
  ord.push_back(p);
  return ord;
}

// blocks that share an XCD (b % 8, the dispatcher's round robin) take consecutive tiles: XCD label x
// gets tiles [x q + min(x, r), ...) with q = total / 8, r = total % 8 — a bijection for any total
// (the plain (b % 8) q + b / 8 only when 8 divides total)
static std::string pm_xcd_remap(uint64_t total) {
  const unsigned long long q = total / 8, r = total % 8;
  std::string o;
  if (r == 0)
    pgmi_appendf(o, "  b = (b %% 8u) * %lluu + b / 8u;  // blocks of one XCD are consecutive tiles\n", q);
  else
    pgmi_appendf(o, "  { const unsigned x = b %% 8u, y = b / 8u; b = (x < %lluu ? x * %lluu : %lluu + (x - %lluu) * %lluu) + y; }"
                    "  // blocks of one XCD are consecutive tiles\n", r, q + 1, r * (q + 1), r, q);
  return o;
}

// a body's signature: its block index, its n operands, then the product (C) and marginal (M) outputs
static std::string pm_signature(const std::string &name, int n) {
  std::string o = "__device__ __forceinline__ void " + name + "(unsigned b";
  for (int i = 0; i < n; ++i) o += ", const double *__restrict__ o" + std::to_string(i);
  o += ", double *__restrict__ C, double *__restrict__ M) {\n  (void)C; (void)M;\n";
  return o;
}

// operand pointers a body takes (its PMBound::ptrs are these, then C and M)
static int pm_nops(const PMSpec &sp) { return sp.multi ? sp.mm.n_ops : sp.k.n_ops; }

// body `name` of one step: a device function of its block index within the step
static std::string pm_body(const PMSpec &sp, const std::string &name) {
  const ProdMK &k = sp.k;
  const int red = sp.red, XI = sp.XI, unroll = sp.unroll;
  const bool store = sp.store, xcd = sp.xcd, nt = sp.nt, has_m = sp.has_m;
  const unsigned gx = sp.gx;
  const uint64_t total = sp.total;
  const int td = sp.tdim;
  const unsigned T = td >= 0 ? sp.T : 1;
  auto tsfx = [&](unsigned t) { return T > 1 ? "t" + std::to_string(t) : std::string(); };
  auto tiled = [&](int i) { return td >= 0 && k.ks[i][td] != 0; };  // operand i varies along the tile dim
  std::string o;
  o += pm_signature(name, k.n_ops);
  if (xcd) o += pm_xcd_remap(total);
  pgmi_appendf(o, "  const unsigned xb = b %% %uu, ob = b / %uu;\n", gx, gx);
  o += "  unsigned idx = ob;\n  long long oc = 0, om = 0";
  for (int i = 0; i < k.n_ops; ++i) pgmi_appendf(o, ", f%d = 0", i);
  o += ";\n  (void)oc; (void)idx;\n";
  const int kx = k.nk - 1;  // kept outer dims 0..kx-1 (kx-1 fastest), the row dim last
  unsigned kc[KMAX] = {};
  for (int q = 0; q < kx; ++q) kc[q] = k.kdiv[q].d;
  auto op_bytes = [&](int i) {  // entries of operand i over the step's index space (rows included)
    double b = k.vec[i] ? 16.0 * k.NP : 8.0;
    for (int q = 0; q < kx; ++q)
      if (k.ks[i][q]) b *= kc[q];
    for (int r = 0; r < k.nr; ++r)
      if (k.rs[i][r]) b *= k.rdiv[r].d;
    return b;
  };
  const std::vector<int> kord = pm_kept_order(kx, kc, [&](int q) {
    double t = 0.0;
    for (int i = 0; i < k.n_ops; ++i)
      if (k.vec[i] && k.ks[i][q]) t += op_bytes(i);
    return t;
  });
  for (int q : kord) {
    if (q == td) continue;  // walked inside the block
    const unsigned dq = k.kdiv[q].d;
    pgmi_appendf(o, "  { const unsigned q = idx / %uu, g = idx - q * %uu; idx = q;", dq, dq);
    if (k.ksc[q]) pgmi_appendf(o, " oc += (long long)g * %lldLL;", (long long)k.ksc[q]);
    if (k.ksm[q]) pgmi_appendf(o, " om += (long long)g * %lldLL;", (long long)k.ksm[q]);
    for (int i = 0; i < k.n_ops; ++i)
      if (k.ks[i][q]) pgmi_appendf(o, " f%d += (long long)g * %lldLL;", i, (long long)k.ks[i][q]);
    o += " }\n";
  }
  const uint32_t NP = k.NP;
  const bool tail = NP % (256u * XI) != 0;
  pgmi_appendf(o, "  const unsigned xbase = xb * %uu + threadIdx.x;\n", 256u * XI);
  for (int u = 0; u < XI; ++u) {
    pgmi_appendf(o, "  const unsigned x%d = xbase + %uu;\n", u, 256u * u);
    if (tail)
      pgmi_appendf(o, "  const unsigned c%d = x%d < %uu ? x%d : %uu;\n", u, u, NP, u, NP - 1);
    else
      pgmi_appendf(o, "  const unsigned c%d = x%d;\n", u, u);
  }
  // operands constant over the reduced entries: once per block
  for (int i = 0; i < k.n_ops; ++i) {
    if (k.jvar[i]) continue;
    if (k.vec[i]) {
      for (int u = 0; u < XI; ++u)
        pgmi_appendf(o, "  const pgm_d2 h%d_%d = ((const pgm_d2 *)(o%d + f%d))[c%d];\n", i, u, i, i, u);
    } else if (tiled(i)) {
      for (unsigned t = 0; t < T; ++t)
        pgmi_appendf(o, "  const double h%d%s = o%d[f%d + %lldLL];\n", i, tsfx(t).c_str(), i, i,
                     (long long)t * (long long)k.ks[i][td]);
    } else {
      pgmi_appendf(o, "  const double h%d = o%d[f%d];\n", i, i, i);
    }
  }
  const char *init = red == PGM_RED_MAX ? "-__builtin_inf()" : "0.0";
  for (unsigned t = 0; t < T && has_m; ++t)
    for (int u = 0; u < XI; ++u) pgmi_appendf(o, "  pgm_d2 a%d%s = {%s, %s};\n", u, tsfx(t).c_str(), init, init);
  // reduced dims as nested loops (dim 0 outermost: the generic kernel's entry order); the innermost
  // dims whose trip product stays within `unroll` are unrolled
  int first_unrolled = k.nr;
  {
    uint64_t prod = 1;
    for (int r = k.nr - 1; r >= 0; --r) {
      prod *= k.rdiv[r].d;
      if (prod > (uint64_t)unroll) break;
      first_unrolled = r;
    }
  }
  std::string ind = "  ";
  for (int r = 0; r < k.nr; ++r) {
    if (r >= first_unrolled)
      pgmi_appendf(o, "%s#pragma unroll\n", ind.c_str());
    else if (r == k.nr - 1)  // an innermost loop too long to unroll fully: `unroll` entries at a time
      pgmi_appendf(o, "%s#pragma unroll %d\n", ind.c_str(), std::max(1, unroll));
    else
      pgmi_appendf(o, "%s#pragma unroll 1\n", ind.c_str());
    pgmi_appendf(o, "%sfor (int r%d = 0; r%d < %u; ++r%d) {\n", ind.c_str(), r, r, k.rdiv[r].d, r);
    ind += "  ";
  }
  auto lin = [&](const int64_t *s) {  // literal offset of the current reduced entry
    std::string e = "0LL";
    for (int r = 0; r < k.nr; ++r)
      if (s[r]) e += " + (long long)r" + std::to_string(r) + " * " + std::to_string((long long)s[r]) + "LL";
    return e;
  };
  for (int i = 0; i < k.n_ops; ++i) {
    if (!k.jvar[i]) continue;
    const std::string J = lin(k.rs[i]);
    if (k.vec[i]) {
      pgmi_appendf(o, "%sconst pgm_d2 *p%d = (const pgm_d2 *)(o%d + f%d + %s);\n", ind.c_str(), i, i, i, J.c_str());
      for (int u = 0; u < XI; ++u) pgmi_appendf(o, "%sconst pgm_d2 v%d_%d = p%d[c%d];\n", ind.c_str(), i, u, i, u);
    } else if (tiled(i)) {
      for (unsigned t = 0; t < T; ++t)
        pgmi_appendf(o, "%sconst double s%d%s = o%d[f%d + %s + %lldLL];\n", ind.c_str(), i, tsfx(t).c_str(), i, i,
                     J.c_str(), (long long)t * (long long)k.ks[i][td]);
    } else {
      pgmi_appendf(o, "%sconst double s%d = o%d[f%d + %s];\n", ind.c_str(), i, i, i, J.c_str());
    }
  }
  for (unsigned t = 0; t < T; ++t) {
    const std::string ts = tsfx(t);
    for (int u = 0; u < XI; ++u) {
      for (int h = 0; h < 2; ++h) {
        const char cx = h ? 'y' : 'x';
        auto term = [&](int i) {
          char buf[64];
          const char *sf = tiled(i) ? ts.c_str() : "";
          if (k.jvar[i] && k.vec[i]) snprintf(buf, sizeof buf, "v%d_%d.%c", i, u, cx);
          else if (k.jvar[i]) snprintf(buf, sizeof buf, "s%d%s", i, sf);
          else if (k.vec[i]) snprintf(buf, sizeof buf, "h%d_%d.%c", i, u, cx);
          else snprintf(buf, sizeof buf, "h%d%s", i, sf);
          return std::string(buf);
        };
        std::string e = "1.0";
        for (int i = 0; i < k.n_ops; ++i) {
          if (k.kind[i] == PGM_PRODN_MUL) e = "(" + e + " * " + term(i) + ")";
          else if (k.kind[i] == PGM_PRODN_RATIO && i + 1 < MOPS)
            e = "(" + e + " * pgm_ratio(" + term(i) + ", " + term(i + 1) + "))";
        }
        pgmi_appendf(o, "%sconst double w%d%s%c = %s;\n", ind.c_str(), u, ts.c_str(), cx, e.c_str());
      }
      pgmi_appendf(o, "%sconst pgm_d2 w%d%s = {w%d%sx, w%d%sy};\n", ind.c_str(), u, ts.c_str(), u, ts.c_str(), u,
                   ts.c_str());
    }
  }
  if (store) {
    pgmi_appendf(o, "%spgm_d2 *cj = (pgm_d2 *)(C + oc + %s);\n", ind.c_str(), lin(k.rsc).c_str());
    for (int u = 0; u < XI; ++u) {
      const std::string guard = tail ? "if (x" + std::to_string(u) + " < " + std::to_string(NP) + "u) " : "";
      if (nt)
        pgmi_appendf(o, "%s%s__builtin_nontemporal_store(w%d, cj + x%d);\n", ind.c_str(), guard.c_str(), u, u);
      else
        pgmi_appendf(o, "%s%scj[x%d] = w%d;\n", ind.c_str(), guard.c_str(), u, u);
    }
  }
  for (unsigned t = 0; t < T && has_m; ++t) {
    const std::string tss = tsfx(t);
    const char *ts = tss.c_str();
    for (int u = 0; u < XI; ++u) {
      if (red == PGM_RED_MAX)
        pgmi_appendf(o, "%sa%d%s.x = pgm_maxn(a%d%s.x, w%d%s.x); a%d%s.y = pgm_maxn(a%d%s.y, w%d%s.y);\n", ind.c_str(),
                     u, ts, u, ts, u, ts, u, ts, u, ts, u, ts);
      else
        pgmi_appendf(o, "%sa%d%s += w%d%s;\n", ind.c_str(), u, ts, u, ts);
    }
  }
  for (int r = k.nr - 1; r >= 0; --r) {
    ind.resize(ind.size() - 2);
    pgmi_appendf(o, "%s}\n", ind.c_str());
  }
  // a marginal divided by an operand constant over the summed entries (PGM_PRODN_MDIV: sigma' / mu)
  if (has_m && k.mdiv >= 0) {
    const int i = k.mdiv;
    for (int u = 0; u < XI; ++u) {
      if (k.vec[i])
        pgmi_appendf(o, "  a%d = (pgm_d2){pgm_ratio(a%d.x, h%d_%d.x), pgm_ratio(a%d.y, h%d_%d.y)};\n", u, u, i, u, u, i, u);
      else
        pgmi_appendf(o, "  a%d = (pgm_d2){pgm_ratio(a%d.x, h%d), pgm_ratio(a%d.y, h%d)};\n", u, u, i, u, i);
    }
  }
  // marginal stores: nontemporal when the step stores no product (a marginal-only pass writes nothing
  // else), plain (write-back L2) otherwise
  for (unsigned t = 0; t < T && has_m; ++t) {
    const std::string ts = tsfx(t);
    const std::string mo = T > 1 ? "M + om + " + std::to_string((long long)t * (long long)k.ksm[td]) + "LL" : "M + om";
    for (int u = 0; u < XI; ++u) {
      const std::string guard = tail ? "if (x" + std::to_string(u) + " < " + std::to_string(NP) + "u) " : "";
      if (!store)
        pgmi_appendf(o, "  %s__builtin_nontemporal_store(a%d%s, (pgm_d2 *)(%s) + x%d);\n", guard.c_str(), u, ts.c_str(),
                     mo.c_str(), u);
      else
        pgmi_appendf(o, "  %s((pgm_d2 *)(%s))[x%d] = a%d%s;\n", guard.c_str(), mo.c_str(), u, u, ts.c_str());
    }
  }
  o += "}\n";
  return o;
}

static std::string pm_multi_body(const PMSpec &sp, const std::string &name) {
  // the target with fewer states of its own dims (R_reg) keeps one register accumulator per state,
  // its dims unrolled innermost; the other target's own dims (R_str) are runtime loops outermost, and
  // its marginal is complete after each of their iterations (everything inside is summed), so it is
  // stored there — registers stay bounded by the smaller target
  const PMMulti &q = sp.mm;
  const int red = sp.red;
  const int treg = q.n1 <= q.n2 ? 0 : 1;  // 0: M1 (C slot) in registers, 1: M2 (M slot)
  const int64_t *sreg = treg == 0 ? q.u1 : q.u2;
  const int64_t *sstr = treg == 0 ? q.u2 : q.u1;
  const char *preg = treg == 0 ? "C" : "M", *pstr = treg == 0 ? "M" : "C";
  const char *mreg = treg == 0 ? "m1" : "m2", *mstr = treg == 0 ? "m2" : "m1";
  const unsigned nreg = treg == 0 ? q.n1 : q.n2;
  std::string o;
  o += pm_signature(name, q.n_ops);
  if (sp.xcd) o += pm_xcd_remap(sp.total);
  pgmi_appendf(o, "  const unsigned xb = b %% %uu, ob = b / %uu;\n", sp.gx, sp.gx);
  o += "  unsigned idx = ob;\n  long long m1 = 0, m2 = 0";
  for (int i = 0; i < q.n_ops; ++i) pgmi_appendf(o, ", f%d = 0", i);
  o += ";\n  (void)idx;\n";
  auto op_bytes = [&](int i) {
    double b = q.vec[i] ? 16.0 * q.NP : 8.0;
    for (int d = 0; d < q.nK; ++d)
      if (q.ks[i][d]) b *= q.kcard[d];
    for (int d = 0; d < q.nU; ++d)
      if (q.us[i][d]) b *= q.ucard[d];
    for (int d = 0; d < q.nZ; ++d)
      if (q.zs[i][d]) b *= q.zcard[d];
    return b;
  };
  const std::vector<int> kord = pm_kept_order(q.nK, q.kcard, [&](int d) {
    double t = 0.0;
    for (int i = 0; i < q.n_ops; ++i)
      if (q.vec[i] && q.ks[i][d]) t += op_bytes(i);
    return t;
  });
  for (int d : kord) {
    pgmi_appendf(o, "  { const unsigned q = idx / %uu, g = idx - q * %uu; idx = q;", q.kcard[d], q.kcard[d]);
    if (q.k1[d]) pgmi_appendf(o, " m1 += (long long)g * %lldLL;", (long long)q.k1[d]);
    if (q.k2[d]) pgmi_appendf(o, " m2 += (long long)g * %lldLL;", (long long)q.k2[d]);
    for (int i = 0; i < q.n_ops; ++i)
      if (q.ks[i][d]) pgmi_appendf(o, " f%d += (long long)g * %lldLL;", i, (long long)q.ks[i][d]);
    o += " }\n";
  }
  const bool tail = q.NP % 256u != 0;
  o += "  const unsigned x = xb * 256u + threadIdx.x;\n";
  if (tail) pgmi_appendf(o, "  const unsigned c = x < %uu ? x : %uu;\n", q.NP, q.NP - 1);
  else o += "  const unsigned c = x;\n";
  const std::string guard = tail ? "if (x < " + std::to_string(q.NP) + "u) " : "";
  const char *init = red == PGM_RED_MAX ? "-__builtin_inf()" : "0.0";
  for (unsigned a = 0; a < nreg; ++a) pgmi_appendf(o, "  pgm_d2 ar_%u = {%s, %s};\n", a, init, init);
  // runtime loops: the streamed target's own dims (u), then the dims neither keeps (z)
  std::string ind = "  ";
  std::vector<int> ustr, ureg;
  for (int d = 0; d < q.nU; ++d) (sstr[d] ? ustr : ureg).push_back(d);
  for (int d : ustr) {
    pgmi_appendf(o, "%s#pragma unroll 1\n%sfor (int u%d = 0; u%d < %u; ++u%d) {\n", ind.c_str(), ind.c_str(), d, d,
            q.ucard[d], d);
    ind += "  ";
  }
  pgmi_appendf(o, "%spgm_d2 as = {%s, %s};\n", ind.c_str(), init, init);
  for (int z = 0; z < q.nZ; ++z) {
    pgmi_appendf(o, "%s#pragma unroll %s\n", ind.c_str(), z == q.nZ - 1 ? "2" : "1");
    pgmi_appendf(o, "%sfor (int z%d = 0; z%d < %u; ++z%d) {\n", ind.c_str(), z, z, q.zcard[z], z);
    ind += "  ";
  }
  auto runtime_off = [&](const int64_t *zs, const int64_t (*us)[KMAX], int i) {
    std::string e;
    for (int z = 0; z < q.nZ; ++z)
      if (zs[z]) e += " + (long long)z" + std::to_string(z) + " * " + std::to_string((long long)zs[z]) + "LL";
    for (int d : ustr)
      if (us[i][d]) e += " + (long long)u" + std::to_string(d) + " * " + std::to_string((long long)us[i][d]) + "LL";
    return e;
  };
  uint64_t nr = 1;
  for (int d : ureg) nr *= q.ucard[d];
  for (uint64_t ra = 0; ra < nr; ++ra) {
    unsigned dig[KMAX] = {};
    uint64_t rem = ra;
    for (int k = (int)ureg.size() - 1; k >= 0; --k) {
      dig[ureg[k]] = (unsigned)(rem % q.ucard[ureg[k]]);
      rem /= q.ucard[ureg[k]];
    }
    int64_t off[MOPS] = {};
    for (int d : ureg)
      for (int i = 0; i < q.n_ops; ++i) off[i] += (int64_t)dig[d] * q.us[i][d];
    pgmi_appendf(o, "%s{\n", ind.c_str());
    for (int i = 0; i < q.n_ops; ++i) {
      const std::string ro = runtime_off(q.zs[i], q.us, i);
      if (q.vec[i])
        pgmi_appendf(o, "%s  const pgm_d2 v%d = ((const pgm_d2 *)(o%d + f%d + %lldLL%s))[c];\n", ind.c_str(), i, i, i,
                (long long)off[i], ro.c_str());
      else
        pgmi_appendf(o, "%s  const double s%d = o%d[f%d + %lldLL%s];\n", ind.c_str(), i, i, i, (long long)off[i],
                ro.c_str());
    }
    for (int h = 0; h < 2; ++h) {
      const char cx = h ? 'y' : 'x';
      auto term = [&](int i) {
        char buf[32];
        if (q.vec[i]) snprintf(buf, sizeof buf, "v%d.%c", i, cx);
        else snprintf(buf, sizeof buf, "s%d", i);
        return std::string(buf);
      };
      std::string e = "1.0";
      for (int i = 0; i < q.n_ops; ++i) {
        if (q.kind[i] == PGM_PRODN_MUL) e = "(" + e + " * " + term(i) + ")";
        else if (q.kind[i] == PGM_PRODN_RATIO && i + 1 < MOPS)
          e = "(" + e + " * pgm_ratio(" + term(i) + ", " + term(i + 1) + "))";
      }
      pgmi_appendf(o, "%s  const double w%c = %s;\n", ind.c_str(), cx, e.c_str());
    }
    pgmi_appendf(o, "%s  const pgm_d2 w = {wx, wy};\n", ind.c_str());
    if (red == PGM_RED_MAX)
      pgmi_appendf(o, "%s  ar_%llu.x = pgm_maxn(ar_%llu.x, w.x); ar_%llu.y = pgm_maxn(ar_%llu.y, w.y); "
                 "as.x = pgm_maxn(as.x, w.x); as.y = pgm_maxn(as.y, w.y);\n",
              ind.c_str(), (unsigned long long)ra, (unsigned long long)ra, (unsigned long long)ra,
              (unsigned long long)ra);
    else
      pgmi_appendf(o, "%s  ar_%llu += w; as += w;\n", ind.c_str(), (unsigned long long)ra);
    pgmi_appendf(o, "%s}\n", ind.c_str());
  }
  for (int z = q.nZ - 1; z >= 0; --z) {
    ind.resize(ind.size() - 2);
    pgmi_appendf(o, "%s}\n", ind.c_str());
  }
  {  // the streamed target's marginal for this iteration is complete
    std::string e;
    for (int d : ustr)
      e += " + (long long)u" + std::to_string(d) + " * " + std::to_string((long long)sstr[d]) + "LL";
    pgmi_appendf(o, "%s%s((pgm_d2 *)(%s + %s%s))[x] = as;\n", ind.c_str(), guard.c_str(), pstr, mstr, e.c_str());
  }
  for (size_t k = 0; k < ustr.size(); ++k) {
    ind.resize(ind.size() - 2);
    pgmi_appendf(o, "%s}\n", ind.c_str());
  }
  for (uint64_t ra = 0; ra < nr; ++ra) {  // register target: accumulator ra at its digits' offset
    uint64_t rem = ra;
    int64_t off = 0;
    for (int k = (int)ureg.size() - 1; k >= 0; --k) {
      off += (int64_t)(rem % q.ucard[ureg[k]]) * sreg[ureg[k]];
      rem /= q.ucard[ureg[k]];
    }
    pgmi_appendf(o, "  %s((pgm_d2 *)(%s + %s + %lldLL))[x] = ar_%llu;\n", guard.c_str(), preg, mreg, (long long)off,
            (unsigned long long)ra);
  }
  o += "}\n";
  return o;
}

// kernel pgm_pm over the bodies (kernel argument: each body's operand pointers, then C and M); starts[i] = first block of
// body i, returns the grid size through *blocks
static std::string pm_source(const std::vector<PMSpec> &specs, std::vector<uint64_t> &starts, uint64_t *blocks) {
  std::string o =
      "#pragma clang fp contract(off)\n"  // products rounded before they are summed, as numpy does
      "typedef double pgm_d2 __attribute__((ext_vector_type(2)));\n"
      "typedef unsigned int pgm_u32x4 __attribute__((ext_vector_type(4)));\n"
      "__device__ __forceinline__ double pgm_ratio(double a, double b) { const double r = a / b; "
      "return r != r ? 0.0 : r; }\n"
      "__device__ __forceinline__ double pgm_maxn(double a, double b) { return (a > b || a != a) ? a : b; }\n";
  const size_t n = specs.size();
  starts.assign(n, 0);
  uint64_t at = 0;
  for (size_t i = 0; i < n; ++i) {
    at = (at + 7) / 8 * 8;
    starts[i] = at;
    at += specs[i].total;
    o += specs[i].multi ? pm_multi_body(specs[i], "pm" + std::to_string(i)) : pm_body(specs[i], "pm" + std::to_string(i));
  }
  *blocks = at;
  size_t nptr = 0;
  for (const PMSpec &sp : specs) nptr += (size_t)pm_nops(sp) + 2;
  pgmi_appendf(o, "struct pgm_pm_args { const double *p[%zu]; };\n", nptr);
  o += "extern \"C\" __global__ void __launch_bounds__(256) pgm_pm(const pgm_pm_args a) {\n"
       "  const unsigned b = blockIdx.x;\n";
  std::vector<std::string> calls(n);
  size_t base = 0;
  for (size_t i = 0; i < n; ++i) {
    const int no = pm_nops(specs[i]);
    std::string call = "pm" + std::to_string(i) + "(b - " + std::to_string((unsigned long long)starts[i]) + "u";
    for (int t = 0; t < no; ++t) call += ", a.p[" + std::to_string(base + t) + "]";
    call += ", (double *)a.p[" + std::to_string(base + no) + "], (double *)a.p[" + std::to_string(base + no + 1) + "])";
    base += (size_t)no + 2;
    calls[i] = call;
  }
  if (n == 1) {
    o += "  " + calls[0] + ";\n";
  } else {
    // a block finds its body through a balanced tree of literal block-range comparisons (log2 of the bodies
    // instead of up to one compare per body; C4 rate unchanged, r05p); blocks in the padding between bodies
    // fall out at the leaf's upper bound
    std::function<void(size_t, size_t, int)> tree = [&](size_t lo, size_t hi, int depth) {
      const std::string ind(2 * (size_t)depth, ' ');
      if (hi - lo == 1) {
        pgmi_appendf(o, "%sif (b < %lluu) %s;\n", ind.c_str(), (unsigned long long)(starts[lo] + specs[lo].total),
                     calls[lo].c_str());
        return;
      }
      const size_t mid = (lo + hi) / 2;
      pgmi_appendf(o, "%sif (b < %lluu) {\n", ind.c_str(), (unsigned long long)starts[mid]);
      tree(lo, mid, depth + 1);
      o += ind + "} else {\n";
      tree(mid, hi, depth + 1);
      o += ind + "}\n";
    };
    tree(0, n, 1);
  }
  o += "}\n";
  return o;
}

// source -> loaded kernel and its code object (process lifetime; the code object is what a direct AQL
// dispatch loads into its own HSA executable, pgm_dq_bind_pm)
struct PMLoaded {
  std::string src;
  hipFunction_t fn;
  std::vector<char> code;
};
static std::mutex g_pm_mu;
static std::vector<PMLoaded> g_pm_cache;

static const PMLoaded *pm_entry(const std::string &src) {  // caller holds g_pm_mu
  for (auto &e : g_pm_cache)
    if (e.src == src) return &e;
  return nullptr;
}

static hipFunction_t pm_cached(const std::string &src) {  // caller holds g_pm_mu
  const PMLoaded *e = pm_entry(src);
  return e ? e->fn : nullptr;
}

static hipFunction_t pm_load(const std::string &src, const std::vector<char> &code) {  // caller holds g_pm_mu
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  if (hipModuleLoadData(&mod, code.data()) != hipSuccess || hipModuleGetFunction(&fn, mod, "pgm_pm") != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  g_pm_cache.push_back(PMLoaded{src, fn, code});
  return fn;
}

static hipFunction_t pm_compile(const std::string &src) {
  std::lock_guard<std::mutex> lk(g_pm_mu);
  if (hipFunction_t f = pm_cached(src)) return f;
  std::vector<char> code;
  if (!pgmi_rtc_code(src, "specialised product+marginal kernel", code)) return nullptr;
  return pm_load(src, code);
}

// compile every bound step's kernel that is not loaded yet: distinct sources on up to
// PGM_RTC_THREADS threads (default 1: hipRTC serialises compiles internally — pathfinder's 20 kernels
// take 2.5 s on 1 thread and 2.6 s on 16), then load the modules
static int pm_prepare(PMBound *const *bs, int n) {
  std::vector<std::string> todo;
  {
    std::lock_guard<std::mutex> lk(g_pm_mu);
    for (int i = 0; i < n; ++i) {
      if (!bs[i] || bs[i]->fn) continue;
      if (hipFunction_t f = pm_cached(bs[i]->src)) {
        bs[i]->fn = f;
        continue;
      }
      if (std::find(todo.begin(), todo.end(), bs[i]->src) == todo.end()) todo.push_back(bs[i]->src);
    }
  }
  if (!todo.empty()) {
    std::vector<std::vector<char>> codes(todo.size());
    std::vector<char> ok(todo.size(), 0);
    const char *te = getenv("PGM_RTC_THREADS");
    const size_t nt = std::max<size_t>(1, std::min<size_t>(todo.size(), te ? (size_t)atoi(te) : 1));
    std::atomic<size_t> next(0);
    auto work = [&] {
      for (size_t i; (i = next.fetch_add(1)) < todo.size();)
        ok[i] = pgmi_rtc_code(todo[i], "specialised product+marginal kernel", codes[i]) ? 1 : 0;
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    std::lock_guard<std::mutex> lk(g_pm_mu);
    for (size_t i = 0; i < todo.size(); ++i) {
      if (!ok[i] || (!pm_cached(todo[i]) && !pm_load(todo[i], codes[i])))
        return pgmi_failf(PGM_EDEVICE, "specialised product+marginal kernel: compile / load failed");
    }
    for (int i = 0; i < n; ++i)
      if (bs[i] && !bs[i]->fn) bs[i]->fn = pm_cached(bs[i]->src);
  }
  return PGM_OK;
}


// ============================================================================= C-ABI
extern "C" {

static int pm_bind(const pgm_productn_desc *d, const double *const *ops, double *C, const int64_t *marg_s,
                   int32_t reduce, double *M, void **bound, std::string *src_out, bool has_m = true) {
  *bound = nullptr;
  if (reduce != PGM_RED_SUM && reduce != PGM_RED_MAX)
    return pgmi_failf(PGM_EINVAL, "product_n_marginal: reduce must be PGM_RED_SUM or PGM_RED_MAX");
  ProdMK k;
  dim3 g;
  const int r = pgmi_plan_product_marg(d, ops, C, marg_s, M, k, g);
  if (r < 0) return r;
  if (r == 0)
    return pgmi_failf(PGM_EINVAL, "product_n_marginal: shape not supported by the fused kernel "
                            "(pgm_product_n_marginal_ok is 0: run pgm_product_n + pgm_contract)");
  // PGM_PM_JIT=0 keeps the generic kernel (the specialised steps' reference path)
  static const int on = pm_knob("PGM_PM_JIT", 1);
  // defaults measured on MI355X, pathfinder C4 (4,000 / 1,000 rows: generic 781K / 515K calibrations/s;
  // specialised above 2M entries 911K / 601K; + one row pair per lane, nontemporal belief stores and
  // XCD-grouped blocks 933K; threshold 256K entries 648K at 1,000 rows)
  // r03ag, after the schedule changes (direct collect operands, 128-block fused floor): 2^18 / 2^16 / 2^14
  // -> 0.96-0.97 / 1.024-1.026 / 1.026-1.028 M calibrations/s at 1,000 rows, 1.27-1.28 / 1.28-1.29 /
  // 1.29 M at 4,000 (small steps specialised join their level's merged launch instead of launching alone)
  // r06at: 2^12 (was 2^14) — C4's smallest steps (the 4-state F29/F92 clique) join their level's merged launch
  // instead of running as generic kernels: +0.5-0.7 % at 4,000 / 1,000 rows (PGM_PM_MIN_ENTRIES A/B knob)
  static const int64_t min_entries = getenv("PGM_PM_MIN_ENTRIES") ? atoll(getenv("PGM_PM_MIN_ENTRIES")) : (1ll << 12);
  // per step, at least this many row pairs per lane when the rows fill them: 2 measured (MI355X, C4
  // 4,000 rows: 1.146 -> 1.18 M calibrations/s; 1,000 rows unchanged, too few rows; forced 2 / 4 for
  // every step, or a minimum of 4: slower, profiles/r02bw_c4_xi.txt)
  static constexpr int xi_min = 2;
  // reduced entries unrolled (4 / 16: -2 % / -10 % at 4,000 rows, profiles/r04v/; 16 on the steps of few
  // blocks only: +1.7 % at 1,000 rows, -3 to -5 % at 4,000, profiles/r04z/)
  static constexpr int unroll = 8;
  // nontemporal belief stores (default-policy stores: -5 % / -9 % at 4,000 / 1,000 rows; write-through
  // product stores: -4 % / -8 %; profiles/r04v/)
  static constexpr bool nt = true;
  static const bool no_jit = getenv("PGM_NO_JIT") != nullptr;
  const uint64_t entries = (uint64_t)k.n_outer * (uint64_t)k.n_red * 2ull * k.NP;
  if (!on || no_jit || entries < (uint64_t)min_entries) return PGM_OK;  // *bound NULL: generic kernel
  // row pairs per lane: a block of a step with few reduced entries (separator messages from small
  // operands, products without a reduction) does little work per lane — one 16-B store and a few
  // loads — so its lifetime, not HBM, bounds the step; XI pairs per lane give each lane ~8 entries of
  // work while keeping >= 2,048 blocks (8 per CU) in the step
  int XI = (uint64_t)k.NP >= 256ull * xi_min ? xi_min : 1;
  {
    const uint64_t red = std::max<uint64_t>(1, (uint64_t)k.n_red);
    while (XI < 8 && red * (uint64_t)XI < 8) {
      const int nx = XI * 2;
      const uint64_t gx2 = (k.NP + 256ull * nx - 1) / (256ull * nx);
      const uint64_t pad = gx2 * 256ull * nx - k.NP;  // idle lanes in the last block of a row range
      if (gx2 * (uint64_t)k.n_outer < 2048 || pad * 4 > k.NP) break;
      XI = nx;
    }
  }
  const uint64_t gx = (k.NP + 256ull * XI - 1) / (256ull * XI);
  const uint64_t total = gx * (uint64_t)k.n_outer;
  if (total >= (1ull << 31)) return PGM_OK;
  PMSpec sp;
  sp.k = k;
  sp.red = reduce;
  sp.XI = XI;
  // entries unrolled: `unroll`, fewer when many row operands vary over the reduced entries (each unrolled
  // entry keeps XI 16-B loads per such operand in flight: at most ~48, the 3-operand steps' budget)
  int nvj = 0;
  for (int t = 0; t < k.n_ops; ++t) nvj += k.vec[t] && k.jvar[t];
  sp.unroll = std::max(1, std::min(unroll, 48 / std::max(1, nvj * XI)));
  sp.store = C != nullptr;
  sp.has_m = has_m;
  sp.xcd = true;  // blocks grouped by XCD for any block count (bijective remap; r04c)
  sp.nt = nt;
  sp.gx = (unsigned)gx;
  sp.total = total;
  // a marginal-only pass re-loads its row operands (child messages) for every state of a kept dim that
  // only row-less operands (psi) carry — an L2-bound walk (C4 level 2: 64 states of the 32,256-state
  // clique); walk the largest such dim (2..8 states) inside the block instead, its states sharing the
  // loaded values, while >= 2,048 blocks remain and T x XI accumulators fit (C4, 4,000 rows: one batch in
  // flight 1.32-1.33 -> 1.36 M calibrations/s, two 1.39-1.43 -> 1.42-1.45 M; 1,000 rows unchanged; r05ac)
  if (!C && has_m && k.mdiv < 0) {
    unsigned best = 1;
    for (int q = 0; q + 1 < k.nk; ++q) {
      const unsigned d = k.kdiv[q].d;
      bool rowless = d >= 2 && d <= 8 && k.ksm[q] != 0;
      for (int t = 0; rowless && t < k.n_ops; ++t)
        if (k.vec[t] && k.ks[t][q]) rowless = false;
      if (rowless && d > best && total / d >= 2048 && d * (unsigned)XI <= 16) best = d, sp.tdim = q;
    }
    if (sp.tdim >= 0) {
      sp.T = best;
      sp.total = total / best;
    }
  }
  std::vector<uint64_t> starts;
  uint64_t blocks = 0;
  const std::string src = pm_source({sp}, starts, &blocks);
  if (src_out) {
    *src_out = src;
    return PGM_OK;
  }
  PMBound *b = new (std::nothrow) PMBound;
  if (!b) return pgmi_failf(PGM_ENOMEM, "product_n_marginal_bind: out of host memory");
  b->src = src;
  b->blocks = (unsigned)blocks;
  b->specs.push_back(sp);
  for (int t = 0; t < k.n_ops; ++t) b->ptrs.push_back(k.ops[t]);
  b->ptrs.push_back(C);
  b->ptrs.push_back(M);
  *bound = b;
  return PGM_OK;
}

int pgm_product_n_marginal_bind(const pgm_productn_desc *d, const double *const *ops, double *C,
                                const int64_t *marg_s, int32_t reduce, double *M, void **bound) {
  STALE_PROBE();
  if (!bound) return pgmi_failf(PGM_EINVAL, "product_n_marginal_bind: null bound");
  return pm_bind(d, ops, C, marg_s, reduce, M, bound, nullptr);
}

int pgm_product_n_bind(const pgm_productn_desc *d, const double *const *ops, double *C, void **bound) {
  STALE_PROBE();
  if (!bound || !d || !C) return pgmi_failf(PGM_EINVAL, "product_n_bind: null argument");
  *bound = nullptr;
  if (d->n_keep < 1 || d->n_keep > PGM_MAX_DIMS) return pgmi_failf(PGM_EINVAL, "product_n_bind: n_keep out of range");
  // the product as a fused step whose every dim is kept (no reduced entries) and no marginal stored
  int64_t ms[PGM_MAX_DIMS];
  for (int i = 0; i < d->n_keep; ++i) ms[i] = d->keep_sc[i] ? d->keep_sc[i] : 1;
  ProdMK k;
  dim3 g;
  const int r = pgmi_plan_product_marg(d, ops, C, ms, C, k, g);
  if (r <= 0) return r < 0 ? r : PGM_OK;  // shape not handled: *bound NULL, the generic kernel runs
  return pm_bind(d, ops, C, ms, PGM_RED_SUM, C, bound, nullptr, false);
}

// plan of the two-marginal pass; 1 = supported (q filled), 0 = not (caller runs two passes)
static int plan_two_marginals(const pgm_productn_desc *d, const double *const *ops, const int64_t *s1,
                              const int64_t *s2, const double *M1, const double *M2, PMMulti &q) {
  if (!d || !ops || !s1 || !s2 || !M1 || !M2) return pgmi_failf(PGM_EINVAL, "product_n_marginals: null argument");
  if (d->n_ops < 1 || d->n_ops > MOPS || d->n_keep < 2 || d->n_keep > PGM_MAX_DIMS) return 0;
  const int last = d->n_keep - 1;
  const int64_t NX = d->keep_card[last];
  if (NX < 64 || NX % 2 || d->keep_sc[last] != 1 || s1[last] != 1 || s2[last] != 1) return 0;
  if (((uintptr_t)M1 & 15) || ((uintptr_t)M2 & 15)) return 0;
  q = PMMulti();
  q.n_ops = d->n_ops;
  for (int t = 0; t < d->n_ops; ++t) {
    if (!ops[t] || d->op_kind[t] < 0 || d->op_kind[t] > 2) return pgmi_failf(PGM_EINVAL, "product_n_marginals: operand %d", t);
    const int64_t sx = d->keep_s[t][last];
    if (sx != 0 && sx != 1) return 0;
    if (sx == 1 && ((uintptr_t)ops[t] & 15)) return 0;
    q.vec[t] = sx == 1;
    q.kind[t] = d->op_kind[t];
  }
  uint64_t nk = 1, nu = 1;
  for (int i = 0; i < last; ++i) {
    const int64_t c = d->keep_card[i];
    if (c <= 0) return pgmi_failf(PGM_EINVAL, "product_n_marginals: keep_card[%d] <= 0", i);
    if (c == 1) continue;
    if ((s1[i] && s1[i] % 2) || (s2[i] && s2[i] % 2)) return 0;
    for (int t = 0; t < d->n_ops; ++t)
      if (q.vec[t] && d->keep_s[t][i] % 2) return 0;
    if (s1[i] && s2[i]) {
      if (q.nK >= KMAX) return 0;
      q.kcard[q.nK] = (unsigned)c;
      q.k1[q.nK] = s1[i];
      q.k2[q.nK] = s2[i];
      for (int t = 0; t < d->n_ops; ++t) q.ks[t][q.nK] = d->keep_s[t][i];
      ++q.nK;
      nk *= (uint64_t)c;
    } else if (s1[i] || s2[i]) {
      if (q.nU >= KMAX) return 0;
      q.ucard[q.nU] = (unsigned)c;
      q.u1[q.nU] = s1[i];
      q.u2[q.nU] = s2[i];
      for (int t = 0; t < d->n_ops; ++t) q.us[t][q.nU] = d->keep_s[t][i];
      ++q.nU;
      nu *= (uint64_t)c;
      if (s1[i]) q.n1 *= (unsigned)c;
      else q.n2 *= (unsigned)c;
    } else {
      if (q.nZ >= KMAX) return 0;
      q.zcard[q.nZ] = (unsigned)c;
      for (int t = 0; t < d->n_ops; ++t) q.zs[t][q.nZ] = d->keep_s[t][i];
      ++q.nZ;
    }
  }
  // register accumulators: the smaller target's own states, unrolled (8 / 32: no better, profiles/r02bv_c4_knobs.txt)
  static constexpr unsigned max_acc = 16u;
  (void)nu;
  if (std::min(q.n1, q.n2) > max_acc || nk >= (1ull << 31)) return 0;
  q.n_outer = (uint32_t)nk;
  q.NP = (uint32_t)(NX / 2);
  const uint64_t gx = (q.NP + 255) / 256;
  if (gx * nk < 256) return 0;  // fewer blocks than CUs: two single-marginal passes fill the chip better
  return 1;
}

int pgm_product_n_marginals_bind(const pgm_productn_desc *d, const double *const *ops, const int64_t *marg_s1,
                                 double *M1, const int64_t *marg_s2, double *M2, int32_t reduce, void **bound) {
  STALE_PROBE();
  if (!bound) return pgmi_failf(PGM_EINVAL, "product_n_marginals_bind: null bound");
  *bound = nullptr;
  if (reduce != PGM_RED_SUM && reduce != PGM_RED_MAX)
    return pgmi_failf(PGM_EINVAL, "product_n_marginals: reduce must be PGM_RED_SUM or PGM_RED_MAX");
  static const bool no_jit = getenv("PGM_NO_JIT") != nullptr || pm_knob("PGM_PM_JIT", 1) == 0;
  if (no_jit) return PGM_OK;
  PMSpec sp;
  const int r = plan_two_marginals(d, ops, marg_s1, marg_s2, M1, M2, sp.mm);
  if (r <= 0) return r;
  sp.multi = 1;
  sp.red = reduce;
  sp.store = false;
  sp.gx = (sp.mm.NP + 255) / 256;
  sp.total = (uint64_t)sp.gx * sp.mm.n_outer;
  sp.xcd = true;
  std::vector<uint64_t> starts;
  uint64_t blocks = 0;
  const std::string src = pm_source({sp}, starts, &blocks);
  PMBound *b = new (std::nothrow) PMBound;
  if (!b) return pgmi_failf(PGM_ENOMEM, "product_n_marginals_bind: out of host memory");
  b->src = src;
  b->blocks = (unsigned)blocks;
  b->specs.push_back(sp);
  for (int t = 0; t < d->n_ops; ++t) b->ptrs.push_back(ops[t]);
  b->ptrs.push_back(M1);  // the C slot
  b->ptrs.push_back(M2);  // the M slot
  *bound = b;
  return PGM_OK;
}

int pgm_product_n_marginal_source(const pgm_productn_desc *d, const double *const *ops, double *C,
                                  const int64_t *marg_s, int32_t reduce, double *M, char *buf, size_t len) {
  STALE_PROBE();
  if (!buf || len == 0) return pgmi_failf(PGM_EINVAL, "product_n_marginal_source: null buffer");
  void *unused = nullptr;
  std::string src;
  const int r = pm_bind(d, ops, C, marg_s, reduce, M, &unused, &src);
  if (r < 0) return r;
  const size_t n = std::min(len - 1, src.size());
  memcpy(buf, src.data(), n);
  buf[n] = 0;
  return (int)src.size();
}

int pgm_pm_bound_run(void *bound, void *stream) {
  STALE_PROBE();
  PMBound *b = (PMBound *)bound;
  if (!b) return pgmi_failf(PGM_EINVAL, "pm_bound_run: null bound");
  if (!b->fn) {
    const int r = pm_prepare(&b, 1);
    if (r != PGM_OK) return r;
  }
  size_t sz = b->ptrs.size() * sizeof(void *);
  void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, (void *)b->ptrs.data(), HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
  HIP_TRY(hipModuleLaunchKernel(b->fn, b->blocks, 1, 1, b->threads, 1, 1, 0, S(stream), nullptr, extra));
  return PGM_OK;
}

// a merged launch's kernel arguments stay within 4 KB (512 pointers); bodies per merged launch (a block finds
// its body through a balanced tree of block-range compares, so the count costs log2 compares; r06: 64 -> 128,
// C4's level 1 holds 74 specialised steps)
static constexpr size_t kPmMaxArgPtrs = 512;
static constexpr size_t kPmMaxTablePtrs = 8192;  // a specialised contraction batch's pointers through a table
static constexpr int kPmMaxBodies = 128;

int pgm_pm_merge(void *const *bounds, int32_t n, void **merged) {
  STALE_PROBE();
  if (!bounds || !merged || n < 1 || n > kPmMaxBodies) return pgmi_failf(PGM_EINVAL, "pm_merge: 1..%d bound steps", kPmMaxBodies);
  *merged = nullptr;
  std::vector<PMSpec> specs;
  std::vector<const double *> ptrs;
  for (int i = 0; i < n; ++i) {
    const PMBound *b = (const PMBound *)bounds[i];
    if (!b) return pgmi_failf(PGM_EINVAL, "pm_merge: null bound %d", i);
    if (b->specs.empty()) return pgmi_failf(PGM_EINVAL, "pm_merge: bound %d is a specialised contraction batch", i);
    specs.insert(specs.end(), b->specs.begin(), b->specs.end());
    ptrs.insert(ptrs.end(), b->ptrs.begin(), b->ptrs.end());
  }
  if (specs.size() > (size_t)kPmMaxBodies) return pgmi_failf(PGM_EINVAL, "pm_merge: more than %d bodies", kPmMaxBodies);
  if (ptrs.size() > kPmMaxArgPtrs) return PGM_OK;  // kernel arguments over 4 KB: keep the separate launches
  std::vector<uint64_t> starts;
  uint64_t blocks = 0;
  const std::string src = pm_source(specs, starts, &blocks);
  if (blocks >= (1ull << 31)) return PGM_OK;  // too large for one grid: keep the separate launches
  PMBound *m = new (std::nothrow) PMBound;
  if (!m) return pgmi_failf(PGM_ENOMEM, "pm_merge: out of host memory");
  m->src = src;
  m->blocks = (unsigned)blocks;
  m->specs = specs;
  m->ptrs = ptrs;
  *merged = m;
  return PGM_OK;
}

int pgm_pm_bound_source(void *bound, char *buf, size_t len) {
  STALE_PROBE();
  const PMBound *b = (const PMBound *)bound;
  if (!b || !buf || len == 0) return pgmi_failf(PGM_EINVAL, "pm_bound_source: null argument");
  const size_t n = std::min(len - 1, b->src.size());
  memcpy(buf, b->src.data(), n);
  buf[n] = 0;
  return (int)b->src.size();
}

int pgm_pm_prepare(void *const *bounds, int32_t n) {
  STALE_PROBE();
  if (!bounds || n < 0) return pgmi_failf(PGM_EINVAL, "pm_prepare: null bounds");
  return pm_prepare((PMBound *const *)bounds, n);
}

// a bound specialised launch as a direct AQL dispatch sees it (pgmdq.cpp): its code object, kernel name,
// grid and explicit argument segment (the flat pointer array)
int pgmi_pm_bound_jit(void *bound, pgmi_jit_launch *out) {
  PMBound *b = (PMBound *)bound;
  if (!b || !out) return pgmi_failf(PGM_EINVAL, "pm_bound_jit: null argument");
  if (!b->fn) {
    const int r = pm_prepare(&b, 1);
    if (r != PGM_OK) return r;
  }
  std::lock_guard<std::mutex> lk(g_pm_mu);
  const PMLoaded *e = pm_entry(b->src);
  if (!e || e->code.empty()) return pgmi_failf(PGM_EINVAL, "pm_bound_jit: no code object kept for this launch");
  out->code = e->code.data();
  out->code_size = e->code.size();
  out->kernel = "pgm_pm";
  out->args = b->ptrs.data();
  out->args_size = b->ptrs.size() * sizeof(void *);
  out->blocks = b->blocks;
  out->wg = b->threads;
  out->owner = b;
  out->write_through = 0;
  return PGM_OK;
}

int pgm_pm_bound_destroy(void *bound) {
  STALE_PROBE();
  delete (PMBound *)bound;
  return PGM_OK;
}

}  // extern "C"

// ----------------------------------------------------------------------------- specialised contraction batches
// A batch of contraction jobs (one dependency level of a compiled contraction path, C1 / C2; or the
// single-workgroup chain of its tiny last levels) as ONE generated kernel: each job's output decode
// (literal divisors), operand strides, reduction walk (literal nested loops, the generic kernels' entry
// order: reduction-outer dims slowest first, the innermost dim last) and lanes per output are
// literals, and a block finds its job by comparing its index with literal ranges — no block map, no
// descriptor loads (the generic k_batch_c reads a block map entry, then ~600 B of descriptor, before
// its first operand load; k_batch_wg_c reads its descriptors field by field from LDS).

static std::string cs_combine(int cmb, const std::string &a, const std::string &b) {
  switch (cmb) {
    case PGM_COMBINE_MUL: return "(" + a + " * " + b + ")";
    case PGM_COMBINE_ADD: return "(" + a + " + " + b + ")";
    case PGM_COMBINE_DIV: return "pgm_div0(" + a + ", " + b + ")";
    case PGM_COMBINE_DIV_RAW: return "(" + a + " / " + b + ")";
    default: return a;  // COPY
  }
}

static std::string cs_red(int red, const std::string &acc, const std::string &v) {
  if (red == PGM_RED_SUM) return acc + " = " + acc + " + " + v + ";";
  if (red == PGM_RED_MAX) return acc + " = pgm_maxn(" + acc + ", " + v + ");";
  return acc + " = " + v + ";";
}

// the job's output index decode: oa / ob / oc from idx (the kept dims, the last one fastest)
static void cs_decode(std::string &o, const ContractK &k, int nk, bool use_b, const char *ind) {
  for (int i = nk - 1; i >= 0; --i) {
    const unsigned d = k.kdiv[i].d;
    if (i == 0)
      pgmi_appendf(o, "%s{ const unsigned g_ = idx;", ind);
    else
      pgmi_appendf(o, "%s{ const unsigned q_ = idx / %uu, g_ = idx - q_ * %uu; idx = q_;", ind, d, d);
    if (k.ksa[i]) pgmi_appendf(o, " oa += (long long)g_ * %lldLL;", (long long)k.ksa[i]);
    if (use_b && k.ksb[i]) pgmi_appendf(o, " ob += (long long)g_ * %lldLL;", (long long)k.ksb[i]);
    if (k.ksc[i]) pgmi_appendf(o, " oc += (long long)g_ * %lldLL;", (long long)k.ksc[i]);
    o += " }\n";
  }
}

// nested loops over the reduction-outer dims (dim 0 outermost) opening; returns the offset expressions
static void cs_red_loops_open(std::string &o, const ContractK &k, std::string &ind, uint64_t inner_trip) {
  uint64_t prod = inner_trip;
  int first_unrolled = k.nr - 1;
  // the innermost reduction dims are unrolled while their trip product stays <= 64, so a 48-entry walk issues
  // its loads together instead of in six dependent rounds (r06q/r06r: C2 91.4 -> 88.6 us; 16 before, 256 no
  // better; PGM_CS_UNROLL_PROD is the A/B knob)
  static const uint64_t unroll_prod = getenv("PGM_CS_UNROLL_PROD") ? strtoull(getenv("PGM_CS_UNROLL_PROD"), nullptr, 10) : 64;
  for (int r = k.nr - 2; r >= 0; --r) {
    prod *= k.rdiv[r].d;
    if (prod > unroll_prod) break;
    first_unrolled = r;
  }
  for (int r = 0; r < k.nr - 1; ++r) {
    pgmi_appendf(o, "%s#pragma unroll%s\n", ind.c_str(), r >= first_unrolled ? "" : " 1");
    pgmi_appendf(o, "%sfor (unsigned r%d = 0; r%d < %uu; ++r%d) {\n", ind.c_str(), r, r, k.rdiv[r].d, r);
    ind += "  ";
  }
}

static void cs_red_loops_close(std::string &o, const ContractK &k, std::string &ind) {
  for (int r = 0; r < k.nr - 1; ++r) {
    ind.resize(ind.size() - 2);
    pgmi_appendf(o, "%s}\n", ind.c_str());
  }
}

static std::string cs_ro_off(const ContractK &k, bool a) {
  std::string e = "0LL";
  for (int r = 0; r < k.nr - 1; ++r) {
    const long long s = a ? (long long)k.rsa[r] : (long long)k.rsb[r];
    if (s) e += " + (long long)r" + std::to_string(r) + " * " + std::to_string(s) + "LL";
  }
  return e;
}

static std::string cs_job_body(const pgmi_cs_job &J, const std::string &name) {
  const ContractK &k = J.k;
  const bool use_b = J.cmb != PGM_COMBINE_COPY;
  const char *init = J.red == PGM_RED_MAX ? "-__builtin_inf()" : "0.0";
  std::string o;
  pgmi_appendf(o, "__device__ __forceinline__ void %s(unsigned tid, unsigned nth, const double *__restrict__ A, "
                  "const double *__restrict__ B, double *__restrict__ C) {\n  (void)B;\n", name.c_str());
  const std::string ra = cs_ro_off(k, true), rb = cs_ro_off(k, false);
  const unsigned RI = k.ri_card;
  if (k.row_mode == 2) {  // output pairs along the innermost kept dim, 16-B accesses (contract_flat2)
    const int kx = k.nk - 1;
    const bool va = k.ksa[kx] != 0, vb = use_b && k.ksb[kx] != 0;
    pgmi_appendf(o, "  for (unsigned q = tid; q < %uu; q += nth) {\n", k.n_out >> 1);
    o += "    unsigned idx = q << 1;\n    long long oa = 0, ob = 0, oc = 0; (void)ob;\n";
    cs_decode(o, k, k.nk, use_b, "    ");
    pgmi_appendf(o, "    double lo = %s, hi = %s;\n", init, init);
    std::string ind = "    ";
    cs_red_loops_open(o, k, ind, RI);
    pgmi_appendf(o, "%s#pragma unroll%s\n", ind.c_str(), RI <= 16 ? "" : " 4");
    pgmi_appendf(o, "%sfor (unsigned ri = 0; ri < %uu; ++ri) {\n", ind.c_str(), RI);
    const std::string in = ind + "  ";
    pgmi_appendf(o, "%sconst double *a_ = A + oa + %s + (long long)ri * %lldLL;\n", in.c_str(), ra.c_str(), (long long)k.ri_sa);
    if (va) pgmi_appendf(o, "%sconst pgm_d2 xa = *(const pgm_d2 *)a_;\n", in.c_str());
    else pgmi_appendf(o, "%sconst double xs_ = *a_; const pgm_d2 xa = {xs_, xs_};\n", in.c_str());
    if (use_b) {
      pgmi_appendf(o, "%sconst double *b_ = B + ob + %s + (long long)ri * %lldLL;\n", in.c_str(), rb.c_str(), (long long)k.ri_sb);
      if (vb) pgmi_appendf(o, "%sconst pgm_d2 xb = *(const pgm_d2 *)b_;\n", in.c_str());
      else pgmi_appendf(o, "%sconst double ys_ = *b_; const pgm_d2 xb = {ys_, ys_};\n", in.c_str());
    }
    pgmi_appendf(o, "%s%s\n", in.c_str(), cs_red(J.red, "lo", cs_combine(J.cmb, "xa.x", "xb.x")).c_str());
    pgmi_appendf(o, "%s%s\n", in.c_str(), cs_red(J.red, "hi", cs_combine(J.cmb, "xa.y", "xb.y")).c_str());
    pgmi_appendf(o, "%s}\n", ind.c_str());
    cs_red_loops_close(o, k, ind);
    o += "    *(pgm_d2 *)(C + oc) = (pgm_d2){lo, hi};\n  }\n}\n";
    return o;
  }
  const unsigned G = 1u << k.g_log2;
  // G lanes of an output at stride 64/G within a wave, as the n-ary jobs (cs_nary_body; PGM_NARY_LANEMAP)
  static const bool lanemap = !getenv("PGM_NARY_LANEMAP") || getenv("PGM_NARY_LANEMAP")[0] != '0';
  const bool lm = G > 1 && G < 64 && lanemap;
  if (lm) {
    const unsigned P = 64u / G;
    pgmi_appendf(o, "  const unsigned lane_g = (tid & 63u) / %uu;\n", P);
    pgmi_appendf(o, "  for (unsigned out = (tid >> 6) * %uu + (tid & %uu); out < %uu; out += (nth >> 6) * %uu) {\n", P, P - 1,
                 k.n_out, P);
  } else {
    if (G > 1) pgmi_appendf(o, "  const unsigned lane_g = tid & %uu;\n", G - 1);
    pgmi_appendf(o, "  for (unsigned out = tid >> %d; out < %uu; out += nth >> %d) {\n", k.g_log2, k.n_out, k.g_log2);
  }
  o += "    unsigned idx = out;\n    long long oa = 0, ob = 0, oc = 0; (void)ob;\n";
  cs_decode(o, k, k.nk, use_b, "    ");
  pgmi_appendf(o, "    double acc = %s;\n", init);
  std::string ind = "    ";
  cs_red_loops_open(o, k, ind, G > 1 ? (RI + G - 1) / G : RI);
  if (G > 1) {
    pgmi_appendf(o, "%sfor (unsigned ri = lane_g; ri < %uu; ri += %uu) {\n", ind.c_str(), RI, G);
  } else {
    pgmi_appendf(o, "%s#pragma unroll%s\n", ind.c_str(), RI <= 16 ? "" : " 8");
    pgmi_appendf(o, "%sfor (unsigned ri = 0; ri < %uu; ++ri) {\n", ind.c_str(), RI);
  }
  const std::string in = ind + "  ";
  std::string va = "A[oa + " + ra + " + (long long)ri * " + std::to_string((long long)k.ri_sa) + "LL]";
  std::string vb = "B[ob + " + rb + " + (long long)ri * " + std::to_string((long long)k.ri_sb) + "LL]";
  pgmi_appendf(o, "%s%s\n", in.c_str(), cs_red(J.red, "acc", cs_combine(J.cmb, va, vb)).c_str());
  pgmi_appendf(o, "%s}\n", ind.c_str());
  cs_red_loops_close(o, k, ind);
  if (G > 1 && J.red != PGM_RED_NONE)
    for (unsigned off = lm ? 32u : G >> 1; off > 0 && off >= (lm ? 64u / G : 1u); off >>= 1)
      pgmi_appendf(o, "    %s\n", cs_red(J.red, "acc", "__shfl_xor(acc, " + std::to_string(off) + ", 64)").c_str());
  pgmi_appendf(o, "    %sC[oc] = acc;\n  }\n}\n", G > 1 ? "if (lane_g == 0) " : "");
  return o;
}

// an evidence gather job (gather_body): C[out] = A[kept offset + sum_j code_j x stride_j], a code out of its
// variable's range raises the error flag and reads state 0
static std::string cs_gather_body(const pgmi_cs_job &J, const std::string &name) {
  const GatherK &g = J.g;
  std::string o;
  pgmi_appendf(o, "__device__ __forceinline__ void %s(unsigned tid, unsigned nth, const double *__restrict__ A, "
                  "const unsigned char *__restrict__ K, double *__restrict__ C, int *__restrict__ E) {\n"
                  "  (void)K; (void)E;\n", name.c_str());
  pgmi_appendf(o, "  for (unsigned out = tid; out < %uu; out += nth) {\n", g.n_out);
  o += "    unsigned idx = out, row = 0;\n    long long oa = 0, oc = 0;\n    (void)row;\n";
  for (int i = g.nk - 1; i >= 0; --i) {
    const unsigned d = g.kdiv[i].d;
    if (i == 0) o += "    { const unsigned g_ = idx;";
    else pgmi_appendf(o, "    { const unsigned q_ = idx / %uu, g_ = idx - q_ * %uu; idx = q_;", d, d);
    if (g.ksa[i]) pgmi_appendf(o, " oa += (long long)g_ * %lldLL;", (long long)g.ksa[i]);
    if (g.ksc[i]) pgmi_appendf(o, " oc += (long long)g_ * %lldLL;", (long long)g.ksc[i]);
    if (i == g.batch_dim) o += " row = g_;";
    o += " }\n";
  }
  for (int j = 0; j < g.n_ev; ++j) {
    pgmi_appendf(o, "    { unsigned c_ = K[%lldLL + (long long)row];", (long long)(g.ev_col[j] * g.ld + g.row0));
    pgmi_appendf(o, " if (c_ >= %uu) { if (E) atomicOr(E, 1); c_ = 0; }", (unsigned)g.ev_card[j]);
    pgmi_appendf(o, " oa += (long long)c_ * %lldLL; }\n", (long long)g.ev_stride[j]);
  }
  o += "    C[oc] = A[oa];\n  }\n}\n";
  return o;
}

// an n-ary contraction job (r06; pgm_batch_add_contract_n): C[out] = reduce over the reduction space of
// X_0 * X_1 * ... (a left fold), every decode and stride a literal; G lanes per output stride through the
// flattened reduction index (its digits decoded with literal divisors), else literal nested loops
static std::string cs_nary_body(const pgmi_cs_job &J, const std::string &name) {
  const ContractNK &k = J.n;
  const int n = k.n_ops;
  const bool mx = k.red == PGM_RED_MAX;
  const char *init = mx ? "-__builtin_inf()" : "0.0";
  std::string o;
  pgmi_appendf(o, "__device__ __forceinline__ void %s(unsigned tid, unsigned nth", name.c_str());
  for (int t = 0; t < n; ++t) pgmi_appendf(o, ", const double *__restrict__ X%d", t);
  o += ", double *__restrict__ C) {\n";
  const unsigned G = 1u << k.g_log2;
  // lanes of an output: G > 1 takes the G lanes of an output at stride 64/G within a wave (lane_g = the high
  // lane bits), so a wave's consecutive lanes hold consecutive outputs and an operand that is unit-stride
  // along the output's fastest dim is read in runs instead of one line per lane (PGM_NARY_LANEMAP=0: the G
  // lanes of an output adjacent, as before)
  static const bool lanemap = !getenv("PGM_NARY_LANEMAP") || getenv("PGM_NARY_LANEMAP")[0] != '0';
  if (G > 1 && G < 64 && lanemap) {
    const unsigned P = 64u / G;
    pgmi_appendf(o, "  const unsigned lane_g = (tid & 63u) / %uu;\n", P);
    pgmi_appendf(o, "  for (unsigned out = (tid >> 6) * %uu + (tid & %uu); out < %uu; out += (nth >> 6) * %uu) {\n", P, P - 1,
                 k.n_out, P);
  } else {
    if (G > 1) pgmi_appendf(o, "  const unsigned lane_g = tid & %uu;\n", G - 1);
    pgmi_appendf(o, "  for (unsigned out = tid >> %d; out < %uu; out += nth >> %d) {\n", k.g_log2, k.n_out, k.g_log2);
  }
  o += "    unsigned idx = out; long long oc = 0;";
  for (int t = 0; t < n; ++t) pgmi_appendf(o, " long long o%d = 0;", t);
  o += "\n";
  for (int i = k.nk - 1; i >= 0; --i) {
    const unsigned d = k.kcard[i];
    if (i == 0) o += "    { const unsigned g_ = idx;";
    else pgmi_appendf(o, "    { const unsigned q_ = idx / %uu, g_ = idx - q_ * %uu; idx = q_;", d, d);
    if (k.ksc[i]) pgmi_appendf(o, " oc += (long long)g_ * %lldLL;", (long long)k.ksc[i]);
    for (int t = 0; t < n; ++t)
      if (k.ks[t][i]) pgmi_appendf(o, " o%d += (long long)g_ * %lldLL;", t, (long long)k.ks[t][i]);
    o += " }\n";
  }
  auto prod = [&](const std::vector<std::string> &off) {
    std::string e = "X0[" + off[0] + "]";
    for (int t = 1; t < n; ++t) e = "(" + e + " * X" + std::to_string(t) + "[" + off[t] + "])";
    return e;
  };
  auto upd = [&](const std::string &v) {
    return mx ? "acc = pgm_maxn(acc, " + v + ");" : "acc = acc + " + v + ";";
  };
  pgmi_appendf(o, "    double acc = %s;\n", init);
  if (k.nr == 0) {
    std::vector<std::string> off;
    for (int t = 0; t < n; ++t) off.push_back("o" + std::to_string(t));
    o += "    acc = " + prod(off) + ";\n";
  } else if (G > 1) {
    // the G lanes of an output stride over the flattened index of the OUTER reduction dims [0, s) only — the
    // fewest outer dims whose product reaches G — and walk the inner dims [s, nr) as literal nested loops:
    // digits are decoded once per outer index instead of once per summed entry (r06; PGM_NARY_SPLIT=0: the
    // whole reduction index flattened and decoded per entry, as before)
    static const bool split = !getenv("PGM_NARY_SPLIT") || getenv("PGM_NARY_SPLIT")[0] != '0';
    int sd = k.nr;
    uint64_t pout = 1;
    for (int i = 0; i < k.nr; ++i) {
      pout *= k.rcard[i];
      if (pout >= G) {
        sd = i + 1;
        break;
      }
    }
    if (!split || sd >= k.nr) {
      sd = k.nr;
      pout = k.n_red;
    }
    pgmi_appendf(o, "    #pragma unroll %d\n    for (unsigned r = lane_g; r < %lluu; r += %uu) {\n      unsigned ri = r;",
                 sd == k.nr ? 4 : 1, (unsigned long long)pout, G);
    for (int t = 0; t < n; ++t) pgmi_appendf(o, " long long p%d = o%d;", t, t);
    o += "\n";
    if (sd < k.nr) {
      for (int i = sd - 1; i >= 0; --i) {
        const unsigned d = k.rcard[i];
        if (i == 0) o += "      { const unsigned g_ = ri;";
        else pgmi_appendf(o, "      { const unsigned q_ = ri / %uu, g_ = ri - q_ * %uu; ri = q_;", d, d);
        for (int t = 0; t < n; ++t)
          if (k.rs[t][i]) pgmi_appendf(o, " p%d += (long long)g_ * %lldLL;", t, (long long)k.rs[t][i]);
        o += " }\n";
      }
      static const uint64_t unroll_in = getenv("PGM_NARY_UNROLL_PROD") ? strtoull(getenv("PGM_NARY_UNROLL_PROD"), nullptr, 10) : 64;
      uint64_t inner = 1;
      int first_unrolled = k.nr;
      for (int r = k.nr - 1; r >= sd; --r) {
        inner *= k.rcard[r];
        if (inner > unroll_in) break;
        first_unrolled = r;
      }
      std::string ind = "      ";
      for (int r = sd; r < k.nr; ++r) {
        pgmi_appendf(o, "%s#pragma unroll%s\n", ind.c_str(), r >= first_unrolled ? "" : " 2");
        pgmi_appendf(o, "%sfor (unsigned r%d = 0; r%d < %uu; ++r%d) {\n", ind.c_str(), r, r, k.rcard[r], r);
        ind += "  ";
      }
      std::vector<std::string> off;
      for (int t = 0; t < n; ++t) {
        std::string e = "p" + std::to_string(t);
        for (int r = sd; r < k.nr; ++r)
          if (k.rs[t][r]) e += " + (long long)r" + std::to_string(r) + " * " + std::to_string((long long)k.rs[t][r]) + "LL";
        off.push_back(e);
      }
      o += ind + upd(prod(off)) + "\n";
      for (int r = sd; r < k.nr; ++r) {
        ind.resize(ind.size() - 2);
        o += ind + "}\n";
      }
      o += "    }\n";
    } else {
    for (int i = k.nr - 1; i >= 0; --i) {
      const unsigned d = k.rcard[i];
      if (i == 0) o += "      { const unsigned g_ = ri;";
      else pgmi_appendf(o, "      { const unsigned q_ = ri / %uu, g_ = ri - q_ * %uu; ri = q_;", d, d);
      for (int t = 0; t < n; ++t)
        if (k.rs[t][i]) pgmi_appendf(o, " p%d += (long long)g_ * %lldLL;", t, (long long)k.rs[t][i]);
      o += " }\n";
    }
    std::vector<std::string> off;
    for (int t = 0; t < n; ++t) off.push_back("p" + std::to_string(t));
    o += "      " + upd(prod(off)) + "\n    }\n";
    }
  } else {
    std::string ind = "    ";
    static const uint64_t unroll_prod = getenv("PGM_NARY_UNROLL_PROD") ? strtoull(getenv("PGM_NARY_UNROLL_PROD"), nullptr, 10) : 64;
    uint64_t inner = 1;
    int first_unrolled = k.nr;
    for (int r = k.nr - 1; r >= 0; --r) {
      inner *= k.rcard[r];
      if (inner > unroll_prod) break;
      first_unrolled = r;
    }
    for (int r = 0; r < k.nr; ++r) {
      pgmi_appendf(o, "%s#pragma unroll%s\n", ind.c_str(), r >= first_unrolled ? "" : " 2");
      pgmi_appendf(o, "%sfor (unsigned r%d = 0; r%d < %uu; ++r%d) {\n", ind.c_str(), r, r, k.rcard[r], r);
      ind += "  ";
    }
    std::vector<std::string> off;
    for (int t = 0; t < n; ++t) {
      std::string e = "o" + std::to_string(t);
      for (int r = 0; r < k.nr; ++r)
        if (k.rs[t][r]) e += " + (long long)r" + std::to_string(r) + " * " + std::to_string((long long)k.rs[t][r]) + "LL";
      off.push_back(e);
    }
    o += ind + upd(prod(off)) + "\n";
    for (int r = 0; r < k.nr; ++r) {
      ind.resize(ind.size() - 2);
      o += ind + "}\n";
    }
  }
  if (G > 1 && G < 64 && lanemap)
    for (unsigned off = 32; off >= 64u / G; off >>= 1)
      pgmi_appendf(o, "    %s\n", upd("__shfl_xor(acc, " + std::to_string(off) + ", 64)").c_str());
  else if (G > 1)
    for (unsigned off = G >> 1; off > 0; off >>= 1)
      pgmi_appendf(o, "    %s\n", upd("__shfl_xor(acc, " + std::to_string(off) + ", 64)").c_str());
  pgmi_appendf(o, "    %sC[oc] = acc;\n  }\n}\n", G > 1 ? "if (lane_g == 0) " : "");
  return o;
}

static int cs_nptrs(const pgmi_cs_job &J) { return J.kind == 2 ? J.n.n_ops + 1 : J.kind == 1 ? 4 : 3; }

int pgmi_cs_bind(const pgmi_cs_job *jobs, int n, const uint32_t *level_off, int n_levels, int one_wg, void **bound) {
  *bound = nullptr;
  static const bool no_jit = getenv("PGM_NO_JIT") != nullptr;
  // (a block finds its job through a balanced tree of literal comparisons: with a linear chain the
  // 130 / 87 / 64-job C2 levels ran 3-4x slower than the generic kernel; with the tree every level is
  // faster specialised, r05i: C2 0.148 ms/query with 24 jobs at most per specialised level, 0.129 with
  // no limit but the kernel-argument budget of 170 jobs)
  std::vector<int> base(n + 1, 0);
  for (int j = 0; j < n; ++j) base[j + 1] = base[j] + cs_nptrs(jobs[j]);
  // over 512 pointers (4 KB of kernel arguments) the kernel reads them from a table in device memory instead
  // (r06: C2's first path level is 106 jobs / ~600 pointers; as two kernels its second packet cost ~2.5 us)
  const bool table = base[n] > (int)kPmMaxArgPtrs;
  if (no_jit || n < 1 || base[n] > (int)kPmMaxTablePtrs) return PGM_OK;
  for (int j = 0; j < n; ++j) {
    if (jobs[j].kind == 1) {
      const GatherK &g = jobs[j].g;
      if (g.nk < 0 || g.nk > KMAX || g.n_ev < 0 || g.n_ev > PGM_MAX_DIMS) return PGM_OK;  // nk 0: one output
      continue;
    }
    if (jobs[j].kind == 2) {
      const ContractNK &c = jobs[j].n;
      if (c.n_ops < 1 || c.n_ops > MOPS || c.nk < 0 || c.nk > KMAX || c.nr < 0 || c.nr > KMAX) return PGM_OK;
      continue;
    }
    const ContractK &k = jobs[j].k;
    if (k.n_split != 1 || (k.row_mode != 0 && k.row_mode != 2) || k.nk < 0 || k.nk > KMAX || k.nr > KMAX ||
        (k.row_mode == 2 && k.nk < 1))
      return PGM_OK;
  }
  std::string o =
      "#pragma clang fp contract(off)\n"  // products rounded before they are summed, as numpy does
      "typedef double pgm_d2 __attribute__((ext_vector_type(2)));\n"
      "__device__ __forceinline__ double pgm_div0(double a, double b) { const double r = a / b; "
      "return r != r ? 0.0 : r; }\n"
      "__device__ __forceinline__ double pgm_maxn(double a, double b) { return (a > b || a != a) ? a : b; }\n";
  for (int j = 0; j < n; ++j)
    o += jobs[j].kind == 1   ? cs_gather_body(jobs[j], "cj" + std::to_string(j))
         : jobs[j].kind == 2 ? cs_nary_body(jobs[j], "cj" + std::to_string(j))
                             : cs_job_body(jobs[j], "cj" + std::to_string(j));
  if (table)
    o += "struct pgm_pm_args { const double *const *__restrict__ p; };\n";
  else
    pgmi_appendf(o, "struct pgm_pm_args { const double *p[%d]; };\n", base[n]);
  // jobs [j0, j1) by block b: a balanced tree of literal comparisons (the jobs' block ranges ascend)
  std::function<void(std::string &, int, int, std::string)> dispatch = [&](std::string &s, int j0, int j1,
                                                                            std::string ind) {
    if (j1 - j0 == 1) {
      const pgmi_cs_job &J = jobs[j0];
      const int p0 = base[j0];
      if (J.kind == 1)
        pgmi_appendf(s, "%scj%d((b - %uu) * 256u + lt, %uu, a.p[%d], (const unsigned char *)a.p[%d], (double *)a.p[%d], "
                        "(int *)a.p[%d]);\n", ind.c_str(), j0, J.block0, J.nblocks * 256u, p0, p0 + 1, p0 + 2, p0 + 3);
      else if (J.kind == 2) {
        pgmi_appendf(s, "%scj%d((b - %uu) * 256u + lt, %uu", ind.c_str(), j0, J.block0, J.nblocks * 256u);
        for (int t = 0; t < J.n.n_ops; ++t) pgmi_appendf(s, ", a.p[%d]", p0 + t);
        pgmi_appendf(s, ", (double *)a.p[%d]);\n", p0 + J.n.n_ops);
      } else
        pgmi_appendf(s, "%scj%d((b - %uu) * 256u + lt, %uu, a.p[%d], a.p[%d], (double *)a.p[%d]);\n", ind.c_str(), j0,
                     J.block0, J.nblocks * 256u, p0, p0 + 1, p0 + 2);
      return;
    }
    const int m = (j0 + j1) / 2;
    pgmi_appendf(s, "%sif (b < %uu) {\n", ind.c_str(), jobs[m].block0);
    dispatch(s, j0, m, ind + "  ");
    pgmi_appendf(s, "%s} else {\n", ind.c_str());
    dispatch(s, m, j1, ind + "  ");
    pgmi_appendf(s, "%s}\n", ind.c_str());
  };
  unsigned blocks = 0, threads = 256;
  if (!one_wg) {
    uint64_t nb = 0;
    for (int j = 0; j < n; ++j) nb = std::max<uint64_t>(nb, (uint64_t)jobs[j].block0 + jobs[j].nblocks);
    if (nb == 0 || nb >= (1ull << 31)) return PGM_OK;
    blocks = (unsigned)nb;
    o += "extern \"C\" __global__ void __launch_bounds__(256) pgm_pm(const pgm_pm_args a) {\n"
         "  const unsigned b = blockIdx.x, lt = threadIdx.x;\n";
    dispatch(o, 0, n, "  ");
    o += "}\n";
  } else {
    // one 1,024-thread workgroup: each level's blocks four at a time (virtual 256-thread blocks), a
    // workgroup barrier after each level (the next level reads what this workgroup wrote)
    blocks = 1;
    threads = 1024;
    o += "extern \"C\" __global__ void __launch_bounds__(1024) pgm_pm(const pgm_pm_args a) {\n"
         "  const unsigned vb = threadIdx.x / 256u, lt = threadIdx.x % 256u;\n";
    int j = 0;
    for (int l = 0; l < n_levels; ++l) {
      const uint32_t b0 = level_off[l], b1 = level_off[l + 1];
      int j1 = j;
      while (j1 < n && jobs[j1].block0 < b1) ++j1;
      pgmi_appendf(o, "  for (unsigned b = %uu + vb; b < %uu; b += 4u) {\n", b0, b1);
      if (j1 > j) dispatch(o, j, j1, "    ");
      o += "  }\n  __syncthreads();\n";
      j = j1;
    }
    if (j != n) return PGM_OK;  // jobs outside the level table: not a shape this form takes
    o += "}\n";
  }
  PMBound *b = new (std::nothrow) PMBound;
  if (!b) return pgmi_failf(PGM_ENOMEM, "batch_specialise: out of host memory");
  b->src = o;
  b->blocks = blocks;
  b->threads = threads;
  for (int q = 0; q < n; ++q) {
    if (jobs[q].kind == 2) {
      for (int t = 0; t < jobs[q].n.n_ops; ++t) b->ptrs.push_back(jobs[q].ops[t]);
      b->ptrs.push_back(jobs[q].C);
      continue;
    }
    b->ptrs.push_back(jobs[q].A);
    if (jobs[q].kind == 1) {
      b->ptrs.push_back((const double *)jobs[q].codes);
      b->ptrs.push_back(jobs[q].C);
      b->ptrs.push_back((const double *)jobs[q].err);
    } else {
      b->ptrs.push_back(jobs[q].B);
      b->ptrs.push_back(jobs[q].C);
    }
  }
  if (table) {
    const size_t bytes = b->ptrs.size() * sizeof(void *);
    hipError_t e = hipMalloc(&b->table, bytes);
    if (e == hipSuccess) e = hipMemcpy(b->table, b->ptrs.data(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      delete b;
      return pgmi_failf(e == hipErrorOutOfMemory ? PGM_ENOMEM : PGM_EDEVICE, "batch_specialise: pointer table: %s",
                        hipGetErrorString(e));
    }
    b->ptrs.assign(1, (const double *)b->table);
  }
  *bound = b;
  return PGM_OK;
}
