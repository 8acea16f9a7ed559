// pgmhip.hip — gfx950 (MI355X / CDNA4) kernels + C-ABI of the discrete-factor engine.
//
// Built for gfx950 only:  hipcc --offload-arch=gfx950 -O3 -fPIC -shared
// (pgmpy_amd/build.py).  Declarations and the reference call site each entry
// point replaces: include/pgmhip.h.  Design, data layout and the roofline of
// every kernel: DESIGN.md.
//
// Kernels
//   k_contract / k_contract_final  generic strided broadcast-combine + axis reduce (HBM-bound)
//   k_gather                       batched evidence reduce (gather by per-row state codes)
//   k_indicator                    0/1 evidence indicators (BP findings)
//   k_argmax                       first-index argmax per row
//   k_rows                         fused per-row plan: reduce -> sum-product -> normalize ->
//                                  marginals / joint / MAP, one lane per evidence row
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <sys/stat.h>
#include <unistd.h>

#include "pgmhip.h"
#include "pgm_internal.h"

#define PGM_ABI_VERSION 23  // 23: pgm_batch_add_contract_n (n-ary contraction jobs), pgm_dq_timer_dispatch_times, pgm_host_scan_* / pgm_host_lut_map_u8; 22: pgm_dq_bind_pm / pgm_dq_run_chain / pgm_dq_profiling; 21: pgm_batch_specialise; 20: pgm_batch_info and the grid-barrier levelled batch removed (levels: single-workgroup mode only); 19: pgm_stream_sync_spin; 18: pgm_batch_set_mode (single-workgroup levelled batch), pgm_batch_blocks; 17: pgm_rows_shard_run (rows sharded over several GPUs from host buffers); 16: pgm_rows_ring_start_ready; 15: pgm_batch_add_level / pgm_batch_info (levelled batch), pgm_memcpy_d2h_async; 14: pgm_rows_ring_* (resident ring of row batches); 13: pgm_dq_timer_dispatch_stats, pgm_rows_bound_kernel; 12: pgm_dq_launch_group, pgm_dq_timer_stop_ticks, PGM_ROWS_FLOOR; 11: pgm_product_n_marginal_bind / pgm_pm_bound_*; 10: pgm_dq_* direct AQL dispatch, pgm_codes_remap; 9: gemm lane_order, batch product_n / indicator

// ----------------------------------------------------------------------------- errors
static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      (void)hipGetLastError();                                                           \
      return fail(e_ == hipErrorOutOfMemory ? PGM_ENOMEM : PGM_EDEVICE, "%s: %s", #expr, \
                  hipGetErrorString(e_));                                                \
    }                                                                                    \
  } while (0)

// debugging aid (PGM_STALE_PROBE=1): report a pending HIP error left by an earlier call when a C-ABI
// entry point starts, so a launch check is not blamed for someone else's error
void pgmi_stale_probe(const char *fn) {
  static const bool on = getenv("PGM_STALE_PROBE") != nullptr;
  if (!on) return;
  const hipError_t e = hipPeekAtLastError();
  if (e != hipSuccess) fprintf(stderr, "pgmhip: pending HIP error at entry of %s: %s\n", fn, hipGetErrorString(e));
}

static inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ----------------------------------------------------------------------------- fast division
// n / d for n < 2^31 with one mul-hi and one shift (Granlund-Montgomery round-up method).
static FDiv make_fdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FDiv{d, (uint32_t)m, l};
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FDiv &f) {
  uint32_t t = __umulhi(n, f.m);
  return (t + n) >> f.s;
}

__device__ __forceinline__ double max_nan(double a, double b) {
  // np.max semantics: NaN propagates
  return (a > b || a != a) ? a : b;
}

// ----------------------------------------------------------------------------- contract

// ContractK (the planned flat / row-mode contraction): pgm_internal.h

template <int CMB>
__device__ __forceinline__ double combine(double a, double b) {
  if constexpr (CMB == PGM_COMBINE_MUL) return a * b;
  if constexpr (CMB == PGM_COMBINE_ADD) return a + b;
  if constexpr (CMB == PGM_COMBINE_DIV) {
    double r = a / b;
    return (r != r) ? 0.0 : r;  // DiscreteFactor.py:863 values[isnan] = 0
  }
  if constexpr (CMB == PGM_COMBINE_DIV_RAW) return a / b;
  return a;  // COPY
}

template <int RED>
__device__ __forceinline__ double red_init() {
  if constexpr (RED == PGM_RED_MAX) return -__builtin_inf();
  return 0.0;
}

template <int RED>
__device__ __forceinline__ double red_op(double acc, double v) {
  if constexpr (RED == PGM_RED_SUM) return acc + v;
  if constexpr (RED == PGM_RED_MAX) return max_nan(acc, v);
  return v;
}

// reduction-outer index -> offsets (wave-uniform when ro is)
__device__ __forceinline__ void decode_ro(const ContractK &p, uint32_t ro, int64_t &ra, int64_t &rb) {
  ra = 0;
  rb = 0;
  for (int k = p.nr - 2; k >= 0; --k) {
    const uint32_t q = fdiv(ro, p.rdiv[k]);
    const uint32_t dg = ro - q * p.rdiv[k].d;
    ra += (int64_t)dg * p.rsa[k];
    rb += (int64_t)dg * p.rsb[k];
    ro = q;
  }
}

// Flat mode: G lanes cooperate on one output (any keep layout); lanes stride the innermost
// reduction dim, the reduction-outer index is walked wave-uniformly.  `tid` / `nthreads` are the
// thread's index and the thread count of the launch (or of its job in a batched launch).
template <int CMB, int RED>
__device__ __forceinline__ void contract_flat(const ContractK &p, const double *__restrict__ A,
                                              const double *__restrict__ B, double *__restrict__ C,
                                              double *__restrict__ ws, uint64_t tid, uint64_t nthreads,
                                              uint32_t split) {
  const uint32_t G = 1u << p.g_log2;
  const uint32_t lane_g = (uint32_t)tid & (G - 1);
  const uint64_t ngroups = nthreads >> p.g_log2;
  const uint32_t r0 = split * p.red_chunk;
  const uint32_t r1 = min(p.n_ro, r0 + p.red_chunk);
  for (uint64_t out = tid >> p.g_log2; out < p.n_out; out += ngroups) {
    int64_t oa = 0, ob = 0, oc = 0;
    uint32_t idx = (uint32_t)out;
    for (int k = p.nk - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
      oa += (int64_t)dg * p.ksa[k];
      if constexpr (CMB != PGM_COMBINE_COPY) ob += (int64_t)dg * p.ksb[k];
      oc += (int64_t)dg * p.ksc[k];
      idx = q;
    }
    double acc = red_init<RED>();
    if (G == 1) {
      // one lane per output: the reduction entries (reduction-outer major, innermost minor — the
      // summation order of the loop below) UNR at a time, every operand load of a group issued before
      // the group is summed, so a long reduction is not one memory round trip per entry (the entry
      // walk is wave-uniform: scalar offsets and branches)
      constexpr int UNR = 8;
      const uint32_t total = (r1 > r0 ? r1 - r0 : 0u) * p.ri_card;
      uint32_t ro = r0, ri = 0;
      int64_t ra = 0, rb = 0;
      if (total) decode_ro(p, ro, ra, rb);
      for (uint32_t e = 0; e < total; e += UNR) {
        double xa[UNR], xb[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (e + u < total) {
            xa[u] = A[oa + ra + (int64_t)ri * p.ri_sa];
            if constexpr (CMB != PGM_COMBINE_COPY) xb[u] = B[ob + rb + (int64_t)ri * p.ri_sb];
            if (++ri == p.ri_card) {
              ri = 0;
              if (++ro < r1) decode_ro(p, ro, ra, rb);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (e + u < total) {
            if constexpr (CMB == PGM_COMBINE_COPY)
              acc = red_op<RED>(acc, xa[u]);
            else
              acc = red_op<RED>(acc, combine<CMB>(xa[u], xb[u]));
          }
        }
      }
    } else {
      // G lanes per output, each striding the innermost reduction dim from its lane; this lane's entries
      // (reduction-outer major, its innermost indices minor — the summation order of the r03 loop) are
      // walked UNR at a time with every operand load of a group issued before the group is summed (r04:
      // the r03 loop waited for each load before the next, one memory round trip per entry — C2's levels
      // with long reduction-outer walks; same order, bit-identical sums).  G <= ri_card (host plan), so
      // every lane has at least one entry per reduction-outer index.
      constexpr int UNR = 8;
      uint32_t ro = r0, ri = lane_g;
      int64_t ra = 0, rb = 0;
      bool live = ro < r1;
      if (live) decode_ro(p, ro, ra, rb);
      while (live) {
        double xa[UNR], xb[UNR];
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (live) {
            xa[u] = A[oa + ra + (int64_t)ri * p.ri_sa];
            if constexpr (CMB != PGM_COMBINE_COPY) xb[u] = B[ob + rb + (int64_t)ri * p.ri_sb];
            cnt = u + 1;
            ri += G;
            if (ri >= p.ri_card) {
              ri = lane_g;
              if (++ro < r1) decode_ro(p, ro, ra, rb);
              else live = false;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (u < cnt) {
            if constexpr (CMB == PGM_COMBINE_COPY)
              acc = red_op<RED>(acc, xa[u]);
            else
              acc = red_op<RED>(acc, combine<CMB>(xa[u], xb[u]));
          }
        }
      }
    }
    if constexpr (RED != PGM_RED_NONE) {
      for (uint32_t off = G >> 1; off > 0; off >>= 1) acc = red_op<RED>(acc, __shfl_xor(acc, (int)off, 64));
    }
    if (lane_g == 0) {
      if (p.n_split == 1)
        C[oc] = acc;
      else
        ws[(uint64_t)split * p.n_out + out] = acc;
    }
  }
}

// Flat mode over output PAIRS along the innermost kept dim, one lane per pair, 16-B accesses (batched
// BP separator marginals: rows innermost).  Host-checked (pgm_batch_add_contract): even innermost kept
// extent, output innermost stride 1, each operand's innermost kept stride 0 or 1, every other stride
// of a 16-B-read operand even, bases 16-B aligned.  Same summation order as contract_flat with G = 1.
template <int CMB, int RED>
__device__ __forceinline__ void contract_flat2(const ContractK &p, const double *__restrict__ A,
                                               const double *__restrict__ B, double *__restrict__ C, uint64_t tid,
                                               uint64_t nthreads) {
  const int kx = p.nk - 1;
  const bool va = p.ksa[kx] != 0, vb = p.ksb[kx] != 0;
  const uint32_t n_pairs = p.n_out >> 1;
  for (uint64_t q = tid; q < n_pairs; q += nthreads) {
    int64_t oa = 0, ob = 0, oc = 0;
    uint32_t idx = (uint32_t)q << 1;
    for (int k = kx; k >= 0; --k) {
      const uint32_t qq = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - qq * p.kdiv[k].d;
      oa += (int64_t)dg * p.ksa[k];
      if constexpr (CMB != PGM_COMBINE_COPY) ob += (int64_t)dg * p.ksb[k];
      oc += (int64_t)dg * p.ksc[k];
      idx = qq;
    }
    double lo = red_init<RED>(), hi = red_init<RED>();
    // the reduction entries in order (reduction-outer major), UNR at a time with every load of a group
    // issued before it is summed (see contract_flat)
    constexpr int UNR = 4;
    const uint32_t total = p.n_ro * p.ri_card;
    uint32_t ro = 0, ri = 0;
    int64_t ra = 0, rb = 0;
    if (total) decode_ro(p, ro, ra, rb);
    for (uint32_t e = 0; e < total; e += UNR) {
      double2 xa[UNR], xb[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (e + u < total) {
          const double *a = A + oa + ra + (int64_t)ri * p.ri_sa;
          if (va) {
            xa[u] = *(const double2 *)a;
          } else {
            xa[u].x = xa[u].y = *a;
          }
          if constexpr (CMB != PGM_COMBINE_COPY) {
            const double *b = B + ob + rb + (int64_t)ri * p.ri_sb;
            if (vb) {
              xb[u] = *(const double2 *)b;
            } else {
              xb[u].x = xb[u].y = *b;
            }
          }
          if (++ri == p.ri_card) {
            ri = 0;
            if (++ro < p.n_ro) decode_ro(p, ro, ra, rb);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (e + u < total) {
          double xl = xa[u].x, xh = xa[u].y;
          if constexpr (CMB != PGM_COMBINE_COPY) {
            xl = combine<CMB>(xl, xb[u].x);
            xh = combine<CMB>(xh, xb[u].y);
          }
          lo = red_op<RED>(lo, xl);
          hi = red_op<RED>(hi, xh);
        }
      }
    }
    *(double2 *)(C + oc) = make_double2(lo, hi);
  }
}

template <int CMB, int RED>
__global__ __launch_bounds__(256) void k_contract(const ContractK p, const double *__restrict__ A,
                                                  const double *__restrict__ B, double *__restrict__ C,
                                                  double *__restrict__ ws) {
  contract_flat<CMB, RED>(p, A, B, C, ws, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x,
                          (uint64_t)gridDim.x * blockDim.x, blockIdx.y);
}

// Row mode: the innermost keep dim runs across the lanes (coalesced when it is innermost in the
// operands, e.g. the evidence-row axis), the outer keep index and the reduction-outer index are
// wave-uniform (scalar decode), the innermost reduction dim is walked by increments.
template <int CMB>
__device__ __forceinline__ double ld_combine(const double *a, const double *b, int64_t ia, int64_t ib) {
  if constexpr (CMB == PGM_COMBINE_COPY)
    return a[ia];
  else
    return combine<CMB>(a[ia], b[ib]);
}

// Row mode: the innermost keep dim runs across the lanes (coalesced when it is innermost in the
// operands, e.g. the evidence-row axis), the outer keep index and the reduction-outer index are
// wave-uniform (scalar decode), the innermost reduction dim is walked by increments.  Loops are
// unrolled 4-wide with independent accumulators so each lane keeps 4-8 loads in flight.
template <int CMB, int RED>
__global__ __launch_bounds__(256) void k_contract_rows(const ContractK p, const double *__restrict__ A,
                                                       const double *__restrict__ B, double *__restrict__ C,
                                                       double *__restrict__ ws) {
  // grid: x-blocks stride the innermost keep dim, y-blocks stride the outer keep index, z = split.
  // A block decodes an outer index once (wave-uniform, scalar) and reuses it for all its rows.
  const int kx = p.nk - 1;
  const uint32_t NX = p.kdiv[kx].d;
  const int64_t sxa = p.ksa[kx], sxb = p.ksb[kx], sxc = p.ksc[kx];
  const uint32_t n_outer = p.n_out / NX;
  const uint32_t xstep = gridDim.x * blockDim.x;
  auto decode_o = [&](uint32_t idx, int64_t &oa, int64_t &ob, int64_t &oc) {
    oa = ob = oc = 0;
    for (int k = kx - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
      oa += (int64_t)dg * p.ksa[k];
      if constexpr (CMB != PGM_COMBINE_COPY) ob += (int64_t)dg * p.ksb[k];
      oc += (int64_t)dg * p.ksc[k];
      idx = q;
    }
  };
  if constexpr (RED == PGM_RED_NONE) {
    for (uint32_t o = blockIdx.y; o < n_outer; o += gridDim.y) {
      int64_t oa, ob, oc;
      decode_o(o, oa, ob, oc);
      uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
      for (; x + 3 * xstep < NX; x += 4 * xstep) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t xx = x + u * xstep;
          v[u] = ld_combine<CMB>(A, B, oa + xx * sxa, ob + xx * sxb);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) C[oc + (int64_t)(x + u * xstep) * sxc] = v[u];
      }
      for (; x < NX; x += xstep) C[oc + (int64_t)x * sxc] = ld_combine<CMB>(A, B, oa + (int64_t)x * sxa, ob + (int64_t)x * sxb);
    }
    return;
  }
  const uint32_t split = blockIdx.z;
  const uint32_t v0 = split * p.red_chunk;
  const uint32_t v1 = min(p.n_v, v0 + p.red_chunk);
  const uint32_t nb = p.ri_nb, CH = p.ri_chunk, RI = p.ri_card;
  for (uint32_t o = blockIdx.y; o < n_outer; o += gridDim.y) {
    int64_t oa, ob, oc;
    decode_o(o, oa, ob, oc);
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < NX; x += xstep) {
      const double *a = A + oa + (int64_t)x * sxa;
      const double *b = B + ob + (int64_t)x * sxb;
      double acc0 = red_init<RED>(), acc1 = acc0, acc2 = acc0, acc3 = acc0;
      for (uint32_t v = v0; v < v1; ++v) {
        const uint32_t ro = nb == 1 ? v : v / nb;
        const uint32_t bk = v - ro * nb;
        int64_t ra, rb;
        decode_ro(p, ro, ra, rb);
        const uint32_t ri1 = min(RI, (bk + 1) * CH);
        uint32_t ri = bk * CH;
        for (; ri + 4 <= ri1; ri += 4) {
          const double w0 = ld_combine<CMB>(a, b, ra + (int64_t)ri * p.ri_sa, rb + (int64_t)ri * p.ri_sb);
          const double w1 = ld_combine<CMB>(a, b, ra + (int64_t)(ri + 1) * p.ri_sa, rb + (int64_t)(ri + 1) * p.ri_sb);
          const double w2 = ld_combine<CMB>(a, b, ra + (int64_t)(ri + 2) * p.ri_sa, rb + (int64_t)(ri + 2) * p.ri_sb);
          const double w3 = ld_combine<CMB>(a, b, ra + (int64_t)(ri + 3) * p.ri_sa, rb + (int64_t)(ri + 3) * p.ri_sb);
          acc0 = red_op<RED>(acc0, w0);
          acc1 = red_op<RED>(acc1, w1);
          acc2 = red_op<RED>(acc2, w2);
          acc3 = red_op<RED>(acc3, w3);
        }
        for (; ri < ri1; ++ri) acc0 = red_op<RED>(acc0, ld_combine<CMB>(a, b, ra + (int64_t)ri * p.ri_sa, rb + (int64_t)ri * p.ri_sb));
      }
      const double acc = red_op<RED>(red_op<RED>(acc0, acc1), red_op<RED>(acc2, acc3));
      if (p.n_split == 1)
        C[oc + (int64_t)x * sxc] = acc;
      else
        ws[(uint64_t)split * p.n_out + (uint64_t)o * NX + x] = acc;
    }
  }
}

// Row mode, short reduction (n_red <= 512, no split): every reduction offset is decoded once per
// block into LDS, then each row sums flat over them with 8 loads and 8 accumulators in flight
// (a BP separator marginal: a few clique variables summed for every (separator state, row)).
#define RTAB_MAX 512
template <int CMB, int RED>
__global__ __launch_bounds__(256) void k_contract_rows_tab(const ContractK p, const double *__restrict__ A,
                                                           const double *__restrict__ B, double *__restrict__ C) {
  __shared__ int64_t sra[RTAB_MAX], srb[RTAB_MAX];
  const uint32_t NR = p.n_red;
  for (uint32_t j = threadIdx.x; j < NR; j += blockDim.x) {
    const uint32_t ro = j / p.ri_card, ri = j - ro * p.ri_card;
    int64_t ra, rb;
    decode_ro(p, ro, ra, rb);
    sra[j] = ra + (int64_t)ri * p.ri_sa;
    srb[j] = rb + (int64_t)ri * p.ri_sb;
  }
  __syncthreads();
  const int kx = p.nk - 1;
  const uint32_t NX = p.kdiv[kx].d;
  const int64_t sxa = p.ksa[kx], sxb = p.ksb[kx], sxc = p.ksc[kx];
  const uint32_t n_outer = p.n_out / NX;
  const uint32_t xstep = gridDim.x * blockDim.x;
  for (uint32_t o = blockIdx.y; o < n_outer; o += gridDim.y) {
    int64_t oa = 0, ob = 0, oc = 0;
    uint32_t idx = o;
    for (int k = kx - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
      oa += (int64_t)dg * p.ksa[k];
      if constexpr (CMB != PGM_COMBINE_COPY) ob += (int64_t)dg * p.ksb[k];
      oc += (int64_t)dg * p.ksc[k];
      idx = q;
    }
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < NX; x += xstep) {
      const double *a = A + oa + (int64_t)x * sxa;
      const double *b = B + ob + (int64_t)x * sxb;
      double acc[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] = red_init<RED>();
      uint32_t j = 0;
      for (; j + 8 <= NR; j += 8) {
        double w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = ld_combine<CMB>(a, b, sra[j + u], srb[j + u]);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = red_op<RED>(acc[u], w[u]);
      }
      for (; j < NR; ++j) acc[0] = red_op<RED>(acc[0], ld_combine<CMB>(a, b, sra[j], srb[j]));
#pragma unroll
      for (int u = 1; u < 8; ++u) acc[0] = red_op<RED>(acc[0], acc[u]);
      C[oc + (int64_t)x * sxc] = acc[0];
    }
  }
}

// k_contract_rows_tab for a plain marginal (COPY), two rows per lane with 16-B loads/stores.
// Host-checked: even row count, row stride 1 in A and C, every other A/C stride even, bases 16-B aligned.
template <int RED>
__global__ __launch_bounds__(256) void k_contract_rows_tab2(const ContractK p, const double *__restrict__ A,
                                                            double *__restrict__ C) {
  __shared__ int64_t sra[RTAB_MAX];
  const uint32_t NR = p.n_red;
  for (uint32_t j = threadIdx.x; j < NR; j += blockDim.x) {
    const uint32_t ro = j / p.ri_card, ri = j - ro * p.ri_card;
    int64_t ra, rb;
    decode_ro(p, ro, ra, rb);
    sra[j] = (ra + (int64_t)ri * p.ri_sa) >> 1;  // in double2 units
  }
  __syncthreads();
  const int kx = p.nk - 1;
  const uint32_t NP = p.kdiv[kx].d >> 1;
  const uint32_t n_outer = p.n_out / p.kdiv[kx].d;
  const uint32_t xstep = gridDim.x * blockDim.x;
  for (uint32_t o = blockIdx.y; o < n_outer; o += gridDim.y) {
    int64_t oa = 0, oc = 0;
    uint32_t idx = o;
    for (int k = kx - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
      oa += (int64_t)dg * p.ksa[k];
      oc += (int64_t)dg * p.ksc[k];
      idx = q;
    }
    const double2 *a2 = (const double2 *)(A + oa);
    double2 *c2 = (double2 *)(C + oc);
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < NP; x += xstep) {
      const double2 *a = a2 + x;
      double2 acc[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] = make_double2(red_init<RED>(), red_init<RED>());
      uint32_t j = 0;
      for (; j + 8 <= NR; j += 8) {
        double2 w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = a[sra[j + u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc[u].x = red_op<RED>(acc[u].x, w[u].x);
          acc[u].y = red_op<RED>(acc[u].y, w[u].y);
        }
      }
      for (; j < NR; ++j) {
        const double2 w = a[sra[j]];
        acc[0].x = red_op<RED>(acc[0].x, w.x);
        acc[0].y = red_op<RED>(acc[0].y, w.y);
      }
#pragma unroll
      for (int u = 1; u < 8; ++u) {
        acc[0].x = red_op<RED>(acc[0].x, acc[u].x);
        acc[0].y = red_op<RED>(acc[0].y, acc[u].y);
      }
      c2[x] = acc[0];
    }
  }
}

template <int RED>
__global__ __launch_bounds__(256) void k_contract_final(const ContractK p, const double *__restrict__ ws,
                                                        double *__restrict__ C) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t out = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; out < p.n_out; out += stride) {
    int64_t oc = 0;
    uint32_t idx = (uint32_t)out;
    for (int k = p.nk - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      oc += (int64_t)(idx - q * p.kdiv[k].d) * p.ksc[k];
      idx = q;
    }
    double acc = ws[out];
    for (int s = 1; s < p.n_split; ++s) acc = red_op<RED>(acc, ws[(uint64_t)s * p.n_out + out]);
    C[oc] = acc;
  }
}

// host: drop card-1 dims, merge dims that are contiguous for every operand
struct Dims {
  int n = 0;
  int64_t card[PGM_MAX_DIMS];
  int64_t s[3][PGM_MAX_DIMS];
};

static void coalesce(Dims &d, int nops) {
  Dims o;
  for (int i = 0; i < d.n; ++i) {
    if (d.card[i] == 1) continue;
    if (o.n > 0) {
      bool ok = true;
      const int j = o.n - 1;
      for (int t = 0; t < nops; ++t)
        if (o.s[t][j] != d.card[i] * d.s[t][i]) ok = false;
      if (ok) {
        o.card[j] *= d.card[i];
        for (int t = 0; t < nops; ++t) o.s[t][j] = d.s[t][i];
        continue;
      }
    }
    o.card[o.n] = d.card[i];
    for (int t = 0; t < nops; ++t) o.s[t][o.n] = d.s[t][i];
    ++o.n;
  }
  d = o;
}

static constexpr bool g_no_rows2 = false;  // (r01's 8-B-only row paths: 0.54-0.70x the 16-B rate)

static const uint64_t kTargetThreads = 256ull * 2048;  // 256 CUs x 32 waves x 64 lanes

struct ContractLaunch {
  ContractK k;
  dim3 grid;
  uint64_t ws_doubles;
  bool empty;
};

static int plan_contract(const pgm_contract_desc *d, ContractLaunch &L) {
  if (!d) return fail(PGM_EINVAL, "contract: null descriptor");
  if (d->n_keep < 0 || d->n_keep > PGM_MAX_DIMS || d->n_red < 0 || d->n_red > PGM_MAX_DIMS)
    return fail(PGM_EINVAL, "contract: n_keep/n_red out of range (%d, %d)", d->n_keep, d->n_red);
  if (d->combine < 0 || d->combine > 4 || d->reduce < 0 || d->reduce > 2)
    return fail(PGM_EINVAL, "contract: bad combine/reduce (%d, %d)", d->combine, d->reduce);
  if (d->reduce == PGM_RED_NONE && d->n_red > 0)
    return fail(PGM_EINVAL, "contract: reduction dims given with PGM_RED_NONE");
  Dims kd, rd;
  kd.n = d->n_keep;
  uint64_t n_out = 1, n_red = 1;
  for (int i = 0; i < d->n_keep; ++i) {
    if (d->keep_card[i] <= 0) return fail(PGM_EINVAL, "contract: keep_card[%d] = %lld", i, (long long)d->keep_card[i]);
    kd.card[i] = d->keep_card[i];
    kd.s[0][i] = d->keep_sa[i];
    kd.s[1][i] = d->keep_sb[i];
    kd.s[2][i] = d->keep_sc[i];
    n_out *= (uint64_t)d->keep_card[i];
  }
  rd.n = d->n_red;
  for (int i = 0; i < d->n_red; ++i) {
    if (d->red_card[i] <= 0) return fail(PGM_EINVAL, "contract: red_card[%d] = %lld", i, (long long)d->red_card[i]);
    rd.card[i] = d->red_card[i];
    rd.s[0][i] = d->red_sa[i];
    rd.s[1][i] = d->red_sb[i];
    n_red *= (uint64_t)d->red_card[i];
  }
  if (n_out >= (1ull << 31) || n_red >= (1ull << 31))
    return fail(PGM_EINVAL, "contract: index space too large (%llu x %llu; limit 2^31 each)",
                (unsigned long long)n_out, (unsigned long long)n_red);
  coalesce(kd, 3);
  coalesce(rd, 2);
  // few outputs (flat mode) and one long reduction run: cut the run into (outer x chunk) so the
  // split-K below has reduction-outer indices to distribute (a batched dot product over a packed
  // operand pair would otherwise leave 64 lanes per output walking the whole run)
  if (d->reduce != PGM_RED_NONE && rd.n > 0 && rd.n < KMAX && kd.n <= KMAX && n_out <= 4096 &&
      !(kd.n > 0 && kd.card[kd.n - 1] >= 64)) {
    const int64_t ri = rd.card[rd.n - 1];
    if (ri >= 8192 && n_red / (uint64_t)ri < 256) {
      for (int64_t c = 4096; c >= 256; c >>= 1) {
        if (ri % c) continue;
        const int last = rd.n - 1;
        rd.card[rd.n] = c;
        rd.s[0][rd.n] = rd.s[0][last];
        rd.s[1][rd.n] = rd.s[1][last];
        rd.card[last] = ri / c;
        rd.s[0][last] *= c;
        rd.s[1][last] *= c;
        ++rd.n;
        break;
      }
    }
  }
  if (kd.n > KMAX || rd.n > KMAX)
    return fail(PGM_EINVAL, "contract: %d keep / %d reduce dims after coalescing (limit %d)", kd.n, rd.n, KMAX);
  ContractK &k = L.k;
  memset(&k, 0, sizeof k);
  k.nk = kd.n;
  k.nr = rd.n;
  for (int i = 0; i < kd.n; ++i) {
    k.kdiv[i] = make_fdiv((uint32_t)kd.card[i]);
    k.ksa[i] = kd.s[0][i];
    k.ksb[i] = kd.s[1][i];
    k.ksc[i] = kd.s[2][i];
  }
  for (int i = 0; i < rd.n; ++i) {
    k.rdiv[i] = make_fdiv((uint32_t)rd.card[i]);
    k.rsa[i] = rd.s[0][i];
    k.rsb[i] = rd.s[1][i];
  }
  k.n_out = (uint32_t)n_out;
  k.n_red = (uint32_t)n_red;
  L.empty = (n_out == 0);
  // reduction = outer (decoded, wave-uniform) x innermost (walked by increments)
  if (rd.n > 0) {
    k.ri_card = (uint32_t)rd.card[rd.n - 1];
    k.ri_sa = rd.s[0][rd.n - 1];
    k.ri_sb = rd.s[1][rd.n - 1];
  } else {
    k.ri_card = 1;
    k.ri_sa = k.ri_sb = 0;
  }
  k.n_ro = (uint32_t)(n_red / k.ri_card);
  const bool has_red = d->reduce != PGM_RED_NONE && n_red > 1;
  const uint64_t NX = kd.n > 0 ? (uint64_t)kd.card[kd.n - 1] : 1;
  // row mode when the innermost output dim fills waves and no lane-parallel reduction is needed
  const bool red_contig = rd.n > 0 && rd.s[0][rd.n - 1] == 1;
  k.row_mode = (kd.n > 0 && NX >= 64 && !(has_red && red_contig && NX < 256 && n_out < kTargetThreads)) ? 1 : 0;
  int g_log2 = 0;
  uint32_t n_split = 1;
  if (k.row_mode) {
    const uint64_t n_outer = n_out / NX;
    const uint64_t xchunks = (NX + 255) / 256;
    const uint64_t target_blocks = 2048;
    uint64_t gy = std::min<uint64_t>(n_outer, 65535);
    uint64_t gx = std::min<uint64_t>(xchunks, std::max<uint64_t>(1, target_blocks / gy));
    k.ri_chunk = k.ri_card;
    k.ri_nb = 1;
    if (has_red && gx * gy < target_blocks / 2) {
      // few outputs and a long reduction: split it (virtual outer index = (ro, chunk of the inner dim))
      const uint64_t want = (target_blocks / 2 + gx * gy - 1) / (gx * gy);
      if (k.n_ro < want && k.ri_card >= 64) {
        const uint64_t nb = std::min<uint64_t>((want + k.n_ro - 1) / k.n_ro, k.ri_card / 16);
        k.ri_nb = (uint32_t)std::max<uint64_t>(nb, 1);
        k.ri_chunk = (uint32_t)((k.ri_card + k.ri_nb - 1) / k.ri_nb);
        k.ri_nb = (k.ri_card + k.ri_chunk - 1) / k.ri_chunk;
      }
      n_split = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(want, (uint64_t)k.n_ro * k.ri_nb), 256);
    }
    k.n_v = k.n_ro * k.ri_nb;
    L.grid = dim3((unsigned)gx, (unsigned)gy, n_split);
  } else {
    if (has_red) {
      while (g_log2 < 6 && (n_out << g_log2) < kTargetThreads && (1ull << (g_log2 + 1)) <= k.ri_card) ++g_log2;
      const uint64_t par = n_out << g_log2;
      if (par < kTargetThreads / 4 && k.n_ro > 1) {
        uint64_t want = (kTargetThreads / 4 + par - 1) / par;
        n_split = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(want, k.n_ro), 1024);
      }
    }
    const uint64_t threads = n_out << g_log2;
    uint64_t blocks = (threads + 255) / 256;
    blocks = std::min<uint64_t>(std::max<uint64_t>(blocks, 1), 65535);
    L.grid = dim3((unsigned)blocks, n_split, 1);
  }
  k.g_log2 = g_log2;
  k.n_split = (int32_t)n_split;
  k.red_chunk = k.row_mode ? (uint32_t)((k.n_v + n_split - 1) / n_split) : (uint32_t)((k.n_ro + n_split - 1) / n_split);
  L.ws_doubles = n_split > 1 ? (uint64_t)n_split * n_out : 0;
  return PGM_OK;
}

// two-rows-per-lane eligibility of a row-mode COPY contraction (A read, C written)
static bool rows2_ok(const ContractK &k, const double *A, const double *C) {
  if (g_no_rows2 || !k.row_mode || k.nk < 1) return false;
  const int kx = k.nk - 1;
  if (k.kdiv[kx].d % 2 || k.ksa[kx] != 1 || k.ksc[kx] != 1) return false;
  if (((uintptr_t)A & 15) || ((uintptr_t)C & 15)) return false;
  for (int i = 0; i < kx; ++i)
    if (k.ksa[i] % 2 || k.ksc[i] % 2) return false;
  for (int i = 0; i < k.nr; ++i)
    if (k.rsa[i] % 2) return false;
  return k.nr == 0 || k.ri_sa % 2 == 0;
}

template <int CMB, int RED>
static void launch_contract_t(const ContractLaunch &L, const double *A, const double *B, double *C, double *ws,
                              hipStream_t s) {
  if (L.k.row_mode && RED != PGM_RED_NONE && L.k.n_split == 1 && L.k.ri_nb == 1 && L.k.n_red <= RTAB_MAX) {
    if (CMB == PGM_COMBINE_COPY && rows2_ok(L.k, A, C)) {
      dim3 g = L.grid;
      g.x = (unsigned)std::max<uint64_t>(1, (g.x + 1) / 2);
      hipLaunchKernelGGL((k_contract_rows_tab2<RED>), g, dim3(256), 0, s, L.k, A, C);
    } else {
      hipLaunchKernelGGL((k_contract_rows_tab<CMB, RED>), L.grid, dim3(256), 0, s, L.k, A, B, C);
    }
  }
  else if (L.k.row_mode)
    hipLaunchKernelGGL((k_contract_rows<CMB, RED>), L.grid, dim3(256), 0, s, L.k, A, B, C, ws);
  else
    hipLaunchKernelGGL((k_contract<CMB, RED>), L.grid, dim3(256), 0, s, L.k, A, B, C, ws);
  if (L.k.n_split > 1) {
    uint64_t blocks = std::min<uint64_t>((L.k.n_out + 255) / 256, 65535);
    hipLaunchKernelGGL((k_contract_final<RED>), dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, s,
                       L.k, (const double *)ws, C);
  }
}

template <int CMB>
static void launch_contract_c(int red, const ContractLaunch &L, const double *A, const double *B, double *C,
                              double *ws, hipStream_t s) {
  switch (red) {
    case PGM_RED_NONE: launch_contract_t<CMB, PGM_RED_NONE>(L, A, B, C, ws, s); break;
    case PGM_RED_SUM: launch_contract_t<CMB, PGM_RED_SUM>(L, A, B, C, ws, s); break;
    default: launch_contract_t<CMB, PGM_RED_MAX>(L, A, B, C, ws, s); break;
  }
}

// ----------------------------------------------------------------------------- n-ary product
#define PMAX PGM_PRODN_MAX_OPS
struct ProdNK {
  int32_t n_ops, nk;
  int32_t kind[PMAX];
  uint32_t n_out, row_mode;
  uint32_t pairs, _pad;  // batched jobs: two innermost elements per lane with 16-B accesses
  FDiv kdiv[KMAX];
  int64_t ksc[KMAX];
  int64_t ks[PMAX][KMAX];
  const double *ops[PMAX];
};

// all operand values first (unused slots alias operand 0 with stride 0, so every load is valid and
// no load sits behind a branch), then the product with the per-operand kinds (uniform branches)
template <int NOPS>
__device__ __forceinline__ double prodn_combine(const ProdNK &p, const double (&v)[NOPS]) {
  double prod = 1.0;
#pragma unroll
  for (int i = 0; i < NOPS; ++i) {
    if (i < p.n_ops) {
      if (p.kind[i] == PGM_PRODN_MUL) {
        prod *= v[i];
      } else if (p.kind[i] == PGM_PRODN_RATIO && i + 1 < NOPS) {
        const double r = v[i] / v[i + 1];
        prod *= (r != r) ? 0.0 : r;
      }
    }
  }
  return prod;
}

// flat mode: every output decoded on its own (grid-stride over tid / nthreads); also the body of a
// batched product_n job (k_batch)
template <int NOPS>
__device__ __forceinline__ void prodn_flat(const ProdNK &p, double *__restrict__ C, uint64_t tid, uint64_t nthreads) {
  for (uint64_t out = tid; out < p.n_out; out += nthreads) {
    uint32_t idx = (uint32_t)out;
    int64_t off[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) off[i] = 0;
    int64_t oc = 0;
    for (int k = p.nk - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
#pragma unroll
      for (int i = 0; i < NOPS; ++i) off[i] += (int64_t)dg * p.ks[i][k];
      oc += (int64_t)dg * p.ksc[k];
      idx = q;
    }
    double v[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) v[i] = p.ops[i][off[i]];
    C[oc] = prodn_combine<NOPS>(p, v);
  }
}

// flat mode over element PAIRS along the innermost dim (host-checked: even innermost card, output
// innermost stride 1, every operand's innermost stride 0 or 1, all other strides of 16-B accessed
// arrays even, bases 16-B aligned): 16-B loads/stores for batched jobs
template <int NOPS>
__device__ __forceinline__ void prodn_flat2(const ProdNK &p, double *__restrict__ C, uint64_t tid, uint64_t nthreads) {
  const int kx = p.nk - 1;
  bool vec[NOPS];
#pragma unroll
  for (int i = 0; i < NOPS; ++i) vec[i] = p.ks[i][kx] != 0;
  const uint32_t n_pairs = p.n_out >> 1;
  for (uint64_t q = tid; q < n_pairs; q += nthreads) {
    uint32_t idx = (uint32_t)q << 1;
    int64_t off[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) off[i] = 0;
    int64_t oc = 0;
    for (int k = kx; k >= 0; --k) {
      const uint32_t qq = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - qq * p.kdiv[k].d;
#pragma unroll
      for (int i = 0; i < NOPS; ++i) off[i] += (int64_t)dg * p.ks[i][k];
      oc += (int64_t)dg * p.ksc[k];
      idx = qq;
    }
    double lo[NOPS], hi[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) {
      if (vec[i]) {
        const double2 w = *(const double2 *)(p.ops[i] + off[i]);
        lo[i] = w.x;
        hi[i] = w.y;
      } else {
        lo[i] = hi[i] = p.ops[i][off[i]];
      }
    }
    *(double2 *)(C + oc) = make_double2(prodn_combine<NOPS>(p, lo), prodn_combine<NOPS>(p, hi));
  }
}

template <int NOPS>
__global__ __launch_bounds__(256) void k_productn(const ProdNK p, double *__restrict__ C) {
  if (p.row_mode) {
    constexpr int U = NOPS <= 4 ? 4 : 2;  // rows in flight per thread
    const int kx = p.nk - 1;
    const uint32_t NX = p.kdiv[kx].d;
    const uint32_t n_outer = p.n_out / NX;
    const uint32_t xstep = gridDim.x * blockDim.x;
    int64_t sx[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) sx[i] = p.ks[i][kx];
    const int64_t scx = p.ksc[kx];
    for (uint32_t o = blockIdx.y; o < n_outer; o += gridDim.y) {
      // outer decode once per block and outer index (wave-uniform), reused for all rows
      int64_t off[NOPS];
#pragma unroll
      for (int i = 0; i < NOPS; ++i) off[i] = 0;
      int64_t oc = 0;
      uint32_t idx = o;
      for (int k = kx - 1; k >= 0; --k) {
        const uint32_t q = fdiv(idx, p.kdiv[k]);
        const uint32_t dg = idx - q * p.kdiv[k].d;
#pragma unroll
        for (int i = 0; i < NOPS; ++i) off[i] += (int64_t)dg * p.ks[i][k];
        oc += (int64_t)dg * p.ksc[k];
        idx = q;
      }
      const double *op[NOPS];
#pragma unroll
      for (int i = 0; i < NOPS; ++i) op[i] = p.ops[i] + off[i];
      for (uint32_t x0 = blockIdx.x * blockDim.x + threadIdx.x; x0 < NX; x0 += U * xstep) {
        double v[U][NOPS];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t x = x0 + u * xstep;
          const int64_t xc = x < NX ? x : NX - 1;
#pragma unroll
          for (int i = 0; i < NOPS; ++i) v[u][i] = op[i][xc * sx[i]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t x = x0 + u * xstep;
          if (x < NX) C[oc + (int64_t)x * scx] = prodn_combine<NOPS>(p, v[u]);
        }
      }
    }
    return;
  }
  prodn_flat<NOPS>(p, C, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, (uint64_t)gridDim.x * blockDim.x);
}

// Row mode, two rows per lane (16-B loads/stores; the 8-B form runs at 0.54-0.70x the 16-B rate on
// gfx950).  Host-checked: even row count, output row stride 1, every operand's row stride 0 (broadcast,
// one scalar per outer index) or 1, every base 16-B aligned (all outer strides even).
template <int NOPS>
__global__ __launch_bounds__(256) void k_productn_rows2(const ProdNK p, double *__restrict__ C) {
  constexpr int U = NOPS <= 4 ? 2 : 1;  // row pairs in flight per thread
  const int kx = p.nk - 1;
  const uint32_t NP = p.kdiv[kx].d >> 1;
  const uint32_t n_outer = p.n_out / p.kdiv[kx].d;
  const uint32_t xstep = gridDim.x * blockDim.x;
  bool vec[NOPS];
#pragma unroll
  for (int i = 0; i < NOPS; ++i) vec[i] = p.ks[i][kx] != 0;
  for (uint32_t o = blockIdx.y; o < n_outer; o += gridDim.y) {
    int64_t off[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) off[i] = 0;
    int64_t oc = 0;
    uint32_t idx = o;
    for (int k = kx - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
#pragma unroll
      for (int i = 0; i < NOPS; ++i) off[i] += (int64_t)dg * p.ks[i][k];
      oc += (int64_t)dg * p.ksc[k];
      idx = q;
    }
    const double *op[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) op[i] = p.ops[i] + off[i];
    double2 *c2 = (double2 *)(C + oc);
    for (uint32_t x0 = blockIdx.x * blockDim.x + threadIdx.x; x0 < NP; x0 += U * xstep) {
      double2 v[U][NOPS];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t x = x0 + u * xstep;
        const uint32_t xc = x < NP ? x : NP - 1;
#pragma unroll
        for (int i = 0; i < NOPS; ++i) {
          if (vec[i]) {
            v[u][i] = ((const double2 *)op[i])[xc];
          } else {
            const double b = op[i][0];
            v[u][i] = make_double2(b, b);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t x = x0 + u * xstep;
        double lo[NOPS], hi[NOPS];
#pragma unroll
        for (int i = 0; i < NOPS; ++i) {
          lo[i] = v[u][i].x;
          hi[i] = v[u][i].y;
        }
        if (x < NP) c2[x] = make_double2(prodn_combine<NOPS>(p, lo), prodn_combine<NOPS>(p, hi));
      }
    }
  }
}

// ----------------------------------------------------------------------------- n-ary product + marginal
// C = prod_i X_i (as pgm_product_n) and, in the same pass, M = SUM/MAX of C over the keep dims M
// does not have: a batched-BP clique belief written together with its separator message (collect)
// or updated in place together with the marginal onto its children's separator (distribute), so
// the belief is not read again.  Rows (the last keep dim) two per lane with 16-B accesses as in
// k_productn_rows2.  A block owns one kept outer index (separator state); the reduction (the
// clique's other states) is walked from an LDS offset table with the next entry's operands in
// flight while the current product is stored and accumulated.
#define RMAX_MARG 512

template <int NOPS>
__device__ __forceinline__ double prodm_combine(const ProdMK &p, const double (&v)[NOPS]) {
  double prod = 1.0;
#pragma unroll
  for (int i = 0; i < NOPS; ++i) {
    if (i < p.n_ops) {
      if (p.kind[i] == PGM_PRODN_MUL) {
        prod *= v[i];
      } else if (p.kind[i] == PGM_PRODN_RATIO && i + 1 < NOPS) {
        const double r = v[i] / v[i + 1];
        prod *= (r != r) ? 0.0 : r;
      }
    }
  }
  return prod;
}


// j-outer form: for each reduced entry j the block sweeps its x range (XI row pairs per lane,
// x = x0 + i*256), so every store instruction of the block lands in one contiguous run of the
// belief and XI x NOPS 16-B operand loads are in flight per lane; the marginal stays in XI
// register accumulators until the last j.  Block = (kept outer index, 256*XI row pairs).
template <int NOPS, int RED, int XI>
__global__ __launch_bounds__(256) void k_productn_marg_jx(const ProdMK p, double *C, double *__restrict__ M) {
  __shared__ int64_t tc[RMAX_MARG];
  __shared__ int64_t to[NOPS][RMAX_MARG];
  const uint32_t NR = p.n_red;
  for (uint32_t j = threadIdx.x; j < NR; j += blockDim.x) {
    uint32_t idx = j;
    int64_t oc = 0, oo[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) oo[i] = 0;
    for (int k = p.nr - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.rdiv[k]);
      const uint32_t dg = idx - q * p.rdiv[k].d;
      oc += (int64_t)dg * p.rsc[k];
#pragma unroll
      for (int i = 0; i < NOPS; ++i) oo[i] += (int64_t)dg * p.rs[i][k];
      idx = q;
    }
    tc[j] = oc;
#pragma unroll
    for (int i = 0; i < NOPS; ++i) to[i][j] = oo[i];
  }
  __syncthreads();
  const int kx = p.nk - 1;
  for (uint32_t o = blockIdx.y; o < p.n_outer; o += gridDim.y) {
    int64_t oc = 0, om = 0, off[NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) off[i] = 0;
    uint32_t idx = o;
    for (int k = kx - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
      oc += (int64_t)dg * p.ksc[k];
      om += (int64_t)dg * p.ksm[k];
#pragma unroll
      for (int i = 0; i < NOPS; ++i) off[i] += (int64_t)dg * p.ks[i][k];
      idx = q;
    }
    const uint32_t x0 = blockIdx.x * (256u * XI) + threadIdx.x;
    uint32_t xs[XI];
#pragma unroll
    for (int u = 0; u < XI; ++u) {
      const uint32_t x = x0 + 256u * u;
      xs[u] = x < p.NP ? x : p.NP - 1;
    }
    double2 acc[XI];
#pragma unroll
    for (int u = 0; u < XI; ++u) acc[u] = make_double2(red_init<RED>(), red_init<RED>());
    // operands that do not vary over the reduced entries: loaded once per outer index
    double2 h[XI][NOPS];
#pragma unroll
    for (int i = 0; i < NOPS; ++i) {
      if (p.jvar[i]) continue;
      const double *b = p.ops[i] + off[i];
      if (p.vec[i]) {
#pragma unroll
        for (int u = 0; u < XI; ++u) h[u][i] = ((const double2 *)b)[xs[u]];
      } else {
        const double sv = b[0];
#pragma unroll
        for (int u = 0; u < XI; ++u) h[u][i] = make_double2(sv, sv);
      }
    }
    for (uint32_t j = 0; j < NR; ++j) {
      double2 v[XI][NOPS];
#pragma unroll
      for (int i = 0; i < NOPS; ++i) {
        const double *b = p.ops[i] + off[i] + to[i][j];
        if (!p.jvar[i]) {
#pragma unroll
          for (int u = 0; u < XI; ++u) v[u][i] = h[u][i];
        } else if (p.vec[i]) {
#pragma unroll
          for (int u = 0; u < XI; ++u) v[u][i] = ((const double2 *)b)[xs[u]];
        } else {
          const double sv = b[0];
#pragma unroll
          for (int u = 0; u < XI; ++u) v[u][i] = make_double2(sv, sv);
        }
      }
      double2 *cj = (double2 *)(C + oc + tc[j]);
#pragma unroll
      for (int u = 0; u < XI; ++u) {
        double lo[NOPS], hi[NOPS];
#pragma unroll
        for (int i = 0; i < NOPS; ++i) {
          lo[i] = v[u][i].x;
          hi[i] = v[u][i].y;
        }
        const double2 pr = make_double2(prodm_combine<NOPS>(p, lo), prodm_combine<NOPS>(p, hi));
        if (C && x0 + 256u * u < p.NP) cj[x0 + 256u * u] = pr;  // C == nullptr: the marginal only
        acc[u].x = red_op<RED>(acc[u].x, pr.x);
        acc[u].y = red_op<RED>(acc[u].y, pr.y);
      }
    }
#pragma unroll
    for (int u = 0; u < XI; ++u) {
      if (p.mdiv >= 0) {  // the marginal over the operand that does not vary over the summed entries
        double2 dv = h[u][0];
#pragma unroll
        for (int i = 1; i < NOPS; ++i)
          if (i == p.mdiv) dv = h[u][i];
        const double rx = acc[u].x / dv.x, ry = acc[u].y / dv.y;
        acc[u] = make_double2(rx != rx ? 0.0 : rx, ry != ry ? 0.0 : ry);
      }
      if (x0 + 256u * u < p.NP) ((double2 *)(M + om))[x0 + 256u * u] = acc[u];
    }
  }
}

// 1 = the fused kernel applies (k filled), 0 = it does not (use product_n + contract), < 0 error
int pgmi_plan_product_marg(const pgm_productn_desc *d, const double *const *ops, const double *C,
                             const int64_t *marg_s, const double *M, ProdMK &k, dim3 &grid) {
  if (!d || !ops || !marg_s || !M) return fail(PGM_EINVAL, "product_n_marginal: null argument");
  if (d->n_ops < 1 || d->n_ops > PMAX || d->n_keep < 1 || d->n_keep > PGM_MAX_DIMS)
    return fail(PGM_EINVAL, "product_n_marginal: n_ops %d / n_keep %d out of range", d->n_ops, d->n_keep);
  if (g_no_rows2 || d->n_ops > MOPS || d->n_keep < 2) return 0;
  memset(&k, 0, sizeof k);
  const int last = d->n_keep - 1;
  const int64_t NX = d->keep_card[last];
  if (NX < 64 || NX % 2 || d->keep_sc[last] != 1 || marg_s[last] != 1) return 0;
  if (((uintptr_t)C & 15) || ((uintptr_t)M & 15)) return 0;
  k.n_ops = d->n_ops;
  k.mdiv = -1;
  for (int t = 0; t < MOPS; ++t) {
    const bool real = t < d->n_ops;
    k.ops[t] = real ? ops[t] : ops[0];
    k.kind[t] = real ? d->op_kind[t] : PGM_PRODN_MUL;
    if (real && (!ops[t] || d->op_kind[t] < 0 || d->op_kind[t] > PGM_PRODN_MDIV))
      return fail(PGM_EINVAL, "product_n_marginal: operand %d", t);
    if (real && d->op_kind[t] == PGM_PRODN_MDIV) {  // a factor of the product, and the marginal's divisor
      if (k.mdiv >= 0) return fail(PGM_EINVAL, "product_n_marginal: more than one PGM_PRODN_MDIV operand");
      k.mdiv = t;
      k.kind[t] = PGM_PRODN_MUL;
    }
    const int64_t sx = real ? d->keep_s[t][last] : 0;
    if (sx != 0 && sx != 1) return 0;
    if (sx == 1 && ((uintptr_t)ops[t] & 15)) return 0;
    k.vec[t] = sx == 1;
  }
  uint64_t n_outer = 1, n_red = 1;
  for (int i = 0; i < last; ++i) {
    const int64_t c = d->keep_card[i];
    if (c <= 0) return fail(PGM_EINVAL, "product_n_marginal: keep_card[%d] <= 0", i);
    if (c == 1) continue;
    const bool kept = marg_s[i] != 0;
    if (d->keep_sc[i] % 2 || (kept && marg_s[i] % 2)) return 0;
    for (int t = 0; t < d->n_ops; ++t)
      if (k.vec[t] && d->keep_s[t][i] % 2) return 0;
    if (kept) {
      if (k.nk >= KMAX - 1) return 0;
      k.kdiv[k.nk] = make_fdiv((uint32_t)c);
      k.ksc[k.nk] = d->keep_sc[i];
      k.ksm[k.nk] = marg_s[i];
      for (int t = 0; t < d->n_ops; ++t) k.ks[t][k.nk] = d->keep_s[t][i];
      ++k.nk;
      n_outer *= (uint64_t)c;
    } else {
      if (k.nr >= KMAX) return 0;
      k.rdiv[k.nr] = make_fdiv((uint32_t)c);
      k.rsc[k.nr] = d->keep_sc[i];
      for (int t = 0; t < d->n_ops; ++t) k.rs[t][k.nr] = d->keep_s[t][i];
      ++k.nr;
      n_red *= (uint64_t)c;
    }
  }
  if (n_red > RMAX_MARG || n_outer >= (1ull << 31)) return 0;
  // kept-dim order of the block schedule: blocks are dispatched with the LAST kept dim fastest.  A
  // row-dim operand that lacks a kept dim is read again by every block along that dim, so the dims
  // lacked by the largest such operands go innermost: the blocks sharing an operand slice then run
  // back to back and find it in L2 (pathfinder's root: 129-258 MB separator aggregates broadcast over
  // its other variables).
  if (k.nk > 1) {
    double score[KMAX];
    for (int i = 0; i < k.nk; ++i) {
      score[i] = 0.0;
      for (int t = 0; t < d->n_ops; ++t) {
        if (!k.vec[t] || k.ks[t][i] != 0) continue;
        double size = 1.0;  // the operand's elements per row
        for (int q = 0; q < k.nk; ++q)
          if (k.ks[t][q] != 0) size *= (double)k.kdiv[q].d;
        for (int r = 0; r < k.nr; ++r)
          if (k.rs[t][r] != 0) size *= (double)k.rdiv[r].d;
        score[i] += size;
      }
    }
    int ord[KMAX];
    for (int i = 0; i < k.nk; ++i) ord[i] = i;
    std::stable_sort(ord, ord + k.nk, [&](int a, int b) { return score[a] < score[b]; });
    ProdMK k2 = k;
    for (int i = 0; i < k.nk; ++i) {
      const int o = ord[i];
      k2.kdiv[i] = k.kdiv[o];
      k2.ksc[i] = k.ksc[o];
      k2.ksm[i] = k.ksm[o];
      for (int t = 0; t < MOPS; ++t) k2.ks[t][i] = k.ks[t][o];
    }
    k = k2;
  }
  for (int t = 0; t < MOPS; ++t) {
    k.jvar[t] = 0;
    for (int r = 0; t < d->n_ops && r < k.nr; ++r) k.jvar[t] |= k.rs[t][r] != 0;
  }
  if (k.mdiv >= 0 && k.jvar[k.mdiv]) return 0;  // the divisor varies over the summed entries: not this kernel
  k.kdiv[k.nk] = make_fdiv((uint32_t)NX);  // the row dim, last
  ++k.nk;
  k.n_red = (int32_t)n_red;
  k.n_outer = (uint32_t)n_outer;
  k.NP = (uint32_t)(NX / 2);
  const uint64_t xb = (k.NP + 255) / 256;
  const uint64_t gy = std::min<uint64_t>(n_outer, 65535);
  // target block count
  static constexpr uint64_t target = 2048;
  const uint64_t gx = std::min<uint64_t>(xb, std::max<uint64_t>(1, target / gy));
  // too few blocks to fill the chip: the two-kernel path (product_n + contract) was faster for a lone
  // launch below 512 blocks, but inside a levelled schedule it costs a second dependency level.  C4
  // (r03ae, two runs each): floor 512 / 256 / 128 / 64 -> 0.87-0.88 / 0.92 / 0.95 / 0.85 M
  // calibrations/s at 1,000 rows, 1.20-1.21 / 1.25 / 1.24-1.25 / 1.24-1.25 M at 4,000.  Once small steps are specialised and merged into their level's launch
  // (PGM_PM_JIT_MIN 2^14, r03ag) a small fused pass costs no launch of its own: floor 128 -> 32 gives
  // 1.03 -> 1.09 M at 1,000 rows, 4,000 rows unchanged at 1.29-1.30 M (r03ah); 32 / 8 / 2 -> 1.08 / 1.08
  // / 1.09-1.10 M (r03ai): no floor by default.
  static constexpr uint64_t min_blocks = 1;
  // (also accepting short reductions on 16+ blocks was slower at 1,000 rows, 0.95 -> 0.87 M: each such
  // pass is a launch of its own, where the two-kernel path's jobs join the level's batch launch; r03af)
  if (gx * gy < min_blocks) return 0;
  grid = dim3((unsigned)gx, (unsigned)gy, 1);
  return 1;
}

// ----------------------------------------------------------------------------- gather
// GatherK (a planned per-row evidence gather): pgm_internal.h

__device__ __forceinline__ void gather_body(const GatherK &p, const double *__restrict__ A,
                                            const uint8_t *__restrict__ codes, double *__restrict__ C,
                                            int32_t *__restrict__ err, uint64_t tid, uint64_t nthreads) {
  for (uint64_t out = tid; out < p.n_out; out += nthreads) {
    int64_t oa = 0, oc = 0, row = 0;
    uint32_t idx = (uint32_t)out;
    for (int k = p.nk - 1; k >= 0; --k) {
      const uint32_t q = fdiv(idx, p.kdiv[k]);
      const uint32_t dg = idx - q * p.kdiv[k].d;
      oa += (int64_t)dg * p.ksa[k];
      oc += (int64_t)dg * p.ksc[k];
      if (k == p.batch_dim) row = dg;
      idx = q;
    }
    for (int j = 0; j < p.n_ev; ++j) {
      uint32_t c = codes[p.ev_col[j] * p.ld + p.row0 + row];
      if (c >= (uint32_t)p.ev_card[j]) {
        if (err) atomicOr(err, 1);
        c = 0;
      }
      oa += (int64_t)c * p.ev_stride[j];
    }
    C[oc] = A[oa];
  }
}

__global__ __launch_bounds__(256) void k_gather(const GatherK p, const double *__restrict__ A,
                                                const uint8_t *__restrict__ codes, double *__restrict__ C,
                                                int32_t *__restrict__ err) {
  gather_body(p, A, codes, C, err, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, (uint64_t)gridDim.x * blockDim.x);
}

// findings as 0/1 indicators (BP): out[k, r] = (codes[r] == k), 1 for a missing code (PGM_EV_MISSING)
__device__ __forceinline__ void indicator_body(const uint8_t *__restrict__ codes, int64_t n_rows, int64_t card,
                                               double *__restrict__ out, int64_t s_state, int64_t s_row,
                                               int32_t *__restrict__ err, int64_t tid, int64_t stride) {
  const int64_t n = n_rows * card;
  for (int64_t i = tid; i < n; i += stride) {
    const int64_t r = i % n_rows, k = i / n_rows;
    const uint32_t c = codes[r];
    double v;
    if (c == PGM_EV_MISSING)
      v = 1.0;
    else {
      if (c >= (uint64_t)card && err) atomicOr(err, 1);
      v = (c == (uint64_t)k) ? 1.0 : 0.0;
    }
    out[k * s_state + r * s_row] = v;
  }
}

// ----------------------------------------------------------------------------- batched small jobs
// Many independent small contractions / evidence gathers in ONE launch: workgroup -> job through a
// block map, each job runs the flat-mode contraction (or the gather) over its own blocks.  One
// level of a compiled contraction path (all steps whose inputs are ready) is one launch instead
// of one launch per step.
struct BatchJob {
  int32_t kind, cmb, red, _pad;  // kind 0: contraction, 1: gather, 2: n-ary product, 3: findings indicator
  int64_t ind_rows, ind_card, ind_s_state, ind_s_row;
  uint32_t block0, nblocks;
  const double *A, *B;
  double *C;
  const uint8_t *codes;
  int32_t *err;
  ContractK c;
  GatherK g;
  ProdNK pn;
};

template <int CMB>
__device__ __forceinline__ void batch_contract_c(const BatchJob &J, uint64_t tid, uint64_t n) {
  if (J.c.row_mode == 2) {  // output pairs, 16-B accesses
    switch (J.red) {
      case PGM_RED_NONE: contract_flat2<CMB, PGM_RED_NONE>(J.c, J.A, J.B, J.C, tid, n); break;
      case PGM_RED_SUM: contract_flat2<CMB, PGM_RED_SUM>(J.c, J.A, J.B, J.C, tid, n); break;
      default: contract_flat2<CMB, PGM_RED_MAX>(J.c, J.A, J.B, J.C, tid, n); break;
    }
    return;
  }
  switch (J.red) {
    case PGM_RED_NONE: contract_flat<CMB, PGM_RED_NONE>(J.c, J.A, J.B, J.C, nullptr, tid, n, 0); break;
    case PGM_RED_SUM: contract_flat<CMB, PGM_RED_SUM>(J.c, J.A, J.B, J.C, nullptr, tid, n, 0); break;
    default: contract_flat<CMB, PGM_RED_MAX>(J.c, J.A, J.B, J.C, nullptr, tid, n, 0); break;
  }
}

__device__ __forceinline__ void batch_block(const BatchJob *__restrict__ jobs, const uint32_t *__restrict__ block_job,
                                            uint32_t b);

__global__ __launch_bounds__(256) void k_batch(const BatchJob *__restrict__ jobs,
                                               const uint32_t *__restrict__ block_job) {
  batch_block(jobs, block_job, blockIdx.x);
}

// A single-workgroup levelled batch of contractions only (the tail of a contraction path, C1 / C2): the
// job descriptors (contraction part only), the block map and the level table are copied into LDS once at
// the start — every load of them independent, issued together — so each level's blocks read their
// descriptor from LDS instead of a block-map load followed by a dependent descriptor load from memory
// (two round trips per level).  Same per-job code as k_batch_c, so the same results bit for bit.
struct alignas(16) ChainJob {
  int32_t cmb, red;
  uint32_t block0, nblocks;
  const double *A, *B;
  double *C;
  ContractK c;
};

template <int CMB>
__device__ __forceinline__ void chain_contract_c(const ChainJob &J, uint64_t tid, uint64_t n) {
  if (J.c.row_mode == 2) {
    switch (J.red) {
      case PGM_RED_NONE: contract_flat2<CMB, PGM_RED_NONE>(J.c, J.A, J.B, J.C, tid, n); break;
      case PGM_RED_SUM: contract_flat2<CMB, PGM_RED_SUM>(J.c, J.A, J.B, J.C, tid, n); break;
      default: contract_flat2<CMB, PGM_RED_MAX>(J.c, J.A, J.B, J.C, tid, n); break;
    }
    return;
  }
  switch (J.red) {
    case PGM_RED_NONE: contract_flat<CMB, PGM_RED_NONE>(J.c, J.A, J.B, J.C, nullptr, tid, n, 0); break;
    case PGM_RED_SUM: contract_flat<CMB, PGM_RED_SUM>(J.c, J.A, J.B, J.C, nullptr, tid, n, 0); break;
    default: contract_flat<CMB, PGM_RED_MAX>(J.c, J.A, J.B, J.C, nullptr, tid, n, 0); break;
  }
}

// 1,024 threads = kChainVB virtual 256-thread blocks: a level's blocks run kChainVB at a time (each
// virtual block's 4 waves as one block of k_batch), one workgroup barrier per level.
static constexpr uint32_t kChainVB = 4;

__global__ __launch_bounds__(256 * kChainVB) void k_batch_wg_c(const ChainJob *__restrict__ jobs,
                                                    const uint32_t *__restrict__ block_job,
                                                    const uint32_t *__restrict__ level_off, uint32_t n_levels,
                                                    uint32_t n_jobs, uint32_t n_blocks) {
  extern __shared__ uint4 chain_lds[];
  const uint32_t jq = n_jobs * (uint32_t)(sizeof(ChainJob) / 16);
  const uint4 *src = reinterpret_cast<const uint4 *>(jobs);
  for (uint32_t i = threadIdx.x; i < jq; i += blockDim.x) chain_lds[i] = src[i];  // all loads independent
  uint32_t *lmap = reinterpret_cast<uint32_t *>(chain_lds + jq);
  for (uint32_t i = threadIdx.x; i < n_blocks; i += blockDim.x) lmap[i] = block_job[i];
  uint32_t *llev = lmap + n_blocks;
  for (uint32_t i = threadIdx.x; i <= n_levels; i += blockDim.x) llev[i] = level_off[i];
  __syncthreads();
  const ChainJob *sj = reinterpret_cast<const ChainJob *>(chain_lds);
  const uint32_t vb = threadIdx.x / 256, lt = threadIdx.x % 256;
  for (uint32_t l = 0; l < n_levels; ++l) {
    const uint32_t e = llev[l + 1];
    for (uint32_t b = llev[l] + vb; b < e; b += kChainVB) {
      const ChainJob &J = sj[lmap[b]];
      const uint64_t tid = (uint64_t)(b - J.block0) * 256 + lt;
      const uint64_t n = (uint64_t)J.nblocks * 256;
      switch (J.cmb) {
        case PGM_COMBINE_MUL: chain_contract_c<PGM_COMBINE_MUL>(J, tid, n); break;
        case PGM_COMBINE_ADD: chain_contract_c<PGM_COMBINE_ADD>(J, tid, n); break;
        case PGM_COMBINE_DIV: chain_contract_c<PGM_COMBINE_DIV>(J, tid, n); break;
        case PGM_COMBINE_DIV_RAW: chain_contract_c<PGM_COMBINE_DIV_RAW>(J, tid, n); break;
        default: chain_contract_c<PGM_COMBINE_COPY>(J, tid, n); break;
      }
    }
    __syncthreads();  // the level's outputs are complete before the next level reads them
  }
}

// A batch whose jobs are all contractions with one (combine, reduce) pair — every C2 / C1 path level —
// runs this instead of k_batch: k_batch carries every job kind's code (167 KB of instructions, 123
// VGPRs), this one only the two contraction bodies.  Same per-job code, so bit-identical results
// (r04: C2 0.175 / 0.178 against 0.179 / 0.180 ms with k_batch, profiles/r04k/).
template <int CMB, int RED>
__global__ __launch_bounds__(256) void k_batch_c(const BatchJob *__restrict__ jobs,
                                                 const uint32_t *__restrict__ block_job) {
  const uint32_t b = blockIdx.x;
  const uint32_t j = __builtin_amdgcn_readfirstlane(block_job[b]);
  const BatchJob &J = jobs[j];
  const uint64_t tid = (uint64_t)(b - J.block0) * blockDim.x + threadIdx.x;
  const uint64_t n = (uint64_t)J.nblocks * blockDim.x;
  if (J.c.row_mode == 2)
    contract_flat2<CMB, RED>(J.c, J.A, J.B, J.C, tid, n);
  else
    contract_flat<CMB, RED>(J.c, J.A, J.B, J.C, nullptr, tid, n, 0);
}

// The same for a batch of n-ary products only (C4's levelled BP sweep: the separator-sized products).
__global__ __launch_bounds__(256) void k_batch_p(const BatchJob *__restrict__ jobs,
                                                 const uint32_t *__restrict__ block_job) {
  const uint32_t b = blockIdx.x;
  const uint32_t j = __builtin_amdgcn_readfirstlane(block_job[b]);
  const BatchJob &J = jobs[j];
  const uint64_t tid = (uint64_t)(b - J.block0) * blockDim.x + threadIdx.x;
  const uint64_t n = (uint64_t)J.nblocks * blockDim.x;
  if (J.pn.pairs) {
    if (J.pn.n_ops <= 2) prodn_flat2<2>(J.pn, J.C, tid, n);
    else if (J.pn.n_ops <= 4) prodn_flat2<4>(J.pn, J.C, tid, n);
    else prodn_flat2<PMAX>(J.pn, J.C, tid, n);
    return;
  }
  if (J.pn.n_ops <= 2) prodn_flat<2>(J.pn, J.C, tid, n);
  else if (J.pn.n_ops <= 4) prodn_flat<4>(J.pn, J.C, tid, n);
  else prodn_flat<PMAX>(J.pn, J.C, tid, n);
}

__device__ __forceinline__ void batch_block(const BatchJob *__restrict__ jobs, const uint32_t *__restrict__ block_job,
                                            uint32_t b) {
  const uint32_t j = __builtin_amdgcn_readfirstlane(block_job[b]);
  const BatchJob &J = jobs[j];
  const uint64_t tid = (uint64_t)(b - J.block0) * blockDim.x + threadIdx.x;
  const uint64_t n = (uint64_t)J.nblocks * blockDim.x;
  if (J.kind == 1) {
    gather_body(J.g, J.A, J.codes, J.C, J.err, tid, n);
    return;
  }
  if (J.kind == 3) {
    indicator_body(J.codes, J.ind_rows, J.ind_card, J.C, J.ind_s_state, J.ind_s_row, J.err, (int64_t)tid, (int64_t)n);
    return;
  }
  if (J.kind == 2) {
    if (J.pn.pairs) {
      if (J.pn.n_ops <= 2) prodn_flat2<2>(J.pn, J.C, tid, n);
      else if (J.pn.n_ops <= 4) prodn_flat2<4>(J.pn, J.C, tid, n);
      else prodn_flat2<PMAX>(J.pn, J.C, tid, n);
      return;
    }
    if (J.pn.n_ops <= 2) prodn_flat<2>(J.pn, J.C, tid, n);
    else if (J.pn.n_ops <= 4) prodn_flat<4>(J.pn, J.C, tid, n);
    else prodn_flat<PMAX>(J.pn, J.C, tid, n);
    return;
  }
  switch (J.cmb) {
    case PGM_COMBINE_MUL: batch_contract_c<PGM_COMBINE_MUL>(J, tid, n); break;
    case PGM_COMBINE_ADD: batch_contract_c<PGM_COMBINE_ADD>(J, tid, n); break;
    case PGM_COMBINE_DIV: batch_contract_c<PGM_COMBINE_DIV>(J, tid, n); break;
    case PGM_COMBINE_DIV_RAW: batch_contract_c<PGM_COMBINE_DIV_RAW>(J, tid, n); break;
    default: batch_contract_c<PGM_COMBINE_COPY>(J, tid, n); break;
  }
}

__global__ __launch_bounds__(256) void k_indicator(const uint8_t *__restrict__ codes, int64_t n_rows, int64_t card,
                                                   double *__restrict__ out, int64_t s_state, int64_t s_row,
                                                   int32_t *__restrict__ err) {
  indicator_body(codes, n_rows, card, out, s_state, s_row, err, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                 (int64_t)gridDim.x * blockDim.x);
}

// ----------------------------------------------------------------------------- argmax
__device__ __forceinline__ bool am_better(double v, uint32_t i, double bv, uint32_t bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn) return !bn || i < bi;  // np.argmax: first NaN wins
  if (bn) return false;
  return v > bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(256) void k_argmax(const double *__restrict__ X, uint64_t n_rows, uint32_t row_len,
                                                int64_t s_row, int64_t s_elem, int g_log2,
                                                int64_t *__restrict__ out, int32_t *__restrict__ out32) {
  const uint32_t G = 1u << g_log2;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane_g = (uint32_t)tid & (G - 1);
  const uint64_t ngroups = ((uint64_t)gridDim.x * blockDim.x) >> g_log2;
  for (uint64_t r = tid >> g_log2; r < n_rows; r += ngroups) {
    double bv = -__builtin_inf();
    uint32_t bi = 0xffffffffu;
    for (uint32_t i = lane_g; i < row_len; i += G) {
      const double v = X[(int64_t)r * s_row + (int64_t)i * s_elem];
      if (am_better(v, i, bv, bi)) {
        bv = v;
        bi = i;
      }
    }
    for (uint32_t off = G >> 1; off > 0; off >>= 1) {
      const double ov = __shfl_xor(bv, (int)off, 64);
      const uint32_t oi = (uint32_t)__shfl_xor((int)bi, (int)off, 64);
      if (am_better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane_g == 0) {
      const int64_t v = (bi == 0xffffffffu) ? 0 : (int64_t)bi;
      if (out) out[r] = v;
      if (out32) out32[r] = (int32_t)v;
    }
  }
}

// ----------------------------------------------------------------------------- dense pairwise step
// C[b, m, n] = sum_k A[b, m, k] B[b, k, n], FP64 MFMA (v_mfma_f64_16x16x4_f64), every index a
// group of variables addressed through a per-index offset table (any label interleaving, no
// packing copies; C written directly in the planner's label order).  A 64x64 output tile per
// workgroup, 4 waves in 2x2, each wave a 32x32 block = 2x2 MFMA tiles (4 independent
// accumulators).  K advances 16 at a time through LDS, A staged transposed (As[k][m]) so each
// operand read is 16 consecutive doubles per k row; the next K tile's global loads are issued
// before the current tile's MFMAs (register prefetch).  Operand maps (gfx950 f64): lane l holds
// A[l&15][k=l>>4], B[k=l>>4][l&15]; D[reg r] is row (l>>4)+4r, col l&15.
struct GemmK {
  int64_t batch, M, N, K;
  const int64_t *a_b, *b_b, *c_b, *a_m, *c_m, *a_k, *b_k, *b_n, *c_n;
  int64_t s_ab, s_bb, s_cb, s_am, s_cm, s_ak, s_bk, s_bn, s_cn;  // >= 0: strided group, -1: table
  uint32_t tiles_n;
  uint32_t a_mfast, b_kfast;  // tile-load lane order: A along m (else k), B along k (else n) — the unit-stride axis
};
// offset of index i of a group: the table (TAB) or a single stride (the group collapses)
template <bool TAB>
__device__ __forceinline__ int64_t goff(int64_t s, const int64_t *tab, int64_t i) {
  if constexpr (TAB) return tab[i];
  else return i * s;
}

// TA / TB / TC: operand A, B, C addressed through its offset tables (some group does not collapse).
// BM x BN block tile, 4 waves in a WY x WX grid, each wave FM x FN 16x16 f64 MFMA tiles; BK = 16.
// Tiles: 64x64 (2x2 waves of 32x32), 16x128 for M <= 16 (1x4 waves of 16x32: no MFMA rows wasted on
// a 16-row step), 128x64 for 64 < M <= 128 (2x2 waves of 64x32: B read once per batch, not twice).
template <int BM, int BN, bool TA, bool TB, bool TC>
__global__ __launch_bounds__(256) void k_gemm_f64(const GemmK p, const double *__restrict__ A,
                                                  const double *__restrict__ B, double *__restrict__ C) {
  constexpr int BK = 16;
  constexpr int WY = BM >= 32 ? 2 : 1, WX = 4 / WY;
  constexpr int FM = BM / 16 / WY, FN = BN / 16 / WX;
  constexpr int NA = BM * BK / 256, NB = BN * BK / 256;  // tile elements per thread per k tile
  static_assert(FM >= 1 && FN >= 1 && NA >= 1 && NB >= 1, "tile shape");
#ifndef PGM_GEMM_PAD
#define PGM_GEMM_PAD 1
#endif
  __shared__ double As[BK][BM + PGM_GEMM_PAD];  // +1: the k-fast tile stores (16 lanes down a column) hit 32 distinct banks
  __shared__ double Bs[BK][BN + PGM_GEMM_PAD];
  typedef double d4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wy = wave / WX, wx = wave % WX;
  const uint32_t t = blockIdx.x;  // n fastest within an m row of tiles (A rows stay hot in L2)
  const int64_t n0 = (int64_t)(t % p.tiles_n) * BN, m0 = (int64_t)(t / p.tiles_n) * BM;
  const int64_t b = (int64_t)blockIdx.z * gridDim.y + blockIdx.y;  // batches beyond 65,535 continue in z
  if (b >= p.batch) return;  // (whole block: uniform)
  const double *Ab = A + goff<TA>(p.s_ab, p.a_b, b);
  const double *Bb = B + goff<TB>(p.s_bb, p.b_b, b);
  // this thread's tile elements per operand and k tile (e = tid + 256 i), lanes along the operand's
  // unit-stride axis: A k-fast (k = e % 16, m = e / 16) or m-fast (m = e % BM, k = e / BM);
  // B n-fast (n = e % BN, k = e / BN) or k-fast (k = e % 16, n = e / 16)
  const bool amf = p.a_mfast, bkf = p.b_kfast;
  int am[NA], ak[NA], bk[NB], bn[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int e = tid + 256 * i;
    am[i] = amf ? (e % BM) : (e >> 4);
    ak[i] = amf ? (e / BM) : (e & 15);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int e = tid + 256 * i;
    bk[i] = bkf ? (e & 15) : (e / BN);
    bn[i] = bkf ? (e >> 4) : (e % BN);
  }
  int64_t arow[NA], bcol[NB];
  bool aok[NA], bok[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int64_t gm = m0 + am[i];
    aok[i] = gm < p.M;
    arow[i] = aok[i] ? goff<TA>(p.s_am, p.a_m, gm) : 0;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int64_t gn = n0 + bn[i];
    bok[i] = gn < p.N;
    bcol[i] = bok[i] ? goff<TB>(p.s_bn, p.b_n, gn) : 0;
  }
  double ra[NA], rb[NB];
  // k offsets.  SR (64 x 64 tiles): strided groups keep a running offset advanced by BK strides per
  // tile (one 64-bit add instead of a multiply and a clamp per element and tile: the plain 64 x 64
  // kernel was VALU-bound on that address arithmetic, 4096^2 x 512: 35 -> 40 TF/s); tiles wholly
  // inside K take unguarded loads, the last tile guards each k.  The 128 x 64 and 16 x 128 tiles keep
  // the clamped per-tile form (the running form costs them registers: 500 x (100 x 576 x 125)
  // 307 -> 400 us, profiles/r02bo_gemm_ab.txt).  Table groups read their entries one k tile ahead of
  // the loads that use them, so a table lookup never sits in series with its data load.
  constexpr bool SR = BM == 64 && BN == 64;
  int64_t oa[NA], ob[NB];
  const int64_t dka = (int64_t)BK * p.s_ak, dkb = (int64_t)BK * p.s_bk;
  auto offs = [&](int64_t k0) {
    const bool full = SR && k0 + BK <= p.K;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (TA || !SR) {
        const int64_t gka = k0 + ak[i];
        oa[i] = goff<TA>(p.s_ak, p.a_k, full ? gka : (gka < p.K ? gka : p.K - 1));
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (TB || !SR) {
        const int64_t gkb = k0 + bk[i];
        ob[i] = goff<TB>(p.s_bk, p.b_k, full ? gkb : (gkb < p.K ? gkb : p.K - 1));
      }
    }
  };
  if constexpr (SR && !TA) {
#pragma unroll
    for (int i = 0; i < NA; ++i) oa[i] = (int64_t)ak[i] * p.s_ak;
  }
  if constexpr (SR && !TB) {
#pragma unroll
    for (int i = 0; i < NB; ++i) ob[i] = (int64_t)bk[i] * p.s_bk;
  }
  // rows / columns past M / N (and, in the clamped form, k past K) read an in-bounds element and
  // are zeroed
  auto load = [&](int64_t k0) {
    double va[NA], vb[NB];
    if (!SR || k0 + BK <= p.K) {
#pragma unroll
      for (int i = 0; i < NA; ++i) va[i] = Ab[arow[i] + oa[i]];
#pragma unroll
      for (int i = 0; i < NB; ++i) vb[i] = Bb[ob[i] + bcol[i]];
#pragma unroll
      for (int i = 0; i < NA; ++i) ra[i] = (aok[i] && (SR || k0 + ak[i] < p.K)) ? va[i] : 0.0;
#pragma unroll
      for (int i = 0; i < NB; ++i) rb[i] = (bok[i] && (SR || k0 + bk[i] < p.K)) ? vb[i] : 0.0;
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        double v = 0.0;
        if (aok[i] && k0 + ak[i] < p.K) v = Ab[arow[i] + oa[i]];
        ra[i] = v;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        double v = 0.0;
        if (bok[i] && k0 + bk[i] < p.K) v = Bb[ob[i] + bcol[i]];
        rb[i] = v;
      }
    }
    if constexpr (SR && !TA) {
#pragma unroll
      for (int i = 0; i < NA; ++i) oa[i] += dka;
    }
    if constexpr (SR && !TB) {
#pragma unroll
      for (int i = 0; i < NB; ++i) ob[i] += dkb;
    }
  };
  d4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  offs(0);
  load(0);
  offs(BK);
  for (int64_t k0 = 0; k0 < p.K; k0 += BK) {
#pragma unroll
    for (int i = 0; i < NA; ++i) As[ak[i]][am[i]] = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) Bs[bk[i]][bn[i]] = rb[i];
    __syncthreads();
    if (k0 + BK < p.K) {  // in flight during this tile's MFMAs
      load(k0 + BK);
      offs(k0 + 2 * BK);
    }
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const int kq = 4 * s + (lane >> 4);
      double av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) av[i] = As[kq][(wy * FM + i) * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[j] = Bs[kq][(wx * FN + j) * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  double *Cb = C + goff<TC>(p.s_cb, p.c_b, b);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int64_t cn = n0 + (wx * FN + j) * 16 + (lane & 15);
    if (cn >= p.N) continue;
    const int64_t ocn = goff<TC>(p.s_cn, p.c_n, cn);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t cm = m0 + (wy * FM + i) * 16 + (lane >> 4) + 4 * r;
        if (cm < p.M) Cb[goff<TC>(p.s_cm, p.c_m, cm) + ocn] = acc[i][j][r];
      }
  }
}

template <int BM, int BN>
static void launch_gemm(int tabs, dim3 g, hipStream_t s, const GemmK &k, const double *A, const double *B, double *C) {
  const dim3 b(256);
  switch (tabs) {
    case 0: hipLaunchKernelGGL((k_gemm_f64<BM, BN, false, false, false>), g, b, 0, s, k, A, B, C); break;
    case 1: hipLaunchKernelGGL((k_gemm_f64<BM, BN, false, false, true>), g, b, 0, s, k, A, B, C); break;
    case 2: hipLaunchKernelGGL((k_gemm_f64<BM, BN, false, true, false>), g, b, 0, s, k, A, B, C); break;
    case 3: hipLaunchKernelGGL((k_gemm_f64<BM, BN, false, true, true>), g, b, 0, s, k, A, B, C); break;
    case 4: hipLaunchKernelGGL((k_gemm_f64<BM, BN, true, false, false>), g, b, 0, s, k, A, B, C); break;
    case 5: hipLaunchKernelGGL((k_gemm_f64<BM, BN, true, false, true>), g, b, 0, s, k, A, B, C); break;
    case 6: hipLaunchKernelGGL((k_gemm_f64<BM, BN, true, true, false>), g, b, 0, s, k, A, B, C); break;
    default: hipLaunchKernelGGL((k_gemm_f64<BM, BN, true, true, true>), g, b, 0, s, k, A, B, C); break;
  }
}

// ----------------------------------------------------------------------------- evidence column select
__global__ __launch_bounds__(256) void k_codes_select(const uint8_t *__restrict__ codes, int64_t ld, int64_t row0,
                                                      const int32_t *__restrict__ cols, int64_t n_rows,
                                                      uint8_t *__restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (r < n_rows) out[(int64_t)j * n_rows + r] = codes[(int64_t)cols[j] * ld + row0 + r];
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// ----------------------------------------------------------------------------- evidence ingestion
// DataFrame columns -> evidence codes (the reference maps each state name with
// name_to_no per row and evidence variable, state_name.py:71-84, DiscreteFactor.py:589-597).  Input:
// per-column int8 indices into that column's categories (pandas Categorical / Arrow dictionary
// indices, -1 = NaN); a per-column LUT maps a category index to the variable's state number (254 =
// a category that is not a state name of the variable).  Output: uint8 state codes (255 = NaN) and,
// per row, the key of its missing-column pattern (XOR of the missing columns' 64-bit keys) and its
// number of missing columns, from which the host groups rows by evidence pattern.  One thread per
// row over a chunk of columns (blockIdx.y); byte accesses along the rows are coalesced.
__global__ __launch_bounds__(256) void k_codes_remap(const int8_t *__restrict__ raw, int64_t ld_raw,
                                                     const uint8_t *__restrict__ lut, int32_t lut_stride,
                                                     int32_t n_cols, int64_t n_rows, int32_t chunk,
                                                     const uint64_t *__restrict__ col_key, uint8_t *__restrict__ out,
                                                     int64_t ld_out, unsigned long long *__restrict__ row_key,
                                                     uint32_t *__restrict__ row_nmiss,
                                                     unsigned long long *__restrict__ row_hash,
                                                     int32_t *__restrict__ err) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n_rows) return;
  const int c0 = blockIdx.y * chunk;
  const int c1 = min(n_cols, c0 + chunk);
  unsigned long long key = 0, h0 = 0, h1 = 0;
  uint32_t nm = 0;
  bool bad = false;
  for (int c = c0; c < c1; ++c) {
    const int v = raw[(int64_t)c * ld_raw + r];
    uint8_t st;
    if (v < 0) {
      st = 255;
      key ^= col_key[c];
      ++nm;
    } else if (v >= lut_stride) {
      st = 254;
      bad = true;
    } else {
      st = lut[(int64_t)c * lut_stride + v];
      bad |= st == 254;
    }
    out[(int64_t)c * ld_out + r] = st;
    if (row_hash) {  // row content: XOR of two independent mixes of (column, state)
      const unsigned long long x = ((unsigned long long)c << 8) | st;
      h0 ^= mix64(x ^ 0x9e3779b97f4a7c15ull);
      h1 ^= mix64(x ^ 0xc2b2ae3d27d4eb4full);
    }
  }
  if (nm && row_key) {
    atomicXor(&row_key[r], key);
    atomicAdd(&row_nmiss[r], nm);
  }
  if (row_hash) {
    atomicXor(&row_hash[2 * r], h0);
    atomicXor(&row_hash[2 * r + 1], h1);
  }
  if (bad && err) atomicOr(err, 1);
}

// numpy's float64 add.reduce of a strided run (the pairwise summation of numpy's umath loops): runs
// of < 8 summed in order; runs of <= 128 in 8 interleaved accumulators combined as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail in order; longer runs split in two at a
// multiple of 8 below the half, each half summed the same way.  Post-order over an explicit stack.
// numpy hands the loop at most one 8,192-element buffer at a time and adds the buffers' sums in
// order (np_sum); checked bit for bit against numpy 2.2 up to 40,000 elements (tests).
__device__ double np_block_sum(const double *a, int64_t n, int64_t s) {
  if (n < 8) {
    double res = 0.0;
    for (int64_t i = 0; i < n; ++i) res += a[i * s];
    return res;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j * s];
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[(i + j) * s];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i * s];
  return res;
}

__device__ double np_pairwise_sum(const double *a, int64_t n, int64_t s) {
  if (n <= 128) return np_block_sum(a, n, s);
  int64_t off[40], len[40];
  double left[40];
  int stage[40];
  int top = 0;
  off[0] = 0, len[0] = n, stage[0] = 0;
  double val = 0.0;
  bool have = false;
  for (;;) {
    if (!have) {
      if (len[top] <= 128) {
        val = np_block_sum(a + off[top] * s, len[top], s);
        have = true;
        --top;
      } else {  // descend into the left half
        int64_t n2 = len[top] / 2;
        n2 -= n2 % 8;
        stage[top] = 1;
        off[top + 1] = off[top], len[top + 1] = n2, stage[top + 1] = 0;
        ++top;
      }
    } else {
      if (top < 0) return val;
      if (stage[top] == 1) {  // left done: the right half next
        int64_t n2 = len[top] / 2;
        n2 -= n2 % 8;
        left[top] = val;
        stage[top] = 2;
        off[top + 1] = off[top] + n2, len[top + 1] = len[top] - n2, stage[top + 1] = 0;
        ++top;
        have = false;
      } else {
        val = left[top] + val;
        --top;
      }
    }
  }
}

// predict(stochastic=True) (DiscreteBayesianNetwork.py:889-892 -> DiscreteFactor.sample L868-912):
// sample() normalises the joint (values / values.sum(), DiscreteFactor.py:530: numpy's pairwise sum)
// and numpy's Generator.choice(P, p=p) then takes cdf = cumsum(p) (in order), cdf /= cdf[-1] and
// index = searchsorted(cdf, u, side="right") = the number of cdf entries <= u.  The same operations
// in the same order per output row r, so a uniform on a CDF boundary lands where numpy puts it; the
// uniforms u come from the reference's seeded stream on the host.  joint column group[r].
__global__ __launch_bounds__(256) void k_sample_joint(const double *__restrict__ joint, int64_t ld, int64_t P,
                                                      const int32_t *__restrict__ group,
                                                      const double *__restrict__ u, int64_t n,
                                                      int32_t *__restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const double *q = joint + group[r];
  double total = 0.0;
  for (int64_t c = 0; c < P; c += 8192) total += np_pairwise_sum(q + c * ld, P - c < 8192 ? P - c : 8192, ld);
  double last = 0.0;
  for (int64_t i = 0; i < P; ++i) last = i ? last + q[i * ld] / total : q[0] / total;
  const double x = u[r];
  double acc = 0.0;
  int64_t idx = 0;
  for (int64_t i = 0; i < P; ++i) {
    acc = i ? acc + q[i * ld] / total : q[0] / total;
    if (acc / last <= x) idx = i + 1;
  }
  out[r] = (int32_t)(idx < P ? idx : P - 1);
}

// ----------------------------------------------------------------------------- fused row plan
// One workgroup owns 64 evidence rows (one per lane) for RG consecutive row groups; its waves split
// the plan's independent components (wave w takes components w, w+W, ...), so every descriptor
// read, loop bound and branch is wave-uniform (scalar) and a row's work is spread over W
// wavefronts.  A wave loads only its components' evidence codes (all in flight at once) and
// stages only their CPT values into LDS.  Components meet once per row group through LDS: masses
// (impossible evidence makes every marginal NaN), MAP index digits and MAP gaps.
//
// Descriptors live in device memory as packed structs (one s_load_dwordx16 per component, one
// s_load_dwordx4 per evidence term).  Table-driven components: for every entry e of a component's
// (query x hidden) index space the host precomputes each factor's offset (tab[off_base + e*nf + j]),
// the marginal rows each query dim accumulates into (tab[marg_base + qi*nq + i]) and the entry's MAP
// index digit (tab[map_base + qi]).  Affine components (one query dim, no hidden dim) need no
// table: factor j sits at base_j + s * fstride[j] for query state s.
struct RowsComp {
  int32_t nf, nt, P, H;
  int32_t simple, mstride, q_lo, q_hi;
  int32_t off_base, marg_base, map_base, ev_lo;  // ev_lo: first evidence term (n_ev when none)
  int32_t val_lo, val_hi, marg0, nq;              // marg0: marginal row of the (affine) query dim
  int32_t fbase[PGM_ROWS_MAX_FAC];
  int32_t fstride[PGM_ROWS_MAX_FAC];
  // affine fast kernel: evidence terms folded into per-slot strides (term j adds code_j * aS[j][k]
  // to factor slot k), padded to 8 terms (stride 0, card 256, a real column)
  int32_t a_S[8][4];
  int32_t a_col[8], a_card[8];
};
struct RowsTerm {
  int32_t col, stride, card, slot;  // evidence column, stride in its factor, cardinality, factor slot
};
struct RowsK {
  int32_t n_values, n_marg, n_joint, n_comp;  // n_values includes the trailing 1.0 (index one_idx)
  int32_t n_waves, terms_off, tab_off, one_idx;  // offsets (in int32) into the descriptor buffer
  int32_t q_marg_off[PGM_ROWS_MAX_LOOP], q_card[PGM_ROWS_MAX_LOOP];
};

struct RowsHandle {
  RowsK k;
  int max_nf, max_nt;
  bool any_table, all_affine;
  double *d_values;
  int32_t *d_desc;
  // plan-specialised kernel (hipRTC): generated at create for all-affine plans, compiled on first use
  std::string jit_src;
  std::mutex jit_mu;
  int jit_state = 0;  // 0 not compiled, 1 ready, -1 unavailable (the AOT kernels run instead)
  hipModule_t jit_mod = nullptr;
  hipFunction_t jit_fn = nullptr;
  hipFunction_t jit_fn2 = nullptr;  // two rows per thread
  hipFunction_t jit_fn_floor = nullptr;  // PGM_ROWS_FLOOR: the same dispatch's loads + stores only
  hipFunction_t jit_fn_floor2 = nullptr;  // ... of the two-rows-per-thread dispatch
  hipFunction_t jit_fn_ring = nullptr;    // the resident ring kernel (pgm_rows_ring_*)
  std::vector<char> jit_code;         // the compiled code object (the direct AQL path loads it again)
  bool jit_write_through = false;     // its output stores are write-through (jit_store() == 2)
  int device = 0;                     // the HIP device current at create (its buffers / module live there)
  int n_cols = 0;                     // 1 + the largest evidence column the plan reads (0: none)
  std::vector<int> cols;              // the evidence columns the plan reads, ascending
  // pgm_rows_shard_run's resources on this handle's device, created on first use and kept until the
  // handle is destroyed: two streams, each with its own grow-only device chunk buffer (codes of the
  // columns the plan reads, outputs, error flag) and a pinned error word, so consecutive chunks
  // alternate between them (chunk c + 1's copy-in and pass overlap chunk c's copy-out)
  struct ShardSide {
    hipStream_t s = nullptr;
    char *buf = nullptr;
    size_t cap = 0;
    int32_t *h_err = nullptr;
  };
  ShardSide shard[2];
  std::mutex shard_mu;  // one pgm_rows_shard_run shard at a time per handle
};

template <bool VL, bool AL, int MAXFC, int MAXT>
__global__ __launch_bounds__(64 * PGM_ROWS_MAX_COMP) void k_rows(
    const RowsK p, const double *__restrict__ gvals, const int32_t *__restrict__ desc,
    const uint8_t *__restrict__ codes, int64_t ld_codes, int64_t row0, int64_t n_rows, int32_t mode, int32_t RG,
    double *__restrict__ marg, double *__restrict__ joint, int64_t ld_out, int32_t *__restrict__ map,
    double *__restrict__ gap, int32_t *__restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // this wave's component
  const int NC = p.n_comp;
  const RowsComp &cd = ((const RowsComp *)desc)[c];
  const RowsTerm *__restrict__ tt = (const RowsTerm *)(desc + p.terms_off) + cd.ev_lo;
  const int32_t *__restrict__ tab = desc + p.tab_off;
  double *svals = lds;
  double *xmass = lds + (VL ? ((p.n_values + 1) & ~1) : 0);  // [NC][64]
  double *xgap = xmass + NC * 64;                              // [NC][64]
  int32_t *xmap = (int32_t *)(xgap + NC * 64);                 // [NC][64]
  double *sacc = (double *)(xmap + NC * 64);                   // [n_marg][64]
  const bool do_marg = (mode & PGM_ROWS_MARGINALS) != 0;
  const bool do_joint = (mode & PGM_ROWS_JOINT) != 0;
  const bool do_map = (mode & (PGM_ROWS_MAP | PGM_ROWS_MAPGAP)) != 0;
  const int nf = cd.nf, nq = cd.nq, nt = cd.nt;
  const uint32_t P = cd.P, H = cd.H;
  auto val = [&](int32_t i) -> double {
    if constexpr (VL) return svals[i];
    else return gvals[i];
  };
  // stage this component's CPT values once per workgroup (no other wave reads them: no barrier)
  if constexpr (VL) {
    if (lane == 0) svals[p.one_idx] = 1.0;
    for (int i = cd.val_lo + lane; i < cd.val_hi; i += 64) svals[i] = gvals[i];
  }
  // evidence codes of row group g (MAXT <= 8: padded terms, static descriptor offsets)
  constexpr int NT = MAXT <= 8 ? MAXT : 1;
  auto load_codes = [&](int g, uint32_t (&code)[NT]) {
    const int64_t r = ((int64_t)blockIdx.x * RG + g) * 64 + lane;
    const uint8_t *crow = codes + row0 + (r < n_rows ? r : 0);
#pragma unroll
    for (int j = 0; j < NT; ++j) code[j] = crow[(int64_t)tt[j].col * ld_codes];
  };
  uint32_t nxt[NT];
  if (MAXT <= 8 && nt > 0) load_codes(0, nxt);
  for (int g = 0; g < RG; ++g) {
    const int64_t r = ((int64_t)blockIdx.x * RG + g) * 64 + lane;
    const bool live = r < n_rows;
    auto acc = [&](int32_t t) -> double & {
      if constexpr (AL) return sacc[t * 64 + lane];
      else return marg[(int64_t)t * ld_out + r];
    };
    int32_t cb[MAXFC];  // slots >= nf point at the constant 1.0 (fbase = one_idx, fstride = 0)
#pragma unroll
    for (int j = 0; j < MAXFC; ++j) cb[j] = cd.fbase[j];
    bool bad = false;
    if (nt == 0) {
      // no evidence in this component: nothing to load (codes may have no columns at all)
    } else if constexpr (MAXT <= 8) {
      uint32_t code[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) code[j] = nxt[j];
      if (g + 1 < RG) load_codes(g + 1, nxt);  // next row group's codes in flight during this one
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const RowsTerm &t = tt[j];
        const bool oob = code[j] >= (uint32_t)t.card;
        bad |= oob;
        const int32_t w = oob ? 0 : (int32_t)code[j] * t.stride;
#pragma unroll
        for (int k = 0; k < MAXFC; ++k) cb[k] += (k == t.slot) ? w : 0;
      }
    } else {
      const uint8_t *crow = codes + row0 + (live ? r : 0);
      for (int j = 0; j < nt; ++j) {
        const RowsTerm &t = tt[j];
        uint32_t cv = crow[(int64_t)t.col * ld_codes];
        if (cv >= (uint32_t)t.card) {
          bad = true;
          cv = 0;
        }
        const int32_t w = (int32_t)cv * t.stride;
#pragma unroll
        for (int k = 0; k < MAXFC; ++k) cb[k] += (k == t.slot) ? w : 0;
      }
    }
    if (bad && live && err) atomicOr(err, 1);
    double mass = 0.0, best = -1.0, second = -1.0;
    int32_t best_map = 0;
    if (cd.simple) {
      // affine: states [0, RC) stay in registers (branch-free clamped loads, all LDS reads of
      // the pass in flight at once); states >= RC are recomputed in the write pass
      const int32_t ms = cd.mstride;
      constexpr int RC = 8;
      double pc[RC];
      const int32_t plast = (int32_t)P - 1;
#pragma unroll
      for (int qs = 0; qs < RC; ++qs) {
        const int32_t q = qs < plast ? qs : plast;
        double prod = val(cb[0] + q * cd.fstride[0]);
#pragma unroll
        for (int j = 1; j < MAXFC; ++j) prod *= val(cb[j] + q * cd.fstride[j]);
        pc[qs] = prod;
      }
      auto visit = [&](uint32_t qs, double prod) {
        mass += prod;
        if (do_joint && live) joint[(int64_t)qs * ms * ld_out + r] = prod;
        if (do_map) {
          if (prod > best) {
            second = best;
            best = prod;
            best_map = (int32_t)qs * ms;
          } else if (prod > second) {
            second = prod;
          }
        }
      };
#pragma unroll
      for (int qs = 0; qs < RC; ++qs)
        if ((uint32_t)qs < P) visit(qs, pc[qs]);
      for (uint32_t qs = RC; qs < P; ++qs) {
        double prod = val(cb[0] + (int32_t)qs * cd.fstride[0]);
#pragma unroll
        for (int j = 1; j < MAXFC; ++j) prod *= val(cb[j] + (int32_t)qs * cd.fstride[j]);
        visit(qs, prod);
      }
      if (do_marg && nq && live) {  // normalised marginal streamed straight to HBM
        const double inv = 1.0 / mass;
        double *out = marg + (int64_t)cd.marg0 * ld_out + r;
#pragma unroll
        for (int qs = 0; qs < RC; ++qs)
          if ((uint32_t)qs < P) __builtin_nontemporal_store(pc[qs] * inv, out + (int64_t)qs * ld_out);
        for (uint32_t qs = RC; qs < P; ++qs) {
          double prod = val(cb[0] + (int32_t)qs * cd.fstride[0]);
#pragma unroll
          for (int j = 1; j < MAXFC; ++j) prod *= val(cb[j] + (int32_t)qs * cd.fstride[j]);
          __builtin_nontemporal_store(prod * inv, out + (int64_t)qs * ld_out);
        }
      }
    } else if (live) {
      const int32_t *toff = tab + cd.off_base;
      const int32_t *tmarg = tab + cd.marg_base;
      const int32_t *tmap = tab + cd.map_base;
      if (do_marg && nq > 1) {
        for (int q = cd.q_lo; q < cd.q_hi; ++q)
          for (int s = 0; s < p.q_card[q]; ++s) acc(p.q_marg_off[q] + s) = 0.0;
      }
      uint32_t e = 0;
#pragma unroll 2
      for (uint32_t qi = 0; qi < P; ++qi) {
        double v = 0.0;
        if (H == 1) {  // no hidden dims: one product per query entry
          const int32_t *o = toff + qi * nf;
          double prod = 1.0;
#pragma unroll
          for (int j = 0; j < MAXFC; ++j)
            if (j < nf) prod *= val(cb[j] + o[j]);
          v = prod;
        } else {
          for (uint32_t hi = 0; hi < H; ++hi, ++e) {
            const int32_t *o = toff + e * nf;
            double prod = 1.0;
#pragma unroll
            for (int j = 0; j < MAXFC; ++j)
              if (j < nf) prod *= val(cb[j] + o[j]);
            v += prod;
          }
        }
        mass += v;
        if (do_marg) {
          if (nq == 1) {
            acc(tmarg[qi]) = v;  // each marginal row is hit exactly once
          } else {
            for (int i = 0; i < nq; ++i) acc(tmarg[qi * nq + i]) += v;
          }
        }
        if (do_joint) joint[(int64_t)tmap[qi] * ld_out + r] = v;
        if (do_map) {
          if (v > best) {
            second = best;
            best = v;
            best_map = tmap[qi];
          } else if (v > second) {
            second = v;
          }
        }
      }
      if (do_marg && nq > 0) {  // component marginals normalised by the component mass
        const double inv = 1.0 / mass;
        for (int q = cd.q_lo; q < cd.q_hi; ++q)
          for (int s = 0; s < p.q_card[q]; ++s) {
            const int a = p.q_marg_off[q] + s;
            if constexpr (AL) marg[(int64_t)a * ld_out + r] = acc(a) * inv;
            else acc(a) *= inv;
          }
      }
    }
    if (NC > 1 || do_map) {
      xmass[c * 64 + lane] = mass;
      if (do_map) {
        xmap[c * 64 + lane] = best_map;
        xgap[c * 64 + lane] = (P > 1) ? (best > 0.0 ? (best - (second < 0.0 ? 0.0 : second)) / best : 0.0) : 1.0;
      }
    }
    if (NC > 1) __syncthreads();
    if (live) {
      double z = mass;
      if (NC > 1) {
        z = 1.0;
        for (int c2 = 0; c2 < NC; ++c2) z *= xmass[c2 * 64 + lane];
      }
      // impossible evidence (zero total mass): every marginal is 0/0 = NaN and np.argmax gives 0
      const bool dead = !(z > 0.0);
      if (do_marg && dead) {
        const double nan = __builtin_nan("");
        for (int q = cd.q_lo; q < cd.q_hi; ++q)
          for (int s = 0; s < p.q_card[q]; ++s) marg[(int64_t)(p.q_marg_off[q] + s) * ld_out + r] = nan;
      }
      if (do_joint && c == 0) {  // single-component plans only
        const double inv = 1.0 / z;
        for (int q = 0; q < p.n_joint; ++q) {
          double *j = joint + (int64_t)q * ld_out + r;
          *j = dead ? __builtin_nan("") : *j * inv;
        }
      }
      if (do_map && c == 0) {
        int32_t m = 0;
        double mg = 1.0;
        for (int c2 = 0; c2 < NC; ++c2) {
          m += xmap[c2 * 64 + lane];
          mg = fmin(mg, xgap[c2 * 64 + lane]);
        }
        if (map) map[r] = dead ? 0 : m;
        if (gap && (mode & PGM_ROWS_MAPGAP)) gap[r] = dead ? 0.0 : mg;
      }
    }
    if (NC > 1 && g + 1 < RG) __syncthreads();  // the exchange slots are reused by the next row group
  }
}

// workgroup barrier for LDS-only exchanges: waits for this wave's LDS traffic, not for its global
// loads/stores (__syncthreads' release fence would wait for every outstanding store to be acked)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// All-affine plans (every component one query dim, no hidden dim, <= 4 factors, <= 8 evidence
// terms: the common batched-predict shape, e.g. munin C3).  Same work split as k_rows, but each
// wave loads its component's descriptor into registers once, folds evidence with multiply-adds
// against host-precomputed per-slot strides, and carries the MAP bookkeeping only when asked.
// Latency shape (one row group per wave at 100k rows): descriptor -> {codes, CPT staging} in
// flight together (staging issues every load before any LDS write) -> products -> LDS-only
// exchange of component masses -> stores.  PGM_ROWS_TIMELINE builds add per-wave s_memrealtime
// stamps (tools/rows_timeline.py).
template <bool VL, int NF, int NT, bool MAP>
__global__ __launch_bounds__(64 * PGM_ROWS_MAX_COMP) void k_rows_affine(
    const RowsK p, const double *__restrict__ gvals, const int32_t *__restrict__ desc,
    const uint8_t *__restrict__ codes, int64_t ld_codes, int64_t row0, int64_t n_rows, int32_t mode, int32_t RG,
    double *__restrict__ marg, int64_t ld_out, int32_t *__restrict__ map, double *__restrict__ gap,
    int32_t *__restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
#ifdef PGM_ROWS_TIMELINE
  const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
#endif
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // this wave's component
  const int NC = p.n_comp;
  const RowsComp &cd = ((const RowsComp *)desc)[c];
  double *svals = lds;
  double *xmass = lds + (VL ? ((p.n_values + 1) & ~1) : 0);  // [NC][64]
  double *xgap = xmass + NC * 64;                              // [NC][64] (MAP only)
  int32_t *xmap = (int32_t *)(xgap + NC * 64);                 // [NC][64] (MAP only)
  const bool do_marg = (mode & PGM_ROWS_MARGINALS) != 0;
  // descriptor -> registers (wave-uniform)
  int32_t fb[NF], fs[NF], S[NT][NF];
  uint32_t card[NT];
  int64_t cofs[NT];
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    fb[k] = cd.fbase[k];
    fs[k] = cd.fstride[k];
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    card[j] = (uint32_t)cd.a_card[j];
    cofs[j] = (int64_t)cd.a_col[j] * ld_codes + row0;
#pragma unroll
    for (int k = 0; k < NF; ++k) S[j][k] = cd.a_S[j][k];
  }
  const int nt = cd.nt;
  const uint32_t P = (uint32_t)cd.P;
  const int32_t ms = cd.mstride;
  double *mrow = marg + (int64_t)cd.marg0 * ld_out;
  auto val = [&](int32_t i) -> double {
    if constexpr (VL) return svals[i];
    else return gvals[i];
  };
  auto load_codes = [&](int g, uint32_t (&code)[NT]) {
    const int64_t r = ((int64_t)blockIdx.x * RG + g) * 64 + lane;
    const uint8_t *crow = codes + (r < n_rows ? r : 0);
#pragma unroll
    for (int j = 0; j < NT; ++j) code[j] = crow[cofs[j]];
  };
  // this wave's first 256 CPT values, then the first row group's codes, all in flight before the
  // LDS writes (vmcnt is in order: the writes wait only for the value loads); larger components
  // stage the rest in further 256-value batches
  uint32_t nx[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) nx[j] = 0;
  const int vlo = cd.val_lo, vhi = cd.val_hi;
  double t[4];
  if constexpr (VL) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = vlo + u * 64 + lane;
      t[u] = gvals[i < vhi ? i : vhi - 1];
    }
  }
  if (nt > 0) load_codes(0, nx);
  if constexpr (VL) {
    if (lane == 0) svals[p.one_idx] = 1.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // clamped lanes rewrite the last value with itself: no branches
      const int i = vlo + u * 64 + lane;
      svals[i < vhi ? i : vhi - 1] = t[u];
    }
    for (int base = vlo + 256; base < vhi; base += 256) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = base + u * 64 + lane;
        t[u] = gvals[i < vhi ? i : vhi - 1];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = base + u * 64 + lane;
        if (i < vhi) svals[i] = t[u];
      }
    }
  }
#ifdef PGM_ROWS_TIMELINE
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const uint64_t t_ready = __builtin_amdgcn_s_memrealtime();
#endif
  for (int g = 0; g < RG; ++g) {
    const int64_t r = ((int64_t)blockIdx.x * RG + g) * 64 + lane;
    const bool live = r < n_rows;
    uint32_t code[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) code[j] = nx[j];
    if (nt > 0 && g + 1 < RG) load_codes(g + 1, nx);  // next group's codes in flight during this one
    int32_t cb[NF];
#pragma unroll
    for (int k = 0; k < NF; ++k) cb[k] = fb[k];
    bool bad = false;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const bool oob = code[j] >= card[j];
      bad |= oob;
      const int32_t cj = oob ? 0 : (int32_t)code[j];
#pragma unroll
      for (int k = 0; k < NF; ++k) cb[k] += cj * S[j][k];
    }
    if (bad && live && err) atomicOr(err, 1);
    constexpr int RC = 8;
    double pc[RC];
    const int32_t plast = (int32_t)P - 1;
#pragma unroll
    for (int qs = 0; qs < RC; ++qs) {
      const int32_t q = qs < plast ? qs : plast;
      double prod = val(cb[0] + q * fs[0]);
#pragma unroll
      for (int k = 1; k < NF; ++k) prod *= val(cb[k] + q * fs[k]);
      pc[qs] = prod;
    }
    double mass = 0.0, best = -1.0, second = -1.0;
    int32_t best_s = 0;
    auto visit = [&](uint32_t qs, double prod) {
      mass += prod;
      if constexpr (MAP) {
        if (prod > best) {
          second = best;
          best = prod;
          best_s = (int32_t)qs;
        } else if (prod > second) {
          second = prod;
        }
      }
    };
#pragma unroll
    for (int qs = 0; qs < RC; ++qs)
      if ((uint32_t)qs < P) visit(qs, pc[qs]);
    for (uint32_t qs = RC; qs < P; ++qs) {
      double prod = val(cb[0] + (int32_t)qs * fs[0]);
#pragma unroll
      for (int k = 1; k < NF; ++k) prod *= val(cb[k] + (int32_t)qs * fs[k]);
      visit(qs, prod);
    }
    // the component waves of a row group meet BEFORE any store, through an LDS-only barrier
    // (no wait for global stores to be acknowledged, as __syncthreads' release fence would)
    double z = mass;
    if (NC > 1) {
      xmass[c * 64 + lane] = mass;
      if constexpr (MAP) {
        xmap[c * 64 + lane] = best_s * ms;
        xgap[c * 64 + lane] = (P > 1) ? (best > 0.0 ? (best - (second < 0.0 ? 0.0 : second)) / best : 0.0) : 1.0;
      }
      lds_barrier();
      z = 1.0;
      for (int c2 = 0; c2 < NC; ++c2) z *= xmass[c2 * 64 + lane];
    }
    // impossible evidence (zero total mass): every marginal is 0/0 = NaN and np.argmax gives 0
    const bool dead = !(z > 0.0);
    if (do_marg && live) {  // normalised marginal streamed straight to HBM
      const double inv = dead ? __builtin_nan("") : 1.0 / mass;
      double *out = mrow + r;
#pragma unroll
      for (int qs = 0; qs < RC; ++qs)
        if ((uint32_t)qs < P) out[(int64_t)qs * ld_out] = pc[qs] * inv;
      for (uint32_t qs = RC; qs < P; ++qs) {
        double prod = val(cb[0] + (int32_t)qs * fs[0]);
#pragma unroll
        for (int k = 1; k < NF; ++k) prod *= val(cb[k] + (int32_t)qs * fs[k]);
        out[(int64_t)qs * ld_out] = prod * inv;
      }
    }
    if constexpr (MAP) {
      if (live && c == 0) {
        int32_t m = best_s * ms;
        double mg = (P > 1) ? (best > 0.0 ? (best - (second < 0.0 ? 0.0 : second)) / best : 0.0) : 1.0;
        if (NC > 1) {
          m = 0;
          mg = 1.0;
          for (int c2 = 0; c2 < NC; ++c2) {
            m += xmap[c2 * 64 + lane];
            mg = fmin(mg, xgap[c2 * 64 + lane]);
          }
        }
        if (map) map[r] = dead ? 0 : m;
        if (gap && (mode & PGM_ROWS_MAPGAP)) gap[r] = dead ? 0.0 : mg;
      }
    }
    if (NC > 1 && g + 1 < RG) lds_barrier();  // the exchange slots are reused by the next row group
  }
#ifdef PGM_ROWS_TIMELINE
  {  // [entry, ready, stores issued, stores acked, HW_ID, XCC_ID] per wave into `gap`
    const uint64_t t_issued = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const uint64_t t_done = __builtin_amdgcn_s_memrealtime();
    if (gap && !(mode & PGM_ROWS_MAPGAP) && lane == 0) {
      double *tl = gap + ((int64_t)blockIdx.x * (blockDim.x >> 6) + c) * 6;
      tl[0] = (double)t_entry;
      tl[1] = (double)t_ready;
      tl[2] = (double)t_issued;
      tl[3] = (double)t_done;
      tl[4] = (double)__builtin_amdgcn_s_getreg(4 | (31 << 11));
      tl[5] = (double)__builtin_amdgcn_s_getreg(20 | (15 << 11));
    }
  }
#endif
}

template <bool VL, int NF, int NT>
static void launch_affine_m(bool do_map, dim3 g, dim3 b, size_t lds, hipStream_t s, const RowsK &k,
                            const double *v, const int32_t *t, const uint8_t *codes, int64_t ldc, int64_t row0,
                            int64_t n, int32_t mode, int32_t RG, double *marg, int64_t ldo, int32_t *map,
                            double *gap, int32_t *err) {
  if (do_map)
    hipLaunchKernelGGL((k_rows_affine<VL, NF, NT, true>), g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, ldo, map, gap, err);
  else
    hipLaunchKernelGGL((k_rows_affine<VL, NF, NT, false>), g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, ldo, map, gap, err);
}

template <bool VL>
static void launch_affine(int max_nf, int max_nt, bool do_map, dim3 g, dim3 b, size_t lds, hipStream_t s,
                          const RowsK &k, const double *v, const int32_t *t, const uint8_t *codes, int64_t ldc,
                          int64_t row0, int64_t n, int32_t mode, int32_t RG, double *marg, int64_t ldo,
                          int32_t *map, double *gap, int32_t *err) {
#define PGM_AFF(NF, NT) launch_affine_m<VL, NF, NT>(do_map, g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, ldo, map, gap, err)
  if (max_nt <= 4) {
    if (max_nf <= 1) PGM_AFF(1, 4);
    else if (max_nf <= 2) PGM_AFF(2, 4);
    else PGM_AFF(4, 4);
  } else {
    if (max_nf <= 1) PGM_AFF(1, 8);
    else if (max_nf <= 2) PGM_AFF(2, 8);
    else PGM_AFF(4, 8);
  }
#undef PGM_AFF
}

template <bool VL, bool AL, int MAXT>
static void launch_rows_t(int max_nf, dim3 g, dim3 b, size_t lds, hipStream_t s, const RowsK &k, const double *v,
                          const int32_t *t, const uint8_t *codes, int64_t ldc, int64_t row0, int64_t n, int32_t mode,
                          int32_t RG, double *marg, double *joint, int64_t ldo, int32_t *map, double *gap, int32_t *err) {
  if (max_nf <= 2)
    hipLaunchKernelGGL((k_rows<VL, AL, 2, MAXT>), g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, joint, ldo, map, gap, err);
  else if (max_nf <= 4)
    hipLaunchKernelGGL((k_rows<VL, AL, 4, MAXT>), g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, joint, ldo, map, gap, err);
  else if (max_nf <= 8)
    hipLaunchKernelGGL((k_rows<VL, AL, 8, MAXT>), g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, joint, ldo, map, gap, err);
  else
    hipLaunchKernelGGL((k_rows<VL, AL, PGM_ROWS_MAX_FAC, MAXT>), g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, joint, ldo, map, gap, err);
}

template <bool VL, bool AL>
static void launch_rows_f(int max_nt, int max_nf, dim3 g, dim3 b, size_t lds, hipStream_t s, const RowsK &k,
                          const double *v, const int32_t *t, const uint8_t *codes, int64_t ldc, int64_t row0, int64_t n,
                          int32_t mode, int32_t RG, double *marg, double *joint, int64_t ldo, int32_t *map, double *gap,
                          int32_t *err) {
  if (max_nt <= 4)
    launch_rows_t<VL, AL, 4>(max_nf, g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, joint, ldo, map, gap, err);
  else if (max_nt <= 8)
    launch_rows_t<VL, AL, 8>(max_nf, g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, joint, ldo, map, gap, err);
  else
    launch_rows_t<VL, AL, PGM_ROWS_MAX_EV>(max_nf, g, b, lds, s, k, v, t, codes, ldc, row0, n, mode, RG, marg, joint, ldo, map, gap, err);
}

// ----------------------------------------------------------------------------- plan-specialised row kernel
// For plans whose components each have one query variable and no hidden variable (the batched
// predict shape, munin C3), pgm_rows_plan_create also writes a kernel source with every column,
// stride, base offset and cardinality as a literal; hipRTC compiles it for gfx950 on first use.
// One thread per evidence row, 256-row workgroups: the CPT values are staged in LDS with every
// load issued before any LDS write, all evidence codes are loaded once per distinct column, and
// each component's products stay in registers between the mass and the stores.  No descriptor
// loads, no inter-wave exchange, a few hundred bytes of code.  Arithmetic order is exactly the
// generic kernels' (factor products left to right, masses summed in state order, components'
// masses multiplied in order), so results are bit-identical to k_rows_affine / k_rows.
void pgmi_appendf(std::string &o, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  o += buf;
}

// workgroup size of the specialised row kernels (tuning knob PGM_ROWS_JIT_WG: a multiple of 64, <= 1024).
// 512 (r02br, MI355X, C3 = 100k-row launches on 4 queues, two rows per thread): 98 blocks of 1,024
// rows per launch — one CPT staging per 1,024 rows and a quarter of the workgroup dispatches of
// 256 x one row — 26.4 -> 29.1-31.1 G rows/s at 20 steps, 36.2 -> 47.1 G at 400; one queue and
// 1M-row launches unchanged (profiles/r02bq_c3_wg_rowform_sweep.txt, r02br_c3_wg_rowform_confirm.txt)
// r04 (96 resident batches, the HBM regime: profiles/r04e, r04f): 320 — 157 blocks of 640 rows per
// 100 k-row launch keep more CUs streaming than 98 x 1,024 once the outputs go to HBM instead of the
// Infinity Cache; three interleaved repeats, 20 steps: 26.6 / 26.7 / 27.9 G rows/s against 27.3 / 25.1 /
// 25.3 G at 512 (192: 27.0 / 26.7 / 26.0; 128: 25.7 / 25.6 / 26.6; 1,024: 25.5 / 24.7 / 25.5)
// r06 (one 157-block launch never covers the 256 CUs): 192 — 261 blocks of 384 rows per
// 100 k-row launch, every CU a block from each launch; three interleaved repeats at the driver's 20 steps
// (profiles/r06b/): 26.29 / 26.82 / 26.04 G rows/s, frac 0.607 / 0.613 / 0.612, against 25.20 / 26.20 /
// 25.74 G, frac 0.572 / 0.606 / 0.588 at 320; the 400-batch ring is unchanged (0.70-0.71).  A/B knob
// PGM_ROWS_JIT_WG (a multiple of 64 in [64, 1024]), read once.
static int jit_wg() {
  static const int wg = [] {
    const char *e = getenv("PGM_ROWS_JIT_WG");
    const int v = e ? atoi(e) : 0;
    return (v >= 64 && v <= 1024 && v % 64 == 0) ? v : 192;
  }();
  return wg;
}

// output store form of the specialised kernels: write-through — 8-B relaxed agent-scope atomic stores /
// 16-B buffer stores with the sc1 bit — so every output line goes past the XCD's L2 in the dispatch that
// writes it (no dirty output left for an end-of-dispatch release to write back; measured MI355X, 100k
// rows: HIP launch 4.7 -> 3.8 us, direct queue 6.2 -> 4.0 us with the per-dispatch release dropped,
// WRITE_SIZE 13.28 MB per launch either way; r02 also measured plain (write-back) and nontemporal forms)
static constexpr int jit_store() { return 2; }

// workgroup size of the ring kernel: 256 = one wave per
// SIMD per workgroup; the loop around the two-row body takes ~147 VGPRs (3 waves per SIMD), so three
// workgroups are resident per CU (a 1,024-thread bound caps it at 128 VGPRs and spills to scratch;
// 512 threads fit one workgroup per CU)
static constexpr int ring_wg() { return 256; }

// the ring's waiting waves back off: the workgroup's token wave reads the chip-wide poll token before
// trying to take it, and sleeps longer the longer it has waited (4 -> 12 -> 32 x 64 clocks).  768 token
// waves retrying one atomic every ~0.1 us while the ring idles saturate that address and delay the one
// wave that reads the host counter (r03: ring-ready 20 steps 17.1 -> 29.5-30.8 G rows/s)
static constexpr bool ring_backoff() { return true; }

static std::vector<int> rows_cols(const pgm_rows_plan *pl);
static void emit_rows_code_loads(std::string &o, const std::vector<int> &cols, int R, bool coherent = false);
static void emit_rows_compute(std::string &o, const pgm_rows_plan *pl, int R, const std::vector<int> &cols,
                              const char *leave);

// R rows per thread (1, or 2 with 16-B marginal stores / 2-byte code loads); names carry the row's suffix
static void emit_rows_kernel(std::string &o, const pgm_rows_plan *pl, int R) {
  const int NV = pl->n_values + 1;  // + trailing 1.0
  // CPT values staged in LDS when they fit (else gathered straight from global memory through L1/L2)
  const bool lds = NV * 8 <= 48 * 1024;
  const int WG = jit_wg();
  pgmi_appendf(o, "extern \"C\" __global__ void __launch_bounds__(%d) pgm_rows_jit%s(const double *__restrict__ V, "
             "const unsigned char *__restrict__ C, long long ldc, long long row0, long long n, "
             "double *__restrict__ M, long long ldo, int *__restrict__ MP, double *__restrict__ G, "
             "int *__restrict__ E, int mode) {\n", WG, R == 2 ? "2" : "");
  o += "  const int t = threadIdx.x;\n";
  pgmi_appendf(o, "  const long long r = ((long long)blockIdx.x * %d + t) * %d;\n", WG, R);
  pgmi_appendf(o, "  const long long rc = r < n ? r : n - %d;\n", R);
  if (R == 2 && jit_store() == 2)
    o += "  const __amdgpu_buffer_rsrc_t rsM = __builtin_amdgcn_make_buffer_rsrc(M, 0, 0x7fffffff, 0x00020000);\n"
         "  const __amdgpu_buffer_rsrc_t rsG = __builtin_amdgcn_make_buffer_rsrc(G, 0, 0x7fffffff, 0x00020000);\n";
  const int K = (NV + WG - 1) / WG;
  if (lds) {
    pgmi_appendf(o, "  __shared__ double S[%d];\n", K * WG);
    for (int i = 0; i < K; ++i) pgmi_appendf(o, "  const double s%d = V[t + %d < %d ? t + %d : %d];\n", i, WG * i, NV, WG * i, NV - 1);
  }
  const std::vector<int> cols = rows_cols(pl);
  emit_rows_code_loads(o, cols, R);
  if (lds) {
    for (int i = 0; i < K; ++i) pgmi_appendf(o, "  S[t + %d < %d ? t + %d : %d] = s%d;\n", WG * i, NV, WG * i, NV - 1, i);
    o += "  __syncthreads();\n#define VAL(i) S[i]\n";
  } else {
    o += "#define VAL(i) V[i]\n";
  }
  emit_rows_compute(o, pl, R, cols, "return");
  o += "}\n#undef VAL\n";
}

// the distinct evidence columns of a plan, each loaded once per row
static std::vector<int> rows_cols(const pgm_rows_plan *pl) {
  std::vector<int> cols;
  for (int j = 0; j < pl->n_ev; ++j)
    if (std::find(cols.begin(), cols.end(), pl->ev_col[j]) == cols.end()) cols.push_back(pl->ev_col[j]);
  return cols;
}

// the row's evidence codes (row rc of the columns at C + row0, leading dimension ldc): e<i>_<u>
// coherent: system-scope relaxed loads (past every non-coherent cache, no invalidation needed) — the
// ring kernel's codes, which may be written after the launch started
static void emit_rows_code_loads(std::string &o, const std::vector<int> &cols, int R, bool coherent) {
  if (!cols.empty()) o += "  const unsigned char *cr = C + row0 + rc;\n";
  for (size_t i = 0; i < cols.size(); ++i) {
    if (R == 1) {
      pgmi_appendf(o, "  const unsigned e%zu_0 = cr[%dLL * ldc];\n", i, cols[i]);
    } else if (coherent) {
      pgmi_appendf(o, "  const unsigned w%zu = __hip_atomic_load((__attribute__((address_space(1))) unsigned short *)(cr + %dLL * ldc), __ATOMIC_RELAXED, "
                   "__HIP_MEMORY_SCOPE_SYSTEM);\n", i, cols[i]);
      pgmi_appendf(o, "  const unsigned e%zu_0 = w%zu & 255u, e%zu_1 = w%zu >> 8;\n", i, i, i, i);
    } else {
      pgmi_appendf(o, "  const unsigned w%zu = *(const unsigned short *)(cr + %dLL * ldc);\n", i, cols[i]);
      pgmi_appendf(o, "  const unsigned e%zu_0 = w%zu & 255u, e%zu_1 = w%zu >> 8;\n", i, i, i, i);
    }
  }
}

// the row's sum-product, normalisation and stores (r, rc, n, M, ldo, MP, G, E, mode, rsM / rsG and the
// loaded codes in scope; VAL(i) = CPT value i); rows past n leave through `leave` ("return" in a grid
// kernel, "break" inside the ring kernel's do-while)
static void emit_rows_compute(std::string &o, const pgm_rows_plan *pl, int R, const std::vector<int> &cols,
                              const char *leave) {
  o += "  unsigned bad = 0u;\n";
  const int NC = pl->n_comp;
  for (int u = 0; u < R; ++u) {
    for (int c = 0; c < NC; ++c) {
      const int lb = pl->comp_loop_begin[c], nq = pl->comp_n_query[c];
      const int fb = pl->comp_fac_begin[c], fe = pl->comp_fac_end[c];
      const int P = nq == 1 ? pl->loop_card[lb] : 1;
      for (int f = fb; f < fe; ++f) {
        pgmi_appendf(o, "  int o%d_%d_%d = %d;\n", c, f - fb, u, pl->fac_base[f]);
        for (int j = pl->fac_ev_begin[f]; j < pl->fac_ev_end[f]; ++j) {
          const int ci = (int)(std::find(cols.begin(), cols.end(), pl->ev_col[j]) - cols.begin());
          const unsigned cd = (unsigned)pl->ev_card[j];
          pgmi_appendf(o, "  { const unsigned x = e%d_%d; bad |= (unsigned)(x >= %uu); o%d_%d_%d += (x >= %uu ? 0 : (int)x) * %d; }\n",
                  ci, u, cd, c, f - fb, u, cd, pl->ev_stride[j]);
        }
      }
      for (int q = 0; q < P; ++q) {
        pgmi_appendf(o, "  const double p%d_%d_%d = ", c, q, u);
        if (fe == fb) o += "1.0";
        for (int f = fb; f < fe; ++f) {
          const int qs = nq == 1 ? pl->fac_stride[f][lb] : 0;
          pgmi_appendf(o, "%sVAL(o%d_%d_%d + %d)", f > fb ? " * " : "", c, f - fb, u, q * qs);
        }
        o += ";\n";
      }
      pgmi_appendf(o, "  const double m%d_%d = p%d_0_%d", c, u, c, u);
      for (int q = 1; q < P; ++q) pgmi_appendf(o, " + p%d_%d_%d", c, q, u);
      o += ";\n";
    }
    pgmi_appendf(o, "  const double z_%d = ", u);
    if (NC == 1) pgmi_appendf(o, "m0_%d", u);
    else {
      o += "1.0";
      for (int c = 0; c < NC; ++c) pgmi_appendf(o, " * m%d_%d", c, u);
    }
    pgmi_appendf(o, ";\n  const bool dead_%d = !(z_%d > 0.0);\n", u, u);
  }
  pgmi_appendf(o, "  if (bad && r < n && E) atomicOr(E, 1);\n  if (r >= n) %s;\n", leave);
  o += "  if (mode & 1) {\n";
  for (int c = 0; c < NC; ++c) {
    const int lb = pl->comp_loop_begin[c], nq = pl->comp_n_query[c];
    if (nq != 1) continue;
    o += "    {";
    for (int u = 0; u < R; ++u)
      pgmi_appendf(o, " const double iv_%d = dead_%d ? __builtin_nan(\"\") : 1.0 / m%d_%d;", u, u, c, u);
    o += "\n";
    for (int q = 0; q < pl->loop_card[lb]; ++q) {
      const int mo = pl->loop_marg_off[lb] + q;
      if (R == 1 && jit_store() == 1)
        pgmi_appendf(o, "      __builtin_nontemporal_store(p%d_%d_0 * iv_0, &M[%dLL * ldo + r]);\n", c, q, mo);
      else if (R == 1 && jit_store() == 2)
        pgmi_appendf(o, "      PGM_WT8(double, &M[%dLL * ldo + r], p%d_%d_0 * iv_0);\n", mo, c, q);
      else if (R == 1)
        pgmi_appendf(o, "      M[%dLL * ldo + r] = p%d_%d_0 * iv_0;\n", mo, c, q);
      else if (jit_store() == 2)
        pgmi_appendf(o, "      PGM_WT16(rsM, %dLL * ldo + r, p%d_%d_0 * iv_0, p%d_%d_1 * iv_1);\n", mo, c, q, c, q);
      else
        pgmi_appendf(o, "      *(double2 *)(M + %dLL * ldo + r) = make_double2(p%d_%d_0 * iv_0, p%d_%d_1 * iv_1);\n",
                mo, c, q, c, q);
    }
    o += "    }\n";
  }
  o += "  }\n  if (mode & 12) {\n";
  for (int u = 0; u < R; ++u) {
    pgmi_appendf(o, "    int m_%d = 0;\n    double mg_%d = 1.0;\n", u, u);
    for (int c = 0; c < NC; ++c) {
      const int lb = pl->comp_loop_begin[c], nq = pl->comp_n_query[c];
      const int P = nq == 1 ? pl->loop_card[lb] : 1;
      const int ms = nq == 1 ? pl->loop_map_stride[lb] : 0;
      o += "    { double b = -1.0, s = -1.0; int bs = 0;\n";
      for (int q = 0; q < P; ++q)
        pgmi_appendf(o, "      if (p%d_%d_%d > b) { s = b; b = p%d_%d_%d; bs = %d; } else if (p%d_%d_%d > s) { s = p%d_%d_%d; }\n",
                c, q, u, c, q, u, q, c, q, u, c, q, u);
      pgmi_appendf(o, "      m_%d += bs * %d;\n", u, ms);
      if (P > 1)
        o += "      const double g = b > 0.0 ? (b - (s < 0.0 ? 0.0 : s)) / b : 0.0;\n";
      else
        o += "      const double g = 1.0;\n";
      pgmi_appendf(o, NC == 1 ? "      mg_%d = g; }\n" : "      mg_%d = fmin(mg_%d, g); }\n", u, u);
    }
  }
  const bool wt = jit_store() == 2;
  if (R == 1 && wt) {
    o += "    if (MP) PGM_WT4(int, &MP[r], dead_0 ? 0 : m_0);\n"
         "    if ((mode & 8) && G) PGM_WT8(double, &G[r], dead_0 ? 0.0 : mg_0);\n  }\n";
  } else if (R == 1) {
    o += "    if (MP) MP[r] = dead_0 ? 0 : m_0;\n    if ((mode & 8) && G) G[r] = dead_0 ? 0.0 : mg_0;\n  }\n";
  } else if (wt) {
    o += "    if (MP) PGM_WT8(unsigned long long, (unsigned long long *)(MP + r), "
         "((unsigned long long)(unsigned)(dead_1 ? 0 : m_1) << 32) | (unsigned)(dead_0 ? 0 : m_0));\n";
    o += "    if ((mode & 8) && G) PGM_WT16(rsG, r, dead_0 ? 0.0 : mg_0, dead_1 ? 0.0 : mg_1);\n  }\n";
  } else {
    o += "    if (MP) *(int2 *)(MP + r) = make_int2(dead_0 ? 0 : m_0, dead_1 ? 0 : m_1);\n";
    o += "    if ((mode & 8) && G) *(double2 *)(G + r) = make_double2(dead_0 ? 0.0 : mg_0, dead_1 ? 0.0 : mg_1);\n  }\n";
  }
}

// ---------------------------------------------------------------------------------------- ring kernel
// pgm_rows_ring: the plan-specialised two-rows-per-thread body run by a RESIDENT grid over a stream of
// row batches (pgm_rows_ring_*).  One launch consumes n_batches batches of n rows; batch b reads and
// writes the buffers of slot b % n_slots (descriptor table D in device memory).  The host publishes
// batches by raising a counter in pinned host memory (ctl[0] = batches posted); the launch may start
// before the first post.  Work item = 128 rows (one wave, two rows per lane) of one batch; item j
// goes to wave j mod W (W = resident waves), so consecutive batches overlap across the chip instead of
// each paying a dispatch.
// Learning that a batch is posted, three levels deep so the host counter sees ONE reader at a time
// (reads of host memory from the GPU are serialised: 768 concurrent first polls cost ~150 us, r03a):
//   1. the count the wave's workgroup last saw (LDS seen_s);
//   2. one wave per workgroup (LDS token) reads the device-memory mirror g[0];
//   3. one wave on the chip (token g[1], agent scope) reads ctl[0] with a system-scope acquire and
//      raises the mirror.
// No acquire fences (an L2 invalidation per workgroup serialises per XCD: ~100 us per launch, r03b):
// the counters are read with relaxed system/agent-scope atomics, and the evidence codes with
// system-scope loads, which go past every non-coherent cache — so codes written (by DMA) after the
// launch started but before their batch was posted are read fresh.  Exit conditions every wave reaches:
// all items done; ctl[1] (cancel) set by the host; or `timeout` ticks of the constant 100 MHz wall
// clock without the needed batch (ctl[2] |= 2); either of the last two raises g[2] (stop) for all.
// The CPT values are staged in LDS once per workgroup for the whole stream.
static void emit_rows_ring(std::string &o, const pgm_rows_plan *pl) {
  const int NV = pl->n_values + 1;
  const int WG = ring_wg();
  const int K = (NV + WG - 1) / WG;
  pgmi_appendf(o, "#define BACKOFF %d\n", ring_backoff() ? 1 : 0);
  o += "struct pgm_ring_slot { const unsigned char *C; long long ldc, row0; double *M; long long ldo; int *MP; "
       "double *G; long long pad; };\n";
  pgmi_appendf(o, "extern \"C\" __global__ void __launch_bounds__(%d) pgm_rows_ring(const double *__restrict__ V, "
             "const pgm_ring_slot *__restrict__ D, unsigned n_slots, unsigned *ctl, unsigned *g, unsigned n_batches, "
             "unsigned base, long long n, int *__restrict__ E, int mode, unsigned long long timeout, int signal) {\n", WG);
  o += "  const int t = threadIdx.x;\n";
  pgmi_appendf(o, "  __shared__ double S[%d];\n  __shared__ unsigned seen_s, token_s, stop_s;\n", K * WG);
  for (int i = 0; i < K; ++i) pgmi_appendf(o, "  const double s%d = V[t + %d < %d ? t + %d : %d];\n", i, WG * i, NV, WG * i, NV - 1);
  for (int i = 0; i < K; ++i) pgmi_appendf(o, "  S[t + %d < %d ? t + %d : %d] = s%d;\n", WG * i, NV, WG * i, NV - 1, i);
  o += "  if (t == 0) { seen_s = base; token_s = 0u; stop_s = 0u; }\n  __syncthreads();\n#define VAL(i) S[i]\n";
  // readiness (pgm_rows_ring_wait_ready): every workgroup counts itself in g[4..5] (64-bit, never reset:
  // each launch adds exactly gridDim.x) once its CPT copy is staged; the last one raises ctl[3] for the host
  o += "  if (signal && t == 0) {\n"
       "    const unsigned long long s = atomicAdd((unsigned long long *)(g + 4), 1ull) + 1ull;\n"
       "    if (s % gridDim.x == 0ull) __hip_atomic_store(&ctl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);\n"
       "  }\n";
  pgmi_appendf(o, "  const unsigned long long W = (unsigned long long)gridDim.x * %d;\n", WG / 64);
  pgmi_appendf(o, "  const unsigned long long wv0 = (unsigned long long)blockIdx.x * %d + (t >> 6);\n", WG / 64);
  o += "  const unsigned long long chunks = (unsigned long long)(n + 127) / 128;\n"
       "  const unsigned long long items = chunks * n_batches;\n"
       "  const unsigned long long t0 = wall_clock64();\n"
       "  const bool lead = (t & 63) == 0;\n"
       "  unsigned seen = base;  /* counts are absolute over the ring's lifetime */\n"
       "  for (unsigned long long j = wv0; j < items; j += W) {\n"
       "    const unsigned bt = (unsigned)(j / chunks);\n"
       "    const unsigned ab = base + bt;  /* the batch's absolute number: posted once ctl[0] > ab */\n"
       "    bool stop = false;\n"
       "    while (ab >= seen) {\n"
       "      const unsigned sl = __hip_atomic_load(&seen_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n"
       "      if (sl > seen) { seen = sl; continue; }\n"
       "      if (__hip_atomic_load(&stop_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) { stop = true; break; }\n"
       "      unsigned mine = 0u;\n"
       "      if (lead) mine = atomicCAS(&token_s, 0u, 1u) == 0u ? 1u : 0u;\n"
       "      mine = __builtin_amdgcn_readfirstlane(mine);\n"
       "      if (!mine) {\n"
       "        if (wall_clock64() - t0 > timeout) { stop = true; break; }\n"
       "        __builtin_amdgcn_s_sleep(2);\n"
       "        continue;\n"
       "      }\n"
       "      unsigned nap = 0u;\n"
       "      for (;;) {  /* this wave speaks for its workgroup */\n"
       "        unsigned m = __hip_atomic_load(&g[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
       "        if (m <= ab) {\n"
       "          if (__hip_atomic_load(&g[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { stop = true; break; }\n"
       "          unsigned poll = 0u;\n"
       "          if (lead && (!BACKOFF || __hip_atomic_load(&g[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u))\n"
       "            poll = atomicCAS(&g[1], 0u, 1u) == 0u ? 1u : 0u;\n"
       "          poll = __builtin_amdgcn_readfirstlane(poll);\n"
       "          if (poll) {  /* the one reader of the host counter */\n"
       "            const unsigned p = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);\n"
       "            if (p > m && lead) __hip_atomic_fetch_max(&g[0], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
       "            if (p > m) m = p;\n"
       "            if (m <= ab) {\n"
       "              const bool cancel = __hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;\n"
       "              const bool late = wall_clock64() - t0 > timeout;\n"
       "              if ((cancel || late) && lead) {\n"
       "                if (late) __hip_atomic_fetch_or(&ctl[2], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);\n"
       "                __hip_atomic_store(&g[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
       "              }\n"
       "              stop = cancel || late;\n"
       "            }\n"
       "            if (lead) __hip_atomic_store(&g[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
       "            if (stop) break;\n"
       "          } else if (wall_clock64() - t0 > timeout) {\n"
       "            stop = true;\n"
       "            break;\n"
       "          }\n"
       "        }\n"
       "        if (m > ab) {\n"
       "          seen = m;\n"
       "          if (lead) atomicMax(&seen_s, m);\n"
       "          break;\n"
       "        }\n"
       "        if (!BACKOFF || ++nap <= 2u) __builtin_amdgcn_s_sleep(4);\n"
       "        else if (nap <= 8u) __builtin_amdgcn_s_sleep(12);\n"
       "        else __builtin_amdgcn_s_sleep(32);\n"
       "      }\n"
       "      if (stop && lead) atomicExch(&stop_s, 1u);\n"
       "      if (lead) atomicExch(&token_s, 0u);\n"
       "      if (stop) break;\n"
       "    }\n"
       "    if (stop) break;\n"
       "    const pgm_ring_slot d = D[bt % n_slots];\n"
       "    const unsigned char *__restrict__ C = d.C;\n"
       "    const long long ldc = d.ldc, row0 = d.row0, ldo = d.ldo;\n"
       "    double *__restrict__ M = d.M;\n"
       "    int *__restrict__ MP = d.MP;\n"
       "    double *__restrict__ G = d.G;\n"
       "    const long long r = (long long)(j - (unsigned long long)bt * chunks) * 128 + (t & 63) * 2;\n"
       "    const long long rc = r < n ? r : n - 2;\n";
  if (jit_store() == 2)
    o += "    const __amdgpu_buffer_rsrc_t rsM = __builtin_amdgcn_make_buffer_rsrc(M, 0, 0x7fffffff, 0x00020000);\n"
         "    const __amdgpu_buffer_rsrc_t rsG = __builtin_amdgcn_make_buffer_rsrc(G, 0, 0x7fffffff, 0x00020000);\n";
  o += "    do {\n";
  const std::vector<int> cols = rows_cols(pl);
  emit_rows_code_loads(o, cols, 2, true);
  emit_rows_compute(o, pl, 2, cols, "break");
  o += "    } while (0);\n  }\n}\n#undef VAL\n";
}

// the dispatch floor of a plan (PGM_ROWS_FLOOR, measurement only): the row kernel's grid (R rows per
// thread, as pgm_rows_jit / pgm_rows_jit2), its evidence-column loads and its output stores (same
// addresses, same widths, same cache policy), with the CPT staging, gathers and arithmetic replaced by
// one conversion of the loaded codes
static void emit_rows_floor(std::string &o, const pgm_rows_plan *pl, int R) {
  const int WG = jit_wg();
  const bool wt = jit_store() == 2;
  pgmi_appendf(o, "extern \"C\" __global__ void __launch_bounds__(%d) pgm_rows_floor%s(const double *__restrict__ V, "
             "const unsigned char *__restrict__ C, long long ldc, long long row0, long long n, "
             "double *__restrict__ M, long long ldo, int *__restrict__ MP, double *__restrict__ G, "
             "int *__restrict__ E, int mode) {\n", WG, R == 2 ? "2" : "");
  pgmi_appendf(o, "  const long long r = ((long long)blockIdx.x * %d + threadIdx.x) * %d;\n  if (r >= n) return;\n", WG, R);
  if (R == 2 && wt)
    o += "  const __amdgpu_buffer_rsrc_t rsM = __builtin_amdgcn_make_buffer_rsrc(M, 0, 0x7fffffff, 0x00020000);\n"
         "  const __amdgpu_buffer_rsrc_t rsG = __builtin_amdgcn_make_buffer_rsrc(G, 0, 0x7fffffff, 0x00020000);\n";
  std::vector<int> cols;
  for (int j = 0; j < pl->n_ev; ++j)
    if (std::find(cols.begin(), cols.end(), pl->ev_col[j]) == cols.end()) cols.push_back(pl->ev_col[j]);
  o += "  unsigned x = 0u;\n";
  if (!cols.empty()) o += "  const unsigned char *cr = C + row0 + r;\n";
  for (size_t i = 0; i < cols.size(); ++i) {
    if (R == 1) pgmi_appendf(o, "  x += cr[%dLL * ldc];\n", cols[i]);
    else pgmi_appendf(o, "  x += *(const unsigned short *)(cr + %dLL * ldc);\n", cols[i]);
  }
  o += "  const double v = (double)x;\n  if (mode & 1) {\n";
  for (int c = 0; c < pl->n_comp; ++c) {
    const int lb = pl->comp_loop_begin[c];
    if (pl->comp_n_query[c] != 1) continue;
    for (int q = 0; q < pl->loop_card[lb]; ++q) {
      const int mo = pl->loop_marg_off[lb] + q;
      if (R == 2 && wt) pgmi_appendf(o, "    PGM_WT16(rsM, %dLL * ldo + r, v, v);\n", mo);
      else if (R == 2) pgmi_appendf(o, "    *(double2 *)(M + %dLL * ldo + r) = make_double2(v, v);\n", mo);
      else if (wt) pgmi_appendf(o, "    PGM_WT8(double, &M[%dLL * ldo + r], v);\n", mo);
      else pgmi_appendf(o, "    M[%dLL * ldo + r] = v;\n", mo);
    }
  }
  o += "  }\n  if (mode & 12) {\n";
  if (R == 2 && wt)
    o += "    if (MP) PGM_WT8(unsigned long long, (unsigned long long *)(MP + r), (unsigned long long)x);\n"
         "    if ((mode & 8) && G) PGM_WT16(rsG, r, v, v);\n  }\n}\n";
  else if (R == 2)
    o += "    if (MP) *(int2 *)(MP + r) = make_int2((int)x, (int)x);\n"
         "    if ((mode & 8) && G) *(double2 *)(G + r) = make_double2(v, v);\n  }\n}\n";
  else if (wt)
    o += "    if (MP) PGM_WT4(int, &MP[r], (int)x);\n    if ((mode & 8) && G) PGM_WT8(double, &G[r], v);\n  }\n}\n";
  else
    o += "    if (MP) MP[r] = (int)x;\n    if ((mode & 8) && G) G[r] = v;\n  }\n}\n";
}

static std::string rows_jit_source(const pgm_rows_plan *pl) {
  // write-through stores: 4/8 B as relaxed agent-scope atomic stores (global_store ... sc1), 16 B as
  // a buffer store with the sc1 cache bit (element offset into the resource's base, bytes < 2 GiB)
  std::string o =
      "typedef unsigned int pgm_u32x4 __attribute__((ext_vector_type(4)));\n"
      "#define PGM_WT4(T, p, v) __hip_atomic_store((__attribute__((address_space(1))) T *)(p), (v), "
      "__ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)\n"
      "#define PGM_WT8(T, p, v) PGM_WT4(T, p, v)\n"
      "#define PGM_WT16(rs, off, a, b) do { const double2 v_ = make_double2((a), (b)); pgm_u32x4 w_; "
      "__builtin_memcpy(&w_, &v_, 16); __builtin_amdgcn_raw_buffer_store_b128(w_, rs, (int)((off) * 8), 0, 16); } "
      "while (0)\n";
  emit_rows_kernel(o, pl, 1);
  o += "\n";
  emit_rows_kernel(o, pl, 2);
  o += "\n";
  emit_rows_floor(o, pl, 1);
  o += "\n";
  emit_rows_floor(o, pl, 2);
  o += "\n";
  emit_rows_ring(o, pl);
  return o;
}

static bool rows2_aligned(int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0, int64_t n_rows,
                          const double *marg, int64_t ld_out, const int32_t *map, const double *gap, int n_marg);

// whether a launch runs the two-rows-per-thread kernel: big enough, and its alignment contract holds
// (else the one-row kernel runs)
static bool rows_jit2_ok(int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0, int64_t n_rows,
                         const double *marg, int64_t ld_out, const int32_t *map, const double *gap, int n_marg) {
  // measured (MI355X): two rows with 16-B stores once the launch is HBM-bound (4M rows: 110 vs 126 us)
  // and, since the 512-thread workgroups and concurrent queues, at 100k rows too (one queue: equal,
  // 3.9 us; four queues: 2.7 -> 2.1 us per launch of GPU span, r02br); one row below 50k rows
  static constexpr int64_t min_rows = 50000;
  if (n_rows < min_rows) return false;
  return rows2_aligned(mode, codes, ld_codes, row0, n_rows, marg, ld_out, map, gap, n_marg);
}

// the alignment / addressing contract of the two-rows-per-lane body (pgm_rows_jit2, pgm_rows_ring)
static bool rows2_aligned(int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0, int64_t n_rows,
                          const double *marg, int64_t ld_out, const int32_t *map, const double *gap, int n_marg) {
  if (n_rows % 2 || ld_codes % 2 || row0 % 2 || ((uintptr_t)codes & 1)) return false;
  if ((mode & PGM_ROWS_MARGINALS) && (((uintptr_t)marg & 15) || ld_out % 2)) return false;
  if (map && ((uintptr_t)map & 7)) return false;
  if ((mode & PGM_ROWS_MAPGAP) && gap && ((uintptr_t)gap & 15)) return false;
  // the write-through 16-B stores address outputs as 32-bit byte offsets below 2 GiB
  if (jit_store() == 2 && (mode & PGM_ROWS_MARGINALS) && (uint64_t)(n_marg + 1) * (uint64_t)ld_out * 8 >= (1ull << 31))
    return false;
  if (jit_store() == 2 && (uint64_t)n_rows * 8 >= (1ull << 31)) return false;
  return true;
}


// compile + load the handle's specialised kernel once; false when unavailable (AOT kernels run)
static bool rows_jit_ready(RowsHandle *h) {
  if (h->jit_src.empty()) return false;
  std::lock_guard<std::mutex> lk(h->jit_mu);
  if (h->jit_state != 0) return h->jit_state > 0;
  h->jit_state = -1;
  static const bool disabled = getenv("PGM_NO_JIT") != nullptr;  // testing: AOT kernels only
  if (disabled) return false;
  std::vector<char> code;
  if (!pgmi_rtc_code(h->jit_src, "specialised row kernel", code)) return false;
  h->jit_code = code;
  if (hipModuleLoadData(&h->jit_mod, code.data()) != hipSuccess) {
    (void)hipGetLastError();
    h->jit_mod = nullptr;
    return false;
  }
  if (hipModuleGetFunction(&h->jit_fn, h->jit_mod, "pgm_rows_jit") != hipSuccess ||
      hipModuleGetFunction(&h->jit_fn2, h->jit_mod, "pgm_rows_jit2") != hipSuccess ||
      hipModuleGetFunction(&h->jit_fn_floor, h->jit_mod, "pgm_rows_floor") != hipSuccess ||
      hipModuleGetFunction(&h->jit_fn_floor2, h->jit_mod, "pgm_rows_floor2") != hipSuccess ||
      hipModuleGetFunction(&h->jit_fn_ring, h->jit_mod, "pgm_rows_ring") != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  h->jit_state = 1;
  return true;
}

// ============================================================================= C-ABI
extern "C" {

int pgm_version(void) { return PGM_ABI_VERSION; }

int pgm_last_error(char *buf, size_t len) {
  if (!buf || len == 0) return PGM_EINVAL;
  size_t n = std::min(len - 1, g_err.size());
  memcpy(buf, g_err.data(), n);
  buf[n] = 0;
  return PGM_OK;
}

int pgm_device_count(int *n) {
  STALE_PROBE();
  if (!n) return fail(PGM_EINVAL, "null pointer");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *n = 0;
    return fail(PGM_EDEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *n = c;
  return PGM_OK;
}

int pgm_set_device(int device) {
  STALE_PROBE();
  HIP_TRY(hipSetDevice(device));
  return PGM_OK;
}

int pgm_alloc(void **ptr, size_t bytes) {
  STALE_PROBE();
  if (!ptr) return fail(PGM_EINVAL, "null pointer");
  *ptr = nullptr;
  if (bytes == 0) return PGM_OK;
  HIP_TRY(hipMalloc(ptr, bytes));
  return PGM_OK;
}

int pgm_free(void *ptr) {
  STALE_PROBE();
  if (ptr) HIP_TRY(hipFree(ptr));
  return PGM_OK;
}

int pgm_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
  STALE_PROBE();
  if (bytes == 0) return PGM_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, S(stream)));
  return PGM_OK;
}

int pgm_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
  STALE_PROBE();
  if (bytes == 0) return PGM_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, S(stream)));
  HIP_TRY(hipStreamSynchronize(S(stream)));
  return PGM_OK;
}

int pgm_memcpy_d2h_async(void *dst, const void *src, size_t bytes, void *stream) {
  STALE_PROBE();
  if (bytes == 0) return PGM_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, S(stream)));
  return PGM_OK;
}

int pgm_memcpy_d2d(void *dst, const void *src, size_t bytes, void *stream) {
  STALE_PROBE();
  if (bytes == 0) return PGM_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, S(stream)));
  return PGM_OK;
}

int pgm_host_alloc(void **ptr, size_t bytes) {
  STALE_PROBE();
  if (!ptr) return fail(PGM_EINVAL, "host_alloc: null pointer");
  *ptr = nullptr;
  if (bytes == 0) bytes = 1;
  const hipError_t e = hipHostMalloc(ptr, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *ptr = nullptr;
    return fail(e == hipErrorOutOfMemory ? PGM_ENOMEM : PGM_EDEVICE, "host_alloc: %s", hipGetErrorString(e));
  }
  memset(*ptr, 0, bytes);
  return PGM_OK;
}

int pgm_host_free(void *ptr) {
  STALE_PROBE();
  if (ptr) HIP_TRY(hipHostFree(ptr));
  return PGM_OK;
}

int pgm_memset(void *dst, int value, size_t bytes, void *stream) {
  STALE_PROBE();
  if (bytes == 0) return PGM_OK;
  HIP_TRY(hipMemsetAsync(dst, value, bytes, S(stream)));
  return PGM_OK;
}

int pgm_stream_sync(void *stream) {
  STALE_PROBE();
  HIP_TRY(hipStreamSynchronize(S(stream)));
  return PGM_OK;
}

// the same wait by polling the stream (hipStreamQuery in a loop): no blocking wait's wake-up latency, one
// host core busy meanwhile — for latency-bound single queries (C2: 0.223 -> 0.210 ms/query, r03ab)
int pgm_stream_sync_spin(void *stream) {
  STALE_PROBE();
  hipError_t e;
  while ((e = hipStreamQuery(S(stream))) == hipErrorNotReady) {
  }
  HIP_TRY(e);
  return PGM_OK;
}

int pgm_event_create(void **ev) {
  STALE_PROBE();
  if (!ev) return fail(PGM_EINVAL, "null pointer");
  hipEvent_t e;
  HIP_TRY(hipEventCreate(&e));
  *ev = (void *)e;
  return PGM_OK;
}

int pgm_event_destroy(void *ev) {
  STALE_PROBE();
  if (ev) HIP_TRY(hipEventDestroy((hipEvent_t)ev));
  return PGM_OK;
}

int pgm_event_record(void *ev, void *stream) {
  STALE_PROBE();
  HIP_TRY(hipEventRecord((hipEvent_t)ev, S(stream)));
  return PGM_OK;
}

int pgm_event_elapsed_ms(void *start, void *stop, float *ms) {
  STALE_PROBE();
  HIP_TRY(hipEventSynchronize((hipEvent_t)stop));
  HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return PGM_OK;
}

int pgm_contract_workspace(const pgm_contract_desc *d, size_t *bytes) {
  STALE_PROBE();
  if (!bytes) return fail(PGM_EINVAL, "null pointer");
  ContractLaunch L;
  int rc = plan_contract(d, L);
  if (rc) return rc;
  *bytes = L.ws_doubles * sizeof(double);
  return PGM_OK;
}

int pgm_contract(const pgm_contract_desc *d, const double *A, const double *B, double *C, void *workspace,
                 size_t workspace_bytes, void *stream) {
  STALE_PROBE();
  ContractLaunch L;
  int rc = plan_contract(d, L);
  if (rc) return rc;
  if (L.empty) return PGM_OK;
  if (!A || !C) return fail(PGM_EINVAL, "contract: null A or C");
  if (d->combine != PGM_COMBINE_COPY && !B) return fail(PGM_EINVAL, "contract: null B for a binary combine");
  if (L.ws_doubles * sizeof(double) > workspace_bytes || (L.ws_doubles && !workspace))
    return fail(PGM_EINVAL, "contract: workspace of %zu bytes needed, %zu given",
                (size_t)(L.ws_doubles * sizeof(double)), workspace_bytes);
  double *ws = (double *)workspace;
  hipStream_t s = S(stream);
  switch (d->combine) {
    case PGM_COMBINE_MUL: launch_contract_c<PGM_COMBINE_MUL>(d->reduce, L, A, B, C, ws, s); break;
    case PGM_COMBINE_ADD: launch_contract_c<PGM_COMBINE_ADD>(d->reduce, L, A, B, C, ws, s); break;
    case PGM_COMBINE_DIV: launch_contract_c<PGM_COMBINE_DIV>(d->reduce, L, A, B, C, ws, s); break;
    case PGM_COMBINE_DIV_RAW: launch_contract_c<PGM_COMBINE_DIV_RAW>(d->reduce, L, A, B, C, ws, s); break;
    default: launch_contract_c<PGM_COMBINE_COPY>(d->reduce, L, A, B, C, ws, s); break;
  }
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

}  // extern "C"

// descriptor -> kernel parameters (coalesced dims, aliased unused operand slots); shared by
// pgm_product_n and the batched product_n job
static int plan_prodn(const pgm_productn_desc *d, const double *const *ops, ProdNK &k) {
  if (!d || !ops) return fail(PGM_EINVAL, "product_n: null argument");
  if (d->n_ops < 1 || d->n_ops > PMAX || d->n_keep < 0 || d->n_keep > PGM_MAX_DIMS)
    return fail(PGM_EINVAL, "product_n: n_ops %d (1..%d) / n_keep %d", d->n_ops, PMAX, d->n_keep);
  // coalesce: one Dims per group of up to 3 operand strides is not enough -> do it by hand
  int n = 0;
  int64_t card[PGM_MAX_DIMS], sc[PGM_MAX_DIMS], so[PMAX][PGM_MAX_DIMS];
  uint64_t n_out = 1;
  for (int i = 0; i < d->n_keep; ++i) {
    if (d->keep_card[i] <= 0) return fail(PGM_EINVAL, "product_n: keep_card[%d] <= 0", i);
    n_out *= (uint64_t)d->keep_card[i];
    if (d->keep_card[i] == 1) continue;
    if (n > 0) {
      bool ok = sc[n - 1] == d->keep_card[i] * d->keep_sc[i];
      for (int t = 0; t < d->n_ops; ++t) ok = ok && so[t][n - 1] == d->keep_card[i] * d->keep_s[t][i];
      if (ok) {
        card[n - 1] *= d->keep_card[i];
        sc[n - 1] = d->keep_sc[i];
        for (int t = 0; t < d->n_ops; ++t) so[t][n - 1] = d->keep_s[t][i];
        continue;
      }
    }
    card[n] = d->keep_card[i];
    sc[n] = d->keep_sc[i];
    for (int t = 0; t < d->n_ops; ++t) so[t][n] = d->keep_s[t][i];
    ++n;
  }
  if (n_out >= (1ull << 31)) return fail(PGM_EINVAL, "product_n: output too large");
  if (n > KMAX) return fail(PGM_EINVAL, "product_n: %d dims after coalescing (limit %d)", n, KMAX);
  memset(&k, 0, sizeof k);
  k.n_ops = d->n_ops;
  k.nk = n;
  k.n_out = (uint32_t)n_out;
  for (int i = 0; i < n; ++i) {
    k.kdiv[i] = make_fdiv((uint32_t)card[i]);
    k.ksc[i] = sc[i];
    for (int t = 0; t < d->n_ops; ++t) k.ks[t][i] = so[t][i];
  }
  for (int t = 0; t < d->n_ops; ++t) {
    if (!ops[t]) return fail(PGM_EINVAL, "product_n: null operand %d", t);
    k.ops[t] = ops[t];
    k.kind[t] = d->op_kind[t];
    if (d->op_kind[t] < 0 || d->op_kind[t] > 2) return fail(PGM_EINVAL, "product_n: bad op_kind[%d]", t);
    if (d->op_kind[t] == PGM_PRODN_RATIO && (t + 1 >= d->n_ops || d->op_kind[t + 1] != PGM_PRODN_DEN))
      return fail(PGM_EINVAL, "product_n: a RATIO operand must be followed by its DEN operand");
    if (d->op_kind[t] == PGM_PRODN_DEN && (t == 0 || d->op_kind[t - 1] != PGM_PRODN_RATIO))
      return fail(PGM_EINVAL, "product_n: a DEN operand must follow a RATIO operand");
  }
  for (int t = d->n_ops; t < PMAX; ++t) {  // unused slots alias operand 0 with stride 0 (valid loads)
    k.ops[t] = k.ops[0];
    k.kind[t] = PGM_PRODN_MUL;
    for (int i = 0; i < n; ++i) k.ks[t][i] = 0;
  }
  const uint64_t NX = n > 0 ? (uint64_t)card[n - 1] : 1;
  k.row_mode = (n > 0 && NX >= 64) ? 1 : 0;
  return PGM_OK;
}

extern "C" {

int pgm_product_n(const pgm_productn_desc *d, const double *const *ops, double *C, void *stream) {
  STALE_PROBE();
  if (!d || !ops || !C) return fail(PGM_EINVAL, "product_n: null argument");
  ProdNK k;
  const int prc = plan_prodn(d, ops, k);
  if (prc != PGM_OK) return prc;
  const int n = k.nk;
  const uint64_t n_out = k.n_out;
  const uint64_t NX = n > 0 ? (uint64_t)k.kdiv[n - 1].d : 1;
  const int64_t *sc = k.ksc;
  // two rows per lane when every access is 16-B aligned (batched BP: rows innermost, even count)
  bool rows2 = k.row_mode && (NX % 2 == 0) && sc[n - 1] == 1 && ((uintptr_t)C & 15) == 0 && !g_no_rows2;
  for (int i = 0; rows2 && i < n - 1; ++i) rows2 = (sc[i] % 2) == 0;
  for (int t = 0; rows2 && t < d->n_ops; ++t) {
    const int64_t sx = k.ks[t][n - 1];
    rows2 = sx == 0 || (sx == 1 && ((uintptr_t)ops[t] & 15) == 0);
    for (int i = 0; rows2 && sx == 1 && i < n - 1; ++i) rows2 = (k.ks[t][i] % 2) == 0;
  }
  dim3 grid;
  if (rows2) {
    const uint64_t NP = NX / 2, n_outer = n_out / NX;
    const uint64_t bs = std::min<uint64_t>(256, (NP + 63) / 64 * 64);
    const uint64_t gy = std::min<uint64_t>(n_outer, 65535);
    const uint64_t gx = std::min<uint64_t>((NP + bs - 1) / bs, std::max<uint64_t>(1, 2048 / gy));
    hipStream_t s = S(stream);
    const dim3 g2((unsigned)gx, (unsigned)gy, 1), b2((unsigned)bs);
    switch (d->n_ops <= 2 ? 2 : d->n_ops <= 4 ? 4 : 8) {
      case 2: hipLaunchKernelGGL((k_productn_rows2<2>), g2, b2, 0, s, k, C); break;
      case 4: hipLaunchKernelGGL((k_productn_rows2<4>), g2, b2, 0, s, k, C); break;
      default: hipLaunchKernelGGL((k_productn_rows2<8>), g2, b2, 0, s, k, C); break;
    }
    HIP_TRY(hipGetLastError());
    return PGM_OK;
  }
  if (k.row_mode) {
    const uint64_t xchunks = (NX + 255) / 256, n_outer = n_out / NX;
    const uint64_t gy = std::min<uint64_t>(n_outer, 65535);
    const uint64_t gx = std::min<uint64_t>(xchunks, std::max<uint64_t>(1, 2048 / gy));
    grid = dim3((unsigned)gx, (unsigned)gy, 1);
  } else {
    grid = dim3((unsigned)std::min<uint64_t>(std::max<uint64_t>((n_out + 255) / 256, 1), 65535), 1, 1);
  }
  hipStream_t s = S(stream);
  switch (d->n_ops <= 2 ? 2 : d->n_ops <= 4 ? 4 : 8) {
    case 2: hipLaunchKernelGGL((k_productn<2>), grid, dim3(256), 0, s, k, C); break;
    case 4: hipLaunchKernelGGL((k_productn<4>), grid, dim3(256), 0, s, k, C); break;
    default: hipLaunchKernelGGL((k_productn<8>), grid, dim3(256), 0, s, k, C); break;
  }
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_product_n_marginal_ok(const pgm_productn_desc *d, const double *const *ops, const double *C,
                              const int64_t *marg_s, const double *M) {
  STALE_PROBE();
  ProdMK k;
  dim3 g;
  return pgmi_plan_product_marg(d, ops, C, marg_s, M, k, g) == 1 ? 1 : 0;
}

int pgm_product_n_marginal(const pgm_productn_desc *d, const double *const *ops, double *C, const int64_t *marg_s,
                           int32_t reduce, double *M, void *stream) {
  STALE_PROBE();
  if (reduce != PGM_RED_SUM && reduce != PGM_RED_MAX)
    return fail(PGM_EINVAL, "product_n_marginal: reduce must be PGM_RED_SUM or PGM_RED_MAX");
  ProdMK k;
  dim3 g;
  const int r = pgmi_plan_product_marg(d, ops, C, marg_s, M, k, g);
  if (r < 0) return r;
  if (r == 0)
    return fail(PGM_EINVAL, "product_n_marginal: shape not supported by the fused kernel "
                            "(pgm_product_n_marginal_ok is 0: run pgm_product_n + pgm_contract)");
  hipStream_t s = S(stream);
  const bool two = k.n_ops <= 2;
  // j-outer form: 2 row pairs per lane from 1,024 row pairs up, else 1 (MI355X, pathfinder's largest
  // clique: collect 413 -> 272 us at 4,000 rows, 94 -> 80 us at 1,000, against r02's j-inner kernel)
  const int XI = k.NP >= 1024 ? 2 : 1;
  const uint64_t gxj = (k.NP + 256ull * XI - 1) / (256ull * XI);
  const dim3 gj((unsigned)gxj, g.y, 1);
#define PGM_MARGJ_NOPS(NO, XX)                                                                               \
  if (reduce == PGM_RED_SUM) hipLaunchKernelGGL((k_productn_marg_jx<NO, PGM_RED_SUM, XX>), gj, dim3(256), 0, s, k, C, M); \
  else hipLaunchKernelGGL((k_productn_marg_jx<NO, PGM_RED_MAX, XX>), gj, dim3(256), 0, s, k, C, M);
#define PGM_MARGJ_LAUNCH(XX)                                                                                 \
  if (two) {                                                                                                 \
    PGM_MARGJ_NOPS(2, XX)                                                                                    \
  } else if (k.n_ops <= 4) {                                                                                 \
    PGM_MARGJ_NOPS(4, XX)                                                                                    \
  } else {                                                                                                   \
    PGM_MARGJ_NOPS(MOPS, XX)                                                                                 \
  }
  if (XI == 2) {
    PGM_MARGJ_LAUNCH(2)
  } else {
    PGM_MARGJ_LAUNCH(1)
  }
#undef PGM_MARGJ_LAUNCH
#undef PGM_MARGJ_NOPS
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_graph_capture_begin(void *stream) {
  STALE_PROBE();
  if (!stream) return fail(PGM_EINVAL, "graph capture needs a non-default stream");
  HIP_TRY(hipStreamBeginCapture(S(stream), hipStreamCaptureModeRelaxed));
  return PGM_OK;
}

int pgm_graph_capture_end(void *stream, void **graph_exec) {
  STALE_PROBE();
  if (!graph_exec) return fail(PGM_EINVAL, "null pointer");
  hipGraph_t g = nullptr;
  HIP_TRY(hipStreamEndCapture(S(stream), &g));
  hipGraphExec_t e = nullptr;
  hipError_t err = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (err != hipSuccess) {
    (void)hipGetLastError();
    return fail(PGM_EDEVICE, "hipGraphInstantiate: %s", hipGetErrorString(err));
  }
  *graph_exec = (void *)e;
  return PGM_OK;
}

int pgm_graph_launch(void *graph_exec, void *stream) {
  STALE_PROBE();
  if (!graph_exec) return fail(PGM_EINVAL, "null graph");
  HIP_TRY(hipGraphLaunch((hipGraphExec_t)graph_exec, S(stream)));
  return PGM_OK;
}

int pgm_graph_destroy(void *graph_exec) {
  STALE_PROBE();
  if (graph_exec) HIP_TRY(hipGraphExecDestroy((hipGraphExec_t)graph_exec));
  return PGM_OK;
}

}  // extern "C"

static int plan_gather(const pgm_gather_desc *d, GatherK &k) {
  if (d->n_keep < 0 || d->n_keep > KMAX || d->n_ev < 0 || d->n_ev > PGM_MAX_DIMS)
    return fail(PGM_EINVAL, "gather: n_keep %d (limit %d) / n_ev %d", d->n_keep, KMAX, d->n_ev);
  if (d->batch_dim >= d->n_keep) return fail(PGM_EINVAL, "gather: batch_dim out of range");
  memset(&k, 0, sizeof k);
  k.nk = d->n_keep;
  k.n_ev = d->n_ev;
  k.batch_dim = d->batch_dim;
  k.ld = d->ld;
  k.row0 = d->row0;
  uint64_t n_out = 1;
  for (int i = 0; i < d->n_keep; ++i) {
    if (d->keep_card[i] <= 0) return fail(PGM_EINVAL, "gather: keep_card[%d] <= 0", i);
    n_out *= (uint64_t)d->keep_card[i];
    k.kdiv[i] = make_fdiv((uint32_t)d->keep_card[i]);
    k.ksa[i] = d->keep_sa[i];
    k.ksc[i] = d->keep_sc[i];
  }
  if (n_out >= (1ull << 31)) return fail(PGM_EINVAL, "gather: output too large");
  for (int j = 0; j < d->n_ev; ++j) {
    k.ev_col[j] = d->ev_col[j];
    k.ev_stride[j] = d->ev_stride[j];
    k.ev_card[j] = (int32_t)d->ev_card[j];
  }
  k.n_out = (uint32_t)n_out;
  return PGM_OK;
}

struct BatchHandle {
  std::vector<BatchJob> jobs;
  std::vector<uint32_t> block_job;
  std::vector<uint32_t> level_off{0};  // single-workgroup levelled batch: first block of each level (+ the end)
  BatchJob *d_jobs = nullptr;
  uint32_t *d_map = nullptr;
  uint32_t *d_level = nullptr;
  int32_t mode = PGM_BATCH_GRID;  // PGM_BATCH_ONE_WORKGROUP: k_batch_wg_c
  int32_t spec = -1;  // every job a contraction with one (combine, reduce): combine * 3 + reduce; products: 100
  ChainJob *d_chain = nullptr;  // ONE_WORKGROUP batch (contractions only): descriptors staged in LDS
  size_t chain_lds = 0;         // dynamic LDS bytes of k_batch_wg_c
  // r06: n-ary contraction jobs (kind 4; BatchJob::_pad indexes these): specialised kernel only
  std::vector<ContractNK> njobs;
  std::vector<std::vector<const double *>> nops;
};

static const int32_t kBatchSpecProducts = 100;  // BatchHandle::spec of a products-only batch
// single-workgroup chains of contractions: descriptors, block map and level table staged in LDS
// (k_batch_wg_c) up to this many bytes
static const size_t kChainLdsMax = 48 * 1024;

template <int CMB>
static void launch_batch_cr(int red, dim3 g, hipStream_t s, const BatchJob *jobs, const uint32_t *map) {
  switch (red) {
    case PGM_RED_NONE: hipLaunchKernelGGL((k_batch_c<CMB, PGM_RED_NONE>), g, dim3(256), 0, s, jobs, map); break;
    case PGM_RED_SUM: hipLaunchKernelGGL((k_batch_c<CMB, PGM_RED_SUM>), g, dim3(256), 0, s, jobs, map); break;
    default: hipLaunchKernelGGL((k_batch_c<CMB, PGM_RED_MAX>), g, dim3(256), 0, s, jobs, map); break;
  }
}

static void launch_batch_c(int spec, dim3 g, hipStream_t s, const BatchJob *jobs, const uint32_t *map) {
  const int red = spec % 3;
  switch (spec / 3) {
    case PGM_COMBINE_MUL: launch_batch_cr<PGM_COMBINE_MUL>(red, g, s, jobs, map); break;
    case PGM_COMBINE_ADD: launch_batch_cr<PGM_COMBINE_ADD>(red, g, s, jobs, map); break;
    case PGM_COMBINE_DIV: launch_batch_cr<PGM_COMBINE_DIV>(red, g, s, jobs, map); break;
    case PGM_COMBINE_DIV_RAW: launch_batch_cr<PGM_COMBINE_DIV_RAW>(red, g, s, jobs, map); break;
    default: launch_batch_cr<PGM_COMBINE_COPY>(red, g, s, jobs, map); break;
  }
}

// a batch contraction job with a reduction takes G lanes per output (G a power of two up to the innermost
// reduction extent) while its outputs x G stay under this many lanes (r04: 32 K / 128 K slower on C2,
// profiles/r04p/)
static uint64_t env_u64(const char *name, uint64_t dflt) {
  const char *v = getenv(name);
  return v && *v ? strtoull(v, nullptr, 10) : dflt;
}
static const uint64_t kBatchLanesCap = env_u64("PGM_BATCH_LANES_CAP", 4096);
// workgroups one batch job may take (its lanes grid-stride over the job's outputs beyond that; r04:
// 1,024 / 4,096 no faster on C1 / C2 / C4, profiles/r04j/)
static const uint64_t kBatchMaxBlocks = env_u64("PGM_BATCH_MAX_BLOCKS", 256);
// a batch contraction without a reduction (a broadcast product or a copy: one load per operand per output)
// may take more workgroups than one that reduces: its lanes otherwise walk several outputs one after
// another, a full memory round trip each (C2's 448,000-output product level: 11.7 -> 8.9 us at 1,024
// blocks, profiles/r04t/), while the reducing jobs of a level were measured slower with more
static const uint64_t kBatchMaxBlocksProduct = env_u64("PGM_BATCH_MAX_BLOCKS_PRODUCT", 1024);

extern "C" {

int pgm_gather(const pgm_gather_desc *d, const double *A, const uint8_t *codes, double *C, int32_t *err_flag,
               void *stream) {
  STALE_PROBE();
  if (!d || !A || !C) return fail(PGM_EINVAL, "gather: null argument");
  if (d->n_ev > 0 && !codes) return fail(PGM_EINVAL, "gather: null codes");
  GatherK k;
  int rc = plan_gather(d, k);
  if (rc != PGM_OK) return rc;
  if (k.n_out == 0) return PGM_OK;
  uint64_t blocks = std::min<uint64_t>((k.n_out + 255) / 256, 65535);
  hipLaunchKernelGGL(k_gather, dim3((unsigned)blocks), dim3(256), 0, S(stream), k, A, codes, C, err_flag);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_batch_create(void **handle) {
  STALE_PROBE();
  if (!handle) return fail(PGM_EINVAL, "batch_create: null handle");
  *handle = new (std::nothrow) BatchHandle;
  return *handle ? PGM_OK : fail(PGM_ENOMEM, "batch_create: host allocation");
}

static int batch_append(BatchHandle *h, BatchJob &J, uint64_t threads, uint64_t cap = 0) {
  if (h->d_jobs) return fail(PGM_EINVAL, "batch: already finalized");
  const uint64_t nb = std::min<uint64_t>(std::max<uint64_t>((threads + 255) / 256, 1), cap ? cap : kBatchMaxBlocks);
  if (h->block_job.size() + nb > 0x7fffffffull) return fail(PGM_EINVAL, "batch: too many blocks");
  J.block0 = (uint32_t)h->block_job.size();
  J.nblocks = (uint32_t)nb;
  h->block_job.insert(h->block_job.end(), nb, (uint32_t)h->jobs.size());
  h->jobs.push_back(J);
  return PGM_OK;
}

int pgm_batch_add_contract(void *handle, const pgm_contract_desc *d, const double *A, const double *B, double *C) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h || !A || !C) return fail(PGM_EINVAL, "batch_add_contract: null argument");
  if (d && d->combine != PGM_COMBINE_COPY && !B) return fail(PGM_EINVAL, "batch_add_contract: null B");
  ContractLaunch L;
  int rc = plan_contract(d, L);
  if (rc != PGM_OK) return rc;
  if (L.empty) return PGM_OK;
  BatchJob J;
  memset(&J, 0, sizeof J);
  J.kind = 0;
  J.cmb = d->combine;
  J.red = d->reduce;
  J.A = A;
  J.B = B;
  J.C = C;
  J.c = L.k;
  // flat mode, no split: lanes per output grow while the job is small and the reduction long
  ContractK &k = J.c;
  k.row_mode = 0;
  k.n_split = 1;
  k.red_chunk = k.n_ro;
  // (a single-workgroup levelled batch runs its blocks one after another: spread a job over at most
  // one block's lanes there)
  const uint64_t lanes_cap = h->mode == PGM_BATCH_ONE_WORKGROUP ? 256 : kBatchLanesCap;
  int g = 0;
  if (d->reduce != PGM_RED_NONE && (uint64_t)k.n_ro * k.ri_card > 1)
    while (g < 6 && ((uint64_t)k.n_out << g) < lanes_cap && (1u << (g + 1)) <= k.ri_card) ++g;
  k.g_log2 = g;
  // output pairs with 16-B accesses when one lane per output is the choice anyway and every access
  // along the innermost kept dim is aligned and unit-stride (or broadcast)
  const int kx = k.nk - 1;
  const bool use_b = d->combine != PGM_COMBINE_COPY;
  bool pairs = g == 0 && kx >= 0 && !g_no_rows2 && k.kdiv[kx].d % 2 == 0 && k.ksc[kx] == 1 && ((uintptr_t)C & 15) == 0;
  const bool va = pairs && k.ksa[kx] != 0, vb = pairs && use_b && k.ksb[kx] != 0;
  pairs = pairs && (k.ksa[kx] == 0 || k.ksa[kx] == 1) && (!use_b || k.ksb[kx] == 0 || k.ksb[kx] == 1);
  for (int i = 0; pairs && i < kx; ++i) pairs = k.ksc[i] % 2 == 0 && (!va || k.ksa[i] % 2 == 0) && (!vb || k.ksb[i] % 2 == 0);
  for (int i = 0; pairs && i + 1 < k.nr; ++i) pairs = (!va || k.rsa[i] % 2 == 0) && (!vb || k.rsb[i] % 2 == 0);
  if (pairs) pairs = (!va || (k.ri_sa % 2 == 0 && ((uintptr_t)A & 15) == 0)) && (!vb || (k.ri_sb % 2 == 0 && ((uintptr_t)B & 15) == 0));
  if (pairs) {
    k.row_mode = 2;
    return batch_append(h, J, (uint64_t)k.n_out / 2, k.n_red <= 1 ? kBatchMaxBlocksProduct : 0);
  }
  return batch_append(h, J, (uint64_t)k.n_out << g, k.n_red <= 1 ? kBatchMaxBlocksProduct : 0);
}

int pgm_batch_add_gather(void *handle, const pgm_gather_desc *d, const double *A, const uint8_t *codes, double *C,
                         int32_t *err_flag) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h || !d || !A || !C) return fail(PGM_EINVAL, "batch_add_gather: null argument");
  if (d->n_ev > 0 && !codes) return fail(PGM_EINVAL, "batch_add_gather: null codes");
  BatchJob J;
  memset(&J, 0, sizeof J);
  int rc = plan_gather(d, J.g);
  if (rc != PGM_OK) return rc;
  if (J.g.n_out == 0) return PGM_OK;
  J.kind = 1;
  J.A = A;
  J.C = C;
  J.codes = codes;
  J.err = err_flag;
  return batch_append(h, J, J.g.n_out);
}

int pgm_batch_add_product_n(void *handle, const pgm_productn_desc *d, const double *const *ops, double *C) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h || !C) return fail(PGM_EINVAL, "batch_add_product_n: null argument");
  BatchJob J;
  memset(&J, 0, sizeof J);
  int rc = plan_prodn(d, ops, J.pn);
  if (rc != PGM_OK) return rc;
  if (J.pn.n_out == 0) return PGM_OK;
  J.kind = 2;
  J.C = C;
  // pairs: 16-B accesses when every access along the innermost dim is aligned and unit/zero stride
  ProdNK &k = J.pn;
  const int kx = k.nk - 1;
  bool pairs = kx >= 0 && k.kdiv[kx].d % 2 == 0 && k.ksc[kx] == 1 && ((uintptr_t)C & 15) == 0 && !g_no_rows2;
  for (int i = 0; pairs && i < kx; ++i) pairs = k.ksc[i] % 2 == 0;
  for (int t = 0; pairs && t < k.n_ops; ++t) {
    const int64_t sx = k.ks[t][kx];
    pairs = sx == 0 || (sx == 1 && ((uintptr_t)k.ops[t] & 15) == 0);
    for (int i = 0; pairs && sx == 1 && i < kx; ++i) pairs = k.ks[t][i] % 2 == 0;
  }
  k.pairs = pairs ? 1u : 0u;
  return batch_append(h, J, pairs ? k.n_out / 2 : k.n_out);
}

// an n-ary contraction's plan: unit dims dropped, adjacent dims merged where every operand (and C, for
// kept dims) steps through them as one, G lanes per output for long reductions of few outputs
static int plan_contract_n(const pgm_contractn_desc *d, const double *const *ops, ContractNK &k) {
  if (!d || !ops) return fail(PGM_EINVAL, "contract_n: null argument");
  const int n = d->n_ops;
  if (n < 1 || n > MOPS) return fail(PGM_EINVAL, "contract_n: %d operands (1..%d)", n, MOPS);
  if (d->reduce != PGM_RED_SUM && d->reduce != PGM_RED_MAX) return fail(PGM_EINVAL, "contract_n: reduce must be sum or max");
  if (d->n_keep < 0 || d->n_keep > PGM_MAX_DIMS || d->n_red < 0 || d->n_red > PGM_MAX_DIMS)
    return fail(PGM_EINVAL, "contract_n: %d kept / %d reduced dims", d->n_keep, d->n_red);
  for (int t = 0; t < n; ++t)
    if (!ops[t]) return fail(PGM_EINVAL, "contract_n: operand %d is null", t);
  memset(&k, 0, sizeof k);
  k.n_ops = n;
  k.red = d->reduce;
  // kept dims (C-order: the last fastest), then reduced dims; each side merged from the inside out
  struct Dim {
    int64_t card, sc, s[MOPS];
  };
  auto collect = [&](int nd, const int64_t *card, const int64_t *sc, const int64_t (*st)[PGM_MAX_DIMS], std::vector<Dim> &out) {
    for (int i = 0; i < nd; ++i) {
      if (card[i] < 0) return false;
      if (card[i] == 1) continue;
      Dim x;
      x.card = card[i];
      x.sc = sc ? sc[i] : 0;
      for (int t = 0; t < n; ++t) x.s[t] = st[t][i];
      if (!out.empty()) {  // merge into the previous (outer) dim when it is this one's continuation
        Dim &o = out.back();
        bool ok = !sc || o.sc == x.sc * x.card;
        for (int t = 0; ok && t < n; ++t) ok = o.s[t] == x.s[t] * x.card;
        if (ok) {
          o.card *= x.card;
          o.sc = x.sc;
          for (int t = 0; t < n; ++t) o.s[t] = x.s[t];
          continue;
        }
      }
      out.push_back(x);
    }
    return true;
  };
  std::vector<Dim> kd, rd;
  for (int i = 0; i < d->n_keep; ++i)
    if (d->keep_card[i] == 0) {
      k.n_out = 0;
      return PGM_OK;  // empty output: nothing to do
    }
  if (!collect(d->n_keep, d->keep_card, d->keep_sc, d->keep_s, kd) || !collect(d->n_red, d->red_card, nullptr, d->red_s, rd))
    return fail(PGM_EINVAL, "contract_n: negative cardinality");
  if ((int)kd.size() > KMAX || (int)rd.size() > KMAX)
    return fail(PGM_EINVAL, "contract_n: %zu kept / %zu reduced dims after merging (at most %d each)", kd.size(), rd.size(), KMAX);
  uint64_t n_out = 1, n_red = 1;
  k.nk = (int)kd.size();
  k.nr = (int)rd.size();
  for (int i = 0; i < k.nk; ++i) {
    n_out *= (uint64_t)kd[i].card;
    if (n_out > 0x7fffffffull) return fail(PGM_EINVAL, "contract_n: output over 2^31 entries");
    k.kcard[i] = (uint32_t)kd[i].card;
    k.ksc[i] = kd[i].sc;
    for (int t = 0; t < n; ++t) k.ks[t][i] = kd[i].s[t];
  }
  for (int i = 0; i < k.nr; ++i) {
    if (rd[i].card == 0) {
      n_red = 0;
      break;
    }
    n_red *= (uint64_t)rd[i].card;
    if (n_red > 0x7fffffffull) return fail(PGM_EINVAL, "contract_n: reduction over 2^31 entries");
    k.rcard[i] = (uint32_t)rd[i].card;
    for (int t = 0; t < n; ++t) k.rs[t][i] = rd[i].s[t];
  }
  if (n_red == 0) return fail(PGM_EINVAL, "contract_n: an empty reduction");
  k.n_out = (uint32_t)n_out;
  k.n_red = (uint32_t)n_red;
  // lanes per output: up to 64 while the job's lanes stay under 4x a batch contraction's cap (a fused
  // step's reduction is a walk of dependent load rounds; more lanes, fewer rounds each)
  static const uint64_t nary_lanes = env_u64("PGM_NARY_LANES", 4 * kBatchLanesCap);
  int g = 0;
  if (k.nr > 0)
    while (g < 6 && ((uint64_t)k.n_out << g) < nary_lanes && (1ull << (g + 1)) <= n_red) ++g;
  k.g_log2 = g;
  return PGM_OK;
}

int pgm_batch_add_contract_n(void *handle, const pgm_contractn_desc *d, const double *const *ops, double *C) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h || !C) return fail(PGM_EINVAL, "batch_add_contract_n: null argument");
  ContractNK k;
  int rc = plan_contract_n(d, ops, k);
  if (rc != PGM_OK) return rc;
  if (k.n_out == 0) return PGM_OK;
  BatchJob J;
  memset(&J, 0, sizeof J);
  J.kind = 4;
  J.red = k.red;
  J.C = C;
  J._pad = (int32_t)h->njobs.size();
  rc = batch_append(h, J, (uint64_t)k.n_out << k.g_log2, k.nr == 0 ? kBatchMaxBlocksProduct : 0);
  if (rc != PGM_OK) return rc;
  h->njobs.push_back(k);
  h->nops.emplace_back(ops, ops + k.n_ops);
  return PGM_OK;
}

int pgm_batch_add_indicator(void *handle, const uint8_t *codes, int64_t n_rows, int64_t card, double *out,
                            int64_t s_state, int64_t s_row, int32_t *err_flag) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h || !codes || !out) return fail(PGM_EINVAL, "batch_add_indicator: null argument");
  if (n_rows <= 0 || card <= 0) return PGM_OK;
  BatchJob J;
  memset(&J, 0, sizeof J);
  J.kind = 3;
  J.codes = codes;
  J.C = out;
  J.err = err_flag;
  J.ind_rows = n_rows;
  J.ind_card = card;
  J.ind_s_state = s_state;
  J.ind_s_row = s_row;
  return batch_append(h, J, (uint64_t)(n_rows * card));
}

int pgm_batch_set_mode(void *handle, int32_t mode) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h) return fail(PGM_EINVAL, "batch_set_mode: null handle");
  if (h->d_jobs || !h->jobs.empty()) return fail(PGM_EINVAL, "batch_set_mode: set before the first job");
  if (mode != PGM_BATCH_GRID && mode != PGM_BATCH_ONE_WORKGROUP) return fail(PGM_EINVAL, "batch_set_mode: mode %d", mode);
  h->mode = mode;
  return PGM_OK;
}

int pgm_batch_blocks(void *handle, int64_t *blocks) {
  BatchHandle *h = (BatchHandle *)handle;
  if (!h || !blocks) return fail(PGM_EINVAL, "batch_blocks: null argument");
  *blocks = (int64_t)h->block_job.size();
  return PGM_OK;
}

int pgm_batch_add_level(void *handle) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h) return fail(PGM_EINVAL, "batch_add_level: null handle");
  if (h->d_jobs) return fail(PGM_EINVAL, "batch_add_level: already finalized");
  if (h->mode != PGM_BATCH_ONE_WORKGROUP) return fail(PGM_EINVAL, "batch_add_level: levels need PGM_BATCH_ONE_WORKGROUP");
  if (h->block_job.size() > h->level_off.back()) h->level_off.push_back((uint32_t)h->block_job.size());
  return PGM_OK;
}

static void batch_free(BatchHandle *h) {
  if (h->d_jobs) (void)hipFree(h->d_jobs);
  if (h->d_map) (void)hipFree(h->d_map);
  if (h->d_level) (void)hipFree(h->d_level);
  if (h->d_chain) (void)hipFree(h->d_chain);
  h->d_chain = nullptr;
  h->chain_lds = 0;
  h->d_jobs = nullptr;
  h->d_map = nullptr;
  h->d_level = nullptr;
}

int pgm_batch_finalize(void *handle) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h) return fail(PGM_EINVAL, "batch_finalize: null handle");
  if (h->d_jobs || h->jobs.empty()) return PGM_OK;
  if (h->level_off.back() < h->block_job.size()) h->level_off.push_back((uint32_t)h->block_job.size());
  h->spec = -1;
  bool uni = true, prod = true, contract_only = true;
  for (const BatchJob &J : h->jobs) {
    uni = uni && J.kind == 0 && J.cmb == h->jobs[0].cmb && J.red == h->jobs[0].red;
    prod = prod && J.kind == 2;
    contract_only = contract_only && (J.kind == 0 || J.kind == 4);  // (kind 4: specialised kernel only)
  }
  if (uni) h->spec = h->jobs[0].cmb * 3 + h->jobs[0].red;
  if (prod) h->spec = kBatchSpecProducts;
  const size_t lds = h->jobs.size() * sizeof(ChainJob) + 4 * (h->block_job.size() + h->level_off.size());
  if (h->mode == PGM_BATCH_ONE_WORKGROUP && !contract_only)
    return fail(PGM_EINVAL, "batch_finalize: a single-workgroup batch takes contractions only");
  if (h->mode == PGM_BATCH_ONE_WORKGROUP && lds > kChainLdsMax)
    return fail(PGM_EINVAL, "batch_finalize: single-workgroup tables of %zu bytes exceed the LDS budget", lds);
  hipError_t e = hipMalloc((void **)&h->d_jobs, sizeof(BatchJob) * h->jobs.size());
  if (e == hipSuccess) e = hipMalloc((void **)&h->d_map, sizeof(uint32_t) * h->block_job.size());
  if (e == hipSuccess)
    e = hipMemcpy(h->d_jobs, h->jobs.data(), sizeof(BatchJob) * h->jobs.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(h->d_map, h->block_job.data(), sizeof(uint32_t) * h->block_job.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && h->mode == PGM_BATCH_ONE_WORKGROUP) {  // k_batch_wg_c: staged descriptors + level table
    e = hipMalloc((void **)&h->d_level, sizeof(uint32_t) * h->level_off.size());
    if (e == hipSuccess)
      e = hipMemcpy(h->d_level, h->level_off.data(), sizeof(uint32_t) * h->level_off.size(), hipMemcpyHostToDevice);
    std::vector<ChainJob> cj(h->jobs.size());
    for (size_t i = 0; i < h->jobs.size(); ++i) {
      const BatchJob &J = h->jobs[i];
      ChainJob &c = cj[i];
      memset(&c, 0, sizeof c);
      c.cmb = J.cmb;
      c.red = J.red;
      c.block0 = J.block0;
      c.nblocks = J.nblocks;
      c.A = J.A;
      c.B = J.B;
      c.C = J.C;
      c.c = J.c;
    }
    if (e == hipSuccess) e = hipMalloc((void **)&h->d_chain, sizeof(ChainJob) * cj.size());
    if (e == hipSuccess) e = hipMemcpy(h->d_chain, cj.data(), sizeof(ChainJob) * cj.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) h->chain_lds = lds;
    if (e == hipSuccess) e = hipDeviceSynchronize();
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    batch_free(h);
    return fail(e == hipErrorOutOfMemory ? PGM_ENOMEM : PGM_EDEVICE, "batch_finalize: %s", hipGetErrorString(e));
  }
  return PGM_OK;
}

int pgm_batch_run(void *handle, void *stream) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h) return fail(PGM_EINVAL, "batch_run: null handle");
  if (h->jobs.empty()) return PGM_OK;
  if (!h->d_jobs) return fail(PGM_EINVAL, "batch_run: not finalized");
  if (!h->njobs.empty())
    return fail(PGM_EINVAL, "batch_run: n-ary contraction jobs run only in the batch's specialised kernel (pgm_batch_specialise)");
  if (h->mode == PGM_BATCH_ONE_WORKGROUP) {
    const uint32_t n_levels = (uint32_t)h->level_off.size() - 1;
    hipLaunchKernelGGL(k_batch_wg_c, dim3(1), dim3(256 * kChainVB), h->chain_lds, S(stream), (const ChainJob *)h->d_chain,
                       h->d_map, h->d_level, n_levels, (uint32_t)h->jobs.size(), (uint32_t)h->block_job.size());
  } else if (h->spec == kBatchSpecProducts) {
    hipLaunchKernelGGL(k_batch_p, dim3((unsigned)h->block_job.size()), dim3(256), 0, S(stream), h->d_jobs, h->d_map);
  } else if (h->spec >= 0) {
    launch_batch_c(h->spec, dim3((unsigned)h->block_job.size()), S(stream), h->d_jobs, h->d_map);
  } else {
    hipLaunchKernelGGL(k_batch, dim3((unsigned)h->block_job.size()), dim3(256), 0, S(stream), h->d_jobs, h->d_map);
  }
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_batch_specialise(void *handle, void **bound) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h || !bound) return fail(PGM_EINVAL, "batch_specialise: null argument");
  *bound = nullptr;
  if (!h->d_jobs) return fail(PGM_EINVAL, "batch_specialise: not finalized");
  std::vector<pgmi_cs_job> jobs;
  for (const BatchJob &J : h->jobs) {
    if ((J.kind > 1 && J.kind != 4) || (J.kind == 0 && J.c.n_split != 1)) return PGM_OK;  // contractions and gathers only
    pgmi_cs_job c;
    memset(&c, 0, sizeof c);
    if (J.kind == 4) {  // n-ary contraction
      c.kind = 2;
      c.red = J.red;
      c.block0 = J.block0;
      c.nblocks = J.nblocks;
      c.C = J.C;
      c.n = h->njobs[J._pad];
      for (int t = 0; t < c.n.n_ops; ++t) c.ops[t] = h->nops[J._pad][t];
      jobs.push_back(c);
      continue;
    }
    c.kind = J.kind;
    c.cmb = J.cmb;
    c.red = J.red;
    c.block0 = J.block0;
    c.nblocks = J.nblocks;
    c.A = J.A;
    c.B = J.B;
    c.C = J.C;
    c.codes = J.codes;
    c.err = J.err;
    if (J.kind == 0) c.k = J.c;
    else c.g = J.g;
    jobs.push_back(c);
  }
  if (jobs.empty()) return PGM_OK;
  return pgmi_cs_bind(jobs.data(), (int)jobs.size(), h->level_off.data(), (int)h->level_off.size() - 1,
                      h->mode == PGM_BATCH_ONE_WORKGROUP ? 1 : 0, bound);
}

int pgm_batch_destroy(void *handle) {
  STALE_PROBE();
  BatchHandle *h = (BatchHandle *)handle;
  if (!h) return PGM_OK;
  batch_free(h);
  delete h;
  return PGM_OK;
}

int pgm_indicator(const uint8_t *codes, int64_t n_rows, int64_t card, double *out, int64_t s_state, int64_t s_row,
                  int32_t *err_flag, void *stream) {
  STALE_PROBE();
  if (!codes || !out) return fail(PGM_EINVAL, "indicator: null argument");
  if (n_rows <= 0 || card <= 0) return PGM_OK;
  uint64_t blocks = std::min<uint64_t>((uint64_t)(n_rows * card + 255) / 256, 65535);
  hipLaunchKernelGGL(k_indicator, dim3((unsigned)blocks), dim3(256), 0, S(stream), codes, n_rows, card, out, s_state,
                     s_row, err_flag);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_argmax(const double *X, int64_t n_rows, int64_t row_len, int64_t s_row, int64_t s_elem, int64_t *out_idx,
               int32_t *out_idx32, void *stream) {
  STALE_PROBE();
  if (!X || (!out_idx && !out_idx32)) return fail(PGM_EINVAL, "argmax: null argument");
  if (n_rows <= 0) return PGM_OK;
  if (row_len <= 0) return fail(PGM_EINVAL, "argmax: empty rows (np.argmax of an empty sequence)");
  if (row_len >= (1ll << 31)) return fail(PGM_EINVAL, "argmax: row too long");
  int g = 0;
  while (g < 6 && ((uint64_t)n_rows << g) < kTargetThreads && (1ll << (g + 1)) <= row_len) ++g;
  uint64_t threads = (uint64_t)n_rows << g;
  uint64_t blocks = std::min<uint64_t>((threads + 255) / 256, 65535);
  hipLaunchKernelGGL(k_argmax, dim3((unsigned)blocks), dim3(256), 0, S(stream), X, (uint64_t)n_rows,
                     (uint32_t)row_len, s_row, s_elem, g, out_idx, out_idx32);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_gemm(const pgm_gemm_desc *d, const double *A, const double *B, double *C, void *stream) {
  STALE_PROBE();
  if (!d || !A || !B || !C || !d->offsets) return fail(PGM_EINVAL, "gemm: null argument");
  if (d->batch < 0 || d->m < 0 || d->n < 0 || d->k < 0) return fail(PGM_EINVAL, "gemm: negative extent");
  if (d->batch == 0 || d->m == 0 || d->n == 0) return PGM_OK;
  GemmK k;
  k.batch = d->batch;
  k.M = d->m;
  k.N = d->n;
  k.K = d->k;
  const int64_t *o = d->offsets;
  k.a_b = o;
  k.b_b = o + d->batch;
  k.c_b = o + 2 * d->batch;
  k.a_m = o + 3 * d->batch;
  k.c_m = k.a_m + d->m;
  k.a_k = k.c_m + d->m;
  k.b_k = k.a_k + d->k;
  k.b_n = k.b_k + d->k;
  k.c_n = k.b_n + d->n;
  k.s_ab = d->stride[0];
  k.s_bb = d->stride[1];
  k.s_cb = d->stride[2];
  k.s_am = d->stride[3];
  k.s_cm = d->stride[4];
  k.s_ak = d->stride[5];
  k.s_bk = d->stride[6];
  k.s_bn = d->stride[7];
  k.s_cn = d->stride[8];
  // block tile by M
  // 128-row tile only while it still gives >= 4 blocks per CU (it halves the blocks of a 65..128-row
  // step; it pays when B is large and would be read twice: C2's 500 x (100 x 576 x 125) step 495 -> 396 us)
  const bool tall_ok = d->m > 64 && d->m <= 128 && (uint64_t)d->batch * (((uint64_t)d->n + 63) / 64) >= 1024;
  const int cfg = d->m <= 16 ? 1 : tall_ok ? 2 : 0;
  const uint64_t BM = cfg == 1 ? 16 : cfg == 2 ? 128 : 64, BN = cfg == 1 ? 128 : 64;
  const uint64_t tn = ((uint64_t)d->n + BN - 1) / BN, tm = ((uint64_t)d->m + BM - 1) / BM;
  if (tn * tm > 0x7fffffffull || d->batch > 65535ll * 65535ll) return fail(PGM_EINVAL, "gemm: grid too large");
  k.tiles_n = (uint32_t)tn;
  if (d->k == 0) return fail(PGM_EINVAL, "gemm: k == 0 (nothing to sum; use the generic contraction)");
  // tile-load lane order along each operand's unit-stride axis (r01: 28.7 -> 32.6 TF/s on plain layouts)
  const bool am_unit = d->stride[3] == 1 || (d->stride[3] < 0 && (d->lane_order & 1));
  const bool bk_unit = d->stride[6] == 1 || (d->stride[6] < 0 && (d->lane_order & 2));
  k.a_mfast = (am_unit && d->stride[5] != 1) ? 1u : 0u;
  k.b_kfast = (bk_unit && d->stride[7] != 1) ? 1u : 0u;
  const bool ta = d->stride[0] < 0 || d->stride[3] < 0 || d->stride[5] < 0;
  const bool tb = d->stride[1] < 0 || d->stride[6] < 0 || d->stride[7] < 0;
  const bool tc = d->stride[2] < 0 || d->stride[4] < 0 || d->stride[8] < 0;
  const int tabs = (ta ? 4 : 0) | (tb ? 2 : 0) | (tc ? 1 : 0);
  const uint64_t gy = std::min<int64_t>(d->batch, 65535), gz = ((uint64_t)d->batch + gy - 1) / gy;
  const dim3 g((unsigned)(tn * tm), (unsigned)gy, (unsigned)gz);
  hipStream_t s = S(stream);
  if (cfg == 1) launch_gemm<16, 128>(tabs, g, s, k, A, B, C);
  else if (cfg == 2) launch_gemm<128, 64>(tabs, g, s, k, A, B, C);
  else launch_gemm<64, 64>(tabs, g, s, k, A, B, C);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_codes_select(const uint8_t *codes, int64_t ld, int64_t row0, const int32_t *cols, int32_t n_cols,
                     int64_t n_rows, uint8_t *out, void *stream) {
  STALE_PROBE();
  if (n_cols <= 0 || n_rows <= 0) return PGM_OK;
  if (!codes || !cols || !out) return fail(PGM_EINVAL, "codes_select: null argument");
  if (n_cols > 65535) return fail(PGM_EINVAL, "codes_select: too many columns");
  const uint64_t bx = ((uint64_t)n_rows + 255) / 256;
  if (bx > 0x7fffffffull) return fail(PGM_EINVAL, "codes_select: too many rows");
  hipLaunchKernelGGL(k_codes_select, dim3((unsigned)bx, (unsigned)n_cols), dim3(256), 0, S(stream), codes, ld, row0,
                     cols, n_rows, out);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_codes_remap(const int8_t *raw, int64_t ld_raw, int32_t n_cols, int64_t n_rows, const uint8_t *lut,
                    int32_t lut_stride, const uint64_t *col_key, uint8_t *out, int64_t ld_out, uint64_t *row_key,
                    uint32_t *row_nmiss, uint64_t *row_hash, int32_t *err_flag, void *stream) {
  STALE_PROBE();
  if (n_cols <= 0 || n_rows <= 0) return PGM_OK;
  if (!raw || !lut || !out || (row_key && (!row_nmiss || !col_key)))
    return fail(PGM_EINVAL, "codes_remap: null argument");
  if (ld_raw < n_rows || ld_out < n_rows || lut_stride < 1 || lut_stride > 256)
    return fail(PGM_EINVAL, "codes_remap: bad leading dimension or LUT stride");
  const uint64_t bx = ((uint64_t)n_rows + 255) / 256;
  if (bx > 0x7fffffffull) return fail(PGM_EINVAL, "codes_remap: too many rows");
  // enough (row block x column chunk) workgroups to fill the chip, each chunk >= 16 columns
  int chunks = 1;
  while (chunks < 64 && bx * chunks < 2048 && n_cols / (chunks * 2) >= 16) chunks *= 2;
  const int chunk = (n_cols + chunks - 1) / chunks;
  hipLaunchKernelGGL(k_codes_remap, dim3((unsigned)bx, (unsigned)chunks), dim3(256), 0, S(stream), raw, ld_raw, lut,
                     lut_stride, n_cols, n_rows, chunk, col_key, out, ld_out, (unsigned long long *)row_key, row_nmiss,
                     (unsigned long long *)row_hash, err_flag);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

// host-side scan (no device): for each of n_cols int8 code columns (n cells each), whether any cell is
// negative (pandas Categorical NaN = -1).  Columns are split over up to `threads` host threads; each
// column is OR-reduced 8 cells per 64-bit word and tested on the sign bits.
// pgm_host_any_negative_i8: pgmhost.cpp (r06: one persistent host thread pool)

int pgm_sample_joint(const double *joint, int64_t ld, int64_t P, const int32_t *group, const double *u, int64_t n,
                     int32_t *out_idx, void *stream) {
  STALE_PROBE();
  if (n <= 0) return PGM_OK;
  if (!joint || !group || !u || !out_idx || P <= 0 || P > 0x7fffffff) return fail(PGM_EINVAL, "sample_joint: bad argument");
  const uint64_t bx = ((uint64_t)n + 255) / 256;
  if (bx > 0x7fffffffull) return fail(PGM_EINVAL, "sample_joint: too many rows");
  hipLaunchKernelGGL(k_sample_joint, dim3((unsigned)bx), dim3(256), 0, S(stream), joint, ld, P, group, u, n, out_idx);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

int pgm_rows_plan_create(const pgm_rows_plan *pl, const double *host_values, void **handle) {
  STALE_PROBE();
  if (!pl || !handle || (!host_values && pl->n_values > 0)) return fail(PGM_EINVAL, "rows_plan_create: null argument");
  *handle = nullptr;
  if (pl->n_loop < 0 || pl->n_loop > PGM_ROWS_MAX_LOOP || pl->n_query < 0 || pl->n_query > pl->n_loop ||
      pl->n_fac < 0 || pl->n_fac > PGM_ROWS_MAX_FAC || pl->n_ev < 0 || pl->n_ev > PGM_ROWS_MAX_EV ||
      pl->n_values < 0 || pl->n_comp < 1 || pl->n_comp > PGM_ROWS_MAX_COMP || pl->n_marg < 0 ||
      pl->n_marg > PGM_ROWS_MAX_MARG)
    return fail(PGM_EINVAL, "rows_plan_create: plan out of range (loop %d query %d fac %d ev %d comp %d marg %d)",
                pl->n_loop, pl->n_query, pl->n_fac, pl->n_ev, pl->n_comp, pl->n_marg);
  RowsK k;
  memset(&k, 0, sizeof k);
  k.one_idx = pl->n_values;  // a trailing 1.0 multiplies into the products of unused factor slots
  k.n_values = pl->n_values + 1;
  k.n_marg = pl->n_marg;
  k.n_joint = pl->n_joint;
  k.n_comp = pl->n_comp;
  // factors: value ranges and evidence ownership
  std::vector<int64_t> fac_hi(pl->n_fac);
  for (int f = 0; f < pl->n_fac; ++f) {
    if (pl->fac_ev_begin[f] < 0 || pl->fac_ev_end[f] > pl->n_ev || pl->fac_ev_begin[f] > pl->fac_ev_end[f])
      return fail(PGM_EINVAL, "rows_plan_create: factor %d evidence range", f);
    int64_t mx = pl->fac_base[f];
    for (int kk = 0; kk < pl->n_loop; ++kk) mx += (int64_t)(pl->loop_card[kk] - 1) * pl->fac_stride[f][kk];
    for (int j = pl->fac_ev_begin[f]; j < pl->fac_ev_end[f]; ++j) mx += (int64_t)(pl->ev_card[j] - 1) * pl->ev_stride[j];
    if (mx >= pl->n_values || pl->fac_base[f] < 0)
      return fail(PGM_EINVAL, "rows_plan_create: factor %d reads past values", f);
    fac_hi[f] = mx + 1;
  }
  std::vector<int> ev_owner(pl->n_ev, -1);
  for (int f = 0; f < pl->n_fac; ++f)
    for (int j = pl->fac_ev_begin[f]; j < pl->fac_ev_end[f]; ++j) {
      if (ev_owner[j] != -1) return fail(PGM_EINVAL, "rows_plan_create: evidence term %d feeds two factors", j);
      ev_owner[j] = f;
    }
  std::vector<RowsComp> comps(pl->n_comp);
  std::vector<int32_t> tab;
  int covered_loop = 0, covered_fac = 0, nq_total = 0, max_nf = 1, max_nt = 0;
  bool any_table = false;
  for (int c = 0; c < pl->n_comp; ++c) {
    const int lb = pl->comp_loop_begin[c], nq = pl->comp_n_query[c], le = pl->comp_loop_end[c];
    const int fb = pl->comp_fac_begin[c], fe = pl->comp_fac_end[c];
    if (lb != covered_loop || nq < 0 || lb + nq > le || le > pl->n_loop || fb != covered_fac || fe < fb ||
        fe > pl->n_fac)
      return fail(PGM_EINVAL, "rows_plan_create: component %d ranges (loops [%d,%d,%d) factors [%d,%d))", c, lb,
                  lb + nq, le, fb, fe);
    covered_loop = le;
    covered_fac = fe;
    uint64_t P = 1, H = 1;
    for (int kk = lb; kk < le; ++kk) {
      if (pl->loop_card[kk] <= 0) return fail(PGM_EINVAL, "rows_plan_create: loop_card[%d] <= 0", kk);
      (kk < lb + nq ? P : H) *= (uint64_t)pl->loop_card[kk];
      if (kk < lb + nq && (pl->loop_marg_off[kk] < 0 || pl->loop_marg_off[kk] + pl->loop_card[kk] > pl->n_marg))
        return fail(PGM_EINVAL, "rows_plan_create: loop %d marginal rows out of range", kk);
    }
    const int nf = fe - fb;
    if (P * H * (uint64_t)std::max(nf, 1) + tab.size() >= (1ull << 26))
      return fail(PGM_EINVAL, "rows_plan_create: component %d index space too large for the fused kernel", c);
    for (int f = fb; f < fe; ++f)
      for (int kk = 0; kk < pl->n_loop; ++kk)
        if ((kk < lb || kk >= le) && pl->fac_stride[f][kk] != 0)
          return fail(PGM_EINVAL, "rows_plan_create: factor %d strides a loop dim outside its component", f);
    max_nf = std::max(max_nf, nf);
    RowsComp &cd = comps[c];
    memset(&cd, 0, sizeof cd);
    cd.nf = nf;
    cd.nq = nq;
    cd.P = (int32_t)P;
    cd.H = (int32_t)H;
    cd.q_lo = nq_total;
    for (int kk = lb; kk < lb + nq; ++kk) {
      k.q_marg_off[nq_total] = pl->loop_marg_off[kk];
      k.q_card[nq_total] = pl->loop_card[kk];
      ++nq_total;
    }
    cd.q_hi = nq_total;
    cd.marg0 = nq >= 1 ? pl->loop_marg_off[lb] : 0;
    cd.simple = (nq <= 1 && H == 1) ? 1 : 0;
    any_table |= !cd.simple;
    cd.mstride = nq == 1 ? pl->loop_map_stride[lb] : 0;
    int64_t vlo = pl->n_values, vhi = 0;
    for (int j = 0; j < PGM_ROWS_MAX_FAC; ++j) cd.fbase[j] = k.one_idx;
    for (int f = fb; f < fe; ++f) {
      cd.fbase[f - fb] = pl->fac_base[f];
      cd.fstride[f - fb] = nq == 1 ? pl->fac_stride[f][lb] : 0;
      vlo = std::min<int64_t>(vlo, pl->fac_base[f]);
      vhi = std::max<int64_t>(vhi, fac_hi[f]);
    }
    cd.val_lo = vlo < vhi ? (int32_t)vlo : 0;
    cd.val_hi = vlo < vhi ? (int32_t)vhi : 0;
    // evidence terms: one contiguous run per component
    int lo = pl->n_ev, hi = 0;
    for (int f = fb; f < fe; ++f)
      if (pl->fac_ev_end[f] > pl->fac_ev_begin[f]) {
        lo = std::min(lo, pl->fac_ev_begin[f]);
        hi = std::max(hi, pl->fac_ev_end[f]);
      }
    if (lo >= hi) lo = hi = pl->n_ev;
    for (int j = lo; j < hi; ++j)
      if (ev_owner[j] < fb || ev_owner[j] >= fe)
        return fail(PGM_EINVAL, "rows_plan_create: component %d evidence terms are not contiguous", c);
    cd.ev_lo = lo;
    cd.nt = hi - lo;
    max_nt = std::max(max_nt, hi - lo);
    for (int j = 0; j < 8; ++j) {
      cd.a_col[j] = hi > lo ? pl->ev_col[lo] : 0;
      cd.a_card[j] = 256;
    }
    if (hi - lo <= 8)
      for (int j = lo; j < hi; ++j) {
        cd.a_col[j - lo] = pl->ev_col[j];
        cd.a_card[j - lo] = pl->ev_card[j];
        if (ev_owner[j] - fb < 4) cd.a_S[j - lo][ev_owner[j] - fb] = pl->ev_stride[j];
      }
    if (cd.simple) continue;
    // per-entry tables, entries in C-order over [query dims..., hidden dims...] (last fastest)
    const int nl = le - lb;
    std::vector<int32_t> dig(nl, 0);
    cd.off_base = (int32_t)tab.size();
    for (uint64_t e = 0; e < P * H; ++e) {
      uint64_t t = e;
      for (int d = nl - 1; d >= 0; --d) {
        dig[d] = (int32_t)(t % (uint64_t)pl->loop_card[lb + d]);
        t /= (uint64_t)pl->loop_card[lb + d];
      }
      for (int f = fb; f < fe; ++f) {
        int64_t o = 0;
        for (int d = 0; d < nl; ++d) o += (int64_t)dig[d] * pl->fac_stride[f][lb + d];
        tab.push_back((int32_t)o);
      }
    }
    cd.marg_base = (int32_t)tab.size();
    for (uint64_t qi = 0; qi < P; ++qi) {
      uint64_t t = qi;
      for (int d = nq - 1; d >= 0; --d) {
        dig[d] = (int32_t)(t % (uint64_t)pl->loop_card[lb + d]);
        t /= (uint64_t)pl->loop_card[lb + d];
      }
      for (int d = 0; d < nq; ++d) tab.push_back(pl->loop_marg_off[lb + d] + dig[d]);
    }
    cd.map_base = (int32_t)tab.size();
    for (uint64_t qi = 0; qi < P; ++qi) {
      uint64_t t = qi;
      int64_t m = 0;
      for (int d = nq - 1; d >= 0; --d) {
        m += (int64_t)(t % (uint64_t)pl->loop_card[lb + d]) * pl->loop_map_stride[lb + d];
        t /= (uint64_t)pl->loop_card[lb + d];
      }
      tab.push_back((int32_t)m);
    }
  }
  if (covered_loop != pl->n_loop || covered_fac != pl->n_fac || nq_total != pl->n_query)
    return fail(PGM_EINVAL, "rows_plan_create: components do not cover the loop dims / factors");
  // descriptor buffer: [RowsComp x n_comp][RowsTerm blocks][tables].  Each component's terms are
  // padded with no-op terms to the kernel's static term count (4 or 8) when they fit it.
  const int padt = max_nt <= 4 ? 4 : max_nt <= 8 ? 8 : 0;
  std::vector<RowsTerm> terms;
  for (int c = 0; c < pl->n_comp; ++c) {
    RowsComp &cd = comps[c];
    const int lo = cd.ev_lo, nt = cd.nt, fb = pl->comp_fac_begin[c];
    cd.ev_lo = (int32_t)terms.size();
    for (int j = lo; j < lo + nt; ++j)
      terms.push_back(RowsTerm{pl->ev_col[j], pl->ev_stride[j], pl->ev_card[j], ev_owner[j] - fb});
    if (nt > 0)
      for (int j = nt; j < padt; ++j) terms.push_back(RowsTerm{pl->ev_col[lo], 0, 256, -1});
  }
  terms.push_back(RowsTerm{0, 0, 256, -1});
  static_assert(sizeof(RowsComp) % 16 == 0 && sizeof(RowsTerm) == 16, "descriptor packing");
  std::vector<int32_t> buf(comps.size() * (sizeof(RowsComp) / 4));
  if (!comps.empty()) memcpy(buf.data(), comps.data(), comps.size() * sizeof(RowsComp));
  k.terms_off = (int32_t)buf.size();
  buf.resize(buf.size() + terms.size() * 4);
  memcpy(buf.data() + k.terms_off, terms.data(), terms.size() * sizeof(RowsTerm));
  k.tab_off = (int32_t)buf.size();
  buf.insert(buf.end(), tab.begin(), tab.end());
  buf.push_back(0);
  RowsHandle *h = new (std::nothrow) RowsHandle;
  if (!h) return fail(PGM_ENOMEM, "rows_plan_create: host allocation");
  h->k = k;
  h->max_nf = max_nf;
  h->max_nt = max_nt;
  h->any_table = any_table;
  h->all_affine = !any_table && max_nf <= 4 && max_nt <= 8;
  h->d_values = nullptr;
  h->d_desc = nullptr;
  (void)hipGetDevice(&h->device);
  for (int j = 0; j < pl->n_ev; ++j) h->n_cols = std::max(h->n_cols, pl->ev_col[j] + 1);
  for (int j = 0; j < pl->n_ev; ++j) h->cols.push_back(pl->ev_col[j]);
  std::sort(h->cols.begin(), h->cols.end());
  h->cols.erase(std::unique(h->cols.begin(), h->cols.end()), h->cols.end());
  if (!any_table) {
    h->jit_src = rows_jit_source(pl);
    h->jit_write_through = jit_store() == 2;
  }
  hipError_t e = hipSuccess;
  e = hipMalloc((void **)&h->d_values, sizeof(double) * (pl->n_values + 1));
  if (e == hipSuccess && pl->n_values > 0)
    e = hipMemcpy(h->d_values, host_values, sizeof(double) * pl->n_values, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    const double one = 1.0;
    e = hipMemcpy(h->d_values + pl->n_values, &one, sizeof(double), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMalloc((void **)&h->d_desc, sizeof(int32_t) * buf.size());
  if (e == hipSuccess) e = hipMemcpy(h->d_desc, buf.data(), sizeof(int32_t) * buf.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    if (h->d_values) (void)hipFree(h->d_values);
    if (h->d_desc) (void)hipFree(h->d_desc);
    delete h;
    return fail(e == hipErrorOutOfMemory ? PGM_ENOMEM : PGM_EDEVICE, "rows_plan_create: %s", hipGetErrorString(e));
  }
  *handle = h;
  return PGM_OK;
}

int pgm_rows_plan_source(const pgm_rows_plan *pl, char *buf, size_t len, size_t *needed) {
  STALE_PROBE();
  if (!pl) return fail(PGM_EINVAL, "rows_plan_source: null plan");
  if (pl->n_comp < 1 || pl->n_comp > PGM_ROWS_MAX_COMP || pl->n_fac < 0 || pl->n_fac > PGM_ROWS_MAX_FAC ||
      pl->n_ev < 0 || pl->n_ev > PGM_ROWS_MAX_EV || pl->n_loop < 0 || pl->n_loop > PGM_ROWS_MAX_LOOP)
    return fail(PGM_EINVAL, "rows_plan_source: plan out of range");
  for (int c = 0; c < pl->n_comp; ++c)
    if (pl->comp_n_query[c] > 1 || pl->comp_loop_end[c] - pl->comp_loop_begin[c] != pl->comp_n_query[c])
      return fail(PGM_EINVAL, "rows_plan_source: component %d is not specialisable (query dims %d, loop dims %d)", c,
                  pl->comp_n_query[c], pl->comp_loop_end[c] - pl->comp_loop_begin[c]);
  const std::string src = rows_jit_source(pl);
  if (needed) *needed = src.size() + 1;
  if (buf && len > 0) {
    const size_t n = std::min(len - 1, src.size());
    memcpy(buf, src.data(), n);
    buf[n] = 0;
  }
  return PGM_OK;
}

int pgm_rows_plan_destroy(void *handle) {
  STALE_PROBE();
  RowsHandle *h = (RowsHandle *)handle;
  if (!h) return PGM_OK;
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (h->shard[0].s || h->shard[1].s) (void)hipSetDevice(h->device);
  for (auto &sd : h->shard) {
    if (sd.s) (void)hipStreamSynchronize(sd.s);
    if (sd.buf) (void)hipFree(sd.buf);
    if (sd.h_err) (void)hipHostFree(sd.h_err);
    if (sd.s) (void)hipStreamDestroy(sd.s);
  }
  (void)hipSetDevice(prev);
  if (h->d_values) (void)hipFree(h->d_values);
  if (h->d_desc) (void)hipFree(h->d_desc);
  if (h->jit_mod) (void)hipModuleUnload(h->jit_mod);
  delete h;
  return PGM_OK;
}

}  // extern "C"

// dry: validate and size the launch only (pgm_rows_plan_bind)
static int rows_plan_run(void *handle, int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0,
                         int64_t n_rows, double *marg, double *joint, int64_t ld_out, int32_t *map, double *gap,
                         int32_t *err_flag, void *stream, bool dry) {
  RowsHandle *h = (RowsHandle *)handle;
  if (!h) return fail(PGM_EINVAL, "rows_plan_run: null handle");
  if (n_rows <= 0) return PGM_OK;
  if (h->max_nt > 0 && !codes) return fail(PGM_EINVAL, "rows_plan_run: null codes");
  if ((mode & PGM_ROWS_MARGINALS) && !marg) return fail(PGM_EINVAL, "rows_plan_run: marginals requested, marg is null");
  if ((mode & PGM_ROWS_JOINT) && !joint) return fail(PGM_EINVAL, "rows_plan_run: joint requested, joint is null");
  if ((mode & PGM_ROWS_JOINT) && h->k.n_comp != 1)
    return fail(PGM_EINVAL, "rows_plan_run: joint output needs a single-component plan");
  if ((mode & PGM_ROWS_MAP) && !map) return fail(PGM_EINVAL, "rows_plan_run: MAP requested, map is null");
  if ((mode & PGM_ROWS_MAPGAP) && !gap) return fail(PGM_EINVAL, "rows_plan_run: MAP gap requested, gap is null");
  if ((mode & (PGM_ROWS_MARGINALS | PGM_ROWS_JOINT)) && ld_out < n_rows)
    return fail(PGM_EINVAL, "rows_plan_run: ld_out %lld < n_rows %lld", (long long)ld_out, (long long)n_rows);
  // one workgroup = 64 rows x RG row groups; W waves split the components
  RowsK k = h->k;
  k.n_waves = k.n_comp;  // one wave per component
  const size_t kLds = 64 * 1024;
  size_t vals_bytes = (size_t)((k.n_values + 1) & ~1) * sizeof(double);
  const bool vals_lds = vals_bytes <= 40 * 1024 && !(mode & PGM_ROWS_VALUES_GLOBAL);
  if (!vals_lds) vals_bytes = 0;
  const size_t x_bytes = (size_t)k.n_comp * 64 * (2 * sizeof(double) + sizeof(int32_t));
  const size_t acc_bytes = (size_t)k.n_marg * 64 * sizeof(double);
  const bool acc_lds = (mode & PGM_ROWS_MARGINALS) && h->any_table && vals_bytes + x_bytes + acc_bytes <= kLds;
  const size_t lds = vals_bytes + x_bytes + (acc_lds ? acc_bytes : 0);
  const uint64_t groups = ((uint64_t)n_rows + 63) / 64;
  // amortise the LDS staging of the CPT values over several row groups once the grid is large
  int32_t RG = 1;
  if (vals_lds && !(mode & PGM_ROWS_ONE_GROUP)) RG = (int32_t)std::max<uint64_t>(1, std::min<uint64_t>(8, groups / 4096));
  hipStream_t s = S(stream);
  const double *v = h->d_values;
  const int32_t *t = h->d_desc;
  if (!(mode & (PGM_ROWS_JOINT | PGM_ROWS_GENERIC | PGM_ROWS_NO_JIT | PGM_ROWS_VALUES_GLOBAL | PGM_ROWS_ONE_GROUP)) &&
      rows_jit_ready(h)) {
    const bool two = rows_jit2_ok(mode, codes, ld_codes, row0, n_rows, marg, ld_out, map, gap, h->k.n_marg);
    const uint64_t rpb = (uint64_t)jit_wg() * (two ? 2 : 1);  // rows per block
    const uint64_t jblocks = ((uint64_t)n_rows + rpb - 1) / rpb;
    if (jblocks > 0x7fffffffull) return fail(PGM_EINVAL, "rows_plan_run: too many rows");
    if (dry) return PGM_OK;
    const uint8_t *cp = codes;
    int64_t ldc = ld_codes, r0 = row0, nr = n_rows, ldo = ld_out;
    double *mg = marg, *gp = gap;
    int32_t *mp = map, *ef = err_flag;
    int32_t md = mode;
    void *args[] = {(void *)&v, (void *)&cp, &ldc, &r0, &nr, (void *)&mg, &ldo, (void *)&mp, (void *)&gp, (void *)&ef, &md};
    HIP_TRY(hipModuleLaunchKernel(two ? h->jit_fn2 : h->jit_fn, (unsigned)jblocks, 1, 1, (unsigned)jit_wg(), 1, 1, 0, s,
                                  args, nullptr));
    return PGM_OK;
  }
  if (h->all_affine && !(mode & PGM_ROWS_JOINT) && !(mode & PGM_ROWS_GENERIC)) {
    RG = 1;
    if (vals_lds && !(mode & PGM_ROWS_ONE_GROUP))
      RG = (int32_t)std::max<uint64_t>(1, std::min<uint64_t>(8, groups / 4096));
    const uint64_t ablocks = (groups + RG - 1) / RG;
    if (ablocks > 0x7fffffffull) return fail(PGM_EINVAL, "rows_plan_run: too many rows");
    const bool do_map = (mode & (PGM_ROWS_MAP | PGM_ROWS_MAPGAP)) != 0;
    // exchange slots: masses only, unless MAP digits / gaps are combined too
    const size_t x_aff = k.n_comp > 1 ? (size_t)k.n_comp * 64 * (do_map ? 2 * sizeof(double) + sizeof(int32_t) : sizeof(double)) : 0;
    const dim3 ag((unsigned)ablocks), ab(64 * k.n_comp);
    if (dry) return PGM_OK;
    if (vals_lds)
      launch_affine<true>(h->max_nf, h->max_nt, do_map, ag, ab, vals_bytes + x_aff, s, k, v, t, codes, ld_codes, row0, n_rows, mode, RG, marg, ld_out, map, gap, err_flag);
    else
      launch_affine<false>(h->max_nf, h->max_nt, do_map, ag, ab, vals_bytes + x_aff, s, k, v, t, codes, ld_codes, row0, n_rows, mode, RG, marg, ld_out, map, gap, err_flag);
    HIP_TRY(hipGetLastError());
    return PGM_OK;
  }
  const uint64_t blocks = (groups + RG - 1) / RG;
  if (blocks > 0x7fffffffull) return fail(PGM_EINVAL, "rows_plan_run: too many rows");
  const dim3 g((unsigned)blocks), b(64 * k.n_waves);
  if (dry) return PGM_OK;
  if (vals_lds && acc_lds)
    launch_rows_f<true, true>(h->max_nt, h->max_nf, g, b, lds, s, k, v, t, codes, ld_codes, row0, n_rows, mode, RG, marg, joint, ld_out, map, gap, err_flag);
  else if (vals_lds)
    launch_rows_f<true, false>(h->max_nt, h->max_nf, g, b, lds, s, k, v, t, codes, ld_codes, row0, n_rows, mode, RG, marg, joint, ld_out, map, gap, err_flag);
  else if (acc_lds)
    launch_rows_f<false, true>(h->max_nt, h->max_nf, g, b, lds, s, k, v, t, codes, ld_codes, row0, n_rows, mode, RG, marg, joint, ld_out, map, gap, err_flag);
  else
    launch_rows_f<false, false>(h->max_nt, h->max_nf, g, b, lds, s, k, v, t, codes, ld_codes, row0, n_rows, mode, RG, marg, joint, ld_out, map, gap, err_flag);
  HIP_TRY(hipGetLastError());
  return PGM_OK;
}

extern "C" {

int pgm_rows_plan_run(void *handle, int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0, int64_t n_rows,
                      double *marg, double *joint, int64_t ld_out, int32_t *map, double *gap, int32_t *err_flag,
                      void *stream) {
  STALE_PROBE();
  return rows_plan_run(handle, mode, codes, ld_codes, row0, n_rows, marg, joint, ld_out, map, gap, err_flag, stream,
                       false);
}

// A validated, fully bound pgm_rows_plan_run (a prepared launch): repeated batches over the same
// buffers pay one argument-free call each instead of re-marshalling thirteen arguments.
struct RowsJitArgs {  // pgm_rows_jit's parameters, packed as the kernel's argument segment
  const double *V;
  const uint8_t *C;
  int64_t ldc, row0, n;
  double *M;
  int64_t ldo;
  int32_t *MP;
  double *G;
  int32_t *E;
  int32_t mode;
  int32_t pad;
};

struct RowsBound {
  // specialised kernel bound: the packed argument segment and launch shape, launched directly
  hipFunction_t fn = nullptr;
  RowsJitArgs args;
  size_t args_size = sizeof(RowsJitArgs);
  unsigned blocks = 0;
  void *handle;
  int32_t mode;
  const uint8_t *codes;
  int64_t ld_codes, row0, n_rows;
  double *marg, *joint;
  int64_t ld_out;
  int32_t *map;
  double *gap;
  int32_t *err;
  void *stream;
};

int pgm_rows_plan_bind(void *handle, int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0,
                       int64_t n_rows, double *marg, double *joint, int64_t ld_out, int32_t *map, double *gap,
                       int32_t *err_flag, void *stream, void **bound) {
  STALE_PROBE();
  if (!bound) return fail(PGM_EINVAL, "rows_plan_bind: null output pointer");
  *bound = nullptr;
  const bool floor = (mode & PGM_ROWS_FLOOR) != 0;
  mode &= ~PGM_ROWS_FLOOR;
  if (floor && (mode & (PGM_ROWS_JOINT | PGM_ROWS_GENERIC | PGM_ROWS_NO_JIT | PGM_ROWS_VALUES_GLOBAL | PGM_ROWS_ONE_GROUP)))
    return fail(PGM_EINVAL, "rows_plan_bind: the floor kernel exists for the specialised kernel's modes only");
  const int st = rows_plan_run(handle, mode, codes, ld_codes, row0, n_rows, marg, joint, ld_out, map, gap, err_flag,
                               stream, true);
  if (st != PGM_OK) return st;
  RowsBound *b = new (std::nothrow) RowsBound;
  if (!b) return fail(PGM_ENOMEM, "rows_plan_bind: out of host memory");
  b->handle = handle;
  b->mode = mode;
  b->codes = codes;
  b->ld_codes = ld_codes;
  b->row0 = row0;
  b->n_rows = n_rows;
  b->marg = marg;
  b->joint = joint;
  b->ld_out = ld_out;
  b->map = map;
  b->gap = gap;
  b->err = err_flag;
  b->stream = stream;
  RowsHandle *h = (RowsHandle *)handle;
  // the same choice rows_plan_run makes (the dry run above compiled the kernel if it applies)
  if (n_rows > 0 && h->jit_state > 0 &&
      !(mode & (PGM_ROWS_JOINT | PGM_ROWS_GENERIC | PGM_ROWS_NO_JIT | PGM_ROWS_VALUES_GLOBAL | PGM_ROWS_ONE_GROUP))) {
    const bool two = rows_jit2_ok(mode, codes, ld_codes, row0, n_rows, marg, ld_out, map, gap, h->k.n_marg);
    b->fn = floor ? (two ? h->jit_fn_floor2 : h->jit_fn_floor) : two ? h->jit_fn2 : h->jit_fn;
    b->args = RowsJitArgs{h->d_values, codes, ld_codes, row0, n_rows, marg, ld_out, map, gap, err_flag, mode, 0};
    const uint64_t rpb = (uint64_t)jit_wg() * (two ? 2 : 1);
    b->blocks = (unsigned)(((uint64_t)n_rows + rpb - 1) / rpb);
  } else if (floor) {
    delete b;
    return fail(PGM_EINVAL, "rows_plan_bind: the floor kernel needs the plan-specialised (hipRTC) kernel");
  }
  *bound = b;
  return PGM_OK;
}

int pgm_rows_bound_run(void *bound) {
  STALE_PROBE();
  RowsBound *b = (RowsBound *)bound;
  if (!b) return fail(PGM_EINVAL, "rows_bound_run: null handle");
  if (b->fn) {
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &b->args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &b->args_size,
                     HIP_LAUNCH_PARAM_END};
    HIP_TRY(hipModuleLaunchKernel(b->fn, b->blocks, 1, 1, (unsigned)jit_wg(), 1, 1, 0, S(b->stream), nullptr, extra));
    return PGM_OK;
  }
  return rows_plan_run(b->handle, b->mode, b->codes, b->ld_codes, b->row0, b->n_rows, b->marg, b->joint, b->ld_out,
                       b->map, b->gap, b->err, b->stream, false);
}

int pgm_rows_bound_kernel(void *bound, char *name, size_t cap, uint32_t *blocks, uint32_t *wg) {
  RowsBound *b = (RowsBound *)bound;
  if (!b || !name || cap == 0) return fail(PGM_EINVAL, "rows_bound_kernel: null argument");
  RowsHandle *h = (RowsHandle *)b->handle;
  const char *k = !b->fn ? "" : b->fn == h->jit_fn2 ? "pgm_rows_jit2" : b->fn == h->jit_fn_floor ? "pgm_rows_floor" : b->fn == h->jit_fn_floor2 ? "pgm_rows_floor2" : "pgm_rows_jit";
  snprintf(name, cap, "%s", k);
  if (blocks) *blocks = b->fn ? b->blocks : 0;
  if (wg) *wg = b->fn ? (uint32_t)jit_wg() : 0;
  return PGM_OK;
}

int pgm_rows_bound_destroy(void *bound) {
  STALE_PROBE();
  delete (RowsBound *)bound;
  return PGM_OK;
}

// ---------------------------------------------------------------------------- rows sharded over GPUs
// One shard of pgm_rows_shard_run on its plan's device, on its own host thread: its rows in chunks of
// at most shard_chunk_rows(), chunk c on side c % 2 of the handle's kept resources (stream + device
// buffer): the chunk's rows of the columns the plan reads in (one copy per run of adjacent columns),
// the plan's pass, its outputs out to the caller's host arrays at the chunk's columns.  Each side's
// stream orders its own chunks, so chunk c + 2 reuses the buffer only after chunk c's copy-out; with
// pinned host arrays (pgm_host_alloc / hipHostRegister) the two sides' DMA and kernels overlap.
static constexpr int64_t shard_chunk_rows() { return 262144; }  // 256 K rows: 36 MB of marginals per chunk

static int shard_side_ready(RowsHandle::ShardSide &sd, size_t need) {
  if (!sd.s) HIP_TRY(hipStreamCreateWithFlags(&sd.s, hipStreamNonBlocking));
  if (!sd.h_err) HIP_TRY(hipHostMalloc((void **)&sd.h_err, 64, hipHostMallocDefault));
  if (sd.cap < need) {
    if (sd.buf) {
      HIP_TRY(hipStreamSynchronize(sd.s));
      (void)hipFree(sd.buf);
      sd.buf = nullptr;
      sd.cap = 0;
    }
    HIP_TRY(hipMalloc((void **)&sd.buf, need));
    sd.cap = need;
  }
  return PGM_OK;
}

static int rows_shard_one(RowsHandle *h, int32_t mode, const uint8_t *host_codes, int64_t ld_codes, int64_t r0,
                          int64_t nr, double *host_marg, int64_t ld_out, int32_t *host_map, int32_t *err_any) {
  std::lock_guard<std::mutex> lk(h->shard_mu);
  HIP_TRY(hipSetDevice(h->device));
  const int64_t chunk = std::min<int64_t>(nr, shard_chunk_rows());
  // device layout of a chunk: codes [h->n_cols][ldc] (only the plan's columns are written), marg
  // [n_marg][ldc], map [ldc], err; ldc a multiple of 16 so the two-rows-per-lane kernel takes full chunks
  const int64_t ldc = (chunk + 15) & ~(int64_t)15;
  const bool want_m = (mode & PGM_ROWS_MARGINALS) != 0, want_p = (mode & PGM_ROWS_MAP) != 0;
  const size_t b_codes = (size_t)std::max(h->n_cols, 1) * ldc;
  const size_t o_marg = (b_codes + 255) & ~(size_t)255;
  const size_t b_marg = want_m ? (size_t)h->k.n_marg * ldc * sizeof(double) : 0;
  const size_t o_map = o_marg + ((b_marg + 255) & ~(size_t)255);
  const size_t b_map = want_p ? (size_t)ldc * sizeof(int32_t) : 0;
  const size_t o_err = o_map + ((b_map + 255) & ~(size_t)255);
  const int n_sides = nr > chunk ? 2 : 1;
  for (int i = 0; i < n_sides; ++i) {
    const int st = shard_side_ready(h->shard[i], o_err + 256);
    if (st != PGM_OK) return st;
    h->shard[i].h_err[0] = 0;
    HIP_TRY(hipMemsetAsync(h->shard[i].buf + o_err, 0, sizeof(int32_t), h->shard[i].s));
  }
  // runs of adjacent plan columns: one 2-D copy each
  std::vector<std::pair<int, int>> runs;
  for (int c : h->cols) {
    if (!runs.empty() && runs.back().first + runs.back().second == c) ++runs.back().second;
    else runs.push_back({c, 1});
  }
  int st = PGM_OK;
  hipError_t e = hipSuccess;
  int64_t c = 0;
  for (int64_t a = r0; a < r0 + nr && st == PGM_OK && e == hipSuccess; a += chunk, ++c) {
    RowsHandle::ShardSide &sd = h->shard[c % n_sides];
    const int64_t m = std::min(chunk, r0 + nr - a);
    uint8_t *d_codes = (uint8_t *)sd.buf;
    double *d_marg = want_m ? (double *)(sd.buf + o_marg) : nullptr;
    int32_t *d_map = want_p ? (int32_t *)(sd.buf + o_map) : nullptr;
    int32_t *d_err = (int32_t *)(sd.buf + o_err);
    for (size_t k = 0; k < runs.size() && e == hipSuccess; ++k)
      e = hipMemcpy2DAsync(d_codes + (size_t)runs[k].first * ldc, (size_t)ldc,
                           host_codes + (size_t)runs[k].first * ld_codes + a, (size_t)ld_codes, (size_t)m,
                           (size_t)runs[k].second, hipMemcpyHostToDevice, sd.s);
    if (e != hipSuccess) break;
    st = rows_plan_run(h, mode, d_codes, ldc, 0, m, d_marg, nullptr, ldc, d_map, nullptr, d_err, sd.s, false);
    if (st == PGM_OK && want_m)
      e = hipMemcpy2DAsync(host_marg + a, (size_t)ld_out * sizeof(double), d_marg, (size_t)ldc * sizeof(double),
                           (size_t)m * sizeof(double), (size_t)h->k.n_marg, hipMemcpyDeviceToHost, sd.s);
    if (st == PGM_OK && e == hipSuccess && want_p)
      e = hipMemcpyAsync(host_map + a, d_map, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost, sd.s);
  }
  int32_t h_err = 0;
  for (int i = 0; i < n_sides; ++i) {
    RowsHandle::ShardSide &sd = h->shard[i];
    if (e == hipSuccess && st == PGM_OK)
      e = hipMemcpyAsync(sd.h_err, sd.buf + o_err, sizeof(int32_t), hipMemcpyDeviceToHost, sd.s);
    const hipError_t es = hipStreamSynchronize(sd.s);
    if (e == hipSuccess) e = es;
    h_err |= sd.h_err[0];
  }
  if (st != PGM_OK) return st;
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(PGM_EDEVICE, "rows_shard_run: %s", hipGetErrorString(e));
  }
  if (h_err && err_any) __atomic_fetch_or(err_any, h_err, __ATOMIC_RELAXED);
  return PGM_OK;
}

int pgm_rows_shard_run(void *const *handles, int32_t n_shards, int32_t mode, const uint8_t *host_codes,
                       int64_t ld_codes, int64_t n_cols, int64_t n_rows, double *host_marg, int64_t ld_out,
                       int32_t *host_map, int32_t *err_any) {
  STALE_PROBE();
  if (!handles || n_shards < 1) return fail(PGM_EINVAL, "rows_shard_run: no plan handles");
  if (n_rows < 0 || ld_codes < n_rows || n_cols < 0) return fail(PGM_EINVAL, "rows_shard_run: bad shape");
  if (mode & ~(PGM_ROWS_MARGINALS | PGM_ROWS_MAP))
    return fail(PGM_EINVAL, "rows_shard_run: mode takes PGM_ROWS_MARGINALS | PGM_ROWS_MAP only");
  if (!(mode & (PGM_ROWS_MARGINALS | PGM_ROWS_MAP))) return fail(PGM_EINVAL, "rows_shard_run: no output requested");
  if ((mode & PGM_ROWS_MARGINALS) && (!host_marg || ld_out < n_rows))
    return fail(PGM_EINVAL, "rows_shard_run: marginals need host_marg with ld_out >= n_rows");
  if ((mode & PGM_ROWS_MAP) && !host_map) return fail(PGM_EINVAL, "rows_shard_run: MAP needs host_map");
  int32_t n_marg = -1;
  for (int32_t i = 0; i < n_shards; ++i) {
    const RowsHandle *h = (const RowsHandle *)handles[i];
    if (!h) return fail(PGM_EINVAL, "rows_shard_run: null handle %d", i);
    if (h->n_cols > n_cols) return fail(PGM_EINVAL, "rows_shard_run: plan %d reads column %d of %lld", i, h->n_cols - 1,
                                        (long long)n_cols);
    if (n_marg >= 0 && h->k.n_marg != n_marg) return fail(PGM_EINVAL, "rows_shard_run: plans differ (marginal rows)");
    n_marg = h->k.n_marg;
  }
  if (n_rows == 0) return PGM_OK;
  if (n_cols > 0 && !host_codes) return fail(PGM_EINVAL, "rows_shard_run: null codes");
  int prev = 0;
  (void)hipGetDevice(&prev);
  // contiguous shards (distributed.shard_bounds): shard i = rows [i n / S, (i + 1) n / S)
  std::vector<int> st(n_shards, PGM_OK);
  std::vector<std::string> msg(n_shards);
  std::vector<std::thread> th;
  th.reserve(n_shards);
  for (int32_t i = 0; i < n_shards; ++i) {
    const int64_t a = n_rows * i / n_shards, b = n_rows * (i + 1) / n_shards;
    th.emplace_back([&, i, a, b] {
      if (b > a) {
        st[i] = rows_shard_one((RowsHandle *)handles[i], mode, host_codes, ld_codes, a, b - a, host_marg, ld_out,
                               host_map, err_any);
        if (st[i] != PGM_OK) msg[i] = g_err;  // the worker's thread-local message
      }
    });
  }
  for (auto &t : th) t.join();
  (void)hipSetDevice(prev);
  for (int32_t i = 0; i < n_shards; ++i)
    if (st[i] != PGM_OK) return fail(st[i], "rows_shard_run: shard %d: %s", i, msg[i].c_str());
  return PGM_OK;
}

// ---------------------------------------------------------------------------- resident ring of batches
struct PgmRingSlot {  // pgm_ring_slot of the generated source (64 B)
  const uint8_t *C;
  int64_t ldc, row0;
  double *M;
  int64_t ldo;
  int32_t *MP;
  double *G;
  int64_t pad;
};
static_assert(sizeof(PgmRingSlot) == 64, "ring slot layout");

struct RowsRing {
  RowsHandle *h = nullptr;
  int32_t mode = 0;
  int64_t n_rows = 0;
  uint32_t n_slots = 0;
  PgmRingSlot *d_slots = nullptr;  // device
  unsigned *ctl = nullptr;         // pinned host: [0] batches posted, [1] cancel, [2] status (|2: timed out)
  unsigned *ctl_dev = nullptr;     // its device address
  unsigned *gctl = nullptr;        // device memory: [0] mirror of ctl[0], [1] host-poll token, [2] stop
  int32_t *err = nullptr;
  hipStream_t stream = nullptr;
  unsigned blocks = 0;
  bool running = false;
  bool reset_gctl = true;   // the device counters need zeroing before the next launch (first / after a stop)
  uint32_t n_batches = 0, posted = 0;  // this launch: batches to run, batches posted
  uint32_t base = 0;        // absolute number of batches posted over the ring's lifetime before this launch
  int wall_khz = 100000;    // the device's constant wall clock (timeout ticks)
};

int pgm_rows_ring_create(void *handle, int32_t mode, int32_t n_slots, const uint8_t *const *codes,
                         const int64_t *ld_codes, const int64_t *row0, int64_t n_rows, double *const *marg,
                         int64_t ld_out, int32_t *const *map, double *const *gap, int32_t *err_flag, void *stream,
                         void **ring) {
  STALE_PROBE();
  if (!ring) return fail(PGM_EINVAL, "rows_ring_create: null output pointer");
  *ring = nullptr;
  RowsHandle *h = (RowsHandle *)handle;
  if (!h) return fail(PGM_EINVAL, "rows_ring_create: null plan");
  if (n_slots < 1 || !codes || !ld_codes || !row0) return fail(PGM_EINVAL, "rows_ring_create: no slots");
  if (n_rows < 2) return fail(PGM_EINVAL, "rows_ring_create: n_rows %lld < 2", (long long)n_rows);
  if (mode & ~(PGM_ROWS_MARGINALS | PGM_ROWS_MAP | PGM_ROWS_MAPGAP))
    return fail(PGM_EINVAL, "rows_ring_create: the ring runs marginals / MAP / MAP-gap outputs only");
  if (!(mode & (PGM_ROWS_MARGINALS | PGM_ROWS_MAP | PGM_ROWS_MAPGAP)))
    return fail(PGM_EINVAL, "rows_ring_create: no output requested");
  if (!rows_jit_ready(h)) return fail(PGM_EINVAL, "rows_ring_create: the ring needs the plan-specialised (hipRTC) kernel");
  std::vector<PgmRingSlot> slots((size_t)n_slots);
  for (int32_t i = 0; i < n_slots; ++i) {
    double *m = (mode & PGM_ROWS_MARGINALS) ? (marg ? marg[i] : nullptr) : nullptr;
    int32_t *mp = (mode & (PGM_ROWS_MAP | PGM_ROWS_MAPGAP)) && map ? map[i] : nullptr;
    double *g = (mode & PGM_ROWS_MAPGAP) && gap ? gap[i] : nullptr;
    if ((mode & PGM_ROWS_MARGINALS) && !m) return fail(PGM_EINVAL, "rows_ring_create: slot %d has no marginal buffer", i);
    if ((mode & PGM_ROWS_MAP) && !mp) return fail(PGM_EINVAL, "rows_ring_create: slot %d has no MAP buffer", i);
    if ((mode & PGM_ROWS_MAPGAP) && !g) return fail(PGM_EINVAL, "rows_ring_create: slot %d has no MAP-gap buffer", i);
    if (h->max_nt > 0 && !codes[i]) return fail(PGM_EINVAL, "rows_ring_create: slot %d has no evidence codes", i);
    if ((mode & PGM_ROWS_MARGINALS) && ld_out < n_rows)
      return fail(PGM_EINVAL, "rows_ring_create: ld_out %lld < n_rows %lld", (long long)ld_out, (long long)n_rows);
    if (!rows2_aligned(mode, codes[i], ld_codes[i], row0[i], n_rows, m, ld_out, mp, g, h->k.n_marg))
      return fail(PGM_EINVAL, "rows_ring_create: slot %d breaks the two-rows-per-lane contract (even rows, row0 and "
                  "leading dimensions, 16-B aligned outputs)", i);
    slots[i] = PgmRingSlot{codes[i], ld_codes[i], row0[i], m, ld_out, mp, g, 0};
  }
  RowsRing *rg = new (std::nothrow) RowsRing;
  if (!rg) return fail(PGM_ENOMEM, "rows_ring_create: out of host memory");
  rg->h = h;
  rg->mode = mode;
  rg->n_rows = n_rows;
  rg->n_slots = (uint32_t)n_slots;
  rg->err = err_flag;
  rg->stream = S(stream);
  hipError_t e = hipMalloc((void **)&rg->d_slots, sizeof(PgmRingSlot) * slots.size());
  if (e == hipSuccess)
    e = hipMemcpy(rg->d_slots, slots.data(), sizeof(PgmRingSlot) * slots.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipHostMalloc((void **)&rg->ctl, 64, hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&rg->ctl_dev, rg->ctl, 0);
  if (e == hipSuccess) e = hipMalloc((void **)&rg->gctl, 64);
  int dev = 0, cus = 0, per_cu = 0;
  if (e == hipSuccess) e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess)
    e = hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, h->jit_fn_ring, ring_wg(), 0);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    if (rg->d_slots) (void)hipFree(rg->d_slots);
    if (rg->gctl) (void)hipFree(rg->gctl);
    if (rg->ctl) (void)hipHostFree(rg->ctl);
    delete rg;
    return fail(e == hipErrorOutOfMemory ? PGM_ENOMEM : PGM_EDEVICE, "rows_ring_create: %s", hipGetErrorString(e));
  }
  memset(rg->ctl, 0, 64);
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0) rg->wall_khz = khz;
  (void)hipGetLastError();
  // every workgroup resident at once (one per CU at the default 1,024 threads)
  rg->blocks = (unsigned)std::max(1, cus * std::max(1, per_cu));
  *ring = rg;
  return PGM_OK;
}

static int ring_start(RowsRing *rg, uint32_t n_batches, double timeout_s, int signal);

int pgm_rows_ring_start(void *ring, uint32_t n_batches, double timeout_s) {
  STALE_PROBE();
  return ring_start((RowsRing *)ring, n_batches, timeout_s, 0);
}

int pgm_rows_ring_start_ready(void *ring, uint32_t n_batches, double timeout_s, double ready_timeout_s) {
  STALE_PROBE();
  RowsRing *rg = (RowsRing *)ring;
  if (!(ready_timeout_s > 0.0) || ready_timeout_s > 600.0)
    return fail(PGM_EINVAL, "rows_ring_start_ready: ready timeout must be in (0, 600] s");
  if (rg) __atomic_store_n(&rg->ctl[3], 0u, __ATOMIC_SEQ_CST);
  const int st = ring_start(rg, n_batches, timeout_s, 1);
  if (st != PGM_OK || n_batches == 0) return st;
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(&rg->ctl[3], __ATOMIC_ACQUIRE) == 0u) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > ready_timeout_s) {
      (void)pgm_rows_ring_cancel(ring);
      return fail(PGM_EDEVICE, "rows_ring_start_ready: the resident grid did not come up within %.3g s",
                  ready_timeout_s);
    }
  }
  return PGM_OK;
}

static int ring_start(RowsRing *rg, uint32_t n_batches, double timeout_s, int signal) {
  if (!rg) return fail(PGM_EINVAL, "rows_ring_start: null ring");
  if (rg->running) return fail(PGM_EINVAL, "rows_ring_start: the ring is running (finish or cancel it first)");
  if (!(timeout_s > 0.0) || timeout_s > 600.0) return fail(PGM_EINVAL, "rows_ring_start: timeout must be in (0, 600] s");
  unsigned long long ticks = (unsigned long long)(timeout_s * (double)rg->wall_khz * 1000.0);
  // ctl[0] counts batches posted over the ring's lifetime (never reset: a launch's batch b is
  // absolute batch base + b), so no device-side reset is needed between launches
  __atomic_store_n(&rg->ctl[1], 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(&rg->ctl[2], 0u, __ATOMIC_SEQ_CST);
  rg->base = __atomic_load_n(&rg->ctl[0], __ATOMIC_SEQ_CST);
  if (rg->base > 0xF0000000u) return fail(PGM_EINVAL, "rows_ring_start: batch counter exhausted (recreate the ring)");
  rg->n_batches = n_batches;
  rg->posted = 0;
  if (n_batches == 0) return PGM_OK;
  const double *v = rg->h->d_values;
  const PgmRingSlot *d = rg->d_slots;
  unsigned ns = rg->n_slots, nb = n_batches;
  unsigned *ctl = rg->ctl_dev, *gc = rg->gctl;
  unsigned base = rg->base;
  long long n = rg->n_rows;
  int32_t *ef = rg->err;
  int32_t md = rg->mode;
  int sg = signal;
  void *args[] = {(void *)&v, (void *)&d, &ns, (void *)&ctl, (void *)&gc, &nb, &base, &n, (void *)&ef, &md, &ticks, &sg};
  if (rg->reset_gctl) {  // mirror = base, token free, stop clear, readiness count 0
    unsigned init[16] = {base, 0u, 0u};
    HIP_TRY(hipMemcpyAsync(rg->gctl, init, sizeof init, hipMemcpyHostToDevice, rg->stream));
    HIP_TRY(hipStreamSynchronize(rg->stream));
    rg->reset_gctl = false;
  }
  HIP_TRY(hipModuleLaunchKernel(rg->h->jit_fn_ring, rg->blocks, 1, 1, (unsigned)ring_wg(), 1, 1, 0, rg->stream, args,
                                nullptr));
  rg->running = true;
  return PGM_OK;
}

int pgm_rows_ring_post(void *ring, uint32_t n_posted) {
  RowsRing *rg = (RowsRing *)ring;
  if (!rg) return fail(PGM_EINVAL, "rows_ring_post: null ring");
  if (!rg->running) return fail(PGM_EINVAL, "rows_ring_post: the ring is not running");
  rg->posted = std::max(rg->posted, __atomic_load_n(&rg->ctl[0], __ATOMIC_SEQ_CST) - rg->base);  // direct stores
  if (n_posted < rg->posted || n_posted > rg->n_batches)
    return fail(PGM_EINVAL, "rows_ring_post: %u batches posted, %u started, asked for %u", rg->posted, rg->n_batches,
                n_posted);
  rg->posted = n_posted;
  // a sequentially consistent store: drained from the store buffer before this call returns
  __atomic_store_n(&rg->ctl[0], rg->base + n_posted, __ATOMIC_SEQ_CST);
  return PGM_OK;
}

static int ring_wait(RowsRing *rg) {
  HIP_TRY(hipStreamSynchronize(rg->stream));
  rg->running = false;
  return PGM_OK;
}

int pgm_rows_ring_finish(void *ring) {
  STALE_PROBE();
  RowsRing *rg = (RowsRing *)ring;
  if (!rg) return fail(PGM_EINVAL, "rows_ring_finish: null ring");
  if (!rg->running) return PGM_OK;
  rg->posted = std::max(rg->posted, __atomic_load_n(&rg->ctl[0], __ATOMIC_SEQ_CST) - rg->base);  // direct stores
  if (rg->posted < rg->n_batches)
    return fail(PGM_EINVAL, "rows_ring_finish: only %u of %u batches posted (post them or cancel)", rg->posted,
                rg->n_batches);
  const int st = ring_wait(rg);
  if (st != PGM_OK) return st;
  if (__atomic_load_n(&rg->ctl[2], __ATOMIC_SEQ_CST) & 2u) {
    rg->reset_gctl = true;
    return fail(PGM_EDEVICE, "rows_ring_finish: the resident kernel timed out waiting for a batch");
  }
  return PGM_OK;
}

int pgm_rows_ring_cancel(void *ring) {
  STALE_PROBE();
  RowsRing *rg = (RowsRing *)ring;
  if (!rg) return fail(PGM_EINVAL, "rows_ring_cancel: null ring");
  if (!rg->running) return PGM_OK;
  __atomic_store_n(&rg->ctl[1], 1u, __ATOMIC_SEQ_CST);
  rg->reset_gctl = true;
  return ring_wait(rg);
}

int pgm_rows_ring_counter(void *ring, uint32_t **counter, uint32_t *base) {
  RowsRing *rg = (RowsRing *)ring;
  if (!rg || !counter || !base) return fail(PGM_EINVAL, "rows_ring_counter: null argument");
  *counter = rg->ctl;
  *base = rg->base;
  return PGM_OK;
}

int pgm_rows_ring_kernel(void *ring, char *name, size_t cap, uint32_t *blocks, uint32_t *wg) {
  RowsRing *rg = (RowsRing *)ring;
  if (!rg || !name || cap == 0) return fail(PGM_EINVAL, "rows_ring_kernel: null argument");
  snprintf(name, cap, "%s", "pgm_rows_ring");
  if (blocks) *blocks = rg->blocks;
  if (wg) *wg = (uint32_t)ring_wg();
  return PGM_OK;
}

int pgm_rows_ring_destroy(void *ring) {
  STALE_PROBE();
  RowsRing *rg = (RowsRing *)ring;
  if (!rg) return PGM_OK;
  int st = PGM_OK;
  if (rg->running) st = pgm_rows_ring_cancel(rg);
  if (rg->d_slots) (void)hipFree(rg->d_slots);
  if (rg->gctl) (void)hipFree(rg->gctl);
  if (rg->ctl) (void)hipHostFree(rg->ctl);
  delete rg;
  return st;
}

// internal (pgm_internal.h): what the direct AQL path (pgmdq.cpp) needs to dispatch a bound
// specialised launch on its own queue; PGM_EINVAL when the bound launch is not the hipRTC kernel
int pgmi_rows_bound_jit(void *bound, pgmi_jit_launch *out) {
  RowsBound *b = (RowsBound *)bound;
  if (!b || !out) return fail(PGM_EINVAL, "rows_bound_jit: null argument");
  if (!b->fn) return fail(PGM_EINVAL, "direct launch needs the plan-specialised kernel (hipRTC), not an AOT kernel");
  RowsHandle *h = (RowsHandle *)b->handle;
  if (h->jit_code.empty()) return fail(PGM_EINVAL, "direct launch: no code object kept for this plan");
  out->code = h->jit_code.data();
  out->code_size = h->jit_code.size();
  out->kernel = b->fn == h->jit_fn2 ? "pgm_rows_jit2" : b->fn == h->jit_fn_floor ? "pgm_rows_floor" : b->fn == h->jit_fn_floor2 ? "pgm_rows_floor2" : "pgm_rows_jit";
  out->args = &b->args;
  out->args_size = b->args_size;
  out->blocks = b->blocks;
  out->wg = (unsigned)jit_wg();
  out->owner = h;
  out->write_through = h->jit_write_through ? 1 : 0;
  return PGM_OK;
}

int pgmi_fail(int code, const char *msg) { return fail(code, "%s", msg); }

int pgmi_failf(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return fail(code, "%s", buf);
}

}  // extern "C"
