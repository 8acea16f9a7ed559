// Launch-floor microbenchmark for the C3 row kernel's shape (100k rows, 7 uint8 evidence
// columns in, 17 fp64 marginal columns out, column-major).  Decomposes the fused row kernel's
// per-launch time into launch/drain floor, store floor and load->store chain.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/floor tools/floor.hip && ./tools/floor [rows]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_empty(int *flag) {
  if (flag && threadIdx.x == 1023) flag[0] = 1;
}

// lane = row, NCOL output columns, RPL rows per lane (strided by blockDim*grid)
template <int NCOL, int RPL>
__global__ void k_store(double *out, int64_t n, int64_t ld) {
#pragma unroll
  for (int k = 0; k < RPL; ++k) {
    int64_t r = ((int64_t)blockIdx.x * RPL + k) * blockDim.x + threadIdx.x;
    if (r < n) {
#pragma unroll
      for (int c = 0; c < NCOL; ++c) __builtin_nontemporal_store((double)c, out + c * ld + r);
    }
  }
}

// write-through stores (relaxed agent-scope atomic store = global_store ... sc1), as the specialised
// row kernel's default output form
template <int NCOL, int RPL>
__global__ void k_store_wt(double *out, int64_t n, int64_t ld) {
#pragma unroll
  for (int k = 0; k < RPL; ++k) {
    int64_t r = ((int64_t)blockIdx.x * RPL + k) * blockDim.x + threadIdx.x;
    if (r < n) {
#pragma unroll
      for (int c = 0; c < NCOL; ++c)
        __hip_atomic_store((__attribute__((address_space(1))) double *)(out + c * ld + r), (double)c,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int NCOL, int RPL>
__global__ void k_store_plain(double *out, int64_t n, int64_t ld) {
#pragma unroll
  for (int k = 0; k < RPL; ++k) {
    int64_t r = ((int64_t)blockIdx.x * RPL + k) * blockDim.x + threadIdx.x;
    if (r < n) {
#pragma unroll
      for (int c = 0; c < NCOL; ++c) out[c * ld + r] = (double)c;
    }
  }
}

// 7 code loads -> 17 stores depending on them
template <int NCOL>
__global__ void k_load_store(const uint8_t *codes, int64_t ldc, double *out, int64_t n, int64_t ld) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 7; ++j) s += codes[j * ldc + r];
  const double v = (double)s;
#pragma unroll
  for (int c = 0; c < NCOL; ++c) __builtin_nontemporal_store(v + c, out + c * ld + r);
}


// the fused row kernel's shape step by step: 1563 x 192 (one wave per component, 3 components
// storing 6/5/6 columns); DESC: column offsets read from a device descriptor (dependent s_load);
// LDS: 240 doubles per wave staged from global and gathered by the codes
struct Desc { int32_t col[4]; int32_t ncol; int32_t vlo; int32_t pad[2]; };
template <bool DESC, bool LDS>
__global__ __launch_bounds__(192) void k_shape(const uint8_t *codes, int64_t ldc, const Desc *desc, const double *vals,
                                               double *out, int64_t n, int64_t ld) {
  __shared__ double sv[3 * 256];
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int32_t col[4], ncol, vlo;
  if (DESC) {
    const Desc &d = desc[c];
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j] = d.col[j];
    ncol = d.ncol;
    vlo = d.vlo;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j] = c * 2 + (j & 1);
    ncol = c == 1 ? 5 : 6;
    vlo = c * 256;
  }
  if (LDS) {
    for (int i = lane; i < 240; i += 64) sv[c * 256 + i] = vals[vlo + i];
  }
  const int64_t r = (int64_t)blockIdx.x * 64 + lane;
  const uint8_t *cr = codes + (r < n ? r : 0);
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += cr[(int64_t)col[j] * ldc];
  double v = (double)s;
  if (LDS) v = sv[c * 256 + (s & 31)] * sv[c * 256 + 32 + (s & 63)];
  if (r < n) {
    double *o = out + (int64_t)(c * 6) * ld + r;
    for (int q = 0; q < ncol; ++q) __builtin_nontemporal_store(v + q, o + (int64_t)q * ld);
  }
}


// kernarg / LDS / block-shape sensitivity: the row kernel's launch envelope with store-only bodies
struct BigArg { int32_t v[32]; };
template <bool BIG, bool DYN>
__global__ __launch_bounds__(768) void k_env(const BigArg a, const Desc *desc, double *out, int64_t n, int64_t ld) {
  extern __shared__ double dl[];
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r = (int64_t)blockIdx.x * 64 + lane;
  int ncol = c == 1 ? 5 : 6;
  double v = 1.0;
  if (BIG) v += a.v[c];
  if (DYN) { dl[threadIdx.x] = v; v += dl[threadIdx.x ^ 1]; }
  if (r < n) {
    double *o = out + (int64_t)(c * 6) * ld + r;
    for (int q = 0; q < ncol; ++q) __builtin_nontemporal_store(v + q, o + (int64_t)q * ld);
  }
}


// instruction-footprint sensitivity: the store body behind N straight-line s_nop (4 B each)
template <int N>
__global__ __launch_bounds__(192) void k_bigcode(double *out, int64_t n, int64_t ld) {
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r = (int64_t)blockIdx.x * 64 + lane;
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("s_nop 0");
  if (r < n) {
    double *o = out + (int64_t)(c * 6) * ld + r;
#pragma unroll
    for (int q = 0; q < 6; ++q) __builtin_nontemporal_store((double)q, o + (int64_t)q * ld);
  }
}

template <typename F>
static void timeit(const char *name, F launch, int reps, double bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 10; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  double us = ms * 1e3 / reps;
  printf("{\"kernel\": \"%s\", \"us_per_launch\": %.3f, \"GBps\": %.1f}\n", name, us, bytes / (us * 1e3));
  CK(hipGetLastError());
}

int main(int argc, char **argv) {
  int64_t n = argc > 1 ? atoll(argv[1]) : 100000;
  const int reps = 200;
  double *out;
  uint8_t *codes;
  CK(hipMalloc(&out, 17 * n * sizeof(double)));
  CK(hipMalloc(&codes, 7 * n));
  CK(hipMemset(codes, 1, 7 * n));
  const double sb = 17.0 * 8 * n, lb = sb + 7.0 * n;
  int g64 = (int)((n + 63) / 64);
  timeit("empty 1563x192", [&] { hipLaunchKernelGGL(k_empty, dim3(g64), dim3(192), 0, 0, nullptr); }, reps, 0);
  timeit("empty 1x64", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, nullptr); }, reps, 0);
  timeit("store nt wg64", [&] { hipLaunchKernelGGL((k_store<17, 1>), dim3(g64), dim3(64), 0, 0, out, n, n); }, reps, sb);
  timeit("store plain wg64", [&] { hipLaunchKernelGGL((k_store_plain<17, 1>), dim3(g64), dim3(64), 0, 0, out, n, n); }, reps, sb);
  timeit("store wt wg256", [&] { hipLaunchKernelGGL((k_store_wt<17, 1>), dim3((n + 255) / 256), dim3(256), 0, 0, out, n, n); }, reps, sb);
  timeit("store wt wg128", [&] { hipLaunchKernelGGL((k_store_wt<17, 1>), dim3((n + 127) / 128), dim3(128), 0, 0, out, n, n); }, reps, sb);
  timeit("store nt wg256", [&] { hipLaunchKernelGGL((k_store<17, 1>), dim3((n + 255) / 256), dim3(256), 0, 0, out, n, n); }, reps, sb);
  timeit("store plain wg256", [&] { hipLaunchKernelGGL((k_store_plain<17, 1>), dim3((n + 255) / 256), dim3(256), 0, 0, out, n, n); }, reps, sb);
  timeit("store nt wg256 rpl2", [&] { hipLaunchKernelGGL((k_store<17, 2>), dim3((n + 511) / 512), dim3(256), 0, 0, out, n, n); }, reps, sb);
  timeit("store plain wg256 rpl2", [&] { hipLaunchKernelGGL((k_store_plain<17, 2>), dim3((n + 511) / 512), dim3(256), 0, 0, out, n, n); }, reps, sb);
  timeit("store nt wg1024", [&] { hipLaunchKernelGGL((k_store<17, 1>), dim3((n + 1023) / 1024), dim3(1024), 0, 0, out, n, n); }, reps, sb);
  timeit("load+store wg64", [&] { hipLaunchKernelGGL((k_load_store<17>), dim3(g64), dim3(64), 0, 0, codes, n, out, n, n); }, reps, lb);
  timeit("load+store wg256", [&] { hipLaunchKernelGGL((k_load_store<17>), dim3((n + 255) / 256), dim3(256), 0, 0, codes, n, out, n, n); }, reps, lb);
  Desc hd[3];
  for (int c = 0; c < 3; ++c) { for (int j = 0; j < 4; ++j) hd[c].col[j] = c * 2 + (j & 1); hd[c].ncol = c == 1 ? 5 : 6; hd[c].vlo = c * 256; }
  Desc *dd; double *vals;
  CK(hipMalloc(&dd, sizeof(hd)));
  CK(hipMemcpy(dd, hd, sizeof(hd), hipMemcpyHostToDevice));
  CK(hipMalloc(&vals, 1024 * sizeof(double)));
  CK(hipMemset(vals, 0, 1024 * sizeof(double)));
  timeit("shape 192 plain", [&] { hipLaunchKernelGGL((k_shape<false, false>), dim3(g64), dim3(192), 0, 0, codes, n, dd, vals, out, n, n); }, reps, lb);
  timeit("shape 192 desc", [&] { hipLaunchKernelGGL((k_shape<true, false>), dim3(g64), dim3(192), 0, 0, codes, n, dd, vals, out, n, n); }, reps, lb);
  timeit("shape 192 lds", [&] { hipLaunchKernelGGL((k_shape<false, true>), dim3(g64), dim3(192), 0, 0, codes, n, dd, vals, out, n, n); }, reps, lb);
  timeit("shape 192 desc+lds", [&] { hipLaunchKernelGGL((k_shape<true, true>), dim3(g64), dim3(192), 0, 0, codes, n, dd, vals, out, n, n); }, reps, lb);
  {  // the same kernel reading 7 columns spread over a 1035-column evidence matrix (as the bench stores it)
    uint8_t *big;
    CK(hipMalloc(&big, 1035 * n));
    CK(hipMemset(big, 1, 1035 * n));
    Desc hs[3];
    const int cols[12] = {17, 171, 333, 402, 590, 611, 777, 801, 950, 1000, 1020, 1034};
    for (int c = 0; c < 3; ++c) { for (int j = 0; j < 4; ++j) hs[c].col[j] = cols[c * 4 + j]; hs[c].ncol = c == 1 ? 5 : 6; hs[c].vlo = c * 256; }
    Desc *ds;
    CK(hipMalloc(&ds, sizeof(hs)));
    CK(hipMemcpy(ds, hs, sizeof(hs), hipMemcpyHostToDevice));
    timeit("shape 192 desc+lds scattered cols", [&] { hipLaunchKernelGGL((k_shape<true, true>), dim3(g64), dim3(192), 0, 0, big, n, ds, vals, out, n, n); }, reps, lb);
    CK(hipFree(big));
  }
  {
    BigArg ba;
    for (int i = 0; i < 32; ++i) ba.v[i] = i;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    timeit("env small", [&] { hipLaunchKernelGGL((k_env<false, false>), dim3(g64), dim3(192), 0, 0, ba, dd, out, n, n); }, reps, sb);
    timeit("env bigarg", [&] { hipLaunchKernelGGL((k_env<true, false>), dim3(g64), dim3(192), 0, 0, ba, dd, out, n, n); }, reps, sb);
    timeit("env dynlds 9.6K", [&] { hipLaunchKernelGGL((k_env<false, true>), dim3(g64), dim3(192), 9600, 0, ba, dd, out, n, n); }, reps, sb);
    timeit("env bigarg+dynlds", [&] { hipLaunchKernelGGL((k_env<true, true>), dim3(g64), dim3(192), 9600, 0, ba, dd, out, n, n); }, reps, sb);
    timeit("env bigarg+dynlds stream", [&] { hipLaunchKernelGGL((k_env<true, true>), dim3(g64), dim3(192), 9600, st, ba, dd, out, n, n); }, reps, sb);
    timeit("shape desc+lds stream", [&] { hipLaunchKernelGGL((k_shape<true, true>), dim3(g64), dim3(192), 0, st, codes, n, dd, vals, out, n, n); }, reps, lb);
  }
  timeit("bigcode 0 nops", [&] { hipLaunchKernelGGL((k_bigcode<0>), dim3(g64), dim3(192), 0, 0, out, n, n); }, reps, sb);
  timeit("bigcode 256 nops (1 KB)", [&] { hipLaunchKernelGGL((k_bigcode<256>), dim3(g64), dim3(192), 0, 0, out, n, n); }, reps, sb);
  timeit("bigcode 1024 nops (4 KB)", [&] { hipLaunchKernelGGL((k_bigcode<1024>), dim3(g64), dim3(192), 0, 0, out, n, n); }, reps, sb);
  timeit("bigcode 2048 nops (8 KB)", [&] { hipLaunchKernelGGL((k_bigcode<2048>), dim3(g64), dim3(192), 0, 0, out, n, n); }, reps, sb);
  timeit("bigcode 1024 nops 1 block", [&] { hipLaunchKernelGGL((k_bigcode<1024>), dim3(1), dim3(192), 0, 0, out, 64, n); }, reps, 0);
  timeit("bigcode 0 nops 1 block", [&] { hipLaunchKernelGGL((k_bigcode<0>), dim3(1), dim3(192), 0, 0, out, 64, n); }, reps, 0);
  timeit("memset out", [&] { CK(hipMemsetAsync(out, 0, 17 * n * sizeof(double), 0)); }, reps, sb);
  CK(hipFree(out));
  CK(hipFree(codes));
  return 0;
}
