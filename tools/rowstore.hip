// Write-rate microbenchmark for the batched-BP row layout: out[o][x], x = evidence row (1000),
// o = clique outer index (32,256) -> 258 MB per pass.  Block shapes as k_productn_rows2 uses them.
//   hipcc --offload-arch=gfx950 -O3 -o tools/rowstore tools/rowstore.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%d %s\n", __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

// one block per outer index (grid.y), pairs of rows across threads
__global__ void k_rowstore2(double *C, int NX, int n_outer) {
  const int NP = NX / 2;
  for (int o = blockIdx.y; o < n_outer; o += gridDim.y) {
    double2 *c2 = (double2 *)(C + (long long)o * NX);
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < NP; x += gridDim.x * blockDim.x) c2[x] = make_double2(1.0, 2.0);
  }
}
// flat: thread per pair over the whole tensor
__global__ void k_flatstore2(double *C, long long npairs) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += (long long)gridDim.x * blockDim.x)
    ((double2 *)C)[i] = make_double2(1.0, 2.0);
}
// read A (same shape) and write C: the in-place update's traffic
__global__ void k_rowcopy2(const double *A, double *C, int NX, int n_outer) {
  const int NP = NX / 2;
  for (int o = blockIdx.y; o < n_outer; o += gridDim.y) {
    const double2 *a2 = (const double2 *)(A + (long long)o * NX);
    double2 *c2 = (double2 *)(C + (long long)o * NX);
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < NP; x += gridDim.x * blockDim.x) {
      double2 v = a2[x];
      v.x *= 1.0000001;
      v.y *= 1.0000001;
      c2[x] = v;
    }
  }
}

template <typename F>
static void timeit(const char *name, F f, double bytes) {
  for (int i = 0; i < 3; ++i) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < 10; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"kernel\": \"%s\", \"us\": %.1f, \"TBps\": %.2f}\n", name, ms * 100, bytes / (ms * 1e-4) / 1e12);
}

int main() {
  const int NX = 1000, n_outer = 32256;
  const long long n = (long long)NX * n_outer;
  double *C, *A;
  CK(hipMalloc(&C, n * 8));
  CK(hipMalloc(&A, n * 8));
  CK(hipMemset(A, 0, n * 8));
  const double wb = n * 8.0;
  timeit("rowstore2 grid(1,32256)x256", [&] { hipLaunchKernelGGL(k_rowstore2, dim3(1, n_outer), dim3(256), 0, 0, C, NX, n_outer); }, wb);
  timeit("rowstore2 grid(1,32256)x512", [&] { hipLaunchKernelGGL(k_rowstore2, dim3(1, n_outer), dim3(512), 0, 0, C, NX, n_outer); }, wb);
  timeit("rowstore2 grid(1,4096)x512", [&] { hipLaunchKernelGGL(k_rowstore2, dim3(1, 4096), dim3(512), 0, 0, C, NX, n_outer); }, wb);
  timeit("flatstore2 2048x256", [&] { hipLaunchKernelGGL(k_flatstore2, dim3(2048), dim3(256), 0, 0, C, n / 2); }, wb);
  timeit("flatstore2 full x256", [&] { hipLaunchKernelGGL(k_flatstore2, dim3((unsigned)((n / 2 + 255) / 256)), dim3(256), 0, 0, C, n / 2); }, wb);
  timeit("memset", [&] { CK(hipMemsetAsync(C, 0, n * 8, 0)); }, wb);
  timeit("rowcopy2 grid(1,32256)x256", [&] { hipLaunchKernelGGL(k_rowcopy2, dim3(1, n_outer), dim3(256), 0, 0, A, C, NX, n_outer); }, 2 * wb);
  timeit("rowcopy2 inplace grid(1,32256)x256", [&] { hipLaunchKernelGGL(k_rowcopy2, dim3(1, n_outer), dim3(256), 0, 0, C, C, NX, n_outer); }, 2 * wb);
  timeit("memcpy d2d", [&] { CK(hipMemcpyAsync(C, A, n * 8, hipMemcpyDeviceToDevice, 0)); }, 2 * wb);
  return 0;
}
