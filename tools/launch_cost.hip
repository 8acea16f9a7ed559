// Host cost of a kernel launch: hipLaunchKernelGGL (AOT) vs hipModuleLaunchKernel (hipRTC module;
// args array or packed `extra` buffer).  Prints us per launch, host-measured, for back-to-back launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_cost tools/launch_cost.hip -lhiprtc
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto e = (x); if (e != 0) { printf("%s:%d err %d\n", __FILE__, __LINE__, (int)e); exit(1); } } while (0)

__global__ void k_aot(double *out, long long n) {
  long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r < n && out) out[r] = 1.0;
}

static const char *kSrc = "extern \"C\" __global__ void k_rtc(double *out, long long n) {\n"
                          "  long long r = (long long)blockIdx.x * 256 + threadIdx.x;\n"
                          "  if (r < n && out) out[r] = 1.0;\n}\n";

template <typename F>
static void bench(const char *name, F f, int reps) {
  for (int i = 0; i < 50; ++i) f();
  CK(hipDeviceSynchronize());
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  CK(hipDeviceSynchronize());
  auto t2 = std::chrono::steady_clock::now();
  printf("{\"launch\": \"%s\", \"host_us\": %.3f, \"wall_us\": %.3f}\n", name,
         std::chrono::duration<double, std::micro>(t1 - t0).count() / reps,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / reps);
}

int main() {
  hiprtcProgram prog;
  CK(hiprtcCreateProgram(&prog, kSrc, "k.hip", 0, nullptr, nullptr));
  const char *opts[] = {"--offload-arch=gfx950", "-O3"};
  CK(hiprtcCompileProgram(prog, 2, opts));
  size_t sz;
  CK(hiprtcGetCodeSize(prog, &sz));
  std::vector<char> code(sz);
  CK(hiprtcGetCode(prog, code.data()));
  hipModule_t mod;
  hipFunction_t fn;
  CK(hipModuleLoadData(&mod, code.data()));
  CK(hipModuleGetFunction(&fn, mod, "k_rtc"));
  double *out;
  long long n = 100000;
  CK(hipMalloc(&out, n * 8));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int reps = 2000;
  unsigned g = (unsigned)((n + 255) / 256);
  bench("aot hipLaunchKernelGGL null stream", [&] { hipLaunchKernelGGL(k_aot, dim3(g), dim3(256), 0, 0, out, n); }, reps);
  bench("aot hipLaunchKernelGGL stream", [&] { hipLaunchKernelGGL(k_aot, dim3(g), dim3(256), 0, s, out, n); }, reps);
  bench("module args stream", [&] {
    void *args[] = {&out, &n};
    hipModuleLaunchKernel(fn, g, 1, 1, 256, 1, 1, 0, s, args, nullptr);
  }, reps);
  struct { double *o; long long n; } pk{out, n};
  size_t psz = sizeof pk;
  bench("module extra stream", [&] {
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &pk, HIP_LAUNCH_PARAM_BUFFER_SIZE, &psz, HIP_LAUNCH_PARAM_END};
    hipModuleLaunchKernel(fn, g, 1, 1, 256, 1, 1, 0, s, nullptr, extra);
  }, reps);
  bench("module extra null stream", [&] {
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &pk, HIP_LAUNCH_PARAM_BUFFER_SIZE, &psz, HIP_LAUNCH_PARAM_END};
    hipModuleLaunchKernel(fn, g, 1, 1, 256, 1, 1, 0, 0, nullptr, extra);
  }, reps);
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  bench("module extra nonblocking stream", [&] {
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &pk, HIP_LAUNCH_PARAM_BUFFER_SIZE, &psz, HIP_LAUNCH_PARAM_END};
    hipModuleLaunchKernel(fn, g, 1, 1, 256, 1, 1, 0, s2, nullptr, extra);
  }, reps);
  bench("aot nonblocking stream", [&] { hipLaunchKernelGGL(k_aot, dim3(g), dim3(256), 0, s2, out, n); }, reps);
  return 0;
}
