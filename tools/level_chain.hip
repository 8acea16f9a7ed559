// Cost of one dependency level in a captured HIP graph (C2's 23-level contraction path is one launch
// per level): a chain of N dependent single-workgroup launches replayed as one graph, with 0..3
// dependent global loads before each level's store (kernel argument -> descriptor -> pointer -> data),
// and the same chain with 64 workgroups per level.  Prints us per level.
//   hipcc --offload-arch=gfx950 -O3 -o tools/level_chain tools/level_chain.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

static const size_t LV = 256 * 512;  // doubles per level (the widest grid: 512 blocks x 256)
#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct Desc {
  const double *const *src;  // -> pointer to the previous level's output
  double *dst;
};

// depth 0: store only; 1: read the previous level's value (data); 2: + a pointer load; 3: + a descriptor load
template <int DEPTH>
__global__ void k_level(const Desc *d, const double *prev, double *out, int level) {
  double v = 1.0;
  if (DEPTH == 1) v = prev[threadIdx.x] + 1.0;
  if (DEPTH == 2) {
    const double *p = *(const double *const *)prev;  // prev holds a pointer to the data
    v = p[threadIdx.x] + 1.0;
  }
  if (DEPTH == 3) {
    const Desc dd = d[level];
    v = (*dd.src)[threadIdx.x] + 1.0;
    out = dd.dst;
  }
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

// a ContractK-sized argument (640 B) passed by value, every word used (the generic contraction kernels
// take their descriptor this way)
struct Big {
  long long w[80];
};
__global__ void k_level_big(const Big b, const double *prev, double *out) {
  double v = prev[threadIdx.x];
#pragma unroll
  for (int i = 0; i < 80; ++i) v += (double)b.w[i];
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

static double run_big(int n_levels, int blocks, int reps) {
  double *buf;
  CK(hipMalloc(&buf, sizeof(double) * LV * (n_levels + 1)));
  CK(hipMemset(buf, 0, sizeof(double) * LV * (n_levels + 1)));
  Big b;
  for (int i = 0; i < 80; ++i) b.w[i] = i;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int l = 1; l <= n_levels; ++l)
    hipLaunchKernelGGL(k_level_big, dim3(blocks), dim3(256), 0, s, b, buf + (size_t)(l - 1) * LV, buf + (size_t)l * LV);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipStreamSynchronize(s));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  CK(hipFree(buf));
  return ms * 1e3 / reps / n_levels;
}

template <int DEPTH>
static double run(int n_levels, int blocks, int reps) {
  double *buf;
  CK(hipMalloc(&buf, sizeof(double) * LV * (n_levels + 1)));
  CK(hipMemset(buf, 0, sizeof(double) * LV * (n_levels + 1)));
  const double **ptrs;  // ptrs[l] = the data of level l
  CK(hipMalloc(&ptrs, sizeof(double *) * (n_levels + 1)));
  Desc *descs;
  CK(hipMalloc(&descs, sizeof(Desc) * (n_levels + 1)));
  const double *hp[256];
  Desc hd[256];
  for (int l = 0; l <= n_levels; ++l) {
    hp[l] = buf + (size_t)l * LV;
    hd[l].src = ptrs + (l ? l - 1 : 0);
    hd[l].dst = buf + (size_t)l * LV;
  }
  CK(hipMemcpy(ptrs, hp, sizeof(double *) * (n_levels + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(descs, hd, sizeof(Desc) * (n_levels + 1), hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int l = 1; l <= n_levels; ++l) {
    const double *prev = DEPTH == 2 ? (const double *)(ptrs + l - 1) : buf + (size_t)(l - 1) * LV;
    hipLaunchKernelGGL(k_level<DEPTH>, dim3(blocks), dim3(256), 0, s, descs, prev, buf + (size_t)l * LV, l);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipStreamSynchronize(s));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  {  // host time of one hipGraphLaunch call on an idle stream, and launch -> completion
    double h = 0, w = 0;
    for (int i = 0; i < 20; ++i) {
      auto t0 = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(ge, s));
      auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(s));
      auto t2 = std::chrono::steady_clock::now();
      h += std::chrono::duration<double, std::micro>(t1 - t0).count();
      w += std::chrono::duration<double, std::micro>(t2 - t0).count();
    }
    if (DEPTH == 1 && blocks == 1)
      printf("  one %d-node graph: hipGraphLaunch host %.1f us, launch -> synchronized %.1f us\n", n_levels, h / 20,
             w / 20);
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  CK(hipFree(buf));
  CK(hipFree(ptrs));
  CK(hipFree(descs));
  return ms * 1e3 / reps / n_levels;
}

int main() {
  const int n = 24, reps = 200;
  for (int blocks : {1, 64, 512}) {
    printf("blocks %3d: depth0 %.2f us/level  depth1 %.2f  depth2 %.2f  depth3 %.2f\n", blocks, run<0>(n, blocks, reps),
           run<1>(n, blocks, reps), run<2>(n, blocks, reps), run<3>(n, blocks, reps));
  }
  for (int blocks : {1, 64})
    printf("blocks %3d: 640-B by-value argument %.2f us/level\n", blocks, run_big(n, blocks, reps));
  return 0;
}
