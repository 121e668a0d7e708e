// Cold instruction-fetch micro-benchmark: a kernel that runs N straight-line VALU instructions
// once per wave (as a fully unrolled GEMM epilogue does) vs the same count in a small loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int N>
__global__ __launch_bounds__(512) void straight(float* out) {
  float a = threadIdx.x, b = 1.0001f;
  asm volatile(".rept %2\n\tv_fma_f32 %0, %0, %1, %1\n\t.endr" : "+v"(a) : "v"(b), "i"(N));
  if (a == 12345.f) out[threadIdx.x] = a;
}
template <int N>
__global__ __launch_bounds__(512) void looped(float* out) {
  float a = threadIdx.x, b = 1.0001f;
  for (int i = 0; i < N / 64; ++i) {
    asm volatile(".rept 64\n\tv_fma_f32 %0, %0, %1, %1\n\t.endr" : "+v"(a) : "v"(b));
  }
  if (a == 12345.f) out[threadIdx.x] = a;
}

template <typename F>
static void run(const char* name, F k, int nwg, float* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(nwg), dim3(512), 0, 0, out);
  CK(hipDeviceSynchronize());
  // one launch at a time: each launch sees a cold instruction cache only if the code is evicted;
  // time single launches bracketed by events
  float tot = 0.f;
  const int it = 20;
  for (int w = 0; w < it; ++w) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k, dim3(nwg), dim3(512), 0, 0, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  printf("%-28s %4d WGs %9.2f us\n", name, nwg, tot * 1e3 / it);
}

int main() {
  float* out;
  CK(hipMalloc(&out, 4096 * 4));
  for (int nwg : {256, 192}) {
    run("straight 64", straight<64>, nwg, out);
    run("straight 1024 (8 KB)", straight<1024>, nwg, out);
    run("straight 4096 (32 KB)", straight<4096>, nwg, out);
    run("straight 8192 (64 KB)", straight<8192>, nwg, out);
    run("looped 1024", looped<1024>, nwg, out);
    run("looped 4096", looped<4096>, nwg, out);
    run("looped 8192", looped<8192>, nwg, out);
  }
  return 0;
}
