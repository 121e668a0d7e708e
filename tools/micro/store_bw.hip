// Store-throughput micro-benchmark: the GEMM epilogue's write pattern (a 256 x 256 bf16 tile
// per workgroup, 16-B stores, one wave = 2 rows x 512 B) vs contiguous 128-KB blocks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// mode 0: tile rows (ld elements per row), mode 1: contiguous block per workgroup
__global__ __launch_bounds__(512) void store_tile(unsigned short* out, int ld, int mode, int ntn, int passes) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int c8 = tid & 31, rr = tid >> 5;  // 16 rows per pass
  uint4 v = make_uint4(b, tid, 7, 9);
  if (mode == 0) {
    const int m0 = (b / ntn) * 256, n0 = (b % ntn) * 256;
    for (int q = 0; q < passes; ++q) {
      const int row = m0 + rr + 16 * q;
      *reinterpret_cast<uint4*>(out + (size_t)row * ld + n0 + 8 * c8) = v;
    }
  } else {
    unsigned short* base = out + (size_t)b * passes * 512 * 8;
    for (int q = 0; q < passes; ++q)
      *reinterpret_cast<uint4*>(base + ((size_t)q * 512 + tid) * 8) = v;
  }
}

int main() {
  const int M = 24576;
  unsigned short* out;
  CK(hipMalloc(&out, (size_t)M * 1024 * 2));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  struct Cfg { const char* name; int ld, mode, nwg, ntn; } cfgs[] = {
      {"tile ld504 192wg", 504, 0, 192, 2}, {"tile ld512 192wg", 512, 0, 192, 2},
      {"tile ld504 256wg (M=32768 rows)", 504, 0, 256, 2}, {"linear 192wg", 0, 1, 192, 2},
      {"linear 256wg", 0, 1, 256, 2}};
  for (auto& c : cfgs) {
    const int passes = 16;  // 256 rows
    const int nwg = c.nwg;
    if (c.mode == 0 && (nwg / c.ntn) * 256 > M + 8192) continue;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(store_tile, dim3(nwg), dim3(512), 0, 0, out, c.ld, c.mode, c.ntn, passes);
    CK(hipEventRecord(a));
    const int it = 20;
    for (int w = 0; w < it; ++w) hipLaunchKernelGGL(store_tile, dim3(nwg), dim3(512), 0, 0, out, c.ld, c.mode, c.ntn, passes);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = (double)nwg * 512 * 16 * passes;
    printf("%-34s %8.2f us  %7.2f MB  %6.2f TB/s\n", c.name, ms * 1e3 / it, bytes / 1e6, bytes / (ms * 1e-3 / it) / 1e12);
  }
  return 0;
}
