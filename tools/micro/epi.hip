// Epilogue micro-benchmark: the ring GEMM kernel's row-major epilogue (256 x 256 tile, 8 waves,
// 4 bands of 64 rows through LDS, 16-B bf16 stores), built up step by step to find what makes
// its store phase take ~17 us per workgroup in the GEMM (stores alone: ~5 us).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ unsigned short bf(float v) { return __builtin_bit_cast(unsigned short, __float2bfloat16(v)); }

// flags: 1 LDS writer + barrier, 2 LDS reads, 4 partial last chunk (N = 500), 8 tanh-ish math,
// 16 a bf16 operand row per pass (loaded at band start), 32 BCE math (sigmoid, one log, dU),
// 64 BCE row partial (xor-shuffle tree + 4-B store per 16 lanes)
template <int FL>
__global__ __launch_bounds__(512, 1) void epi(unsigned short* out, int ld, int N, int M, float seed,
                                               const unsigned short* x, float* rowpart) {
  __shared__ __attribute__((aligned(16))) float lds[2 * 64 * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 2, wn = wave & 3;
  const int ntn = 2, b = blockIdx.x, m0 = (b / ntn) * 256, n0 = (b % ntn) * 256;
  f32x16 acc[4][2];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = seed * (i + 1) + j * r + lane;
  const int c8 = tid & 31, rr = tid >> 5;
  const int col0 = n0 + 8 * c8;
#pragma unroll 1
  for (int mi = 0; mi < 4; ++mi) {
    float* band = lds + (mi & 1) * 64 * 256;
    uint4 xb[4];
    if constexpr (FL & 16) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int br = rr + 16 * q;
        const int row = m0 + (br >> 5) * 128 + mi * 32 + (br & 31);
        xb[q] = *reinterpret_cast<const uint4*>(x + (size_t)row * ld + col0);
      }
    }
    if constexpr (FL & 1) {
      for (int ni = 0; ni < 2; ++ni)
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          band[row * 256 + wn * 64 + ni * 32 + (lane & 31)] = acc[0][ni][r];
        }
      for (int j = 0; j < 3; ++j)
        for (int ni = 0; ni < 2; ++ni) acc[j][ni] = acc[j + 1][ni];
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int br = rr + 16 * q;
      const int row = m0 + (br >> 5) * 128 + mi * 32 + (br & 31);
      float v[8];
      if constexpr (FL & 2) {
        const float4 a = *reinterpret_cast<const float4*>(band + br * 256 + 8 * c8);
        const float4 c = *reinterpret_cast<const float4*>(band + br * 256 + 8 * c8 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
      } else {
        for (int j = 0; j < 8; ++j) v[j] = seed + j + q;
      }
      if constexpr (FL & 8) {
        for (int j = 0; j < 8; ++j) v[j] = 1.f - 2.f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(v[j] * 2.885f) + 1.f);
      }
      float rs = 0.f;
      if constexpr (FL & 32) {
        float sv[8];
        const unsigned ww[4] = {xb[q].x, xb[q].y, xb[q].z, xb[q].w};
        for (int j = 0; j < 4; ++j) { sv[2 * j] = __uint_as_float(ww[j] << 16); sv[2 * j + 1] = __uint_as_float(ww[j] & 0xffff0000u); }
        for (int j = 0; j < 8; ++j) {
          const float y = __builtin_amdgcn_rcpf(1.f + __expf(-v[j]));
          rs += __logf(sv[j] != 0.f ? y : 1.f - y);
          v[j] = (y - sv[j]) * 1e-4f;
        }
      } else if constexpr (FL & 16) {
        v[0] += __uint_as_float(xb[q].x);
      }
      if constexpr (FL & 64) {
        for (int off = 8; off >= 1; off >>= 1) rs += __shfl_xor(rs, off, 64);
        if ((c8 & 15) == 0) rowpart[(size_t)row * 4 + (c8 >> 4)] = -rs;
      }
      const int nv = row >= M ? 0 : (col0 >= N ? 0 : (N - col0 < 8 ? N - col0 : 8));
      unsigned short* o = out + (size_t)row * ld + col0;
      if (nv == 8) {
        unsigned w[4];
        for (int j = 0; j < 4; ++j) w[j] = (unsigned)bf(v[2 * j]) | (unsigned)bf(v[2 * j + 1]) << 16;
        *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
      } else if (FL & 4) {
        for (int j = 0; j < nv; ++j) o[j] = bf(v[j]);
      }
    }
  }
}

template <int FL>
static void run(const char* name, unsigned short* out, int N, const unsigned short* x = nullptr,
                float* rp = nullptr) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int M = 24576, nwg = 192, ld = 504;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(epi<FL>, dim3(nwg), dim3(512), 0, 0, out, ld, N, M, 0.5f, x, rp);
  CK(hipEventRecord(a));
  const int it = 20;
  for (int w = 0; w < it; ++w) hipLaunchKernelGGL(epi<FL>, dim3(nwg), dim3(512), 0, 0, out, ld, N, M, 0.5f, x, rp);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("%-40s N %d  %8.2f us per launch\n", name, N, ms * 1e3 / it);
}

int main() {
  unsigned short* out;
  CK(hipMalloc(&out, (size_t)24576 * 504 * 2));
  run<0>("stores only", out, 512);
  run<0>("stores only", out, 500);
  run<2>("+ LDS reads", out, 512);
  run<3>("+ LDS writer/barrier", out, 512);
  run<7>("+ partial chunk", out, 500);
  run<15>("+ math", out, 500);
  run<11>("writer+reads+math, no partial", out, 512);
  unsigned short* x; float* rp;
  CK(hipMalloc(&x, (size_t)24576 * 504 * 2));
  CK(hipMemset(x, 0, (size_t)24576 * 504 * 2));
  CK(hipMalloc(&rp, (size_t)24576 * 4 * 4));
  run<3 | 2 | 16>("writer+reads + operand loads", out, 512, x, rp);
  run<3 | 2 | 16 | 32>("+ BCE math", out, 512, x, rp);
  run<3 | 2 | 16 | 32 | 64>("+ BCE row partials", out, 512, x, rp);
  run<3 | 2 | 16 | 64>("operand + row partials, no BCE math", out, 512, x, rp);
  return 0;
}
