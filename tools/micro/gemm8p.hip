// The 256^2 8-phase bf16 GEMM of cdna_hip_programming.md ("The 256^2 8-phase template", §5 T1-T5),
// written from the guide's specification as a yardstick for the library's eight-phase kernel
// (VERDICT r4 item 1a): C[M][N] (bf16) = A[M][K] . B^T where B is given as Bt[N][K] (both
// k-contiguous), uniform random [-1, 1) operands.
//
//   * 256 x 256 x 64 tile, 512 threads = 8 waves (2 M x 4 N), each wave 128 x 64 of
//     v_mfma_f32_16x16x32_bf16 accumulators (2 x 4 x 2 x 2 f32x4 = 128 registers);
//   * operand tiles as HALF images (128 rows x 64 k, 16 KB): half h of A = rows 64 h .. 64 h + 63 of
//     both wave rows, half h of B = columns 32 h .. 32 h + 31 of all four wave columns; 2 buffers
//     (even / odd k-tile) x {A0, A1, B0, B1} = 128 KB of LDS in ONE __shared__ array;
//   * images are [16-row block][32-k half] subtiles of 1024 B (one global_load_lds_dwordx4 wave
//     instruction each) with the st_16x32 swizzle byte ^= ((byte >> 9) & 1) << 5 applied to the
//     per-lane SOURCE address and undone on the ds_read_b128;
//   * a k-tile is 4 phases, one C-quadrant (64 x 32) x K = 64 = 16 MFMAs each:
//       p1 (0,0) reads B-sub 0 (4), sched_barrier, A-sub 0 (8); DMA A1(t+1); lgkmcnt(8)
//       p2 (0,1) reads B-sub 1 (4);                               DMA B0(t+2)
//       p3 (1,1) reads A-sub 1 (8);                               DMA A0(t+2)
//       p4 (1,0) reads nothing;                                   DMA B1(t+2); vmcnt(6)
//     each phase: reads + DMA -> s_barrier -> lgkmcnt(0) -> setprio 1, 16 MFMAs, setprio 0 ->
//     s_barrier; vmcnt(6) only in phases 4 and 8 (3 half-tiles = 6 DMA instructions stay in
//     flight across the barriers); waves 4-7 run one barrier behind waves 0-3;
//   * bijective XCD remap, then 4 x 8 tile groups per XCD.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/micro/gemm8p tools/micro/gemm8p.hip -ldl
// Run:   tools/micro/gemm8p [M N K] [--rounds R] [--iters I] [--lib magic_amd/libmvae.so]
//   prints per-round TF/s of the template (and, with --lib, of the library's eight-phase kernel
//   and its default plan on the same NT shape through mvae_bench_gemm, interleaved in the same
//   process), then the stamped build's in-kernel clock and cycles per k-tile.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) unsigned char lds_u8;

constexpr int HALF = 16384;  // bytes per half image
constexpr int NT = 512;

__host__ __device__ inline unsigned swz(unsigned b) { return b ^ (((b >> 9) & 1u) << 5); }

template <int OFF>
__device__ __forceinline__ bf16x8 rd(unsigned a) {
  s16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

struct Args {
  const unsigned short* A;
  const unsigned short* Bt;
  unsigned short* C;
  int M, N, K;
  unsigned long long* stamps;
  int gm;  // m-tiles per tile group (the guide's 4; the library's 8)
};

template <bool ST>
struct T8 {
  f32x4 acc[2][4][2][2];  // [m-sub][16-row block][n-sub][16-col block]
  bf16x8 fa0[8], fa1[8], fb0[4], fb1[4];  // [block * 2 + k-half]
  unsigned aA, aB;                         // fragment read bases (LDS byte addresses)
  const unsigned short* gA[2][2];          // [dma j][half h]: lane's source at k0 = 0
  const unsigned short* gB[2][2];
  unsigned char* smem;
  int wave;

  template <int H, int BF>
  __device__ __forceinline__ void dma_a(int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(gA[j][H] + kt * 64,
                                       (lds_u8*)(smem + (BF * 2 + H) * HALF + (j * 8 + wave) * 1024), 16, 0, 0);
  }
  template <int H, int BF>
  __device__ __forceinline__ void dma_b(int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(gB[j][H] + kt * 64,
                                       (lds_u8*)(smem + (4 + BF * 2 + H) * HALF + (j * 8 + wave) * 1024), 16, 0, 0);
  }
  template <int H, int BF>
  __device__ __forceinline__ void rd_a(bf16x8 (&f)[8]) {
    constexpr int O = (BF * 2 + H) * HALF;
    f[0] = rd<O + 0 * 1024>(aA); f[1] = rd<O + 1 * 1024>(aA);
    f[2] = rd<O + 2 * 1024>(aA); f[3] = rd<O + 3 * 1024>(aA);
    f[4] = rd<O + 4 * 1024>(aA); f[5] = rd<O + 5 * 1024>(aA);
    f[6] = rd<O + 6 * 1024>(aA); f[7] = rd<O + 7 * 1024>(aA);
  }
  template <int H, int BF>
  __device__ __forceinline__ void rd_b(bf16x8 (&f)[4]) {
    constexpr int O = (BF * 2 + H) * HALF;
    f[0] = rd<O + 0 * 1024>(aB); f[1] = rd<O + 1 * 1024>(aB);
    f[2] = rd<O + 2 * 1024>(aB); f[3] = rd<O + 3 * 1024>(aB);
  }
  template <int MS, int NS>
  __device__ __forceinline__ void mma(const bf16x8 (&fa)[8], const bf16x8 (&fb)[4]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[MS][mb][NS][nb] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mb * 2 + kh], fb[nb * 2 + kh], acc[MS][mb][NS][nb], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  // k-tile t in buffer BF (t + 1 in BF ^ 1, t + 2 back in BF)
  template <int BF>
  __device__ __forceinline__ void tile(int t, int nkt) {
    constexpr int BN = BF ^ 1;
    const bool h1 = t + 1 < nkt, h2 = t + 2 < nkt;
    // p1 (0,0)
    rd_b<0, BF>(fb0);
    __builtin_amdgcn_sched_barrier(0);
    rd_a<0, BF>(fa0);
    if (h1) dma_a<1, BN>(t + 1);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // the B-sub 0 reads: B0 is restaged in p2
    bar();
    mma<0, 0>(fa0, fb0);
    bar();
    // p2 (0,1)
    rd_b<1, BF>(fb1);
    if (h2) dma_b<0, BF>(t + 2);
    bar();
    mma<0, 1>(fa0, fb1);
    bar();
    // p3 (1,1)
    rd_a<1, BF>(fa1);
    if (h2) dma_a<0, BF>(t + 2);
    bar();
    mma<1, 1>(fa1, fb1);
    bar();
    // p4 (1,0)
    if (h2) {
      dma_b<1, BF>(t + 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // k-tile t + 1 landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    mma<1, 0>(fa1, fb0);
    bar();
  }
};

template <bool ST>
__global__ __launch_bounds__(NT, 1) void gemm8p_kernel(Args a) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[8 * HALF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int ntm = a.M / 256, ntn = a.N / 256, nwg = ntm * ntn;
  // bijective XCD remap (blocks b and b + 8 share an XCD), then groups of 4 m-tiles
  const int orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int GM = a.gm;
  const int grp = wg / (GM * ntn), first = grp * GM, gsz = min(ntm - first, GM);
  const int tm = first + (wg % (GM * ntn)) % gsz, tn = (wg % (GM * ntn)) / gsz;
  const int m0 = tm * 256, n0 = tn * 256;

  T8<ST> s;
  s.smem = smem;
  s.wave = __builtin_amdgcn_readfirstlane(wave);
  // DMA sources: wave instruction j covers subtile j * 8 + wave of a half image
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int sub = j * 8 + wave, rb = sub >> 1, kh = sub & 1;
    const unsigned p = swz(lane * 16);
    const int i = rb * 16 + (p >> 6), k = kh * 32 + ((p >> 4) & 3) * 8;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ra = (i >> 6) * 128 + h * 64 + (i & 63);
      const int cb = (i >> 5) * 64 + h * 32 + (i & 31);
      s.gA[j][h] = a.A + (size_t)(m0 + ra) * a.K + k;
      s.gB[j][h] = a.Bt + (size_t)(n0 + cb) * a.K + k;
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u8*)smem;
  const unsigned fo = swz((lane & 15) * 64 + (lane >> 4) * 16);
  s.aA = lds0 + (wm * 4) * 2 * 1024 + fo;
  s.aB = lds0 + 4 * HALF + (wn * 2) * 2 * 1024 + fo;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int l = 0; l < 2; ++l) s.acc[i][j][k][l] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = a.K / 64;
  const bool lag = __builtin_amdgcn_readfirstlane(wave) >= 4;
  // prologue: A0 B0 B1 A1 of k-tile 0, then B0 A0 B1 of k-tile 1 (its A1 goes in k-tile 0's p1)
  s.template dma_a<0, 0>(0);
  s.template dma_b<0, 0>(0);
  s.template dma_b<1, 0>(0);
  s.template dma_a<1, 0>(0);
  if (nkt > 1) {
    s.template dma_b<0, 1>(1);
    s.template dma_a<0, 1>(1);
    s.template dma_b<1, 1>(1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (lag) bar();
  unsigned long long t0 = 0, r0 = 0;
  if constexpr (ST) {
    r0 = __builtin_amdgcn_s_memrealtime();
    t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int t = 0; t < nkt; t += 2) {
    s.template tile<0>(t, nkt);
    if (t + 1 < nkt) s.template tile<1>(t + 1, nkt);
  }
  if (!lag) bar();
  if constexpr (ST) {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      unsigned long long* o = a.stamps + 4 * ((size_t)blockIdx.x * 8 + wave);
      o[0] = t1 - t0;
      o[1] = r1 - r0;
      o[2] = nkt;
    }
  }
  // C/D layout of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + j
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int ns = 0; ns < 2; ++ns)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const int row = m0 + wm * 128 + ms * 64 + mb * 16 + (lane >> 4) * 4;
          const int col = n0 + wn * 64 + ns * 32 + nb * 16 + (lane & 15);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const __bf16 v = (__bf16)s.acc[ms][mb][ns][nb][j];
            a.C[(size_t)(row + j) * a.N + col] = __builtin_bit_cast(unsigned short, v);
          }
        }
}

// naive fp32-accumulate reference, one thread per output
__global__ void ref_kernel(const unsigned short* A, const unsigned short* Bt, float* C, int M, int N, int K) {
  const int col = blockIdx.x * 64 + threadIdx.x % 64, row = blockIdx.y * 4 + threadIdx.x / 64;
  if (row >= M || col >= N) return;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) {
    const float x = __uint_as_float((unsigned)A[(size_t)row * K + k] << 16);
    const float y = __uint_as_float((unsigned)Bt[(size_t)col * K + k] << 16);
    acc = fmaf(x, y, acc);
  }
  C[(size_t)row * N + col] = acc;
}

static unsigned short to_bf16(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
static float from_bf16(unsigned short h) {
  unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

typedef int (*bench_fn)(int, int, int, int, int, int, int, int, void*, float*);

int main(int argc, char** argv) {
  int M = 4096, N = 4096, K = 4096, rounds = 5, iters = 50, gm = 4;
  const char* libpath = nullptr;
  int pos = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--rounds")) rounds = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--iters")) iters = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--lib")) libpath = argv[++i];
    else if (!strcmp(argv[i], "--gm")) gm = atoi(argv[++i]);
    else if (pos == 0) { M = atoi(argv[i]); ++pos; }
    else if (pos == 1) { N = atoi(argv[i]); ++pos; }
    else if (pos == 2) { K = atoi(argv[i]); ++pos; }
  }
  if (M % 256 || N % 256 || K % 64 || M <= 0 || N <= 0 || K <= 0) {
    fprintf(stderr, "M, N must be multiples of 256 and K of 64\n");
    return 2;
  }
  const size_t na = (size_t)M * K, nb = (size_t)N * K, nc = (size_t)M * N;
  std::vector<unsigned short> hA(na), hB(nb);
  unsigned long long x = 0x9E3779B97F4A7C15ull;
  auto uni = [&]() {  // uniform [-1, 1)
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    return (float)((x >> 40) * (1.0 / (1ull << 24))) * 2.f - 1.f;
  };
  for (auto& v : hA) v = to_bf16(uni());
  for (auto& v : hB) v = to_bf16(uni());
  unsigned short *dA, *dB, *dC;
  float* dR;
  unsigned long long* dS;
  const int nwg = (M / 256) * (N / 256);
  CK(hipMalloc(&dA, na * 2));
  CK(hipMalloc(&dB, nb * 2));
  CK(hipMalloc(&dC, nc * 2));
  CK(hipMalloc(&dR, nc * 4));
  CK(hipMalloc(&dS, (size_t)nwg * 8 * 4 * 8));
  CK(hipMemcpy(dA, hA.data(), na * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), nb * 2, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  Args a{dA, dB, dC, M, N, K, dS, gm};

  // correctness: every output against the naive kernel
  hipLaunchKernelGGL(ref_kernel, dim3((N + 63) / 64, (M + 3) / 4), dim3(256), 0, st, dA, dB, dR, M, N, K);
  hipLaunchKernelGGL(gemm8p_kernel<false>, dim3(nwg), dim3(NT), 0, st, a);
  CK(hipStreamSynchronize(st));
  {
    std::vector<unsigned short> hc(nc);
    std::vector<float> hr(nc);
    CK(hipMemcpy(hc.data(), dC, nc * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), dR, nc * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    double worst = 0;
    for (size_t i = 0; i < nc; ++i) {
      const double d = std::fabs((double)from_bf16(hc[i]) - hr[i]);
      const double tol = std::fabs(hr[i]) / 128.0 + 1e-3 * std::sqrt((double)K);
      worst = std::max(worst, d / tol);
      if (d > tol) ++bad;
    }
    printf("check %dx%dx%d: %zu of %zu outputs outside tolerance (worst err/tol %.3f)\n", M, N, K, bad, nc, worst);
    if (bad) return 1;
  }

  bench_fn lib_bench = nullptr;
  if (libpath) {
    void* h = dlopen(libpath, RTLD_NOW);
    if (!h) { fprintf(stderr, "dlopen %s: %s\n", libpath, dlerror()); return 1; }
    lib_bench = (bench_fn)dlsym(h, "mvae_bench_gemm");
    if (!lib_bench) { fprintf(stderr, "no mvae_bench_gemm\n"); return 1; }
  }
  const double flops = 2.0 * M * N * K;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // >= 2 s of back-to-back launches first (DVFS settles under load)
  {
    const auto t_end = 2000.f;
    float el = 0;
    CK(hipEventRecord(e0, st));
    while (el < t_end) {
      for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(gemm8p_kernel<false>, dim3(nwg), dim3(NT), 0, st, a);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&el, e0, e1));
    }
  }
  std::vector<double> tt, tl_e8, tl_def;
  for (int r = 0; r < rounds; ++r) {
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(gemm8p_kernel<false>, dim3(nwg), dim3(NT), 0, st, a);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    tt.push_back(flops / (ms / iters * 1e-3) / 1e12);
    if (lib_bench) {
      // NT layout (at = 0, bt = 1), bf16 (prec 1 << 4): variant 13 = the eight-phase kernel forced,
      // 0 = the planner's default kernel
      float avg = 0;
      int rc = lib_bench(M, N, K, 0, 1, 1, 13 | 16, iters, st, &avg);
      if (rc) { fprintf(stderr, "mvae_bench_gemm rc %d\n", rc); return 1; }
      tl_e8.push_back(flops / (avg * 1e-3) / 1e12);
      rc = lib_bench(M, N, K, 0, 1, 1, 0 | 16, iters, st, &avg);
      if (rc) { fprintf(stderr, "mvae_bench_gemm rc %d\n", rc); return 1; }
      tl_def.push_back(flops / (avg * 1e-3) / 1e12);
    }
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  printf("template 8-phase  %dx%dx%d: median %.1f TF/s over %d rounds (", M, N, K, med(tt), rounds);
  for (double v : tt) printf(" %.1f", v);
  printf(" )\n");
  if (lib_bench) {
    printf("library e8 (var13) %dx%dx%d: median %.1f TF/s (", M, N, K, med(tl_e8));
    for (double v : tl_e8) printf(" %.1f", v);
    printf(" )\nlibrary default    %dx%dx%d: median %.1f TF/s (", M, N, K, med(tl_def));
    for (double v : tl_def) printf(" %.1f", v);
    printf(" )\n");
  }
  // stamped build: in-kernel clock and cycles per k-tile (after the timed runs, chip warm)
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(gemm8p_kernel<true>, dim3(nwg), dim3(NT), 0, st, a);
  CK(hipStreamSynchronize(st));
  {
    std::vector<unsigned long long> hs((size_t)nwg * 8 * 4);
    CK(hipMemcpy(hs.data(), dS, hs.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> cyc, clk;
    for (int w = 0; w < nwg * 8; ++w) {
      const unsigned long long* o = &hs[(size_t)w * 4];
      if (!o[1] || !o[2]) continue;
      cyc.push_back((double)o[0] / o[2]);
      clk.push_back((double)o[0] / o[1] * 0.1);  // memrealtime ticks at 100 MHz -> GHz
    }
    printf("stamped: k-loop %.0f cycles per 256x256x64 k-tile (median over waves; MFMA issue floor 2048), "
           "in-kernel clock %.3f GHz\n", med(cyc), med(clk));
  }
  return 0;
}
