// The encoder's hidden layers in one launch (bf16 mode): H_l = act(H_{l-1} W_l), l = 1 .. n-1,
// over the stacked 3B rows (11a/vae.py:353-356 applied to the rot / lock / key blocks). Each
// workgroup owns TM rows for the whole chain: its activation block stays in LDS (TM x 512 bf16)
// from layer to layer, and only the weights stream in (32-row k-steps of W_l, 2-4 x 32 KB of LDS,
// global_load_lds_dwordx4 by every wave); each layer's block is copied out to the layer's bf16
// plane (the backward's operand) before the next layer runs. One launch replaces n-1 GEMM launches,
// their prologues / epilogue tails, and the activation round trips through HBM.
//
// 512 threads = 8 waves, wave w owns output columns 64 w .. 64 w + 63 (TM x 64 in
// v_mfma_f32_16x16x32_bf16 accumulators). Layouts in LDS:
//   activation: row r, 16-B chunk c (8 columns) at byte r * 1024 + 16 (c ^ (r & 15)): the 16 rows
//     of an A fragment read one chunk each from 16 distinct 16-B slots (conflict-free);
//   weight step image (per 128-column quarter q): [32 k-rows][16 chunks of 8 columns], chunk c of
//     k-row k at slot c ^ tr_swz(k); B fragments by two ds_read_b64_tr_b16 (gemm_bf16e.hip's
//     row-contiguous image, k-half 0).
// Columns >= N of a layer's output hold the constant row padding (1.0 at N -- the next layer's
// bias input -- and 0 beyond), as the GEMM epilogue with GemmEpi::padw = 2 writes them.
#include "gemm_common.h"

#include <cstdint>

namespace mvae {
namespace {

using namespace gemm;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short lds_short;
typedef __attribute__((address_space(3))) void* lds_ptr;

constexpr int CT = 512;          // threads
constexpr int KS = 32;           // k-rows per weight step
constexpr int QIMG = KS * 128;   // bf16 elements per quarter image (8 KB)
constexpr int STEP = 4 * QIMG;   // ... per step (32 KB)
constexpr int AROW = 512;        // activation row (bf16 elements, 1 KB)
constexpr int TMMAX = 96;

__device__ __attribute__((aligned(16))) unsigned short c_zero16[8] = {0, 0, 0, 0, 0, 0, 0, 0};

__device__ __forceinline__ int tr_swz(int k) { return (4 * (k & 3)) ^ (2 * ((k >> 3) & 1)); }

template <int OFF>
__device__ __forceinline__ bf16x8 rd_b128(unsigned a) {
  s16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ bf16x8 rd_tr(unsigned a) {
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a), "i"(4 * 256));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// weight steps in flight beside the one being read: the LDS the activation block leaves
constexpr int nstages(int tm) { return tm > 64 ? 2 : (tm > 32 ? 3 : 4); }

template <int MB>
__global__ __launch_bounds__(CT, 1) void enc_chain_kernel(ChainArgs a) {
  constexpr int TM = 16 * MB;
  constexpr int NS = nstages(TM);
  static_assert(TM * AROW + NS * STEP <= 160 * 512, "LDS");
  __shared__ __attribute__((aligned(1024))) short smem[TM * AROW + NS * STEP];
  short* const act = smem;
  short* const wst = smem + TM * AROW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * TM;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_short*)smem;
  const unsigned wst0 = lds0 + TM * AROW * 2;

  // ---- the input block (the layer-0 output plane) -> act, every wave; chunks past the row's
  // stored width (and rows past M) read the zero page
  {
    constexpr int NCH = TM * 64;  // 16-B chunks
#pragma unroll 1
    for (int base = wave * 64; base < NCH; base += CT) {
      const int L = base + lane;
      const int r = L >> 6, c = (L & 63) ^ (r & 15);
      const bool ok = m0 + r < a.M && 8 * c + 8 <= a.ldx;
      const unsigned short* src = ok ? a.x + (size_t)(m0 + r) * a.ldx + 8 * c : c_zero16;
      __builtin_amdgcn_global_load_lds(src, (lds_ptr)(act + base * 8), 16, 0, 0);
    }
  }
  // ---- weight steps: (layer, k-step) flattened; step s of layer l covers k-rows 32 s .. + 31
  auto steps = [&](int ll) { return (a.l[ll].K + KS - 1) / KS; };
  int G = 0;
  for (int ll = 0; ll < a.nl; ++ll) G += steps(ll);
  // every wave issues 4 of a step's 32 DMA instructions (64 lanes x 16 B each); (il, is): the
  // layer / step of the next step to issue
  int il = 0, is = 0, ig = 0;
  // per-lane source offsets of the current layer's step image (k-row within the step, column
  // clamped to the layer's last 8-column chunk), recomputed when the issue cursor changes layer
  unsigned doff[4];
  int dkr[4];
  auto layer_offsets = [&]() {
    const ChainLayer& w = a.l[il];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int Lc = (j * 8 + wave) * 64 + lane;  // chunk of the step image (linear LDS order)
      const int q = Lc >> 9, i = Lc & 511;
      const int krow = i >> 4, c = (i & 15) ^ tr_swz(krow);
      int col = 128 * q + 8 * c;
      col = col < w.N ? col : ((w.N - 1) & ~7);
      doff[j] = (unsigned)(krow * w.ldw + col);
      dkr[j] = krow;
    }
  };
  layer_offsets();
  auto issue = [&]() {
    const ChainLayer& w = a.l[il];
    short* img = wst + (ig % NS) * STEP;
    const int k0 = is * KS;
    const unsigned short* wk = w.w + (size_t)k0 * w.ldw;
    const int kl = w.K - k0;  // k-rows >= kl read the zero page
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned short* src = dkr[j] < kl ? wk + doff[j] : c_zero16;
      __builtin_amdgcn_global_load_lds(src, (lds_ptr)(img + (j * 8 + wave) * 512), 16, 0, 0);
    }
    ++ig;
    if (++is == steps(il)) {
      is = 0;
      if (++il < a.nl) layer_offsets();
    }
  };
  for (int i = 0; i < NS && i < G; ++i) issue();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the act block and the first steps)
  __syncthreads();

  // fragment addresses: A row block rb = rows 16 rb + (lane & 15), chunk 4 s + (lane >> 4)
  // (XOR-swizzled per row: added per step below); B column block nb of this wave's 64 columns
  const int ar = lane & 15, akc = lane >> 4;
  unsigned bad[4];
  {
    const int g4 = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
    const int krow = 8 * g4 + qq;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int col = 64 * (wave & 1) + 16 * nb + 4 * p;  // within the quarter
      const int c = (col >> 3) ^ tr_swz(krow);
      bad[nb] = wst0 + (wave >> 1) * QIMG * 2 + krow * 256 + c * 16 + 8 * (p & 1);
    }
  }
  f32x4 acc[MB][4];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int l = 0, s = 0;
  bool stored = false;  // a layer's block was stored since the last wait: wait for everything
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
    if (g > 0) {  // step g landed (its DMA is this wave's; the barrier publishes every wave's)
      // steps issued after g: 4 DMA instructions each (stores and loads may retire out of order)
      const int after = stored ? 0 : min(NS - 1, G - 1 - g);
      if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stored = false;
      bar();
    }
    const unsigned boff = (unsigned)((g % NS) * STEP * 2);
    bf16x8 fa[MB], fb[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) fb[nb] = rd_tr(bad[nb] + boff);
#pragma unroll
    for (int rb = 0; rb < MB; ++rb) {
      const int r = 16 * rb + ar, c = 4 * s + akc;
      fa[rb] = rd_b128<0>(lds0 + (unsigned)(r * 1024 + 16 * (c ^ (r & 15))));
    }
    // the first half of the row blocks' MFMAs as soon as B and their A fragments landed, the
    // second half's reads still in flight
    constexpr int H = (MB + 1) / 2;
    if constexpr (MB - H == 3) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
    else if constexpr (MB - H == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
    else if constexpr (MB - H == 1) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if (!(a.diag & 2)) {
#pragma unroll
      for (int rb = 0; rb < H; ++rb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rb], fb[nb], acc[rb][nb], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (!(a.diag & 2)) {
#pragma unroll
      for (int rb = H; rb < MB; ++rb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rb], fb[nb], acc[rb][nb], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    bar();  // step g's image (and, at a layer's end, the activation block) no longer read
    if (g + NS < G && !(a.diag & 1)) issue();
    if (++s < steps(l)) continue;
    // ---- layer l done: act(acc) -> the activation block (bf16, RN), padding past N
    const ChainLayer& w = a.l[l];
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        float v[4] = {acc[rb][nb][0], acc[rb][nb][1], acc[rb][nb][2], acc[rb][nb][3]};
        act_n(v, a.act);
        const int col = 64 * wave + 16 * nb + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 16 * rb + 4 * (lane >> 4) + j;
          const unsigned short h = col < w.N ? __builtin_bit_cast(unsigned short, __float2bfloat16(v[j]))
                                             : (col == w.N ? (unsigned short)0x3f80 : (unsigned short)0);
          act[r * AROW + 8 * ((col >> 3) ^ (r & 15)) + (col & 7)] = (short)h;
        }
        acc[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    __syncthreads();
    // the block -> the layer's plane (16-B chunks of the round8(N + 1) stored columns)
    {
      const int nch = (w.N + 8) >> 3;  // chunks holding columns 0 .. N
      const int tot = TM * nch;
#pragma unroll 1
      for (int i = tid; i < tot && !(a.diag & 4); i += CT) {
        const int r = i / nch, c = i - r * nch;
        if (m0 + r < a.M) {
          const uint4 v = *reinterpret_cast<const uint4*>(act + r * AROW + 8 * (c ^ (r & 15)));
          *reinterpret_cast<uint4*>(w.out + (size_t)(m0 + r) * w.ldo + 8 * c) = v;
        }
      }
    }
    stored = true;
    ++l;
    s = 0;
  }
}

}  // namespace

int enc_chain_rows(int M, int forced) {
  if (forced >= 16 && forced <= TMMAX && forced % 16 == 0) return forced;
  // rows per workgroup: one round of 256 workgroups when it fits (TM <= 96: LDS)
  int tm = 16 * ((M + 256 * 16 - 1) / (256 * 16));
  return tm > TMMAX ? TMMAX : (tm < 16 ? 16 : tm);
}

hipError_t launch_enc_chain(const ChainArgs& a, hipStream_t st) {
  if (a.nl < 1 || a.nl > 4 || a.M <= 0) return hipErrorInvalidValue;
  for (int l = 0; l < a.nl; ++l)
    if (a.l[l].K > 512 || a.l[l].N > 511 || (a.l[l].ldw & 7) || (a.l[l].ldo & 7) ||
        a.l[l].ldo < ((a.l[l].N + 8) & ~7) || (reinterpret_cast<uintptr_t>(a.l[l].w) & 15) ||
        (reinterpret_cast<uintptr_t>(a.l[l].out) & 15))
      return hipErrorInvalidValue;
  if ((a.ldx & 7) || (reinterpret_cast<uintptr_t>(a.x) & 15)) return hipErrorInvalidValue;
  const int tm = enc_chain_rows(a.M, a.rows);
  const dim3 grid((a.M + tm - 1) / tm);
  switch (tm / 16) {
    case 1: hipLaunchKernelGGL(enc_chain_kernel<1>, grid, dim3(CT), 0, st, a); break;
    case 2: hipLaunchKernelGGL(enc_chain_kernel<2>, grid, dim3(CT), 0, st, a); break;
    case 3: hipLaunchKernelGGL(enc_chain_kernel<3>, grid, dim3(CT), 0, st, a); break;
    case 4: hipLaunchKernelGGL(enc_chain_kernel<4>, grid, dim3(CT), 0, st, a); break;
    case 5: hipLaunchKernelGGL(enc_chain_kernel<5>, grid, dim3(CT), 0, st, a); break;
    default: hipLaunchKernelGGL(enc_chain_kernel<6>, grid, dim3(CT), 0, st, a); break;
  }
  return hipGetLastError();
}

}  // namespace mvae
