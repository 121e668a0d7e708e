// bf16-MFMA GEMM family for gfx950 (v_mfma_f32_32x32x16_bf16, fp32 accumulate), operands
// read as bf16 PLANES that their producers wrote (GEMM epilogues, de-interleave, latent
// kernels, Adam):
//   MVAE_PREC_BF16: one plane, x ~ RN_bf16(x);
//   MVAE_PREC_F32X: three planes, x = x0 + x1 + x2 EXACTLY (8+8+8 significand bits, each
//     residual an exact fp32 difference). sum_{i+j<3} A_i B_j reproduces the fp32 product
//     to ~2^-24 relative and is ONE bf16 GEMM over the K-concatenated plane pairs
//     (0,0),(0,1),(0,2),(1,0),(1,1),(2,0): the k-loop walks (pair, k-tile). When the A
//     operand's residual planes are all zero (dyn flag from its producer: binary pixels),
//     only the three pairs with i = 0 run. gfx950 has no xf32 and its bf16 MFMA rate is 16x
//     the fp32 rate, so fp32-accurate GEMMs cost 3-6 bf16 GEMMs instead of one fp32 GEMM.
//
// Tile 128x128xBK, 256 threads = 4 waves (2x2), each wave 2x2 MFMA 32x32 accumulators.
// LDS images (register-staged 16-B loads, next tile in registers during the MFMAs; single
// LDS buffer by default, two barriers per k-tile):
//   k-contiguous operand ([rows][K] in HBM): [row][k], stride BK+8 bf16 -> fragments by
//     ds_read_b128 (8 consecutive k), conflict-free;
//   row-contiguous operand ([K][rows]): [k][row], stride 160 bf16 -> fragments by two
//     ds_read_b64_tr_b16 (CDNA4 transposing LDS read), conflict-free.
#include "gemm_common.h"

#include <cmath>
#include <cstdlib>
#include <cstdint>

namespace mvae {
namespace {

using namespace gemm;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int SR = 160;     // [k][row] stride (bf16): 320 B = 64 mod 256 -> tr reads conflict-free

template <int BK>
struct Geo {
  static constexpr int SK = BK + 8;  // [row][k] stride (bf16): b128 fragment reads conflict-free
  static constexpr int STAGE = 128 * SK > BK * SR ? 128 * SK : BK * SR;  // bf16 elements / image
  static constexpr int NLD = 128 * BK / 8 / NT;                         // 16-B loads / thread
};

// 100 MHz constant-rate stamp, workgroup-comparable (diagnostics builds only)
__device__ __forceinline__ unsigned long long realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

template <bool KC, int BK>
struct Stage {
  static constexpr int SK = Geo<BK>::SK;
  static constexpr int NLD = Geo<BK>::NLD;
  static constexpr int CPR = BK / 8;  // 16-B chunks per row of a k-contiguous tile
  int4 r[NLD];

  __device__ __forceinline__ void load(const unsigned short* __restrict__ g, int ld, int row0,
                                       int nrows, int k0, int kend, int tid) {
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int c = tid + NT * j;
      int gr, gk;
      if constexpr (KC) {
        gr = row0 + c / CPR;
        gr = gr < nrows ? gr : nrows - 1;
        gk = k0 + 8 * (c % CPR);
        const unsigned short* p = g + (size_t)gr * ld + gk;
        if (gk + 8 <= kend) {
          r[j] = *reinterpret_cast<const int4*>(p);
        } else {
          unsigned short v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gk + e < kend ? p[e] : (unsigned short)0;
          r[j] = *reinterpret_cast<int4*>(v);
        }
      } else {
        gk = k0 + (c >> 4);
        gr = row0 + 8 * (c & 15);
        if (gk < kend) {
          const unsigned short* p = g + (size_t)gk * ld + gr;
          if (gr + 8 <= nrows) {
            r[j] = *reinterpret_cast<const int4*>(p);
          } else {
            unsigned short v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = gr + e < nrows ? p[e] : (unsigned short)0;
            r[j] = *reinterpret_cast<int4*>(v);
          }
        } else {
          r[j] = make_int4(0, 0, 0, 0);
        }
      }
    }
  }

  __device__ __forceinline__ void store(short* s, int tid) const {
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int c = tid + NT * j;
      const int off = KC ? (c / CPR) * SK + 8 * (c % CPR) : (c >> 4) * SR + 8 * (c & 15);
      *reinterpret_cast<int4*>(s + off) = r[j];
    }
  }

  // fragment (8 consecutive k) for the 32-row block at rb, k16-step ks
  __device__ __forceinline__ bf16x8 frag(const short* s, int rb, int ks, int lane) const {
    if constexpr (KC) {
      const s16x8 v = *reinterpret_cast<const s16x8*>(s + (rb + (lane & 31)) * SK + 16 * ks +
                                                      8 * (lane >> 5));
      return __builtin_bit_cast(bf16x8, v);
    } else {
      const int i = lane & 15, q = i >> 2, pp = i & 3;
      const int h = lane >> 5, g1 = (lane >> 4) & 1;
      const short* a0 = s + (16 * ks + 8 * h + q) * SR + rb + 16 * g1 + 4 * pp;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * SR));
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  }
};

// DB: double-buffered LDS (one barrier per k-tile) vs single buffer (two barriers; half the
// LDS, so more workgroups fit per CU).
template <bool AT, bool BT, int EPI, int BK, bool DB>
__global__ __launch_bounds__(NT, 2) void gemm_bf16p_kernel(PParams pp) {
  constexpr int STAGE = Geo<BK>::STAGE;
  constexpr int NB = DB ? 2 : 1;
  const Params& p = pp.g;
  if (epi_skip<EPI>(p.epi)) return;
  __shared__ __attribute__((aligned(16))) short smem[2 * NB * STAGE];
  // image b of A at smem + b*STAGE, of B at smem + (NB+b)*STAGE

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const Tile t = tile_of(p, true);
  const unsigned short* __restrict__ A = pp.A + t.bi * p.sA;
  const unsigned short* __restrict__ Bm = pp.B + t.bi * p.sB;

  Stage<!AT, BK> la;
  Stage<BT, BK> lb;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int npairs = (pp.dyn && *pp.dyn == 0) ? pp.npairs0 : pp.npairs;
  const int nkt = t.ks < t.ke ? (t.ke - t.ks + BK - 1) / BK : 0;
  const int total = npairs * nkt;
  auto load = [&](int it) {
    const int pr = it / nkt, kt = it - pr * nkt;
    const int k0 = t.ks + kt * BK;
    la.load(A + pp.pa[pr] * pp.pA, p.lda, t.m0, p.M, k0, t.ke, tid);
    lb.load(Bm + pp.pb[pr] * pp.pB, p.ldb, t.n0, p.N, k0, t.ke, tid);
  };
  if (total > 0) {
    load(0);
    la.store(smem, tid);
    lb.store(smem + NB * STAGE, tid);
  }
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    const int cur = DB ? (it & 1) : 0;
    const bool more = it + 1 < total;
    if (more) load(it + 1);
    const short* sa = smem + cur * STAGE;
    const short* sb = smem + (NB + cur) * STAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) fa[mi] = la.frag(sa, wm * 64 + mi * 32, ks, lane);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) fb[ni] = lb.frag(sb, wn * 64 + ni * 32, ks, lane);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
    }
    if constexpr (!DB) __syncthreads();
    if (more) {
      const int nxt = DB ? (cur ^ 1) : 0;
      la.store(smem + nxt * STAGE, tid);
      lb.store(smem + (NB + nxt) * STAGE, tid);
    }
    __syncthreads();
  }
  epilogue<EPI>(p, t, acc, reinterpret_cast<float*>(smem));
}

// ---------------------------------------------------------------------------------------
// Wide kernels: 256x256x64 tile, 512 threads = 8 waves (2 along M x 4 along N), each wave
// 128x64 = 4x2 MFMA 32x32x16 accumulators (1024 MFMA cycles per k-tile per wave). Operand
// tiles are copied HBM -> LDS by global_load_lds_dwordx4 (no VGPR staging). The LDS images
// are lane-linear (the DMA's destination is wave base +
// 16 B x lane); bank-conflict-free fragment reads come from XOR swizzles applied to the
// per-lane SOURCE address and undone on the read:
//   k-contiguous operand: image [256 rows][8 chunks of 8 k], chunk c of row r at position
//     c ^ ((r >> 1) & 7)  -> ds_read_b128 of 16 consecutive rows hits 16 distinct 16-B slots;
//   row-contiguous operand: image [64 k][32 chunks of 8 rows], chunk c of k-row k at
//     position c ^ (4 (k & 3))  -> the 32 lanes of a ds_read_b64_tr_b16 pass hit 32 slots.
// Out-of-range chunks (k >= ke, rows >= nrows of a row-contiguous operand) are loaded from a
// zero page, so partial tiles need no masking; rows past the end of a k-contiguous operand
// are clamped (their outputs are not stored). Requires every ld, batch and plane stride and
// the K padding [K, round8(K)) of k-contiguous operands to be zero-filled multiples of 8.
constexpr int WT = 256, WNT = 512;

__device__ __attribute__((aligned(16))) int4 g_zero16[1];
typedef __attribute__((address_space(3))) short lds_short;

// operand image of one k-tile (BK = 64 or 32) of ROWS (256 or 128) rows: NG DMA instructions
// per thread (NW waves x 64 lanes x 16 B each)
template <bool KC, int BK, int ROWS = 256, int NW = 8>
struct WLoad {
  // (an image of 192 rows x 32 k is 1.5 instructions per thread: the last one by half the waves)
  static constexpr int NCH = ROWS * BK / 8;  // 16-B chunks per image
  static constexpr int NG = (NCH + NW * 64 - 1) / (NW * 64);
  static constexpr int CPR = BK / 8;    // 16-B chunks per row of a k-contiguous image
  static constexpr int RPB = 128 / BK;  // k-contiguous rows per 256-B bank row
  static constexpr int CPK = ROWS / 8;  // 16-B chunks per k-row of a row-contiguous image
  long long off[NG];
  int kc[NG];
  bool rv[NG];
  __device__ __forceinline__ static int swz(int row) { return (row / RPB) & (CPR - 1); }
  __device__ __forceinline__ void init(int ld, int r0, int nrows, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int q = (j * NW + wave) * 64 + lane;  // chunk this lane copies
      if constexpr (KC) {
        const int row = q / CPR;
        const int c = (q % CPR) ^ swz(row);
        int gr = r0 + row;
        gr = gr < nrows ? gr : nrows - 1;
        off[j] = (long long)gr * ld + 8 * c;
        kc[j] = 8 * c;
        rv[j] = true;
      } else {
        const int krow = q / CPK;
        const int c = (q % CPK) ^ (4 * (krow & 3));
        const int col = r0 + 8 * c;
        rv[j] = col < nrows;
        off[j] = (long long)krow * ld + col;
        kc[j] = krow;
      }
    }
  }
  __device__ __forceinline__ void issue(const unsigned short* __restrict__ g, int ld, int k0,
                                        int kend, short* img, int wave) const {
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      if constexpr (NCH % (NW * 64) != 0)
        if ((j * NW + wave) * 64 >= NCH) continue;  // (wave-uniform)
      const bool ok = rv[j] && k0 + kc[j] < kend;
      const unsigned short* src = KC ? g + off[j] + k0 : g + off[j] + (long long)k0 * ld;
      src = ok ? src : reinterpret_cast<const unsigned short*>(g_zero16);
      __builtin_amdgcn_global_load_lds(src, (lds_short*)(img + (j * NW + wave) * 512), 16, 0, 0);
    }
  }
  // LDS instructions per fragment
  static constexpr int NRD = KC ? 1 : 2;
  // fragment (8 consecutive k) of the 32-row block at rb, k16-step ks. All fragment reads are
  // inline asm and their results are waited for explicitly (wait_lds) before use: the
  // transposing-read builtin makes hipcc wait for every outstanding LDS-DMA (vmcnt(0)), and a
  // compiler-visible ds_read_b128 next to the asm reads makes it wait lgkmcnt(0) before the
  // first use, which also waits for the NEXT k16-step's prefetched fragments (measured: the
  // MFMA-only loop then ran at ~47 % of peak).
  __device__ __forceinline__ bf16x8 frag(const short* s, unsigned s_lds, int rb, int ks,
                                         int lane) const {
    if constexpr (KC) {
      const int row = rb + (lane & 31);
      const int pos = (2 * ks + (lane >> 5)) ^ swz(row);
      const unsigned a = s_lds + 2u * (unsigned)(row * BK + pos * 8);
      s16x8 v;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
      return __builtin_bit_cast(bf16x8, v);
    } else {
      const int i = lane & 15, q = i >> 2, pp = i & 3;
      const int kk = 16 * ks + 8 * (lane >> 5) + q;
      const int ro = rb + 16 * ((lane >> 4) & 1) + 4 * pp;
      const int pos = (ro >> 3) ^ (4 * (kk & 3));
      const unsigned a0 = s_lds + 2u * (unsigned)(kk * ROWS + pos * 8 + (ro & 4));
      s16x4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a0), "i"(8 * ROWS));
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  }
};

// wait until at most N LDS instructions are outstanding (N is a literal per instantiation)
template <int N>
__device__ __forceinline__ void wait_lds() {
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
// wait until at most N vector-memory operations are outstanding (N literal per instantiation)
template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------
// Interleaved ring kernel: the k-loop walks (k-tile, plane pair) with the pairs INNERMOST, and
// the A and B operand images live in LDS rings of 3 and 2 slots (5 x 32 KB = the CU's 160 KB):
// an image is copied only when the iteration's (plane, k-tile) differs from the previous
// iteration's (with binary pixels the layer-0 operand is copied once per k-tile for its three
// pairs). The LDS fragment reads of the NEXT k16-step issued between the MFMAs of the current one
// (one fragment per MFMA gap; MI355X_MICROARCH.md §LDS: up to three reads per 32x32x16 gap are
// free), so no k16-step waits for its reads and no read burst stalls the MFMA issue. The
// iteration hand-off sits inside the last k16-step: once the step's fragments are in registers
// every read of the iteration's images is done, so after half of its MFMAs the waves wait for
// the next iteration's images (counted vmcnt), pass one raw s_barrier, issue the copies into the
// slots the iteration freed, and read the next iteration's first fragments behind the remaining
// MFMAs. Copies: B image of it+2 and A image of it+3 are issued in iteration it (B ring 2 slots,
// A ring 3 slots), each only when the (plane, k-tile) changes.
// Tile 256 x TN (TN = 256 or 128), 8 waves 2 (M) x 4 (N), each 128 x TN/4 = 4 x NI 32x32
// accumulators. TN = 128 doubles the tile count of a narrow GEMM (N ~ 500: the hidden encoder
// and decoder layers) so it fills the chip without split-K slabs and their reduction.
// MVAE_QGAP (build-time A/B): the next k16-step's fragment reads are spread over the first
// NM - MVAE_QGAP MFMA gaps, so the last one has MVAE_QGAP more MFMAs to land before the step's
// lgkmcnt(0)
#ifndef MVAE_QGAP
#define MVAE_QGAP 0
#endif
// MI = 3 (k-contiguous A only): a 192 x TN tile (each wave 96 x TN/4), so a 3B-row GEMM of
// 24576 rows is 128 x 2 = 256 workgroups -- one per CU -- instead of 96 x 2 = 192 (256 rows).
template <bool AT, bool BT, int EPI, bool TE, int TN, int MI = 4, bool ST = false>
__global__ __launch_bounds__(WNT, 1) void gemm_bf16q_kernel(PParams pp) {
  constexpr int BK = 64;
  constexpr int NI = TN / 128;
  constexpr int TM = 64 * MI;                  // tile rows: 2 wave rows x MI 32-row blocks
  static_assert(MI == 4 || (MI == 3 && !AT), "192-row tiles need a k-contiguous A operand");
  constexpr int IMA = TM * BK, IMB = TN * BK;  // bf16 elements per operand image
  constexpr int KS = BK / 16;
  constexpr int NM = MI * NI;                  // MFMAs per wave per k16-step
  constexpr int NF = NI + MI;                  // fragments per wave per k16-step (B first)
  const Params& p = pp.g;
  if (epi_skip<EPI>(p.epi)) return;
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st_wait = 0, st_vmw = 0;
  if constexpr (ST) {
    __builtin_amdgcn_sched_barrier(0);
    st0 = realtime();
    __builtin_amdgcn_sched_barrier(0);
  }
  // A ring slots | B ring slots; the row-major epilogue's two 64-row bands (and the BCE row
  // partials) reuse it after the k-loop
  constexpr int RING = 3 * IMA + 2 * IMB;
  constexpr int EPIL = TE ? 2 * (2 * 64 * TN + 64 * MI * (TN / 8)) : 0;
  __shared__ __attribute__((aligned(16))) short smem[RING > EPIL ? RING : EPIL];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const Tile t = tile_of_t<TM, TN>(p, true);
  const unsigned short* __restrict__ A = pp.A + t.bi * p.sA;
  const unsigned short* __restrict__ Bm = pp.B + t.bi * p.sB;

  WLoad<!AT, BK, TM> la;
  WLoad<BT, BK, TN> lb;
  la.init(p.lda, t.m0, p.M, wave, lane);
  lb.init(p.ldb, t.n0, p.N, wave, lane);

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int np = (pp.dyn && *pp.dyn == 0) ? pp.npairs0 : pp.npairs;
  const int nkt = t.ks < t.ke ? (t.ke - t.ks + BK - 1) / BK : 0;
  const int total = (pp.diag & 16) ? 0 : np * nkt;  // diag bit 4: the epilogue alone
  // s_setprio 1 around each k16-step's MFMAs (cdna_hip_programming.md T5): +1-3 % on the step's
  // GEMMs, +3-7 % on 4096^3 (profiles/r3/gemm_ab_setprio_r3u.txt); diag bit 5 turns it off (A/B)
  const bool sprio = (pp.diag & 32) == 0;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_short*)smem;
  auto pa_of = [&](int pr) { return (pp.pab >> (4 * pr)) & 3; };
  auto pb_of = [&](int pr) { return (pp.pab >> (4 * pr + 2)) & 3; };
  auto adv = [&](int& kt, int& pr) { if (++pr == np) { pr = 0; ++kt; } };
  // A cursor: iteration ia (k-tile, pair) of the last A image considered and its slot; B likewise
  int akt = 0, apr = 0, ia = 0, asl = 0;
  int bkt = 0, bpr = 0, ib = 0, bsl = 0;
  bool pend_a = false;  // the A copy issued with the last B copy (vmcnt accounting)
  const bool dma = !(pp.diag & 1);
  constexpr int GA = WLoad<!AT, BK, TM>::NG;  // DMA instructions per A image per thread
  // move the A cursor to ia+1 and copy its image if it differs from ia's
  auto next_a = [&]() -> bool {
    if (ia + 1 >= total || !dma) return false;
    const int k0 = akt, p0 = apr;
    adv(akt, apr);
    ++ia;
    if (akt == k0 && pa_of(apr) == pa_of(p0)) return false;
    asl = asl == 2 ? 0 : asl + 1;
    la.issue(A + pa_of(apr) * pp.pA, p.lda, t.ks + akt * BK, t.ke, smem + asl * IMA, wave);
    return true;
  };
  auto next_b = [&]() -> bool {
    if (ib + 1 >= total || !dma) return false;
    const int k0 = bkt, p0 = bpr;
    adv(bkt, bpr);
    ++ib;
    if (bkt == k0 && pb_of(bpr) == pb_of(p0)) return false;
    bsl ^= 1;
    lb.issue(Bm + pb_of(bpr) * pp.pB, p.ldb, t.ks + bkt * BK, t.ke, smem + 3 * IMA + bsl * IMB, wave);
    return true;
  };
  // slots of the images of iterations it .. it+2 (A) and it .. it+1 (B)
  int sa_q[3] = {0, 0, 0};
  int sb_q[2] = {0, 0};

  bf16x8 fa[2][MI], fb[2][NI];
  auto rd_a = [&](int slot, int ks, int mi, bf16x8& a) {
    a = la.frag(smem + slot * IMA, lds0 + 2u * (unsigned)(slot * IMA), wm * (MI * 32) + mi * 32, ks, lane);
  };
  auto rd_b = [&](int slot, int ks, int ni, bf16x8& b) {
    b = lb.frag(smem + 3 * IMA + slot * IMB, lds0 + 2u * (unsigned)(3 * IMA + slot * IMB),
                wn * (TN / 4) + ni * 32, ks, lane);
  };
  // fragment f of a k16-step: B fragments first, then the four A fragments
  auto rd_f = [&](int sa, int sb, int ks, int f, int buf) {
    if (f < NI) rd_b(sb, ks, f, fb[buf][f]);
    else rd_a(sa, ks, f - NI, fa[buf][f - NI]);
  };
  auto mfma = [&](int i, int cur) {
    const int mi = i / NI, ni = i % NI;
    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][mi], fb[cur][ni], acc[mi][ni], 0, 0, 0);
  };

  if (total > 0) {
    // prologue: A(0), B(0), A(1); wait for A(0), B(0); barrier; B(1), A(2)
    la.issue(A + pa_of(0) * pp.pA, p.lda, t.ks, t.ke, smem, wave);
    lb.issue(Bm + pb_of(0) * pp.pB, p.ldb, t.ks, t.ke, smem + 3 * IMA, wave);
    const bool a1 = next_a();
    sa_q[0] = 0; sa_q[1] = asl;
    if (a1) {
      wait_vm<GA>();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (ST) {
      __builtin_amdgcn_sched_barrier(0);
      st1 = realtime();
      __builtin_amdgcn_sched_barrier(0);
    }
    next_b();
    sb_q[0] = 0; sb_q[1] = bsl;
    pend_a = next_a();
    sa_q[2] = asl;
#pragma unroll
    for (int f = 0; f < NF; ++f) rd_f(sa_q[0], sb_q[0], 0, f, 0);
  }
  for (int it = 0; it < total; ++it) {
    const int sa = sa_q[0], sb = sb_q[0];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int cur = ks & 1, nx = cur ^ 1;
      wait_lds<0>();  // this step's fragments (read during the previous step's MFMAs)
      __builtin_amdgcn_sched_barrier(0);
      if (sprio) __builtin_amdgcn_s_setprio(1);
      if (ks + 1 < KS) {
        // MFMA i, then the fragments of step ks+1 assigned to its gap
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          mfma(i, cur);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int f = 0; f < NF; ++f)
            if (f * (NM - MVAE_QGAP) / NF == i) rd_f(sa, sb, ks + 1, f, nx);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NM / 2; ++i) mfma(i, cur);
        __builtin_amdgcn_sched_barrier(0);
        const bool more = it + 1 < total;
        if (more) {
          unsigned long long tw0 = 0;
          if constexpr (ST) tw0 = realtime();
          // images of it+1 landed (only the A copy issued after its B copy may be in flight),
          // every wave's reads of it's images are done: its freed slots can be refilled
          if (pend_a) {
            wait_vm<GA>();
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          if constexpr (ST) {  // stamped builds: time in the vmcnt wait, then in the barrier
            const unsigned long long tw1 = realtime();
            st_vmw += tw1 - tw0;
            tw0 = tw1;
          }
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          if constexpr (ST) st_wait += realtime() - tw0;
        }
        __builtin_amdgcn_sched_barrier(0);
        // fragments of it+1's first step (its images: the slot queues' second entries), then
        // the copies into the freed slots: B of it+2, A of it+3
#pragma unroll
        for (int i = NM / 2; i < NM; ++i) {
          mfma(i, cur);
          __builtin_amdgcn_sched_barrier(0);
          if (more) {
            constexpr int H = NM / 2;  // gaps after the barrier
#pragma unroll
            for (int f = 0; f < NF; ++f)
              if (f * (H - 1) / NF + H == i) rd_f(sa_q[1], sb_q[1], 0, f, nx);
            if (i == NM - 2) {
              next_b();
              sb_q[0] = sb_q[1]; sb_q[1] = bsl;
              pend_a = next_a();
              sa_q[0] = sa_q[1]; sa_q[1] = sa_q[2]; sa_q[2] = asl;
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (sprio) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // KS is even: the next iteration's step 0 reads land in fa/fb[0]
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (ST) {
    __builtin_amdgcn_sched_barrier(0);
    st2 = realtime();
    __builtin_amdgcn_sched_barrier(0);
  }
  unsigned long long st_iss = 0;
  // BCE row partials in the LDS past the two 64-row bands (2 x 64 x TN floats), 64 MI x TN / 8
  // floats (EPIL above)
  if constexpr (TE) epilogue_rm<EPI, MI, NI, 4, WNT>(p, t, acc, reinterpret_cast<float*>(smem), wm, wn, pp.diag,
                                                     ST ? &st_iss : nullptr,
                                                     reinterpret_cast<float*>(smem) + 2 * 64 * TN);
  else epilogue_g<EPI, MI, NI, TM, 4>(p, t, acc, reinterpret_cast<float*>(smem), wm, wn);
  if constexpr (ST) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long st3 = realtime();
    if (threadIdx.x == 0) {
      unsigned long long* o = pp.stamps + 8 * (size_t)blockIdx.x;
      o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = st_iss; o[5] = st_wait; o[6] = st_vmw;
    }
  }
}

template <bool AT, bool BT, int EPI, bool TE, int TN, int MI = 4>
hipError_t launch_q(const PParams& p, hipStream_t st) {
  const int nwg = p.g.ntm * p.g.ntn * p.g.batch * p.g.split;
  // stamped diagnostics builds (bench only): the hidden forward (ACT), the BCE head (BCEB, bf16 binary target as in the step) and
  // the hidden dgrad (DACTB: bf16 aux, B = W^T)
  if constexpr (TE && !AT && ((EPI == EPI_ACT && !BT) || (EPI == EPI_BCEB && !BT) || (EPI == EPI_DACTB && BT))) {
    if (p.stamps) {
      hipLaunchKernelGGL((gemm_bf16q_kernel<AT, BT, EPI, TE, TN, MI, true>), dim3(nwg), dim3(WNT), 0, st, p);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_bf16q_kernel<AT, BT, EPI, TE, TN, MI>), dim3(nwg), dim3(WNT), 0, st, p);
  return hipGetLastError();
}

template <int EPI, bool TE, int TN>
hipError_t launch_q_l(const PParams& p, bool at, bool bt, hipStream_t st) {
  // 192-row tiles (planner: Params::tm == 192) for the A-k-contiguous non-BCE epilogues
  constexpr bool T192 = EPI != EPI_BCE && EPI != EPI_BCEB && EPI != EPI_SIGMOID;
  if constexpr (T192) {
    if (p.g.tm == 192 && !at)
      return bt ? launch_q<false, true, EPI, TE, TN, 3>(p, st) : launch_q<false, false, EPI, TE, TN, 3>(p, st);
  }
  if (!at && !bt) return launch_q<false, false, EPI, TE, TN>(p, st);
  if (at && !bt) return launch_q<true, false, EPI, TE, TN>(p, st);
  if (!at && bt) return launch_q<false, true, EPI, TE, TN>(p, st);
  return launch_q<true, true, EPI, TE, TN>(p, st);
}

template <int EPI, bool TE>
hipError_t launch_q_t(const PParams& p, bool at, bool bt, hipStream_t st) {
  return p.g.tn == 128 ? launch_q_l<EPI, TE, 128>(p, at, bt, st) : launch_q_l<EPI, TE, 256>(p, at, bt, st);
}

// ---------------------------------------------------------------------------------------
// Plane-stacked f32x ring kernel (create option x3; tile TM x 128, TM = 64 MI). The ring kernel
// above walks (k-tile, plane pair) iterations: six pairs make six iterations per 64 k, each with its
// own barrier and image copies (3 A + 5 B images per k-tile) and two fragment reads per MFMA. Here
// one stage holds a 32-k tile of EVERY plane the pairs read (A planes 0..NA-1, B planes 0..NB-1; two
// stages, 120 / 144 KB), each k16-step reads every plane's fragments once and issues all its pair
// MFMAs from them: per 64 k two barriers, 3 + 3 images and one fragment read per MFMA for each
// pair -- the short-K f32x GEMMs of the hidden layers (K = 501: 48 ring iterations per tile) are
// bound by those per-iteration costs, not by their MFMAs. The same pairs as the ring kernel
// (i + j < 3, sum of 2^-24-exact plane products), summed (k16-step, pair) instead of (pair, k16).
// The epilogues are the ring kernel's (32x32 accumulators, TN = 128: one per 32 rows per wave).
constexpr __host__ __device__ int x3_pa(int na, int nb, int i) {
  return na == 1 ? 0 : (nb == 1 ? i : (i < 3 ? 0 : (i == 5 ? 2 : 1)));  // (0,0) (0,1) (0,2) (1,1) (1,0) (2,0)
}
constexpr __host__ __device__ int x3_pb(int na, int nb, int i) {
  return nb == 1 ? 0 : (na == 1 ? i : (i < 3 ? i : (i == 3 ? 1 : 0)));
}
template <int NA, int NB, int MI, bool AT, bool BT>
__device__ __forceinline__ void x3_kloop(const PParams& pp, const Tile& t, const unsigned short* __restrict__ A,
                                         const unsigned short* __restrict__ Bm, short* smem,
                                         f32x16 (&acc)[MI][1], int wave, int lane, int wm, int wn) {
  constexpr int BK = 32, TM = 64 * MI, TN = 128;
  constexpr int IMA = TM * BK, IMB = TN * BK, STG = 3 * IMA + 3 * IMB;
  constexpr int NP = (NA == 1 || NB == 1) ? 3 : 6;  // pairs i + j < 3
  constexpr int NF = NB + NA * MI;                   // fragments per k16-step (B first)
  constexpr int NM = NP * MI;                        // MFMAs per wave per k16-step
  constexpr int H = NM / 2;                          // MFMAs before the stage hand-off
  const Params& p = pp.g;
  WLoad<!AT, BK, TM> la;
  WLoad<BT, BK, TN> lb;
  la.init(p.lda, t.m0, p.M, wave, lane);
  lb.init(p.ldb, t.n0, p.N, wave, lane);
  const int nkt = t.ks < t.ke ? (t.ke - t.ks + BK - 1) / BK : 0;
  const bool sprio = (pp.diag & 32) == 0;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_short*)smem;
  auto issue = [&](int kt, int st) {
    const int k0 = t.ks + kt * BK;
#pragma unroll
    for (int a = 0; a < NA; ++a) la.issue(A + a * pp.pA, p.lda, k0, t.ke, smem + st * STG + a * IMA, wave);
#pragma unroll
    for (int b = 0; b < NB; ++b) lb.issue(Bm + b * pp.pB, p.ldb, k0, t.ke, smem + st * STG + 3 * IMA + b * IMB, wave);
  };
  // a wave whose 32 columns all lie past N (the latent head's N = 2L = 40 in a 128-wide tile)
  // issues no fragment reads and no MFMAs: its outputs are never stored (it still copies and syncs)
  const bool live = t.n0 + wn * 32 < p.N;
  bf16x8 fa[2][NA][MI], fb[2][NB];
  // fragment f of k16-step ks of stage st into buffer buf: the B planes' first, then A's by plane
  auto rd_f = [&](int st, int ks, int f, int buf) {
    if (!live) return;
    if (f < NB) {
      const int o = st * STG + 3 * IMA + f * IMB;
      fb[buf][f] = lb.frag(smem + o, lds0 + 2u * (unsigned)o, wn * 32, ks, lane);
    } else {
      const int a = (f - NB) / MI, mi = (f - NB) % MI;
      const int o = st * STG + a * IMA;
      fa[buf][a][mi] = la.frag(smem + o, lds0 + 2u * (unsigned)o, wm * (MI * 32) + mi * 32, ks, lane);
    }
  };
  auto mfma = [&](int i, int cur) {
    const int pr = i / MI, mi = i % MI;
    if (live)
      acc[mi][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][x3_pa(NA, NB, pr)][mi], fb[cur][x3_pb(NA, NB, pr)],
                                                           acc[mi][0], 0, 0, 0);
  };
  if (nkt <= 0) return;
  // prologue: stages 0 and 1 in flight, wait for both (one wait: waves issue unequal counts of
  // a 192-row image), step 0's fragments
  issue(0, 0);
  if (nkt > 1) issue(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int f = 0; f < NF; ++f) rd_f(0, 0, f, 0);
  for (int kt = 0; kt < nkt; ++kt) {
    const int st = kt & 1;
    // k16-step 0: its fragments landed; step 1's read into buffer 1 between the MFMAs
    wait_lds<0>();
    __builtin_amdgcn_sched_barrier(0);
    if (sprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      mfma(i, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 0; f < NF; ++f)
        if (f * NM / NF == i) rd_f(st, 1, f, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (sprio) __builtin_amdgcn_s_setprio(0);
    // k16-step 1: once its fragments are in registers this wave reads stage st no more; after
    // half its MFMAs wait for stage st ^ 1 (k-tile kt + 1, the only copy in flight), one barrier
    // (every wave done with stage st), then the copy of k-tile kt + 2 into stage st and the next
    // k-tile's step-0 fragments behind the remaining MFMAs
    wait_lds<0>();
    __builtin_amdgcn_sched_barrier(0);
    if (sprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < H; ++i) mfma(i, 1);
    __builtin_amdgcn_sched_barrier(0);
    const bool more = kt + 1 < nkt;
    if (more) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = H; i < NM; ++i) {
      mfma(i, 1);
      __builtin_amdgcn_sched_barrier(0);
      if (more) {
#pragma unroll
        for (int f = 0; f < NF; ++f)
          if (f * (NM - H - 1) / NF + H == i) rd_f(st ^ 1, 0, f, 0);
        if (i == NM - 2 && kt + 2 < nkt) issue(kt + 2, st);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (sprio) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The 256 x 256 form (the ring kernel's 256x256 plans: C2's hidden weight gradients): a 16-k stage
// of all six planes is 48 KB, three stages; each k16-step reads its 18 fragments (A 3 x 4, B 3 x 2)
// once, after the stage's barrier, and issues the 48 pair MFMAs from them -- no fragment double
// buffer (18 + 128 accumulator registers; the other wave of the SIMD covers the read latency)
template <int NA, int NB, bool AT, bool BT>
__device__ __forceinline__ void x3w_kloop(const PParams& pp, const Tile& t, const unsigned short* __restrict__ A,
                                          const unsigned short* __restrict__ Bm, short* smem,
                                          f32x16 (&acc)[4][2], int wave, int lane, int wm, int wn) {
  constexpr int BK = 16, TM = 256, TN = 256, MI = 4, NI = 2;
  constexpr int IMA = TM * BK, IMB = TN * BK, STG = 3 * IMA + 3 * IMB;
  constexpr int NP = (NA == 1 || NB == 1) ? 3 : 6;
  constexpr int NG = NA * WLoad<!AT, BK, TM>::NG + NB * WLoad<BT, BK, TN>::NG;  // DMA instructions per stage
  const Params& p = pp.g;
  WLoad<!AT, BK, TM> la;
  WLoad<BT, BK, TN> lb;
  la.init(p.lda, t.m0, p.M, wave, lane);
  lb.init(p.ldb, t.n0, p.N, wave, lane);
  const int nkt = t.ks < t.ke ? (t.ke - t.ks + BK - 1) / BK : 0;
  const bool sprio = (pp.diag & 32) == 0;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_short*)smem;
  const bool live = t.n0 + wn * (TN / 4) < p.N;
  auto issue = [&](int kt, int st) {
    const int k0 = t.ks + kt * BK;
#pragma unroll
    for (int a = 0; a < NA; ++a) la.issue(A + a * pp.pA, p.lda, k0, t.ke, smem + st * STG + a * IMA, wave);
#pragma unroll
    for (int b = 0; b < NB; ++b) lb.issue(Bm + b * pp.pB, p.ldb, k0, t.ke, smem + st * STG + 3 * IMA + b * IMB, wave);
  };
  if (nkt <= 0) return;
  issue(0, 0);
  if (nkt > 1) issue(1, 1);
  for (int kt = 0; kt < nkt; ++kt) {
    const int st = kt % 3;
    // stage kt landed (only k-tile kt + 1's copies may still be in flight), every wave done with
    // k-tile kt - 1's stage: the copy of kt + 2 goes into it
    if (kt + 1 < nkt) {
      if constexpr (NG == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (NG == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 2 < nkt) issue(kt + 2, (kt + 2) % 3);
    if (!live) continue;
    bf16x8 fa[NA][MI], fb[NB][NI];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int o = st * STG + 3 * IMA + b * IMB;
        fb[b][ni] = lb.frag(smem + o, lds0 + 2u * (unsigned)o, wn * (TN / 4) + ni * 32, 0, lane);
      }
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int o = st * STG + a * IMA;
        fa[a][mi] = la.frag(smem + o, lds0 + 2u * (unsigned)o, wm * (MI * 32) + mi * 32, 0, lane);
      }
    wait_lds<0>();
    __builtin_amdgcn_sched_barrier(0);
    if (sprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int pr = 0; pr < NP; ++pr)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[x3_pa(NA, NB, pr)][mi], fb[x3_pb(NA, NB, pr)][ni],
                                                                acc[mi][ni], 0, 0, 0);
    if (sprio) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool AT, bool BT, int EPI, bool TE>
__global__ __launch_bounds__(WNT, 1) void gemm_bf16xw_kernel(PParams pp) {
  constexpr int TM = 256, TN = 256;
  const Params& p = pp.g;
  if (epi_skip<EPI>(p.epi)) return;
  constexpr int RING = 3 * (3 * TM * 16 + 3 * TN * 16);
  constexpr int EPIL = TE ? 2 * (2 * 64 * TN + 64 * 4 * (TN / 8)) : 0;
  __shared__ __attribute__((aligned(16))) short smem[RING > EPIL ? RING : EPIL];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const Tile t = tile_of_t<TM, TN>(p, true);
  const unsigned short* __restrict__ A = pp.A + t.bi * p.sA;
  const unsigned short* __restrict__ Bm = pp.B + t.bi * p.sB;
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if (!(pp.diag & 16)) {
    if (pp.dyn && *pp.dyn == 0) x3w_kloop<1, 3, AT, BT>(pp, t, A, Bm, smem, acc, wave, lane, wm, wn);
    else x3w_kloop<3, 3, AT, BT>(pp, t, A, Bm, smem, acc, wave, lane, wm, wn);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (TE) epilogue_rm<EPI, 4, 2, 4, WNT>(p, t, acc, reinterpret_cast<float*>(smem), wm, wn, pp.diag, nullptr,
                                                   reinterpret_cast<float*>(smem) + 2 * 64 * TN);
  else epilogue_g<EPI, 4, 2, TM, 4>(p, t, acc, reinterpret_cast<float*>(smem), wm, wn);
}

template <bool AT, bool BT, int EPI, bool TE, int MI>
__global__ __launch_bounds__(WNT, 1) void gemm_bf16x_kernel(PParams pp) {
  constexpr int TM = 64 * MI, TN = 128;
  static_assert(MI == 4 || (MI == 3 && !AT), "192-row tiles need a k-contiguous A operand");
  const Params& p = pp.g;
  if (epi_skip<EPI>(p.epi)) return;
  constexpr int RING = 2 * (3 * TM * 32 + 3 * TN * 32);
  constexpr int EPIL = TE ? 2 * (2 * 64 * TN + 64 * MI * (TN / 8)) : 0;
  __shared__ __attribute__((aligned(16))) short smem[RING > EPIL ? RING : EPIL];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const Tile t = tile_of_t<TM, TN>(p, true);
  const unsigned short* __restrict__ A = pp.A + t.bi * p.sA;
  const unsigned short* __restrict__ Bm = pp.B + t.bi * p.sB;
  f32x16 acc[MI][1];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][0][r] = 0.f;
  if (!(pp.diag & 16)) {  // diag bit 4: the epilogue alone
    if (pp.dyn && *pp.dyn == 0) x3_kloop<1, 3, MI, AT, BT>(pp, t, A, Bm, smem, acc, wave, lane, wm, wn);
    else x3_kloop<3, 3, MI, AT, BT>(pp, t, A, Bm, smem, acc, wave, lane, wm, wn);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (TE) epilogue_rm<EPI, MI, 1, 4, WNT>(p, t, acc, reinterpret_cast<float*>(smem), wm, wn, pp.diag, nullptr,
                                                    reinterpret_cast<float*>(smem) + 2 * 64 * TN);
  else epilogue_g<EPI, MI, 1, TM, 4>(p, t, acc, reinterpret_cast<float*>(smem), wm, wn);
}

template <int EPI, bool TE>
hipError_t launch_x_t(const PParams& p, bool at, bool bt, hipStream_t st) {
  const int nwg = p.g.ntm * p.g.ntn * p.g.batch * p.g.split;
  const dim3 g(nwg), b(WNT);
  if (p.g.tn == 256) {  // (x3_serves: 256-row tiles)
    if (!at && !bt) hipLaunchKernelGGL((gemm_bf16xw_kernel<false, false, EPI, TE>), g, b, 0, st, p);
    else if (at && !bt) hipLaunchKernelGGL((gemm_bf16xw_kernel<true, false, EPI, TE>), g, b, 0, st, p);
    else if (!at && bt) hipLaunchKernelGGL((gemm_bf16xw_kernel<false, true, EPI, TE>), g, b, 0, st, p);
    else hipLaunchKernelGGL((gemm_bf16xw_kernel<true, true, EPI, TE>), g, b, 0, st, p);
    return hipGetLastError();
  }
  if (p.g.tm == 192 && !at) {
    if (bt) hipLaunchKernelGGL((gemm_bf16x_kernel<false, true, EPI, TE, 3>), g, b, 0, st, p);
    else hipLaunchKernelGGL((gemm_bf16x_kernel<false, false, EPI, TE, 3>), g, b, 0, st, p);
  } else if (!at && !bt) {
    hipLaunchKernelGGL((gemm_bf16x_kernel<false, false, EPI, TE, 4>), g, b, 0, st, p);
  } else if (at && !bt) {
    hipLaunchKernelGGL((gemm_bf16x_kernel<true, false, EPI, TE, 4>), g, b, 0, st, p);
  } else if (!at && bt) {
    hipLaunchKernelGGL((gemm_bf16x_kernel<false, true, EPI, TE, 4>), g, b, 0, st, p);
  } else {
    hipLaunchKernelGGL((gemm_bf16x_kernel<true, true, EPI, TE, 4>), g, b, 0, st, p);
  }
  return hipGetLastError();
}

// the plane-stacked kernel serves this ring plan: option x3, tile N 128, the six f32x pairs of
// three-plane operands (A's residual planes possibly zero at run time: its three-pair loop)
bool x3_serves(const PParams& p) {
  if (!p.x3 || p.npairs != 6) return false;
  if (p.g.tn != 128 && !(p.g.tn == 256 && p.g.tm == 256 && p.x3 >= 2)) return false;
  // (the 256x256 form's BCE instantiations spill: the head keeps the eight-phase / ring kernels)
  if (p.g.tn == 256 && (p.g.epi.mode == EPI_BCE || p.g.epi.mode == EPI_BCEB)) return false;
  for (int i = 0; i < 6; ++i)
    if (p.pa[i] != x3_pa(3, 3, i) || p.pb[i] != x3_pb(3, 3, i)) return false;
  return !p.dyn || p.npairs0 == 3;
}

// the row-major 16-B epilogue (epilogue_wide) applies: bases and strides keep every 8-column
// chunk of every operand it touches 16-B aligned
bool wide_epi_vec_ok(const Params& g) {
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const GemmEpi& e = g.epi;
  if (e.c32 && (!al(g.C) || (g.ldc & 3) || (g.sC & 3))) return false;
  if (e.cp && (!al(e.cp) || (g.ldc & 7) || (g.sC & 7) || (e.pc & 7))) return false;
  if (e.mode == EPI_DACT && !e.auxp && (!al(e.aux) || (e.ld_aux & 3))) return false;
  if (e.mode == EPI_DACT && e.auxp && (!al(e.auxp) || (e.ld_aux & 7))) return false;
  if (e.mode == EPI_BCE || e.mode == EPI_BCEB) {
    if (e.x && (!al(e.x) || (e.ldx & 3))) return false;
    if (e.xp && (!al(e.xp) || (e.ldx & 7))) return false;
    if (e.y && (!al(e.y) || (e.ldy & 3))) return false;
  }
  return true;
}

// The planned 256-row kernel: the eight-phase kernel (tile N = TN_E8, gemm_bf16e.hip) or the
// interleaved ring kernel. Their epilogue goes through LDS (row-major 16-B stores) when the tile
// writes bf16 planes or is the BCE head (2-B plane stores and 4-B target loads per element
// otherwise), and stays in the C/D layout for fp32-only outputs (split-K slabs: 128-B row
// segments already, where the LDS round trip measured 5-10 % slower); the eight-phase kernel's
// accumulators are not in the C/D row-segment order, so its epilogue always goes through LDS
// (variant 14 = 13); variant 10 keeps the ring kernel on the C/D layout.
template <int EPI>
hipError_t launch_wide(const PParams& p, bool at, bool bt, int variant, hipStream_t st) {
  constexpr bool BCE = EPI == EPI_BCE || EPI == EPI_BCEB;
  if (p.g.tn == TN_E8) {  // always the LDS epilogue: 16-B accesses where aligned, else element-wise
    (void)variant;
    return gemm_bf16e_launch(p, at, bt, EPI, wide_epi_vec_ok(p.g), st);
  }
  const bool te = (p.g.epi.cp || BCE) && variant != 10 && wide_epi_vec_ok(p.g);
  if (x3_serves(p)) return te ? launch_x_t<EPI, true>(p, at, bt, st) : launch_x_t<EPI, false>(p, at, bt, st);
  if (te) return launch_q_t<EPI, true>(p, at, bt, st);
  return launch_q_t<EPI, false>(p, at, bt, st);
}

template <bool AT, bool BT, int EPI, int BK, bool DB>
hipError_t launch_t(const PParams& p, hipStream_t st) {
  const int nwg = p.g.ntm * p.g.ntn * p.g.batch * p.g.split;
  hipLaunchKernelGGL((gemm_bf16p_kernel<AT, BT, EPI, BK, DB>), dim3(nwg), dim3(NT), 0, st, p);
  return hipGetLastError();
}

template <int EPI, int BK, bool DB>
hipError_t launch_layout(const PParams& p, bool at, bool bt, hipStream_t st) {
  if (!at && !bt) return launch_t<false, false, EPI, BK, DB>(p, st);
  if (at && !bt) return launch_t<true, false, EPI, BK, DB>(p, st);
  if (!at && bt) return launch_t<false, true, EPI, BK, DB>(p, st);
  return launch_t<true, true, EPI, BK, DB>(p, st);
}

// variant (diagnostics): 0 = single-buffered BK 64 (default: 40 KB LDS, 2-3 WGs/CU),
// 1 = double-buffered BK 32, 2 = double-buffered BK 64 (80 KB LDS: one workgroup per CU).
// Measured on the C2 shapes (profiles/r1/gemm_ab_bf16_variants.txt): BK-64 single buffer
// fastest everywhere (e.g. 308 vs 274 vs 179 TF/s on the layer-0 forward).
template <int EPI>
hipError_t launch_var(const PParams& p, bool at, bool bt, int variant, hipStream_t st) {
  if constexpr (EPI == EPI_STORE) {
    if (variant == 1) return launch_layout<EPI, 32, true>(p, at, bt, st);
    if (variant == 2) return launch_layout<EPI, 64, true>(p, at, bt, st);
  }
  return launch_layout<EPI, 64, false>(p, at, bt, st);
}

}  // namespace

bool gemm_bf16_wide(const GemmDesc& d) {
  if (d.prec == GEMM_F32) return false;
  // 10-12, 15: default-shape variants of the ring kernel (C/D epilogue, forced tile N, no
  // eight-phase kernel); 3: the ring kernel, 6 / 13 / 14: the eight-phase kernel, on any shape
  const int v = (d.variant >= 10 && d.variant != 13 && d.variant != 14) ? 0 : d.variant;
  if (v == 1 || v == 2 || v == 4) return false;  // 128x128 register-staged variants
  // output dimensions >= 128 (the thin decoder / latent-head GEMMs of C3-C5: a 256-row ring
  // tile ran them 1.6-1.7x faster than the 128x128 register-staged kernel, profiles/r4/README.md)
  if (v != 3 && v != 6 && v != 13 && v != 14 && (d.M < 128 || d.N < 128)) return false;
  // one k-tile and under a CU's worth of 256x256 tiles (dec layer 1: K = L + 1; the head's
  // dgrad: K = 2L): epilogue-bound on few CUs, the 128x128 kernels spread it wider
  const long long t256 = (long long)((d.M + 255) / 256) * ((d.N + 255) / 256) * d.batch;
  if (v == 0 && d.K <= 64 && t256 < 256) return false;
  auto a8 = [](long long v) { return (v & 7) == 0; };
  if (!a8(d.lda) || !a8(d.ldb) || !a8(d.pA) || !a8(d.pB)) return false;
  if (d.batch > 1 && (!a8(d.sA) || !a8(d.sB))) return false;
  if ((reinterpret_cast<uintptr_t>(d.Ap) | reinterpret_cast<uintptr_t>(d.Bp)) & 15) return false;
  return true;
}

// Joint choice of the kernel (256 x 256 eight-phase kernel; 256 x 256 / 256 x 128 / 192 x 256 /
// 192 x 128 ring kernels) and split-K: each kernel's time is its rounds of resident workgroups
// (one per CU) x (k-tiles + fixed prologue/epilogue cost) x its time per k-tile; split-K adds the
// fp32 slab round trip and the reduction launch. Variants 11 / 12 force the ring kernel at tile
// N 128 / 256, 13 / 14 the eight-phase kernel, 15 the ring kernels only.
struct WidePlan { int split = 1; int tn = 256; int tm = 256; };
static WidePlan wide_plan(const GemmDesc& d, size_t max_ws) {
  const bool fixed = d.epi.mode == EPI_BCE || d.epi.mode == EPI_BCEB || d.epi.mode == EPI_SIGMOID;
  const int kt = (d.K + 63) / 64;
  const bool x3 = d.x3 && d.prec == GEMM_F32X && d.nA == 3 && d.nB == 3;
  const int T = d.nA > d.nB ? d.nA : d.nB;
  int np = 0;
  for (int i = 0; i < d.nA; ++i)
    for (int j = 0; j < d.nB; ++j) np += i + j < T;
  if (d.dynA) np = (np + (d.nB < T ? d.nB : T)) / 2;  // A's residual planes often all zero
  const bool big = d.M >= 256 && d.N >= 256;
  const bool force_e8 = d.variant == 13 || d.variant == 14 || d.variant == 6;
  // the eight-phase kernel where it measured faster than the ring kernels (profiles/r4): enough
  // 256x256 tiles to fill the chip, or a long k-loop over >= 32 tiles; its (k-tile, pair)
  // iterations copy both operand images (the ring kernel reuses an unchanged image)
  const long long t256 = (long long)((d.M + 255) / 256) * ((d.N + 255) / 256) * d.batch;
  // 192-row ring tiles: k-contiguous A, epilogues other than the BCE head / sigmoid
  const bool t192 = !d.at && d.epi.mode != EPI_BCE && d.epi.mode != EPI_BCEB &&
                    d.epi.mode != EPI_SIGMOID;
  const long long tl192 = (long long)((d.M + 191) / 192) * ((d.N + 255) / 256) * d.batch;
  // ... except (in-step A/B, profiles/r4/README.md) single-product GEMMs where one round of
  // 192-row ring tiles keeps >= 4/3 as many CUs busy (C3 layer-0 forward: 256 vs 192 workgroups,
  // 0.255 vs 0.276 ms; hidden forward 31.7 vs 32.7 us)
  // (a real one-round fill: not a tile count split-K multiplies anyway -- the C3 decoder-output
  // dgrad, 86 vs 64 tiles, stays on the eight-phase kernel: 0.107 vs 0.115 ms in r4n)
  const bool ring_fills = t192 && np == 1 && tl192 > 128 && tl192 <= 256 && 3 * tl192 >= 4 * t256;
  const bool e8_rule = big && t256 >= 32 && (t256 >= 256 || (long long)np * kt >= 64) && !ring_fills;
  // the eight-phase kernel addresses an operand plane by 32-bit per-lane element offsets
  const long long ea = (long long)(d.at ? d.K : d.M) * d.lda, eb = (long long)(d.bt ? d.N : d.K) * d.ldb;
  const bool e8_fits = ea < (1LL << 32) && eb < (1LL << 32);
  // A as bits (a 0/1 operand): the eight-phase kernel, whose bits path reads it (its plane path
  // runs the rare batch with another pixel value)
  const bool allow_e8 = e8_fits && (force_e8 || (d.variant == 0 && (e8_rule || d.Abits)));
  double best = 1e30;
  WidePlan pl;
  for (int cand = 0; cand < 5; ++cand) {
    // candidates: ring 256x256, 256x128, eight-phase 256x256, ring 192x256, 192x128
    const bool e8 = cand == 2;
    const int w = cand == 0 || cand == 3 ? 256 : cand == 1 || cand == 4 ? 128 : TN_E8;
    const int tmr = cand >= 3 ? 192 : 256;
    if (e8 ? !allow_e8 : allow_e8 || (force_e8 && e8_fits)) continue;
    if (!e8 && d.Abits && e8_fits && d.variant == 0) continue;
    if (cand >= 3 && !t192) continue;
    if ((d.tm == 192 && t192 && cand != 3 && cand != 4) || (d.tm == 256 && cand >= 3)) continue;
    if (d.variant == 11 && w != 128) continue;
    if (d.variant == 12 && w != 256) continue;
    if (!e8 && (d.M < 128 || d.N < 128) && d.variant != 3 && d.variant < 10) continue;
    const int tnn = e8 ? 256 : w;
    const long long tiles = (long long)((d.M + tmr - 1) / tmr) * ((d.N + tnn - 1) / tnn) * d.batch;
    // ring kernels, measured: 4096^3 at 1.06 PF/s = 1.94 us per 256x256 k-tile per CU; the
    // 256x128 tile does half the MFMA work per k-tile in ~1.5 us (profiles/r2/gemm_ab_tile_n.txt);
    // 192-row tiles interpolated (a fixed ~1.1 us per k-tile plus ~0.1 us per 32x32 block).
    // eight-phase kernel: per 256x256 k-tile (gemm_bf16e.hip)
    double t_kt = e8 ? 1.35e-6 : tmr == 192 ? (w == 256 ? 1.7e-6 : 1.4e-6) : (w == 256 ? 1.9e-6 : 1.5e-6);
    // the plane-stacked kernel (option x3) serves the six-pair f32x ring plans at tile N 128:
    // C2 hidden forward 60 -> 50 us, hidden dgrad 72 -> 67 us in the region pass (r6zi)
    if (x3 && !e8 && w == 128) t_kt *= 0.88;
    const double fix = 3.0;
    for (int s = 1; s <= (fixed ? 1 : 32); ++s) {
      if (s > 1 && kt / s < 2) break;
      if (s > 1 && (size_t)d.batch * s * d.M * d.N > max_ws) break;
      const double rounds = std::ceil(tiles * s / 256.0);
      double t = rounds * (np * std::ceil((double)kt / s) + fix) * t_kt;
      // split-K: the slabs' write + read and the reduction launch (8 us fixed: C2's f32x hidden
      // forward, 12288 x 500 x 501, ran 65.6 us at 192x256 split 2 against 61.0 us as one round
      // of 192x128 tiles unsplit, where the model with 4 us preferred the split, r5zq)
      if (s > 1) t += (double)d.batch * s * d.M * d.N * 8.0 / 4.5e12 + 8e-6;
      if (t < best * 0.97) { best = t; pl.split = s; pl.tn = w; pl.tm = tmr; }
    }
  }
  return pl;
}

int gemm_bf16_wide_split(const GemmDesc& d, size_t max_ws) { return wide_plan(d, max_ws).split; }

int gemm_bf16_wide_tn(const GemmDesc& d, size_t max_ws) { return wide_plan(d, max_ws).tn; }

int gemm_bf16_wide_tm(const GemmDesc& d, size_t max_ws) { return wide_plan(d, max_ws).tm; }

void gemm_bf16_wide_plan(const GemmDesc& d, size_t max_ws, int* split, int* tn, int* tm) {
  const WidePlan pl = wide_plan(d, max_ws);
  *split = pl.split; *tn = pl.tn; *tm = pl.tm;
}

hipError_t gemm_bf16_launch(const gemm::Params& g, const GemmDesc& d, int epi, hipStream_t st) {
  PParams p;
  p.g = g;
  p.A = d.Ap; p.pA = d.pA;
  p.B = d.Bp; p.pB = d.pB;
  p.dyn = d.dynA;
  p.diag = d.diag;
  p.stamps = d.stamps;
  p.abits = d.Abits; p.abits_kts = d.abits_kts; p.abits_sb = d.abits_sb; p.anb = d.anb;
  p.dj = d.dj;
  p.bits_reg = d.bits_reg;
  p.prio = d.prio;
  p.x3 = d.x3;
  // the fused de-interleave rides on the eight-phase kernel's bits path only
  if (d.dj.nworkers && (g.tn != TN_E8 || !d.Abits || d.at || d.bt || (epi != EPI_STORE && epi != EPI_ACT)))
    return hipErrorInvalidValue;
  // tile order: bands of 8 m-tiles walked n by n when a row has >= 8 n-tiles, so the 32 tiles
  // an XCD holds at once share 8 A and 4 B tiles in its L2 (C5 latent-head forward
  // 24576 x 4000 x 501: 0.177 -> 0.161 ms; neutral on the BCE head and the other shapes,
  // profiles/r4/r4u_tile_group.txt); GemmDesc::group >= 0 overrides (A/B: mvae_bench_gemm)
  const int tile_group = d.group;
  // plane pairs (i, j), i + j < max(nA, nB); the pairs with i = 0 first, j snaking (ascending for
  // even i, descending for odd i): (0,0) (0,1) (0,2) (1,1) (1,0) (2,0), so consecutive pairs share
  // the B plane at both A-plane changes and the ring kernel copies 3 A + 5 B images per k-tile
  // instead of 3 + 6
  int n = 0;
  const int T = d.nA > d.nB ? d.nA : d.nB;
  for (int i = 0; i < d.nA; ++i)
    for (int jj = 0; jj < d.nB; ++jj) {
      const int j = (i & 1) ? d.nB - 1 - jj : jj;
      if (i + j < T) { p.pa[n] = (unsigned char)i; p.pb[n] = (unsigned char)j; ++n; }
    }
  p.npairs = n;
  p.npairs0 = d.nB < T ? d.nB : T;  // pairs with i == 0
  p.npairs_a0 = p.npairs0;
  if (!p.dyn) p.npairs0 = n;
  p.pab = 0;
  for (int i = 0; i < n; ++i) p.pab |= (p.pa[i] | p.pb[i] << 2) << (4 * i);
  // the eight-phase kernel's image-reusing walk (plane pairs only; the BCE head's whole-round
  // launch then sums in another order than its 256x128 ring-tile remainder, bce_split: the same
  // values to fp32 rounding)
  p.reuse = n > 1;
  if (gemm_bf16_wide(d)) {
    // tile N: the planner's (gemm_run), 256 for the diagnostic variants of the 256x256 forms
    const bool q = d.variant == 0 || d.variant == 3 || d.variant == 6 || (d.variant >= 10 && d.variant <= 15);
    p.g.tn = q && (g.tn == 128 || g.tn == TN_E8) ? g.tn : 256;
    p.g.tm = q && p.g.tn != TN_E8 && g.tm == 192 && !d.at ? 192 : 256;
    const int tm = p.g.tm, tn = p.g.tn == TN_E8 ? 256 : p.g.tn;
    p.g.ntm = (d.M + tm - 1) / tm;
    p.g.ntn = (d.N + tn - 1) / tn;
    p.g.group = tile_group >= 0 ? tile_group : (p.g.ntn >= 8 ? 8 : 0);
    switch (epi) {
      case EPI_STORE: return launch_wide<EPI_STORE>(p, d.at, d.bt, d.variant, st);
      case EPI_ACT: return launch_wide<EPI_ACT>(p, d.at, d.bt, d.variant, st);
      case EPI_DACT:
        return d.epi.auxp ? launch_wide<EPI_DACTB>(p, d.at, d.bt, d.variant, st)
                          : launch_wide<EPI_DACT>(p, d.at, d.bt, d.variant, st);
      case EPI_BCE: return launch_wide<EPI_BCE>(p, d.at, d.bt, d.variant, st);
      case EPI_BCEB: return launch_wide<EPI_BCEB>(p, d.at, d.bt, d.variant, st);
      case EPI_SIGMOID: return launch_wide<EPI_SIGMOID>(p, d.at, d.bt, d.variant, st);
      default: return hipErrorInvalidValue;
    }
  }
  switch (epi) {
    case EPI_STORE: return launch_var<EPI_STORE>(p, d.at, d.bt, d.variant, st);
    case EPI_ACT: return launch_var<EPI_ACT>(p, d.at, d.bt, d.variant, st);
    case EPI_DACT: return launch_var<EPI_DACT>(p, d.at, d.bt, d.variant, st);
    case EPI_BCE: return launch_var<EPI_BCE>(p, d.at, d.bt, d.variant, st);
    case EPI_BCEB: return launch_var<EPI_BCEB>(p, d.at, d.bt, d.variant, st);
    case EPI_SIGMOID: return launch_var<EPI_SIGMOID>(p, d.at, d.bt, d.variant, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mvae
