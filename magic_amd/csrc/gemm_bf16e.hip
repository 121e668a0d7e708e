// Eight-phase bf16-MFMA GEMM for gfx950: 256 x 256 x 64 tiles, 512 threads = 8 waves in
// 2 (M) x 4 (N), each wave 128 x 64 = 4 x 2 accumulators of v_mfma_f32_32x32x16_bf16 (fp32).
// Same operands (bf16 plane images, f32x plane pairs walked (k-tile, pair) pairs-innermost),
// tile order, epilogues and results as the ring kernel (gemm_bf16.hip); what differs is the
// main loop, rebuilt on the ping-pong schedule of cdna_hip_programming.md "The 256^2 8-phase
// template" (T3+T4, T5):
//
// * each wave's 128 x 64 block is four quadrants (m, n) of 64 x 32 (2 x 1 accumulators); one
//   PHASE = the fragment reads one quadrant needs + one half-tile LDS-DMA -> s_barrier ->
//   lgkmcnt(0) -> 8 MFMAs at s_setprio 1 -> s_barrier. A k-tile is 4 phases:
//     q1: (0,0) reads A-sub 0 and B-sub 0   q2: (0,1) reads B-sub 1
//     q3: (1,1) reads A-sub 1               q4: (1,0) reads nothing (B-sub 0 still in registers)
// * waves 4-7 run one barrier behind waves 0-3 (one extra s_barrier before the loop), so on
//   every SIMD -- which holds one wave of each half -- one wave issues its LDS reads and DMA
//   while its partner runs MFMAs, and the roles swap at each barrier;
// * operand tiles travel as HALF images (128 rows x 64 k, 16 KB): half h of A holds the rows
//   of A-sub h of both wave rows, half h of B the columns of B-sub h of all four wave columns,
//   so a quadrant's reads touch one A half and one B half only. Two buffers (even / odd
//   k-tile) x {A0, A1, B0, B1} = 128 KB of LDS. A half is re-filled once its last reader is
//   two phases back: k-tile t issues B1(t+1) in q1, A1(t+1) in q2, A0(t+2) in q3, B0(t+2) in
//   q4; the data a phase reads is waited for (counted vmcnt, never 0 in steady state: three
//   half-tiles stay in flight across the barriers) one phase earlier, before that phase's
//   first barrier, which every reader passes after the wait (MI355X_MICROARCH.md, two waves
//   per SIMD, item 7).
// The LDS images are lane-linear (global_load_lds_dwordx4) with the conflict-free XOR swizzles
// of the ring kernel applied to the per-lane source address and undone on the read.
#include "gemm_common.h"

#include <cstdint>

namespace mvae {
namespace {

using namespace gemm;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) short lds_short;

constexpr int EBK = 64;          // k-tile
constexpr int EH = 128 * EBK;    // bf16 elements per half image (16 KB)
constexpr int EHB = 2 * EH;      // ... bytes
constexpr int ENT = 512;

// One operand's half images, copied by buffer_load_dwordx4 ... lds (a buffer resource over the
// operand's plane, 2 GB range): per lane only a 32-bit byte offset; the k-tile's offset is the
// scalar soffset, and chunks that must read as zero (past K, or row chunks past the operand's
// rows) take an offset past the resource's range, which the hardware returns as zeros.
// Image row i (0..127) of half h is tile row (column, for B) 128 h + i, so a row-contiguous
// operand's DMA reads whole 256-B row segments. Each lane copies 2 16-B chunks per half (8 waves
// x 64 lanes x 2 = 1024 chunks = 16 KB):
//   k-contiguous ([rows][K] in HBM): image [128 rows][8 chunks of 8 k], chunk c of row i stored
//     at c ^ ((i >> 1) & 7) -> ds_read_b128 fragment reads conflict-free;
//   row-contiguous ([K][rows]): image [64 k][16 chunks of 8 rows], chunk c of k-row k stored
//     at c ^ tr_swz(k) -> the 32 lanes of a ds_read_b64_tr_b16 pass hit 32 distinct slots.
// Rows past the end of a k-contiguous operand are clamped (their outputs are not stored).
constexpr unsigned OOB = 0x80000000u;  // >= the resource's num_records: loads zeros
// chunk swizzle of a row-contiguous image's k-row k: the 4 (k & 3) term spreads the four k-rows
// of one ds_read_b64_tr_b16 block over the bank row (the 2 ((k >> 3) & 1) term, constant within a
// 32-lane half, kept from the removed 16x16x32 form: conflict-free either way)
__device__ __forceinline__ int tr_swz(int k) { return (4 * (k & 3)) ^ (2 * ((k >> 3) & 1)); }
template <bool KC>
struct HLoad {
  unsigned voff[2][2];  // [chunk j][half h]: byte offset of the chunk at k0 = 0, or OOB
  int kc[2];            // its k within the tile (k-contiguous: 8c; else the k row)
  __device__ __forceinline__ static int map(int i, int h) { return h * 128 + i; }
  __device__ __forceinline__ void init(int ld, int r0, int nrows, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = (j * 8 + wave) * 64 + lane;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (KC) {
          const int i = q >> 3;
          const int c = (q & 7) ^ ((i >> 1) & 7);
          int gr = r0 + map(i, h);
          gr = gr < nrows ? gr : nrows - 1;
          voff[j][h] = 2u * ((unsigned)gr * (unsigned)ld + 8u * c);
          kc[j] = 8 * c;
        } else {
          const int krow = q >> 4;
          const int c = (q & 15) ^ tr_swz(krow);
          const int col = r0 + map(8 * c, h);
          voff[j][h] = col < nrows ? 2u * ((unsigned)krow * (unsigned)ld + (unsigned)col) : OOB;
          kc[j] = krow;
        }
      }
    }
  }
  // half H of the k-tile at k0 (tile k-range ends at kend) from the plane at g into img;
  // wave: the wave index as a scalar
  // chunks J0 .. J1-1 of the lane (the half's 2 DMA instructions, or one of them)
  template <int H, int J0 = 0, int J1 = 2>
  __device__ __forceinline__ void issue(const unsigned short* g, int ld, int k0, int kend, short* img,
                                        int wave, bool lin = false) const {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(g), (short)0, (int)OOB, 0x00020000);
    const unsigned soff = KC ? 2u * (unsigned)k0 : 2u * (unsigned)k0 * (unsigned)ld;
    const int kl = k0 + EBK <= kend ? (1 << 30) : kend - k0;  // chunks at k >= kl read zeros
#pragma unroll
    for (int j = J0; j < J1; ++j) {
      unsigned v = kc[j] < kl ? voff[j][H] : OOB;
      if (lin) v = 16u * (threadIdx.x + 512u * j);  // diagnostics: linear source (wrong data)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(img + (j * 8 + wave) * 512), 16, v, soff, 0, 0);
    }
  }
};

// fragment reads (8 consecutive k of one 32-row block) at an LDS byte address + immediate
// offset, in inline asm: hipcc neither waits vmcnt(0) for the in-flight DMA (the transposing-
// read builtin makes it) nor lgkmcnt(0) early; each phase waits for its own reads
template <int OFF>
__device__ __forceinline__ bf16x8 rd_b128(unsigned a) {
  s16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return __builtin_bit_cast(bf16x8, v);
}
template <int OFF>
__device__ __forceinline__ bf16x8 rd_tr(unsigned a) {
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a), "i"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a), "i"(OFF + 4 * 256));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
// per-lane byte offset within a half image of the fragment of the 32-row block at image row rb,
// k16-step ks
template <bool KC>
__device__ __forceinline__ unsigned frag_addr(int rb, int ks, int lane) {
  if constexpr (KC) {
    const int row = rb + (lane & 31);
    const int pos = (2 * ks + (lane >> 5)) ^ ((row >> 1) & 7);
    return (unsigned)(row * 128 + pos * 16);
  } else {
    const int i = lane & 15, q = i >> 2, pp = i & 3;
    const int kk = 16 * ks + 8 * (lane >> 5) + q;
    const int ro = rb + 16 * ((lane >> 4) & 1) + 4 * pp;
    const int pos = (ro >> 3) ^ tr_swz(kk);
    return (unsigned)(kk * 256 + pos * 16 + 2 * (ro & 4));
  }
}

// at most 2n LDS-DMA instructions (n half-tiles) of this wave outstanding
__device__ __forceinline__ void wait_halves(int n) {
  if (n >= 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// main-loop state of one workgroup (registers once inlined). ST: stamped diagnostics build --
// per wave, the shader-clock cycles of each of a k-tile's 8 barrier-delimited slots summed over
// the k-loop (mvae_bench_gemm with MVAE_STAMPS=2; never in the step)
// (Measured and removed, profiles/r4/README.md: a 16x16x32-MFMA form -- higher clock, more
// cycles, no faster -- and issuing the DMA between the MFMAs -- 25 % slower.)
template <bool AT, bool BT, bool ST = false>
struct E8 {
  static constexpr bool KA = !AT, KB = BT;  // operand images k-contiguous?
  HLoad<KA> la;
  HLoad<KB> lb;
  f32x16 acc[4][2];
  // A-sub 0 / 1 (64 rows x 64 k) and B-sub 0 / 1 (32 cols x 64 k) fragments: fa[4 r + ks]
  // (32-row block r 0..1, k16-step ks 0..3), fb[ks]
  bf16x8 fa0[8], fa1[8], fb0[4], fb1[4];
  // fragment base addresses: A [ks] (k-contiguous) / [r], B [ks] / [0]
  unsigned aA[4], aB[4];
  const unsigned short* A;
  const unsigned short* Bm;
  short* smem;
  int wave;
  unsigned long long st_last, st_acc[ST ? 8 : 1];

  // the barrier closing slot K of a k-tile (stamped builds: its cycles since the previous one)
  template <int K>
  __device__ __forceinline__ void sbar() {
    bar();
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      st_acc[K] += t - st_last;
      st_last = t;
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // A half H of buffer Bf at byte (2 H + Bf) EHB; B half H at (4 + 2 H + Bf) EHB (aB includes 4 EHB)
  template <int H, int Bf>
  __device__ __forceinline__ void rd_a(bf16x8 (&fa)[8]) {
    constexpr int O = (2 * H + Bf) * EHB;
    if constexpr (KA) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        fa[ks] = rd_b128<O>(aA[ks]);
        fa[4 + ks] = rd_b128<O + 32 * 128>(aA[ks]);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        fa[4 * r] = rd_tr<O>(aA[r]);
        fa[4 * r + 1] = rd_tr<O + 4096>(aA[r]);
        fa[4 * r + 2] = rd_tr<O + 2 * 4096>(aA[r]);
        fa[4 * r + 3] = rd_tr<O + 3 * 4096>(aA[r]);
      }
    }
  }
  template <int H, int Bf>
  __device__ __forceinline__ void rd_b(bf16x8 (&fb)[4]) {
    constexpr int O = (2 * H + Bf) * EHB;
    if constexpr (KB) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) fb[ks] = rd_b128<O>(aB[ks]);
    } else {
      fb[0] = rd_tr<O>(aB[0]);
      fb[1] = rd_tr<O + 4096>(aB[0]);
      fb[2] = rd_tr<O + 2 * 4096>(aB[0]);
      fb[3] = rd_tr<O + 3 * 4096>(aB[0]);
    }
  }
  // the quadrant's 8 MFMAs once this wave's reads have landed
  template <int M, int N>
  __device__ __forceinline__ void mfma_q(const bf16x8 (&fa)[8], const bf16x8 (&fb)[4]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int r = 0; r < 2; ++r)
        acc[2 * M + r][N] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[4 * r + ks], fb[ks], acc[2 * M + r][N], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  template <int H, int Bf, int J0 = 0, int J1 = 2>
  __device__ __forceinline__ void issue_a(const PParams& pp, const Tile& t, int kt, int pr) {
    const int pa = (pp.pab >> (4 * pr)) & 3;
    la.template issue<H, J0, J1>(A + pa * pp.pA, pp.g.lda, t.ks + kt * EBK, t.ke, smem + (2 * H + Bf) * EH, wave,
                                 ST && (pp.diag & 2));
  }
  template <int H, int Bf, int J0 = 0, int J1 = 2>
  __device__ __forceinline__ void issue_b(const PParams& pp, const Tile& t, int kt, int pr) {
    const int pb = (pp.pab >> (4 * pr + 2)) & 3;
    lb.template issue<H, J0, J1>(Bm + pb * pp.pB, pp.g.ldb, t.ks + kt * EBK, t.ke, smem + (4 + 2 * H + Bf) * EH, wave,
                                 ST && (pp.diag & 2));
  }
  // k-tile `it` (its images in buffer Bf); (kt1, pr1), (kt2, pr2): (k-tile, pair) of it+1, it+2.
  // Fragment reads 4 / 4 / 8 / 8 per phase: B-sub 0 in q1, B-sub 1 in q2, A-sub 1 in q3 and the
  // NEXT k-tile's A-sub 0 in q4 (its registers are free after q2), each waited for (vmcnt) in the
  // phase before; the DMA of B1(it+1), A1(it+1), A0(it+2), B0(it+2) in q1..q4 refills a half
  // >= 3 phases after its last read.
  template <int Bf>
  __device__ __forceinline__ void tile(const PParams& pp, const Tile& t, int it, int total, int kt1, int pr1,
                                       int kt2, int pr2) {
    constexpr int Bn = Bf ^ 1;
    // stamped builds' A/B switches (results meaningless): diag 1 = no DMA after the prologue,
    // 2 = linear DMA source addresses, 64 = no fragment reads
    const bool dma = !ST || !(pp.diag & 1), rdf = !ST || !(pp.diag & 64);
    const bool n1 = it + 1 < total;  // a next k-tile exists (its A-sub 0 is read in q4)
    const bool m1 = n1 && dma, m2 = it + 2 < total && dma;
    // q1: (0,0) reads B0(it); B1(it) for q2 landed; B1(it+1)
    if (rdf) rd_b<0, Bf>(fb0);
    wait_halves(m1 ? 3 : 1);
    if (m1) issue_b<1, Bn>(pp, t, kt1, pr1);
    sbar<0>();
    mfma_q<0, 0>(fa0, fb0);
    sbar<1>();
    // q2: (0,1) reads B1(it); A1(it) for q3 landed; A1(it+1)
    if (rdf) rd_b<1, Bf>(fb1);
    wait_halves(m1 ? 3 : 0);
    if (m1) issue_a<1, Bn>(pp, t, kt1, pr1);
    sbar<2>();
    mfma_q<0, 1>(fa0, fb1);
    sbar<3>();
    // q3: (1,1) reads A1(it); A0(it+1) for q4 landed; A0(it+2) into the half A0(it) was read from
    if (rdf) rd_a<1, Bf>(fa1);
    if (m1) wait_halves(3);
    if (m2) issue_a<0, Bf>(pp, t, kt2, pr2);
    sbar<4>();
    mfma_q<1, 1>(fa1, fb1);
    sbar<5>();
    // q4: (1,0) reads A0(it+1); B0(it+1) for the next q1 landed; B0(it+2)
    if (rdf && n1) rd_a<0, Bn>(fa0);
    if (m1) wait_halves(m2 ? 3 : 2);
    if (m2) issue_b<0, Bf>(pp, t, kt2, pr2);
    sbar<6>();
    mfma_q<1, 0>(fa1, fb0);
    sbar<7>();
  }
};

template <bool AT, bool BT, int EPI, bool TE, bool ST = false>
__global__ __launch_bounds__(ENT, 1) void gemm_bf16e_kernel(PParams pp) {
  const Params& p = pp.g;
  if (epi_skip<EPI>(p.epi)) return;
  // [A0 b0 | A0 b1 | A1 b0 | A1 b1 | B0 b0 | B0 b1 | B1 b0 | B1 b1]; the row-major epilogue's two
  // 64-row bands and the BCE row partials reuse it after the k-loop
  constexpr int RING = 8 * EH;
  constexpr int EPIL = 2 * (2 * 64 * 256 + 64 * 4 * 32);
  __shared__ __attribute__((aligned(16))) short smem[RING > EPIL ? RING : EPIL];

  unsigned long long st_k0 = 0, st_k2 = 0;  // stamped builds: kernel start, k-loop end (realtime)
  if constexpr (ST) st_k0 = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const Tile t = tile_of_t<256, 256>(p, true);

  E8<AT, BT, ST> s;
  s.A = pp.A + t.bi * p.sA;
  s.Bm = pp.B + t.bi * p.sB;
  s.smem = smem;
  s.wave = __builtin_amdgcn_readfirstlane(wave);
  s.la.init(p.lda, t.m0, p.M, wave, lane);
  s.lb.init(p.ldb, t.n0, p.N, wave, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) s.acc[i][j][r] = 0.f;
  constexpr bool KA = E8<AT, BT, ST>::KA, KB = E8<AT, BT, ST>::KB;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_short*)smem;
#pragma unroll
  for (int i = 0; i < (KA ? 4 : 2); ++i)
    s.aA[i] = lds0 + (KA ? frag_addr<true>(wm * 64, i, lane) : frag_addr<false>(wm * 64 + 32 * i, 0, lane));
#pragma unroll
  for (int i = 0; i < (KB ? 4 : 1); ++i)
    s.aB[i] = lds0 + 4 * EHB + (KB ? frag_addr<true>(wn * 32, i, lane) : frag_addr<false>(wn * 32, 0, lane));

  const int np = (pp.dyn && *pp.dyn == 0) ? pp.npairs0 : pp.npairs;
  const int nkt = t.ks < t.ke ? (t.ke - t.ks + EBK - 1) / EBK : 0;
  const int total = np * nkt;
  // waves 4-7 (the second half of every SIMD pair), as a scalar condition: s_barrier ignores EXEC
  // (stamped builds, diag 128: no stagger -- both halves in the same phase)
  const bool lag = __builtin_amdgcn_readfirstlane(wave) >= 4 && !(ST && (pp.diag & 128));

  if (total > 0) {
    // (k-tile, pair) cursors of tiles it+1 and it+2
    int kt1 = 0, pr1 = 0, kt2 = 0, pr2 = 0;
    auto adv = [&](int& kt, int& pr) { if (++pr == np) { pr = 0; ++kt; } };
    // prologue: A0 B0 B1 A1 of tile 0, A0 B0 of tile 1
    s.template issue_a<0, 0>(pp, t, 0, 0);
    s.template issue_b<0, 0>(pp, t, 0, 0);
    s.template issue_b<1, 0>(pp, t, 0, 0);
    s.template issue_a<1, 0>(pp, t, 0, 0);
    adv(kt1, pr1);
    kt2 = kt1; pr2 = pr1;
    adv(kt2, pr2);
    if (total > 1) {
      s.template issue_a<0, 1>(pp, t, kt1, pr1);
      s.template issue_b<0, 1>(pp, t, kt1, pr1);
    }
    wait_halves(total > 1 ? 4 : 2);
    bar();
    s.template rd_a<0, 0>(s.fa0);  // tile 0's A-sub 0 (later tiles': read in the previous q4)
    if (lag) bar();
    unsigned long long st_t0 = 0, st_r0 = 0;
    if constexpr (ST) {
#pragma unroll
      for (int k = 0; k < 8; ++k) s.st_acc[k] = 0;
      st_r0 = __builtin_amdgcn_s_memrealtime();
      st_t0 = s.st_last = __builtin_amdgcn_s_memtime();
    }
    for (int it = 0; it < total; it += 2) {
      s.template tile<0>(pp, t, it, total, kt1, pr1, kt2, pr2);
      kt1 = kt2; pr1 = pr2; adv(kt2, pr2);
      if (it + 1 < total) {
        s.template tile<1>(pp, t, it + 1, total, kt1, pr1, kt2, pr2);
        kt1 = kt2; pr1 = pr2; adv(kt2, pr2);
      }
    }
    if (!lag) bar();
    if constexpr (ST) {
      const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) {
        unsigned long long* o = pp.stamps + 16 * ((size_t)blockIdx.x * 8 + wave);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = s.st_acc[k];
        o[8] = t1 - st_t0; o[9] = r1 - st_r0; o[10] = total;
        o[11] = st_r0 - st_k0;  // prologue (realtime ticks, 100 MHz)
      }
      st_k2 = r1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // The LDS row-major epilogue for every output (16-B global accesses when te, else element-wise).
  // A wave's accumulator block (m, r) (A-sub m, 32-row block r) is tile rows 128 m + 64 wm + 32 r
  // and its block n (B-sub n) tile columns 128 n + 32 wn (contiguous half images); band mi holds
  // block (mi >> 1, mi & 1) of both wave rows (RMAP 1). The band's blocks are always the first
  // ones (rotated down after each band: the band loop is not unrolled).
  float* const lds_f = reinterpret_cast<float*>(smem);
  {  // 32x32 blocks (C/D layout: col lane & 31, row (r & 3) + 8 (r >> 2) + 4 (lane >> 5))
    auto wb = [&](float* band, int) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          band[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 256 + n * 128 + wn * 32 + (lane & 31)] =
              s.acc[0][n][r];
#pragma unroll
      for (int i = 0; i + 1 < 4; ++i)
#pragma unroll
        for (int n = 0; n < 2; ++n) s.acc[i][n] = s.acc[i + 1][n];
    };
    epilogue_rm_w<EPI, 4, 256, ENT, decltype(wb)&, 1>(p, t, wb, lds_f, 0, nullptr, lds_f + 2 * 64 * 256, TE);
  }
  if constexpr (ST) {  // epilogue: from the k-loop's end until every store of the workgroup issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane == 0 && st_k2) pp.stamps[16 * ((size_t)blockIdx.x * 8 + wave) + 12] = __builtin_amdgcn_s_memrealtime() - st_k2;
  }
}

template <bool AT, bool BT, int EPI, bool TE>
hipError_t launch_e(const PParams& p, hipStream_t st) {
  const int nwg = p.g.ntm * p.g.ntn * p.g.batch * p.g.split;
  if constexpr (EPI == EPI_STORE) {  // the stamped diagnostics build (mvae_bench_gemm)
    if (p.stamps) {
      hipLaunchKernelGGL((gemm_bf16e_kernel<AT, BT, EPI, TE, true>), dim3(nwg), dim3(ENT), 0, st, p);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_bf16e_kernel<AT, BT, EPI, TE>), dim3(nwg), dim3(ENT), 0, st, p);
  return hipGetLastError();
}

template <int EPI, bool TE>
hipError_t launch_e_l(const PParams& p, bool at, bool bt, hipStream_t st) {
  if (!at && !bt) return launch_e<false, false, EPI, TE>(p, st);
  if (at && !bt) return launch_e<true, false, EPI, TE>(p, st);
  if (!at && bt) return launch_e<false, true, EPI, TE>(p, st);
  return launch_e<true, true, EPI, TE>(p, st);
}

template <int EPI>
hipError_t launch_e_t(const PParams& p, bool at, bool bt, bool te, hipStream_t st) {
  return te ? launch_e_l<EPI, true>(p, at, bt, st) : launch_e_l<EPI, false>(p, at, bt, st);
}

}  // namespace

// the eight-phase kernel for a planned 256 x 256 tile (PParams::g.tn == TN_E8): te = the row-major
// LDS epilogue (planes / BCE outputs with 16-B aligned rows), else the C/D-layout epilogue
hipError_t gemm_bf16e_launch(const PParams& p, bool at, bool bt, int epi, bool te, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_e_t<EPI_STORE>(p, at, bt, te, st);
    case EPI_ACT: return launch_e_t<EPI_ACT>(p, at, bt, te, st);
    case EPI_DACT: return launch_e_t<EPI_DACT>(p, at, bt, te, st);
    case EPI_DACTB: return launch_e_t<EPI_DACTB>(p, at, bt, te, st);
    case EPI_BCE: return launch_e_t<EPI_BCE>(p, at, bt, te, st);
    case EPI_BCEB: return launch_e_t<EPI_BCEB>(p, at, bt, te, st);
    case EPI_SIGMOID: return launch_e_t<EPI_SIGMOID>(p, at, bt, te, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mvae
