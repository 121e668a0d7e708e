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
// Image row i (0..127) of half h is tile row map(i, h): SUB rows of each wave slice (A: 2 wave
// rows x 64, B: 4 wave columns x 32). Each lane copies 2 16-B chunks per half (8 waves x 64
// lanes x 2 = 1024 chunks = 16 KB):
//   k-contiguous ([rows][K] in HBM): image [128 rows][8 chunks of 8 k], chunk c of row i stored
//     at c ^ ((i >> 1) & 7) -> ds_read_b128 fragment reads conflict-free;
//   row-contiguous ([K][rows]): image [64 k][16 chunks of 8 rows], chunk c of k-row k stored
//     at c ^ (4 (k & 3)) -> the 32 lanes of a ds_read_b64_tr_b16 pass hit 32 distinct slots.
// Rows past the end of a k-contiguous operand are clamped (their outputs are not stored).
constexpr unsigned OOB = 0x80000000u;  // >= the resource's num_records: loads zeros
template <bool KC, int SUB>
struct HLoad {
  unsigned voff[2][2];  // [chunk j][half h]: byte offset of the chunk at k0 = 0, or OOB
  int kc[2];            // its k within the tile (k-contiguous: 8c; else the k row)
  __device__ __forceinline__ static int map(int i, int h) {
    return (i / SUB) * (2 * SUB) + h * SUB + (i % SUB);
  }
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
          const int c = (q & 15) ^ (4 * (krow & 3));
          const int col = r0 + map(8 * c, h);
          voff[j][h] = col < nrows ? 2u * ((unsigned)krow * (unsigned)ld + (unsigned)col) : OOB;
          kc[j] = krow;
        }
      }
    }
  }
  // half H of the k-tile at k0 (tile k-range ends at kend) from the plane at g into img;
  // wave: the wave index as a scalar
  template <int H>
  __device__ __forceinline__ void issue(const unsigned short* g, int ld, int k0, int kend, short* img,
                                        int wave) const {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(g), (short)0, (int)OOB, 0x00020000);
    const unsigned soff = KC ? 2u * (unsigned)k0 : 2u * (unsigned)k0 * (unsigned)ld;
    const int kl = k0 + EBK <= kend ? (1 << 30) : kend - k0;  // chunks at k >= kl read zeros
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned v = kc[j] < kl ? voff[j][H] : OOB;
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
// per-lane byte offset within a half image of the fragment of the 32-row block at image row
// rb, k16-step ks
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
    const int pos = (ro >> 3) ^ (4 * (kk & 3));
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

// main-loop state of one workgroup (registers once inlined)
template <bool AT, bool BT>
struct E8 {
  static constexpr bool KA = !AT, KB = BT;  // operand images k-contiguous?
  HLoad<KA, 64> la;
  HLoad<KB, 32> lb;
  f32x16 acc[4][2];
  bf16x8 fa[2][4], fb0[4], fb1[4];  // A-sub [block][k16-step], B-sub 0 / 1 [k16-step]
  unsigned aA[KA ? 4 : 2], aB[KB ? 4 : 1];
  const unsigned short* A;
  const unsigned short* Bm;
  short* smem;
  int wave;

  // A half H of buffer Bf at byte (2 H + Bf) EHB; B half H at (4 + 2 H + Bf) EHB (aB includes 4 EHB)
  template <int H, int Bf>
  __device__ __forceinline__ void rd_a() {
    constexpr int O = (2 * H + Bf) * EHB;
    if constexpr (KA) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        fa[0][ks] = rd_b128<O>(aA[ks]);
        fa[1][ks] = rd_b128<O + 32 * 128>(aA[ks]);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        fa[r][0] = rd_tr<O>(aA[r]);
        fa[r][1] = rd_tr<O + 4096>(aA[r]);
        fa[r][2] = rd_tr<O + 2 * 4096>(aA[r]);
        fa[r][3] = rd_tr<O + 3 * 4096>(aA[r]);
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
  __device__ __forceinline__ void mfma_q(const bf16x8 (&fb)[4]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int r = 0; r < 2; ++r)
        acc[2 * M + r][N] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[r][ks], fb[ks], acc[2 * M + r][N], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  template <int H, int Bf>
  __device__ __forceinline__ void issue_a(const PParams& pp, const Tile& t, int kt, int pr) {
    const int pa = (pp.pab >> (4 * pr)) & 3;
    la.template issue<H>(A + pa * pp.pA, pp.g.lda, t.ks + kt * EBK, t.ke, smem + (2 * H + Bf) * EH, wave);
  }
  template <int H, int Bf>
  __device__ __forceinline__ void issue_b(const PParams& pp, const Tile& t, int kt, int pr) {
    const int pb = (pp.pab >> (4 * pr + 2)) & 3;
    lb.template issue<H>(Bm + pb * pp.pB, pp.g.ldb, t.ks + kt * EBK, t.ke, smem + (4 + 2 * H + Bf) * EH, wave);
  }
  // k-tile `it` (its images in buffer Bf); (kt1, pr1), (kt2, pr2): (k-tile, pair) of it+1, it+2
  template <int Bf>
  __device__ __forceinline__ void tile(const PParams& pp, const Tile& t, int it, int total, int kt1, int pr1,
                                       int kt2, int pr2) {
    constexpr int Bn = Bf ^ 1;
    const bool m1 = it + 1 < total, m2 = it + 2 < total;
    // q1: (0,0); B1(it) for q2 landed; B1(it+1)
    rd_a<0, Bf>();
    rd_b<0, Bf>(fb0);
    wait_halves(m1 ? 3 : 1);
    if (m1) issue_b<1, Bn>(pp, t, kt1, pr1);
    bar();
    mfma_q<0, 0>(fb0);
    bar();
    // q2: (0,1); A1(it) for q3 landed; A1(it+1)
    rd_b<1, Bf>(fb1);
    wait_halves(m1 ? 3 : 0);
    if (m1) issue_a<1, Bn>(pp, t, kt1, pr1);
    bar();
    mfma_q<0, 1>(fb1);
    bar();
    // q3: (1,1); A0(it+2) into the A0 half q1 read
    rd_a<1, Bf>();
    if (m2) issue_a<0, Bf>(pp, t, kt2, pr2);
    bar();
    mfma_q<1, 1>(fb1);
    bar();
    // q4: (1,0); A0(it+1), B0(it+1) for the next q1 landed; B0(it+2)
    if (m1) wait_halves(m2 ? 3 : 2);
    if (m2) issue_b<0, Bf>(pp, t, kt2, pr2);
    bar();
    mfma_q<1, 0>(fb0);
    bar();
  }
};

template <bool AT, bool BT, int EPI, bool TE>
__global__ __launch_bounds__(ENT, 1) void gemm_bf16e_kernel(PParams pp) {
  const Params& p = pp.g;
  if (epi_skip<EPI>(p.epi)) return;
  // [A0 b0 | A0 b1 | A1 b0 | A1 b1 | B0 b0 | B0 b1 | B1 b0 | B1 b1]; the row-major epilogue's two
  // 64-row bands and the BCE row partials reuse it after the k-loop
  constexpr int RING = 8 * EH;
  constexpr int EPIL = TE ? 2 * (2 * 64 * 256 + 64 * 4 * 32) : 0;
  __shared__ __attribute__((aligned(16))) short smem[RING > EPIL ? RING : EPIL];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const Tile t = tile_of_t<256, 256>(p, true);

  E8<AT, BT> s;
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
  constexpr bool KA = E8<AT, BT>::KA, KB = E8<AT, BT>::KB;
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
  const bool lag = __builtin_amdgcn_readfirstlane(wave) >= 4;

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
    if (lag) bar();
    for (int it = 0; it < total; it += 2) {
      s.template tile<0>(pp, t, it, total, kt1, pr1, kt2, pr2);
      kt1 = kt2; pr1 = pr2; adv(kt2, pr2);
      if (it + 1 < total) {
        s.template tile<1>(pp, t, it + 1, total, kt1, pr1, kt2, pr2);
        kt1 = kt2; pr1 = pr2; adv(kt2, pr2);
      }
    }
    if (!lag) bar();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (TE) epilogue_rm<EPI, 4, 2, 4, ENT>(p, t, s.acc, reinterpret_cast<float*>(smem), wm, wn, 0, nullptr,
                                                   reinterpret_cast<float*>(smem) + 2 * 64 * 256);
  else epilogue_g<EPI, 4, 2, 256, 4>(p, t, s.acc, reinterpret_cast<float*>(smem), wm, wn);
}

template <bool AT, bool BT, int EPI, bool TE>
hipError_t launch_e(const PParams& p, hipStream_t st) {
  const int nwg = p.g.ntm * p.g.ntn * p.g.batch * p.g.split;
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
