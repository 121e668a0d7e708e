// Eight-phase bf16-MFMA GEMM for gfx950: 256 x 256 x 64 tiles, 512 threads = 8 waves in
// 2 (M) x 4 (N), each wave 128 x 64 of v_mfma_f32_16x16x32_bf16 accumulators (fp32). Same
// operands (bf16 plane images, f32x plane pairs walked (k-tile, pair) pairs-innermost), tile
// order, epilogues and results as the ring kernel (gemm_bf16.hip). The main loop is the 256^2
// 8-phase schedule of cdna_hip_programming.md ("The 256^2 8-phase template") as its
// specification states it -- the form tools/micro/gemm8p.hip measured at 1414 TF/s on 4096^3
// (2437 cycles per k-tile) against 1135 for round 4's 32x32x16 form of this kernel (3630 cycles,
// profiles/r5/r5a_template_vs_e8.txt):
//
// * each wave's 128 x 64 block is four quadrants (m-sub, n-sub) of 64 x 32 = 4 x 2 16x16 blocks;
//   one PHASE = fragment reads + one half-tile LDS-DMA -> s_barrier -> lgkmcnt(0) -> 16 MFMAs
//   (the quadrant over K = 64) at s_setprio 1 -> s_barrier. A k-tile t is 4 phases:
//     p1 (0,0): reads B-sub 0, then A-sub 0; DMA A1(t+1); lgkmcnt retires the B-sub 0 reads
//     p2 (0,1): reads B-sub 1;                DMA B0(t+2)
//     p3 (1,1): reads A-sub 1;                DMA A0(t+2)
//     p4 (1,0): reads nothing;                DMA B1(t+2); vmcnt(6): k-tile t+1 landed
//   (vmcnt only in p4: three half-tiles = 6 DMA instructions stay in flight across barriers);
// * waves 4-7 run one barrier behind waves 0-3 (one extra s_barrier before the loop), so on
//   every SIMD -- one wave of each half -- one wave issues its reads and DMA while its partner
//   runs MFMAs; a restaged half was last read >= 2 phases earlier, or 1 phase with its reads
//   retired before that phase's first barrier (B-sub 0); data waited for in p4 is read in the
//   next p1, one barrier after the staggered half's wait (cdna_hip_programming.md, "Read a
//   staged buffer one phase AFTER the wait that retires it");
// * operand tiles travel as HALF images (128 rows x 64 k, 16 KB): half h of A = tile rows
//   128 h .. 128 h + 127, of which wave row wm reads rows 64 wm .. 64 wm + 63 (its m-sub h); half
//   h of B = tile columns 128 h .., of which wave column wn reads 32 wn .. 32 wn + 31. Two
//   buffers (even / odd k-tile) x {A0, A1, B0, B1} = 128 KB of LDS in one __shared__ array.
//
// Images (global -> LDS by global_load_lds_dwordx4; linear LDS destination, the swizzle applied
// to the per-lane SOURCE and undone on the read):
//   k-contiguous operand ([rows][K] in HBM): [8 row-blocks of 16][2 k-halves of 32] subtiles of
//     1 KB, each [16 rows][64 B] with the st_16x32 swizzle byte ^= ((byte >> 9) & 1) << 5;
//     fragments by ds_read_b128;
//   row-contiguous operand ([K][rows]): [64 k-rows][16 chunks of 8 rows], chunk c of k-row k at
//     slot c ^ tr_swz(k); a fragment is two ds_read_b64_tr_b16 (k 0-3 and 4-7 of its 8),
//     conflict-free (the 16 lanes of a group: 4 k-rows x 4 row quads; the two groups of a
//     32-lane half: k-rows 8 apart, slots XORed by 2).
#include "gemm_common.h"
#include "deint_bits.h"

#include <cstdint>

namespace mvae {
namespace {

using namespace gemm;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short lds_short;

constexpr int EBK = 64;          // k-tile
constexpr int EH = 128 * EBK;    // bf16 elements per half image (16 KB)
constexpr int EHB = 2 * EH;      // ... bytes
constexpr int ENT = 512;

// st_16x32: within a [16 rows][64 B] subtile, byte bit 5 ^= bit 9 (rows 8-15 swap 32-B halves)
__device__ __forceinline__ unsigned st_swz(unsigned b) { return b ^ (((b >> 9) & 1u) << 5); }
// chunk swizzle of a row-contiguous image's k-row k
__device__ __forceinline__ int tr_swz(int k) { return (4 * (k & 3)) ^ (2 * ((k >> 3) & 1)); }

// the source of every chunk that must read as zero (past K): 16 zero bytes in the code object
__device__ __attribute__((aligned(16))) unsigned short g_zero16[8] = {0, 0, 0, 0, 0, 0, 0, 0};

// One operand's DMA (global_load_lds_dwordx4, a per-lane 64-bit source: measured 2437 cycles per
// k-tile against 3320 with buffer_load_dwordx4 ... lds through a buffer resource on the same
// schedule, profiles/r5/r5c_*): per lane 2 chunks (instructions j = 0, 1: subtile / k-row quad
// 8 j + wave of the half) per half h, as element offsets into the plane at k0 = 0. Rows (columns)
// past the operand are clamped to its last row (8-column chunk): their outputs are not stored.
// Chunks past K read g_zero16 (both operands, so the tail products are exact zeros).
template <bool KC>
struct HLoad {
  unsigned voff[2][2];  // [j][h] element offsets (a plane of < 2^32 elements: gemm_bf16_wide)
  int kc[2];            // the chunk's k within the tile (KC: first k of its 8; else its k-row)
  __device__ __forceinline__ void init(int ld, int r0, int nrows, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int sub = j * 8 + wave;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (KC) {
          const unsigned pos = st_swz(16u * lane);  // logical byte of the subtile stored at 16 lane
          const int i = (sub >> 1) * 16 + (int)(pos >> 6);
          const int k = (sub & 1) * 32 + (int)((pos >> 4) & 3) * 8;
          int gr = r0 + 128 * h + i;
          gr = gr < nrows ? gr : nrows - 1;
          voff[j][h] = (unsigned)gr * (unsigned)ld + (unsigned)k;
          kc[j] = k;
        } else {
          const int q = sub * 64 + lane;
          const int krow = q >> 4;
          const int c = (q & 15) ^ tr_swz(krow);
          int col = r0 + 128 * h + 8 * c;
          col = col < nrows ? col : ((nrows - 1) & ~7);
          voff[j][h] = (unsigned)krow * (unsigned)ld + (unsigned)col;
          kc[j] = krow;
        }
      }
    }
  }
  // half H of the k-tile at k0 (tile k-range ends at kend) from the plane at g into img
  template <int H>
  __device__ __forceinline__ void issue(const unsigned short* g, int ld, int k0, int kend, short* img,
                                        int wave) const {
    const unsigned short* gk = g + (KC ? (size_t)k0 : (size_t)k0 * (size_t)ld);
    typedef __attribute__((address_space(3))) void* lds_ptr;
    if (k0 + EBK <= kend) {  // a whole k-tile (wave-uniform)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_global_load_lds(gk + voff[j][H], (lds_ptr)(img + (j * 8 + wave) * 512), 16, 0, 0);
    } else {
      const int kl = kend - k0;  // chunks at k >= kl read zeros
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const unsigned short* src = kc[j] < kl ? gk + voff[j][H] : g_zero16;
        __builtin_amdgcn_global_load_lds(src, (lds_ptr)(img + (j * 8 + wave) * 512), 16, 0, 0);
      }
    }
  }
};

// fragment reads at an LDS byte address + immediate offset, in inline asm: hipcc neither waits
// vmcnt(0) for the in-flight DMA (the transposing-read builtin makes it) nor lgkmcnt(0) early
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
// per-lane LDS byte offset (within a half image) of the 16x16x32 fragment whose 16 rows start at
// image row r0 (k-half 0; k-half 1 is + 1024 (KC) / + 8192 (row-contiguous))
template <bool KC>
__device__ __forceinline__ unsigned frag_addr(int r0, int lane) {
  if constexpr (KC) {
    return (unsigned)((r0 >> 4) * 2048) + st_swz((unsigned)((lane & 15) * 64 + (lane >> 4) * 16));
  } else {
    // lane 16 g + 4 q + p: k-row 8 g + q, rows r0 + 4 p .. + 3 (ds_read_b64_tr_b16 gather)
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int krow = 8 * g + q;
    const int c = ((r0 + 4 * p) >> 3) ^ tr_swz(krow);
    return (unsigned)(krow * 256 + c * 16 + 8 * (p & 1));
  }
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// ---- the bits path (BitMat A, mvae_internal.h): a k-tile's A image is its 2 KB block, copied by
// one 256-B global_load_lds_dword per wave into one of two bits buffers at LDS 0 / 2048 (the A
// half-image area is otherwise unused); each wave reads its two 64-row quarters (8 B per lane
// each) with ds_read_b64 and expands them in registers into its 8 + 8 A fragments: 1.0 / 0.0
// bf16 pairs, two VALU operations per dword (the fragments the plane path reads from LDS).
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <int OFF>
__device__ __forceinline__ u32x2 rd_b64(unsigned a) {
  u32x2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return v;
}
// fragments (2 j + h, kh) of one quarter's word j: element pair d = bits (p, p + 16) of w >> 8 h,
// p = 4 kh + d, as bf16 pair (1.0 | 0.0) = that masked word times 0x3F80 >> p (v_mul_u32_u24)
__device__ __forceinline__ bf16x8 bits_frag(unsigned s, int kh) {
  unsigned d[4];
#pragma unroll
  for (int dd = 0; dd < 4; ++dd) {
    const int p = 4 * kh + dd;
    d[dd] = (unsigned)__umul24(s & (0x10001u << p), 0x3F80u >> p);
  }
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(bf16x8, u32x4{d[0], d[1], d[2], d[3]});
}
__device__ __forceinline__ void bits_expand(u32x2 w, bf16x8 (&fa)[8]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const unsigned wj = j ? w.y : w.x;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned s = h ? wj >> 8 : wj;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) fa[2 * (2 * j + h) + kh] = bits_frag(s, kh);
    }
  }
}

// main-loop state of one workgroup (registers once inlined). ST: stamped diagnostics build --
// per wave the k-loop's shader-clock cycles and, with diag 16, each of a k-tile's 8
// barrier-delimited slots summed over the k-loop (mvae_bench_gemm with MVAE_STAMPS=2; never in
// the step). BITS: A from a BitMat, its fragments expanded in registers per wave (the plane
// path's A images, reads and DMA unused) -- 1: each k-tile's block copied into LDS by one
// 256-B LDS-DMA per wave, each wave reading its two quarters from there; 2: each wave loads its
// two quarters' words straight into registers (two 8-B `sc1` loads per lane), the form of the
// fused de-interleave's consumers (DeintJob)
template <bool AT, bool BT, bool ST = false, int BITS = 0>
struct E8 {
  static constexpr bool KA = !AT, KB = BT;  // operand images k-contiguous?
  HLoad<KA> la;
  HLoad<KB> lb;
  // accumulators [band 2 ms + (mb >> 1)][mb & 1][ns][nb]: 16x16 block mb (0..3) of m-sub ms,
  // block nb (0..1) of n-sub ns; band b = the epilogue's 64-row band b
  f32x4 acc[4][2][2][2];
  // A-sub 0 / 1 (64 rows x 64 k) and B-sub 0 / 1 (32 cols x 64 k) fragments [block * 2 + k-half]
  bf16x8 fa0[8], fa1[8], fb0[4], fb1[4];
  // fragment base addresses: k-contiguous A / B one base; row-contiguous one per 16-row block
  unsigned aA[KA ? 1 : 4], aB[KB ? 1 : 2];
  const unsigned short* A;
  const unsigned short* Bm;
  short* smem;
  int wave;
  unsigned long long st_last, st_acc[ST ? 8 : 1];
  bool st_slots;  // stamped builds, diag 16: per-slot stamps (each waits lgkmcnt(0): intrusive)
  // BITS: this tile's strip (its first k-tile's block at Ab + 512 * (ks / 64)); LDS byte address
  // of this wave's quarter-0 words in bits buffer 0 (quarter 1: + 1024, buffer 1: + 2048); the
  // current k-tile's words of quarters 0 (A-sub 0) and 1 (A-sub 1)
  const unsigned* Ab;
  unsigned bA;
  u32x2 wb0, wb1;
  // BITS 2: the words of quarters 0 / 1 (each reloaded for the next k-tile right after its
  // expansion: quarter 0 in p1, quarter 1 in p3), this lane's 8-B index in a block (quarter 0), and
  // the chunks known finished by the fused de-interleave
  u32x2 wn0, wn1;
  int wq, ready;
  // BITS: the 2 KB block of k-tile kt into bits buffer Bf, 256 B per wave
  template <int Bf>
  __device__ __forceinline__ void issue_bits(const Tile& t, int kt) {
    typedef __attribute__((address_space(3))) void* lds_ptr;
    const unsigned* src = Ab + (size_t)(t.ks / EBK + kt) * BITMAT_BLOCK_WORDS + wave * 64 + (threadIdx.x & 63);
    __builtin_amdgcn_global_load_lds(src, (lds_ptr)(reinterpret_cast<char*>(smem) + Bf * 2048 + wave * 256), 4, 0, 0);
  }
  template <int Bf>
  __device__ __forceinline__ void rd_bits() {
    wb0 = rd_b64<Bf * 2048>(bA);
    wb1 = rd_b64<Bf * 2048 + 1024>(bA);
  }
  // BITS 2: a fused launch's chunk c is finished (the workers' done[c] reached B / 64): one `sc1`
  // poll of the next 64 chunks' counters per try (lane i: chunk c + i), so one poll that finds
  // the workers ahead covers every chunk they finished
  __device__ __forceinline__ void gate(const PParams& pp, int c) {
    if (c < ready) return;
    const int lane = threadIdx.x & 63;
    const int R = pp.dj.B >> 6;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const int ci = c + lane;
      const int v = ci < pp.dj.nchunks ? __hip_atomic_load(pp.dj.done + ci, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : R;
      const unsigned long long ok = __ballot(v >= R);
      if (ok & 1ull) {
        ready = c + (~ok ? __builtin_ctzll(~ok) : 64);
        return;
      }
      // (bounded: a worker that never finished -- 0.5 s at the 100 MHz realtime clock -- raises
      // the job's error word; the launch then ends with invalid results instead of hanging)
      if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {
        if (lane == 0) atomicOr(pp.dj.err, 1);
        ready = 1 << 30;
        return;
      }
      __builtin_amdgcn_s_sleep(8);  // (~0.2 us: 1536 pollers stay off the counters' L2 lines)
    }
  }
  // BITS 2: k-tile kt's words of this wave's quarter Q into wn0 / wn1 by an 8-B `sc1` load in
  // inline asm (invisible to hipcc's waitcnt pass, which otherwise drains every load at once: the
  // p4 / p3 waits below retire it); a fused launch first waits until the chunk is finished
  template <int Q>
  __device__ __forceinline__ void load_bits(const PParams& pp, const Tile& t, int kt) {
    const int gk = t.ks / EBK + kt;
    if (Q == 0 && pp.dj.nworkers && !(pp.dj.diag & 1)) gate(pp, gk / DEINT_FUSE_PB);
    const unsigned* q = Ab + (size_t)gk * BITMAT_BLOCK_WORDS + 2 * wq + 256 * Q;
    if constexpr (Q == 0) asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(wn0) : "v"(q) : "memory");
    else asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(wn1) : "v"(q) : "memory");
  }

  template <int K>
  __device__ __forceinline__ void sbar() {
    bar();
    if constexpr (ST) {
      if (!st_slots) return;
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
    if constexpr (KA) {  // block mb, k-half kh: subtile 2 mb + kh of the wave row's 8
      fa[0] = rd_b128<O>(aA[0]);
      fa[1] = rd_b128<O + 1024>(aA[0]);
      fa[2] = rd_b128<O + 2048>(aA[0]);
      fa[3] = rd_b128<O + 3072>(aA[0]);
      fa[4] = rd_b128<O + 4096>(aA[0]);
      fa[5] = rd_b128<O + 5120>(aA[0]);
      fa[6] = rd_b128<O + 6144>(aA[0]);
      fa[7] = rd_b128<O + 7168>(aA[0]);
    } else {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        fa[2 * mb] = rd_tr<O>(aA[mb]);
        fa[2 * mb + 1] = rd_tr<O + 8192>(aA[mb]);
      }
    }
  }
  template <int H, int Bf>
  __device__ __forceinline__ void rd_b(bf16x8 (&fb)[4]) {
    constexpr int O = (2 * H + Bf) * EHB;
    if constexpr (KB) {
      fb[0] = rd_b128<O>(aB[0]);
      fb[1] = rd_b128<O + 1024>(aB[0]);
      fb[2] = rd_b128<O + 2048>(aB[0]);
      fb[3] = rd_b128<O + 3072>(aB[0]);
    } else {
      fb[0] = rd_tr<O>(aB[0]);
      fb[1] = rd_tr<O + 8192>(aB[0]);
      fb[2] = rd_tr<O>(aB[1]);
      fb[3] = rd_tr<O + 8192>(aB[1]);
    }
  }
  // the quadrant's 16 MFMAs once this wave's reads have landed (priority 1 around them unless
  // flips is false: PParams::prio)
  bool flips = true;
  template <int MS, int NS>
  __device__ __forceinline__ void mfma_q(const bf16x8 (&fa)[8], const bf16x8 (&fb)[4]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (flips) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[2 * MS + (mb >> 1)][mb & 1][NS][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              fa[2 * mb + kh], fb[2 * nb + kh], acc[2 * MS + (mb >> 1)][mb & 1][NS][nb], 0, 0, 0);
    if (flips) __builtin_amdgcn_s_setprio(0);
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
  // k-tile `it` (its images in buffer Bf); (kt1, pr1), (kt2, pr2): (k-tile, pair) of it+1, it+2;
  // ka1: it+1's A image is the one its buffer holds (from it-1: not copied again), ka2 / kb2: it+2's
  // A / B images likewise (from it)
  // BITS: ka1 = it+1 has this iteration's k-tile (no block copy), ex = this iteration's k-tile differs
  // from it-1's (expand; else the fragments in fa0 / fa1 are still this k-tile's)
  template <int Bf>
  __device__ __forceinline__ void tile(const PParams& pp, const Tile& t, int it, int total, int kt1, int pr1,
                                       int kt2, int pr2, bool ka1, bool ka2, bool kb2, bool ex = true) {
    constexpr int Bn = Bf ^ 1;
    // stamped builds' A/B switches (results meaningless): diag 1 = no DMA after the prologue,
    // 64 = no fragment reads
    const bool dma = !ST || !(pp.diag & 1), rdf = !ST || !(pp.diag & 64);
    const bool h1 = it + 1 < total && dma, h2 = it + 2 < total && dma;
    const bool ia2 = h2 && !ka2, ib2 = h2 && !kb2;
    // p1 (0,0)
    if (rdf) rd_b<0, Bf>(fb0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (BITS == 2) {
      // quarter 0 of this k-tile (landed by the last p4's wait) expanded, then it+1's quarter 0
      // loaded into the same registers; the B-sub 0 reads retired (B0 is restaged in p2)
      if (ex) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" : "+v"(wn0));
        bits_expand(wn0, fa0);
      }
      if (h1 && !ka1) load_bits<0>(pp, t, kt1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if constexpr (BITS == 1) {
      // both quarters' words (the buffer is next restaged in tile it+1's p1); the whole block of
      // it+1 into the other buffer, whose last reads were tile it-1's p1; quarter 0 expanded once
      // every read retired (B-sub 0's as well: B0 is restaged in p2)
      if (ex) rd_bits<Bf>();
      if (h1 && !ka1) issue_bits<Bn>(t, kt1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (ex) {
        asm volatile("" : "+v"(wb0), "+v"(wb1));
        __builtin_amdgcn_sched_barrier(0);
        bits_expand(wb0, fa0);
      }
    } else {
      if (rdf) rd_a<0, Bf>(fa0);
      if (h1 && !ka1) issue_a<1, Bn>(pp, t, kt1, pr1);
      // the B-sub 0 reads (issued first) retired: B0 is restaged in p2
      // (the A-sub 0 reads: 8 ds_read_b128, or 16 transposing reads -- the count saturates at 15)
      if constexpr (KA) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
    }
    sbar<0>();
    mfma_q<0, 0>(fa0, fb0);
    sbar<1>();
    // p2 (0,1)
    if (rdf) rd_b<1, Bf>(fb1);
    if (ib2) issue_b<0, Bf>(pp, t, kt2, pr2);
    sbar<2>();
    mfma_q<0, 1>(fa0, fb1);
    sbar<3>();
    // p3 (1,1)
    if constexpr (BITS == 2) {
      // quarter 1 (loaded in the last p3: what is younger may stay in flight except this tile's
      // B0 halves), then it+1's
      if (ex) {
        if (ib2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" : "+v"(wn1));
        bits_expand(wn1, fa1);
      }
      if (h1 && !ka1) load_bits<1>(pp, t, kt1);
    } else if constexpr (BITS == 1) {
      if (ex) bits_expand(wb1, fa1);
    } else {
      if (rdf) rd_a<1, Bf>(fa1);
      if (ia2) issue_a<0, Bf>(pp, t, kt2, pr2);
    }
    sbar<4>();
    mfma_q<1, 1>(fa1, fb1);
    sbar<5>();
    // p4 (1,0): k-tile it+1 landed -- what stays in flight is the halves of it+2 issued in this
    // tile (2 DMA instructions each; the bits path's block of it+1 went out in p1, before them)
    if (ib2) issue_b<1, Bf>(pp, t, kt2, pr2);
    if constexpr (BITS) {
      if (ib2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ib2 && ia2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (ib2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (ia2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sbar<6>();
    mfma_q<1, 0>(fa1, fb0);
    sbar<7>();
  }
};

// One workgroup's tile: the k-loop and the epilogue. BITS: A from the BitMat pp.abits (its AT
// is then immaterial: the bits path has one A layout)
template <bool AT, bool BT, int EPI, bool TE, bool ST, int BITS>
__device__ __forceinline__ void e8_tile(const PParams& pp, short* smem) {
  const Params& p = pp.g;
  unsigned long long st_k0 = 0, st_k2 = 0;  // stamped builds: kernel start, k-loop end (realtime)
  if constexpr (ST) st_k0 = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const Tile t = tile_of_t<256, 256>(p, true, pp.dj.nworkers);

  using S = E8<AT, BT, ST, BITS>;
  S s;
  s.A = pp.A + t.bi * p.sA;
  s.Bm = pp.B + t.bi * p.sB;
  s.smem = smem;
  s.wave = __builtin_amdgcn_readfirstlane(wave);
  if constexpr (ST) s.st_slots = (pp.diag & 16) != 0;
  if constexpr (BITS) {
    s.Ab = pp.abits + (size_t)t.bi * pp.abits_sb + (size_t)(t.m0 / 256) * pp.abits_kts * BITMAT_BLOCK_WORDS;
  } else {
    s.la.init(p.lda, t.m0, p.M, wave, lane);
  }
  s.lb.init(p.ldb, t.n0, p.N, wave, lane);
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int k = 0; k < 2; ++k) s.acc[b][i][j][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_short*)smem;
  if constexpr (BITS == 1) {
    s.bA = lds0 + (unsigned)(wm * 512 + lane * 8);  // quarter (0, wm): rows 64 wm .. of half 0
  } else if constexpr (BITS == 2) {
    s.wq = wm * 64 + lane;  // (quarter (0, wm): words 128 wm + 2 lane, + 1; quarter 1: + 256)
    s.ready = 0;
  } else if constexpr (S::KA) {
    s.aA[0] = lds0 + frag_addr<true>(64 * wm, lane);
  } else {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) s.aA[mb] = lds0 + frag_addr<false>(64 * wm + 16 * mb, lane);
  }
  if constexpr (S::KB) {
    s.aB[0] = lds0 + 4 * EHB + frag_addr<true>(32 * wn, lane);
  } else {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) s.aB[nb] = lds0 + 4 * EHB + frag_addr<false>(32 * wn + 16 * nb, lane);
  }

  // (bits: A is exact, its residual planes zero -- the pairs with A plane 0)
  const int np = BITS != 0 ? pp.npairs_a0 : (pp.dyn && *pp.dyn == 0) ? pp.npairs0 : pp.npairs;
  const int nkt = t.ks < t.ke ? (t.ke - t.ks + EBK - 1) / EBK : 0;
  const int total = np * nkt;
  // waves 4-7 (the second wave of every SIMD), as a scalar condition: s_barrier ignores EXEC
  // (stamped builds, diag 128: no stagger -- both halves in the same phase)
  const bool lag = __builtin_amdgcn_readfirstlane(wave) >= 4 && !(ST && (pp.diag & 128));
  // priority (PParams::prio): 0 priority 1 around every MFMA quadrant; 1 priority 1 for the
  // lagging half (waves 4-7) for the whole loop, no flips (cdna_hip_programming.md T5, static
  // form); 2 no priorities
  s.flips = pp.prio == 0;
  if (pp.prio == 1 && lag) __builtin_amdgcn_s_setprio(1);

  if (total > 0) {
    // The (k-tile, pair) walk. Default: pairs innermost. reuse (f32x plane pairs): k-tiles in
    // twos, pairs between -- (k0,p0) (k1,p0) (k0,p1) (k1,p1) ... -- so an iteration and the one
    // two before it (the same LDS buffer) share the k-tile, and an operand plane they share is
    // not copied again (binary pixels, 3 pairs: 2 of 6 A images copied; 6 pairs: 16 of 24
    // images). Cursor = (group g of two k-tiles, index r within it).
    struct Cur { int g, r, kt, pr; };
    // (the bits path walks pairs innermost: the pairs of a k-tile reuse its expanded fragments)
    const bool rw = pp.reuse != 0 && BITS == 0;
    auto set = [&](Cur& c) {
      if (!rw) { c.kt = c.g; c.pr = c.r; return; }
      if (2 * c.g + 1 < nkt) { c.kt = 2 * c.g + (c.r & 1); c.pr = c.r >> 1; }
      else { c.kt = 2 * c.g; c.pr = c.r; }
    };
    auto adv = [&](Cur& c) {
      const int span = !rw ? np : (2 * c.g + 1 < nkt ? 2 * np : np);
      if (++c.r == span) { c.r = 0; ++c.g; }
      set(c);
    };
    auto pa_of = [&](int pr) { return (pp.pab >> (4 * pr)) & 3; };
    auto pb_of = [&](int pr) { return (pp.pab >> (4 * pr + 2)) & 3; };
    // cursors of iterations it-1 .. it+2
    Cur cm{0, 0, 0, 0}, c0{0, 0, 0, 0}, c1{0, 0, 0, 0}, c2{0, 0, 0, 0};
    set(c0);
    c1 = c0; adv(c1);
    c2 = c1; adv(c2);
    // iteration j's image (A or B) is already in its buffer: iteration j-2 had the same k-tile
    // and plane (it+1's A: from it-1 -- cm; it+2's: from it -- c0)
    auto ka = [&](const Cur& a, const Cur& b, int j) { return rw && j >= 2 && a.kt == b.kt && pa_of(a.pr) == pa_of(b.pr); };
    auto kb = [&](const Cur& a, const Cur& b, int j) { return rw && j >= 2 && a.kt == b.kt && pb_of(a.pr) == pb_of(b.pr); };
    // prologue: A0 B0 B1 A1 of k-tile 0, then B0 A0 B1 of k-tile 1 (its A1: tile 0's p1); the bits
    // path: k-tile 0's block, B0 B1, then k-tile 1's B0 B1 (its block: tile 0's p1)
    int kt1 = c1.kt, pr1 = c1.pr, kt2 = c2.kt, pr2 = c2.pr;
    if constexpr (BITS != 0) {
      if constexpr (BITS == 2) {
        s.template load_bits<0>(pp, t, 0);
        s.template load_bits<1>(pp, t, 0);
      } else {
        s.template issue_bits<0>(t, 0);
      }
      s.template issue_b<0, 0>(pp, t, 0, 0);
      s.template issue_b<1, 0>(pp, t, 0, 0);
      if (total > 1) {
        s.template issue_b<0, 1>(pp, t, kt1, pr1);
        s.template issue_b<1, 1>(pp, t, kt1, pr1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      s.template issue_a<0, 0>(pp, t, 0, 0);
      s.template issue_b<0, 0>(pp, t, 0, 0);
      s.template issue_b<1, 0>(pp, t, 0, 0);
      s.template issue_a<1, 0>(pp, t, 0, 0);
      if (total > 1) {
        s.template issue_b<0, 1>(pp, t, kt1, pr1);
        s.template issue_a<0, 1>(pp, t, kt1, pr1);
        s.template issue_b<1, 1>(pp, t, kt1, pr1);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    bar();
    if (lag) bar();
    unsigned long long st_t0 = 0, st_r0 = 0;
    if constexpr (ST) {
#pragma unroll
      for (int k = 0; k < 8; ++k) s.st_acc[k] = 0;
      st_r0 = __builtin_amdgcn_s_memrealtime();
      st_t0 = s.st_last = __builtin_amdgcn_s_memtime();
    }
    auto step = [&]() { cm = c0; c0 = c1; c1 = c2; adv(c2); };
    // the bits path: it+1's block is copied only for a new k-tile, and an iteration expands only
    // when its k-tile is not it-1's
    auto ka1_of = [&](int j) { return BITS != 0 ? c1.kt == c0.kt : ka(c1, cm, j); };
    auto ex_of = [&](int j) { return BITS == 0 || j == 0 || c0.kt != cm.kt; };
    for (int it = 0; it < total; it += 2) {
      s.template tile<0>(pp, t, it, total, c1.kt, c1.pr, c2.kt, c2.pr, ka1_of(it + 1), ka(c2, c0, it + 2),
                         kb(c2, c0, it + 2), ex_of(it));
      step();
      if (it + 1 < total) {
        s.template tile<1>(pp, t, it + 1, total, c1.kt, c1.pr, c2.kt, c2.pr, ka1_of(it + 2),
                           ka(c2, c0, it + 3), kb(c2, c0, it + 3), ex_of(it + 1));
        step();
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
  // Band mi = accumulator band mi: tile rows 128 (mi >> 1) + 64 wm + 32 (mi & 1) + 0..31 of both
  // wave rows (RMAP 1); the 16x16 C/D layout: col = lane & 15, row = 4 (lane >> 4) + j. The band's
  // blocks are always acc[0] (rotated down after each band: the band loop is not unrolled).
  float* const lds_f = reinterpret_cast<float*>(smem);
  {
    auto wb = [&](float* band, int) {
#pragma unroll
      for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
        for (int ns = 0; ns < 2; ++ns)
#pragma unroll
          for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              band[(wm * 32 + m2 * 16 + 4 * (lane >> 4) + j) * 256 + ns * 128 + wn * 32 + nb * 16 + (lane & 15)] =
                  s.acc[0][m2][ns][nb][j];
#pragma unroll
      for (int b = 0; b + 1 < 4; ++b)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int k = 0; k < 2; ++k) s.acc[b][i][j][k] = s.acc[b + 1][i][j][k];
    };
    epilogue_rm_w<EPI, 4, 256, ENT, decltype(wb)&, 1>(p, t, wb, lds_f, 0, nullptr, lds_f + 2 * 64 * 256, TE);
  }
  if constexpr (ST) {  // epilogue: from the k-loop's end until every store of the workgroup issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane == 0 && st_k2) pp.stamps[16 * ((size_t)blockIdx.x * 8 + wave) + 12] = __builtin_amdgcn_s_memrealtime() - st_k2;
  }
}

// the bits path is compiled where the step runs it: the layer-0 forward (ACT, or split-K slabs)
// and weight gradient (slabs or output), B row-contiguous
template <bool BT, int EPI, bool ST>
constexpr bool has_bits = !BT && !ST && (EPI == EPI_STORE || EPI == EPI_ACT);

// The fused de-interleave's workers (DeintJob). A worker workgroup takes tasks T = w, w + W, ...
// (task T: chunk order[T / R] of 256 pixels, batch rows 64 (T % R) ..), each in 4 passes of 16
// rows. Each pass's 16 rows x 3 KB of X (the row chunk's interleaved pixels) go HBM -> LDS by 48
// LDS-DMA instructions of 1 KB each (6 per wave) -- whole contiguous KBs: a thread's own 96-B
// pieces at a 96-B lane stride, the standalone kernel's loads, touch 6x the L1 lines they use and
// held a CU to ~25 GB/s -- into a ring of 3 pass buffers, two passes in flight. Per pass each
// thread reads one row octet (96 B) from LDS and writes its block bytes (deint_octet) into the
// task's byte image -- no global store in a pass: the next pass's DMA wait would wait for it too
// (vmcnt retires in order). At a task's first pass the previous task's words (deint_words;
// forward words written through) and target bytes are stored, and counted in done[chunk] one pass
// later, once every wave's vmcnt wait has retired them and the pass barrier has passed.
// Measured at C3 (r6t-r6y): the workers alone 0.69 ms on their 64 CUs (the DMA alone 0.34 ms;
// dedicated loader waves beside 4 transposing waves 0.88), so the fused launch (0.78 ms) loses
// to the separate de-interleave + forward (0.50 ms): the transpose's VALU and LDS work per byte
// needs more CUs than the forward's tiles leave free. Option deint_fuse stays off.
constexpr int DW_ROWB = 64 * DEINT_FUSE_PB * 12;   // bytes of one row's 256-pixel chunk (3 KB)
constexpr int DW_PASSB = 16 * DW_ROWB;              // one pass: 16 rows (48 KB)
constexpr int DW_BT = 3 * 8 * DEINT_FUSE_PB * 72;   // one task's byte image (DeintLds)
constexpr int DW_ORDER = 3 * DW_PASSB + 2 * DW_BT;  // LDS byte offset of the order table
constexpr int DW_LDS = 163840;                      // the workgroup's LDS (160 KB)
constexpr int DW_MAXCH = (DW_LDS - DW_ORDER) / 4;   // chunks the order table can hold
static_assert(DW_ORDER + 4 * 64 <= DW_LDS, "LDS");
__device__ __forceinline__ void deint_worker(const DeintJob& dj, short* smem) {
  constexpr int PB = DEINT_FUSE_PB, OS = 72;
  using Lds = DeintLds<PB, OS>;
  char* lds = reinterpret_cast<char*>(smem);
  int* ord = reinterpret_cast<int*>(lds + DW_ORDER);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int R = dj.B >> 6;
  const int W = dj.nworkers;
  const int ntask = dj.nchunks * R;
  const int D = dj.D;
  if (blockIdx.x == 0 && tid == 0 && dj.dyn_next) {
    dj.dyn_next[0] = 0;
    dj.dyn_next[2] = 0;
  }
  for (int i = tid; i < dj.nchunks; i += ENT) ord[i] = dj.order ? dj.order[i] : i;
  __syncthreads();
  if ((int)blockIdx.x >= ntask) return;
  const int ntw = (ntask - 1 - (int)blockIdx.x) / W + 1;  // this worker's tasks
  const int P = 4 * ntw;                                   // ... and passes
  auto task_of = [&](int k) { return (int)blockIdx.x + k * W; };
  typedef __attribute__((address_space(3))) void* lds_ptr;
  // pass p's 48 KB into ring buffer p % 3: this wave's instructions jj = wave + 8 m (row jj / 3,
  // KB jj % 3 of it)
  auto issue = [&](int p) {
    if (dj.diag & 16) return;
    const int T = task_of(p >> 2);
    const int c = ord[T / R];
    const size_t row0 = (size_t)(64 * (T % R) + 16 * (p & 3));
    const int f0 = 3 * 256 * c;  // first float of the row chunk
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      const int jj = wave + 8 * m, rr = jj / 3, part = jj % 3;
      int f = f0 + part * 256 + 4 * lane;
      f = f + 4 <= 3 * D ? f : 3 * D - 4;  // (past the row: its last 16 B, unused)
      const float* src = dj.x + (row0 + rr) * 3 * (size_t)D + f;
      __builtin_amdgcn_global_load_lds(src, (lds_ptr)(lds + (p % 3) * DW_PASSB + jj * 1024), 16, 0, 0);
    }
  };
  issue(0);
  if (P > 1) issue(1);
  // the BCE target bytes of task t (block 1 of its byte image) to xbits, four per thread: no
  // store in the pass loop, whose next DMA wait would also wait for the store (vmcnt is in order)
  auto target_bytes = [&](int t, const Lds& bt) {
    const int c = ord[t / R], r = tid >> 3, o0 = 4 * (tid & 7);
    const int q0 = 32 * c + o0, nq = D >> 3;  // first octet of the row chunk, octets per row
    unsigned char* dst = dj.xbits + (size_t)(64 * (t % R) + r) * dj.ldbits + q0;
    if (q0 + 4 <= nq) {
      *reinterpret_cast<unsigned*>(dst) = (unsigned)bt[1][o0][r] | (unsigned)bt[1][o0 + 1][r] << 8 |
                                          (unsigned)bt[1][o0 + 2][r] << 16 | (unsigned)bt[1][o0 + 3][r] << 24;
    } else {
      for (int j = 0; j < 4 && q0 + j < nq; ++j) dst[j] = bt[1][o0 + j][r];
    }
  };
  bool nb = false;
  int pend = -1;  // chunk of the task whose words were stored in the last pass
  for (int p = 0; p < P; ++p) {
    const int k = p >> 2, q = p & 3;
    // pass p landed; what is younger: pass p+1's DMA, issued at the end of pass p-1 (the stores
    // of pass p-1, issued before it, retire here too)
    if (p + 1 < P) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (a bare barrier: __syncthreads' release fence would wait for the DMA in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    // (the words stored at the last pass are older than pass p+1's DMA: retired by this pass's
    // wait in every wave)
    if (pend >= 0) {
      if (tid == 0 && dj.done) __hip_atomic_fetch_add(dj.done + pend, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pend = -1;
    }
    const int T = task_of(k);
    const int c = ord[T / R], by = T % R;
    if (q == 0 && k > 0 && !(dj.diag & 8)) {  // the last task's words from its byte image
      const int Tp = task_of(k - 1);
      const int cp = ord[Tp / R];
      const Lds& btp = *reinterpret_cast<const Lds*>(lds + 3 * DW_PASSB + ((k - 1) & 1) * DW_BT);
      deint_words<PB, OS, true>(tid, ENT, dj.B, D, dj.kts_f, dj.kts_w, dj.xbf, dj.xbw, cp, Tp % R, btp);
      target_bytes(Tp, btp);
      pend = cp;
    }
    if (!(dj.diag & 8)) {
      Lds& bt = *reinterpret_cast<Lds*>(lds + 3 * DW_PASSB + (k & 1) * DW_BT);
      const char* raw = lds + (p % 3) * DW_PASSB;
      const int rr = tid >> 5, o = tid & 31;
      const int pix = 256 * c + 8 * o, r = 16 * q + rr;
      unsigned by3[3];
      const unsigned pad = (pix <= D && D < pix + 8) ? 1u << (D - pix) : 0u;
      by3[0] = by3[1] = by3[2] = pad;
      if (pix + 8 <= D) {
        const float4* src = reinterpret_cast<const float4*>(raw + rr * DW_ROWB + o * 96);
        float e[24];
#pragma unroll
        for (int t = 0; t < 6; ++t) {
          const float4 v = src[t];
          e[4 * t] = v.x; e[4 * t + 1] = v.y; e[4 * t + 2] = v.z; e[4 * t + 3] = v.w;
        }
        nb |= deint_octet(e, by3);
      }
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) bt[cc][o][r] = (unsigned char)by3[cc];
    }
    // into the buffer pass p - 1 was read from (free since the barrier), after this pass's stores
    // (issued at the pass's start, the DMA measured slower: 0.77 vs 0.69 ms of workers at C3)
    if (p + 2 < P) issue(p + 2);
  }
  // the last task: its words once every wave's bytes are in (the barrier), then its count
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
  const int Tl = task_of(ntw - 1);
  const int cl = ord[Tl / R];
  if (!(dj.diag & 8)) {
    const Lds& btl = *reinterpret_cast<const Lds*>(lds + 3 * DW_PASSB + ((ntw - 1) & 1) * DW_BT);
    deint_words<PB, OS, true>(tid, ENT, dj.B, D, dj.kts_f, dj.kts_w, dj.xbf, dj.xbw, cl, Tl % R, btl);
    target_bytes(Tl, btl);
  }
  if (dj.dyn && __ballot(nb) != 0 && lane == 0) atomicOr(dj.dyn + 2, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && dj.done) {
    if (pend >= 0) __hip_atomic_fetch_add(dj.done + pend, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(dj.done + cl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the workers alone, one per CU (diagnostics: mvae_bench_deint variant 5; order null = identity)
__global__ __launch_bounds__(ENT, 1) void deint_persist_kernel(DeintJob dj) {
  __shared__ __attribute__((aligned(1024))) short smem[DW_LDS / 2];
  deint_worker(dj, smem);
}

template <bool AT, bool BT, int EPI, bool TE, bool ST = false>
__global__ __launch_bounds__(ENT, 1) void gemm_bf16e_kernel(PParams pp) {
  if (epi_skip<EPI>(pp.g.epi)) return;
  if (pp.g.epi.only_if && *pp.g.epi.only_if == 0) return;
  // [A0 b0 | A0 b1 | A1 b0 | A1 b1 | B0 b0 | B0 b1 | B1 b0 | B1 b1]; the row-major epilogue's two
  // 64-row bands and the BCE row partials reuse it after the k-loop (one __shared__ array: a
  // second one can make hipcc wait vmcnt(0) before the loop's LDS reads)
  constexpr int RING = 8 * EH;
  constexpr int EPIL = 2 * (2 * 64 * 256 + 64 * 4 * 32);
  // (the bits-path instantiations also carry the fused de-interleave's workers: the whole 160 KB)
  constexpr int SM0 = RING > EPIL ? RING : EPIL;
  constexpr int SM = has_bits<BT, EPI, ST> && DW_LDS / 2 > SM0 ? DW_LDS / 2 : SM0;
  __shared__ __attribute__((aligned(1024))) short smem[SM];
  // a 0/1 batch (the de-interleave's not-binary word, a uniform branch): A from its bits
  if constexpr (has_bits<BT, EPI, ST>) {
    if (pp.dj.nworkers) {  // the fused de-interleave: workers first, then the GEMM's tiles
      if ((int)blockIdx.x < pp.dj.nworkers) {
        if (!(pp.dj.diag & 4)) deint_worker(pp.dj, smem);
        return;
      }
      if (pp.dj.diag & 2) return;
      e8_tile<false, BT, EPI, TE, ST, 2>(pp, smem);
      return;
    }
    if (pp.abits && (!pp.anb || *pp.anb == 0)) {
      if (pp.bits_reg) e8_tile<false, BT, EPI, TE, ST, 2>(pp, smem);
      else e8_tile<false, BT, EPI, TE, ST, 1>(pp, smem);
      return;
    }
  }
  e8_tile<AT, BT, EPI, TE, ST, 0>(pp, smem);
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
  if (p.dj.nworkers && (!has_bits<BT, EPI, false> || AT || !p.abits || (p.dj.nworkers & 7))) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_bf16e_kernel<AT, BT, EPI, TE>), dim3(nwg + p.dj.nworkers), dim3(ENT), 0, st, p);
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

hipError_t launch_deint_persist(const DeintJob& j, hipStream_t st) {
  if (j.nworkers <= 0 || j.nchunks > DW_MAXCH || (j.B % 64) || (j.D % 8)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(deint_persist_kernel, dim3(j.nworkers), dim3(ENT), 0, st, j);
  return hipGetLastError();
}

namespace {

// (tests / diagnostics) one BitMat word per thread from a bf16 plane of 0/1 values
__global__ void bits_from_plane_kernel(const unsigned short* __restrict__ plane, int ld, int trans, int M,
                                       int K, unsigned* __restrict__ out, int kts, size_t nwords,
                                       int* __restrict__ nb) {
  const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  const size_t blk = w / BITMAT_BLOCK_WORDS;
  const int r = (int)(w % BITMAT_BLOCK_WORDS);
  const int mt = (int)(blk / kts), kt = (int)(blk % kts);
  const int j = r & 1, lane = (r >> 1) & 63, q = r >> 7;  // q = 2 s + wm
  unsigned word = 0;
  bool bad = false;
  for (int b = 0; b < 32; ++b) {
    const int h = (b >> 3) & 1, kh = (b >> 2) & 1, el = ((b & 3) << 1) | (b >> 4);
    const int row = mt * 256 + 64 * q + 16 * (2 * j + h) + (lane & 15);
    const int k = kt * 64 + 32 * kh + 8 * (lane >> 4) + el;
    if (row >= M || k >= K) continue;
    const unsigned short v = trans ? plane[(size_t)k * ld + row] : plane[(size_t)row * ld + k];
    if (v == 0x3F80u) word |= 1u << b;
    else if (v != 0) bad = true;
  }
  out[w] = word;
  if (bad && nb) atomicOr(nb, 1);
}

}  // namespace

hipError_t launch_bits_from_plane(const unsigned short* plane, int ld, bool trans, int M, int K,
                                  unsigned* out, int kts, int* nb, hipStream_t st) {
  if (M <= 0 || K <= 0 || kts < bitmat_kts(K)) return hipErrorInvalidValue;
  const size_t n = (size_t)((M + 255) / 256) * kts * BITMAT_BLOCK_WORDS;
  hipLaunchKernelGGL(bits_from_plane_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, plane, ld,
                     trans ? 1 : 0, M, K, out, kts, n, nb);
  return hipGetLastError();
}

// the eight-phase kernel for a planned 256 x 256 tile (PParams::g.tn == TN_E8): te = the row-major
// LDS epilogue with 16-B global accesses, else element-wise
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
