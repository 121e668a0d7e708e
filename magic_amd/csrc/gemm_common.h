// Shared pieces of the GEMM kernel families (fp32 MFMA and bf16 MFMA): launch parameters,
// activation math with TF semantics, the XCD-grouped tile order and the fused epilogues.
// Both families use 128x128 workgroup tiles, 4 waves in 2x2, each wave 2x2 MFMA 32x32
// accumulators, so the accumulator -> (row, col) map and the epilogue are identical.
#pragma once
#include "mvae_internal.h"

namespace mvae {
namespace gemm {

constexpr int BM = 128, BN = 128, NT = 256;

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Params {
  int M, N, K;
  const float* A; int lda;
  const float* B; int ldb;
  float* C; int ldc;
  long long sA, sB, sC;     // batch strides
  int batch, split, kchunk;
  int ntm, ntn;
  int tn;                   // bf16 DMA kernels: ring-kernel tile N (256 or 128) or TN_E8
  int tm = 256;             // ... and ring-kernel tile M (256, or 192 for a k-contiguous A)
  int group = 0;            // tile order: 0 = row by row (n fastest); G > 0 = bands of G m-tiles
                            // walked n by n, so an XCD's resident tiles share A and B in its L2
  GemmEpi epi;
};
constexpr int TN_E8 = GEMM_TN_E8;  // Params::tn of the 256 x 256 eight-phase kernel (gemm_bf16e.hip)

// launch parameters of the bf16-plane kernels (gemm_bf16.hip, gemm_bf16e.hip)
struct PParams {
  Params g;                         // shapes, fp32 output, batch/split/tiles, epilogue
  const unsigned short* A; long long pA;
  const unsigned short* B; long long pB;
  int npairs, npairs0;
  unsigned char pa[6], pb[6];
  int pab;                          // pa[i] | pb[i] << 2 packed 4 bits per pair (no memory reads)
  const int* dyn;                   // A residual planes nonzero? (nullptr: use all pairs)
  int diag;                         // timing diagnostics: bit 0 = no operand copies after the
                                    // prologue (the k-loop multiplies stale LDS images)
  int reuse;                        // eight-phase kernel: (k-tile, pair) iterations in pairs of
                                    // k-tiles, pairs between, and an operand image not copied
                                    // again when its buffer already holds it (gemm_bf16e.hip)
  unsigned long long* stamps;       // stamped diagnostics builds (ST): 8 slots per workgroup
                                    // {start, prologue landed, k-loop done, end, stores issued}
  // eight-phase kernel: A as a BitMat (mvae_internal.h) instead of its planes while *anb == 0 --
  // strips of kts blocks per 256 rows, batch stride sb words (GemmDesc::Abits)
  const unsigned* abits = nullptr;
  int abits_kts = 0;
  long long abits_sb = 0;
  const int* anb = nullptr;
  int npairs_a0 = 1;                // the leading pairs with A plane 0 (the bits path's pairs)
  DeintJob dj;                      // eight-phase kernel: the fused de-interleave (GemmDesc::dj)
  int bits_reg = 0;                 // eight-phase bits path: A words by loads to registers (E8 BITS 2)
  int prio = 0;                     // eight-phase kernel: s_setprio form (gemm_bf16e.hip e8_tile)
  int x3 = 0;                       // f32x ring plans at tile N 128: the plane-stacked kernel (GemmDesc::x3)
};

// tanh as an odd [13/6] rational in x on [-7.905, 7.905] (clamped beyond, where tanh rounds to
// +-1): one v_rcp_f32 and FMAs that pair into packed v_pk_fma_f32, relative error < 6e-7
// everywhere (numpy check against float64 tanh on a 2M-point grid, tools/micro/README). The
// previous exp/reciprocal form (two transcendentals plus a Taylor branch near 0) kept the
// hidden-layer epilogues VALU-bound: the quarter-rate transcendentals dominate their math.
__device__ __forceinline__ float tanh_fast(float x) {
  const float c = __builtin_amdgcn_fmed3f(x, -7.90531110763549805f, 7.90531110763549805f);
  const float x2 = c * c;
  float p = fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(x2, p, -8.60467152213735e-11f);
  p = fmaf(x2, p, 5.12229709037114e-08f);
  p = fmaf(x2, p, 1.48572235717979e-05f);
  p = fmaf(x2, p, 6.37261928875436e-04f);
  p = fmaf(x2, p, 4.89352455891786e-03f);
  float q = fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(x2, q, 2.26843463243900e-03f);
  q = fmaf(x2, q, 4.89352518554385e-03f);
  float r = (p * c) * __builtin_amdgcn_rcpf(q);
  asm("" : "+v"(r));  // pinned: the NaN select below stays a v_cndmask, not a branch
  return x != x ? x : r;  // NaN propagates (the clamp would map it to +-1)
}
__device__ __forceinline__ float elu_fast(float v) { return v < 0.f ? __expf(v) - 1.f : v; }
__device__ __forceinline__ float act_f(float v, int act) {
  if (act == ACT_TANH) return tanh_fast(v);
  return elu_fast(v);  // TF elu: exp(x) - 1 for x < 0
}
// the activation (derivative) of n values, the act switch hoisted out of the element loop
template <int n>
__device__ __forceinline__ void act_n(float (&v)[n], int act) {
  if (act == ACT_TANH) {
#pragma unroll
    for (int j = 0; j < n; ++j) v[j] = tanh_fast(v[j]);
  } else {
#pragma unroll
    for (int j = 0; j < n; ++j) v[j] = elu_fast(v[j]);
  }
}
template <int n>
__device__ __forceinline__ void dact_n(float (&v)[n], const float (&y)[n], int act) {
  if (act == ACT_TANH) {
#pragma unroll
    for (int j = 0; j < n; ++j) v[j] = v[j] * (1.f - y[j] * y[j]);
  } else {
#pragma unroll
    for (int j = 0; j < n; ++j) v[j] = y[j] < 0.f ? v[j] * (y[j] + 1.f) : v[j];
  }
}
__device__ __forceinline__ float dact_f(float g, float y, int act) {
  if (act == ACT_TANH) return g * (1.f - y * y);  // TF TanhGrad
  return y < 0.f ? g * (y + 1.f) : g;              // TF EluGrad (on the output)
}
__device__ __forceinline__ float sigmoid_f(float v) { return 1.f / (1.f + expf(-v)); }
// hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1e-7 relative): the BCE
// epilogue evaluates them for every decoder output element (D x B per step)
__device__ __forceinline__ float sigmoid_fast(float v) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-v));
}

// the dgrad epilogue (fp32 aux or its bf16 plane)
template <int EPI>
constexpr bool is_dact = EPI == EPI_DACT || EPI == EPI_DACTB;

// bijective XCD remap: consecutive logical tiles land on the same XCD (blockIdx % 8 group)
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = b & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

__device__ __forceinline__ float bf16_bits_to_f32(unsigned short b) {
  return __uint_as_float((unsigned)b << 16);
}
// BCE epilogues: EPI_BCE reads the fp32 target; EPI_BCEB reads its bf16 plane while *xdyn == 0
// (every pixel of the batch a bf16 value) and the fp32 target otherwise -- one launch, the
// choice a uniform branch in the epilogue (bce_x16). An EPI_BCE launch given xdyn returns at once
// when the plane applies (the two-launch form; gemm_run launches EPI_BCEB alone).
template <int EPI>
__device__ __forceinline__ bool epi_skip(const GemmEpi& e) {
  if constexpr (EPI == EPI_BCE) return e.xdyn != nullptr && *e.xdyn == 0;
  return false;
}
// the BCE target read from its bf16 plane?
template <int EPI>
__device__ __forceinline__ bool bce_x16(const GemmEpi& e) {
  if constexpr (EPI == EPI_BCEB) return e.xdyn == nullptr || *e.xdyn == 0;
  return false;
}
// -log-likelihood term of one pixel, TF semantics log(y^x (1-y)^(1-x)) with pow(0,0) = 1 and
// no epsilon (11a/vae.py:266-269). (A single-log form for binary targets makes hipcc spill
// the wide kernel's accumulators across its main loop.)
// Branch-free: both logs evaluated (pinned by the empty asm statements, else hipcc branches per
// element around them) and each term selected, so a 0 * log(0) never enters the sum.
__device__ __forceinline__ float bce_term(float yv, float xv) {
  float l1 = __logf(yv), l0 = __logf(1.f - yv);
  asm("" : "+v"(l1));
  asm("" : "+v"(l0));
  const float a = xv != 0.f ? xv * l1 : 0.f;
  const float b = xv != 1.f ? (1.f - xv) * l0 : 0.f;
  return a + b;
}

// v -> n bf16 planes (n = 1: round to nearest; n = 3: exact split, each residual exact)
__device__ __forceinline__ void store_planes(unsigned short* cp, long long pc, int n, size_t idx,
                                             float v) {
  float r = v;
  for (int t = 0; t < n; ++t) {
    const unsigned short b = __builtin_bit_cast(unsigned short, __float2bfloat16(r));
    cp[t * pc + idx] = b;
    r -= __uint_as_float((unsigned)b << 16);
  }
}

// logical tile of this workgroup (TBM x TBN tiles)
struct Tile {
  int z, bi, si, m0, n0, nt, ks, ke;
};
template <int TBM, int TBN>
__device__ __forceinline__ Tile tile_of_t(const Params& p, bool remap, int boff = 0) {
  Tile t;
  const int tiles = p.ntm * p.ntn;
  const int nwg = tiles * p.batch * p.split;
  // boff: workgroups ahead of the tiles (the fused de-interleave's workers; a multiple of 8, so
  // blockIdx % 8 still names the XCD)
  const int bx = (int)blockIdx.x - boff;
  const int b = remap ? xcd_remap(bx, nwg) : bx;
  t.z = b / tiles;
  const int rem = b - t.z * tiles;
  int mt;
  if (p.group > 0) {
    const int band = rem / (p.group * p.ntn), m0 = band * p.group;
    const int gsz = min(p.ntm - m0, p.group), r = rem - band * p.group * p.ntn;
    t.nt = r / gsz;
    mt = m0 + (r - t.nt * gsz);
  } else {
    mt = rem / p.ntn;
    t.nt = rem - mt * p.ntn;
  }
  t.bi = t.z / p.split;
  t.si = t.z - t.bi * p.split;
  t.m0 = mt * TBM;
  t.n0 = t.nt * TBN;
  t.ks = t.si * p.kchunk;
  t.ke = min(p.K, t.ks + p.kchunk);
  return t;
}
__device__ __forceinline__ Tile tile_of(const Params& p, bool remap) {
  return tile_of_t<BM, BN>(p, remap);
}

// Epilogue over this wave's MI x NI 32x32 accumulators; the wave owns rows
// [m0 + wm*MI*32, +MI*32) and columns [n0 + wn*NI*32, +NI*32) of a TBM-row tile whose
// columns are split over NWN waves. C/D layout of a 32x32 MFMA:
// col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
// BCE: `red` >= NWN*TBM floats of LDS no longer read by the main loop; the row partials are
// written per 128-column block (rowpart[row][N/128 blocks], gemm_bce_nblk) whatever the tile.
template <int EPI, int MI, int NI, int TBM, int NWN>
__device__ __forceinline__ void epilogue_g(const Params& p, const Tile& t, f32x16 (&acc)[MI][NI],
                                           float* red, int wm, int wn) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int fr = lane & 31, fk = lane >> 5;
  float* __restrict__ C = p.C + (size_t)t.z * p.sC;  // z = bi*split + si (slab) or bi (split==1)
  unsigned short* __restrict__ cp = p.epi.cp ? p.epi.cp + (size_t)t.z * p.sC : nullptr;
  const GemmEpi& e = p.epi;
  const int rbase = t.m0 + wm * MI * 32 + 4 * fk;
  const int cbase = t.n0 + wn * NI * 32 + fr;
  // Each 32-row block: the operand the epilogue reads (aux for DACT, the target x for BCE)
  // is loaded for all 16 x NI elements first, then the outputs are computed and stored.
  // (Interleaving load -> use -> store per element serialises one memory latency per element:
  // the stores may alias the loads.)
  constexpr bool BCE = EPI == EPI_BCE || EPI == EPI_BCEB;
  constexpr bool READS = is_dact<EPI> || BCE;
  const bool x16 = bce_x16<EPI>(e);
  // a 0/1 batch whose target the de-interleave wrote as bits (with the pixel operand as bits it
  // writes no bf16 plane): one bit per element
  const bool tbits = EPI == EPI_BCEB && e.xnb && *e.xnb == 0 && e.xbits;
  const float* __restrict__ src = is_dact<EPI> ? e.aux : e.x;
  const int lds_ = is_dact<EPI> ? e.ld_aux : e.ldx;
  // not unrolled: the block's accumulators are acc[0], rotated down after each block (one copy
  // of the epilogue code, see epilogue_rm)
#pragma unroll 1
  for (int mi = 0; mi < MI; ++mi) {
    float sv[16][NI];
    if constexpr (READS) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + mi * 32 + (r & 3) + 8 * (r >> 2);
        int sr = row < p.M ? row : p.M - 1;
        if constexpr (is_dact<EPI>) sr = sr >= e.remap_split ? sr - e.remap_shift : sr;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          int col = cbase + ni * 32;
          col = col < p.N ? col : p.N - 1;
          if (EPI == EPI_BCEB && tbits) sv[r][ni] = (float)((e.xbits[(size_t)sr * e.ldbits + (col >> 3)] >> (col & 7)) & 1);
          else if (EPI == EPI_BCEB && x16) sv[r][ni] = bf16_bits_to_f32(e.xp[(size_t)sr * lds_ + col]);
          else if constexpr (is_dact<EPI>)
            sv[r][ni] = e.auxp ? bf16_bits_to_f32(e.auxp[(size_t)sr * lds_ + col]) : src[(size_t)sr * lds_ + col];
          else sv[r][ni] = src[(size_t)sr * lds_ + col];
        }
      }
    }
    // ACT / DACT: the activation over the block's 16 x NI values with the act switch hoisted
    // out of the element loop (per-element runtime selects broke the epilogue into branches)
    float av[16 * NI];
    if constexpr (EPI == EPI_ACT || is_dact<EPI>) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) av[r * NI + ni] = acc[0][ni][r];
      if constexpr (EPI == EPI_ACT) {
        act_n(av, e.act);
      } else {
        float yv[16 * NI];
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) yv[r * NI + ni] = sv[r][ni];
        dact_n(av, yv, e.act);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + mi * 32 + (r & 3) + 8 * (r >> 2);
      float rs = 0.f;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int col = cbase + ni * 32;
        if (row < p.M && col < p.N) {
          const size_t o = (size_t)row * p.ldc + col;
          float v = acc[0][ni][r];
          if constexpr (EPI == EPI_ACT || is_dact<EPI>) v = av[r * NI + ni];
          if constexpr (BCE) {
            const float yv = sigmoid_fast(v);
            const float xv = sv[r][ni];
            // -log(y^x (1-y)^(1-x)) with TF pow(0,0) = 1 (no epsilon), 11a/vae.py:266-269
            rs += bce_term(yv, xv);
            v = (yv - xv) * e.scale;
            if (e.y) e.y[(size_t)row * e.ldy + col] = yv;
          }
          if constexpr (EPI == EPI_SIGMOID) v = sigmoid_f(v);
          if (e.c32) C[o] = v;
          if (cp) store_planes(cp, e.pc, e.ncp, o, v);
        }
      }
      if constexpr (BCE) {
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) rs += __shfl_xor(rs, off, 64);
        if (fr == 0) red[wn * TBM + (row - t.m0)] = rs;  // lanes 0 and 32
      }
    }
#pragma unroll
    for (int j = 0; j + 1 < MI; ++j)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[j][ni] = acc[j + 1][ni];
  }
  if constexpr (BCE) {
    __syncthreads();
    constexpr int WPB = 128 / (NI * 32);  // waves per 128-column block
    constexpr int NBT = NWN / WPB;        // 128-column blocks per tile
    const int nblk = (p.N + 127) / 128;
    for (int i = tid; i < NBT * TBM; i += blockDim.x) {
      const int b = i / TBM, r = i - b * TBM;
      const int gb = t.nt * NBT + b;
      if (gb < nblk && t.m0 + r < p.M) {
        float s_ = 0.f;
#pragma unroll
        for (int w = 0; w < WPB; ++w) s_ += red[(b * WPB + w) * TBM + r];
        e.rowpart[(size_t)(t.m0 + r) * (e.rp_ld ? e.rp_ld : nblk) + gb + e.rp_off] = -s_;
      }
    }
  }
}

// Row-major epilogue of the 256x256 wide kernels (8 waves 2x4, each 4x2 32x32 accumulators).
// The C/D layout puts 32 consecutive columns of one row in a half-wave, so a direct store is one
// 2-B (bf16 plane) or 4-B element per lane: a 256x256 tile with three output planes takes 384
// store instructions per thread, and the BCE target/aux loads are as narrow. Here each 64-row
// band (accumulator row block mi of both wave rows) goes through LDS instead: the waves write
// their raw accumulators row-major ([64][256] fp32, 64 KB, two bands in flight), pass a barrier,
// and every thread then owns 8 consecutive columns of 4 rows: 16-B loads of the epilogue's
// operands (DACT aux, BCE target), the math, and 16-B stores of the fp32 output and of each
// bf16 plane. BCE row partials: each 8-column chunk's terms summed in order, then a fixed xor
// tree over the 16 lanes of a 128-column block; lane 0 of the 16 writes rowpart. Requires
// (wide_epi_vec_ok) 16-B aligned bases and ld / plane / batch strides that keep 8-column chunks
// 16-B aligned; chunks that cross N fall back to element stores.
__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8f(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ unsigned short bf16_rn_bits(float v) {
  return __builtin_bit_cast(unsigned short, __float2bfloat16(v));
}
// 8 values -> n bf16 planes, one 16-B store per plane (exact split for n = 3)
__device__ __forceinline__ void st8_planes(unsigned short* cp, long long pc, int n, size_t o,
                                           const float (&v)[8]) {
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = v[j];
  for (int t = 0; t < n; ++t) {
    unsigned w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned short lo = bf16_rn_bits(r[2 * j]), hi = bf16_rn_bits(r[2 * j + 1]);
      r[2 * j] -= bf16_bits_to_f32(lo);
      r[2 * j + 1] -= bf16_bits_to_f32(hi);
      w[j] = (unsigned)lo | (unsigned)hi << 16;
    }
    *reinterpret_cast<uint4*>(cp + t * pc + o) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// diag (timing diagnostics, results meaningless): bit 1 = no global stores, bit 2 = no LDS
// transpose, bit 3 = no transcendental math. Waves 2 (M) x NWN (N), NTH threads, each wave
// acc[MI][NI] 32x32 blocks: tile (64*MI) x TW, TW = NWN*NI*32 (a multiple of 128). Band mi =
// accumulator row block mi of both wave rows (64 rows); `lds` holds two bands (2 x 64 x TW fp32).
// Wide kernels: MI 4, NWN 4, NTH 512 (256 x 128*NI tiles); twin kernel: 2, 2, 2, 256 (128 x 128).
// issued (stamped diagnostics builds only): s_memrealtime once the last store is issued
// rpl (BCE): LDS for the per-chunk row partials, (64 MI) x (TW / 8) floats past the two band
// buffers; nullptr: a 16-lane xor-shuffle tree per pass instead (its four dependent lane
// exchanges behind each pass's transcendentals measured ~9 us per 256x256 tile,
// tools/micro/epi.hip)
// Generic form: write_band(band, mi) writes this wave's part of band mi (row-major, TW floats
// per band row) from its accumulators in whatever MFMA layout they are; vec = false: every
// global access element-wise (bases / strides not 16-B aligned, wide_epi_vec_ok false).
// RMAP: tile row of band row br of band mi -- 0: wave row (br >> 5) owns rows [64 MI wr, +64 MI)
// and band mi is its 32-row block mi; 1 (eight-phase kernel, MI 4): 32-row block mi of wave row
// wr is tile rows 128 (mi >> 1) + 64 wr + 32 (mi & 1)
template <int EPI, int MI, int TW, int NTH, class WB, int RMAP = 0>
__device__ __forceinline__ void epilogue_rm_w(const Params& p, const Tile& t, WB&& write_band,
                                              float* lds, int diag, unsigned long long* issued,
                                              float* rpl, bool vec) {
  constexpr int BAND = 64 * TW;  // floats per band buffer
  static_assert(TW % 128 == 0, "BCE row partials are per 128-column block");
  constexpr int CW = TW / 8;                    // 8-column chunks per band row
  constexpr int RP = NTH / CW;                  // band rows per reader pass
  constexpr bool BCE = EPI == EPI_BCE || EPI == EPI_BCEB;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const GemmEpi& e = p.epi;
  float* __restrict__ C = p.C + (size_t)t.z * p.sC;
  unsigned short* __restrict__ cp = e.cp ? e.cp + (size_t)t.z * p.sC : nullptr;
  const int c8 = tid % CW, rr = tid / CW;   // reader: chunk of 8 columns, row within RP
  const int col0 = t.n0 + 8 * c8;
  const int nblk = (p.N + 127) / 128;
  const int gb = t.nt * (TW / 128) + (c8 >> 4);  // 128-column block of this chunk
  constexpr int NQ = 64 / RP;                   // reader passes per band
  // The operand each pass's math reads (DACT activation, BCE target) for all NQ passes of a
  // band, loaded BEFORE the band's LDS transpose so their latency overlaps it (loading inside
  // each pass exposed one global-load latency per pass: 16 per 256-row tile). bf16 sources
  // stay packed (one uint4 per pass) until use.
  constexpr bool LD = is_dact<EPI> || BCE;
  auto tile_row = [&](int mi, int br) {
    if constexpr (RMAP == 1) return (mi >> 1) * 128 + (br >> 5) * 64 + (mi & 1) * 32 + (br & 31);
    return (br >> 5) * (MI * 32) + mi * 32 + (br & 31);
  };
  auto pass_row = [&](int mi, int q) { return t.m0 + tile_row(mi, rr + RP * q); };  // band row -> global
  auto pass_nv = [&](int row) {
    return row >= p.M ? 0 : (col0 >= p.N ? 0 : (p.N - col0 < 8 ? p.N - col0 : 8));
  };
  // whole-chunk access of a partial last chunk (GemmEpi::padw)
  auto pass_full = [&](int nv) { return vec && (nv == 8 || (e.padw && nv > 0)); };
  const bool bsrc = EPI == EPI_DACTB || bce_x16<EPI>(e);  // the operand is bf16
  // the operand rows of band mi's NQ passes: bf16 packed into sb (b16) or fp32 into sf
  // every target pixel of the batch 0 or 1 (the de-interleave's flag): no per-pixel test, and
  // the targets read as one bit per pixel when the de-interleave wrote them so (e.xbits)
  const bool allbin = EPI == EPI_BCEB && e.xnb && *e.xnb == 0;
  const bool tbits = allbin && e.xbits != nullptr;
  constexpr int SFN_ = (LD && EPI != EPI_BCEB) ? NQ : 1;
  auto load_band = [&](int mi, bool b16, float (&sf)[SFN_][8], uint4 (&sb)[LD ? NQ : 1]) {
    if constexpr (LD) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int row = pass_row(mi, q);
        const int nv = pass_nv(row);
        int sr = row < p.M ? row : p.M - 1;
        if constexpr (is_dact<EPI>) sr = sr >= e.remap_split ? sr - e.remap_shift : sr;
        const int ld_src = is_dact<EPI> ? e.ld_aux : e.ldx;
        if (EPI == EPI_BCEB && tbits) {  // byte col0 / 8 of the row: bit j = column col0 + j
          sb[q] = make_uint4(nv > 0 ? (unsigned)e.xbits[(size_t)sr * e.ldbits + (col0 >> 3)] : 0u, 0u, 0u, 0u);
        } else if (b16) {
          const unsigned short* src = (is_dact<EPI> ? e.auxp : e.xp) + (size_t)sr * ld_src + col0;
          if (pass_full(nv)) {
            sb[q] = *reinterpret_cast<const uint4*>(src);
          } else {
            unsigned short h[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) h[j] = j < nv ? src[j] : (unsigned short)0;
            sb[q] = make_uint4((unsigned)h[0] | (unsigned)h[1] << 16, (unsigned)h[2] | (unsigned)h[3] << 16,
                               (unsigned)h[4] | (unsigned)h[5] << 16, (unsigned)h[6] | (unsigned)h[7] << 16);
          }
        } else if constexpr (EPI != EPI_BCEB) {
          const float* src = (is_dact<EPI> ? e.aux : e.x) + (size_t)sr * ld_src + col0;
          if (pass_full(nv)) ld8f(src, sf[q]);
          else
#pragma unroll
            for (int j = 0; j < 8; ++j) sf[q][j] = j < nv ? src[j] : 0.f;
        }
      }
    }
  };
  // bf16 operands are loaded one band ahead (issued before band mi-1's transpose and passes),
  // so their latency hides behind a whole band of work; fp32 operands (twice the registers:
  // double-buffered they spill) at the start of their own band, before its LDS transpose
  // (the combined BCE epilogue reads its rare fp32 target per pass instead: beside the bf16
  // double buffer a band of fp32 operands spilled)
  constexpr int SFN = (LD && EPI != EPI_BCEB) ? NQ : 1;
  float sf[SFN][8];
  uint4 sb[LD ? NQ : 1], sbn[LD ? NQ : 1];
  if (bsrc) load_band(0, true, sf, sb);
  // One band per iteration of a NON-unrolled loop: the band's accumulators are always acc[0]
  // (the blocks rotate down after the writer), so the epilogue code is emitted once instead of
  // MI times (37.6 -> 13.6 KB for the 256x256 ACT kernel; no time change measured).
#pragma unroll 1
  for (int mi = 0; mi < MI; ++mi) {
    float* band = lds + (mi & 1) * BAND;
    if (bsrc) {
      if (mi + 1 < MI) load_band(mi + 1, true, sf, sbn);
    } else {
      load_band(mi, false, sf, sb);
    }
    if (!(diag & 4)) write_band(band, mi);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int br = rr + RP * q;                                    // band row
      const int row = pass_row(mi, q);
      float v[8];
      const float4 a = *reinterpret_cast<const float4*>(band + br * TW + 8 * c8);
      const float4 b = *reinterpret_cast<const float4*>(band + br * TW + 8 * c8 + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      const bool rok = row < p.M;
      const int nv = pass_nv(row);
      const bool full = pass_full(nv);
      float rs = 0.f;
      if (nv > 0) {
        float sv[8];
        if constexpr (LD) {
          if (EPI == EPI_BCEB && tbits) {
#pragma unroll
            for (int j = 0; j < 8; ++j) sv[j] = (sb[q].x >> j) & 1u ? 1.f : 0.f;
          } else if (bsrc) {
            const unsigned ww[4] = {sb[q].x, sb[q].y, sb[q].z, sb[q].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              sv[2 * j] = __uint_as_float(ww[j] << 16);
              sv[2 * j + 1] = __uint_as_float(ww[j] & 0xffff0000u);
            }
          } else if constexpr (EPI == EPI_BCEB) {  // the fp32 target, read here (see sf)
            const float* src = e.x + (size_t)(row < p.M ? row : p.M - 1) * e.ldx + col0;
            if (full) ld8f(src, sv);
            else
#pragma unroll
              for (int j = 0; j < 8; ++j) sv[j] = j < nv ? src[j] : 0.f;
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) sv[j] = sf[q][j];
          }
        }
        float yv[8];
        if constexpr (BCE) {
          if (diag & 8) {  // timing diagnostics: no transcendental math
#pragma unroll
            for (int j = 0; j < 8; ++j) { yv[j] = v[j]; rs += v[j] * sv[j]; v[j] = (yv[j] - sv[j]) * e.scale; }
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) yv[j] = sigmoid_fast(v[j]);
            // binary targets (every target of the wave's passes 0 or 1, a wave-uniform branch):
            // the term is log(x ? y : 1 - y) -- the same value as the two-log form below, whose
            // other term is exactly 0 -- at one logarithm per pixel instead of two
            // (hardware log2 scaled by ln 2: v_log_f32 + one multiply, where __logf expands to
            // ~12 instructions of denormal scaling and extended-precision correction)
            bool bin = allbin;
            if (!bin) {
              bool b = true;
#pragma unroll
              for (int j = 0; j < 8; ++j) b &= (sv[j] == 0.f) | (sv[j] == 1.f);
              bin = __all(b);
            }
            if (bin) {
              float bt[8];
#pragma unroll
              for (int j = 0; j < 8; ++j)
                bt[j] = __builtin_amdgcn_logf(sv[j] != 0.f ? yv[j] : 1.f - yv[j]) * 0.693147180559945309f;
              if (nv == 8) {  // (the same sum in the same order, without the column mask)
#pragma unroll
                for (int j = 0; j < 8; ++j) rs += bt[j];
              } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) rs += j < nv ? bt[j] : 0.f;
              }
            } else {
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                // -log(y^x (1-y)^(1-x)) with TF pow(0,0) = 1 (no epsilon), 11a/vae.py:266-269
                const float bt = bce_term(yv[j], sv[j]);
                rs += j < nv ? bt : 0.f;
              }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (yv[j] - sv[j]) * e.scale;
          }
        }
        if constexpr (EPI == EPI_ACT)
          if (!(diag & 8)) act_n(v, e.act);
        if constexpr (EPI == EPI_SIGMOID) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = sigmoid_f(v[j]);
        }
        if constexpr (is_dact<EPI>) dact_n(v, sv, e.act);
        if (nv < 8) {  // padding columns of a whole-chunk store (GemmEpi::padw)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j >= nv) v[j] = (e.padw == 2 && col0 + j == p.N) ? 1.f : 0.f;
          if constexpr (BCE)
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (j >= nv) yv[j] = 0.f;
        }
        const size_t o = (size_t)row * p.ldc + col0;
        if (diag & 2) {
        } else if (full) {
          if (e.c32) st8f(C + o, v);
          if (cp) st8_planes(cp, e.pc, e.ncp, o, v);
          if constexpr (BCE)
            if (e.y) st8f(e.y + (size_t)row * e.ldy + col0, yv);
        } else {
          for (int j = 0; j < nv; ++j) {
            if (e.c32) C[o + j] = v[j];
            if (cp) store_planes(cp, e.pc, e.ncp, o + j, v[j]);
            if constexpr (BCE)
              if (e.y) e.y[(size_t)row * e.ldy + col0 + j] = yv[j];
          }
        }
      }
      if constexpr (BCE) {
        if (rpl) {
          rpl[tile_row(mi, br) * CW + c8] = rs;
        } else {
#pragma unroll
          for (int off = 8; off >= 1; off >>= 1) rs += __shfl_xor(rs, off, 64);
          if ((c8 & 15) == 0 && rok && gb < nblk) e.rowpart[(size_t)row * (e.rp_ld ? e.rp_ld : nblk) + gb + e.rp_off] = -rs;
        }
      }
    }
    if constexpr (LD) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) sb[q] = sbn[q];
    }
  }
  if constexpr (BCE) {
    if (rpl) {
      // each (tile row, 128-column block): its 16 chunk partials summed in the order of the
      // xor-shuffle tree (off = 8, 4, 2, 1 -- the same sums, bit for bit)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      constexpr int NB = TW / 128;
      for (int i = tid; i < 64 * MI * NB; i += NTH) {
        const int tr = i / NB, b = i - tr * NB;
        const int row = t.m0 + tr, gbb = t.nt * NB + b;
        const float* q = rpl + tr * CW + 16 * b;
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; j += 4) {
          const float4 a = *reinterpret_cast<const float4*>(q + j);
          v[j] = a.x; v[j + 1] = a.y; v[j + 2] = a.z; v[j + 3] = a.w;
        }
        float t8[8], t4[4];
#pragma unroll
        for (int j = 0; j < 8; ++j) t8[j] = v[j] + v[j + 8];
#pragma unroll
        for (int j = 0; j < 4; ++j) t4[j] = t8[j] + t8[j + 4];
        const float sum = (t4[0] + t4[2]) + (t4[1] + t4[3]);
        if (row < p.M && gbb < nblk) e.rowpart[(size_t)row * (e.rp_ld ? e.rp_ld : nblk) + gbb + e.rp_off] = -sum;
      }
    }
  }
  if (issued) {
    unsigned long long tt;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt) :: "memory");
    *issued = tt;
  }
}

// Row-major epilogue of the 32x32-MFMA kernels (waves 2 (M) x NWN (N), acc[MI][NI] of 32x32 blocks
// in the C/D layout: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)). The band's blocks
// are always acc[0] (rotated down after each band: the band loop is not unrolled).
template <int EPI, int MI, int NI, int NWN, int NTH>
__device__ __forceinline__ void epilogue_rm(const Params& p, const Tile& t, f32x16 (&acc)[MI][NI],
                                            float* lds, int wm, int wn, int diag = 0,
                                            unsigned long long* issued = nullptr,
                                            float* rpl = nullptr, bool vec = true) {
  constexpr int TW = NWN * NI * 32;
  const int lane = threadIdx.x & 63;
  auto wb = [&](float* band, int) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        band[row * TW + wn * (NI * 32) + ni * 32 + (lane & 31)] = acc[0][ni][r];
      }
#pragma unroll
    for (int j = 0; j + 1 < MI; ++j)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[j][ni] = acc[j + 1][ni];
  };
  epilogue_rm_w<EPI, MI, TW, NTH>(p, t, wb, lds, diag, issued, rpl, vec);
}

// the 128x128-tile kernels: 4 waves in 2x2, each 2x2 accumulators
template <int EPI>
__device__ __forceinline__ void epilogue(const Params& p, const Tile& t, f32x16 (&acc)[2][2],
                                         float* red) {
  const int wave = threadIdx.x >> 6;
  epilogue_g<EPI, 2, 2, BM, 2>(p, t, acc, red, wave >> 1, wave & 1);
}

}  // namespace gemm

// the eight-phase 256 x 256 kernel (gemm_bf16e.hip) for a planned tile (g.tn == TN_E8); te: the
// row-major LDS epilogue
hipError_t gemm_bf16e_launch(const gemm::PParams& p, bool at, bool bt, int epi, bool te, hipStream_t st);

}  // namespace mvae
