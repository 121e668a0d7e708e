// bf16-MFMA GEMM family for gfx950 (v_mfma_f32_32x32x16_bf16, fp32 accumulate) with the same
// fused epilogues as the fp32 family. Operands stay fp32 in HBM; the loader converts each
// staged element into TA (TB) bf16 terms in LDS:
//   T = 1: x ~ bf16(x)                         (MVAE_PREC_BF16: bf16 operands, fp32 accumulate)
//   T = 3: x = hi + mid + lo, each bf16, EXACT (8+8+8 significand bits; each residual is an
//          exact fp32 difference), so sum_{i+j<3} a_i b_j reproduces the fp32 product to
//          ~2^-24 relative and the MFMA accumulates in fp32 (MVAE_PREC_F32X: fp32-accurate
//          GEMM at bf16-MFMA rate — gfx950 has no xf32, and bf16 MFMA is 16x the fp32 rate).
// DYNA: when every staged A element of a k-tile is exactly bf16 (e.g. the binary pixels of
// the shape images), the A residual terms are skipped for that k-tile (workgroup-uniform
// decision through per-wave ballots), so an exact-bf16 operand costs 1 term, not 3.
//
// Tile 128x128xBK, 4 waves (2x2), each wave 2x2 MFMA 32x32 tiles. LDS image per term:
//   k-contiguous operand ([rows][K] in HBM): [row][k], row stride BK+8 bf16 -> fragments by
//     ds_read_b128 (8 consecutive k), conflict-free;
//   row-contiguous operand ([K][rows]): [k][row], row stride 160 bf16 -> fragments by two
//     ds_read_b64_tr_b16 (the CDNA4 transposing LDS read), conflict-free;
// both written with 8-byte ds_write_b64 from one 16-B global load each. One LDS buffer,
// next tile's global loads in registers during the MFMAs, two barriers per k-tile.
#include "gemm_common.h"

namespace mvae {
namespace {

using namespace gemm;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int SR = 160;  // [k][row] stride (bf16): 320 B = 64 mod 256 -> tr reads conflict-free

__device__ __forceinline__ unsigned short bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, __float2bfloat16(v));
}
__device__ __forceinline__ float bf16_val(unsigned short b) {
  return __uint_as_float((unsigned)b << 16);
}

// split 4 floats into T bf16 terms (packed 4 x 16 bit per term); returns residual-nonzero
template <int T>
__device__ __forceinline__ bool split4(const float4 v, s16x4 (&o)[T]) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  bool nz = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float r = x[e];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const unsigned short b = bf16_bits(r);
      o[t][e] = (short)b;
      r = r - bf16_val(b);  // exact
      if (t == 0) nz |= r != 0.f;
    }
  }
  return nz;
}

template <bool KC, int T, int BK>
struct Stage {
  static constexpr int SK = BK + 8;                       // [row][k] stride
  static constexpr int PLANE = KC ? 128 * SK : BK * SR;   // bf16 elements per term plane
  static constexpr int NLD = 128 * BK / 4 / NT;           // float4 loads per thread
  float4 r[NLD];

  __device__ __forceinline__ void load(const float* __restrict__ g, int ld, int row0, int nrows,
                                       int k0, int kend, int tid) {
    if constexpr (KC) {
      const bool kfull = k0 + BK <= kend;
#pragma unroll
      for (int j = 0; j < NLD; ++j) {
        const int c = tid + NT * j;
        const int row = c / (BK / 4), kq = c % (BK / 4);
        int gr = row0 + row;
        gr = gr < nrows ? gr : nrows - 1;
        const int gk = k0 + 4 * kq;
        const float* p = g + (size_t)gr * ld + gk;
        if (kfull) {
          r[j] = *reinterpret_cast<const float4*>(p);
        } else {
          r[j].x = gk + 0 < kend ? p[0] : 0.f;
          r[j].y = gk + 1 < kend ? p[1] : 0.f;
          r[j].z = gk + 2 < kend ? p[2] : 0.f;
          r[j].w = gk + 3 < kend ? p[3] : 0.f;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NLD; ++j) {
        const int c = tid + NT * j;
        const int k = c >> 5, rq = c & 31;
        const int gk = k0 + k;
        const int gr = row0 + 4 * rq;
        if (gk < kend) {
          const float* p = g + (size_t)gk * ld + gr;
          if (gr + 3 < nrows) {
            r[j] = *reinterpret_cast<const float4*>(p);
          } else {
            r[j].x = gr + 0 < nrows ? p[0] : 0.f;
            r[j].y = gr + 1 < nrows ? p[1] : 0.f;
            r[j].z = gr + 2 < nrows ? p[2] : 0.f;
            r[j].w = gr + 3 < nrows ? p[3] : 0.f;
          }
        } else {
          r[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  }

  // convert + store the staged tile; returns whether any residual term is nonzero
  __device__ __forceinline__ bool store(short* s, int tid) {
    bool nz = false;
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      s16x4 o[T];
      nz |= split4<T>(r[j], o);
      const int c = tid + NT * j;
      int off;
      if constexpr (KC) {
        const int row = c / (BK / 4), kq = c % (BK / 4);
        off = row * SK + 4 * kq;
      } else {
        const int k = c >> 5, rq = c & 31;
        off = k * SR + 4 * rq;
      }
#pragma unroll
      for (int t = 0; t < T; ++t) *reinterpret_cast<s16x4*>(s + t * PLANE + off) = o[t];
    }
    return nz;
  }

  // fragment (8 consecutive k) of term t for the 32-row block starting at row rb, k-step ks
  __device__ __forceinline__ bf16x8 frag(const short* s, int t, int rb, int ks, int lane) const {
    const short* base = s + t * PLANE;
    if constexpr (KC) {
      const s16x8 v = *reinterpret_cast<const s16x8*>(base + (rb + (lane & 31)) * SK + 16 * ks +
                                                      8 * (lane >> 5));
      return __builtin_bit_cast(bf16x8, v);
    } else {
      const int i = lane & 15, q = i >> 2, p = i & 3;
      const int h = lane >> 5, g1 = (lane >> 4) & 1;
      const short* a0 = base + (16 * ks + 8 * h + q) * SR + rb + 16 * g1 + 4 * p;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * SR));
      const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

template <bool AT, bool BT, int TA, int TB, bool DYNA, int BK, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(Params p) {
  using SA = Stage<!AT, TA, BK>;
  using SB = Stage<BT, TB, BK>;
  constexpr int A_ELEMS = TA * SA::PLANE, B_ELEMS = TB * SB::PLANE;
  __shared__ __attribute__((aligned(16))) short smem[A_ELEMS + B_ELEMS];
  __shared__ int wflag[4];
  short* As = smem;
  short* Bs = smem + A_ELEMS;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const Tile t = tile_of(p, true);
  const float* __restrict__ A = p.A + t.bi * p.sA;
  const float* __restrict__ Bm = p.B + t.bi * p.sB;

  SA la;
  SB lb;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = t.ks < t.ke ? (t.ke - t.ks + BK - 1) / BK : 0;
  if (nk > 0) {
    la.load(A, p.lda, t.m0, p.M, t.ks, t.ke, tid);
    lb.load(Bm, p.ldb, t.n0, p.N, t.ks, t.ke, tid);
    const bool nz = la.store(As, tid);
    lb.store(Bs, tid);
    if constexpr (DYNA) {
      const bool w = __ballot(nz) != 0;
      if (lane == 0) wflag[wave] = w;
    }
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(A, p.lda, t.m0, p.M, t.ks + (kt + 1) * BK, t.ke, tid);
      lb.load(Bm, p.ldb, t.n0, p.N, t.ks + (kt + 1) * BK, t.ke, tid);
    }
    int ta = TA;
    if constexpr (DYNA) ta = (wflag[0] | wflag[1] | wflag[2] | wflag[3]) ? TA : 1;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[TA][2], fb[TB][2];
#pragma unroll
      for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) fa[i][mi] = la.frag(As, i, wm * 64 + mi * 32, ks, lane);
#pragma unroll
      for (int j = 0; j < TB; ++j)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) fb[j][ni] = lb.frag(Bs, j, wn * 64 + ni * 32, ks, lane);
      // products a_i b_j with i + j < max(TA, TB), smallest terms first
      constexpr int T = TA > TB ? TA : TB;
#pragma unroll
      for (int s = T - 1; s >= 0; --s) {
#pragma unroll
        for (int i = 0; i < TA; ++i) {
          const int j = s - i;
          if (j < 0 || j >= TB) continue;
          if (DYNA && i > 0 && ta == 1) continue;
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][mi], fb[j][ni], acc[mi][ni], 0, 0, 0);
        }
      }
    }
    __syncthreads();
    if (more) {
      const bool nz = la.store(As, tid);
      lb.store(Bs, tid);
      if constexpr (DYNA) {
        const bool w = __ballot(nz) != 0;
        if (lane == 0) wflag[wave] = w;
      }
    }
    __syncthreads();
  }
  epilogue<EPI>(p, t, acc, reinterpret_cast<float*>(smem));
}

template <bool AT, bool BT, int TA, int TB, bool DYNA, int BK, int EPI>
hipError_t launch_t(const Params& p, hipStream_t st) {
  const int nwg = p.ntm * p.ntn * p.batch * p.split;
  hipLaunchKernelGGL((gemm_bf16_kernel<AT, BT, TA, TB, DYNA, BK, EPI>), dim3(nwg), dim3(NT), 0, st, p);
  return hipGetLastError();
}

template <int TA, int TB, bool DYNA, int BK, int EPI>
hipError_t launch_layout(const Params& p, bool at, bool bt, hipStream_t st) {
  if (!at && !bt) return launch_t<false, false, TA, TB, DYNA, BK, EPI>(p, st);
  if (at && !bt) return launch_t<true, false, TA, TB, DYNA, BK, EPI>(p, st);
  if (!at && bt) return launch_t<false, true, TA, TB, DYNA, BK, EPI>(p, st);
  return launch_t<true, true, TA, TB, DYNA, BK, EPI>(p, st);
}

template <int EPI>
hipError_t launch_mode(const Params& p, bool at, bool bt, int mode, hipStream_t st) {
  if (mode == GEMM_BF16) return launch_layout<1, 1, false, 64, EPI>(p, at, bt, st);
  return launch_layout<3, 3, true, 32, EPI>(p, at, bt, st);  // GEMM_F32X
}

}  // namespace

hipError_t gemm_bf16_launch(const gemm::Params& p, bool at, bool bt, int mode, int epi, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_mode<EPI_STORE>(p, at, bt, mode, st);
    case EPI_ACT: return launch_mode<EPI_ACT>(p, at, bt, mode, st);
    case EPI_DACT: return launch_mode<EPI_DACT>(p, at, bt, mode, st);
    case EPI_BCE: return launch_mode<EPI_BCE>(p, at, bt, mode, st);
    case EPI_SIGMOID: return launch_mode<EPI_SIGMOID>(p, at, bt, mode, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mvae
