// fp32 VALU GEMM for the step's skinny products (gfx950): C[M,N] = A[M,K] B[K,N] where an MFMA
// tile would be mostly empty — one output dimension or the reduction dimension <= 64 (at small
// latent sizes: the latent head forward / weight gradient (N = 2L), the decoder's first layer
// (K = L + 1) and its weight gradient (M = L + 1), the latent-head dgrad (K = 2L) and the
// decoder's dgrad into z (N = L)). Exact fp32 products and fp32 sums (the fp32 parity class of
// the MFMA paths), the fused epilogues of gemm_common.h's Params, split-K through the ordered
// slab reduction of gemm_f32.hip.
//
// Tile 64x64, K in chunks of 32 staged through LDS in [k][row] order (transposing the
// k-contiguous operands on the way in; two buffers, the next chunk in flight in registers),
// 256 threads each owning a 4x4 output block: per k two 16-B LDS reads (4 rows of A broadcast
// over 16 lanes, 4 columns of B) feed 16 FMAs.
#include "gemm_common.h"

namespace mvae {
namespace {

using namespace gemm;

constexpr int VT = 64, VKC = 32, VNT = 256, VSLD = VT + 4;  // LDS row stride (16-B aligned rows)

// chunk [k0, k0 + VKC) x [r0, r0 + VT) of an operand: 2 float4 per thread held in registers
// (load) while the previous chunk is multiplied, then written to s[k][r] (store)
template <bool KC>
struct VStage {
  float4 v[2];
  __device__ __forceinline__ void load(const float* __restrict__ g, int ld, int r0, int nrows, int k0,
                                       int kend, int tid, bool al) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + VNT * i;  // 512 quads = 2048 floats
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (KC) {
        const int r = idx >> 3, kq = idx & 7;
        const int gr = r0 + r, gk = k0 + 4 * kq;
        if (gr < nrows) {
          const float* p = g + (size_t)gr * ld + gk;
          if (al && gk + 4 <= kend) {
            x = *reinterpret_cast<const float4*>(p);
          } else {
            x.x = gk + 0 < kend ? p[0] : 0.f;
            x.y = gk + 1 < kend ? p[1] : 0.f;
            x.z = gk + 2 < kend ? p[2] : 0.f;
            x.w = gk + 3 < kend ? p[3] : 0.f;
          }
        }
      } else {
        const int k = idx >> 4, rq = idx & 15;
        const int gk = k0 + k, gr = r0 + 4 * rq;
        if (gk < kend) {
          const float* p = g + (size_t)gk * ld + gr;
          if (al && gr + 4 <= nrows) {
            x = *reinterpret_cast<const float4*>(p);
          } else {
            x.x = gr + 0 < nrows ? p[0] : 0.f;
            x.y = gr + 1 < nrows ? p[1] : 0.f;
            x.z = gr + 2 < nrows ? p[2] : 0.f;
            x.w = gr + 3 < nrows ? p[3] : 0.f;
          }
        }
      }
      v[i] = x;
    }
  }
  __device__ __forceinline__ void store(float* s, int tid) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + VNT * i;
      if constexpr (KC) {
        const int r = idx >> 3, kq = idx & 7;
        float* q = s + (4 * kq) * VSLD + r;
        q[0] = v[i].x; q[VSLD] = v[i].y; q[2 * VSLD] = v[i].z; q[3 * VSLD] = v[i].w;
      } else {
        const int k = idx >> 4, rq = idx & 15;
        *reinterpret_cast<float4*>(s + k * VSLD + 4 * rq) = v[i];
      }
    }
  }
};

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(VNT) void gemm_valu_kernel(Params p) {
  // two LDS buffers of [A chunk | B chunk]: the next chunk's global loads are in flight in
  // registers while the current chunk is multiplied; one barrier per chunk
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * VKC * VSLD];
  const int tid = threadIdx.x;
  const int tm = tid >> 4, tn = tid & 15;
  const Tile t = tile_of_t<VT, VT>(p, false);
  const float* __restrict__ A = p.A + t.bi * p.sA;
  const float* __restrict__ Bm = p.B + t.bi * p.sB;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  // 16-B operand loads only where every row start is 16-B aligned (the step's buffers are)
  const bool ala = ((reinterpret_cast<uintptr_t>(A) & 15) | (p.lda & 3)) == 0;
  const bool alb = ((reinterpret_cast<uintptr_t>(Bm) & 15) | (p.ldb & 3)) == 0;
  VStage<!AT> la;
  VStage<BT> lb;
  // DACT: this thread's 4 x 4 activation values loaded before the k-loop, their latency behind
  // it (loaded in the epilogue, each row's loads waited behind the previous row's stores, which
  // may alias them)
  float ax[4][4];
  if constexpr (EPI == EPI_DACT) {
    const GemmEpi& e = p.epi;
    const int c0 = t.n0 + 4 * tn;
    const bool av = c0 + 4 <= p.N && (e.ld_aux & 3) == 0 && (reinterpret_cast<uintptr_t>(e.aux) & 15) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row = t.m0 + 4 * tm + i;
      row = row < p.M ? row : p.M - 1;
      const int ar = row >= e.remap_split ? row - e.remap_shift : row;
      const float* x = e.aux + (size_t)ar * e.ld_aux + c0;
      if (av) {
        const float4 q = *reinterpret_cast<const float4*>(x);
        ax[i][0] = q.x; ax[i][1] = q.y; ax[i][2] = q.z; ax[i][3] = q.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) ax[i][j] = c0 + j < p.N ? x[j] : 0.f;
      }
    }
  }
  const int nch = t.ks < t.ke ? (t.ke - t.ks + VKC - 1) / VKC : 0;
  if (nch > 0) {
    la.load(A, p.lda, t.m0, p.M, t.ks, t.ke, tid, ala);
    lb.load(Bm, p.ldb, t.n0, p.N, t.ks, t.ke, tid, alb);
    la.store(smem, tid);
    lb.store(smem + VKC * VSLD, tid);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const float* As = smem + (c & 1) * 2 * VKC * VSLD;
    const float* Bs = As + VKC * VSLD;
    const bool more = c + 1 < nch;
    if (more) {
      const int k1 = t.ks + (c + 1) * VKC;
      la.load(A, p.lda, t.m0, p.M, k1, t.ke, tid, ala);
      lb.load(Bm, p.ldb, t.n0, p.N, k1, t.ke, tid, alb);
    }
#pragma unroll 8
    for (int k = 0; k < VKC; ++k) {
      const float4 a = *reinterpret_cast<const float4*>(As + k * VSLD + 4 * tm);
      const float4 b = *reinterpret_cast<const float4*>(Bs + k * VSLD + 4 * tn);
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
    }
    if (more) {
      float* nb = smem + ((c + 1) & 1) * 2 * VKC * VSLD;
      la.store(nb, tid);
      lb.store(nb + VKC * VSLD, tid);
    }
    __syncthreads();
  }
  // epilogue: 4 rows x 4 consecutive columns per thread
  float* __restrict__ C = p.C + (size_t)t.z * p.sC;
  unsigned short* __restrict__ cp = p.epi.cp ? p.epi.cp + (size_t)t.z * p.sC : nullptr;
  const GemmEpi& e = p.epi;
  const int c0 = t.n0 + 4 * tn;
  const bool vec = c0 + 4 <= p.N && (p.ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0 &&
                   (!cp || ((reinterpret_cast<uintptr_t>(cp) & 7) == 0 && (e.pc & 3) == 0));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = t.m0 + 4 * tm + i;
    if (row >= p.M) continue;
    float v[4] = {acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
    if constexpr (EPI == EPI_ACT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = act_f(v[j], e.act);
    }
    if constexpr (EPI == EPI_SIGMOID) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = sigmoid_f(v[j]);
    }
    if constexpr (EPI == EPI_DACT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = c0 + j < p.N ? dact_f(v[j], ax[i][j], e.act) : 0.f;
    }
    const size_t o = (size_t)row * p.ldc + c0;
    if (vec) {
      if (e.c32) *reinterpret_cast<float4*>(C + o) = make_float4(v[0], v[1], v[2], v[3]);
      if (cp) {
        float r[4] = {v[0], v[1], v[2], v[3]};
        for (int q = 0; q < e.ncp; ++q) {
          unsigned short b[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            b[j] = __builtin_bit_cast(unsigned short, __float2bfloat16(r[j]));
            r[j] -= bf16_bits_to_f32(b[j]);
          }
          *reinterpret_cast<uint2*>(cp + q * e.pc + o) =
              make_uint2((unsigned)b[0] | (unsigned)b[1] << 16, (unsigned)b[2] | (unsigned)b[3] << 16);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c0 + j >= p.N) break;
        if (e.c32) C[o + j] = v[j];
        if (cp) store_planes(cp, e.pc, e.ncp, o + j, v[j]);
      }
    }
  }
}

template <bool AT, bool BT, int EPI>
hipError_t launch_v(const Params& p, hipStream_t st) {
  const int nwg = p.ntm * p.ntn * p.batch * p.split;
  hipLaunchKernelGGL((gemm_valu_kernel<AT, BT, EPI>), dim3(nwg), dim3(VNT), 0, st, p);
  return hipGetLastError();
}

template <int EPI>
hipError_t launch_v_layout(const Params& p, bool at, bool bt, hipStream_t st) {
  if (!at && !bt) return launch_v<false, false, EPI>(p, st);
  if (at && !bt) return launch_v<true, false, EPI>(p, st);
  if (!at && bt) return launch_v<false, true, EPI>(p, st);
  return launch_v<true, true, EPI>(p, st);
}

}  // namespace

bool gemm_valu_fits(const GemmDesc& d) {
  if (d.variant != 0) return false;
  if (d.epi.mode == EPI_BCE || d.epi.mode == EPI_BCEB) return false;
  // skinny K, or a skinny output with a short K (the long-K weight gradients of the latent head
  // and decoder layer 1 stay on the fp32 MFMA kernel: measured faster, profiles/r2)
  const int lo = d.M < d.N ? d.M : d.N;
  return d.K <= 64 || (lo <= 64 && d.K <= 1024);
}

int gemm_valu_split(const GemmDesc& d, size_t max_ws) {
  const long long tiles = (long long)((d.M + VT - 1) / VT) * ((d.N + VT - 1) / VT) * d.batch;
  const int chunks = (d.K + VKC - 1) / VKC;
  // latency-bound small kernels: aim at >= 4 waves per SIMD (1024 workgroups of 4 waves), at
  // least 2 chunks per slice, at most 16 slices (the ordered reduction reads them serially)
  int s = 1;
  while (s * 2 <= 16 && s * 2 <= chunks / 2 && tiles * s < 1024 &&
         (size_t)d.batch * 2 * s * d.M * d.N <= max_ws)
    s *= 2;
  return s;
}

hipError_t gemm_valu_launch(const gemm::Params& g, const GemmDesc& d, int epi, hipStream_t st) {
  Params p = g;
  p.ntm = (d.M + VT - 1) / VT;
  p.ntn = (d.N + VT - 1) / VT;
  const int chunks = (d.K + VKC - 1) / VKC;
  p.kchunk = ((chunks + p.split - 1) / p.split) * VKC;
  switch (epi) {
    case EPI_STORE: return launch_v_layout<EPI_STORE>(p, d.at, d.bt, st);
    case EPI_ACT: return launch_v_layout<EPI_ACT>(p, d.at, d.bt, st);
    case EPI_DACT: return launch_v_layout<EPI_DACT>(p, d.at, d.bt, st);
    case EPI_SIGMOID: return launch_v_layout<EPI_SIGMOID>(p, d.at, d.bt, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mvae
