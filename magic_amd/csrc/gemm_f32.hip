// fp32-input MFMA GEMM for gfx950 (v_mfma_f32_32x32x2_f32: exact fp32, k-ordered fma chain)
// with the fused epilogues of the metric-VAE step.
//
// C[M,N] = A[M,K] * B[K,N], A stored row-major [M][K] or transposed [K][M] (at),
// B stored [K][N] or transposed [N][K] (bt). Every bias is folded into the GEMM: activation
// buffers carry a constant ones column and each parameter block is the augmented [W; b]
// (rows K+1), so forward = one GEMM, and the weight gradient of [W; b] = one GEMM whose M
// includes the ones column (the bias gradient is its last row).
//
// Tile 128x128x32, 256 threads = 4 waves in 2x2, each wave 64x64 = 2x2 MFMA 32x32 tiles.
// LDS tiles are k-major ([BK][BM+pad]) so every fragment read is a conflict-free ds_read_b32
// at consecutive addresses; the register-staged global loader transposes operands whose
// global layout is k-contiguous (pad 1 -> conflict-free transposing ds_write_b32) and copies
// m-/n-contiguous operands with ds_write_b128 (pad 4). Double-buffered LDS, one barrier per
// k-tile, next tile's global loads issued before the MFMAs of the current one.
// Blocks are remapped so that the column tiles of one row panel share an XCD (L2 reuse of A).
// Split-K (for small grids) writes fp32 partial slabs that a second kernel sums in a fixed
// order and passes through the epilogue: results are deterministic run to run.
#include "gemm_common.h"

#include <algorithm>
#include <cmath>
#include <cstdint>

namespace mvae {
namespace {

using namespace gemm;
constexpr int BK = 32;

template <bool KCONTIG, int SLD, int ROWS>
struct TileLoader;

// operand whose global layout is k-contiguous: [rows][K] -> LDS [BK][rows] (transpose)
template <int SLD, int ROWS>
struct TileLoader<true, SLD, ROWS> {
  float4 r[4];
  __device__ __forceinline__ void load(const float* __restrict__ g, int ld, int row0, int nrows,
                                       int k0, int kend, int tid) {
    const bool kfull = k0 + BK <= kend;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tid + NT * j;
      const int row = c >> 3, kq = c & 7;
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
  }
  __device__ __forceinline__ void store(float* s, int tid) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tid + NT * j;
      const int row = c >> 3, kq = c & 7;
      float* q = s + (4 * kq) * SLD + row;
      q[0] = r[j].x; q[SLD] = r[j].y; q[2 * SLD] = r[j].z; q[3 * SLD] = r[j].w;
    }
  }
};

// operand whose global layout is row(m/n)-contiguous: [K][rows] -> LDS [BK][rows] (copy)
template <int SLD, int ROWS>
struct TileLoader<false, SLD, ROWS> {
  float4 r[4];
  __device__ __forceinline__ void load(const float* __restrict__ g, int ld, int row0, int nrows,
                                       int k0, int kend, int tid) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
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
  __device__ __forceinline__ void store(float* s, int tid) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tid + NT * j;
      const int k = c >> 5, rq = c & 31;
      *reinterpret_cast<float4*>(s + k * SLD + 4 * rq) = r[j];
    }
  }
};

// VAR (diagnostic A/B variants, EPI_STORE only): 0 default; 1 fragments read per k-step
// (no read-ahead); 2 no XCD remap.
template <bool AT, bool BT, int EPI, int VAR = 0>
__global__ __launch_bounds__(NT, 2) void gemm_f32_kernel(Params p) {
  constexpr bool A_KC = !AT;  // A stored [M][K] -> k-contiguous
  constexpr bool B_KC = BT;   // B stored [N][K] -> k-contiguous
  constexpr int SA = A_KC ? BM + 1 : BM + 4;
  constexpr int SB = B_KC ? BN + 1 : BN + 4;
  constexpr int A_TILE = BK * SA, B_TILE = BK * SB;
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_TILE + B_TILE)];
  float* As = smem;
  float* Bs = smem + 2 * A_TILE;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  if (epi_skip<EPI>(p.epi)) return;
  const Tile t = tile_of(p, VAR != 2);
  const int bi = t.bi, m0 = t.m0, n0 = t.n0, ks = t.ks, ke = t.ke;

  const float* __restrict__ A = p.A + bi * p.sA;
  const float* __restrict__ Bm = p.B + bi * p.sB;

  TileLoader<A_KC, SA, BM> la;
  TileLoader<B_KC, SB, BN> lb;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = ks < ke ? (ke - ks + BK - 1) / BK : 0;
  if (nk > 0) {
    la.load(A, p.lda, m0, p.M, ks, ke, tid);
    lb.load(Bm, p.ldb, n0, p.N, ks, ke, tid);
    la.store(As, tid);
    lb.store(Bs, tid);
  }
  __syncthreads();

  const int fr = lane & 31, fk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(A, p.lda, m0, p.M, ks + (kt + 1) * BK, ke, tid);
      lb.load(Bm, p.ldb, n0, p.N, ks + (kt + 1) * BK, ke, tid);
    }
    const float* as = As + cur * A_TILE + wm * 64 + fr + fk * SA;
    const float* bs = Bs + cur * B_TILE + wn * 64 + fr + fk * SB;
    if constexpr (VAR == 1) {
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        const float a0 = as[2 * kk * SA], a1 = as[2 * kk * SA + 32];
        const float b0 = bs[2 * kk * SB], b1 = bs[2 * kk * SB + 32];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    } else {
      // read the whole k-tile's fragments first (distinct registers), then the MFMA chain:
      // the LDS latency overlaps the MFMAs instead of serialising every group of four
      float fa[BK / 2][2], fb[BK / 2][2];
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        fa[kk][0] = as[2 * kk * SA];
        fa[kk][1] = as[2 * kk * SA + 32];
        fb[kk][0] = bs[2 * kk * SB];
        fb[kk][1] = bs[2 * kk * SB + 32];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk][0], fb[kk][0], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk][0], fb[kk][1], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk][1], fb[kk][0], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[kk][1], fb[kk][1], acc[1][1], 0, 0, 0);
      }
    }
    if (more) {
      la.store(As + (cur ^ 1) * A_TILE, tid);
      lb.store(Bs + (cur ^ 1) * B_TILE, tid);
    }
    __syncthreads();
  }

  epilogue<EPI>(p, t, acc, smem);
}

// sum split-K slabs in fixed order and apply the epilogue
template <int EPI>
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int split, int M, int N,
                                     float* __restrict__ C, int ldc, long long sC, GemmEpi e) {
  if (e.only_if && *e.only_if == 0) return;
  const int bi = blockIdx.z;
  const long long slab = (long long)M * N;
  const float* w = ws + (size_t)bi * split * slab;
  float* c = C + bi * sC;
  const long long total = slab;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    // the slab loads in groups of 8 issued before their ordered sum (a load -> wait -> add
    // chain per slab left every thread waiting out `split` memory latencies in a row: 36 us
    // median for the 501 x 500 hidden-layer weight gradients at split 16-32)
    float v = 0.f;
    int s = 0;
    for (; s + 8 <= split; s += 8) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = w[(s + j) * slab + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) v += t[j];
    }
    for (; s < split; ++s) v += w[s * slab + i];
    const int row = (int)(i / N), col = (int)(i - (long long)row * N);
    if constexpr (EPI == EPI_ACT) v = act_f(v, e.act);
    if constexpr (EPI == EPI_SIGMOID) v = sigmoid_f(v);
    if constexpr (EPI == EPI_DACT) {
      const int ar = row >= e.remap_split ? row - e.remap_shift : row;
      const size_t ai = (size_t)ar * e.ld_aux + col;
      v = dact_f(v, e.auxp ? bf16_bits_to_f32(e.auxp[ai]) : e.aux[ai], e.act);
    }
    if (e.c32) c[(size_t)row * ldc + col] = v;
    if (e.cp) store_planes(e.cp + bi * sC, e.pc, e.ncp, (size_t)row * ldc + col, v);
  }
}

// The same, 4 consecutive columns per thread: 16-B slab loads and fp32 stores, one 8-B store
// per bf16 plane (the scalar form above is store-issue bound). Needs N, ldc, the plane and
// batch strides multiples of 4 and 16-B aligned C / 8-B aligned planes (splitk_reduce4_ok).
template <int EPI>
__global__ void splitk_reduce4_kernel(const float* __restrict__ ws, int split, int M, int N,
                                      float* __restrict__ C, int ldc, long long sC, GemmEpi e) {
  if (e.only_if && *e.only_if == 0) return;
  const int bi = blockIdx.z;
  const long long slab = (long long)M * N;
  const float* w = ws + (size_t)bi * split * slab;
  float* c = C + bi * sC;
  unsigned short* cp = e.cp ? e.cp + bi * sC : nullptr;
  const int n4 = N >> 2;
  const long long total = (long long)M * n4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(i / n4), col = 4 * (int)(i - (long long)row * n4);
    const size_t si = (size_t)row * N + col;
    float4 a = *reinterpret_cast<const float4*>(w + si);
    int s = 1;
    for (; s + 4 <= split; s += 4) {  // same order as the scalar kernel: ((s0 + s1) + s2) ...
      float4 u[4];                    // (loads of 4 slabs issued before their sum)
#pragma unroll
      for (int j = 0; j < 4; ++j) u[j] = *reinterpret_cast<const float4*>(w + (s + j) * slab + si);
#pragma unroll
      for (int j = 0; j < 4; ++j) { a.x += u[j].x; a.y += u[j].y; a.z += u[j].z; a.w += u[j].w; }
    }
    for (; s < split; ++s) {
      const float4 u = *reinterpret_cast<const float4*>(w + s * slab + si);
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
    if constexpr (EPI == EPI_ACT) {
      if (e.act == ACT_TANH) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = act_f(v[j], ACT_TANH);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = act_f(v[j], ACT_ELU);
      }
    }
    if constexpr (EPI == EPI_SIGMOID) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = sigmoid_f(v[j]);
    }
    if constexpr (EPI == EPI_DACT) {
      const int ar = row >= e.remap_split ? row - e.remap_shift : row;
      const size_t ai = (size_t)ar * e.ld_aux + col;
      float y[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = e.auxp ? bf16_bits_to_f32(e.auxp[ai + j]) : e.aux[ai + j];
      dact_n(v, y, e.act);
    }
    const size_t o = (size_t)row * ldc + col;
    if (e.c32) *reinterpret_cast<float4*>(c + o) = make_float4(v[0], v[1], v[2], v[3]);
    if (cp) {
      float r[4] = {v[0], v[1], v[2], v[3]};
      for (int t = 0; t < e.ncp; ++t) {
        unsigned short b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          b[j] = __builtin_bit_cast(unsigned short, __float2bfloat16(r[j]));
          r[j] -= bf16_bits_to_f32(b[j]);
        }
        *reinterpret_cast<uint2*>(cp + t * e.pc + o) =
            make_uint2((unsigned)b[0] | (unsigned)b[1] << 16, (unsigned)b[2] | (unsigned)b[3] << 16);
      }
    }
  }
}

bool splitk_reduce4_ok(const GemmDesc& d) {
  auto a = [](const void* p, int n) { return (reinterpret_cast<uintptr_t>(p) & (n - 1)) == 0; };
  if ((d.N & 3) || (d.ldc & 3) || (d.sC & 3) || !a(d.C, 16)) return false;
  if (d.epi.cp && ((d.epi.pc & 3) || !a(d.epi.cp, 8))) return false;
  return true;
}

template <bool AT, bool BT, int EPI, int VAR>
hipError_t launch_t(const Params& p, hipStream_t st) {
  const int nwg = p.ntm * p.ntn * p.batch * p.split;
  hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, EPI, VAR>), dim3(nwg), dim3(NT), 0, st, p);
  return hipGetLastError();
}

template <int EPI, int VAR = 0>
hipError_t launch_layout(const Params& p, bool at, bool bt, hipStream_t st) {
  if (!at && !bt) return launch_t<false, false, EPI, VAR>(p, st);
  if (at && !bt) return launch_t<true, false, EPI, VAR>(p, st);
  if (!at && bt) return launch_t<false, true, EPI, VAR>(p, st);
  return launch_t<true, true, EPI, VAR>(p, st);
}

hipError_t launch_store(const Params& p, bool at, bool bt, int variant, hipStream_t st) {
  switch (variant) {
    case 1: return launch_layout<EPI_STORE, 1>(p, at, bt, st);
    case 2: return launch_layout<EPI_STORE, 2>(p, at, bt, st);
    default: return launch_layout<EPI_STORE, 0>(p, at, bt, st);
  }
}

}  // namespace

int gemm_bce_nblk(int N) { return (N + BN - 1) / BN; }

int gemm_plan_split(const GemmDesc& d, size_t max_ws) {
  if (d.epi.mode == EPI_BCE || d.epi.mode == EPI_BCEB || d.epi.mode == EPI_SIGMOID) return 1;
  if (d.valu) return gemm_valu_split(d, max_ws);
  if (gemm_bf16_wide(d)) return gemm_bf16_wide_split(d, max_ws);
  const int ntm = (d.M + BM - 1) / BM, ntn = (d.N + BN - 1) / BN;
  const long long tiles = (long long)ntm * ntn * d.batch;
  const int ktiles = (d.K + BK - 1) / BK;
  // Throughput model: each CU works through ceil(WGs/256) workgroups (two co-resident WGs
  // overlap each other's stalls but share the MFMA pipes), each WG costs its k-tiles plus a
  // fixed prologue/epilogue; split-K adds the slab round trip and one reduction launch.
  const double cus = 256.0;
  // one 128x128x32 k-tile per CU: fp32 MFMA rate; bf16 / 3-term split are load-bound
  const double t_ktile = d.prec == GEMM_F32 ? 1.75e-6 : (d.prec == GEMM_BF16 ? 0.3e-6 : 0.5e-6);
  double best = 1e30;
  int best_s = 1;
  for (int s = 1; s <= 32; ++s) {
    if (s > 1 && ktiles / s < 4) break;
    if (s > 1 && (size_t)d.batch * s * d.M * d.N > max_ws) break;
    const double rounds = std::ceil(tiles * s / cus);
    double t = rounds * ((double)ktiles / s + 2.0) * t_ktile;
    if (s > 1) t += (double)d.batch * s * d.M * d.N * 8.0 / 4.5e12 + 4e-6;
    if (t < best * 0.97) { best = t; best_s = s; }
  }
  return best_s;
}

size_t gemm_workspace_elems(const GemmDesc& d) {
  const int s = d.split > 0 ? d.split : gemm_plan_split(d, ~size_t(0));
  return s > 1 ? (size_t)d.batch * s * d.M * d.N : 0;
}

hipError_t gemm_run(const GemmDesc& d, float* ws, size_t ws_elems, hipStream_t st) {
  if (d.M <= 0 || d.N <= 0) return hipSuccess;
  Params p;
  p.M = d.M; p.N = d.N; p.K = d.K;
  p.A = d.A; p.lda = d.lda; p.B = d.B; p.ldb = d.ldb;
  p.sA = d.sA; p.sB = d.sB;
  p.batch = d.batch;
  p.ntm = (d.M + BM - 1) / BM; p.ntn = (d.N + BN - 1) / BN;
  p.epi = d.epi;
  if (d.prec == GEMM_F32) p.epi.xdyn = nullptr;  // fp32 kernels read the fp32 BCE target
  // one planner pass: split-K and (bf16 DMA kernels) the ring tile
  const size_t wsz = ws ? ws_elems : 0;
  int split = 1;
  p.tn = 0;
  p.tm = 256;
  if (!d.valu && gemm_bf16_wide(d)) gemm_bf16_wide_plan(d, wsz, &split, &p.tn, &p.tm);
  else split = gemm_plan_split(d, wsz);
  if (d.split > 0) split = d.split;
  if (split > 1 && (!ws || (size_t)d.batch * split * d.M * d.N > ws_elems)) return hipErrorInvalidValue;
  p.split = split;
  const int kb = d.prec == GEMM_F32 ? BK : 64;  // k-tile of the kernel that runs
  const int ktiles = (d.K + kb - 1) / kb;
  p.kchunk = ((ktiles + split - 1) / split) * kb;
  if (split == 1) {
    p.C = d.C; p.ldc = d.ldc; p.sC = d.sC;
    if (d.valu) return gemm_valu_launch(p, d, d.epi.mode, st);
    if (d.prec != GEMM_F32) {
      // BCE with a bf16-plane target: one launch choosing the plane or the fp32 target by *xdyn
      if (d.epi.mode == EPI_BCE && d.epi.xp && d.epi.xdyn) return gemm_bf16_launch(p, d, EPI_BCEB, st);
      Params q = p;
      q.epi.xdyn = nullptr;  // a single BCE launch always runs (fp32 target)
      return gemm_bf16_launch(q, d, d.epi.mode, st);
    }
    switch (d.epi.mode) {
      case EPI_STORE: return launch_store(p, d.at, d.bt, d.variant, st);
      case EPI_ACT: return launch_layout<EPI_ACT>(p, d.at, d.bt, st);
      case EPI_DACT: return launch_layout<EPI_DACT>(p, d.at, d.bt, st);
      case EPI_BCE: return launch_layout<EPI_BCE>(p, d.at, d.bt, st);
      case EPI_SIGMOID: return launch_layout<EPI_SIGMOID>(p, d.at, d.bt, st);
      default: return hipErrorInvalidValue;
    }
  }
  // split-K: raw slabs [batch][split][M][N], then ordered reduction + epilogue
  p.C = ws; p.ldc = d.N; p.sC = (long long)d.M * d.N;
  p.epi.cp = nullptr;  // planes (and the fp32 output, if any) are written by the reduction
  p.epi.c32 = 1;       // the slabs themselves always
  p.epi.padw = 0;      // slab rows are N wide (ldc = N): no whole-chunk stores past column N
  hipError_t err = d.valu ? gemm_valu_launch(p, d, EPI_STORE, st)
                 : d.prec != GEMM_F32 ? gemm_bf16_launch(p, d, EPI_STORE, st)
                                      : launch_store(p, d.at, d.bt, d.variant, st);
  if (err != hipSuccess) return err;
  const long long total = (long long)d.M * d.N;
  int grid = (int)std::min<long long>((total + 255) / 256, 2048);
  dim3 g(grid, 1, d.batch);
  // small outputs (weight gradients of the latent head / decoder layer 1): one element per
  // thread, so the slices' loads spread over more waves
  if (splitk_reduce4_ok(d) && total >= (1 << 18)) {
    dim3 g4((int)std::min<long long>((total / 4 + 255) / 256, 2048), 1, d.batch);
    switch (d.epi.mode) {
      case EPI_STORE:
        hipLaunchKernelGGL(splitk_reduce4_kernel<EPI_STORE>, g4, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
        break;
      case EPI_ACT:
        hipLaunchKernelGGL(splitk_reduce4_kernel<EPI_ACT>, g4, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
        break;
      case EPI_DACT:
        hipLaunchKernelGGL(splitk_reduce4_kernel<EPI_DACT>, g4, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
        break;
      case EPI_SIGMOID:
        hipLaunchKernelGGL(splitk_reduce4_kernel<EPI_SIGMOID>, g4, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
        break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (d.epi.mode) {
    case EPI_STORE:
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_STORE>, g, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
      break;
    case EPI_ACT:
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_ACT>, g, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
      break;
    case EPI_DACT:
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_DACT>, g, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
      break;
    case EPI_SIGMOID:
      hipLaunchKernelGGL(splitk_reduce_kernel<EPI_SIGMOID>, g, dim3(256), 0, st, ws, split, d.M, d.N, d.C, d.ldc, d.sC, d.epi);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mvae
