// Conv-encoder tower of the metric-VAE (BASELINE config 5): the CifarNet
// tower of the reference's siamese overlap regressor (6b/net.py:50-60) in front of the fully
// connected encoder, weights shared by the three encoder passes:
//
//   conv1 5x5x64 SAME + ReLU -> max_pool 2x2/2 -> LRN(4, 1, 1e-3/9, .75)      conv1_fwd_kernel
//   conv2 5x5x64 SAME + ReLU                                                   conv2_* kernels
//   LRN -> max_pool 2x2/2 -> flatten (NHWC, feature (h*W4 + w)*64 + c)         lrn2_pool2_fwd_kernel
//
// Activations are NHWC fp32, one image per row of the stacked batch ([rot | lock | key], 3B rows
// forward; [rot g1 | lock g1 | lock g2 | key g2], 4B rows backward, backward row j reading
// forward row j < 2B ? j : j - B). Every per-pixel op maps the 64 channels onto the 64 lanes of
// one wavefront: LRN's channel window is 8 lane shuffles, pooling is per lane, and loads and
// stores of a pixel are one coalesced 256-B access.
//
// Pooling routes its gradient to the FIRST maximum of the window in row-major order (TF's
// MaxPoolGrad); the ReLU in front of pool 1 is folded into the backward as (pooled value > 0).
// Weight gradients reduce over image chunks into fixed-order slabs (no float atomics): a step
// is bitwise reproducible.
#include "mvae_internal.h"

namespace mvae {
namespace {

constexpr int CH = 64;   // channels of both conv layers (6b/net.py:50,55)
constexpr int KS = 5;    // kernel size
constexpr int NT = KS * KS;
constexpr int LRN_R = 4;
constexpr float LRN_BIAS = 1.f, LRN_ALPHA = 0.001f / 9.f, LRN_BETA = 0.75f;  // 6b/net.py:54,57

inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

__device__ __forceinline__ int remap(int j, int B2) { return j < B2 ? j : j - B2 / 2; }

// whole-wave lane shifts by one (DPP wave_shr:1 / wave_shl:1, GFX9 family): a VALU move, no
// LDS traffic; bound_ctrl: the lane shifted in reads 0 (the LRN window's clipping at the ends)
__device__ __forceinline__ float wave_shr1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float wave_shl1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

// sum over channels |j - c| <= 4 (clipped at 0 and 63) of v_j; lane c holds v_c
__device__ __forceinline__ float win_sum(float v, int c) {
  (void)c;
  float s = v, a = v, b = v;
#pragma unroll
  for (int d = 1; d <= LRN_R; ++d) {
    a = wave_shr1(a);
    b = wave_shl1(b);
    s += a + b;
  }
  return s;
}

// s^-beta for s >= 1 (the LRN scale: bias 1): native v_log_f32 / v_exp_f32
__device__ __forceinline__ float pow_nbeta(float s) {
  return __builtin_amdgcn_exp2f(-LRN_BETA * __builtin_amdgcn_logf(s));
}

__device__ __forceinline__ float lrn_fwd(float a, int c) {
  const float s = LRN_BIAS + LRN_ALPHA * win_sum(a * a, c);
  return a * pow_nbeta(s);
}

// d a_c of out = lrn(a) given d out (g), TF LRNGrad
__device__ __forceinline__ float lrn_bwd(float a, float g, int c) {
  const float s = LRN_BIAS + LRN_ALPHA * win_sum(a * a, c);
  const float sb = pow_nbeta(s);
  const float inner = win_sum(g * a * sb / s, c);
  return g * sb - 2.f * LRN_ALPHA * LRN_BETA * a * inner;
}

__device__ __forceinline__ unsigned short bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, __float2bfloat16(v));
}

// bf16 plane images (1 plane RN, or 3 planes exact split) of one fp32 value
__device__ __forceinline__ void put_planes(unsigned short* p, long long ps, int n, size_t idx, float v) {
  float r = v;
  for (int t = 0; t < n; ++t) {
    const unsigned short b = bf16_bits(r);
    p[t * ps + idx] = b;
    r -= __uint_as_float((unsigned)b << 16);
  }
}

// ---------------------------------------------------------------- conv1 + pool1 + LRN1
// Workgroup: one image, one pooled row qy, a segment of SEG pooled columns. The segment's
// 6 x (2*SEG + 4) input patch is staged in LDS once; each wave then takes pooled pixels
// w, w+4, ... with lane = output channel, reading the 36 patch values it needs as LDS
// broadcasts. The four conv outputs of the 2x2 window are formed in registers, ReLU,
// first-max pooling, then LRN across the lanes. w: conv1 block [26][64] (25 taps, bias row).
// Writes p1 (pooled, for LRN1's backward), arg1 (window position of the max), n1 (conv2's
// input) and, when n1b, its bf16 image.
constexpr int SEG_MAX = 64;
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const float* __restrict__ xs, int ldx,
                                                        const float* __restrict__ w, int S, int seg,
                                                        float* __restrict__ p1, unsigned char* __restrict__ arg1,
                                                        float* __restrict__ n1, unsigned short* __restrict__ n1b) {
  __shared__ float patch[6][2 * SEG_MAX + 4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int S1 = S / 2;
  const int img = blockIdx.z, qy = blockIdx.y, qx0 = blockIdx.x * seg;
  const int nq = min(seg, S1 - qx0);
  const int pw = 2 * nq + 4;
  const float* x = xs + (size_t)img * ldx;
  for (int i = threadIdx.x; i < 6 * pw; i += 256) {
    const int r = i / pw, cc = i % pw;
    const int y = 2 * qy - 2 + r, xx = 2 * qx0 - 2 + cc;
    patch[r][cc] = (y >= 0 && y < S && xx >= 0 && xx < S) ? x[y * S + xx] : 0.f;
  }
  float wr[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wr[t] = w[t * CH + lane];
  const float b = w[NT * CH + lane];
  __syncthreads();
  for (int q = wv; q < nq; q += 4) {
    float pv[36];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) pv[i * 6 + j] = patch[i][2 * q + j];
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int dy = k >> 1, dx = k & 1;
      float acc = b;
#pragma unroll
      for (int ky = 0; ky < KS; ++ky)
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) acc = fmaf(pv[(dy + ky) * 6 + dx + kx], wr[ky * KS + kx], acc);
      const float v = fmaxf(acc, 0.f);
      if (v > best) { best = v; arg = k; }
    }
    const size_t o = (((size_t)img * S1 + qy) * S1 + qx0 + q) * CH + lane;
    p1[o] = best;
    arg1[o] = (unsigned char)arg;
    const float nv = lrn_fwd(best, lane);
    if (n1) n1[o] = nv;
    if (n1b) n1b[o] = bf16_bits(nv);
  }
}

// ---------------------------------------------------------------- conv2 (fp32 VALU)
// out[img][p][n] = sum_{t, k} in[img][p + t][k] * Wt[t][k][n]  (+ bias, ReLU when FWD)
// FWD: Wt[t][k][n] = W[t*64 + k][n]; data gradient (!FWD): Wt[t][k][n] = W[(24 - t)*64 + n][k]
// (the SAME conv's input gradient is the SAME conv of the output gradient with the kernel
// rotated by 180 degrees and its channel axes swapped). Workgroup: one image, an 8x8 output
// tile x 64 channels; its 12x12x64 input patch sits in LDS, the weights stream in one tap at
// a time. Thread: 4 pixels of a tile row x 4 channels.
template <bool FWD>
__global__ __launch_bounds__(256) void conv2_valu_kernel(const float* __restrict__ in, const float* __restrict__ W,
                                                         float* __restrict__ out, int S1) {
  __shared__ float patch[12 * 12 * CH];
  __shared__ float wt[CH * CH];
  const int tid = threadIdx.x;
  const int tilesx = (S1 + 7) / 8;
  const int ty0 = (blockIdx.x / tilesx) * 8, tx0 = (blockIdx.x % tilesx) * 8;
  const size_t imgoff = (size_t)blockIdx.y * S1 * S1 * CH;
  for (int i = tid; i < 144 * (CH / 4); i += 256) {
    const int px = i / (CH / 4), c4 = i % (CH / 4);
    const int y = ty0 - 2 + px / 12, x = tx0 - 2 + px % 12;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y >= 0 && y < S1 && x >= 0 && x < S1)
      v = *reinterpret_cast<const float4*>(in + imgoff + ((size_t)y * S1 + x) * CH + 4 * c4);
    *reinterpret_cast<float4*>(patch + px * CH + 4 * c4) = v;
  }
  const int n0 = 4 * (tid & 15);
  const int pg = tid >> 4;            // 16 groups of 4 pixels: tile row pg/2, cols 4*(pg&1)..
  const int ry = pg >> 1, rx = 4 * (pg & 1);
  float acc[4][4] = {};
  for (int t = 0; t < NT; ++t) {
    __syncthreads();
    for (int i = tid; i < CH * CH; i += 256) {
      const int k = i / CH, n = i % CH;
      wt[i] = FWD ? W[(size_t)(t * CH + k) * CH + n] : W[(size_t)((NT - 1 - t) * CH + n) * CH + k];
    }
    __syncthreads();
    const int ky = t / KS, kx = t % KS;
    const float* pr = patch + ((ry + ky) * 12 + rx + kx) * CH;
#pragma unroll 4
    for (int k = 0; k < CH; ++k) {
      const float4 w4 = *reinterpret_cast<const float4*>(wt + k * CH + n0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = pr[i * CH + k];
        acc[i][0] = fmaf(a, w4.x, acc[i][0]);
        acc[i][1] = fmaf(a, w4.y, acc[i][1]);
        acc[i][2] = fmaf(a, w4.z, acc[i][2]);
        acc[i][3] = fmaf(a, w4.w, acc[i][3]);
      }
    }
  }
  float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
  if (FWD) bias = *reinterpret_cast<const float4*>(W + (size_t)NT * CH * CH + n0);
  const int y = ty0 + ry;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int x = tx0 + rx + i;
    if (y >= S1 || x >= S1) continue;
    float4 v = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
    if (FWD) {
      v.x = fmaxf(v.x + bias.x, 0.f); v.y = fmaxf(v.y + bias.y, 0.f);
      v.z = fmaxf(v.z + bias.z, 0.f); v.w = fmaxf(v.w + bias.w, 0.f);
    }
    *reinterpret_cast<float4*>(out + imgoff + ((size_t)y * S1 + x) * CH + n0) = v;
  }
}

// ---------------------------------------------------------------- LRN2 + pool2 (forward)
// One wave per FPP pooled pixels (loads of all of them issued first): LRN of the four window
// pixels, first max -> the layer-0 operand row (feature (qy*S2 + qx)*64 + c; fp32 and/or bf16
// planes) and the window position.
constexpr int FPP = 2;
__global__ __launch_bounds__(256) void lrn2_pool2_fwd_kernel(const float* __restrict__ a2, int S1, int nimg,
                                                             float* __restrict__ xf, int ldf, int f32,
                                                             unsigned short* __restrict__ xfp, long long pstride,
                                                             int np, unsigned char* __restrict__ arg2) {
  const int lane = threadIdx.x & 63;
  const int S2 = S1 / 2;
  const long long NP = (long long)nimg * S2 * S2;
  const long long P0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * FPP;
  if (P0 >= NP) return;
  float a[FPP][4];
  long long Pu[FPP];
#pragma unroll
  for (int u = 0; u < FPP; ++u) {
    const long long P = P0 + u < NP ? P0 + u : NP - 1;   // a tail duplicate writes the same values
    Pu[u] = P;
    const int img = (int)(P / (S2 * S2));
    const int qq = (int)(P - (long long)img * S2 * S2);
    const int qy = qq / S2, qx = qq - qy * S2;
    const float* src = a2 + (size_t)img * S1 * S1 * CH;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      a[u][q] = src[((size_t)(2 * qy + (q >> 1)) * S1 + 2 * qx + (q & 1)) * CH + lane];
  }
#pragma unroll
  for (int u = 0; u < FPP; ++u) {
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float v = lrn_fwd(a[u][q], lane);
      if (v > best) { best = v; arg = q; }
    }
    const long long P = Pu[u];
    const int img = (int)(P / (S2 * S2));
    const int qq = (int)(P - (long long)img * S2 * S2);
    const size_t o = (size_t)img * ldf + (size_t)qq * CH + lane;
    if (f32) xf[o] = best;
    if (xfp) put_planes(xfp, pstride, np, o, best);
    arg2[(size_t)P * CH + lane] = (unsigned char)arg;
  }
}

// ---------------------------------------------------------------- pool2 + LRN2 + ReLU (backward)
// One wave per PPW (backward image, pooled pixel) pairs: dxf -> the window's argmax pixel ->
// LRNGrad -> ReLU mask; every pixel of the window is written (zeros off the argmax). The loads
// of all PPW pooled pixels are issued before any of them is used (the kernel is bound by load
// latency: one pooled pixel per wave left its waves waiting 77 % of their cycles).
constexpr int PPW = 4;
__global__ __launch_bounds__(256) void pool2_bwd_kernel(const float* __restrict__ dxf, int ldf,
                                                        const float* __restrict__ a2,
                                                        const unsigned char* __restrict__ arg2, int S1,
                                                        int nimg, int B2, float* __restrict__ da2,
                                                        unsigned short* __restrict__ da2b) {
  const int lane = threadIdx.x & 63;
  const int S2 = S1 / 2;
  const long long NP = (long long)nimg * S2 * S2;
  const long long P0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * PPW;
  if (P0 >= NP) return;
  float g[PPW], a[PPW][4];
  int ar[PPW];
  size_t obase[PPW];
  int pw[PPW];
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    const long long P = P0 + u < NP ? P0 + u : NP - 1;   // a tail duplicate writes the same values
    const int j = (int)(P / (S2 * S2));
    const int qq = (int)(P - (long long)j * S2 * S2);
    const int qy = qq / S2, qx = qq - qy * S2;
    const int f = remap(j, B2);
    g[u] = dxf[(size_t)j * ldf + (size_t)qq * CH + lane];
    ar[u] = arg2[((size_t)f * S2 * S2 + qq) * CH + lane];
    const float* src = a2 + (size_t)f * S1 * S1 * CH;
    pw[u] = (2 * qy) * S1 + 2 * qx;
#pragma unroll
    for (int q = 0; q < 4; ++q) a[u][q] = src[(size_t)(pw[u] + (q >> 1) * S1 + (q & 1)) * CH + lane];
    obase[u] = (size_t)j * S1 * S1;
  }
#pragma unroll
  for (int u = 0; u < PPW; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float dn = ar[u] == q ? g[u] : 0.f;
      float d = 0.f;
      if (__ballot(dn != 0.f)) d = lrn_bwd(a[u][q], dn, lane);
      d = a[u][q] > 0.f ? d : 0.f;
      const size_t o = (obase[u] + pw[u] + (q >> 1) * S1 + (q & 1)) * CH + lane;
      if (da2) da2[o] = d;
      if (da2b) da2b[o] = bf16_bits(d);
    }
}

// ---------------------------------------------------------------- conv1 weight gradient
// dn1 = d(LRN-1 output) -> LRNGrad with p1 -> ReLU mask (p1 > 0) = d1, the gradient at the
// argmax pixel's conv1 pre-activation; slab[grp][chunk][t][c] = sum over the chunk's backward
// images j (group grp: rows [grp*2B, grp*2B + 2B)) and pooled pixels of
// d1[j][P][c] * x[fwd row][argmax pixel + tap t], t = 25: the bias row.
// The workgroup walks the chunk's segments (image, pooled row, QS pooled columns): a segment's
// dn1 / p1 / arg1 rows and its 6-row input band are staged in LDS, and the NEXT segment's are
// already loading into registers while this one computes (the walk is otherwise a chain of
// dependent global loads). Compute: each wave takes pooled columns w, w+4, ... with
// lane = channel (LRNGrad across the lanes) and gathers its 25 taps from the band at its own
// argmax offset.
constexpr int QS = 32;
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const float* __restrict__ dn1,
                                                          const float* __restrict__ p1,
                                                          const unsigned char* __restrict__ arg1,
                                                          const float* __restrict__ xs, int ldx, int S,
                                                          int B2, int ipc, float* __restrict__ slab) {
  constexpr int BW = 2 * QS + 4;
  // staging images; the final cross-wave reduction reuses the same LDS (20 KB per workgroup:
  // several workgroups per CU keep enough segment loads in flight)
  constexpr int NSTAGE = 6 * BW + 2 * QS * CH + QS * CH / 4;
  constexpr int NRED = 4 * 13 * CH;   // the 26 accumulator rows reduce in two halves of 13
  __shared__ __attribute__((aligned(16))) float lds[NSTAGE > NRED ? NSTAGE : NRED];
  float* band = lds;
  float* sg = band + 6 * BW;
  float* sa = sg + QS * CH;
  unsigned char* sr = reinterpret_cast<unsigned char*>(sa + QS * CH);
  auto red = reinterpret_cast<float (*)[13][CH]>(lds);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int S1 = S / 2, np1 = S1 * S1;
  const int grp = blockIdx.y, chunk = blockIdx.x;
  const int j0 = grp * B2 + chunk * ipc;
  const int j1 = min(j0 + ipc, grp * B2 + B2);
  const int nseg = (S1 + QS - 1) / QS;
  const int nit = j1 > j0 ? (j1 - j0) * S1 * nseg : 0;
  float rg[8], ra[8], rb[2];
  uint2 rr = make_uint2(0, 0);
  int cur_nq = 0;
  auto fetch = [&](int it) {
    const int j = j0 + it / (S1 * nseg);
    const int rem = it % (S1 * nseg);
    const int qy = rem / nseg, q0 = (rem % nseg) * QS;
    const int nq = min(QS, S1 - q0);
    const int f = remap(j, B2);
    const size_t pg = (size_t)j * np1 + (size_t)qy * S1 + q0;   // first pooled pixel (backward image)
    const size_t pf = (size_t)f * np1 + (size_t)qy * S1 + q0;   // ... (forward image)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, px = e >> 6;
      rg[u] = px < nq ? dn1[pg * CH + e] : 0.f;
      ra[u] = px < nq ? p1[pf * CH + e] : 0.f;
    }
    rr = (tid * 8) / CH < nq ? *reinterpret_cast<const uint2*>(arg1 + pf * CH + tid * 8) : make_uint2(0, 0);
    const float* x = xs + (size_t)f * ldx;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + 256 * u, r = i / BW, cc = i % BW;
      const int y = 2 * qy - 2 + r, xx = 2 * q0 - 2 + cc;
      rb[u] = (i < 6 * BW && y >= 0 && y < S && xx >= 0 && xx < S) ? x[y * S + xx] : 0.f;
    }
    return nq;
  };
  auto commit = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) { sg[tid + 256 * u] = rg[u]; sa[tid + 256 * u] = ra[u]; }
    *reinterpret_cast<uint2*>(sr + tid * 8) = rr;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (tid + 256 * u < 6 * BW) band[tid + 256 * u] = rb[u];
  };
  float acc[NT + 1] = {};
  if (nit > 0) {
    cur_nq = fetch(0);
    commit();
  }
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int nq = cur_nq;
    int next_nq = 0;
    if (it + 1 < nit) next_nq = fetch(it + 1);
    for (int q = wv; q < nq; q += 4) {
      const float g = sg[q * CH + lane], a = sa[q * CH + lane];
      const int ar = sr[q * CH + lane];
      float v = 0.f;
      if (__ballot(g != 0.f)) v = lrn_bwd(a, g, lane);
      v = a > 0.f ? v : 0.f;
      const float* bp = band + (ar >> 1) * BW + 2 * q + (ar & 1);
#pragma unroll
      for (int ky = 0; ky < KS; ++ky)
#pragma unroll
        for (int kx = 0; kx < KS; ++kx)
          acc[ky * KS + kx] = fmaf(v, bp[ky * BW + kx], acc[ky * KS + kx]);
      acc[NT] += v;
    }
    __syncthreads();
    if (it + 1 < nit) {
      commit();
      cur_nq = next_nq;
    }
    __syncthreads();
  }
  // staging images dead: the LDS becomes the reduction buffer (two halves of 13 rows)
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 13; ++t) red[wv][t][lane] = acc[13 * hf + t];
    __syncthreads();
    for (int i = tid; i < 13 * CH; i += 256) {
      const int t = i / CH, c = i % CH;
      slab[((size_t)grp * gridDim.x + chunk) * (NT + 1) * CH + 13 * hf * CH + i] =
          ((red[0][t][c] + red[1][t][c]) + red[2][t][c]) + red[3][t][c];
    }
  }
}

// ---------------------------------------------------------------- conv2 weight gradient (VALU)
// slab[grp][chunk][t*64 + k][n] = sum over the chunk's backward images j and output pixels p of
// n1[fwd row][p + tap t][k] * da2[j][p][n]; blockIdx.z = t (25: the bias row, k = 0 only).
// Tiles of 64 pixels x 64 channels of both operands are staged in LDS; thread: 4 k x 4 n.
__global__ __launch_bounds__(256) void conv2_wgrad_valu_kernel(const float* __restrict__ n1,
                                                               const float* __restrict__ da2, int S1,
                                                               int B2, int ipc, float* __restrict__ slab) {
  __shared__ float As[64 * CH];
  __shared__ float Ds[64 * CH];
  const int tid = threadIdx.x;
  const int grp = blockIdx.y, chunk = blockIdx.x, t = blockIdx.z;
  const int nchunk = gridDim.x;
  const int ky = t / KS - 2, kx = t % KS - 2;
  const int j0 = grp * B2 + chunk * ipc;
  const int j1 = min(j0 + ipc, grp * B2 + B2);
  const int np1 = S1 * S1;
  const int k0 = 4 * (tid >> 4), n0 = 4 * (tid & 15);
  float acc[4][4] = {};
  for (int j = j0; j < j1; ++j) {
    const int f = remap(j, B2);
    for (int p0 = 0; p0 < np1; p0 += 64) {
      __syncthreads();
      for (int i = tid; i < 64 * (CH / 4); i += 256) {
        const int pl = i / (CH / 4), c4 = i % (CH / 4);
        const int p = p0 + pl;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), dv = a;
        if (p < np1) {
          dv = *reinterpret_cast<const float4*>(da2 + ((size_t)j * np1 + p) * CH + 4 * c4);
          if (t == NT) {
            a = make_float4(1.f, 1.f, 1.f, 1.f);
          } else {
            const int y = p / S1 + ky, x = p % S1 + kx;
            if (y >= 0 && y < S1 && x >= 0 && x < S1)
              a = *reinterpret_cast<const float4*>(n1 + ((size_t)f * np1 + y * S1 + x) * CH + 4 * c4);
          }
        }
        *reinterpret_cast<float4*>(As + pl * CH + 4 * c4) = a;
        *reinterpret_cast<float4*>(Ds + pl * CH + 4 * c4) = dv;
      }
      __syncthreads();
#pragma unroll 4
      for (int p = 0; p < 64; ++p) {
        const float4 a = *reinterpret_cast<const float4*>(As + p * CH + k0);
        const float4 d = *reinterpret_cast<const float4*>(Ds + p * CH + n0);
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[i][0] = fmaf(av[i], d.x, acc[i][0]);
          acc[i][1] = fmaf(av[i], d.y, acc[i][1]);
          acc[i][2] = fmaf(av[i], d.z, acc[i][2]);
          acc[i][3] = fmaf(av[i], d.w, acc[i][3]);
        }
      }
    }
  }
  float* out = slab + ((size_t)grp * nchunk + chunk) * (NT * CH + 1) * CH;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (t == NT && k0 + i > 0) break;
    *reinterpret_cast<float4*>(out + (size_t)(t * CH + k0 + i) * CH + n0) =
        make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  }
}

// out_g[i] = sum_{c < nchunk} slab[g][c][i] (g = 0: g1 block, g = 1: g2 block) in a fixed
// order: workgroup = 64 consecutive i x 16 chunk lanes; lane r sums chunks r, r+16, ... and the
// 16 partials are added in lane order (deterministic; many chunks stay parallel)
__global__ __launch_bounds__(1024) void sum_slabs_kernel(const float* __restrict__ slab, int nchunk,
                                                         size_t n, float* __restrict__ out0,
                                                         float* __restrict__ out1) {
  __shared__ float part[16][64];
  const int c = threadIdx.x & 63, r = threadIdx.x >> 6;
  const size_t i = (size_t)blockIdx.x * 64 + c;
  const int g = blockIdx.y;
  float acc = 0.f;
  if (i < n) {
    const float* s = slab + (size_t)g * nchunk * n + i;
    for (int k = r; k < nchunk; k += 16) acc += s[(size_t)k * n];
  }
  part[r][c] = acc;
  __syncthreads();
  if (r == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += part[k][c];
    (g ? out1 : out0)[i] = t;
  }
}

}  // namespace

// ------------------------------------------------------------------ launchers
hipError_t launch_conv1_fwd(const ConvTower& T, const float* xs, int ldx, const float* w1, int nimg,
                            hipStream_t st) {
  const int nseg = (T.S1 + SEG_MAX - 1) / SEG_MAX;
  const int seg = (T.S1 + nseg - 1) / nseg;
  hipLaunchKernelGGL(conv1_fwd_kernel, dim3(nseg, T.S1, nimg), dim3(256), 0, st, xs, ldx, w1, T.S, seg,
                     T.p1, T.arg1, T.n1, T.n1b);
  return hipGetLastError();
}

hipError_t launch_conv2(const ConvTower& T, bool fwd, const float* in, const unsigned short* inb,
                        const float* w2, const unsigned short* w2b, float* out, int nimg, hipStream_t st) {
  if (T.mfma && inb && w2b) return launch_conv2_mfma(T, fwd, inb, w2b, w2, out, nimg, st);
  const int tiles = ((T.S1 + 7) / 8) * ((T.S1 + 7) / 8);
  if (fwd)
    hipLaunchKernelGGL(conv2_valu_kernel<true>, dim3(tiles, nimg), dim3(256), 0, st, in, w2, out, T.S1);
  else
    hipLaunchKernelGGL(conv2_valu_kernel<false>, dim3(tiles, nimg), dim3(256), 0, st, in, w2, out, T.S1);
  return hipGetLastError();
}

hipError_t launch_lrn2_pool2_fwd(const ConvTower& T, int nimg, float* xf, int ldf, int f32,
                                 const Planes& xfp, hipStream_t st) {
  const size_t waves = ((size_t)nimg * T.S2 * T.S2 + FPP - 1) / FPP;
  hipLaunchKernelGGL(lrn2_pool2_fwd_kernel, dim3(nblk(waves, 4)), dim3(256), 0, st, T.a2, T.S1, nimg, xf,
                     ldf, f32, xfp.p, xfp.stride, xfp.n, T.arg2);
  return hipGetLastError();
}

hipError_t launch_pool2_bwd(const ConvTower& T, const float* dxf, int ldf, int B, hipStream_t st) {
  const size_t waves = ((size_t)4 * B * T.S2 * T.S2 + PPW - 1) / PPW;
  hipLaunchKernelGGL(pool2_bwd_kernel, dim3(nblk(waves, 4)), dim3(256), 0, st, dxf, ldf, T.a2, T.arg2,
                     T.S1, 4 * B, 2 * B, T.da2, T.da2b);
  return hipGetLastError();
}

hipError_t launch_conv1_wgrad(const ConvTower& T, const float* xs, int ldx, int B, float* g1, float* g2,
                              hipStream_t st) {
  const int B2 = 2 * B;
  const int nchunk = T.nchunk1, ipc = (B2 + nchunk - 1) / nchunk;
  hipLaunchKernelGGL(conv1_wgrad_kernel, dim3(nchunk, 2), dim3(256), 0, st, T.dn1, T.p1, T.arg1, xs, ldx,
                     T.S, B2, ipc, T.slab);
  const size_t n = (size_t)(NT + 1) * CH;
  hipLaunchKernelGGL(sum_slabs_kernel, dim3(nblk(n, 64), 2), dim3(1024), 0, st, T.slab, nchunk, n, g1, g2);
  return hipGetLastError();
}

hipError_t launch_conv2_wgrad(const ConvTower& T, int B, float* g1, float* g2, hipStream_t st) {
  const int B2 = 2 * B;
  const size_t n = (size_t)(NT * CH + 1) * CH;
  if (T.mfma && T.n1b && T.da2b) {
    hipError_t e = launch_conv2_wgrad_mfma(T, B, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sum_slabs_kernel, dim3(nblk(n, 64), 2), dim3(1024), 0, st, T.slab, T.nchunk2m, n, g1, g2);
    return hipGetLastError();
  }
  const int nchunk = T.nchunk2, ipc = (B2 + nchunk - 1) / nchunk;
  hipLaunchKernelGGL(conv2_wgrad_valu_kernel, dim3(nchunk, 2, NT + 1), dim3(256), 0, st, T.n1, T.da2, T.S1,
                     B2, ipc, T.slab);
  hipLaunchKernelGGL(sum_slabs_kernel, dim3(nblk(n, 64), 2), dim3(1024), 0, st, T.slab, nchunk, n, g1, g2);
  return hipGetLastError();
}

}  // namespace mvae
