// Bandwidth-bound kernels of the metric-VAE step (gfx950): batch de-interleave, the
// counter-based N(0,1) sampler, reparameterisation, the latent loss head forward/backward
// (KL, deformation, cosine / squared-difference distance, training_loss), deterministic
// loss/column reductions, and the fused dual TF-Adam update.
//
// Row order of every stacked encoder buffer: [rotated lock | lock | key] (3B rows), so the
// cost gradient (rotated+lock) and the metric gradient (lock+key) each use a CONTIGUOUS
// 2B-row range. The backward stacks 4B rows: [rot(g1) | lock(g1) | lock(g2) | key(g2)].
#include "mvae_internal.h"
#include "deint_bits.h"
#include <cstdlib>

namespace mvae {
namespace {

constexpr float L2_EPS = 1e-12f;  // tf.nn.l2_normalize default

// bf16 plane images of fp32 values (operands of the bf16 / f32x GEMMs): n = 1 round to
// nearest; n = 3 exact split x = x0 + x1 + x2 (each residual an exact fp32 difference).
// Returns whether the first residual is nonzero (x not exactly representable in bf16).
__device__ __forceinline__ bool planes_put(unsigned short* p, long long ps, int n, size_t idx, float v) {
  float r = v;
  bool nz = false;
  for (int t = 0; t < n; ++t) {
    const unsigned short b = __builtin_bit_cast(unsigned short, __float2bfloat16(r));
    p[t * ps + idx] = b;
    r -= __uint_as_float((unsigned)b << 16);
    if (t == 0) nz = r != 0.f;
  }
  return nz;
}

// internal block (0 rot, 1 lock, 2 key) -> reference eps slot (0 lock, 1 rot, 2 key)
__device__ __forceinline__ int eps_slot(int blk) { return blk == 0 ? 1 : (blk == 1 ? 0 : 2); }

// ---------------------------------------------------------------- de-interleave
// x[b][p*3 + c] (c: 0 lock, 1 rotated lock, 2 key; 11a/overlap_input.py:117-119,201)
//  -> xs[(blk*B + b)][p], blk = {rot:0, lock:1, key:2}. Each thread moves 4 pixels:
// three 16-B loads, three 16-B stores (coalesced both ways).
// bf16 bits of v rounded to nearest even, and the exact remainder v - bf16(v)
__device__ __forceinline__ unsigned short bf16_rn(float v, float& rem) {
  const unsigned short b = __builtin_bit_cast(unsigned short, __float2bfloat16(v));
  rem = v - __uint_as_float((unsigned)b << 16);
  return b;
}
__device__ __forceinline__ uint2 pack4(unsigned short a, unsigned short b, unsigned short c,
                                       unsigned short d) {
  return make_uint2((unsigned)a | (unsigned)b << 16, (unsigned)c | (unsigned)d << 16);
}

// [B, D, 3] interleaved (lock, rotated, key) -> row blocks [rot | lock | key] of the layer-0
// operand: fp32 rows for the blocks in f32mask (bit c: block c; plane modes keep only the lock
// block, the BCE target) and the RN bf16 plane 0 (8-byte stores). In the exact-split mode the
// residual planes are NOT written here: the kernel only raises *dyn when some pixel is not
// exact in bf16, and residual_planes_kernel then writes planes 1 and 2 (binary shape images
// never pay for them; the GEMMs read the residual planes only when *dyn != 0).
__global__ void deinterleave_vec_kernel(const float4* __restrict__ x, float* __restrict__ xs,
                                        unsigned short* __restrict__ xp, int* __restrict__ dyn,
                                        int B, int D, int ldx, int f32mask, int* __restrict__ dyn_next) {
  // the other slot of the flags, for the next de-interleave (no per-step memset launch); this
  // form does not test for 0/1 pixels: it raises the not-binary word (dyn[2]) unconditionally
  if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) {
    if (dyn_next) dyn_next[0] = dyn_next[2] = 0;
    if (dyn) atomicOr(dyn + 2, 1);
  }
  const int b = blockIdx.y;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;  // pixel quad
  bool nz = false;
  if (q * 4 < D) {
    const float4* src = x + ((size_t)b * 3 * D) / 4 + 3 * q;
    const float4 v0 = src[0], v1 = src[1], v2 = src[2];
    // pixels p0..p3: (l,r,k) = (v0.x v0.y v0.z) (v0.w v1.x v1.y) (v1.z v1.w v2.x) (v2.y v2.z v2.w)
    const float4 vv[3] = {make_float4(v0.y, v1.x, v1.w, v2.z),   // rot
                          make_float4(v0.x, v0.w, v1.z, v2.y),   // lock
                          make_float4(v0.z, v1.y, v2.x, v2.w)};  // key
    const size_t col = 4 * (size_t)q;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t o = (size_t)(c * B + b) * ldx + col;
      if (f32mask >> c & 1) *reinterpret_cast<float4*>(xs + o) = vv[c];
      if (xp) {
        float r0, r1, r2, r3;
        const uint2 w = pack4(bf16_rn(vv[c].x, r0), bf16_rn(vv[c].y, r1), bf16_rn(vv[c].z, r2),
                              bf16_rn(vv[c].w, r3));
        *reinterpret_cast<uint2*>(xp + o) = w;
        nz |= (r0 != 0.f) | (r1 != 0.f) | (r2 != 0.f) | (r3 != 0.f);
      }
    }
  }
  if (dyn && __ballot(nz) != 0 && (threadIdx.x & 63) == 0) atomicOr(dyn, 1);
}

// 4 NQ pixels (3 NQ float4 of x in v, pixel order) of row b from column col -> the fp32 rows
// of the blocks in f32mask and bf16 plane 0 (16-B stores); returns whether a pixel is inexact
template <int NQ>
__device__ __forceinline__ bool deint_put(const float4* v, float* __restrict__ xs,
                                          unsigned short* __restrict__ xp, int B, int b,
                                          size_t col, int ldx, int f32mask) {
  static_assert(NQ % 2 == 0, "whole 16-B plane stores");
  constexpr int NP = 4 * NQ;
  bool nz = false;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int ch = c == 0 ? 1 : (c == 1 ? 0 : 2);  // block c (rot, lock, key) <- channel ch
    float f[NP];
#pragma unroll
    for (int h = 0; h < NQ; ++h) {
      const float4 a = v[3 * h], bb = v[3 * h + 1], cc = v[3 * h + 2];
      const float e[12] = {a.x, a.y, a.z, a.w, bb.x, bb.y, bb.z, bb.w, cc.x, cc.y, cc.z, cc.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) f[4 * h + j] = e[3 * j + ch];
    }
    const size_t o = (size_t)(c * B + b) * ldx + col;
    if (f32mask >> c & 1) {
#pragma unroll
      for (int h = 0; h < NQ; ++h)
        *reinterpret_cast<float4*>(xs + o + 4 * h) = make_float4(f[4 * h], f[4 * h + 1], f[4 * h + 2], f[4 * h + 3]);
    }
    if (xp) {
#pragma unroll
      for (int h = 0; h < NQ; h += 2) {
        float r[8];
        unsigned short h16[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) h16[j] = bf16_rn(f[4 * h + j], r[j]);
        const uint2 lo = pack4(h16[0], h16[1], h16[2], h16[3]), hi = pack4(h16[4], h16[5], h16[6], h16[7]);
        *reinterpret_cast<uint4*>(xp + o + 4 * h) = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
        for (int j = 0; j < 8; ++j) nz |= r[j] != 0.f;
      }
    }
  }
  return nz;
}

// The same for 4 NQ pixels per thread (D % (4 NQ) == 0): 3 NQ 16-B loads (48 NQ contiguous
// bytes) issued together, then per block NQ / 2 16-B plane stores. 8 pixels per thread measured
// 0.305 -> 0.287 ms at C3 (profiles/r4/r4y_deinterleave.txt)
template <int NQ>
__global__ void deinterleave_vecn_kernel(const float4* __restrict__ x, float* __restrict__ xs,
                                         unsigned short* __restrict__ xp, int* __restrict__ dyn,
                                         int B, int D, int ldx, int f32mask, int* __restrict__ dyn_next,
                                         unsigned char* __restrict__ xbits, int ldbits) {
  // the other slot of the flags, for the next de-interleave (no per-step memset launch)
  if (dyn_next && (blockIdx.x | blockIdx.y | threadIdx.x) == 0) dyn_next[0] = dyn_next[2] = 0;
  constexpr int NP = 4 * NQ;  // pixels per thread
  const int b = blockIdx.y;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  bool nz = false, nb = false;
  if (q * NP < D) {
    const float4* src = x + ((size_t)b * 3 * D) / 4 + 3 * NQ * q;
    float4 v[3 * NQ];
#pragma unroll
    for (int i = 0; i < 3 * NQ; ++i) v[i] = src[i];
    // some value of the three channels neither 0 nor 1 (the BCE target is one of them)
#pragma unroll
    for (int i = 0; i < 3 * NQ; ++i) {
      const float e[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) nb |= (e[j] != 0.f) & (e[j] != 1.f);
    }
    nz = deint_put<NQ>(v, xs, xp, B, b, (size_t)NP * q, ldx, f32mask);
    if (xbits) {  // the lock channel (element 3 j of pixel j) as bits, 8 pixels per byte
      static_assert(NQ == 2, "one byte per thread");
      const float e[24] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                           v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w,
                           v[4].x, v[4].y, v[4].z, v[4].w, v[5].x, v[5].y, v[5].z, v[5].w};
      unsigned byte = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) byte |= (e[3 * j] != 0.f ? 1u : 0u) << j;
      xbits[(size_t)b * ldbits + q] = (unsigned char)byte;
    }
  }
  if (dyn) {  // (the ballots with every lane of the wave active)
    const bool anz = __ballot(nz) != 0, anb = __ballot(nb) != 0;
    if ((threadIdx.x & 63) == 0) {
      if (anz) atomicOr(dyn, 1);
      if (anb) atomicOr(dyn + 2, 1);
    }
  }
}

// (diagnostics) persistent form: gridDim.x workgroups stride over the B x D/8 pixel groups
__global__ void deinterleave_persist_kernel(const float4* __restrict__ x, unsigned short* __restrict__ xp,
                                            int B, int D, int ldx) {
  const int nq = D / 8;
  const size_t n = (size_t)B * nq;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / nq), q = (int)(i % nq);
    const float4* src = x + ((size_t)b * 3 * D) / 4 + 6 * (size_t)q;
    float4 v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = src[k];
    deint_put<2>(v, nullptr, xp, B, b, (size_t)8 * q, ldx, 0);
  }
}

__global__ void deinterleave_scalar_kernel(const float* __restrict__ x, float* __restrict__ xs,
                                           unsigned short* __restrict__ xp, int* __restrict__ dyn,
                                           int B, int D, int ldx, int f32mask, int* __restrict__ dyn_next) {
  // the other slot of the flags (see deinterleave_vec_kernel: no 0/1 test here)
  if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) {
    if (dyn_next) dyn_next[0] = dyn_next[2] = 0;
    if (dyn) atomicOr(dyn + 2, 1);
  }
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  bool nz = false;
  if (p < D) {
    const float* src = x + (size_t)b * 3 * D + 3 * (size_t)p;
    const float v[3] = {src[1], src[0], src[2]};  // rot, lock, key
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t o = (size_t)(c * B + b) * ldx + p;
      if (f32mask >> c & 1) xs[o] = v[c];
      if (xp) {
        float r;
        xp[o] = bf16_rn(v[c], r);
        nz |= r != 0.f;
      }
    }
  }
  if (dyn && __ballot(nz) != 0 && (threadIdx.x & 63) == 0) atomicOr(dyn, 1);
}

// Only when *dyn != 0 (some pixel of the batch is not a bf16 value): planes 1 and 2 of the
// exact split of the layer-0 operand (3-plane mode), and the fp32 rows of the blocks in
// f32mask (the BCE target, read from bf16 plane 0 while every pixel is exact).
__global__ void residual_planes_kernel(const float* __restrict__ x, float* __restrict__ xs,
                                       unsigned short* __restrict__ xp, long long ps, int np,
                                       int f32mask, const int* __restrict__ dyn, int B, int D,
                                       int ldx) {
  if (*dyn == 0) return;
  const size_t n = (size_t)B * D;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t b = i / D, p = i - b * D;
    const float* src = x + b * 3 * D + 3 * p;
    const float v[3] = {src[1], src[0], src[2]};  // rot, lock, key
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t o = (size_t)(c * B + b) * ldx + p;
      if (f32mask >> c & 1) xs[o] = v[c];
      if (np == 3) {
        float r1, r2, r3;
        (void)bf16_rn(v[c], r1);
        xp[ps + o] = bf16_rn(r1, r2);
        xp[2 * ps + o] = bf16_rn(r2, r3);
      }
    }
  }
}

// ---------------------------------------------------------------- N(0,1) sampler
// Philox4x32-10 counter-based generator + Box-Muller; element i of call `counter` depends
// only on (seed, counter, i): reproducible and independent of the launch geometry.
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = l1; c[2] = n2; c[3] = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// The 4 normals of Philox block q of call `counter`: global elements 4q .. 4q+3 of the stream
// (Box-Muller on the block's two 32-bit pairs). The sampler kernel and the fused latent kernels
// (which regenerate eps in registers instead of reading it) share this code, so a regenerated
// value is bit-identical to the sampled one. Hardware transcendentals (v_log_f32 = log2,
// v_sin/cos_f32 of 2*pi*x, v_sqrt_f32; ~1 ulp): the latent kernels regenerate 3*B*L normals in
// the forward and again in the backward, and the accurate libm forms made them VALU-bound.
__device__ __forceinline__ void normal4(uint64_t q, uint64_t seed, uint64_t counter, float (&r)[4]) {
  uint32_t c[4] = {(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)counter, (uint32_t)(counter >> 32)};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float inv = 2.3283064365386963e-10f;  // 2^-32
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float u1 = __fmul_rn(__fadd_rn((float)c[2 * j], 0.5f), inv);  // (0,1)
    const float u2 = __fmul_rn(__fadd_rn((float)c[2 * j + 1], 0.5f), inv);
    // -2 ln u1 = -2 ln2 log2 u1
    const float rad = __builtin_amdgcn_sqrtf(__fmul_rn(-1.3862943611198906f, __builtin_amdgcn_logf(u1)));
    r[2 * j] = __fmul_rn(rad, __builtin_amdgcn_cosf(u2));      // cos(2 pi u2)
    r[2 * j + 1] = __fmul_rn(rad, __builtin_amdgcn_sinf(u2));  // sin(2 pi u2)
  }
}

// One Philox block per thread -> 4 normals at consecutive GLOBAL element indices. With a
// row-sharded batch the rank's elements of slot s (blockIdx.y) are the contiguous global range
// [(s*Bg + off)*L, +B*L): a data-parallel rank draws exactly its slice of the eps the single
// process would draw for the global batch (off = 0, Bg = B: the plain contiguous stream).
__global__ void normal_kernel(float* __restrict__ out, int B, int L, int Bg, int off, uint64_t seed,
                              uint64_t counter) {
  const size_t n = (size_t)B * L;
  const size_t g0 = ((size_t)blockIdx.y * Bg + off) * L;  // first global element of this slot
  const size_t q = g0 / 4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // Philox block
  if (4 * q >= g0 + n) return;
  float r[4];
  normal4(q, seed, counter, r);
  float* o = out + (size_t)blockIdx.y * n;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t e = 4 * q + j;
    if (e >= g0 && e < g0 + n) o[e - g0] = r[j];
  }
}

// ---------------------------------------------------------------- fused latent head
// eps of the reparameterisation (11a/vae.py:373): the [3][B][L] buffer (given by the caller),
// or the training / inference Philox stream regenerated in registers (internal draws: no eps
// buffer is written or read; mvae_buffer(MVAE_BUF_EPS) materialises it on demand).
struct EpsSrc {
  const float* buf;   // nullptr: regenerate
  uint64_t seed, counter;
  int Bg, off;        // global batch and this rank's first row (the sharded stream)
};

// eps of (internal block blk, row b, columns i .. i+3); V4: L % 4 == 0 and i % 4 == 0, so the
// four elements are exactly one Philox block
template <bool V4>
__device__ __forceinline__ void eps_get(const EpsSrc& es, int blk, int b, int i, int B, int L,
                                        float (&e)[4]) {
  const int sl = eps_slot(blk);
  if (es.buf) {
    const float* p = es.buf + ((size_t)sl * B + b) * L + i;
    if constexpr (V4) {
      const float4 v = *reinterpret_cast<const float4*>(p);
      e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
    } else {
      e[0] = p[0];
    }
    return;
  }
  const size_t g = ((size_t)sl * es.Bg + es.off + b) * L + i;  // global element
  if constexpr (V4) {
    normal4(g >> 2, es.seed, es.counter, e);
  } else {
    float r[4];
    normal4(g >> 2, es.seed, es.counter, r);
    e[0] = r[g & 3];
  }
}

// sigma = sqrt(exp(s)) = exp2(s log2(e) / 2) on v_exp_f32, and z = mu + sigma * eps
// (11a/vae.py:371-377): one explicit rounding sequence shared by the forward and the backward
// (which recomputes z instead of reading it)
__device__ __forceinline__ float sigma_of(float s) {
  return __builtin_amdgcn_exp2f(__fmul_rn(s, 0.72134752044448170f));
}
__device__ __forceinline__ float reparam(float mu, float s, float e) {
  return __fadd_rn(mu, __fmul_rn(sigma_of(s), e));
}

__device__ __forceinline__ void ld4(const float* p, float (&v)[4]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
// 4 values -> n bf16 planes at p[t*ps + o .. +3] (8-B stores; o % 4 == 0)
__device__ __forceinline__ void planes_put4(unsigned short* p, long long ps, int n, size_t o,
                                            const float (&v)[4]) {
  float r[4] = {v[0], v[1], v[2], v[3]};
  for (int t = 0; t < n; ++t) {
    unsigned short q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q[j] = __builtin_bit_cast(unsigned short, __float2bfloat16(r[j]));
      r[j] -= __uint_as_float((unsigned)q[j] << 16);
    }
    *reinterpret_cast<uint2*>(p + t * ps + o) = pack4(q[0], q[1], q[2], q[3]);
  }
}

// Forward of the latent head, one wave per batch row b (V4: 4 columns per lane): mu / s of the
// three passes (ms rows [mu | s], 2L wide) and eps -> z, written only where something reads it
// (zmask bit 1: fp32 lock row, for fp32 decoder GEMMs and the cosine statistics; bit 2: fp32 key
// row, cosine only; the lock row's bf16 planes for the plane-mode decoder GEMMs), and the row
// sums rowfwd[b] = {sum(1 + s - mu^2 - exp s) (KL, lock pass, :281-284), sum (z_lock - z_rot)^2
// (deformation, :293-294), sum (z_lock - z_key)^2 (squared-difference distance, :309)}.
// WPR waves per row: 1 (four rows per 256-thread workgroup) or 4 (one long row per workgroup,
// the four waves' sums combined through LDS in a fixed order), so a 2000-wide row keeps enough
// loads in flight.
template <bool V4, int WPR>
__global__ void latent_fwd_kernel(const float* __restrict__ ms, EpsSrc es, float* __restrict__ z,
                                  unsigned short* __restrict__ zp, long long ps, int np, int zmask,
                                  int B, int L, int ldz, float* __restrict__ rowfwd) {
  const int lane = threadIdx.x & 63;
  const int wr = (threadIdx.x >> 6) % WPR;  // wave within the row
  const int b = blockIdx.x * (4 / WPR) + (threadIdx.x >> 6) / WPR;
  __shared__ float red[4][3];
  if (WPR == 1 && b >= B) return;
  constexpr int W = V4 ? 4 : 1;
  float kl = 0.f, fd = 0.f, sq = 0.f;
  for (int i = W * (lane + 64 * wr); i < L; i += 64 * W * WPR) {
    float zz[3][4], mul[4], sl[4];
#pragma unroll
    for (int blk = 0; blk < 3; ++blk) {
      const float* row = ms + (size_t)(blk * B + b) * 2 * L;
      float mu[4], sg[4], e[4];
      if constexpr (V4) { ld4(row + i, mu); ld4(row + L + i, sg); }
      else { mu[0] = row[i]; sg[0] = row[L + i]; }
      eps_get<V4>(es, blk, b, i, B, L, e);
#pragma unroll
      for (int j = 0; j < W; ++j) zz[blk][j] = reparam(mu[j], sg[j], e[j]);
      if (blk == 1) {
#pragma unroll
        for (int j = 0; j < W; ++j) { mul[j] = mu[j]; sl[j] = sg[j]; }
      }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
      kl += 1.f + sl[j] - mul[j] * mul[j] - __expf(sl[j]);
      const float d = zz[1][j] - zz[0][j], q = zz[1][j] - zz[2][j];
      fd += d * d;
      sq += q * q;
    }
    const size_t ol = (size_t)(B + b) * ldz + i, ok = (size_t)(2 * B + b) * ldz + i;
    if constexpr (V4) {
      if (zmask & 2) *reinterpret_cast<float4*>(z + ol) = make_float4(zz[1][0], zz[1][1], zz[1][2], zz[1][3]);
      if (zmask & 4) *reinterpret_cast<float4*>(z + ok) = make_float4(zz[2][0], zz[2][1], zz[2][2], zz[2][3]);
      if (zp) planes_put4(zp, ps, np, ol, zz[1]);
    } else {
      if (zmask & 2) z[ol] = zz[1][0];
      if (zmask & 4) z[ok] = zz[2][0];
      if (zp) planes_put(zp, ps, np, ol, zz[1][0]);
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    kl += __shfl_xor(kl, off, 64);
    fd += __shfl_xor(fd, off, 64);
    sq += __shfl_xor(sq, off, 64);
  }
  if constexpr (WPR == 1) {
    if (lane == 0) *reinterpret_cast<float4*>(rowfwd + 4 * (size_t)b) = make_float4(kl, fd, sq, 0.f);
  } else {
    if (lane == 0) { red[wr][0] = kl; red[wr][1] = fd; red[wr][2] = sq; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float t[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) t[q] = ((red[0][q] + red[1][q]) + red[2][q]) + red[3][q];
      *reinterpret_cast<float4*>(rowfwd + 4 * (size_t)b) = make_float4(t[0], t[1], t[2], 0.f);
    }
  }
}

// ---------------------------------------------------------------- column statistics
// mode 0 (colsq):  out[j] = sum_b z_lock[b][j]^2 (j < L), sum_b z_key[b][j-L]^2 (j >= L)
// mode 1 (coldot): out[i] = sum_b draw_b * n_lock[b][i] * n_key[b][i]
// Two-stage, fixed-order (deterministic): partials over row chunks, then chunk sums.
// Column statistics of the cosine metric in two fixed-order passes: chunk partials of CS_ROWS
// rows (4 row lanes x CS_ROWS / 4 rows each, their loads issued before the ordered sum), then
// the ordered sum over chunks. (With 128-row chunks every thread waited out 32 dependent
// global loads in a row and the final pass another nchunk: 20-30 us per statistic for a few
// hundred KB.)
// 128-row chunks: 32-row ones left the final pass 256 dependent partials per column at C3
// (colsq + coldot 36.5 -> 23.6 us, profiles/r4/r4aj_colstats.txt)
constexpr int CS_ROWS = 128;
constexpr int CS_PER = CS_ROWS / 4;  // rows per thread

// cnt (one launch): the partials written through (sc1) and counted per column block by an
// agent-scope add after every storing wave's vmcnt(0); the block whose add comes last sums the
// column block's partials in chunk order by sc1 loads -- colstats_final_kernel's order, so the
// same bits -- and resets the counter (MI355X_MICROARCH.md's sc1 hand-off, first row)
__global__ void colstats_part_kernel(int mode, const float* __restrict__ z, int B, int L, int ldz,
                                     const float* __restrict__ colsq, const float* __restrict__ draw,
                                     float* __restrict__ part, int* __restrict__ cnt, float* __restrict__ out) {
  const int ncols = mode == 0 ? 2 * L : L;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 cols x 4 row lanes
  const int j = blockIdx.x * 64 + tx;
  const int r0 = blockIdx.y * CS_ROWS;
  __shared__ float red[4][64];
  float acc = 0.f;
  if (j < ncols) {
    if (mode == 0) {
      const float* src = j < L ? z + (size_t)B * ldz + j : z + (size_t)2 * B * ldz + (j - L);
      float v[CS_PER];
#pragma unroll
      for (int i = 0; i < CS_PER; ++i) {
        const int b = r0 + ty + 4 * i;
        v[i] = b < B ? src[(size_t)b * ldz] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < CS_PER; ++i) acc += v[i] * v[i];
    } else {
      const float rl = rsqrtf(fmaxf(colsq[j], L2_EPS));
      const float rk = rsqrtf(fmaxf(colsq[L + j], L2_EPS));
      float zl[CS_PER], zk[CS_PER], dr[CS_PER];
#pragma unroll
      for (int i = 0; i < CS_PER; ++i) {
        const int b = r0 + ty + 4 * i;
        const bool ok = b < B;
        zl[i] = ok ? z[(size_t)(B + b) * ldz + j] : 0.f;
        zk[i] = ok ? z[(size_t)(2 * B + b) * ldz + j] : 0.f;
        dr[i] = ok ? draw[b] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < CS_PER; ++i) acc += dr[i] * (zl[i] * rl) * (zk[i] * rk);
    }
  }
  red[ty][tx] = acc;
  __syncthreads();
  const float v = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
  if (!cnt) {
    if (ty == 0 && j < ncols) part[(size_t)blockIdx.y * ncols + j] = v;
    return;
  }
  if (ty == 0 && j < ncols) __hip_atomic_store(part + (size_t)blockIdx.y * ncols + j, v, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(cnt + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (int)gridDim.y - 1;
  __syncthreads();
  if (!last) return;
  // every row lane loads a quarter of each 64-chunk group (one round of load latency), row lane 0
  // sums the column in chunk order (colstats_final_kernel's order: the same bits)
  __shared__ float stage[64][64];
  const int nchunk = gridDim.y;
  float a = 0.f;
  for (int c0 = 0; c0 < nchunk; c0 += 64) {
    const int n = min(64, nchunk - c0);
    if (j < ncols) {
      float t[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = ty + 4 * i;
        t[i] = c < n ? __hip_atomic_load(part + (size_t)(c0 + c) * ncols + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) stage[ty + 4 * i][tx] = t[i];
    }
    __syncthreads();
    if (ty == 0 && j < ncols)
      for (int c = 0; c < n; ++c) a += stage[c][tx];
    __syncthreads();
  }
  if (ty == 0 && j < ncols) out[j] = a;
  if (threadIdx.x == 0) cnt[blockIdx.x] = 0;  // (the next launch is ordered behind this one)
}

__global__ void colstats_final_kernel(const float* __restrict__ part, int nchunk, int ncols,
                                      float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ncols) return;
  float acc = 0.f;
  int c = 0;
  for (; c + 8 <= nchunk; c += 8) {  // 8 loads in flight, summed in chunk order
    float t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = part[(size_t)(c + i) * ncols + j];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += t[i];
  }
  for (; c < nchunk; ++c) acc += part[(size_t)c * ncols + j];
  out[j] = acc;
}

// ---------------------------------------------------------------- metric / losses per row
// One wave per batch row b. rowvals[b] = {R_b, K_b, F_b, T_b}; dist[b]; draw[b] = dT/draw_b.
//   R_b: BCE row partials from the decoder-output GEMM epilogue (11a/vae.py:266-269)
//   K_b = -0.5 sum(1 + s - mu^2 - exp(s)), F_b = w sum (z_lock - z_rot)^2: the fused latent
//         forward's row sums (rowfwd, :281-284, :293-294)
//   dist_b: sum (z_lock - z_key)^2 (rowfwd) or cosine (axis-0 l2_normalize, :444-458, from the
//         fp32 lock / key rows and the column sums of squares); 1/raw if recip
//   T_b = (dist_b - area_b)^2                         (:313)
__global__ void metric_kernel(const float* __restrict__ z, int ldz, const float* __restrict__ rowfwd,
                              const float* __restrict__ rowpart, int nblk,
                              const float* __restrict__ areas, const float* __restrict__ colsq,
                              int B, int L, int metric, int recip, float w, float inv_bg,
                              float* __restrict__ rowvals, float* __restrict__ dist,
                              float* __restrict__ draw) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* zl = z + (size_t)(B + b) * ldz;
  const float* zk = z + (size_t)(2 * B + b) * ldz;
  float raw = 0.f, rp = 0.f;
  if (metric == 0) {
    auto term = [&](float l, float k, int i) {
      const float rl = rsqrtf(fmaxf(colsq[i], L2_EPS));
      const float rk = rsqrtf(fmaxf(colsq[L + i], L2_EPS));
      raw += (l * rl) * (k * rk);
    };
    if ((L & 3) == 0 && L >= 64 && (ldz & 3) == 0) {  // 16-B loads, 4 elements per lane
      for (int i = 4 * lane; i < L; i += 256) {
        const float4 l = *reinterpret_cast<const float4*>(zl + i);
        const float4 k = *reinterpret_cast<const float4*>(zk + i);
        term(l.x, k.x, i);
        term(l.y, k.y, i + 1);
        term(l.z, k.z, i + 2);
        term(l.w, k.w, i + 3);
      }
    } else {
      for (int i = lane; i < L; i += 64) term(zl[i], zk[i], i);
    }
  }
  for (int j = lane; j < nblk; j += 64) rp += rowpart[(size_t)b * nblk + j];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    raw += __shfl_xor(raw, off, 64);
    rp += __shfl_xor(rp, off, 64);
  }
  if (lane == 0) {
    const float4 f = *reinterpret_cast<const float4*>(rowfwd + 4 * (size_t)b);
    if (metric == 1) raw = f.z;
    const float dv = recip ? 1.f / raw : raw;
    const float a = areas ? areas[b] : 0.f;
    const float g = 2.f * (dv - a) * inv_bg;
    rowvals[4 * (size_t)b + 0] = rp;
    rowvals[4 * (size_t)b + 1] = -0.5f * f.x;
    rowvals[4 * (size_t)b + 2] = w * f.y;
    rowvals[4 * (size_t)b + 3] = (dv - a) * (dv - a);
    dist[b] = dv;
    draw[b] = recip ? -g * dv * dv : g;  // tf.reciprocal grad: -dy * y^2
  }
}

// single block, fixed-order: losses = {cost, training_loss, r_l, l_l, d_l} (local sums / B_global)
__global__ void loss_reduce_kernel(const float* __restrict__ rowvals, int B, float inv_bg,
                                   float* __restrict__ losses) {
  __shared__ float red[4][256];
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  // rows tid, tid + 256, ... in order; 8 rows' 16-B loads issued before their sums
  const float4* rv = reinterpret_cast<const float4*>(rowvals);
  int b = threadIdx.x;
  for (; b + 7 * 256 < B; b += 8 * 256) {
    float4 t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = rv[b + 256 * i];
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[0] += t[i].x; a[1] += t[i].y; a[2] += t[i].z; a[3] += t[i].w; }
  }
  for (; b < B; b += 256) {
    const float4 t = rv[b];
    a[0] += t.x; a[1] += t.y; a[2] += t.z; a[3] += t.w;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[q][threadIdx.x] = a[q];
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s) {
#pragma unroll
      for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float R = red[0][0] * inv_bg, K = red[1][0] * inv_bg, F = red[2][0] * inv_bg;
    losses[0] = R + K + F;
    losses[1] = red[3][0] * inv_bg;
    losses[2] = R;
    losses[3] = K;
    losses[4] = F;
  }
}

// ---------------------------------------------------------------- latent head backward
// dhead rows (4B): [rot:g1 | lock:g1 | lock:g2 | key:g2], cols [dmu (L) | ds (L)]
//   g1: dz_rot = -2w(zl-zr)/B ; dz_lock = dz_dec + 2w(zl-zr)/B, + KL: dmu += mu/B,
//       ds += 0.5(exp(s)-1)/B
//   g2: sqdiff: dz_lock = 2 draw (zl-zk) = -dz_key
//       cosine: dz = r (draw n_other - n c), c = coldot (summed over the global batch),
//               the n*c term only where sum z^2 >= 1e-12 (tf.maximum routes the gradient)
//   reparameterisation: dmu = dz, ds = 0.5 dz eps sigma
// One thread per (pair b, W consecutive latent elements): the four backward rows from one
// read of the three passes' mu / s and dz_dec; z and eps are recomputed exactly as the forward
// produced them (reparam, eps_get), so neither is read from memory.
template <bool V4>
__global__ void latent_bwd_kernel(const float* __restrict__ ms, EpsSrc es,
                                  const float* __restrict__ dzdec, const float* __restrict__ draw,
                                  const float* __restrict__ colsq, const float* __restrict__ coldot,
                                  int B, int L, int metric, float w, float inv_bg,
                                  float* __restrict__ dhead, int ldh,
                                  unsigned short* __restrict__ hp, long long ps, int np) {
  constexpr int W = V4 ? 4 : 1;
  const int LW = L / W;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * LW) return;
  const int b = (int)(idx / LW), i = W * (int)(idx - (size_t)b * LW);
  float mu[3][4], sg[3][4], e[3][4], dd[4];
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    const float* row = ms + (size_t)(blk * B + b) * 2 * L;
    if constexpr (V4) { ld4(row + i, mu[blk]); ld4(row + L + i, sg[blk]); }
    else { mu[blk][0] = row[i]; sg[blk][0] = row[L + i]; }
    eps_get<V4>(es, blk, b, i, B, L, e[blk]);
  }
  if constexpr (V4) ld4(dzdec + (size_t)b * L + i, dd);
  else dd[0] = dzdec[(size_t)b * L + i];
  const float dr = draw[b];
  float out[4][2][4];  // [row q][dmu | ds][element]
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const float zr = reparam(mu[0][j], sg[0][j], e[0][j]);
    const float zl = reparam(mu[1][j], sg[1][j], e[1][j]);
    const float zk = reparam(mu[2][j], sg[2][j], e[2][j]);
    const float ex_l = __expf(sg[1][j]);
    const float sig_r = sigma_of(sg[0][j]), sig_l = sigma_of(sg[1][j]), sig_k = sigma_of(sg[2][j]);
    const float def = 2.f * w * (zl - zr) * inv_bg;
    float dz2, dz3;  // g2 rows: lock, key
    if (metric == 1) {
      dz2 = 2.f * dr * (zl - zk);
      dz3 = -dz2;
    } else {
      const float ssl = colsq[i + j], ssk = colsq[L + i + j];
      const float rl = rsqrtf(fmaxf(ssl, L2_EPS)), rk = rsqrtf(fmaxf(ssk, L2_EPS));
      const float nl = zl * rl, nk = zk * rk, c = coldot[i + j];
      dz2 = rl * (dr * nk - (ssl >= L2_EPS ? nl * c : 0.f));
      dz3 = rk * (dr * nl - (ssk >= L2_EPS ? nk * c : 0.f));
    }
    const float dz1 = dd[j] + def;
    out[0][0][j] = -def;
    out[1][0][j] = dz1 + mu[1][j] * inv_bg;
    out[2][0][j] = dz2;
    out[3][0][j] = dz3;
    out[0][1][j] = -0.5f * def * e[0][j] * sig_r;
    out[1][1][j] = 0.5f * dz1 * e[1][j] * sig_l + 0.5f * (ex_l - 1.f) * inv_bg;
    out[2][1][j] = 0.5f * dz2 * e[1][j] * sig_l;
    out[3][1][j] = 0.5f * dz3 * e[2][j] * sig_k;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const size_t o = (size_t)(q * B + b) * ldh + h * L + i;
      if constexpr (V4) {
        if (dhead) *reinterpret_cast<float4*>(dhead + o) = make_float4(out[q][h][0], out[q][h][1], out[q][h][2], out[q][h][3]);
        if (hp) planes_put4(hp, ps, np, o, out[q][h]);
      } else {
        if (dhead) dhead[o] = out[q][h][0];
        if (hp) planes_put(hp, ps, np, o, out[q][h][0]);
      }
    }
}

// ---------------------------------------------------------------- dual TF-Adam
// opt1 (lr1, g1) over every trained variable, opt2 (lr2, g2) over the encoder slice;
// both from the pre-step gradients: theta = (theta - d1) - d2.  lr_t precomputed on the
// host in fp32 exactly as TF ApplyAdam (lr*sqrt(1-b2^t)/(1-b1^t) with fp32 beta powers).
template <bool NT>
__device__ __forceinline__ void st_f(float* p, float v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT>
__global__ void adam_kernel(AdamArgs a) {
  const size_t i = a.i0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.i1) return;
  float th = a.theta[i];
  {
    const float g = a.g1[i];
    float m = a.m1[i], v = a.v1[i];
    m += (g - m) * (1.f - a.b1);
    v += (g * g - v) * (1.f - a.b2);
    st_f<NT>(a.m1 + i, m); st_f<NT>(a.v1 + i, v);
    th -= (a.lr1 * m) / (sqrtf(v) + a.eps);
  }
  if (i < a.n_enc) {
    const float g = a.g2[i];
    float m = a.m2[i], v = a.v2[i];
    m += (g - m) * (1.f - a.b1);
    v += (g * g - v) * (1.f - a.b2);
    st_f<NT>(a.m2 + i, m); st_f<NT>(a.v2 + i, v);
    th -= (a.lr2 * m) / (sqrtf(v) + a.eps);
  }
  st_f<NT>(a.theta + i, th);
  if (a.tp.p) planes_put(a.tp.p, a.tp.stride, a.tp.n, i, th);
}

__global__ void split_planes_kernel(const float* __restrict__ s, size_t n, unsigned short* p,
                                    long long ps, int np) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) planes_put(p, ps, np, i, s[i]);
}

__global__ void copy2d_kernel(const float* __restrict__ s, int lds, float* __restrict__ d, int ldd,
                              int rows, int cols) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)rows * cols) return;
  const int r = (int)(idx / cols), c = (int)(idx - (size_t)r * cols);
  d[(size_t)r * ldd + c] = s[(size_t)r * lds + c];
}

// ---------------------------------------------------------------- batch producer
// The reference's input pipeline for one batch (11a/overlap_input.py:127-261): lock and key
// images from uint8 tables, the lock rotated by tf.contrib.image.rotate semantics (output
// (x,y) samples ((c*x - s*y) + x_off, (s*x + c*y) + y_off), NEAREST = roundf, zero fill;
// per-example coefficients precomputed in fp32 on the host), concatenated per pixel as
// (lock, rotated, key) and divided by 255 -> X [B, H*W*3]. No FMA contraction, so the
// gather indices match the host restatement bit for bit (hipcc contracts even the *_rn
// intrinsics into FMAs unless contraction is off: a few pixels per batch then sampled a
// neighbour; caught by tests/test_input_pipeline.py's grey-value tables).
__global__ void make_batch_kernel(const unsigned char* __restrict__ locks,
                                  const unsigned char* __restrict__ keys, int H, int W,
                                  const int* __restrict__ idx, const float4* __restrict__ coef,
                                  float div, float* __restrict__ x) {
#pragma clang fp contract(off)  // (the *_rn intrinsics do not prevent it: their bodies are outside)
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int HW = H * W;
  if (p >= HW) return;
  const int id = idx[b];
  const float4 cf = coef[b];
  const int yy = p / W, xx = p - yy * W;
  const float fx = (float)xx, fy = (float)yy;
  const float xin = (cf.x * fx - cf.y * fy) + cf.z;  // unfused: fp contract(off) above
  const float yin = (cf.y * fx + cf.x * fy) + cf.w;
  const float xr = roundf(xin), yr = roundf(yin);
  const unsigned char* L = locks + (size_t)id * HW;
  float rot = 0.f;
  if (xr >= 0.f && xr <= (float)(W - 1) && yr >= 0.f && yr <= (float)(H - 1))
    rot = (float)L[(int)yr * W + (int)xr];
  float* o = x + (size_t)b * 3 * HW + 3 * (size_t)p;
  o[0] = (float)L[p] / div;
  o[1] = rot / div;
  o[2] = (float)keys[(size_t)id * HW + p] / div;
}

// The same batch (bit for bit) at 4 pixels per thread for H*W % 4 == 0 and a 16-B aligned x:
// one 4-B load each of the lock and key bytes, the 12 output floats of a thread written to LDS,
// and the workgroup's 1024-pixel segment of the output row (12 KB, contiguous in x) stored back
// with 16-B stores that are contiguous across each wave (3 per thread). The per-pixel store of
// make_batch_kernel (three 4-B stores at a 12-B lane stride) ran at ~2.1-2.5 TB/s.
constexpr int MB_PIX = 4 * 256;  // pixels per workgroup
__global__ __launch_bounds__(256) void make_batch4_kernel(const unsigned char* __restrict__ locks,
                                                          const unsigned char* __restrict__ keys, int H,
                                                          int W, const int* __restrict__ idx,
                                                          const float4* __restrict__ coef, float div,
                                                          float* __restrict__ x) {
#pragma clang fp contract(off)  // as make_batch_kernel: the coordinates are unfused mul / add / sub
  __shared__ __attribute__((aligned(16))) float seg[3 * MB_PIX];
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int HW = H * W;
  const int s0 = blockIdx.x * MB_PIX;  // first pixel of the segment
  const int p0 = s0 + 4 * tid;
  const int id = idx[b];
  const float4 cf = coef[b];
  const unsigned char* L = locks + (size_t)id * HW;
  if (p0 < HW) {
    const uchar4 lv = *reinterpret_cast<const uchar4*>(L + p0);
    const uchar4 kv = *reinterpret_cast<const uchar4*>(keys + (size_t)id * HW + p0);
    const unsigned char l[4] = {lv.x, lv.y, lv.z, lv.w}, k[4] = {kv.x, kv.y, kv.z, kv.w};
    float v[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 + j;
      const int yy = p / W, xx = p - yy * W;
      const float fx = (float)xx, fy = (float)yy;
      const float xin = (cf.x * fx - cf.y * fy) + cf.z;  // unfused: fp contract(off) above
      const float yin = (cf.y * fx + cf.x * fy) + cf.w;
      const float xr = roundf(xin), yr = roundf(yin);
      float rot = 0.f;
      if (xr >= 0.f && xr <= (float)(W - 1) && yr >= 0.f && yr <= (float)(H - 1))
        rot = (float)L[(int)yr * W + (int)xr];
      v[3 * j] = (float)l[j] / div;
      v[3 * j + 1] = rot / div;
      v[3 * j + 2] = (float)k[j] / div;
    }
    float4* d = reinterpret_cast<float4*>(seg + 12 * tid);
    d[0] = make_float4(v[0], v[1], v[2], v[3]);
    d[1] = make_float4(v[4], v[5], v[6], v[7]);
    d[2] = make_float4(v[8], v[9], v[10], v[11]);
  }
  __syncthreads();
  const int nf = 3 * min(MB_PIX, HW - s0);  // floats of this segment (a multiple of 12)
  float4* o = reinterpret_cast<float4*>(x + (size_t)b * 3 * HW + 3 * (size_t)s0);
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int f = 4 * (tid + 256 * s);
    if (f < nf) o[tid + 256 * s] = *reinterpret_cast<const float4*>(seg + f);
  }
}

// ---------------------------------------------------------------- de-interleave to bits
// The layer-0 pixel operand of a 0/1 batch as BitMats (deint_bits.h): one workgroup per task of
// 64 batch rows x 64 PB pixels. Raises the not-binary word (*dyn slot 2) when a pixel is neither 0
// nor 1: the step then runs deint_grey_kernel (the planes) and the GEMMs read the planes.
template <int PB, int NT, int OS, bool NTL = false, bool NOW = false, bool CO = false>
__global__ __launch_bounds__(NT) void deint_bits_kernel(const float4* __restrict__ x, int B, int D, int kts_f,
                                                        int kts_w, unsigned* __restrict__ xbf,
                                                        unsigned* __restrict__ xbw,
                                                        unsigned char* __restrict__ xbits, int ldbits,
                                                        int* __restrict__ dyn, int* __restrict__ dyn_next) {
  if (dyn_next && (blockIdx.x | blockIdx.y | threadIdx.x) == 0) dyn_next[0] = dyn_next[2] = 0;
  __shared__ __attribute__((aligned(16))) DeintLds<PB, OS> bt;
  if constexpr (CO) {
    __shared__ __attribute__((aligned(16))) float4 stage[2][16][96];
    deint_bits_task<PB, NT, OS, NTL, NOW, true>(x, B, D, kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, blockIdx.x,
                                                blockIdx.y, bt, stage);
  } else {
    deint_bits_task<PB, NT, OS, NTL, NOW>(x, B, D, kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, blockIdx.x, blockIdx.y,
                                          bt);
  }
}

// The weight gradient's BitMat (pixels x stacked rows) from the forward's (stacked rows x
// pixels): one wave per 64 x 64 bit tile -- a quarter of a block on either side -- its 128 words in,
// the tile as [8 pixel octets][64 rows] bytes in LDS, its 128 transposed words out (the 8 x 8 bit
// transpose of deint_bits.h). The de-interleave then writes only the forward words (deint
// variant 7): the transpose runs on the side stream beside the layer-0 forward, whose 192 tiles
// (C3) leave CUs free, and the layer-0 weight gradient waits for it.
__device__ __forceinline__ unsigned bits_compact(unsigned s) {  // inverse of bits_spread (low byte)
  unsigned e = s & 0xFu, o = (s >> 16) & 0xFu;
  e = (e | (e << 2)) & 0x33u; e = (e | (e << 1)) & 0x55u;
  o = (o | (o << 2)) & 0x33u; o = (o | (o << 1)) & 0x55u;
  return e | (o << 1);
}
__global__ __launch_bounds__(256) void bits_transpose_kernel(const unsigned* __restrict__ xbf, int kts_f,
                                                             unsigned* __restrict__ xbw, int kts_w, int nrow64) {
  __shared__ __attribute__((aligned(16))) unsigned char tb[4][8][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = blockIdx.x * 4 + wave;
  const bool ok = tile < nrow64 * kts_f;
  const int a = ok ? tile % nrow64 : 0, b = ok ? tile / nrow64 : 0;  // stacked-row tile, pixel tile
  if (ok) {
    const uint2 w = *reinterpret_cast<const uint2*>(xbf + ((size_t)(a >> 2) * kts_f + b) * BITMAT_BLOCK_WORDS +
                                                    (a & 3) * 128 + 2 * lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
          tb[wave][4 * kh + (lane >> 4)][16 * (2 * j + h) + (lane & 15)] =
              (unsigned char)bits_compact((j ? w.y : w.x) >> (8 * h + 4 * kh));
  }
  __syncthreads();
  if (!ok) return;
  unsigned out[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    unsigned wo = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int p = 16 * (2 * j + h) + (lane & 15);
        const unsigned long long rows =
            *reinterpret_cast<const unsigned long long*>(&tb[wave][p >> 3][32 * kh + 8 * (lane >> 4)]);
        const unsigned long long col = (rows >> (p & 7)) & 0x0101010101010101ull;
        wo |= bits_spread((unsigned)((col * 0x0102040810204080ull) >> 56)) << (8 * h + 4 * kh);
      }
    out[j] = wo;
  }
  *reinterpret_cast<uint2*>(xbw + ((size_t)(b >> 2) * kts_w + a) * BITMAT_BLOCK_WORDS + (b & 3) * 128 + 2 * lane) =
      make_uint2(out[0], out[1]);
}

// The plane image of a batch with a pixel other than 0 or 1 (after deint_bits_kernel raised the
// not-binary word; else every workgroup returns at once): bf16 plane 0 (planes 1-2 of the exact
// split too when np == 3), the fp32 rows of the blocks in f32mask, and the inexact flag (*dyn) --
// what the plane path's GEMMs and the BCE epilogue read. Workgroups stride over the 8-pixel groups.
// done (the fused launch's chunk counters, DeintJob::done): zeroed for the next launch, whose
// workers count from 0 (this kernel runs after every fused launch, in stream order)
__global__ void deint_grey_kernel(const float4* __restrict__ x, float* __restrict__ xs,
                                  unsigned short* __restrict__ xp, long long ps, int np, int f32mask,
                                  int* __restrict__ dyn, int B, int D, int ldx, int* __restrict__ done,
                                  int ndone) {
  if (done && blockIdx.x == 0)
    for (int i = threadIdx.x; i < ndone; i += blockDim.x) done[i] = 0;
  if (dyn[2] == 0) return;
  const int nq = D / 8;
  const size_t n = (size_t)B * nq;
  bool nz = false;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / nq), q = (int)(i % nq);
    const float4* src = x + ((size_t)b * 3 * D) / 4 + 6 * (size_t)q;
    float4 v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = src[k];
    nz |= deint_put<2>(v, xs, xp, B, b, (size_t)8 * q, ldx, f32mask);
    if (np == 3) {  // the exact split's residual planes of the 24 values
      const float e[24] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                           v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w,
                           v[4].x, v[4].y, v[4].z, v[4].w, v[5].x, v[5].y, v[5].z, v[5].w};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int ch = c == 0 ? 1 : (c == 1 ? 0 : 2);
        const size_t o = (size_t)(c * B + b) * ldx + (size_t)8 * q;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float r1, r2, r3;
          (void)bf16_rn(e[3 * j + ch], r1);
          xp[ps + o + j] = bf16_rn(r1, r2);
          xp[2 * ps + o + j] = bf16_rn(r2, r3);
        }
      }
    }
  }
  if (__ballot(nz) != 0 && (threadIdx.x & 63) == 0) atomicOr(dyn, 1);
}

inline unsigned nblocks(size_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

__global__ void mvae_region_marker() {}

}  // namespace

hipError_t launch_deinterleave(const float* x, float* xs, const Planes& xp, int* dyn, int* dyn_next,
                               int B, int D, int ldx, int f32mask, int f32dyn_mask, hipStream_t st,
                               unsigned char* xbits, int ldbits) {
  // 8 pixels per thread (4 and 16 measured slower, profiles/r4/r4y_deinterleave.txt; an LDS-staged
  // form with lane-contiguous loads too, r4an_deinterleave_lds_rejected.txt); 4 when D % 8 != 0
  const bool al = (reinterpret_cast<uintptr_t>(x) % 16) == 0;
  if ((D % 8) == 0 && al && (ldx % 8) == 0) {
    dim3 g(nblocks(D / 8, 256), B);
    hipLaunchKernelGGL(deinterleave_vecn_kernel<2>, g, dim3(256), 0, st,
                       reinterpret_cast<const float4*>(x), xs, xp.p, dyn, B, D, ldx, f32mask, dyn_next,
                       xbits, ldbits);
  } else if ((D % 4) == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0 && (ldx % 4) == 0) {
    dim3 g(nblocks(D / 4, 256), B);
    hipLaunchKernelGGL(deinterleave_vec_kernel, g, dim3(256), 0, st,
                       reinterpret_cast<const float4*>(x), xs, xp.p, dyn, B, D, ldx, f32mask, dyn_next);
  } else {
    dim3 g(nblocks(D, 256), B);
    hipLaunchKernelGGL(deinterleave_scalar_kernel, g, dim3(256), 0, st, x, xs, xp.p, dyn, B, D, ldx,
                       f32mask, dyn_next);
  }
  f32dyn_mask &= ~f32mask;
  if (dyn && xp.p && (xp.n == 3 || f32dyn_mask))
    hipLaunchKernelGGL(residual_planes_kernel, dim3(2048), dim3(256), 0, st, x, xs, xp.p, xp.stride,
                       xp.n, f32dyn_mask, dyn, B, D, ldx);
  return hipGetLastError();
}

hipError_t launch_deint_bits(const float* x, int B, int D, unsigned* xbf, int kts_f, unsigned* xbw, int kts_w,
                             unsigned char* xbits, int ldbits, int* dyn, int* dyn_next, float* xs,
                             const Planes& xp, int ldx, int f32dyn_mask, hipStream_t st, int variant) {
  if ((D % 8) || (B % 64) || (reinterpret_cast<uintptr_t>(x) % 16) || (ldx % 8) || !dyn || !xp.p ||
      kts_f != bitmat_kts(D + 1) || kts_w != bitmat_kts(3 * B))
    return hipErrorInvalidValue;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  switch (variant) {  // (diagnostics: mvae_bench_deint) 0 = the step's form
    case 5: {  // the fused launch's LDS-DMA workers alone, one per CU
      DeintJob j;
      j.x = x; j.B = B; j.D = D; j.kts_f = kts_f; j.kts_w = kts_w;
      j.xbf = xbf; j.xbw = xbw; j.xbits = xbits; j.ldbits = ldbits; j.dyn = dyn; j.dyn_next = dyn_next;
      j.nchunks = (kts_f + DEINT_FUSE_PB - 1) / DEINT_FUSE_PB;
      j.nworkers = 256;
      const hipError_t e = launch_deint_persist(j, st);
      if (e != hipSuccess) return e;
      break;
    }
    case 7:  // the step's form without the weight-gradient words (launch_bits_transpose writes them)
      hipLaunchKernelGGL((deint_bits_kernel<2, 256, 72, false, true>), dim3((kts_f + 1) / 2, B / 64), dim3(256), 0, st,
                         x4, B, D, kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    case 8:  // the step's form with coalesced loads of X through an LDS stage (deint_load_co)
      hipLaunchKernelGGL((deint_bits_kernel<2, 256, 72, false, false, true>), dim3((kts_f + 1) / 2, B / 64), dim3(256), 0,
                         st, x4, B, D, kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    case 9:  // variant 7 with coalesced loads
      hipLaunchKernelGGL((deint_bits_kernel<2, 256, 72, false, true, true>), dim3((kts_f + 1) / 2, B / 64), dim3(256), 0,
                         st, x4, B, D, kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    case 6:  // the step's form with non-temporal loads of X (2x slower: r6zb_deint_nt_loads.txt)
      hipLaunchKernelGGL((deint_bits_kernel<2, 256, 72, true>), dim3((kts_f + 1) / 2, B / 64), dim3(256), 0, st, x4, B,
                         D, kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    case 1:
      hipLaunchKernelGGL((deint_bits_kernel<2, 256, 64>), dim3((kts_f + 1) / 2, B / 64), dim3(256), 0, st, x4, B, D,
                         kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    case 2:
      hipLaunchKernelGGL((deint_bits_kernel<4, 512, 72>), dim3((kts_f + 3) / 4, B / 64), dim3(512), 0, st, x4, B, D,
                         kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    case 3:
      hipLaunchKernelGGL((deint_bits_kernel<1, 256, 72>), dim3(kts_f, B / 64), dim3(256), 0, st, x4, B, D,
                         kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    case 4:
      hipLaunchKernelGGL((deint_bits_kernel<4, 256, 72>), dim3((kts_f + 3) / 4, B / 64), dim3(256), 0, st, x4, B, D,
                         kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
      break;
    default:
      hipLaunchKernelGGL((deint_bits_kernel<2, 256, 72>), dim3((kts_f + 1) / 2, B / 64), dim3(256), 0, st, x4, B, D,
                         kts_f, kts_w, xbf, xbw, xbits, ldbits, dyn, dyn_next);
  }
  return launch_deint_grey(x, B, D, dyn, xs, xp, ldx, f32dyn_mask, nullptr, 0, st);
}

hipError_t launch_bits_transpose(const unsigned* xbf, int kts_f, unsigned* xbw, int kts_w, int B, hipStream_t st) {
  if (B % 64 || kts_f <= 0 || kts_w != bitmat_kts(3 * B)) return hipErrorInvalidValue;
  const int nrow64 = 3 * B / 64;
  const long long tiles = (long long)nrow64 * kts_f;
  hipLaunchKernelGGL(bits_transpose_kernel, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, st, xbf, kts_f, xbw,
                     kts_w, nrow64);
  return hipGetLastError();
}

hipError_t launch_deint_grey(const float* x, int B, int D, int* dyn, float* xs, const Planes& xp, int ldx,
                             int f32dyn_mask, int* done, int ndone, hipStream_t st) {
  // (256 workgroups striding: for a 0/1 batch every one returns at once, and fewer cost less)
  hipLaunchKernelGGL(deint_grey_kernel, dim3(256), dim3(256), 0, st, reinterpret_cast<const float4*>(x), xs,
                     xp.p, xp.stride, xp.n, f32dyn_mask, dyn, B, D, ldx, done, ndone);
  return hipGetLastError();
}

hipError_t launch_deinterleave_grid(const float* x, unsigned short* xp, int B, int D, int ldx, int grid,
                                    hipStream_t st) {
  if ((D % 8) || (ldx % 8) || (reinterpret_cast<uintptr_t>(x) % 16)) return hipErrorInvalidValue;
  if (grid < 0) {
    dim3 g(nblocks(D / 8, 256), B);
    hipLaunchKernelGGL(deinterleave_vecn_kernel<2>, g, dim3(256), 0, st, reinterpret_cast<const float4*>(x),
                       nullptr, xp, nullptr, B, D, ldx, 0, nullptr, nullptr, 0);
  } else if (grid > 0) {
    hipLaunchKernelGGL(deinterleave_persist_kernel, dim3(grid), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(x), xp, B, D, ldx);
  }
  return hipGetLastError();
}

hipError_t launch_normal(float* out, int slots, int B, int L, int Bg, int off, uint64_t seed,
                         uint64_t counter, hipStream_t st) {
  const size_t n = (size_t)B * L;
  if (n == 0 || slots <= 0) return hipSuccess;
  // Philox blocks touched by one slot's range: at most n/4 + 2
  dim3 g(nblocks(n / 4 + 2, 256), slots);
  hipLaunchKernelGGL(normal_kernel, g, dim3(256), 0, st, out, B, L, Bg, off, seed, counter);
  return hipGetLastError();
}

static EpsSrc eps_src(const LatentEps& le) {
  EpsSrc es;
  es.buf = le.buf;
  es.seed = le.seed;
  es.counter = le.counter;
  es.Bg = le.Bg;
  es.off = le.off;
  return es;
}

hipError_t launch_latent_fwd(const float* ms, const LatentEps& le, float* z, const Planes& zp,
                             int zmask, int B, int L, int ldz, float* rowfwd, hipStream_t st) {
  const EpsSrc es = eps_src(le);
  const bool v4 = L % 4 == 0 && ldz % 4 == 0;
  if (v4 && L >= 1024)
    hipLaunchKernelGGL((latent_fwd_kernel<true, 4>), dim3(B), dim3(256), 0, st, ms, es, z, zp.p,
                       zp.stride, zp.n, zmask, B, L, ldz, rowfwd);
  else if (v4)
    hipLaunchKernelGGL((latent_fwd_kernel<true, 1>), dim3(nblocks(B, 4)), dim3(256), 0, st, ms, es, z,
                       zp.p, zp.stride, zp.n, zmask, B, L, ldz, rowfwd);
  else
    hipLaunchKernelGGL((latent_fwd_kernel<false, 1>), dim3(nblocks(B, 4)), dim3(256), 0, st, ms, es, z,
                       zp.p, zp.stride, zp.n, zmask, B, L, ldz, rowfwd);
  return hipGetLastError();
}

int colstats_nchunk(int B) { return (B + CS_ROWS - 1) / CS_ROWS; }

hipError_t launch_colstats(int mode, const float* z, int B, int L, int ldz, const float* colsq,
                           const float* draw, float* part, int nchunk, float* out, hipStream_t st, int* cnt) {
  const int ncols = mode == 0 ? 2 * L : L;
  dim3 g(nblocks(ncols, 64), nchunk);
  hipLaunchKernelGGL(colstats_part_kernel, g, dim3(256), 0, st, mode, z, B, L, ldz, colsq, draw, part, cnt, out);
  if (!cnt)
    hipLaunchKernelGGL(colstats_final_kernel, dim3(nblocks(ncols, 256)), dim3(256), 0, st, part, nchunk, ncols, out);
  return hipGetLastError();
}

hipError_t launch_metric(const float* z, int ldz, const float* rowfwd, const float* rowpart, int nblk,
                         const float* areas, const float* colsq, int B, int L, int metric, int recip,
                         float w, float inv_bg, float* rowvals, float* dist, float* draw,
                         hipStream_t st) {
  hipLaunchKernelGGL(metric_kernel, dim3(nblocks(B, 4)), dim3(256), 0, st, z, ldz, rowfwd, rowpart, nblk,
                     areas, colsq, B, L, metric, recip, w, inv_bg, rowvals, dist, draw);
  return hipGetLastError();
}

hipError_t launch_loss_reduce(const float* rowvals, int B, float inv_bg, float* losses, hipStream_t st) {
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, st, rowvals, B, inv_bg, losses);
  return hipGetLastError();
}

hipError_t launch_latent_bwd(const float* ms, const LatentEps& le, const float* dzdec, const float* draw,
                             const float* colsq, const float* coldot, int B, int L, int metric, float w,
                             float inv_bg, float* dhead, int ldh, const Planes& hp, hipStream_t st) {
  const EpsSrc es = eps_src(le);
  if (L % 4 == 0 && ldh % 4 == 0) {
    const size_t n = (size_t)B * (L / 4);
    hipLaunchKernelGGL(latent_bwd_kernel<true>, dim3(nblocks(n, 256)), dim3(256), 0, st, ms, es, dzdec,
                       draw, colsq, coldot, B, L, metric, w, inv_bg, dhead, ldh, hp.p, hp.stride, hp.n);
  } else {
    const size_t n = (size_t)B * L;
    hipLaunchKernelGGL(latent_bwd_kernel<false>, dim3(nblocks(n, 256)), dim3(256), 0, st, ms, es, dzdec,
                       draw, colsq, coldot, B, L, metric, w, inv_bg, dhead, ldh, hp.p, hp.stride, hp.n);
  }
  return hipGetLastError();
}

hipError_t launch_adam(const AdamArgs& a, hipStream_t st) {
  AdamArgs r = a;
  r.i1 = a.i1 < a.n_all ? a.i1 : a.n_all;
  if (r.i0 >= r.i1) return hipSuccess;
  if (r.nt) hipLaunchKernelGGL(adam_kernel<true>, dim3(nblocks(r.i1 - r.i0, 256)), dim3(256), 0, st, r);
  else hipLaunchKernelGGL(adam_kernel<false>, dim3(nblocks(r.i1 - r.i0, 256)), dim3(256), 0, st, r);
  return hipGetLastError();
}

hipError_t launch_split_planes(const float* src, size_t n, const Planes& dst, hipStream_t st) {
  if (!dst.p || n == 0) return hipSuccess;
  hipLaunchKernelGGL(split_planes_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, src, n, dst.p,
                     dst.stride, dst.n);
  return hipGetLastError();
}

__global__ void binarize_kernel(float* x, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] > 0.f ? 1.f : 0.f;
}

hipError_t launch_binarize(float* x, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(binarize_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, x, n);
  return hipGetLastError();
}

hipError_t launch_make_batch(const unsigned char* locks, const unsigned char* keys, int H, int W,
                             const int* idx, const float* coef, int B, float div, float* x,
                             hipStream_t st) {
  const size_t hw = (size_t)H * W;
  if (hw % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    dim3 g(nblocks(hw, MB_PIX), B);
    hipLaunchKernelGGL(make_batch4_kernel, g, dim3(256), 0, st, locks, keys, H, W, idx,
                       reinterpret_cast<const float4*>(coef), div, x);
    return hipGetLastError();
  }
  dim3 g(nblocks(hw, 256), B);
  hipLaunchKernelGGL(make_batch_kernel, g, dim3(256), 0, st, locks, keys, H, W, idx,
                     reinterpret_cast<const float4*>(coef), div, x);
  return hipGetLastError();
}

hipError_t launch_marker(int region, hipStream_t st) {
  hipLaunchKernelGGL(mvae_region_marker, dim3(MARKER_GRID + region), dim3(64), 0, st);
  return hipGetLastError();
}

hipError_t launch_copy2d(const float* src, int lds, float* dst, int ldd, int rows, int cols,
                         hipStream_t st) {
  const size_t n = (size_t)rows * cols;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(copy2d_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, src, lds, dst, ldd, rows, cols);
  return hipGetLastError();
}

}  // namespace mvae
