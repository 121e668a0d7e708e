// Bandwidth-bound kernels of the metric-VAE step (gfx950): batch de-interleave, the
// counter-based N(0,1) sampler, reparameterisation, the latent loss head forward/backward
// (KL, deformation, cosine / squared-difference distance, training_loss), deterministic
// loss/column reductions, and the fused dual TF-Adam update.
//
// Row order of every stacked encoder buffer: [rotated lock | lock | key] (3B rows), so the
// cost gradient (rotated+lock) and the metric gradient (lock+key) each use a CONTIGUOUS
// 2B-row range. The backward stacks 4B rows: [rot(g1) | lock(g1) | lock(g2) | key(g2)].
#include "mvae_internal.h"

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
                                        int B, int D, int ldx, int f32mask) {
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

__global__ void deinterleave_scalar_kernel(const float* __restrict__ x, float* __restrict__ xs,
                                           unsigned short* __restrict__ xp, int* __restrict__ dyn,
                                           int B, int D, int ldx, int f32mask) {
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
  uint32_t c[4] = {(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)counter, (uint32_t)(counter >> 32)};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float inv = 2.3283064365386963e-10f;  // 2^-32
  float r[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float u1 = ((float)c[2 * j] + 0.5f) * inv;  // (0,1)
    const float u2 = ((float)c[2 * j + 1] + 0.5f) * inv;
    const float rad = sqrtf(-2.f * logf(u1));
    float s, co;
    sincosf(6.283185307179586f * u2, &s, &co);
    r[2 * j] = rad * co;
    r[2 * j + 1] = rad * s;
  }
  float* o = out + (size_t)blockIdx.y * n;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t e = 4 * q + j;
    if (e >= g0 && e < g0 + n) o[e - g0] = r[j];
  }
}

// ---------------------------------------------------------------- reparameterisation
// z = mu + sqrt(exp(s)) * eps   (11a/vae.py:371-377); ms rows = [mu | s] (2L wide). The bf16
// planes of z are written for the lock block only: the decoder's GEMMs read no other rows.
__global__ void latent_fwd_kernel(const float* __restrict__ ms, const float* __restrict__ eps,
                                  float* __restrict__ z, unsigned short* __restrict__ zp,
                                  long long ps, int np, int B, int L, int ldz) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)3 * B * L) return;
  const int r = (int)(idx / L), i = (int)(idx - (size_t)r * L);
  const int blk = r / B, b = r - blk * B;
  const float mu = ms[(size_t)r * 2 * L + i];
  const float s = ms[(size_t)r * 2 * L + L + i];
  const float e = eps[((size_t)eps_slot(blk) * B + b) * L + i];
  const float v = mu + sqrtf(expf(s)) * e;
  z[(size_t)r * ldz + i] = v;
  if (zp && blk == 1) planes_put(zp, ps, np, (size_t)r * ldz + i, v);
}

// the same, 4 consecutive elements per thread (L % 4 == 0: 16-B rows of ms, eps and z)
__global__ void latent_fwd4_kernel(const float* __restrict__ ms, const float* __restrict__ eps,
                                   float* __restrict__ z, unsigned short* __restrict__ zp,
                                   long long ps, int np, int B, int L, int ldz) {
  const int L4 = L / 4;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)3 * B * L4) return;
  const int r = (int)(idx / L4), i = 4 * (int)(idx - (size_t)r * L4);
  const int blk = r / B, b = r - blk * B;
  const float4 mu = *reinterpret_cast<const float4*>(ms + (size_t)r * 2 * L + i);
  const float4 s = *reinterpret_cast<const float4*>(ms + (size_t)r * 2 * L + L + i);
  const float4 e = *reinterpret_cast<const float4*>(eps + ((size_t)eps_slot(blk) * B + b) * L + i);
  const float4 v = make_float4(mu.x + sqrtf(expf(s.x)) * e.x, mu.y + sqrtf(expf(s.y)) * e.y,
                               mu.z + sqrtf(expf(s.z)) * e.z, mu.w + sqrtf(expf(s.w)) * e.w);
  const size_t o = (size_t)r * ldz + i;
  *reinterpret_cast<float4*>(z + o) = v;
  if (zp && blk == 1) {
    planes_put(zp, ps, np, o, v.x);
    planes_put(zp, ps, np, o + 1, v.y);
    planes_put(zp, ps, np, o + 2, v.z);
    planes_put(zp, ps, np, o + 3, v.w);
  }
}

// ---------------------------------------------------------------- column statistics
// mode 0 (colsq):  out[j] = sum_b z_lock[b][j]^2 (j < L), sum_b z_key[b][j-L]^2 (j >= L)
// mode 1 (coldot): out[i] = sum_b draw_b * n_lock[b][i] * n_key[b][i]
// Two-stage, fixed-order (deterministic): partials over row chunks, then chunk sums.
constexpr int CS_ROWS = 128;
__global__ void colstats_part_kernel(int mode, const float* __restrict__ z, int B, int L, int ldz,
                                     const float* __restrict__ colsq, const float* __restrict__ draw,
                                     float* __restrict__ part) {
  const int ncols = mode == 0 ? 2 * L : L;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 cols x 4 row lanes
  const int j = blockIdx.x * 64 + tx;
  const int r0 = blockIdx.y * CS_ROWS;
  const int r1 = min(B, r0 + CS_ROWS);
  __shared__ float red[4][64];
  float acc = 0.f;
  if (j < ncols) {
    if (mode == 0) {
      const float* src = j < L ? z + (size_t)B * ldz + j : z + (size_t)2 * B * ldz + (j - L);
      for (int b = r0 + ty; b < r1; b += 4) {
        const float v = src[(size_t)b * ldz];
        acc += v * v;
      }
    } else {
      const float rl = rsqrtf(fmaxf(colsq[j], L2_EPS));
      const float rk = rsqrtf(fmaxf(colsq[L + j], L2_EPS));
      for (int b = r0 + ty; b < r1; b += 4) {
        const float zl = z[(size_t)(B + b) * ldz + j], zk = z[(size_t)(2 * B + b) * ldz + j];
        acc += draw[b] * (zl * rl) * (zk * rk);
      }
    }
  }
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && j < ncols)
    part[(size_t)blockIdx.y * ncols + j] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
}

__global__ void colstats_final_kernel(const float* __restrict__ part, int nchunk, int ncols,
                                      float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ncols) return;
  float acc = 0.f;
  for (int c = 0; c < nchunk; ++c) acc += part[(size_t)c * ncols + j];
  out[j] = acc;
}

// ---------------------------------------------------------------- metric / losses per row
// One wave per batch row b. rowvals[b] = {R_b, K_b, F_b, T_b}; dist[b]; draw[b] = dT/draw_b.
//   R_b: BCE row partials from the decoder-output GEMM epilogue (11a/vae.py:266-269)
//   K_b = -0.5 sum(1 + s - mu^2 - exp(s))            (lock pass, :281-284)
//   F_b = w sum (z_lock - z_rot)^2                    (:293-294)
//   dist_b: cosine (axis-0 l2_normalize, :444-458) or sum (z_lock - z_key)^2; 1/raw if recip
//   T_b = (dist_b - area_b)^2                         (:313)
__global__ void metric_kernel(const float* __restrict__ z, int ldz, const float* __restrict__ ms,
                              const float* __restrict__ rowpart, int nblk,
                              const float* __restrict__ areas, const float* __restrict__ colsq,
                              int B, int L, int metric, int recip, float w, float inv_bg,
                              float* __restrict__ rowvals, float* __restrict__ dist,
                              float* __restrict__ draw) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* zr = z + (size_t)b * ldz;
  const float* zl = z + (size_t)(B + b) * ldz;
  const float* zk = z + (size_t)(2 * B + b) * ldz;
  const float* msl = ms + (size_t)(B + b) * 2 * L;
  float kl = 0.f, fd = 0.f, raw = 0.f, rp = 0.f;
  auto term = [&](float mu, float s, float l, float r, float k, int i) {
    kl += 1.f + s - mu * mu - expf(s);
    const float d = l - r;
    fd += d * d;
    if (metric == 0) {
      const float rl = rsqrtf(fmaxf(colsq[i], L2_EPS));
      const float rk = rsqrtf(fmaxf(colsq[L + i], L2_EPS));
      raw += (l * rl) * (k * rk);
    } else {
      const float e = l - k;
      raw += e * e;
    }
  };
  if ((L & 3) == 0 && L >= 256 && (ldz & 3) == 0) {  // 16-B loads, 4 elements per lane (all lanes busy)
    for (int i = 4 * lane; i < L; i += 256) {
      const float4 mu = *reinterpret_cast<const float4*>(msl + i);
      const float4 s = *reinterpret_cast<const float4*>(msl + L + i);
      const float4 l = *reinterpret_cast<const float4*>(zl + i);
      const float4 r = *reinterpret_cast<const float4*>(zr + i);
      const float4 k = *reinterpret_cast<const float4*>(zk + i);
      term(mu.x, s.x, l.x, r.x, k.x, i);
      term(mu.y, s.y, l.y, r.y, k.y, i + 1);
      term(mu.z, s.z, l.z, r.z, k.z, i + 2);
      term(mu.w, s.w, l.w, r.w, k.w, i + 3);
    }
  } else {
    for (int i = lane; i < L; i += 64) term(msl[i], msl[L + i], zl[i], zr[i], zk[i], i);
  }
  for (int j = lane; j < nblk; j += 64) rp += rowpart[(size_t)b * nblk + j];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    kl += __shfl_xor(kl, off, 64);
    fd += __shfl_xor(fd, off, 64);
    raw += __shfl_xor(raw, off, 64);
    rp += __shfl_xor(rp, off, 64);
  }
  if (lane == 0) {
    const float dv = recip ? 1.f / raw : raw;
    const float a = areas ? areas[b] : 0.f;
    const float g = 2.f * (dv - a) * inv_bg;
    rowvals[4 * (size_t)b + 0] = rp;
    rowvals[4 * (size_t)b + 1] = -0.5f * kl;
    rowvals[4 * (size_t)b + 2] = w * fd;
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
  for (int b = threadIdx.x; b < B; b += 256) {
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] += rowvals[4 * (size_t)b + q];
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
__global__ void latent_bwd_kernel(const float* __restrict__ z, int ldz, const float* __restrict__ ms,
                                  const float* __restrict__ eps, const float* __restrict__ dzdec,
                                  const float* __restrict__ draw, const float* __restrict__ colsq,
                                  const float* __restrict__ coldot, int B, int L, int metric,
                                  float w, float inv_bg, float* __restrict__ dhead, int ldh,
                                  unsigned short* __restrict__ hp, long long ps, int np) {
  // one thread per (b, i): the four backward rows of element i of pair b from one read of its
  // three z values, the lock mu/s and the rot/key s, the three eps and dz_dec
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * L) return;
  const int b = (int)(idx / L), i = (int)(idx - (size_t)b * L);
  const float zr = z[(size_t)b * ldz + i];
  const float zl = z[(size_t)(B + b) * ldz + i];
  const float zk = z[(size_t)(2 * B + b) * ldz + i];
  const float s_r = ms[(size_t)b * 2 * L + L + i];
  const float mu_l = ms[(size_t)(B + b) * 2 * L + i];
  const float s_l = ms[(size_t)(B + b) * 2 * L + L + i];
  const float s_k = ms[(size_t)(2 * B + b) * 2 * L + L + i];
  const float e_r = eps[((size_t)eps_slot(0) * B + b) * L + i];
  const float e_l = eps[((size_t)eps_slot(1) * B + b) * L + i];
  const float e_k = eps[((size_t)eps_slot(2) * B + b) * L + i];
  const float ex_l = expf(s_l);
  const float sig_r = sqrtf(expf(s_r)), sig_l = sqrtf(ex_l), sig_k = sqrtf(expf(s_k));
  const float def = 2.f * w * (zl - zr) * inv_bg;
  float dz2, dz3;  // g2 rows: lock, key
  {
    const float dr = draw[b];
    if (metric == 1) {
      dz2 = 2.f * dr * (zl - zk);
      dz3 = -dz2;
    } else {
      const float ssl = colsq[i], ssk = colsq[L + i];
      const float rl = rsqrtf(fmaxf(ssl, L2_EPS)), rk = rsqrtf(fmaxf(ssk, L2_EPS));
      const float nl = zl * rl, nk = zk * rk, c = coldot[i];
      dz2 = rl * (dr * nk - (ssl >= L2_EPS ? nl * c : 0.f));
      dz3 = rk * (dr * nl - (ssk >= L2_EPS ? nk * c : 0.f));
    }
  }
  const float dz1 = dzdec[(size_t)b * L + i] + def;
  const float dmu[4] = {-def, dz1 + mu_l * inv_bg, dz2, dz3};
  const float ds[4] = {-0.5f * def * e_r * sig_r, 0.5f * dz1 * e_l * sig_l + 0.5f * (ex_l - 1.f) * inv_bg,
                       0.5f * dz2 * e_l * sig_l, 0.5f * dz3 * e_k * sig_k};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const size_t o = (size_t)(q * B + b) * ldh;
    if (dhead) {
      dhead[o + i] = dmu[q];
      dhead[o + L + i] = ds[q];
    }
    if (hp) {
      planes_put(hp, ps, np, o + i, dmu[q]);
      planes_put(hp, ps, np, o + L + i, ds[q]);
    }
  }
}

// ---------------------------------------------------------------- dual TF-Adam
// opt1 (lr1, g1) over every trained variable, opt2 (lr2, g2) over the encoder slice;
// both from the pre-step gradients: theta = (theta - d1) - d2.  lr_t precomputed on the
// host in fp32 exactly as TF ApplyAdam (lr*sqrt(1-b2^t)/(1-b1^t) with fp32 beta powers).
__global__ void adam_kernel(AdamArgs a) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_all) return;
  float th = a.theta[i];
  {
    const float g = a.g1[i];
    float m = a.m1[i], v = a.v1[i];
    m += (g - m) * (1.f - a.b1);
    v += (g * g - v) * (1.f - a.b2);
    a.m1[i] = m; a.v1[i] = v;
    th -= (a.lr1 * m) / (sqrtf(v) + a.eps);
  }
  if (i < a.n_enc) {
    const float g = a.g2[i];
    float m = a.m2[i], v = a.v2[i];
    m += (g - m) * (1.f - a.b1);
    v += (g * g - v) * (1.f - a.b2);
    a.m2[i] = m; a.v2[i] = v;
    th -= (a.lr2 * m) / (sqrtf(v) + a.eps);
  }
  a.theta[i] = th;
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
// gather indices match the host restatement bit for bit.
__global__ void make_batch_kernel(const unsigned char* __restrict__ locks,
                                  const unsigned char* __restrict__ keys, int H, int W,
                                  const int* __restrict__ idx, const float4* __restrict__ coef,
                                  float div, float* __restrict__ x) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int HW = H * W;
  if (p >= HW) return;
  const int id = idx[b];
  const float4 cf = coef[b];
  const int yy = p / W, xx = p - yy * W;
  const float fx = (float)xx, fy = (float)yy;
  const float xin = __fadd_rn(__fsub_rn(__fmul_rn(cf.x, fx), __fmul_rn(cf.y, fy)), cf.z);
  const float yin = __fadd_rn(__fadd_rn(__fmul_rn(cf.y, fx), __fmul_rn(cf.x, fy)), cf.w);
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

inline unsigned nblocks(size_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

__global__ void mvae_region_marker() {}

}  // namespace

hipError_t launch_deinterleave(const float* x, float* xs, const Planes& xp, int* dyn, int B, int D,
                               int ldx, int f32mask, int f32dyn_mask, hipStream_t st) {
  if ((D % 4) == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0 && (ldx % 4) == 0) {
    dim3 g(nblocks(D / 4, 256), B);
    hipLaunchKernelGGL(deinterleave_vec_kernel, g, dim3(256), 0, st,
                       reinterpret_cast<const float4*>(x), xs, xp.p, dyn, B, D, ldx, f32mask);
  } else {
    dim3 g(nblocks(D, 256), B);
    hipLaunchKernelGGL(deinterleave_scalar_kernel, g, dim3(256), 0, st, x, xs, xp.p, dyn, B, D, ldx,
                       f32mask);
  }
  f32dyn_mask &= ~f32mask;
  if (dyn && xp.p && (xp.n == 3 || f32dyn_mask))
    hipLaunchKernelGGL(residual_planes_kernel, dim3(2048), dim3(256), 0, st, x, xs, xp.p, xp.stride,
                       xp.n, f32dyn_mask, dyn, B, D, ldx);
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

hipError_t launch_latent_fwd(const float* ms, const float* eps, float* z, const Planes& zp, int B,
                             int L, int ldz, hipStream_t st) {
  if (L % 4 == 0 && ldz % 4 == 0) {
    const size_t n4 = (size_t)3 * B * (L / 4);
    hipLaunchKernelGGL(latent_fwd4_kernel, dim3(nblocks(n4, 256)), dim3(256), 0, st, ms, eps, z, zp.p,
                       zp.stride, zp.n, B, L, ldz);
    return hipGetLastError();
  }
  const size_t n = (size_t)3 * B * L;
  hipLaunchKernelGGL(latent_fwd_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, ms, eps, z, zp.p,
                     zp.stride, zp.n, B, L, ldz);
  return hipGetLastError();
}

int colstats_nchunk(int B) { return (B + CS_ROWS - 1) / CS_ROWS; }

hipError_t launch_colstats(int mode, const float* z, int B, int L, int ldz, const float* colsq,
                           const float* draw, float* part, int nchunk, float* out, hipStream_t st) {
  const int ncols = mode == 0 ? 2 * L : L;
  dim3 g(nblocks(ncols, 64), nchunk);
  hipLaunchKernelGGL(colstats_part_kernel, g, dim3(256), 0, st, mode, z, B, L, ldz, colsq, draw, part);
  hipLaunchKernelGGL(colstats_final_kernel, dim3(nblocks(ncols, 256)), dim3(256), 0, st, part, nchunk, ncols, out);
  return hipGetLastError();
}

hipError_t launch_metric(const float* z, int ldz, const float* ms, const float* rowpart, int nblk,
                         const float* areas, const float* colsq, int B, int L, int metric, int recip,
                         float w, float inv_bg, float* rowvals, float* dist, float* draw,
                         hipStream_t st) {
  hipLaunchKernelGGL(metric_kernel, dim3(nblocks(B, 4)), dim3(256), 0, st, z, ldz, ms, rowpart, nblk,
                     areas, colsq, B, L, metric, recip, w, inv_bg, rowvals, dist, draw);
  return hipGetLastError();
}

hipError_t launch_loss_reduce(const float* rowvals, int B, float inv_bg, float* losses, hipStream_t st) {
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, st, rowvals, B, inv_bg, losses);
  return hipGetLastError();
}

hipError_t launch_latent_bwd(const float* z, int ldz, const float* ms, const float* eps,
                             const float* dzdec, const float* draw, const float* colsq,
                             const float* coldot, int B, int L, int metric, float w, float inv_bg,
                             float* dhead, int ldh, const Planes& hp, hipStream_t st) {
  const size_t n = (size_t)B * L;
  hipLaunchKernelGGL(latent_bwd_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, z, ldz, ms, eps, dzdec,
                     draw, colsq, coldot, B, L, metric, w, inv_bg, dhead, ldh, hp.p, hp.stride, hp.n);
  return hipGetLastError();
}

hipError_t launch_adam(const AdamArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(nblocks(a.n_all, 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_split_planes(const float* src, size_t n, const Planes& dst, hipStream_t st) {
  if (!dst.p || n == 0) return hipSuccess;
  hipLaunchKernelGGL(split_planes_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, src, n, dst.p,
                     dst.stride, dst.n);
  return hipGetLastError();
}

hipError_t launch_make_batch(const unsigned char* locks, const unsigned char* keys, int H, int W,
                             const int* idx, const float* coef, int B, float div, float* x,
                             hipStream_t st) {
  dim3 g(nblocks((size_t)H * W, 256), B);
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
