// The de-interleave to bits, one task (64 batch rows x 64 PB pixels): the body of
// deint_bits_kernel (mvae_kernels.hip) and of the worker workgroups of the layer-0 forward's
// fused launch (gemm_bf16e.hip, DeintJob). Writes the layer-0 pixel operand of a 0/1 batch as the
// eight-phase kernel's BitMats (mvae_internal.h): xbf = A of the forward (rows [rot | lock | key] x
// pixels, the ones column at k = D), xbw = A of the weight gradient (pixels x rows, the ones row at
// pixel D), plus the BCE target (the lock block) as bits per row (GemmEpi::xbits) -- 1.1 bits
// written per pixel triple instead of the 48 of the bf16 plane. Each thread reads 4 x 96
// contiguous bytes (8 pixels of one row, as the plane kernel), writes one byte per block into LDS
// ([block][octet][row]: a row-contiguous 8 x 8 bit block is one u64), then assembles the forward
// words four at a time (one 16-B store; SC1: written through, `sc1`, for a consumer in the same
// launch -- MI355X_MICROARCH.md's sc1 hand-off) and the weight-gradient words one at a time.
// Raises the not-binary word (dyn[2]) when a pixel is neither 0 nor 1. Padding outside the
// written blocks (rows past 3B, pixel quarters past D) is zero from the buffers' creation.
#pragma once
#include "mvae_internal.h"

namespace mvae {

// bits el = 0..7 of b -> positions 0..3 (even el) and 16..19 (odd el): a BitMat word's layout
__device__ __forceinline__ unsigned bits_spread(unsigned b) {
  unsigned e = b & 0x55u, o = (b >> 1) & 0x55u;
  e = (e | (e >> 1)) & 0x33u; e = (e | (e >> 2)) & 0x0Fu;
  o = (o | (o >> 1)) & 0x33u; o = (o | (o >> 2)) & 0x0Fu;
  return e | (o << 16);
}

// LDS of one task: [3 blocks][8 PB octets][OS bytes per octet row] (OS 72: the 16 octets of a
// write land on 16 banks)
template <int PB, int OS>
using DeintLds = unsigned char[3][8 * PB][OS];

// task (bx, by): pixels [64 PB bx, +64 PB), batch rows [64 by, +64), NT threads. Its loads
// (deint_load: 4 x 96 contiguous bytes of NR rows per thread into v) and the rest (deint_finish;
// `written` runs once v is consumed -- this thread's LDS bytes written, v free for the next task's
// loads -- and `synced` once the workgroup has synchronised after everyone's LDS writes)
template <int PB, int NT>
struct DeintShape {
  static constexpr int NO = 8 * PB;    // octets per row
  static constexpr int RPP = NT / NO;  // rows per pass
  static constexpr int NR = 64 / RPP;  // row passes per thread
  static_assert(NT % NO == 0 && 64 % RPP == 0, "whole rows per pass");
};
template <int PB, int NT, bool NTL = false>
__device__ __forceinline__ void deint_load(const float4* __restrict__ x, int D, int bx, int by,
                                           float4 (&v)[DeintShape<PB, NT>::NR][6]) {
  using S = DeintShape<PB, NT>;
  const int tid = threadIdx.x;
  // (unconditional loads -- octets past D read the row's last one, unused -- so the values need no
  // merge with a not-loaded path, whose register copies would wait for every load at once)
  const int b0 = by * 64, pix = min(bx * 64 * PB + 8 * (tid % S::NO), D - 8);
#pragma unroll
  for (int i = 0; i < S::NR; ++i) {
    const float4* src = x + ((size_t)(b0 + tid / S::NO + S::RPP * i) * 3 * D + 3 * (size_t)pix) / 4;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      if constexpr (NTL) {  // (read once: non-temporal)
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src + k));
        v[i][k] = make_float4(t.x, t.y, t.z, t.w);
      } else {
        v[i][k] = src[k];
      }
    }
  }
}
// The same registers loaded coalesced: pass i's 16 rows x 96 float4 (the task's 1.5 KB of each row)
// read by consecutive lanes (one 1 KB contiguous span per wave instruction, where deint_load's
// lanes stride 96 B: each instruction then touches 48 lines of 128 B), passed through an LDS stage
// (two buffers of 24 KB, pass parity) into deint_load's mapping (row tid / 16 + 16 i, octet
// tid % 16). PB 2, 256 threads only. Float4s past the row's end (pixels past D, unused) read its last.
__device__ __forceinline__ void deint_load_co(const float4* __restrict__ x, int D, int bx, int by,
                                              float4 (&v)[4][6], float4 (*stage)[16][96]) {
  const int tid = threadIdx.x;
  const int b0 = by * 64, c40 = 3 * (bx * 128) / 4, rowf4 = 3 * D / 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int q = tid + 256 * k, r = q / 96, c4 = min(c40 + q % 96, rowf4 - 1);
      v[i][k] = x[(size_t)(b0 + 16 * i + r) * rowf4 + c4];
    }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float4 (*st)[96] = stage[i & 1];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int q = tid + 256 * k;
      st[q / 96][q % 96] = v[i][k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 6; ++k) v[i][k] = st[tid / 16][6 * (tid % 16) + k];
  }
}

// one row's 8 pixels x 3 channels (interleaved, as X stores them) -> the byte of each block
// (bit j = pixel j nonzero; block c: rot, lock, key <- channels 1, 0, 2); true if a value is not
// 0 / 1
__device__ __forceinline__ bool deint_octet(const float (&e)[24], unsigned (&by3)[3]) {
  bool nb = false;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int ch = c == 0 ? 1 : (c == 1 ? 0 : 2);
    unsigned byte = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = e[3 * j + ch];
      byte |= (f != 0.f ? 1u : 0u) << j;
      nb |= (f != 0.f) & (f != 1.f);
    }
    by3[c] = byte;
  }
  return nb;
}

// the task's BitMat words from its LDS bytes, by threads t0, t0 + nt, ...: the forward words four
// at a time (lanes 2 q, 2 q + 1 of the fragment layout, words j = 0 / 1 each: rows 16 (2 j + h) +
// (lane & 15), k-octet 8 kk + 4 kh + (lane >> 4); one 16-B store, SC1 written through), the
// weight-gradient words one at a time (pixel 64 kk + 16 (2 j + h) + (lane & 15), rows 32 kh +
// 8 (lane >> 4) + 0..7: bit (pixel & 7) of 8 row bytes of one octet)
template <int PB, int OS, bool SC1, bool NOW = false>
__device__ __forceinline__ void deint_words(int t0, int nt, int B, int D, int kts_f, int kts_w,
                                            unsigned* __restrict__ xbf, unsigned* __restrict__ xbw, int bx,
                                            int by, const DeintLds<PB, OS>& bt) {
  const int b0 = by * 64, p0 = bx * 64 * PB;
  for (int wq = t0; wq < 3 * PB * 32; wq += nt) {
    const int c = wq / (PB * 32), kk = (wq / 32) % PB, wl0 = 4 * (wq & 31);
    const int kt = PB * bx + kk;
    if (kt >= kts_f) continue;
    const int grow = c * B + b0;  // first stacked row of this task's 64
    unsigned w4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int wl = wl0 + q, lane = wl >> 1, j = wl & 1;
      unsigned w = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
          w |= bits_spread(bt[c][8 * kk + 4 * kh + (lane >> 4)][16 * (2 * j + h) + (lane & 15)]) << (8 * h + 4 * kh);
      w4[q] = w;
    }
    unsigned* dst = xbf + ((size_t)(grow >> 8) * kts_f + kt) * BITMAT_BLOCK_WORDS + ((grow >> 6) & 3) * 128 + wl0;
    if constexpr (SC1) {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 val = {w4[0], w4[1], w4[2], w4[3]};
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(val) : "memory");
    } else {
      *reinterpret_cast<uint4*>(dst) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
  for (int wi = t0; wi < (NOW ? 0 : 3 * PB * 128); wi += nt) {  // (NOW: diagnostics, no xbw)
    const int c = wi / (PB * 128), kk = (wi / 128) % PB, wl = wi & 127, lane = wl >> 1, j = wl & 1;
    const int grow = c * B + b0;
    const int pq = p0 + 64 * kk;
    if (pq > D) continue;
    unsigned w = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int pr = 64 * kk + 16 * (2 * j + h) + (lane & 15);
        const unsigned long long rows =
            *reinterpret_cast<const unsigned long long*>(&bt[c][pr >> 3][32 * kh + 8 * (lane >> 4)]);
        const unsigned long long col = (rows >> (pr & 7)) & 0x0101010101010101ull;
        const unsigned byte = (unsigned)((col * 0x0102040810204080ull) >> 56);  // bit i = row i
        w |= bits_spread(byte) << (8 * h + 4 * kh);
      }
    xbw[((size_t)(pq >> 8) * kts_w + (grow >> 6)) * BITMAT_BLOCK_WORDS + ((pq >> 6) & 3) * 128 + wl] = w;
  }
}

template <int PB, int NT, int OS, bool SC1, class FW, class FS, bool NOW = false>
__device__ __forceinline__ void deint_finish(int B, int D, int kts_f, int kts_w, unsigned* __restrict__ xbf,
                                             unsigned* __restrict__ xbw, unsigned char* __restrict__ xbits,
                                             int ldbits, int* __restrict__ dyn, int bx, int by,
                                             const float4 (&v)[DeintShape<PB, NT>::NR][6], DeintLds<PB, OS>& bt,
                                             FW&& written, FS&& synced) {
  using S = DeintShape<PB, NT>;
  constexpr int NO = S::NO, RPP = S::RPP, NR = S::NR;
  const int tid = threadIdx.x;
  const int b0 = by * 64, p0 = bx * 64 * PB;
  const int o = tid % NO, pix = p0 + 8 * o;
  const bool in = pix + 8 <= D;
  bool nb = false;
  // pixels past D: the ones column (pixel D) and zeros
  const unsigned pad = (pix <= D && D < pix + 8) ? 1u << (D - pix) : 0u;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = tid / NO + RPP * i;
    unsigned by3[3] = {pad, pad, pad};
    if (in) {
      const float e[24] = {v[i][0].x, v[i][0].y, v[i][0].z, v[i][0].w, v[i][1].x, v[i][1].y, v[i][1].z, v[i][1].w,
                           v[i][2].x, v[i][2].y, v[i][2].z, v[i][2].w, v[i][3].x, v[i][3].y, v[i][3].z, v[i][3].w,
                           v[i][4].x, v[i][4].y, v[i][4].z, v[i][4].w, v[i][5].x, v[i][5].y, v[i][5].z, v[i][5].w};
      nb |= deint_octet(e, by3);
      xbits[(size_t)(b0 + r) * ldbits + (pix >> 3)] = (unsigned char)by3[1];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) bt[c][o][r] = (unsigned char)by3[c];
  }
  written();
  if (dyn) {
    const bool anb = __ballot(nb) != 0;
    if ((tid & 63) == 0 && anb) atomicOr(dyn + 2, 1);
  }
  __syncthreads();
  synced();
  deint_words<PB, OS, SC1, NOW>(tid, NT, B, D, kts_f, kts_w, xbf, xbw, bx, by, bt);
}

// the whole task (the standalone kernel's workgroup)
template <int PB, int NT, int OS, bool NTL = false, bool NOW = false, bool CO = false>
__device__ __forceinline__ void deint_bits_task(const float4* __restrict__ x, int B, int D, int kts_f, int kts_w,
                                                unsigned* __restrict__ xbf, unsigned* __restrict__ xbw,
                                                unsigned char* __restrict__ xbits, int ldbits,
                                                int* __restrict__ dyn, int bx, int by, DeintLds<PB, OS>& bt,
                                                float4 (*stage)[16][96] = nullptr) {
  float4 v[DeintShape<PB, NT>::NR][6];
  if constexpr (CO) {
    static_assert(PB == 2 && NT == 256, "the coalesced load serves the step's task shape");
    deint_load_co(x, D, bx, by, v, stage);
  } else {
    deint_load<PB, NT, NTL>(x, D, bx, by, v);
  }
  auto none = [] {};
  deint_finish<PB, NT, OS, false, decltype(none)&, decltype(none)&, NOW>(B, D, kts_f, kts_w, xbf, xbw, xbits,
                                                                         ldbits, dyn, bx, by, v, bt, none, none);
}

}  // namespace mvae
