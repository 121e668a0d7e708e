// bf16-MFMA kernels of the conv tower's 5x5x64x64 layer (conv_tower.hip; bf16 mode), gfx950
// v_mfma_f32_32x32x16_bf16 with fp32 accumulate.
//
// conv2_mfma_kernel — the SAME convolution as an implicit GEMM (forward, and the data gradient
// with the rotated/transposed kernel image): M = output pixels of a band of BR image rows,
// N = 64 output channels, K = 25 taps x 64 input channels. The band's input patch
// ((BR+4) x (S1+4) pixels x 64 channels, zero border) sits in LDS once; each tap's 64x64 kernel
// slice streams through a double-buffered LDS slot (one barrier per tap). A tap is a constant
// shift of every lane's patch address, so the A fragments are plain 16-B ds_read_b128 of the
// shifted pixel rows; 16-B chunks are XOR-swizzled by (pixel>>1)&7 so 16 consecutive pixels hit
// 16 distinct bank slots. 4 waves x (2 M-fragments of 32 pixels) x (2 N-fragments): 256 pixel
// slots; for S1 = 50 a band is 5 rows = 250 pixels. LDS 78.6 KB: two workgroups per CU, so one
// stages its patch while the other computes.
// conv2_mfma_half_kernel (the default) walks the input channels in two halves of 32 with
// 8 waves and 10-row bands at S1 = 50: 56 KB of LDS, two workgroups per CU (the full-channel
// 8-wave form needs 113 KB and runs alone on its CU, every per-tap barrier exposed).
//
// conv2_wgrad_mfma_kernel — dW[t][k][n] = sum_p in[p + t][k] d[p][n]: K = pixels, so both
// operands are pixel-major ([pixel][channel] rows) and are read with ds_read_b64_tr_b16 (each
// lane of a 16-lane group addresses its own pixel row: the tap shift is again a constant
// offset). A workgroup owns one 32-channel half of k and of n for all 25 taps (accumulators
// spread over 4 waves by tap), over a chunk of images; the four (k, n) halves of one chunk are
// placed on the same XCD so their shared operand rows hit that XCD's L2.
#include "mvae_internal.h"
#include <algorithm>

namespace mvae {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int CH = 64, NT = 25;

__device__ __forceinline__ int swz(int px) { return (px >> 1) & 7; }

template <bool FWD, int NW, int TPB, int FPW>
__global__ __launch_bounds__(64 * NW) void conv2_mfma_kernel(const unsigned short* __restrict__ in,
                                                            const unsigned short* __restrict__ wimg,
                                                            const float* __restrict__ bias,
                                                            float* __restrict__ out, int S1, int BR) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int PW = S1 + 4, PR = BR + 4;
  unsigned short* patch = lds;                 // [PR*PW][64], 16-B chunks swizzled
  unsigned short* wb = lds + PR * PW * CH;     // 2 slots x TPB x [64 n][64 k], swizzled by n
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img = blockIdx.y;
  const int y0 = blockIdx.x * BR;
  const int rows = min(BR, S1 - y0);
  const int npx = rows * S1;
  const size_t ibase = (size_t)img * S1 * S1 * CH;
  // a tap's 64x64 slice = 512 16-B chunks, 512 / (64 NW) per thread: chunk q -> n = q/8, k chunk q%8.
  // TPB taps per LDS slot (one barrier per slot); two slots
  constexpr int NT_ = 64 * NW, WCH = NT_ >= 512 ? 1 : 512 / NT_, NG = (NT + TPB - 1) / TPB;
  int4 wr[TPB][WCH];
  auto get_w = [&](int g) {
#pragma unroll
    for (int j = 0; j < TPB; ++j)
#pragma unroll
      for (int u = 0; u < WCH; ++u) {
        const int t = g * TPB + j;
        if (t < NT && tid + NT_ * u < 512)
          wr[j][u] = *reinterpret_cast<const int4*>(wimg + (size_t)t * CH * CH + 8 * (tid + NT_ * u));
      }
  };
  get_w(0);
  for (int i = tid; i < PR * PW * 8; i += NT_) {
    const int px = i >> 3, c = i & 7;
    const int y = y0 - 2 + px / PW, x = px % PW - 2;
    int4 v = make_int4(0, 0, 0, 0);
    if (y >= 0 && y < S1 && x >= 0 && x < S1)
      v = *reinterpret_cast<const int4*>(in + ibase + ((size_t)y * S1 + x) * CH + 8 * c);
    *reinterpret_cast<int4*>(patch + px * CH + 8 * (c ^ swz(px))) = v;
  }
  auto put_w = [&](unsigned short* dst) {
#pragma unroll
    for (int j = 0; j < TPB; ++j)
#pragma unroll
      for (int u = 0; u < WCH; ++u) {
        const int q = tid + NT_ * u, n = q >> 3, c = q & 7;
        if (q < 512) *reinterpret_cast<int4*>(dst + j * CH * CH + n * CH + 8 * (c ^ swz(n))) = wr[j][u];
      }
  };
  put_w(wb);
  __syncthreads();
  const int nfr = (npx + 31) >> 5;
  bool has[FPW];  // wave-uniform
  int pb[FPW];
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    has[i] = wave + NW * i < nfr;
    const int pl = (wave + NW * i) * 32 + (lane & 31);
    const int q = pl < npx ? pl : 0;
    pb[i] = (q / S1) * PW + q % S1;
  }
  const int h = lane >> 5;
  f32x16 acc[FPW][2];
#pragma unroll
  for (int i = 0; i < FPW; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (int g = 0; g < NG; ++g) {
    if (g + 1 < NG) get_w(g + 1);
#pragma unroll
   for (int j = 0; j < TPB; ++j) {
    const int t = g * TPB + j;
    if (t >= NT) break;
    const unsigned short* wc = wb + ((g & 1) * TPB + j) * CH * CH;
    const int toff = (t / 5) * PW + t % 5;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = 2 * ks + h;
      bf16x8 fa[FPW], fb[2];
#pragma unroll
      for (int i = 0; i < FPW; ++i) {
        const int px = pb[i] + toff;
        fa[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(patch + px * CH + 8 * (c ^ swz(px))));
      }
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) {
        const int n = nf * 32 + (lane & 31);
        fb[nf] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(wc + n * CH + 8 * (c ^ swz(n))));
      }
#pragma unroll
      for (int i = 0; i < FPW; ++i)
        if (has[i]) {
          acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[0], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[1], acc[i][1], 0, 0, 0);
        }
    }
   }
    if (g + 1 < NG) put_w(wb + ((g + 1) & 1) * TPB * CH * CH);
    __syncthreads();
  }
  // C: row (pixel) (r&3) + 8(r>>2) + 4h of the fragment, column (channel) lane&31 + 32 nf
  const size_t obase = ibase + (size_t)y0 * S1 * CH;
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    if (!has[i]) continue;
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const int n = nf * 32 + (lane & 31);
      const float b = FWD ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pl = (wave + NW * i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (pl >= npx) continue;
        float v = acc[i][nf][r];
        if (FWD) v = fmaxf(v + b, 0.f);
        out[obase + (size_t)pl * CH + n] = v;
      }
    }
  }
}

// Channel-half form of conv2_mfma_kernel (8 waves, 2 M-fragments each): the 64 input channels
// are walked in two halves of 32, each a full pass over the 25 taps with the band patch and the
// kernel slices of that half only (64-B pixel / kernel rows, 16-B chunks swizzled by (row>>2)&3:
// 16 consecutive rows of one chunk column hit 16 distinct slots of a 256-B bank row). LDS is
// half of the full-channel form's (56 KB at S1 = 50), so two workgroups share a CU and one's
// per-tap barrier and LDS latency overlap the other's MFMAs; the accumulators carry over.
__device__ __forceinline__ int swz4(int r) { return (r >> 2) & 3; }

template <bool FWD>
__global__ __launch_bounds__(512, 2) void conv2_mfma_half_kernel(const unsigned short* __restrict__ in,
                                                                 const unsigned short* __restrict__ wimg,
                                                                 const float* __restrict__ bias,
                                                                 float* __restrict__ out, int S1, int BR) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  constexpr int NW = 8, FPW = 2, HC = 32;
  const int PW = S1 + 4, PR = BR + 4;
  unsigned short* patch = lds;                 // [PR*PW][32]
  unsigned short* wb = lds + PR * PW * HC;     // 2 slots x [64 n][32 k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img = blockIdx.y;
  const int y0 = blockIdx.x * BR;
  const int rows = min(BR, S1 - y0);
  const int npx = rows * S1;
  const size_t ibase = (size_t)img * S1 * S1 * CH;
  // a tap's half slice = 256 16-B chunks: thread q < 256 -> n = q / 4, chunk q % 4
  int4 wr = make_int4(0, 0, 0, 0);
  auto get_w = [&](int hh, int t) {
    if (tid < 256) wr = *reinterpret_cast<const int4*>(wimg + (size_t)t * CH * CH + (tid >> 2) * CH + HC * hh + 8 * (tid & 3));
  };
  auto put_w = [&](unsigned short* dst) {
    const int n = tid >> 2, c = tid & 3;
    if (tid < 256) *reinterpret_cast<int4*>(dst + n * HC + 8 * (c ^ swz4(n))) = wr;
  };
  const int nfr = (npx + 31) >> 5;
  bool has[FPW];  // wave-uniform
  int pb[FPW];
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    has[i] = wave + NW * i < nfr;
    const int pl = (wave + NW * i) * 32 + (lane & 31);
    const int q = pl < npx ? pl : 0;
    pb[i] = (q / S1) * PW + q % S1;
  }
  const int h = lane >> 5;
  f32x16 acc[FPW][2];
#pragma unroll
  for (int i = 0; i < FPW; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (int hh = 0; hh < 2; ++hh) {
    // every read of the previous half ended before the tap loop's last barrier
    get_w(hh, 0);
    for (int i = tid; i < PR * PW * 4; i += 64 * NW) {
      const int px = i >> 2, c = i & 3;
      const int y = y0 - 2 + px / PW, x = px % PW - 2;
      int4 v = make_int4(0, 0, 0, 0);
      if (y >= 0 && y < S1 && x >= 0 && x < S1)
        v = *reinterpret_cast<const int4*>(in + ibase + ((size_t)y * S1 + x) * CH + HC * hh + 8 * c);
      *reinterpret_cast<int4*>(patch + px * HC + 8 * (c ^ swz4(px))) = v;
    }
    put_w(wb);
    __syncthreads();
    for (int t = 0; t < NT; ++t) {
      if (t + 1 < NT) get_w(hh, t + 1);
      const unsigned short* wc = wb + (t & 1) * CH * HC;
      const int toff = (t / 5) * PW + t % 5;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = 2 * ks + h;
        bf16x8 fa[FPW], fb[2];
#pragma unroll
        for (int i = 0; i < FPW; ++i) {
          const int px = pb[i] + toff;
          fa[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(patch + px * HC + 8 * (c ^ swz4(px))));
        }
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          const int n = nf * 32 + (lane & 31);
          fb[nf] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(wc + n * HC + 8 * (c ^ swz4(n))));
        }
#pragma unroll
        for (int i = 0; i < FPW; ++i)
          if (has[i]) {
            acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[0], acc[i][0], 0, 0, 0);
            acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[1], acc[i][1], 0, 0, 0);
          }
      }
      if (t + 1 < NT) put_w(wb + ((t + 1) & 1) * CH * HC);
      __syncthreads();
    }
  }
  const size_t obase = ibase + (size_t)y0 * S1 * CH;
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    if (!has[i]) continue;
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const int n = nf * 32 + (lane & 31);
      const float b = FWD ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pl = (wave + NW * i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (pl >= npx) continue;
        float v = acc[i][nf][r];
        if (FWD) v = fmaxf(v + b, 0.f);
        out[obase + (size_t)pl * CH + n] = v;
      }
    }
  }
}

// Weight gradient. The next row block's operand rows are fetched into registers (NA + 4 16-B
// chunks per thread) while the current block computes. Grid: 8 * ceil(2 * nchunk * 4 / 8) workgroups; id -> (XCD = id & 7,
// sibling s = (id >> 3) & 3 = k half * 2 + n half, chunk group). LDS: the image rows of one row
// block [r0, r0 + R) for one channel half: A patch (R+4) x (S1+4) x 32 and d 16*nk x 32 (64-B
// pixel rows: four consecutive pixels of a tr16 group span the 256-B bank row, no swizzle).
template <int NA>
__global__ __launch_bounds__(256, 2) void conv2_wgrad_mfma_kernel(const unsigned short* __restrict__ inb,
                                                                  const unsigned short* __restrict__ db,
                                                                  int S1, int R, int B2, int nchunk, int ipc,
                                                                  float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int PW = S1 + 4;
  const int nslot = ((R * S1 + 15) / 16) * 16;   // pixel slots of a row block (k16 steps * 16)
  unsigned short* ap = lds;                      // [(R+4)*PW][32]
  unsigned short* dp = lds + (R + 4) * PW * 32;  // [nslot][32]
  const int id = blockIdx.x;
  const int xcd = id & 7, sib = (id >> 3) & 3, cgi = (id >> 5) * 8 + xcd;
  if (cgi >= 2 * nchunk) return;                 // workgroup-uniform
  const int grp = cgi / nchunk, chunk = cgi % nchunk;
  const int kh = sib >> 1, nh = sib & 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = grp * B2 + chunk * ipc;
  const int j1 = min(j0 + ipc, grp * B2 + B2);
  const int np1 = S1 * S1;
  const int nrb = (S1 + R - 1) / R;              // row blocks per image
  const int nb = j1 > j0 ? (j1 - j0) * nrb : 0;  // row blocks of this workgroup
  const int nA = (R + 4) * PW * 4, nD = nslot * 4;  // 16-B chunks of the two LDS images
  // taps of this wave: wave, wave + 4, ... (7, 6, 6, 6); bias (ones A fragment) on wave 3 of kh 0
  constexpr int MT = 7;
  f32x16 acc[MT], accb;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) accb[r] = 0.f;
  const bool dobias = kh == 0 && wave == 3;
  const int i16 = lane & 15, q = i16 >> 2, pq = i16 & 3, h = lane >> 5, g1 = (lane >> 4) & 1;
  const int col = 16 * g1 + 4 * pq;             // this lane's 4-element column chunk
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  // the next row block's operand rows are loaded into registers while the current one computes
  int4 ra[NA], rd[4];
  auto fetch = [&](int b) {
    const int j = j0 + b / nrb, r0 = (b % nrb) * R;
    const int f = j < B2 ? j : j - B2 / 2;
    const int npx = min(R, S1 - r0) * S1;
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int i = tid + 256 * u;
      ra[u] = make_int4(0, 0, 0, 0);
      if (i < nA) {
        const int px = i >> 2, c = i & 3;
        const int y = r0 - 2 + px / PW, x = px % PW - 2;
        if (y >= 0 && y < S1 && x >= 0 && x < S1)
          ra[u] = *reinterpret_cast<const int4*>(inb + ((size_t)f * np1 + y * S1 + x) * CH + 32 * kh + 8 * c);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + 256 * u;
      rd[u] = make_int4(0, 0, 0, 0);
      if (i < nD && (i >> 2) < npx)
        rd[u] = *reinterpret_cast<const int4*>(db + ((size_t)j * np1 + (size_t)r0 * S1 + (i >> 2)) * CH + 32 * nh + 8 * (i & 3));
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int i = tid + 256 * u;
      if (i < nA) *reinterpret_cast<int4*>(ap + (i >> 2) * 32 + 8 * (i & 3)) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + 256 * u;
      if (i < nD) *reinterpret_cast<int4*>(dp + (i >> 2) * 32 + 8 * (i & 3)) = rd[u];
    }
  };
  if (nb > 0) {
    fetch(0);
    commit();
  }
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    const int r0 = (b % nrb) * R;
    const int npx = min(R, S1 - r0) * S1;
    if (b + 1 < nb) fetch(b + 1);
    for (int s = 0; s < nslot / 16; ++s) {
      const int klo = 16 * s + 8 * h + q, khi = klo + 4;
      const int plo = klo < npx ? klo : 0, phi = khi < npx ? khi : 0;
      const int alo = (plo / S1) * PW + plo % S1, ahi = (phi / S1) * PW + phi % S1;
      const s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(dp + klo * 32 + col));
      const s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(dp + khi * 32 + col));
      const bf16x8 fb = __builtin_bit_cast(bf16x8, __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int t = wave + 4 * i;
        if (t >= NT) break;
        const int toff = (t / 5) * PW + t % 5;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ap + (alo + toff) * 32 + col));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ap + (ahi + toff) * 32 + col));
        const bf16x8 fa = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[i], 0, 0, 0);
      }
      if (dobias) accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, fb, accb, 0, 0, 0);
    }
    __syncthreads();
    if (b + 1 < nb) commit();
    __syncthreads();
  }
  float* out = slab + ((size_t)grp * nchunk + chunk) * (NT * CH + 1) * CH;
  const int n = 32 * nh + (lane & 31);
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int t = wave + 4 * i;
    if (t >= NT) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * h;
      out[(size_t)(t * CH + k) * CH + n] = acc[i][r];
    }
  }
  if (dobias && h == 0) out[(size_t)NT * CH * CH + n] = accb[0];
}

// Weight gradient, 8-wave form: a workgroup owns one 32-channel half of k and ALL 64 n for the
// 25 taps (waves take taps w, w+8, ...: 4,3,...,3 taps x 2 n-halves of accumulators), so one
// B fragment pair (both n halves) serves every tap of the wave and only the two k halves of a
// chunk read the same d rows. d rows are 128 B (64 n): 16-B chunks of rows with (p>>1)&1 swap
// their 64-B halves, so the four rows of a tr16 group hit four distinct 64-B bank groups.
// Grid: 8 * ceil(2 * nchunk * 2 / 8); id -> (XCD = id & 7, k half = (id >> 3) & 1, chunk group).
template <int NA>
__global__ __launch_bounds__(512) void conv2_wgrad_mfma8_kernel(const unsigned short* __restrict__ inb,
                                                                const unsigned short* __restrict__ db,
                                                                int S1, int R, int B2, int nchunk, int ipc,
                                                                float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int PW = S1 + 4;
  const int nslot = ((R * S1 + 15) / 16) * 16;
  unsigned short* ap = lds;                      // [(R+4)*PW][32]
  unsigned short* dp = lds + (R + 4) * PW * 32;  // [nslot][64], 64-B halves swapped by (p>>1)&1
  // patch row of each pixel slot of a row block: ptab[p] = (p / S1) * PW + p % S1
  int* ptab = reinterpret_cast<int*>(dp + ((R * S1 + 15) / 16 * 16) * 64);
  const int id = blockIdx.x;
  const int xcd = id & 7, kh = (id >> 3) & 1, cgi = (id >> 4) * 8 + xcd;
  if (cgi >= 2 * nchunk) return;                 // workgroup-uniform
  const int grp = cgi / nchunk, chunk = cgi % nchunk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = grp * B2 + chunk * ipc;
  const int j1 = min(j0 + ipc, grp * B2 + B2);
  const int np1 = S1 * S1;
  const int nrb = (S1 + R - 1) / R;
  const int nb = j1 > j0 ? (j1 - j0) * nrb : 0;
  const int nA = (R + 4) * PW * 4, nD = nslot * 8;
  constexpr int MT = 4;                          // taps per wave (at most)
  f32x16 acc[MT][2], accb[2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][n2][r] = 0.f;
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2)
#pragma unroll
    for (int r = 0; r < 16; ++r) accb[n2][r] = 0.f;
  const bool dobias = kh == 0 && wave == 7;      // wave 7 holds 3 taps: room for the bias rows
  for (int p = tid; p < nslot; p += 512) ptab[p] = (p / S1) * PW + p % S1;   // read after 1st barrier
  const int i16 = lane & 15, q = i16 >> 2, pq = i16 & 3, h = lane >> 5, g1 = (lane >> 4) & 1;
  const int col = 16 * g1 + 4 * pq;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  int4 ra[NA], rd[4];
  // this thread's A-image chunks sit at the same (patch row, column) in every row block
  int arow[NA], acol[NA];
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int px = (tid + 512 * u) >> 2;
    arow[u] = px / PW;
    acol[u] = px - arow[u] * PW - 2;
  }
  auto fetch = [&](int b) {
    const int j = j0 + b / nrb, r0 = (b % nrb) * R;
    const int f = j < B2 ? j : j - B2 / 2;
    const int npx = min(R, S1 - r0) * S1;
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int i = tid + 512 * u;
      ra[u] = make_int4(0, 0, 0, 0);
      if (i < nA) {
        const int c = i & 3;
        const int y = r0 - 2 + arow[u], x = acol[u];
        if (y >= 0 && y < S1 && x >= 0 && x < S1)
          ra[u] = *reinterpret_cast<const int4*>(inb + ((size_t)f * np1 + y * S1 + x) * CH + 32 * kh + 8 * c);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + 512 * u;
      rd[u] = make_int4(0, 0, 0, 0);
      if (i < nD && (i >> 3) < npx)
        rd[u] = *reinterpret_cast<const int4*>(db + ((size_t)j * np1 + (size_t)r0 * S1 + (i >> 3)) * CH + 8 * (i & 7));
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int i = tid + 512 * u;
      if (i < nA) *reinterpret_cast<int4*>(ap + (i >> 2) * 32 + 8 * (i & 3)) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + 512 * u;
      const int p = i >> 3, c = (i & 7) ^ (((p >> 1) & 1) << 2);
      if (i < nD) *reinterpret_cast<int4*>(dp + p * 64 + 8 * c) = rd[u];
    }
  };
  if (nb > 0) {
    fetch(0);
    commit();
  }
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    const int r0 = (b % nrb) * R;
    const int npx = min(R, S1 - r0) * S1;
    if (b + 1 < nb) fetch(b + 1);
    for (int s = 0; s < nslot / 16; ++s) {
      const int klo = 16 * s + 8 * h + q, khi = klo + 4;
      const int plo = klo < npx ? klo : 0, phi = khi < npx ? khi : 0;
      const int alo = ptab[plo], ahi = ptab[phi];
      bf16x8 fb[2];
#pragma unroll
      for (int n2 = 0; n2 < 2; ++n2) {
        const int clo = (32 * n2 + col) ^ (((klo >> 1) & 1) << 5);
        const int chi = (32 * n2 + col) ^ (((khi >> 1) & 1) << 5);
        const s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(dp + klo * 64 + clo));
        const s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(dp + khi * 64 + chi));
        fb[n2] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int t = wave + 8 * i;
        if (t >= NT) break;
        const int toff = (t / 5) * PW + t % 5;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ap + (alo + toff) * 32 + col));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ap + (ahi + toff) * 32 + col));
        const bf16x8 fa = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb[0], acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb[1], acc[i][1], 0, 0, 0);
      }
      if (dobias) {
        accb[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, fb[0], accb[0], 0, 0, 0);
        accb[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, fb[1], accb[1], 0, 0, 0);
      }
    }
    __syncthreads();
    if (b + 1 < nb) commit();
    __syncthreads();
  }
  float* out = slab + ((size_t)grp * nchunk + chunk) * (NT * CH + 1) * CH;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int t = wave + 8 * i;
    if (t >= NT) break;
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = 32 * kh + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(size_t)(t * CH + k) * CH + 32 * n2 + (lane & 31)] = acc[i][n2][r];
      }
  }
  if (dobias && h == 0)
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) out[(size_t)NT * CH * CH + 32 * n2 + (lane & 31)] = accb[n2][0];
}

// bf16 kernel images of conv2 for the MFMA kernels, [t][n][k] (k contiguous):
// forward  wf[t][n][k] = W[t*64 + k][n];  data gradient  wd[t][n][k] = W[(24 - t)*64 + n][k]
__global__ void conv2_wprep_kernel(const float* __restrict__ W, unsigned short* __restrict__ wf,
                                   unsigned short* __restrict__ wd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NT * CH * CH) return;
  const int t = i / (CH * CH), n = (i / CH) % CH, k = i % CH;
  wf[i] = __builtin_bit_cast(unsigned short, __float2bfloat16(W[(size_t)(t * CH + k) * CH + n]));
  wd[i] = __builtin_bit_cast(unsigned short, __float2bfloat16(W[(size_t)((NT - 1 - t) * CH + n) * CH + k]));
}

}  // namespace

// band rows of the forward / data-gradient kernel with nw waves (64 nw pixel slots)
int conv2_mfma_band(int S1, int nw, int tpb, int fpw) {
  const size_t wlds = (size_t)2 * tpb * CH * CH * 2;   // two slots of TPB taps
  int br = std::max(1, std::min(S1, 32 * nw * fpw / S1));
  while (br > 1 && (size_t)(br + 4) * (S1 + 4) * CH * 2 + wlds > 160 * 1024) --br;
  return br;
}

size_t conv2_mfma_lds(int S1, int nw, int tpb, int fpw) {
  const int br = conv2_mfma_band(S1, nw, tpb, fpw);
  return (size_t)(br + 4) * (S1 + 4) * CH * 2 + (size_t)2 * tpb * CH * CH * 2;
}

int conv2_wgrad_rows(int S1) { return std::max(1, std::min(S1, 256 / S1)); }

size_t conv2_wgrad_lds(int S1) {
  const int R = conv2_wgrad_rows(S1);
  const size_t nslot = ((size_t)R * S1 + 15) / 16 * 16;
  return ((size_t)(R + 4) * (S1 + 4) + nslot) * 32 * 2;
}

hipError_t launch_conv2_wprep(const ConvTower& T, const float* w2, hipStream_t st) {
  hipLaunchKernelGGL(conv2_wprep_kernel, dim3((NT * CH * CH + 255) / 256), dim3(256), 0, st, w2, T.w2f, T.w2d);
  return hipGetLastError();
}

hipError_t launch_conv2_mfma(const ConvTower& T, bool fwd, const unsigned short* inb,
                             const unsigned short* wimg, const float* w2, float* out, int nimg,
                             hipStream_t st) {
  const int nw = T.conv2_nw == 16 ? 16 : (T.conv2_nw == 8 ? 8 : 4);
  const int tpb = nw == 8 && T.conv2_tpb == 2 ? 2 : 1;
  const int fpw = nw == 16 ? 1 : (nw == 4 && T.conv2_fpw == 4 ? 4 : 2);
  const int br = conv2_mfma_band(T.S1, nw, tpb, fpw);
  const size_t lds = conv2_mfma_lds(T.S1, nw, tpb, fpw);
  dim3 g((T.S1 + br - 1) / br, nimg);
  const float* bias = w2 + (size_t)NT * CH * CH;
#define CONV2_LAUNCH(NW_, TPB_, FPW_)                                                              \
  do {                                                                                             \
    if (fwd)                                                                                       \
      hipLaunchKernelGGL((conv2_mfma_kernel<true, NW_, TPB_, FPW_>), g, dim3(64 * NW_), lds, st,   \
                         inb, wimg, bias, out, T.S1, br);                                          \
    else                                                                                           \
      hipLaunchKernelGGL((conv2_mfma_kernel<false, NW_, TPB_, FPW_>), g, dim3(64 * NW_), lds, st,  \
                         inb, wimg, bias, out, T.S1, br);                                          \
  } while (0)
  if (T.conv2_half) {
    // channel-half form: band of 512 pixel slots, 2 workgroups per CU
    const int hbr = std::max(1, std::min(T.S1, 512 / T.S1));
    const size_t hlds = ((size_t)(hbr + 4) * (T.S1 + 4) * 32 + (size_t)2 * CH * 32) * 2;
    dim3 hg((T.S1 + hbr - 1) / hbr, nimg);
    if (fwd)
      hipLaunchKernelGGL((conv2_mfma_half_kernel<true>), hg, dim3(512), hlds, st, inb, wimg, bias, out, T.S1, hbr);
    else
      hipLaunchKernelGGL((conv2_mfma_half_kernel<false>), hg, dim3(512), hlds, st, inb, wimg, bias, out, T.S1, hbr);
    return hipGetLastError();
  }
  if (nw == 16) CONV2_LAUNCH(16, 1, 1);
  else if (nw == 8 && tpb == 2) CONV2_LAUNCH(8, 2, 2);
  else if (nw == 8) CONV2_LAUNCH(8, 1, 2);
  else if (fpw == 4) CONV2_LAUNCH(4, 1, 4);
  else CONV2_LAUNCH(4, 1, 2);
#undef CONV2_LAUNCH
  return hipGetLastError();
}

hipError_t launch_conv2_wgrad_mfma(const ConvTower& T, int B, hipStream_t st) {
  const int B2 = 2 * B;
  const int nchunk = T.nchunk2m, ipc = (B2 + nchunk - 1) / nchunk;
  const int groups8 = (2 * nchunk + 7) / 8;
  const int R = conv2_wgrad_rows(T.S1);
  const int chunks = (R + 4) * (T.S1 + 4) * 4;   // 16-B chunks of the A image per thread block
  if (T.conv2_wg8 && (size_t)((R * T.S1 + 15) / 16 * 16) * 8 <= 4 * 512) {
    const int g16 = (2 * nchunk + 7) / 8;
    const size_t nsl = (size_t)(R * T.S1 + 15) / 16 * 16;
    const size_t lds = ((size_t)(R + 4) * (T.S1 + 4) * 32 + nsl * 64) * 2 + nsl * 4;
    if (chunks <= 4 * 512)
      hipLaunchKernelGGL(conv2_wgrad_mfma8_kernel<4>, dim3(g16 * 16), dim3(512), lds, st, T.n1b, T.da2b, T.S1,
                         R, B2, nchunk, ipc, T.slab);
    else if (chunks <= 8 * 512)
      hipLaunchKernelGGL(conv2_wgrad_mfma8_kernel<8>, dim3(g16 * 16), dim3(512), lds, st, T.n1b, T.da2b, T.S1,
                         R, B2, nchunk, ipc, T.slab);
    else
      return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (chunks <= 8 * 256)
    hipLaunchKernelGGL(conv2_wgrad_mfma_kernel<8>, dim3(groups8 * 32), dim3(256), conv2_wgrad_lds(T.S1), st,
                       T.n1b, T.da2b, T.S1, R, B2, nchunk, ipc, T.slab);
  else if (chunks <= 16 * 256)
    hipLaunchKernelGGL(conv2_wgrad_mfma_kernel<16>, dim3(groups8 * 32), dim3(256), conv2_wgrad_lds(T.S1), st,
                       T.n1b, T.da2b, T.S1, R, B2, nchunk, ipc, T.slab);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace mvae
