// Internal declarations shared by the libmvae translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstddef>
#include <cstdint>

namespace mvae {

enum EpiMode {
  EPI_STORE = 0,    // C = acc
  EPI_ACT = 1,      // C = act(acc)                     (forward layer, bias folded via ones column)
  EPI_DACT = 2,     // C = acc * act'(aux[remap(row)])  (dgrad through the producing activation)
  EPI_BCE = 3,      // sigmoid + reconstruction BCE row partials + dU = (y - x) * scale (+ optional y)
  EPI_SIGMOID = 4,  // C = sigmoid(acc)                 (generate / reconstruct)
};

enum Act { ACT_TANH = 0, ACT_ELU = 1 };

// GEMM arithmetic: native fp32 MFMA; bf16 operands (fp32 accumulate); fp32-accurate
// 3-term exact bf16 split (see gemm_bf16.hip).
enum GemmPrec { GEMM_F32 = 0, GEMM_BF16 = 1, GEMM_F32X = 2 };

struct GemmEpi {
  int mode = EPI_STORE;
  int act = ACT_TANH;
  const float* aux = nullptr;   // DACT: activation output the gradient flows through
  int ld_aux = 0;
  int remap_split = 1 << 30;    // aux row = row >= remap_split ? row - remap_shift : row
  int remap_shift = 0;
  const float* x = nullptr;     // BCE: target pixels (lock image)
  int ldx = 0;
  float scale = 1.f;            // BCE: 1/global_batch
  float* y = nullptr;           // BCE: optional sigmoid output
  int ldy = 0;
  float* rowpart = nullptr;     // BCE: [M][nblk_n] per-row partial sums of the BCE terms
};

// bf16 operand shadows (precision = bf16). When set, the GEMM reads A/B from these
// instead of the fp32 pointers (same logical layout/ld) and accumulates in fp32.
struct GemmDesc {
  int M = 0, N = 0, K = 0;
  const float* A = nullptr; int lda = 0; bool at = false;  // at: A stored [K][M]
  const float* B = nullptr; int ldb = 0; bool bt = false;  // bt: B stored [N][K]
  float* C = nullptr; int ldc = 0;
  int batch = 1; long long sA = 0, sB = 0, sC = 0;          // per-batch element strides
  const __hip_bfloat16* Ah = nullptr;  // bf16 shadows (nullptr = fp32 operands)
  const __hip_bfloat16* Bh = nullptr;
  __hip_bfloat16* Ch = nullptr;        // optional bf16 copy of the epilogue output (ldc)
  int prec = GEMM_F32;                 // GemmPrec
  int variant = 0;                     // kernel variant (diagnostics / A-B); 0 = default
  int split = 0;                       // forced split-K (0 = planner)
  GemmEpi epi;
};

// Split-K choice for a GEMM (deterministic slab reduction when > 1).
int gemm_plan_split(const GemmDesc& d, size_t max_ws);
// Workspace elements (floats) the GEMM needs for its split-K slabs.
size_t gemm_workspace_elems(const GemmDesc& d);
// Launch. ws: device workspace of >= gemm_workspace_elems(d) floats.
hipError_t gemm_run(const GemmDesc& d, float* ws, size_t ws_elems, hipStream_t st);
namespace gemm { struct Params; }
hipError_t gemm_bf16_launch(const gemm::Params& p, bool at, bool bt, int mode, int epi, hipStream_t st);
// Number of column blocks the BCE epilogue writes per row (rowpart's inner dim).
int gemm_bce_nblk(int N);

// ---- elementwise / reduction kernels (mvae_kernels.hip) ----
hipError_t launch_deinterleave(const float* x, float* xs, __hip_bfloat16* xsh, int B, int D, int ldx,
                               hipStream_t st);
hipError_t launch_normal(float* out, size_t n, uint64_t seed, uint64_t counter, hipStream_t st);
hipError_t launch_latent_fwd(const float* ms, const float* eps, float* z, __hip_bfloat16* zh, int B,
                             int L, int ldz, hipStream_t st);
// out[j] for j in [0, ncols): mode 0 = colsq (z_lock^2 | z_key^2), mode 1 = coldot.
hipError_t launch_colstats(int mode, const float* z, int B, int L, int ldz, const float* colsq,
                           const float* draw, float* part, int nchunk, float* out, hipStream_t st);
int colstats_nchunk(int B);
hipError_t launch_metric(const float* z, int ldz, const float* ms, const float* rowpart, int nblk,
                         const float* areas, const float* colsq, int B, int L, int metric, int recip,
                         float w, float inv_bg, float* rowvals, float* dist, float* draw,
                         hipStream_t st);
hipError_t launch_loss_reduce(const float* rowvals, int B, float inv_bg, float* losses, hipStream_t st);
hipError_t launch_latent_bwd(const float* z, int ldz, const float* ms, const float* eps,
                             const float* dzdec, const float* draw, const float* colsq,
                             const float* coldot, int B, int L, int metric, float w, float inv_bg,
                             float* dhead, __hip_bfloat16* dheadh, hipStream_t st);
struct AdamArgs {
  float* theta; const float* g1; const float* g2; float* m1; float* v1; float* m2; float* v2;
  size_t n_all, n_enc; float lr1, lr2, b1, b2, eps;
  __hip_bfloat16* theta_h;  // optional bf16 shadow refreshed in the same pass
};
hipError_t launch_adam(const AdamArgs& a, hipStream_t st);
hipError_t launch_cast_bf16(const float* src, __hip_bfloat16* dst, size_t n, hipStream_t st);
hipError_t launch_copy2d(const float* src, int lds, float* dst, int ldd, int rows, int cols,
                         hipStream_t st);

}  // namespace mvae
