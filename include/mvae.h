/*
 * mvae.h — C ABI of libmvae, the MI355X (gfx950) training step of the "magic"
 * asymmetric metric-VAE (reference: ag8/magic, class TangoEncoder).
 *
 * The reference has no FFI: its "operator API" is the Python class
 * TangoEncoder(sess) driven through tf.Session.run (11a/vae.py:13,22) and fed by
 * overlap_input.inputs() (11a/overlap_input.py:76). Each entry point below replaces
 * one of those graph evaluations; the Python mirror of the reference interface
 * (magic_amd/vae.py) binds them through ctypes. Plain pointers and sizes only:
 * every float* argument is a DEVICE pointer owned by the caller unless stated.
 *
 *   reference call (file:line)                      -> entry point(s)
 *   TangoEncoder.__init__  11a/vae.py:22-332         -> mvae_create (+ mvae_param_* for init)
 *   partial_fit            11a/vae.py:385-411        -> mvae_train_step
 *                                                      = mvae_forward, mvae_metric,
 *                                                        mvae_backward, mvae_adam
 *                                                      (split so a data-parallel host can
 *                                                       all-reduce between the phases)
 *   get_predictions        11a/vae.py:413-414        -> mvae_predict
 *   transform              11a/vae.py:416-420        -> mvae_transform
 *   generate               11a/vae.py:422-434        -> mvae_generate
 *   reconstruct            11a/vae.py:436-440        -> mvae_reconstruct
 *
 * Errors: 0 = ok; <0 = invalid argument / configuration (MVAE_E*); >0 = hipError_t.
 * No exception crosses the ABI; mvae_last_error() returns a message.
 * Threading: one context per device per process; a context is not thread-safe;
 * all work is enqueued on the caller's stream (hipStream_t passed as void*).
 */
#ifndef MVAE_H_
#define MVAE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVAE_ABI_VERSION 4
#define MVAE_MAX_ENC 8

enum { MVAE_OK = 0, MVAE_EINVAL = -1, MVAE_ECONFIG = -2, MVAE_ESTATE = -3 };
enum { MVAE_ACT_TANH = 0, MVAE_ACT_ELU = 1 };                    /* 8c family : 11a */
enum { MVAE_METRIC_COSINE = 0, MVAE_METRIC_SQDIFF = 1 };        /* 11a/constants.py:5-7 */
/* GEMM arithmetic: F32 = native fp32 MFMA; BF16 = bf16 operands, fp32 accumulate;
 * F32X = fp32-accurate: every fp32 operand split exactly into 3 bf16 terms, products
 * a_i*b_j with i+j<3 on bf16 MFMA, fp32 accumulate (exact-bf16 tiles take 1 term). */
enum { MVAE_PREC_F32 = 0, MVAE_PREC_BF16 = 1, MVAE_PREC_F32X = 2 };

/* Hyper-parameters the reference hard-codes in TangoEncoder.__init__ (11a/vae.py:30-65)
 * and FLAGS (11a/constants.py:32,49,52,60). */
typedef struct mvae_cfg {
  int image_size;        /* H = W; D = H*W pixels per image                    */
  int batch;             /* rows per call on this rank (FLAGS.BATCH_SIZE)      */
  int global_batch;      /* rows over all ranks; losses/grads scale by 1/global */
  int n_enc;             /* encoder depth (1..MVAE_MAX_ENC)                    */
  int enc[MVAE_MAX_ENC]; /* encoder widths, 11a/vae.py:30                      */
  int dec[2];            /* decoder widths, fixed [500,500] (11a/vae.py:36)    */
  int latent;            /* L, 11a/vae.py:49                                   */
  int act;               /* MVAE_ACT_*                                          */
  int metric;            /* MVAE_METRIC_*                                       */
  int reciprocal;        /* distance = 1/raw (11a/vae.py:307,309)              */
  float deform_weight;   /* 10 (8c/vae.py:287) or 100 (11a/vae.py:293)         */
  float lr[2];           /* [cost optimizer, metric optimizer]                 */
  float beta1, beta2, epsilon; /* TF AdamOptimizer defaults .9/.999/1e-8       */
  int precision;         /* MVAE_PREC_*                                         */
  uint64_t seed;         /* counter-based N(0,1) stream for eps when not given */
  int conv;              /* 1: conv-encoder variant (BASELINE config 5): the CifarNet
                            tower of 6b/net.py:50-60 (conv5x5x64, pool, LRN, conv5x5x64,
                            LRN, pool; weights shared by the three encoder passes) in front
                            of the FC encoder, whose first layer then reads the (S/4)^2*64
                            tower features. Variables enc_conv{1,2}_{W,b} come first in
                            mvae_param_info order (W as [25*c_in, 64], TF HWIO flattened).
                            Needs image_size % 4 == 0. bf16 precision runs the 64->64 conv
                            on MFMA; f32 / f32x run the tower in fp32. 0: FC encoder.  */
} mvae_cfg;

typedef struct mvae_ctx mvae_ctx;

/* Named views into context-owned device memory. */
enum {
  MVAE_KIND_PARAM = 0, MVAE_KIND_GRAD1 = 1, MVAE_KIND_GRAD2 = 2,
  MVAE_KIND_M1 = 3, MVAE_KIND_V1 = 4, MVAE_KIND_M2 = 5, MVAE_KIND_V2 = 6
};
typedef struct mvae_tensor {
  char name[48];    /* reference variable meaning, e.g. "enc_h0_W", "dec_out_mean_b" */
  float* data;      /* device pointer of element [0][0]                               */
  int rows, cols;   /* logical shape (a bias is rows=1)                                */
  int ld;           /* row stride in elements                                          */
  int trained_by;   /* bit0: cost optimizer, bit1: metric optimizer, 0: dead variable  */
} mvae_tensor;

/* Flat buffers (for checkpoints and the data-parallel gradient all-reduce). */
enum {
  MVAE_BUF_PARAMS = 0,   /* all trained parameters (augmented [W;b] blocks)            */
  MVAE_BUF_GRADS = 1,    /* [g1 (all trained) | g2 (encoder)] — the all-reduce bucket  */
  MVAE_BUF_ADAM = 2,     /* [m1 | v1 | m2 | v2]                                        */
  MVAE_BUF_LOSSES = 3,   /* float[8]: cost, training_loss, r_l, l_l, d_l (rank-local
                            partial sums scaled by 1/global_batch; global after a sum)  */
  MVAE_BUF_COLSQ = 4,    /* float[2L]: sum_b z_lock^2, sum_b z_key^2 (cosine metric)    */
  MVAE_BUF_COLDOT = 5,   /* float[L]:  sum_b draw_b n_lock n_key     (cosine metric)    */
  MVAE_BUF_DIST = 6,     /* float[B]: distance of the last forward                      */
  MVAE_BUF_GRADS_DEC = 7,/* decoder slice of g1 (ready first in mvae_backward)         */
  MVAE_BUF_DEAD = 8,     /* the never-trained decoder log-sigma variables               */
  MVAE_BUF_EPS = 9,      /* float[3,B,L]: eps of the last forward (given or generated).  */
                         /* A generated draw is regenerated inside the latent kernels and */
                         /* written to this buffer only when it is requested: the call    */
                         /* synchronises the device (hipDeviceSynchronize) and the pointer */
                         /* holds the draw of the forward BEFORE the call -- re-fetch it  */
                         /* after every forward whose eps you read.                        */
  MVAE_BUF_DYN = 10      /* int32[1] (count 1): nonzero when the last batch's pixels are
                            not all exact in bf16 (f32x: the layer-0 GEMMs then run all 6
                            plane pairs instead of 3; bf16/f32x: the BCE target is read in
                            fp32 instead of bf16); absent in f32 mode. The flag alternates
                            between two slots batch by batch: re-fetch the pointer after
                            each forward                                                    */
};

int mvae_abi_version(void);
/* Build id: the first 16 hex digits of the SHA-256 of the library's sources (magic_amd/csrc/*
 * and this header) at compile time (magic_amd/build.py source_hash). The Python loader refuses
 * a library whose id differs from the sources on disk, so a stale libmvae.so fails loudly. */
const char* mvae_build_id(void);
int mvae_create(const mvae_cfg* cfg, int device, mvae_ctx** out);
/* mvae_create with plan-time kernel switches (A/B and tests; NULL or "" = the defaults, which are
 * the measured best plans): "name=value[,name=value...]" with e8 (256-row bf16 GEMMs: 1 planner,
 * 0 ring kernels only, 2 the eight-phase kernel wherever a 256-row kernel runs), thin_ring (0-2),
 * valu (0/1), dact_planes (0/1), bce_split (0/1), plan_log (0/1: GEMM plans on stderr),
 * conv2_half (0/1), conv2_nw (4/8/16), conv2_tpb (1/2), conv2_fpw (2/4), conv2_wg (4/8),
 * conv2_nchunk (> 0), enc_chain (0/1: bf16 mode, the encoder's hidden layers in one launch,
 * default 1), enc_chain_rows (its rows per workgroup, 16..96; 0 auto; both chains), dec_chain
 * (0/1: bf16 mode, the decoder's two hidden layers in one launch, default 1), bits (0/1: bf16 and
 * f32x modes, the layer-0 pixel operand of a 0/1 batch as one bit per pixel -- the de-interleave
 * writes BitMats instead of the bf16 plane and the eight-phase kernel expands the A fragments in
 * registers; a batch with another pixel value takes the planes; default 1), bits_reg (0/1: each
 * wave loads its A words straight to registers, else through an LDS copy of the block; default
 * 1), deint_fuse (0/1: the de-interleave's workers inside the layer-0 forward's launch beside its
 * tiles, handing chunks over by counters; measured slower, default 0), xbw_split (0/1/2: the
 * weight gradient's BitMat transposed from the forward's on the side stream instead of written by
 * the de-interleave; 2 = where the layer-0 forward leaves CUs idle, default), adam_nt (0/1: Adam's
 * moments and fp32 parameters stored non-temporal, default 1), e8_prio (0-2, A/B: the eight-phase
 * kernel's s_setprio form, default 0), deint_variant (0-6 or 8, A/B: the de-interleave's form; 8 = coalesced X loads through LDS), cs_one
 * (0-2: the cosine metric's column statistics in one launch, the last row chunk's workgroup
 * summing the partials in the two-launch order -- the same bits; 2, the default: where L <= 32),
 * x3 (0-2: f32x ring-kernel plans on the plane-stacked kernels, every operand plane of a k-tile in
 * LDS at once -- 1 the tile-N-128 plans, 2 also the 256x256 ones; the same products summed in
 * another order; default 2). Diagnostics, results
 * meaningless: deint_fuse_diag (0-31: parts of the fused launch switched off), diag_skip_deint (1: de-interleave only the first batch -- a timing bound),
 * diag_shadow_deint (-1 or a workgroup count > 0: a second de-interleave of each step's input
 * into a scratch image on a low-priority stream, launched at diag_shadow_at = 0 the forward,
 * 1 the backward, 2 the encoder backward -- the cost of staging), diag_chain (enc_chain's
 * ablations: 1 no weight DMA past the first steps, 2 no MFMAs, 4 no copy-out; bits combine).
 * An unknown name or a value out of range is MVAE_EINVAL. The library reads no environment
 * variables (the diagnostics entry point mvae_bench_gemm aside). */
int mvae_create_ex(const mvae_cfg* cfg, int device, const char* options, mvae_ctx** out);
int mvae_destroy(mvae_ctx* ctx);
const char* mvae_last_error(mvae_ctx* ctx);   /* ctx may be NULL (creation errors) */

int mvae_param_count(mvae_ctx* ctx);
int mvae_param_info(mvae_ctx* ctx, int kind, int index, mvae_tensor* out);
int mvae_buffer(mvae_ctx* ctx, int which, float** ptr, size_t* count);
/* Optimizer step counters (TF beta1_power/beta2_power, kept on the host in fp32). */
int mvae_get_step(mvae_ctx* ctx, int64_t* t1, int64_t* t2);
int mvae_set_step(mvae_ctx* ctx, int64_t t1, int64_t t2);
/* Philox call counters of the internal N(0,1) sampler (eps == NULL): training draws
 * (mvae_forward / mvae_train_step) and inference draws (mvae_predict / mvae_reconstruct)
 * are separate streams, so evaluation never shifts the training noise; save both with a
 * checkpoint to resume the exact sequence. Counters must be < 2^63. */
/* Data parallelism: this rank's rows start at row_offset of the global batch (default 0).
 * The internal sampler then draws exactly this rank's slice of the eps a single process
 * would draw for the whole global batch. 0 <= row_offset <= global_batch - batch. */
int mvae_set_shard(mvae_ctx* ctx, int64_t row_offset);
int mvae_get_rng(mvae_ctx* ctx, uint64_t* train, uint64_t* eval);
int mvae_set_rng(mvae_ctx* ctx, uint64_t train, uint64_t eval);
/* Re-derive the bf16 plane images of the parameters from the fp32 masters: call after
 * writing parameters through mvae_param_info views (bf16 / f32x modes; no-op for f32). */
int mvae_sync_params(mvae_ctx* ctx, void* stream);

/* ---- training step, phase by phase --------------------------------------------- */
/* x: [B, 3*D] f32 HWC-interleaved (lock, rotated lock, key), 11a/overlap_input.py:117-119.
 * eps: [3, B, L] f32 in the reference's draw order (lock, rotated, key), or NULL to draw
 * from the context's counter-based generator (seed, call counter).                   */
int mvae_forward(mvae_ctx* ctx, const float* x, const float* eps, void* stream);
/* areas: [B] f32. Needs MVAE_BUF_COLSQ summed over ranks (cosine) before the call.    */
int mvae_metric(mvae_ctx* ctx, const float* areas, void* stream);
/* Needs MVAE_BUF_COLDOT summed over ranks (cosine). Writes MVAE_BUF_GRADS.           */
int mvae_backward(mvae_ctx* ctx, void* stream);
/* The same backward in mvae_backward_nparts(ctx) = R + 2 parts, R = option "wgrad0_chunks"
 * (0: decoder; 1: latent head, encoder dgrad chain and layer-0 weight-gradient chunk 0;
 * 2 .. R: layer-0 chunks 1 .. R-1; R + 1: the remaining encoder weight gradients). After
 * part k the ranges mvae_grad_range(ctx, k, i = 0, 1, ...) are final: a data-parallel host
 * all-reduces them while the later parts run (returns MVAE_EINVAL past the last range). Over
 * all parts the ranges cover MVAE_BUF_GRADS exactly once. */
int mvae_backward_nparts(mvae_ctx* ctx);
int mvae_backward_part(mvae_ctx* ctx, int part, void* stream);
int mvae_grad_range(mvae_ctx* ctx, int part, int index, float** ptr, size_t* count);
/* Schedule switches: "side_stream" (default 1) runs the weight gradients on a context-owned
 * side stream beside the dgrad chain, joined before the gradients they write are reported
 * final (mvae_backward / the end of each mvae_backward_part); "wgrad0_chunks" (1, 2, 4, 8;
 * default 1) splits the layer-0 weight gradient (40 MB of the 69 MB bucket at C4) into row
 * chunks that finish -- and can be all-reduced -- one after another; "early_adam" (default 0)
 * lets mvae_adam update the blocks after the layer-0 block on the side stream as soon as the
 * backward has written their gradients (beside the layer-0 weight gradient): only for callers
 * that neither read nor modify MVAE_BUF_GRADS between mvae_backward and mvae_adam (no
 * all-reduce): the caller's stream then joins the side stream in mvae_adam;
 * mvae_train_step uses it in the bf16 and f32x modes; "early_chunks" (1, 2, 4, 8; default 1):
 * with the early Adam and "wgrad0_chunks" 1, mvae_backward runs the layer-0 weight gradient in
 * that many row chunks and updates each chunk's parameter rows but the last's on the side stream
 * beside the next chunk's GEMM, i.e. already inside mvae_backward (so with early_adam the
 * parameters, their Adam state and MVAE_BUF_GRADS are not to be read between mvae_backward and
 * mvae_adam; 1: one GEMM, everything in mvae_adam); "bce_split" (default 1) runs a BCE head whose
 * 256x256 tiles leave a partial last round as the whole rounds plus 256x128 tiles for the rest
 * (bitwise the same results in bf16; in f32x equal to fp32 rounding: the two kernels sum the plane
 * pairs in different orders); "side_mask" (0-3, default 3): which weight gradients run on the side
 * stream -- bit 0 the decoder's, bit 1 the encoder's (a cleared bit: in order on the caller's
 * stream; the same results). */
int mvae_set_option(mvae_ctx* ctx, const char* name, int value);
/* Both TF ApplyAdam updates from MVAE_BUF_GRADS (theta -= d1(g1) + d2(g2)).           */
int mvae_adam(mvae_ctx* ctx, void* stream);
/* Single-GPU partial_fit: all four phases. losses_out: device float[5] or NULL;
 * dist_out: device float[B] or NULL.                                                  */
int mvae_train_step(mvae_ctx* ctx, const float* x, const float* areas, const float* eps,
                    float* losses_out, float* dist_out, void* stream);

/* ---- inference surface ------------------------------------------------------------ */
int mvae_predict(mvae_ctx* ctx, const float* x, const float* eps, float* dist_out, void* stream);
/* The same in two phases: a data-parallel host all-reduces MVAE_BUF_COLSQ (cosine metric)
 * between them, so every rank's distances use the global batch's column norms as the
 * single-process call on the whole batch does (8c/vae.py:449-450).                        */
int mvae_predict_encode(mvae_ctx* ctx, const float* x, const float* eps, void* stream);
int mvae_predict_finish(mvae_ctx* ctx, float* dist_out, void* stream);
/* transform: the lock image's latent mean only (no eps draw). */
int mvae_transform(mvae_ctx* ctx, const float* x, float* zmean_out, void* stream);
int mvae_reconstruct(mvae_ctx* ctx, const float* x, const float* eps, float* y_out, void* stream);
/* z: [n, L] (n <= B) -> y: [n, D] */
int mvae_generate(mvae_ctx* ctx, const float* z, int n, float* y_out, void* stream);

/* ---- batch producer (11a/overlap_input.py:127-261) -------------------------------- */
/* locks, keys: uint8 [n][H][W] (decoded PNGs, 0..255) on the device; idx: int [B] example
 * of each row; coef: float [B][4] = (cos, sin, x_off, y_off) of each row's rotation
 * (tf.contrib.image.rotate, computed on the host in fp32, 16-byte aligned).
 * Writes x_out [B, H*W*3] float32: per pixel (lock, rotated lock, key) / divisor
 * (255: inputs(normalize=True), 11a/overlap_input.py:113-115; 1: raw 0..255 pixels).       */
int mvae_make_batch(const unsigned char* locks, const unsigned char* keys, int height, int width,
                    const int* idx, const float* coef, int batch, float divisor, float* x_out,
                    void* stream);

/* ---- diagnostics ------------------------------------------------------------------ */
/* HIP-event timing of named regions (one GEMM incl. its split-K reduction, or one
 * bandwidth kernel group), recorded on the launch stream while enabled.               */
int mvae_timing_enable(mvae_ctx* ctx, int on);
/* Restrict recording to one region (-1: all regions, the default): a timed loop can carry the
   events of the one kernel it reports without the event pairs of every other region. */
int mvae_timing_select(mvae_ctx* ctx, int region);
/* Profiler runs: bracket every launch of `region` with an empty marker kernel of
 * 4096 + region workgroups, so a rocprofv3 kernel trace can attribute dispatches (and their
 * counters) to the region. Off by default. */
int mvae_timing_marker(mvae_ctx* ctx, int region, int on);
int mvae_timing_regions(mvae_ctx* ctx);
const char* mvae_timing_name(mvae_ctx* ctx, int region);
int mvae_timing_read(mvae_ctx* ctx, int region, double* total_ms, int64_t* count);
int mvae_timing_reset(mvae_ctx* ctx);
/* One GEMM of the step's kernel family: C[M,N] = epi(A[M,K] B[K,N]); A stored [M][K]
 * (at=0) or [K][M] (at=1), B stored [K][N] (bt=0) or [N][K] (bt=1). epi: 0 store,
 * 1 act (act: 0 tanh, 1 elu), 2 C = acc * act'(aux), 4 sigmoid; epi | (prec << 4) |
 * (variant << 8) selects the arithmetic (MVAE_PREC_*) and kernel (0 auto, 3 the 256x256
 * bf16 kernel, 4 the 128x128 one, 9 the fp32 VALU kernel for skinny shapes). Workspace is allocated and freed inside
 * (synchronous; tests only). mvae_bench_gemm: variant | (prec << 4) | (epi << 8).    */
int mvae_bench_gemm(int M, int N, int K, int at, int bt, int batch, int variant, int iters,
                    void* stream, float* avg_ms);
/* Diagnostics: the step's de-interleave of a [B][3D] batch of random 0/1 pixels, iters launches
 * (B % 64 == 0, D % 8 == 0): variant 0-4 the bits forms (the pixel operand as BitMats), 100 the
 * bf16-plane pass. Average ms per launch in *avg_ms.                                         */
int mvae_bench_deint(int B, int D, int variant, int iters, void* stream, float* avg_ms);
/* One 5x5x64x64 conv kernel of the conv tower on caller data (tests; synchronous): S1 x S1 x 64
 * NHWC images, B rows (3B forward images, 4B backward). mode 0: relu(conv(x, W2) + b2), 3B
 * images, y = W2 block [1601][64]; mode 1: data gradient of x (4B images), y = W2; mode 2:
 * out[2][1601][64] = the cost / metric weight gradients of x = conv2 input (3B), y = d pre-
 * activation (4B). mfma: bf16 MFMA kernels (operands rounded to bf16), else fp32 VALU.     */
int mvae_debug_conv2(int S1, int B, int mode, int mfma, const float* x, const float* y, float* out,
                     void* stream);
int mvae_debug_gemm(int M, int N, int K, const float* A, int lda, int at, const float* B, int ldb,
                    int bt, float* C, int ldc, int epi, int act, const float* aux, int ld_aux,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MVAE_H_ */
