// libmvae C ABI: context, parameter layout and the training-step schedule.
//
// HBM layout (all fp32, row-major, every row stride a multiple of 4 floats):
//   theta  = [enc blocks | head | dec blocks], each block the augmented [W; b] of one layer
//            ((fan_in+1) x fan_out; the head block is [W_mean W_logsigma; b_mean b_logsigma]).
//   grads  = [g1 (same layout as theta) | g2 (encoder slice)] — ONE all-reduce bucket.
//   adam   = [m1 | v1 | m2 | v2].
//   Activation buffers carry a constant ones column after the last feature so every GEMM
//   folds its bias (see gemm_f32.hip). Stacked encoder rows: [rot | lock | key] (3B),
//   backward rows [rot:g1 | lock:g1 | lock:g2 | key:g2] (4B).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/mvae.h"
#include "mvae_internal.h"

using namespace mvae;

namespace {

struct Block {
  size_t off = 0;  // element offset in theta / g1
  int K = 0, N = 0;
  int ld = 0;      // row stride: N rounded up to 8 (16-B rows for the bf16 plane images)
};

inline int round8(int v) { return (v + 7) & ~7; }
inline size_t align64(size_t v) { return (v + 63) & ~size_t(63); }
// Philox call counters of inference draws carry this bit (a stream disjoint from training's)
constexpr uint64_t EVAL_STREAM = 1ull << 63;

}  // namespace

struct mvae_ctx {
  mvae_cfg cfg{};
  int device = 0;
  bool diag_skip_deint = false;  // create option diag_skip_deint (timing bound only: wrong results)
  // diagnostics (create options diag_shadow_deint / diag_shadow_at): a second de-interleave of
  // the step's input into a scratch image on a low-priority stream beside the step -- the cost
  // to the step of staging the next batch's pass (grid: -1 the normal launch, > 0 persistent)
  int diag_shadow = 0, diag_shadow_at = 0;
  hipStream_t stage = nullptr;
  bool stage_pending = false;
  unsigned short* shadow = nullptr;
  const float* last_x = nullptr;
  int B = 0, D = 0, L = 0, nenc = 0, d0 = 0, d1 = 0;
  float inv_bg = 1.f;
  int ldx = 0, ldz = 0, ld_d1 = 0, ld_d2 = 0, ld_u = 0, lddz = 0, ld_dh = 0, nblk = 0, nchunk = 0;
  std::vector<int> ldh;
  // parameters
  std::vector<Block> enc;
  Block head, v1, v2, vo;
  // conv-encoder variant (cfg.conv): tower blocks [25*c_in; b] x 64 before the FC encoder
  bool conv = false;
  Block cv1, cv2;
  ConvTower tower;
  int F = 0, ldf = 0;        // tower features per image (FC layer-0 fan-in) and row stride
  float* xf = nullptr;       // [3B][ldf] tower features (+ ones column): FC layer-0 operand
  float* dxf = nullptr;      // [4B][ldf] their gradient
  int xf32 = 1;              // write the fp32 xf rows (some fp32 GEMM reads them)
  GemmDesc bwd_feat;         // dxf = dZ_0 W_0^T
  int bwd_feat_r = 0;
  size_t n_all = 0, n_enc = 0;
  float* theta = nullptr;
  float* grads = nullptr;
  float* adam = nullptr;
  float* dead = nullptr;
  // activations / workspaces
  float* xs = nullptr;
  std::vector<float*> H;
  float *ms = nullptr, *z = nullptr, *a1 = nullptr, *a2 = nullptr, *du = nullptr;
  float *rowpart = nullptr, *rowvals = nullptr, *dist = nullptr, *draw = nullptr, *losses = nullptr;
  float *colsq = nullptr, *coldot = nullptr, *cspart = nullptr, *eps = nullptr;
  int* cscnt = nullptr;  // create option cs_one: the column statistics' per-column-block counters
  float* rowfwd = nullptr;   // [B][4] latent forward row sums (KL, deformation, sq-diff distance)
  LatentEps le;              // eps of the last forward (buffer, or the Philox call regenerated)
  bool eps_lazy = false;     // le is a Philox call whose values the eps buffer does not hold yet
  int zmask = 6;             // fp32 z rows the latent forward writes (bit 1 lock, bit 2 key)
  float *dzd2 = nullptr, *dzd1 = nullptr, *dzdec = nullptr, *dhead = nullptr;
  std::vector<float*> dzl;  // dZ of every encoder layer [4B][lddz] (all live until its wgrad)
  int enc_part1 = 0;        // bwd_enc[0, enc_part1): dgrad chain + layer-0 wgrad
  // the layer-0 weight gradient in R row chunks (option "wgrad0_chunks", R = 2, 4, 8): chunk r
  // covers rows [w0m[R][r], w0m[R][r+1]) of the [W_0; b_0] block, one backward part each, so a
  // data-parallel host all-reduces each chunk while the next one computes (R = 1: one GEMM)
  int w0_chunks = 1;
  std::vector<GemmDesc> w0c[9];
  std::vector<int> w0m[9];
  int bpart = 0;            // next backward part expected (phase 4)
  float* zgen = nullptr;
  int dhead32 = 1;           // latent_bwd writes fp32 dhead rows (some fp32 GEMM reads them)
  float* ws = nullptr;       // split-K slabs of GEMMs on the caller's stream
  float* ws_side = nullptr;  // ... and of GEMMs on the side stream (concurrent)
  size_t ws_elems = 0;
  // side stream: the weight gradients run beside the dgrad chain (backward)
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> sync_ev;  // fork/join events (timing disabled), reused round robin
  size_t sync_next = 0;
  bool use_side = true;      // option "side_stream"
  bool side_pending = false; // side stream holds work the caller's stream has not joined
  bool early_adam = false;   // option "early_adam": Adam of the parameters after the layer-0
                             // block runs on the side stream beside the layer-0 weight gradient
  bool early_fork = false;   // ... the side stream waits for the dgrad chain this step
  // ... and, with the layer-0 weight gradient in R > 1 chunks, Adam of chunk k's rows ran on the
  // side stream beside chunk k + 1's GEMM: mvae_adam's layer-0 launch starts here
  size_t adam0_from = 0;
  // the single-call backward with the early Adam runs the layer-0 weight gradient in this many
  // chunks when "wgrad0_chunks" is 1 (option "early_chunks"; 1: one GEMM, the default since the
  // chunks keep the one-GEMM plan: 1 vs 2 chunks C2 -2.5 %, C3 -2.4 %, C5 -1.0 %, r6l)
  int early_chunks = 1;
  int side_mask = 3;         // option "side_mask": weight gradients on the side stream -- bit 0
                             // the decoder's, bit 1 the encoder's (else in order on the caller's)
  bool valu = true;          // skinny GEMMs on the fp32 VALU kernel (env MVAE_NO_VALU=1: off)
  std::vector<void*> allocs;
  // bf16 plane images (bf16 / f32x modes): fp32 buffer -> planes of the same layout
  struct PlaneBuf { float* base; size_t n; Planes pl; };
  std::vector<PlaneBuf> planes;
  int np = 0;            // planes per buffer: 0 (fp32 mode), 1 (bf16), 3 (f32x)
  int* dyn = nullptr;    // bf16/f32x: some de-interleaved pixel not exact in bf16?
  int* dyn_cur = nullptr;  // ... its slot of the last de-interleave (two slots, used in turn)
  int x32mask = 7;       // fp32 row blocks of xs the step reads (bit c: 0 rot, 1 lock, 2 key)
  int x32dyn = 0;        // ... written only when *dyn != 0 (the BCE target, else read as bf16)
  unsigned char* xbits = nullptr;  // the BCE target (lock block) as bits (GemmEpi::xbits)
  int ldbits = 0;
  // the layer-0 pixel operand of a 0/1 batch as bits (create option bits, default on where it
  // applies): BitMats of the forward (3B x (D + 1)) and the weight gradient ((D + 1) x 3B), written
  // by the de-interleave instead of the bf16 plane, read by the eight-phase kernel's bits path
  bool bits_on = false;
  unsigned* xbf = nullptr;
  unsigned* xbw = nullptr;
  int kts_f = 0, kts_w = 0;
  // the de-interleave inside the layer-0 forward's launch (create option deint_fuse; DeintJob):
  // f0f the fused launch (bits path, its own split), f0fb the plane-path fallback that runs only
  // for a batch with a pixel other than 0 / 1; fuse_buf: the chunk counters, error word, order
  int adam_nt = 0;  // create option adam_nt
  int deint_variant = 0;  // create option deint_variant
  int e8_prio = 0;        // create option e8_prio (PParams::prio)
  // create option xbw_split: the de-interleave writes the forward BitMat only and the weight
  // gradient's (xbw) is transposed from it on the side stream (launch_bits_transpose), joined by
  // xbw_ev before the layer-0 weight gradient
  int xbw_split = 0;
  hipEvent_t xbw_ev = nullptr;
  bool xbw_pending = false;
  bool fuse = false;
  GemmDesc f0f, f0fb;
  int* fuse_buf = nullptr;
  int fuse_nchunks = 0;
  // schedule (each GEMM tagged with its timing region)
  std::vector<GemmDesc> fwd_enc;  // encoder layers + head
  // the hidden layers fwd_enc[1 .. nenc-1] as one launch (enc_chain.hip; create option enc_chain)
  bool chain = false;
  ChainArgs chain_args;
  int chain_r = 0;
  GemmDesc f_d1, f_d2, f_out;
  // the decoder's hidden layers f_d1, f_d2 as one launch (the same kernel; option dec_chain)
  bool dchain = false;
  ChainArgs dchain_args;
  int dchain_r = 0;
  GemmDesc f_out_a, f_out_b;  // f_out as whole rounds of 256x256 tiles + the rest (f_split)
  bool f_split = false;
  bool use_split = true;      // option "bce_split" (default 1)
  std::vector<GemmDesc> bwd_dec;  // W_out, D_out, W_d2, D_d2, W_d1, D_d1
  std::vector<GemmDesc> bwd_enc;  // W_head, D_head, (W_i, D_i)..., W_0
  std::vector<int> fwd_enc_r, bwd_dec_r, bwd_enc_r;
  int f_d1_r = 0, f_d2_r = 0, f_out_r = 0;
  // HIP-event timing regions (diagnostics / bench roofline)
  std::vector<std::string> region_names;
  std::vector<double> region_ms;
  std::vector<int64_t> region_n;
  struct Pending { int region; hipEvent_t a, b; };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;
  bool timing = false;
  int timing_sel = -1;   // record only this region (-1: all)
  std::vector<char> marker;  // launch marker kernels around these regions (profiler runs)
  // optimizer state (TF beta1_power / beta2_power are fp32 variables)
  int64_t t1 = 0, t2 = 0;
  float b1p[2] = {0, 0}, b2p[2] = {0, 0};
  uint64_t rng_counter = 0;   // training draws (eps == NULL in mvae_forward / train_step)
  uint64_t rng_eval = 0;      // inference draws (predict / reconstruct): a separate stream, so
                              // evaluation never shifts the training noise sequence
  int row_off = 0;            // this rank's first row in the global batch (eps sampling)
  int phase = 0;  // 0 idle, 1 forward done, 2 metric done, 3 backward done
  std::string err;
};

static thread_local std::string g_create_err;

#define MV_CHECK(expr)                                                              \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
      return (int)e_;                                                               \
    }                                                                               \
  } while (0)

static int fail(mvae_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg; else g_create_err = msg;
  return code;
}

static hipError_t dalloc(mvae_ctx* ctx, float** p, size_t n) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(float));
  if (e != hipSuccess) return e;
  ctx->allocs.push_back(q);
  *p = static_cast<float*>(q);
  return hipMemset(q, 0, std::max<size_t>(n, 1) * sizeof(float));
}

static hipError_t ones_column(float* base, int ld, int col, int rows) {
  std::vector<float> one(rows, 1.f);
  return hipMemcpy2D(base + col, (size_t)ld * sizeof(float), one.data(), sizeof(float), sizeof(float),
                     rows, hipMemcpyHostToDevice);
}

static Planes planes_of(const mvae_ctx* c, const float* p) {
  for (const auto& b : c->planes)
    if (p >= b.base && p < b.base + b.n) {
      Planes r = b.pl;
      r.p += (p - b.base);
      return r;
    }
  return Planes{};
}

static GemmDesc gd(int M, int N, int K, const float* A, int lda, bool at, const float* Bm, int ldb,
                   bool bt, float* C, int ldc, int mode = EPI_STORE) {
  GemmDesc d;
  d.M = M; d.N = N; d.K = K; d.A = A; d.lda = lda; d.at = at; d.B = Bm; d.ldb = ldb; d.bt = bt;
  d.C = C; d.ldc = ldc; d.epi.mode = mode;
  return d;
}

static int region(mvae_ctx* c, const std::string& name) {
  for (size_t i = 0; i < c->region_names.size(); ++i)
    if (c->region_names[i] == name) return (int)i;
  c->region_names.push_back(name);
  c->region_ms.push_back(0.0);
  c->region_n.push_back(0);
  return (int)c->region_names.size() - 1;
}

static hipEvent_t take_event(mvae_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // timing only: no system-scope fence (a cache writeback + invalidate per record otherwise)
  (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return e;
}

// RAII: records a start/stop event pair around one region on the launch stream; in profiler
// runs (mvae_timing_marker) it also brackets the region with marker kernels whose grid size
// (MARKER_GRID + region) names the region in a kernel trace
struct TimeScope {
  mvae_ctx* c; int r; hipStream_t st; hipEvent_t a = nullptr; bool mk = false;
  TimeScope(mvae_ctx* c_, int r_, hipStream_t st_) : c(c_), r(r_), st(st_) {
    mk = r < (int)c->marker.size() && c->marker[r];
    if (mk) (void)launch_marker(r, st);
    if (c->timing && (c->timing_sel < 0 || c->timing_sel == r)) {
      a = take_event(c);
      (void)hipEventRecord(a, st);
    }
  }
  ~TimeScope() {
    if (a) {
      hipEvent_t b = take_event(c);
      (void)hipEventRecord(b, st);
      c->pending.push_back({r, a, b});
    }
    if (mk) (void)launch_marker(r, st);
  }
};

static void build_schedule(mvae_ctx* c) {
  const int B = c->B, L = c->L, n = c->nenc, act = c->cfg.act;
  float* th = c->theta;
  float* g1 = c->grads;
  const long long n_all = (long long)c->n_all;
  // ---- forward: encoder on the stacked 3B rows
  c->fwd_enc.clear();
  const float* X0 = c->conv ? c->xf : c->xs;   // layer-0 operand: pixels or tower features
  const int ld0 = c->conv ? c->ldf : c->ldx;
  for (int i = 0; i < n; ++i) {
    const float* A = i == 0 ? X0 : c->H[i - 1];
    const int lda = i == 0 ? ld0 : c->ldh[i - 1];
    GemmDesc d = gd(3 * B, c->enc[i].N, c->enc[i].K + 1, A, lda, false, th + c->enc[i].off,
                    c->enc[i].ld, false, c->H[i], c->ldh[i], EPI_ACT);
    d.epi.act = act;
    d.epi.padw = 2;  // H[i]: the ones column at N, zeros beyond
    c->fwd_enc.push_back(d);
    c->fwd_enc_r.push_back(region(c, "enc_fwd_" + std::to_string(i)));
  }
  c->fwd_enc.push_back(gd(3 * B, 2 * L, c->head.K + 1, c->H[n - 1], c->ldh[n - 1], false,
                          th + c->head.off, c->head.ld, false, c->ms, 2 * L));
  c->fwd_enc_r.push_back(region(c, "head_fwd"));
  c->f_d1_r = region(c, "dec_fwd_1");
  c->f_d2_r = region(c, "dec_fwd_2");
  c->f_out_r = region(c, "dec_fwd_out_bce");
  for (const char* nm : {"dec_bwd_w_out", "dec_bwd_d_out", "dec_bwd_w_2", "dec_bwd_d_2", "dec_bwd_w_1",
                         "dec_bwd_d_z"})
    c->bwd_dec_r.push_back(region(c, nm));
  // ---- decoder on the lock rows
  c->f_d1 = gd(B, c->d0, L + 1, c->z + (size_t)B * c->ldz, c->ldz, false, th + c->v1.off, c->v1.ld,
               false, c->a1, c->ld_d1, EPI_ACT);
  c->f_d1.epi.act = act;
  c->f_d1.epi.padw = 2;
  c->f_d2 = gd(B, c->d1, c->d0 + 1, c->a1, c->ld_d1, false, th + c->v2.off, c->v2.ld, false, c->a2,
               c->ld_d2, EPI_ACT);
  c->f_d2.epi.act = act;
  c->f_d2.epi.padw = 2;
  c->f_out = gd(B, c->D, c->d1 + 1, c->a2, c->ld_d2, false, th + c->vo.off, c->vo.ld, false, c->du,
                c->ld_u, EPI_BCE);
  c->f_out.epi.x = c->xs + (size_t)B * c->ldx;
  c->f_out.epi.ldx = c->ldx;
  c->f_out.epi.scale = c->inv_bg;
  c->f_out.epi.rowpart = c->rowpart;
  // ---- decoder backward (g1 only)
  c->bwd_dec.clear();
  c->bwd_dec.push_back(gd(c->d1 + 1, c->D, B, c->a2, c->ld_d2, true, c->du, c->ld_u, false,
                          g1 + c->vo.off, c->vo.ld));
  GemmDesc dout = gd(B, c->d1, c->D, c->du, c->ld_u, false, th + c->vo.off, c->vo.ld, true, c->dzd2,
                     c->ld_d2, EPI_DACT);
  dout.epi.act = act; dout.epi.aux = c->a2; dout.epi.ld_aux = c->ld_d2; dout.epi.padw = 1;
  c->bwd_dec.push_back(dout);
  c->bwd_dec.push_back(gd(c->d0 + 1, c->d1, B, c->a1, c->ld_d1, true, c->dzd2, c->ld_d2, false,
                          g1 + c->v2.off, c->v2.ld));
  GemmDesc dd2 = gd(B, c->d0, c->d1, c->dzd2, c->ld_d2, false, th + c->v2.off, c->v2.ld, true, c->dzd1,
                    c->ld_d1, EPI_DACT);
  dd2.epi.act = act; dd2.epi.aux = c->a1; dd2.epi.ld_aux = c->ld_d1; dd2.epi.padw = 1;
  c->bwd_dec.push_back(dd2);
  c->bwd_dec.push_back(gd(L + 1, c->d0, B, c->z + (size_t)B * c->ldz, c->ldz, true, c->dzd1,
                          c->ld_d1, false, g1 + c->v1.off, c->v1.ld));
  c->bwd_dec.push_back(gd(B, L, c->d0, c->dzd1, c->ld_d1, false, th + c->v1.off, c->v1.ld, true,
                          c->dzdec, L));
  // ---- encoder backward: g1 over rows [rot|lock], g2 over [lock|key] (batched GEMMs).
  // Part 1 runs the dgrad chain (head -> layer 1) and then the big layer-0 weight gradient;
  // part 2 the small weight gradients of the head and hidden layers. Each part ends with a
  // set of finished gradient ranges (the all-reduce buckets of mvae_grad_range), so a data-
  // parallel host overlaps the decoder and layer-0 all-reduces with the remaining work.
  c->bwd_enc.clear();
  c->bwd_enc_r.clear();
  auto dgrad = [&](int i) {  // dZ_{i-1} = (dZ_i W_i^T) * act'(H_{i-1}); i == n: the head
    const bool head = i == n;
    const Block& blk = head ? c->head : c->enc[i];
    const float* src = head ? c->dhead : c->dzl[i];
    const int lds = head ? c->ld_dh : c->lddz;
    GemmDesc d = gd(4 * B, blk.K, blk.N, src, lds, false, th + blk.off, blk.ld, true, c->dzl[i - 1],
                    c->lddz, EPI_DACT);
    d.epi.act = act; d.epi.aux = c->H[i - 1]; d.epi.ld_aux = c->ldh[i - 1];
    d.epi.remap_split = 2 * B; d.epi.remap_shift = B;
    d.epi.padw = 1;  // dZ rows: zero padding
    c->bwd_enc.push_back(d);
    c->bwd_enc_r.push_back(region(c, head ? std::string("head_bwd_d") : "enc_bwd_d_" + std::to_string(i)));
  };
  auto wgrad = [&](int i) {  // [W_i; b_i] gradients (g1 and g2 as one batch-2 GEMM); i == n: head
    const bool head = i == n;
    const Block& blk = head ? c->head : c->enc[i];
    const float* A = i == 0 ? X0 : c->H[i - 1];
    const int lda = i == 0 ? ld0 : c->ldh[i - 1];
    const float* src = head ? c->dhead : c->dzl[i];
    const int lds = head ? c->ld_dh : c->lddz;
    GemmDesc w = gd(blk.K + 1, blk.N, 2 * B, A, lda, true, src, lds, false, g1 + blk.off, blk.ld);
    w.batch = 2; w.sA = (long long)B * lda; w.sB = (long long)2 * B * lds; w.sC = n_all;
    c->bwd_enc.push_back(w);
    c->bwd_enc_r.push_back(region(c, head ? std::string("head_bwd_w") : "enc_bwd_w_" + std::to_string(i)));
  };
  for (int i = n; i >= 1; --i) dgrad(i);
  if (c->conv) {  // gradient of the tower features: dxf = dZ_0 W_0^T (no activation)
    c->bwd_feat = gd(4 * B, c->F, c->enc[0].N, c->dzl[0], c->lddz, false, th + c->enc[0].off,
                     c->enc[0].ld, true, c->dxf, c->ldf);
    c->bwd_feat_r = region(c, "enc_bwd_d_0");
  }
  wgrad(0);
  c->enc_part1 = (int)c->bwd_enc.size();
  wgrad(n);
  for (int i = n - 1; i >= 1; --i) wgrad(i);
  for (const char* nm : {"deinterleave", "eps_rng", "latent_fwd", "colsq", "metric_loss", "coldot",
                         "latent_bwd", "adam"})
    region(c, nm);
  if (c->conv)
    for (const char* nm : {"conv1_fwd", "conv2_fwd", "lrn2_pool2_fwd", "pool2_bwd", "conv2_wgrad",
                           "conv2_dgrad", "conv1_wgrad"})
      region(c, nm);
}

static int validate(const mvae_cfg* cfg) {
  if (!cfg) return fail(nullptr, MVAE_EINVAL, "cfg is NULL");
  if (cfg->image_size <= 0 || cfg->batch <= 0 || cfg->latent <= 0)
    return fail(nullptr, MVAE_ECONFIG, "image_size, batch and latent must be positive");
  if (cfg->global_batch < cfg->batch) return fail(nullptr, MVAE_ECONFIG, "global_batch < batch");
  if (cfg->n_enc < 1 || cfg->n_enc > MVAE_MAX_ENC) return fail(nullptr, MVAE_ECONFIG, "n_enc out of range");
  for (int i = 0; i < cfg->n_enc; ++i)
    if (cfg->enc[i] <= 0) return fail(nullptr, MVAE_ECONFIG, "encoder width must be positive");
  if (cfg->dec[0] <= 0 || cfg->dec[1] <= 0) return fail(nullptr, MVAE_ECONFIG, "decoder widths must be positive");
  if (cfg->act != MVAE_ACT_TANH && cfg->act != MVAE_ACT_ELU) return fail(nullptr, MVAE_ECONFIG, "bad act");
  if (cfg->metric != MVAE_METRIC_COSINE && cfg->metric != MVAE_METRIC_SQDIFF)
    return fail(nullptr, MVAE_ECONFIG, "bad metric");
  if (cfg->precision != MVAE_PREC_F32 && cfg->precision != MVAE_PREC_BF16 &&
      cfg->precision != MVAE_PREC_F32X)
    return fail(nullptr, MVAE_ECONFIG, "bad precision");
  if (cfg->conv != 0 && cfg->conv != 1) return fail(nullptr, MVAE_ECONFIG, "conv must be 0 or 1");
  // conv tower: sizes up to BASELINE's 100 x 100 are the tested range (tests/test_gpu_conv.py);
  // larger images would need > 64 KB of dynamic LDS in the conv2 MFMA kernels, never run
  if (cfg->conv && (cfg->image_size % 4 != 0 || cfg->image_size > 100))
    return fail(nullptr, MVAE_ECONFIG, "conv encoder: image_size must be a multiple of 4 (<= 100)");
  const long long D = (long long)cfg->image_size * cfg->image_size;
  if (D * 3 * cfg->batch > (1LL << 31) - 1 || 3LL * cfg->batch * (D + 4) > (1LL << 31) * 8)
    return fail(nullptr, MVAE_ECONFIG, "batch too large for 32-bit row indexing");
  return MVAE_OK;
}

extern "C" {

int mvae_abi_version(void) { return MVAE_ABI_VERSION; }

#ifndef MVAE_BUILD_ID
#error "MVAE_BUILD_ID must be defined by the build (magic_amd/build.py source_hash)"
#endif
const char* mvae_build_id(void) { return MVAE_BUILD_ID; }

const char* mvae_last_error(mvae_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

int mvae_destroy(mvae_ctx* ctx) {
  if (!ctx) return MVAE_EINVAL;
  int dev = 0;
  hipGetDevice(&dev);
  hipSetDevice(ctx->device);
  hipDeviceSynchronize();
  for (auto& pd : ctx->pending) { hipEventDestroy(pd.a); hipEventDestroy(pd.b); }
  for (auto e : ctx->event_pool) hipEventDestroy(e);
  for (auto e : ctx->sync_ev) hipEventDestroy(e);
  if (ctx->xbw_ev) hipEventDestroy(ctx->xbw_ev);
  if (ctx->side) hipStreamDestroy(ctx->side);
  if (ctx->stage) hipStreamDestroy(ctx->stage);
  for (void* p : ctx->allocs) hipFree(p);
  hipSetDevice(dev);
  delete ctx;
  return MVAE_OK;
}

// Plan-time kernel switches of one context (mvae_create_ex options; the library reads no
// environment outside its diagnostics entry points). Defaults are the measured best plans.
struct CreateOpts {
  int e8 = 1;           // 256-row bf16 GEMMs: 1 planner (eight-phase + ring kernels), 0 ring only,
                        // 2 the eight-phase kernel wherever a 256-row kernel runs
  int thin_ring = 2;    // f32x latent head: 2 ring kernel incl. its weight gradient, 1 weight
                        // gradient on the fp32 kernel, 0 the VALU kernel
  int valu = 1;         // skinny products on the fp32 VALU kernel
  int dact_planes = 1;  // bf16 mode: DACT epilogues read the activation's bf16 plane
  int bce_split = 1;    // the BCE head in whole rounds + 256x128 ring tiles
  int plan_log = 0;     // print the GEMM plans on stderr
  int diag_skip_deint = 0;  // diagnostics: de-interleave only the first batch (the step's time
                            // without its streaming pass; results meaningless)
  int diag_shadow_deint = 0, diag_shadow_at = 0;  // diagnostics: see mvae_ctx::diag_shadow
  int enc_chain = 1;    // bf16 mode: the encoder's hidden layers in one launch (0: one GEMM each)
  int enc_chain_rows = 0;  // ... its rows per workgroup forced (16..96, multiple of 16; 0 auto)
  int diag_chain = 0;      // ... its timing ablations (ChainArgs::diag; results meaningless)
  int dec_chain = 1;    // bf16 mode: the decoder's two hidden layers in one launch (0: one GEMM each)
  int bits = 1;         // plane modes: the layer-0 pixel operand of a 0/1 batch as bits (BitMat)
  int bits_reg = 1;     // ... the eight-phase bits path loading A's words to registers (E8 BITS 2;
                        // 0: through an LDS copy -- C3 1.784 vs 1.769 ms, C5 2.450 vs 2.432, r6t)
  int deint_fuse = 0;   // ... the de-interleave run inside the layer-0 forward's launch (DeintJob)
  int deint_fuse_diag = 0;  // ... its timing diagnostics (DeintJob::diag; results invalid)
  int adam_nt = 1;      // Adam's moment / fp32 parameter stores non-temporal (C2 -0.6 %, C3 -0.3 %, r6za)
  int deint_variant = 0;  // the bits de-interleave's form (launch_deint_bits; diagnostics / A-B)
  int e8_prio = 0;      // the eight-phase kernel's s_setprio form (PParams::prio; A-B)
  int x3 = 2;           // f32x: ring plans on the plane-stacked kernels (gemm_bf16.hip): 1 the tile-N-128
                        // plans (C2 -2.1 / -2.9 % on two boxes, r6zi / r6zj), 2 also the 256x256 ones
                        // (C2's hidden weight gradients 68.5 -> 66.5 us, step -0.2 %, r6zp)
  int cs_one = 2;       // the column statistics in one launch (the last chunk's workgroup sums the
                        // partials in colstats_final_kernel's order: the same bits): 0 off, 1 on, 2
                        // where L <= 32 (one 64-column block: C2 -0.9 %; C3, L 200: +0.2 %, r6zh / r6zi)
  int xbw_split = 2;    // the weight gradient's BitMat transposed from the forward's (mvae_ctx):
                        // 0 off, 1 on, 2 where the layer-0 forward's workgroups leave >= 32 CUs
                        // (C3 -0.6 %, C5 -0.4 %; C2, 480 forward workgroups: +3.8 % on, r6zf)
  int conv2_nw = 8, conv2_tpb = 1, conv2_fpw = 2, conv2_wg = 8, conv2_half = 1, conv2_nchunk = 0;
};

static int parse_opts(const char* s, CreateOpts* o) {
  if (!s) return MVAE_OK;
  std::string all(s);
  size_t i = 0;
  while (i < all.size()) {
    size_t j = all.find(',', i);
    if (j == std::string::npos) j = all.size();
    const std::string kv = all.substr(i, j - i);
    i = j + 1;
    if (kv.empty()) continue;
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) return fail(nullptr, MVAE_EINVAL, "option without '=': " + kv);
    const std::string k = kv.substr(0, eq);
    char* end = nullptr;
    const long v = std::strtol(kv.c_str() + eq + 1, &end, 10);
    if (end == kv.c_str() + eq + 1 || *end) return fail(nullptr, MVAE_EINVAL, "option value not an integer: " + kv);
    auto in = [&](long lo, long hi) { return v >= lo && v <= hi; };
    if (k == "e8" && in(0, 2)) o->e8 = (int)v;
    else if (k == "thin_ring" && in(0, 2)) o->thin_ring = (int)v;
    else if (k == "valu" && in(0, 1)) o->valu = (int)v;
    else if (k == "dact_planes" && in(0, 1)) o->dact_planes = (int)v;
    else if (k == "bce_split" && in(0, 1)) o->bce_split = (int)v;
    else if (k == "plan_log" && in(0, 1)) o->plan_log = (int)v;
    else if (k == "diag_skip_deint" && in(0, 1)) o->diag_skip_deint = (int)v;
    else if (k == "diag_shadow_deint" && in(-1, 1 << 16)) o->diag_shadow_deint = (int)v;
    else if (k == "diag_shadow_at" && in(0, 2)) o->diag_shadow_at = (int)v;
    else if (k == "enc_chain" && in(0, 1)) o->enc_chain = (int)v;
    else if (k == "diag_chain" && in(0, 7)) o->diag_chain = (int)v;
    else if (k == "dec_chain" && in(0, 1)) o->dec_chain = (int)v;
    else if (k == "bits" && in(0, 1)) o->bits = (int)v;
    else if (k == "bits_reg" && in(0, 1)) o->bits_reg = (int)v;
    else if (k == "deint_fuse" && in(0, 1)) o->deint_fuse = (int)v;
    else if (k == "deint_fuse_diag" && in(0, 31)) o->deint_fuse_diag = (int)v;
    else if (k == "adam_nt" && in(0, 1)) o->adam_nt = (int)v;
    else if (k == "deint_variant" && (in(0, 6) || v == 8)) o->deint_variant = (int)v;
    else if (k == "e8_prio" && in(0, 2)) o->e8_prio = (int)v;
    else if (k == "xbw_split" && in(0, 2)) o->xbw_split = (int)v;
    else if (k == "cs_one" && in(0, 2)) o->cs_one = (int)v;
    else if (k == "x3" && in(0, 2)) o->x3 = (int)v;
    else if (k == "enc_chain_rows" && (v == 0 || (in(16, 96) && v % 16 == 0))) o->enc_chain_rows = (int)v;
    else if (k == "conv2_nw" && (v == 4 || v == 8 || v == 16)) o->conv2_nw = (int)v;
    else if (k == "conv2_tpb" && in(1, 2)) o->conv2_tpb = (int)v;
    else if (k == "conv2_fpw" && (v == 2 || v == 4)) o->conv2_fpw = (int)v;
    else if (k == "conv2_wg" && (v == 4 || v == 8)) o->conv2_wg = (int)v;
    else if (k == "conv2_half" && in(0, 1)) o->conv2_half = (int)v;
    else if (k == "conv2_nchunk" && in(0, 1 << 20)) o->conv2_nchunk = (int)v;
    else return fail(nullptr, MVAE_EINVAL, "unknown option or value out of range: " + kv);
  }
  return MVAE_OK;
}

int mvae_create(const mvae_cfg* cfg, int device, mvae_ctx** out) {
  return mvae_create_ex(cfg, device, nullptr, out);
}

int mvae_create_ex(const mvae_cfg* cfg, int device, const char* options, mvae_ctx** out) {
  if (!out) return fail(nullptr, MVAE_EINVAL, "out is NULL");
  *out = nullptr;
  int rc = validate(cfg);
  if (rc) return rc;
  CreateOpts opt;
  if ((rc = parse_opts(options, &opt))) return rc;
  mvae_ctx* ctx = new (std::nothrow) mvae_ctx();
  if (!ctx) return fail(nullptr, MVAE_EINVAL, "out of host memory");
  ctx->cfg = *cfg;
  ctx->device = device;
  ctx->diag_skip_deint = opt.diag_skip_deint != 0;
  ctx->adam_nt = opt.adam_nt;
  ctx->deint_variant = opt.deint_variant;
  ctx->e8_prio = opt.e8_prio;
  ctx->xbw_split = opt.xbw_split == 1 ? 1 : 0;  // (2: decided with the forward's plan, below)
  ctx->diag_shadow = opt.diag_shadow_deint;
  ctx->diag_shadow_at = opt.diag_shadow_at;
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) { g_create_err = hipGetErrorString(he); delete ctx; return (int)he; }
  auto c = ctx;
  c->B = cfg->batch;
  c->D = cfg->image_size * cfg->image_size;
  c->L = cfg->latent;
  c->nenc = cfg->n_enc;
  c->d0 = cfg->dec[0];
  c->d1 = cfg->dec[1];
  c->inv_bg = 1.f / (float)cfg->global_batch;
  c->b1p[0] = c->b1p[1] = cfg->beta1;
  c->b2p[0] = c->b2p[1] = cfg->beta2;
  // ---- parameter layout
  size_t off = 0;
  int fan_in = c->D;
  c->conv = cfg->conv != 0;
  if (c->conv) {
    const int S = cfg->image_size;
    c->tower.S = S; c->tower.S1 = S / 2; c->tower.S2 = S / 4;
    c->cv1.off = off; c->cv1.K = 25; c->cv1.N = 64; c->cv1.ld = 64;
    off = align64(off + (size_t)26 * 64);
    c->cv2.off = off; c->cv2.K = 25 * 64; c->cv2.N = 64; c->cv2.ld = 64;
    off = align64(off + (size_t)(25 * 64 + 1) * 64);
    c->F = c->tower.S2 * c->tower.S2 * 64;
    c->ldf = round8(c->F + 1);
    fan_in = c->F;
  }
  for (int i = 0; i < c->nenc; ++i) {
    Block b; b.off = off; b.K = fan_in; b.N = cfg->enc[i]; b.ld = round8(b.N);
    c->enc.push_back(b);
    off = align64(off + (size_t)(b.K + 1) * b.ld);
    fan_in = b.N;
  }
  c->head.off = off; c->head.K = fan_in; c->head.N = 2 * c->L; c->head.ld = round8(2 * c->L);
  off = align64(off + (size_t)(fan_in + 1) * c->head.ld);
  c->n_enc = off;
  c->v1.off = off; c->v1.K = c->L; c->v1.N = c->d0; c->v1.ld = round8(c->d0);
  off = align64(off + (size_t)(c->L + 1) * c->v1.ld);
  c->v2.off = off; c->v2.K = c->d0; c->v2.N = c->d1; c->v2.ld = round8(c->d1);
  off = align64(off + (size_t)(c->d0 + 1) * c->v2.ld);
  c->vo.off = off; c->vo.K = c->d1; c->vo.N = c->D; c->vo.ld = round8(c->D);
  off = align64(off + (size_t)(c->d1 + 1) * c->vo.ld);
  c->n_all = off;
  // ---- strides
  c->ldx = round8(c->D + 1);
  c->ldz = round8(c->L + 1);
  c->ld_d1 = round8(c->d0 + 1);
  c->ld_d2 = round8(c->d1 + 1);
  c->ld_u = round8(c->D);
  c->ld_dh = round8(2 * c->L);
  int maxe = 0;
  for (int i = 0; i < c->nenc; ++i) {
    c->ldh.push_back(round8(cfg->enc[i] + 1));
    maxe = std::max(maxe, cfg->enc[i]);
  }
  c->lddz = round8(maxe);
  c->nblk = gemm_bce_nblk(c->D);
  c->nchunk = colstats_nchunk(c->B);
  const size_t B = c->B, L = c->L;
#define ALLOC(p, n)                                              \
  do {                                                           \
    hipError_t e_ = dalloc(c, &(p), (n));                        \
    if (e_ != hipSuccess) {                                      \
      g_create_err = std::string("hipMalloc ") + #p + ": " + hipGetErrorString(e_); \
      mvae_destroy(c);                                           \
      return (int)e_;                                            \
    }                                                            \
  } while (0)
  ALLOC(c->theta, c->n_all);
  ALLOC(c->grads, c->n_all + c->n_enc);
  ALLOC(c->adam, 2 * c->n_all + 2 * c->n_enc);
  ALLOC(c->dead, (size_t)c->d1 * c->D + c->D);
  ALLOC(c->xs, 3 * B * c->ldx);
  c->H.resize(c->nenc);
  for (int i = 0; i < c->nenc; ++i) ALLOC(c->H[i], 3 * B * c->ldh[i]);
  ALLOC(c->ms, 3 * B * 2 * L);
  ALLOC(c->z, 3 * B * c->ldz);
  ALLOC(c->zgen, B * c->ldz);
  ALLOC(c->a1, B * c->ld_d1);
  ALLOC(c->a2, B * c->ld_d2);
  ALLOC(c->du, B * c->ld_u);
  ALLOC(c->rowpart, B * c->nblk);
  ALLOC(c->rowvals, 4 * B);
  ALLOC(c->dist, B);
  ALLOC(c->draw, B);
  ALLOC(c->losses, 8);
  ALLOC(c->colsq, 2 * L);
  ALLOC(c->coldot, L);
  ALLOC(c->cspart, (size_t)c->nchunk * 2 * L);
  if (opt.cs_one == 1 || (opt.cs_one == 2 && L <= 32)) ALLOC(*reinterpret_cast<float**>(&c->cscnt), (2 * L + 63) / 64);  // (zeroed)
  ALLOC(c->eps, 3 * B * L);
  ALLOC(c->rowfwd, 4 * B);
  ALLOC(c->dzd2, B * c->ld_d2);
  ALLOC(c->dzd1, B * c->ld_d1);
  ALLOC(c->dzdec, B * L);
  ALLOC(c->dhead, 4 * B * c->ld_dh);
  c->dzl.resize(c->nenc);
  for (int i = 0; i < c->nenc; ++i) ALLOC(c->dzl[i], 4 * B * c->lddz);
  if (c->conv) {
    ConvTower& T = c->tower;
    const size_t a1 = (size_t)T.S1 * T.S1 * 64, a2n = (size_t)T.S2 * T.S2 * 64;
    T.mfma = cfg->precision == MVAE_PREC_BF16;
    // kernel-shape options (A/B): conv2_half=0 (full-channel forward / data gradient kernel,
    // shaped by conv2_nw=4|16, conv2_tpb=2, conv2_fpw=4), conv2_wg=4
    T.conv2_nw = opt.conv2_nw;
    T.conv2_tpb = opt.conv2_tpb;
    T.conv2_fpw = opt.conv2_fpw;
    T.conv2_wg8 = opt.conv2_wg == 8;
    T.conv2_half = opt.conv2_half != 0;
    ALLOC(c->xf, 3 * B * c->ldf);
    ALLOC(c->dxf, 4 * B * c->ldf);
    ALLOC(T.p1, 3 * B * a1);
    if (!T.mfma) ALLOC(T.n1, 3 * B * a1);   // the MFMA kernels read the bf16 images only
    ALLOC(T.a2, 3 * B * a1);
    if (!T.mfma) ALLOC(T.da2, 4 * B * a1);
    ALLOC(T.dn1, 4 * B * a1);
    float* tmp = nullptr;
    ALLOC(tmp, (3 * B * a1 + 3) / 4); T.arg1 = reinterpret_cast<unsigned char*>(tmp);
    ALLOC(tmp, (3 * B * a2n + 3) / 4); T.arg2 = reinterpret_cast<unsigned char*>(tmp);
    if (T.mfma) {
      ALLOC(tmp, (3 * B * a1 + 1) / 2); T.n1b = reinterpret_cast<unsigned short*>(tmp);
      ALLOC(tmp, (4 * B * a1 + 1) / 2); T.da2b = reinterpret_cast<unsigned short*>(tmp);
      ALLOC(tmp, 25 * 64 * 64 / 2); T.w2f = reinterpret_cast<unsigned short*>(tmp);
      ALLOC(tmp, 25 * 64 * 64 / 2); T.w2d = reinterpret_cast<unsigned short*>(tmp);
    }
    const int B2 = 2 * (int)B;
    T.nchunk1 = std::min(B2, 1024);
    T.nchunk2 = std::min(B2, 32);
    // image chunks of the MFMA weight gradient: 64 -> 256 workgroups at C5CONV, one per CU
    // (same box: 1.085 ms vs 1.11 at 128 and 1.17 at 256, profiles/r2/conv2_wgrad_ab.txt)
    T.nchunk2m = std::min(B2, 64);
    if (opt.conv2_nchunk > 0) T.nchunk2m = std::min(B2, opt.conv2_nchunk);
    const size_t s1 = (size_t)2 * T.nchunk1 * 26 * 64;
    const size_t s2 = (size_t)2 * (T.mfma ? T.nchunk2m : T.nchunk2) * (25 * 64 + 1) * 64;
    ALLOC(T.slab, std::max(s1, s2));
  }
  // constant ones columns (bias folding)
  hipError_t e = ones_column(c->xs, c->ldx, c->D, 3 * (int)B);
  if (e == hipSuccess && c->conv) e = ones_column(c->xf, c->ldf, c->F, 3 * (int)B);
  for (int i = 0; e == hipSuccess && i < c->nenc; ++i) e = ones_column(c->H[i], c->ldh[i], cfg->enc[i], 3 * (int)B);
  if (e == hipSuccess) e = ones_column(c->z, c->ldz, c->L, 3 * (int)B);
  if (e == hipSuccess) e = ones_column(c->zgen, c->ldz, c->L, (int)B);
  if (e == hipSuccess) e = ones_column(c->a1, c->ld_d1, c->d0, (int)B);
  if (e == hipSuccess) e = ones_column(c->a2, c->ld_d2, c->d1, (int)B);
  if (e != hipSuccess) {
    g_create_err = std::string("ones column: ") + hipGetErrorString(e);
    mvae_destroy(c);
    return (int)e;
  }
  build_schedule(c);
  if (!opt.valu) c->valu = false;
  // option e8: the 256-row bf16 DMA GEMMs are planned over the eight-phase and ring kernels
  // (default, 1), on the ring kernels only (0), or on the eight-phase kernel wherever a 256-row
  // kernel would run (2)
  const int e8_mode = opt.e8;
  // option thin_ring: 0 the f32x latent head on the VALU kernel, 1 the head's weight gradient on
  // the fp32 kernel (A/B); default 2
  const int thin_ring = opt.thin_ring;
  const bool dact_planes = opt.dact_planes != 0;  // 0: bf16-mode DACT reads the fp32 activations (A/B)
  const int gp = cfg->precision == MVAE_PREC_BF16 ? GEMM_BF16
                 : (cfg->precision == MVAE_PREC_F32X ? GEMM_F32X : GEMM_F32);
  c->np = gp == GEMM_BF16 ? 1 : (gp == GEMM_F32X ? 3 : 0);
  if (c->np) {
    // plane images of every GEMM operand buffer (filled from the fp32 buffer once here,
    // then written by each producer: de-interleave, epilogues, latent kernels, Adam)
    auto add = [&](float* base, size_t n) -> hipError_t {
      void* q = nullptr;
      hipError_t e = hipMalloc(&q, (size_t)c->np * n * sizeof(unsigned short));
      if (e != hipSuccess) return e;
      c->allocs.push_back(q);
      mvae_ctx::PlaneBuf pb{base, n, Planes{static_cast<unsigned short*>(q), (long long)n, c->np}};
      c->planes.push_back(pb);
      return launch_split_planes(base, n, pb.pl, nullptr);
    };
    hipError_t e = add(c->theta, c->n_all);
    if (e == hipSuccess) e = add(c->xs, 3 * B * c->ldx);
    if (e == hipSuccess && c->conv) e = add(c->xf, 3 * B * c->ldf);
    for (int i = 0; e == hipSuccess && i < c->nenc; ++i) e = add(c->H[i], 3 * B * c->ldh[i]);
    if (e == hipSuccess) e = add(c->z, 3 * B * c->ldz);
    if (e == hipSuccess) e = add(c->zgen, B * c->ldz);
    if (e == hipSuccess) e = add(c->a1, B * c->ld_d1);
    if (e == hipSuccess) e = add(c->a2, B * c->ld_d2);
    if (e == hipSuccess) e = add(c->du, B * c->ld_u);
    if (e == hipSuccess) e = add(c->dzd2, B * c->ld_d2);
    if (e == hipSuccess) e = add(c->dzd1, B * c->ld_d1);
    if (e == hipSuccess) e = add(c->dhead, 4 * B * c->ld_dh);
    for (int i = 0; e == hipSuccess && i < c->nenc; ++i) e = add(c->dzl[i], 4 * B * c->lddz);
    if (e == hipSuccess) e = dalloc(c, reinterpret_cast<float**>(&c->dyn), 4);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      g_create_err = std::string("plane images: ") + hipGetErrorString(e);
      mvae_destroy(c);
      return (int)e;
    }
  }
  auto wire = [&](GemmDesc& d) {
    d.prec = gp;
    d.x3 = opt.x3;
    // skinny products (an output dimension or K <= 64 and no 256x256 plane-kernel shape: the
    // latent head and the decoder's first layer at small L) run on the fp32 VALU kernel
    const long long t256 = (long long)((d.M + 255) / 256) * ((d.N + 255) / 256) * d.batch;
    const bool wide_shape = d.M >= 256 && d.N >= 256 && !(d.K <= 64 && t256 < 256);
    // ... except the f32x latent head at small L over the tall stacked rows (C2: forward
    // 12288 x 40 x 501, dgrad 16384 x 500 x 40): the ring kernel's plane products (variant 3, any
    // shape) beat the VALU kernel there (24.3 / 23.9 us vs 30.8 / 38.0 us in the step,
    // profiles/r4/r4g_plan_c2.txt and bench_default_r4p_regions.txt), and its weight gradient
    // (501 x 40 x 8192, two products: 35.6 vs 40.7 us on the fp32 kernel, r4ar_thin_gemms.txt)
    const int lo = d.M < d.N ? d.M : d.N;
    const bool tall = d.M >= 4096 || (thin_ring == 2 && d.K >= 4096);
    if (gp == GEMM_F32X && e8_mode == 1 && !wide_shape && tall && lo >= 32 && d.K >= 32 &&
        d.variant == 0 && thin_ring)
      d.variant = 3;
    if (c->valu && gemm_valu_fits(d) && !(gp != GEMM_F32 && wide_shape)) {
      d.prec = GEMM_F32;
      d.valu = 1;
    }
    if (!c->np) return;
    const Planes a = planes_of(c, d.A), b = planes_of(c, d.B), o = planes_of(c, d.C);
    d.Ap = a.p; d.pA = a.stride; d.nA = c->np;
    d.Bp = b.p; d.pB = b.stride; d.nB = c->np;
    d.epi.cp = o.p; d.epi.pc = o.stride; d.epi.ncp = o.p ? c->np : 0;
    d.dynA = (c->np == 3 && d.A >= c->xs && d.A < c->xs + (size_t)3 * B * c->ldx) ? c->dyn : nullptr;
    // exact split: GEMMs the 256x256 bf16 kernel does not serve (a dimension < 256: the
    // latent head, thin decoder layers) run faster as one native fp32 MFMA GEMM than as six
    // bf16 plane products on the 128x128 kernel; same accuracy class
    if (gp == GEMM_F32X && !gemm_bf16_wide(d)) d.prec = GEMM_F32;
    if (d.prec != GEMM_F32 && !d.valu && gemm_bf16_wide(d) && e8_mode != 1)
      d.variant = e8_mode == 0 ? 15 : 13;
    // bf16 mode: a plane-kernel DACT epilogue reads the activation's bf16 plane (act' from the
    // bf16-rounded output, the operand precision of this mode), so the forward epilogues write
    // the activations as planes only (no fp32 copy)
    if (c->np == 1 && d.epi.mode == EPI_DACT && d.prec != GEMM_F32 && !d.valu && dact_planes)
      d.epi.auxp = planes_of(c, d.epi.aux).p;
  };
  for (auto* v : {&c->fwd_enc, &c->bwd_dec, &c->bwd_enc})
    for (auto& d : *v) wire(d);
  if (c->conv) wire(c->bwd_feat);
  wire(c->f_d1);
  wire(c->f_d2);
  wire(c->f_out);
  // fp32 xs rows: everything when a GEMM reads xs in fp32; otherwise only the BCE target
  // (lock block), and only for a batch whose pixels are not all bf16 values (the BCE epilogue
  // reads plane 0 while *dyn == 0)
  if (c->np) {
    c->x32mask = 0;
    c->x32dyn = 2;
    for (auto* v : {&c->fwd_enc, &c->bwd_enc})
      for (auto& d : *v)
        if (d.prec == GEMM_F32 && d.A >= c->xs && d.A < c->xs + (size_t)3 * B * c->ldx) c->x32mask = 7;
    if (c->f_out.prec != GEMM_F32) {
      const Planes xp = planes_of(c, c->xs);
      c->f_out.epi.xp = xp.p + (size_t)B * c->ldx;
      c->f_out.epi.xdyn = c->dyn;
      c->f_out.epi.xnb = c->dyn + 2;
      if (c->D % 8 == 0) {  // the 8-pixel de-interleave writes the target's bits beside its plane
        c->ldbits = (c->D / 8 + 15) & ~15;
        float* xb = nullptr;
        ALLOC(xb, ((size_t)B * c->ldbits + 3) / 4);
        c->xbits = reinterpret_cast<unsigned char*>(xb);
        c->f_out.epi.xbits = c->xbits;
        c->f_out.epi.ldbits = c->ldbits;
      }
    } else {
      c->x32mask |= 2;  // the native fp32 BCE GEMM reads the fp32 target rows
    }
    // fp32 copies only of the GEMM outputs something reads in fp32: an operand of a native
    // fp32 GEMM or the aux of a DACT epilogue (e.g. dU and the dgrads feeding plane GEMMs
    // only are written as planes alone). Outputs without a plane image keep their fp32 store.
    std::vector<GemmDesc*> all;
    for (auto* v : {&c->fwd_enc, &c->bwd_dec, &c->bwd_enc})
      for (auto& d : *v) all.push_back(&d);
    for (GemmDesc* d : {&c->f_d1, &c->f_d2, &c->f_out}) all.push_back(d);
    if (c->conv) all.push_back(&c->bwd_feat);
    for (GemmDesc* d : all) {
      const mvae_ctx::PlaneBuf* pb = nullptr;
      for (const auto& q : c->planes)
        if (d->C >= q.base && d->C < q.base + q.n) pb = &q;
      if (!pb || !d->epi.cp) continue;
      auto in = [&](const float* x) { return x && x >= pb->base && x < pb->base + pb->n; };
      bool fp32_reader = false;
      for (const GemmDesc* g : all) {
        if (g->prec == GEMM_F32 && (in(g->A) || in(g->B))) fp32_reader = true;
        if (g->epi.mode == EPI_DACT && in(g->epi.aux) && !g->epi.auxp) fp32_reader = true;
      }
      d->epi.c32 = fp32_reader ? 1 : 0;
    }
  }
  {  // fp32 z rows: lock for fp32 decoder GEMMs (layer-1 forward, its weight gradient) and the
     // cosine column statistics; key for the cosine statistics only
    const bool cos = cfg->metric == MVAE_METRIC_COSINE;
    const bool lock32 = !c->np || cos || c->f_d1.prec == GEMM_F32 || c->bwd_dec[4].prec == GEMM_F32;
    c->zmask = (lock32 ? 2 : 0) | (cos ? 4 : 0);
  }
  if (c->np) {  // fp32 dhead only for a native-fp32 head GEMM (else its planes alone)
    c->dhead32 = 0;
    for (auto& d : c->bwd_enc)
      if (d.prec == GEMM_F32 && (d.A == c->dhead || d.B == c->dhead)) c->dhead32 = 1;
  }
  if (c->conv) {
    // conv1 reads the fp32 pixels of all three row blocks (forward and weight gradient); the
    // fp32 feature rows are written only when an fp32 GEMM reads them
    c->x32mask = 7;
    c->xf32 = !c->np || c->fwd_enc[0].prec == GEMM_F32 || c->bwd_enc[c->nenc].prec == GEMM_F32;
  }
  for (auto* v : {&c->fwd_enc, &c->bwd_dec, &c->bwd_enc})
    for (auto& d : *v)
      if (c->np && (!d.Ap || !d.Bp)) {
        g_create_err = "internal: GEMM operand without plane image";
        mvae_destroy(c);
        return MVAE_EINVAL;
      }
  {  // the pixel operand as bits: both layer-0 GEMMs on the bf16-plane kernels, the target bits
     // written (D % 8 == 0), whole 64-row blocks, no fp32 pixel rows read
    GemmDesc& f0 = c->fwd_enc[0];
    GemmDesc& w0 = c->bwd_enc[c->nenc];
    auto planek = [](const GemmDesc& d) { return d.prec != GEMM_F32 && !d.valu && gemm_bf16_wide(d); };
    if (opt.bits && c->np && !c->conv && c->xbits && c->B % 64 == 0 && c->x32mask == 0 && planek(f0) &&
        planek(w0) && f0.A == c->xs && w0.A == c->xs) {
      c->kts_f = bitmat_kts(c->D + 1);
      c->kts_w = bitmat_kts(3 * c->B);
      float* q = nullptr;
      ALLOC(q, bitmat_words(3 * c->B, c->D + 1));
      c->xbf = reinterpret_cast<unsigned*>(q);
      ALLOC(q, bitmat_words(c->D + 1, 3 * c->B));
      c->xbw = reinterpret_cast<unsigned*>(q);
      f0.Abits = c->xbf; f0.abits_kts = c->kts_f; f0.anb = c->dyn + 2;
      // the weight gradient's batch 2 (g2) reads stacked rows B .. 3B: k-tiles from B / 64
      w0.Abits = c->xbw; w0.abits_kts = c->kts_w; w0.anb = c->dyn + 2;
      w0.abits_sb = (long long)(c->B / 64) * BITMAT_BLOCK_WORDS;
      f0.bits_reg = w0.bits_reg = opt.bits_reg;
      c->bits_on = true;
    }
  }
  {  // layer-0 weight-gradient row chunks (see w0c): the wired GEMM re-pointed at row ranges,
     // with the whole GEMM's split-K and kernel pinned, so each output row is summed exactly as
     // the one-GEMM backward sums it (chunked and unchunked backwards are bitwise equal: the early
     // Adam's chunks, the data-parallel parts)
    const GemmDesc& w = c->bwd_enc[c->nenc];
    const int w_split = gemm_plan_split(w, ~size_t(0));
    int w_variant = w.variant;
    if (w.prec != GEMM_F32 && !w.valu && gemm_bf16_wide(w) && w.variant == 0) {
      int sp = 0, tn = 0, tm = 0;
      gemm_bf16_wide_plan(w, ~size_t(0), &sp, &tn, &tm);
      w_variant = tn == GEMM_TN_E8 ? 13 : (tn == 128 ? 11 : 12);  // (tm: 256 for an A^T operand)
    }
    for (int R : {2, 4, 8}) {
      const int per = ((w.M + R - 1) / R + 255) / 256 * 256;
      for (int m0 = 0; m0 < w.M; m0 += per) {
        GemmDesc d = w;
        const int m1 = std::min(w.M, m0 + per);
        d.M = m1 - m0;
        d.A = w.A + m0;                  // A stored [K][M] (at): the chunk's columns
        if (d.Ap) d.Ap = w.Ap + m0;
        d.C = w.C + (size_t)m0 * w.ldc;  // output rows
        if (d.Abits) d.Abits = w.Abits + (size_t)(m0 / 256) * w.abits_kts * BITMAT_BLOCK_WORDS;
        d.split = w_split;
        d.variant = w_variant;
        c->w0c[R].push_back(d);
        c->w0m[R].push_back(m0);
      }
      c->w0m[R].push_back(w.M);
    }
  }
  {  // The BCE head in whole rounds: when its 256x256 tiles leave a partial last round on the
     // 256 CUs (C2: 16 x 40 = 640 tiles = 2.5 rounds), the columns of the whole rounds run as one
     // launch and the rest as 256x128 ring tiles (half the work per tile, so the last round takes
     // about half as long); elementwise the same results and the same 128-column row partials.
     // create option bce_split=0: never; set_option "bce_split" 0: one launch (A/B, tests)
    const bool on = opt.bce_split != 0;
    const GemmDesc& f = c->f_out;
    const long long tm = (f.M + 255) / 256, tn = (f.N + 255) / 256, tiles = tm * tn;
    const long long n1 = (tiles / 256) * 256 / tm;  // n-tiles of the whole rounds
    c->f_split = false;
    // (the rest at least 128 columns wide: a narrower one is no ring-kernel shape and would run on
    // the 128x128 plane kernel, which the split's same-results argument does not cover)
    if (on && f.prec != GEMM_F32 && !f.valu && gemm_bf16_wide(f) && tiles > 256 && tiles % 256 != 0 &&
        tiles % 256 <= 128 && n1 >= 1 && n1 < tn && f.N - 256 * n1 >= 128) {
      const int c0 = (int)(256 * n1);
      GemmDesc a = f, b = f;
      a.N = c0;
      a.epi.rp_ld = gemm_bce_nblk(f.N);
      b.N = f.N - c0;
      b.B = f.B + c0;
      if (b.Bp) b.Bp = f.Bp + c0;
      if (b.C) b.C = f.C + c0;
      if (b.epi.cp) b.epi.cp = f.epi.cp + c0;
      if (b.epi.x) b.epi.x = f.epi.x + c0;
      if (b.epi.xp) b.epi.xp = f.epi.xp + c0;
      if (b.epi.xbits) b.epi.xbits = f.epi.xbits + c0 / 8;  // (c0: a multiple of 256)
      b.epi.rp_ld = gemm_bce_nblk(f.N);
      b.epi.rp_off = c0 / 128;
      b.variant = 11;  // the ring kernel at 256x128 tiles
      c->f_out_a = a;
      c->f_out_b = b;
      c->f_split = true;
    }
  }
  {  // the de-interleave inside the layer-0 forward's launch (DeintJob): the forward's 256 x 256
     // tiles x split leave CUs free for its workers (C3: 192 tiles + 64 workers; C2: 96 tiles x
     // split 2 + 64 workers), so its HBM stream runs beside the k-loop instead of before it
    const GemmDesc& f0 = c->fwd_enc[0];
    const long long tiles = (long long)((f0.M + 255) / 256) * ((f0.N + 255) / 256) * f0.batch;
    const int kt = (f0.K + 63) / 64;
    int sp = 0;  // the largest split whose workgroups leave >= 32 CUs (>= 8 k-tiles per slab)
    for (int s = 1; s <= 8 && tiles * s <= 224 && (s == 1 || kt / s >= 8); ++s) sp = s;
    int sp_plan = 0, tn = 0, tm = 0;
    if (c->bits_on) gemm_bf16_wide_plan(f0, ~size_t(0), &sp_plan, &tn, &tm);
    if (opt.deint_fuse && c->bits_on && sp > 0 && f0.batch == 1 && tn == GEMM_TN_E8 && !f0.at && !f0.bt &&
        (f0.epi.mode == EPI_ACT || f0.epi.mode == EPI_STORE) && (c->D % 8) == 0 && (c->ldx % 8) == 0) {
      const int nwg = (int)tiles * sp;
      const int W = (256 - nwg) & ~7;
      const int nch = (c->kts_f + DEINT_FUSE_PB - 1) / DEINT_FUSE_PB;
      if (nch > 640) goto no_fuse;  // (the workers' LDS order table: gemm_bf16e.hip DW_MAXCH)
      float* q = nullptr;
      ALLOC(q, 2 * (size_t)nch + 8);
      c->fuse_buf = reinterpret_cast<int*>(q);
      // production order: by the slab-local k-tile at which a consumer first needs the chunk (the
      // split-K slabs' chunks in turn), then by chunk
      const int kcs = (kt + sp - 1) / sp;  // k-tiles per slab
      std::vector<std::pair<int, int>> key(nch);
      for (int ch = 0; ch < nch; ++ch) {
        const int k0 = DEINT_FUSE_PB * ch, sl = std::min(sp - 1, k0 / kcs);
        key[ch] = {k0 - sl * kcs, ch};
      }
      std::sort(key.begin(), key.end());
      std::vector<int> order(nch);
      for (int i = 0; i < nch; ++i) order[i] = key[i].second;
      if (hipMemcpy(c->fuse_buf + nch + 8, order.data(), nch * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
        g_create_err = "hipMemcpy fuse order";
        mvae_destroy(c);
        return MVAE_EINVAL;
      }
      GemmDesc f = f0;
      f.split = sp;
      f.variant = 13;  // the eight-phase kernel (its bits path carries the workers)
      DeintJob& j = f.dj;
      j.B = c->B; j.D = c->D; j.kts_f = c->kts_f; j.kts_w = c->kts_w;
      j.xbf = c->xbf; j.xbw = c->xbw; j.xbits = c->xbits; j.ldbits = c->ldbits;
      j.done = c->fuse_buf;
      j.err = c->fuse_buf + nch;
      j.order = c->fuse_buf + nch + 8;
      j.nworkers = W;
      j.nchunks = nch;
      j.diag = opt.deint_fuse_diag;
      c->f0f = f;
      c->f0fb = f0;  // (epi.only_if: the not-binary word, set per call)
      c->fuse_nchunks = nch;
      c->fuse = true;
    }
  no_fuse:;
  }
  if (opt.xbw_split == 2 && c->bits_on && !c->fuse) {  // the forward's workgroups leave CUs free?
    const GemmDesc& f0 = c->fwd_enc[0];
    int sp = 0, tn = 0, tm = 0;
    gemm_bf16_wide_plan(f0, ~size_t(0), &sp, &tn, &tm);
    const long long tiles = (long long)((f0.M + tm - 1) / tm) * ((f0.N + (tn == GEMM_TN_E8 ? 256 : tn) - 1) /
                                                                   (tn == GEMM_TN_E8 ? 256 : tn)) * f0.batch;
    c->xbw_split = tiles * sp <= 224 ? 1 : 0;
  }
  if (c->fuse) c->xbw_split = 0;  // (the fused launch's workers write xbw themselves)
  size_t ws = 0;
  auto wsz = [&](const GemmDesc& d) { ws = std::max(ws, gemm_workspace_elems(d)); };
  if (c->fuse) wsz(c->f0f);
  for (int R : {2, 4, 8})
    for (auto& d : c->w0c[R]) wsz(d);
  for (auto& d : c->fwd_enc) wsz(d);
  for (auto& d : c->bwd_dec) wsz(d);
  for (auto& d : c->bwd_enc) wsz(d);
  wsz(c->f_d1);
  wsz(c->f_d2);
  wsz(c->f_out);
  if (c->conv) wsz(c->bwd_feat);
  c->ws_elems = ws;
  // the hidden encoder layers as one launch: bf16 planes in and out, tanh / elu epilogues writing
  // planes only, widths that fit the kernel's 512-column activation block
  // hidden layers as one launch (enc_chain.hip): bf16 planes in and out, tanh / elu epilogues
  // writing planes only, widths that fit the kernel's 512-column activation block; ds[i] reads
  // ds[i - 1]'s output plane
  auto chain_of = [&](std::initializer_list<const GemmDesc*> ds, ChainArgs& ca) {
    const GemmDesc& d0 = **ds.begin();
    ca.x = d0.Ap;
    ca.ldx = d0.lda;
    ca.M = d0.M;
    ca.nl = (int)ds.size();
    ca.act = d0.epi.act;
    ca.rows = opt.enc_chain_rows;
    ca.diag = opt.diag_chain;
    bool ok = ca.nl >= 1 && ca.nl <= 4;
    const GemmDesc* prev = nullptr;
    int i = 0;
    for (const GemmDesc* p : ds) {
      if (i >= 4) break;
      const GemmDesc& d = *p;
      ok = ok && d.prec == GEMM_BF16 && !d.valu && d.epi.mode == EPI_ACT && d.epi.c32 == 0 &&
           d.epi.cp && d.epi.ncp == 1 && d.epi.padw == 2 && d.Ap && d.Bp && d.batch == 1 && !d.at &&
           !d.bt && d.K <= 512 && d.N <= 511 && d.M == ca.M && d.epi.act == ca.act;
      ChainLayer& cl = ca.l[i++];
      cl.w = d.Bp; cl.ldw = d.ldb; cl.K = d.K; cl.N = d.N; cl.out = d.epi.cp; cl.ldo = d.ldc;
      if (prev) ok = ok && d.Ap == prev->epi.cp && d.lda == prev->ldc;
      prev = p;
    }
    return ok;
  };
  if (opt.enc_chain && c->np == 1 && c->nenc == 3)
    c->chain = chain_of({&c->fwd_enc[1], &c->fwd_enc[2]}, c->chain_args);
  else if (opt.enc_chain && c->np == 1 && c->nenc == 4)
    c->chain = chain_of({&c->fwd_enc[1], &c->fwd_enc[2], &c->fwd_enc[3]}, c->chain_args);
  else if (opt.enc_chain && c->np == 1 && c->nenc == 5)
    c->chain = chain_of({&c->fwd_enc[1], &c->fwd_enc[2], &c->fwd_enc[3], &c->fwd_enc[4]}, c->chain_args);
  if (c->chain) c->chain_r = region(c, "enc_fwd_chain");
  if (opt.dec_chain && c->np == 1) c->dchain = chain_of({&c->f_d1, &c->f_d2}, c->dchain_args);
  if (c->dchain) c->dchain_r = region(c, "dec_fwd_chain");
  if (opt.plan_log) {
    // the GEMM plans of this context (diagnostics): shape, arithmetic, kernel, split-K + combine
    auto show = [&](const GemmDesc& d, int r) {
      const int sp = gemm_plan_split(d, ws);
      const bool wide = gemm_bf16_wide(d);
      std::fprintf(stderr, "[mvae plan] %-16s M %6d N %6d K %6d batch %d prec %d valu %d wide %d tile %dx%d split %d\n",
                   r >= 0 ? c->region_names[r].c_str() : "?", d.M, d.N, d.K, d.batch, d.prec, d.valu,
                   (int)wide, wide ? gemm_bf16_wide_tm(d, ws) : 0, wide ? gemm_bf16_wide_tn(d, ws) : 0, sp);
    };
    for (size_t i = 0; i < c->fwd_enc.size(); ++i) show(c->fwd_enc[i], c->fwd_enc_r[i]);
    if (c->chain)
      std::fprintf(stderr, "[mvae plan] enc_fwd_chain    layers 1..%d in one launch, %d rows per workgroup\n",
                   c->nenc - 1, enc_chain_rows(c->chain_args.M, c->chain_args.rows));
    show(c->f_d1, c->f_d1_r); show(c->f_d2, c->f_d2_r); show(c->f_out, c->f_out_r);
    if (c->dchain)
      std::fprintf(stderr, "[mvae plan] dec_fwd_chain    f_d1, f_d2 in one launch, %d rows per workgroup\n",
                   enc_chain_rows(c->dchain_args.M, c->dchain_args.rows));
    for (size_t i = 0; i < c->bwd_dec.size(); ++i) show(c->bwd_dec[i], c->bwd_dec_r[i]);
    for (size_t i = 0; i < c->bwd_enc.size(); ++i) show(c->bwd_enc[i], c->bwd_enc_r[i]);
  }
  ALLOC(c->ws, ws);
  ALLOC(c->ws_side, ws);
#undef ALLOC
  {
    int lo = 0, hi = 0;
    hipError_t se = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (se == hipSuccess) se = hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, lo);
    if (se == hipSuccess && c->diag_shadow) {
      se = hipStreamCreateWithPriority(&c->stage, hipStreamNonBlocking, lo);
      void* q = nullptr;
      if (se == hipSuccess) se = hipMalloc(&q, (size_t)3 * c->B * c->ldx * sizeof(unsigned short));
      if (se == hipSuccess) { c->allocs.push_back(q); c->shadow = static_cast<unsigned short*>(q); }
    }
    if (se == hipSuccess) se = hipEventCreateWithFlags(&c->xbw_ev, hipEventDisableTiming);
    for (int i = 0; se == hipSuccess && i < 16; ++i) {
      hipEvent_t ev = nullptr;
      // stream-to-stream ordering on this device only: no system-scope fence. The producer side
      // of every fork / join is a kernel, and a kernel's end-of-dispatch release is at least agent
      // scope -- the whole device, every XCD's L2 written back -- which is what a consumer kernel
      // on another queue of the same device needs; system scope adds only host / peer visibility,
      // which nothing here reads through these events (they order GPU work; the host waits on
      // stream / device synchronisation, which keeps its own fences). Measured: -0.009 ms per step
      // at C2 / C3 (profiles/r5/r5z_events_without_system_fence.txt); the bitwise tests of the
      // side-stream schedules (test_gpu_r2.py early Adam, side_mask) run with these events.
      se = hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence);
      if (se == hipSuccess) c->sync_ev.push_back(ev);
    }
    if (se != hipSuccess) {
      g_create_err = std::string("side stream: ") + hipGetErrorString(se);
      mvae_destroy(c);
      return (int)se;
    }
  }
  *out = c;
  return MVAE_OK;
}

int mvae_param_count(mvae_ctx* ctx) { return ctx ? 2 * ctx->nenc + 4 + 8 + (ctx->conv ? 4 : 0) : MVAE_EINVAL; }

int mvae_param_info(mvae_ctx* ctx, int kind, int index, mvae_tensor* out) {
  if (!ctx || !out) return MVAE_EINVAL;
  const int n = ctx->nenc;
  const int count = mvae_param_count(ctx);
  if (index < 0 || index >= count) return fail(ctx, MVAE_EINVAL, "param index out of range");
  std::memset(out, 0, sizeof(*out));
  const Block* cvb = nullptr;
  if (ctx->conv) {  // enc_conv1_W, enc_conv1_b, enc_conv2_W, enc_conv2_b come first
    if (index < 4) cvb = index < 2 ? &ctx->cv1 : &ctx->cv2;
    else index -= 4;
  }
  // resolve (name, block-relative pointer) in reference creation order (11a/vae.py:85-153)
  const Block* blk = nullptr;
  bool bias = false;
  int col0 = 0, cols = 0, ld = 0, enc_part = 0;
  std::string name;
  if (cvb) {
    blk = cvb;
    bias = index & 1;
    name = std::string(index < 2 ? "enc_conv1" : "enc_conv2") + (bias ? "_b" : "_W");
    cols = blk->N; ld = blk->ld; enc_part = 1;
  } else if (index < 2 * n) {
    const int i = index / 2;
    bias = index & 1;
    blk = &ctx->enc[i];
    name = "enc_h" + std::to_string(i) + (bias ? "_b" : "_W");
    cols = blk->N; ld = blk->ld; enc_part = 1;
  } else if (index < 2 * n + 4) {
    const int j = index - 2 * n;
    blk = &ctx->head;
    bias = j & 1;
    const bool logsig = j >= 2;
    name = std::string(logsig ? "enc_out_log_sigma" : "enc_out_mean") + (bias ? "_b" : "_W");
    col0 = logsig ? ctx->L : 0; cols = ctx->L; ld = blk->ld; enc_part = 1;
  } else if (index < 2 * n + 10) {
    const int j = index - 2 * n - 4;
    const Block* bl[3] = {&ctx->v1, &ctx->v2, &ctx->vo};
    const char* nm[3] = {"dec_h1", "dec_h2", "dec_out_mean"};
    blk = bl[j / 2];
    bias = j & 1;
    name = std::string(nm[j / 2]) + (bias ? "_b" : "_W");
    cols = blk->N; ld = blk->ld;
  } else {  // dead decoder log-sigma variables (11a/vae.py:147,153): allocated, never trained
    bias = (index - 2 * n - 10) == 1;
    std::strncpy(out->name, bias ? "dec_out_log_sigma_b" : "dec_out_log_sigma_W", sizeof(out->name) - 1);
    if (kind != MVAE_KIND_PARAM) return fail(ctx, MVAE_EINVAL, "dead variables have no optimizer state");
    out->data = ctx->dead + (bias ? (size_t)ctx->d1 * ctx->D : 0);
    out->rows = bias ? 1 : ctx->d1;
    out->cols = ctx->D;
    out->ld = ctx->D;
    out->trained_by = 0;
    return MVAE_OK;
  }
  std::strncpy(out->name, name.c_str(), sizeof(out->name) - 1);
  float* base = nullptr;
  switch (kind) {
    case MVAE_KIND_PARAM: base = ctx->theta; break;
    case MVAE_KIND_GRAD1: base = ctx->grads; break;
    case MVAE_KIND_GRAD2: base = enc_part ? ctx->grads + ctx->n_all : nullptr; break;
    case MVAE_KIND_M1: base = ctx->adam; break;
    case MVAE_KIND_V1: base = ctx->adam + ctx->n_all; break;
    case MVAE_KIND_M2: base = enc_part ? ctx->adam + 2 * ctx->n_all : nullptr; break;
    case MVAE_KIND_V2: base = enc_part ? ctx->adam + 2 * ctx->n_all + ctx->n_enc : nullptr; break;
    default: return fail(ctx, MVAE_EINVAL, "bad kind");
  }
  if (!base) return fail(ctx, MVAE_EINVAL, "decoder variables are not trained by the metric optimizer");
  out->data = base + blk->off + (bias ? (size_t)blk->K * ld : 0) + col0;
  out->rows = bias ? 1 : blk->K;
  out->cols = cols;
  out->ld = ld;
  out->trained_by = enc_part ? 3 : 1;
  return MVAE_OK;
}

int mvae_buffer(mvae_ctx* ctx, int which, float** ptr, size_t* count) {
  if (!ctx || !ptr || !count) return MVAE_EINVAL;
  switch (which) {
    case MVAE_BUF_PARAMS: *ptr = ctx->theta; *count = ctx->n_all; break;
    case MVAE_BUF_GRADS: *ptr = ctx->grads; *count = ctx->n_all + ctx->n_enc; break;
    case MVAE_BUF_ADAM: *ptr = ctx->adam; *count = 2 * ctx->n_all + 2 * ctx->n_enc; break;
    case MVAE_BUF_LOSSES: *ptr = ctx->losses; *count = 5; break;
    case MVAE_BUF_COLSQ: *ptr = ctx->colsq; *count = 2 * (size_t)ctx->L; break;
    case MVAE_BUF_COLDOT: *ptr = ctx->coldot; *count = ctx->L; break;
    case MVAE_BUF_DIST: *ptr = ctx->dist; *count = ctx->B; break;
    case MVAE_BUF_GRADS_DEC: *ptr = ctx->grads + ctx->n_enc; *count = ctx->n_all - ctx->n_enc; break;
    case MVAE_BUF_DEAD: *ptr = ctx->dead; *count = (size_t)ctx->d1 * ctx->D + ctx->D; break;
    case MVAE_BUF_EPS:
      if (ctx->eps_lazy) {  // the last forward's internal draw, written out on request
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess)
          e = launch_normal(ctx->eps, 3, ctx->B, ctx->L, ctx->le.Bg, ctx->le.off, ctx->le.seed,
                            ctx->le.counter, nullptr);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) return fail(ctx, (int)e, std::string("eps: ") + hipGetErrorString(e));
        ctx->eps_lazy = false;
      }
      *ptr = ctx->eps; *count = (size_t)3 * ctx->B * ctx->L; break;
    case MVAE_BUF_DYN:
      if (!ctx->dyn) return fail(ctx, MVAE_EINVAL, "no dyn flag in this precision mode");
      *ptr = reinterpret_cast<float*>(ctx->dyn_cur ? ctx->dyn_cur : ctx->dyn); *count = 1; break;
    default: return fail(ctx, MVAE_EINVAL, "bad buffer id");
  }
  return MVAE_OK;
}

int mvae_get_step(mvae_ctx* ctx, int64_t* t1, int64_t* t2) {
  if (!ctx || !t1 || !t2) return MVAE_EINVAL;
  *t1 = ctx->t1; *t2 = ctx->t2;
  return MVAE_OK;
}

int mvae_set_step(mvae_ctx* ctx, int64_t t1, int64_t t2) {
  if (!ctx || t1 < 0 || t2 < 0) return MVAE_EINVAL;
  ctx->t1 = t1; ctx->t2 = t2;
  // recompute the fp32 beta powers exactly as TF accumulates them (one fp32 multiply per step)
  for (int o = 0; o < 2; ++o) {
    const int64_t t = o == 0 ? t1 : t2;
    float b1p = ctx->cfg.beta1, b2p = ctx->cfg.beta2;
    for (int64_t s = 0; s < t; ++s) { b1p *= ctx->cfg.beta1; b2p *= ctx->cfg.beta2; }
    ctx->b1p[o] = b1p; ctx->b2p[o] = b2p;
  }
  return MVAE_OK;
}

int mvae_get_rng(mvae_ctx* ctx, uint64_t* train, uint64_t* eval) {
  if (!ctx || !train || !eval) return MVAE_EINVAL;
  *train = ctx->rng_counter; *eval = ctx->rng_eval;
  return MVAE_OK;
}

int mvae_set_rng(mvae_ctx* ctx, uint64_t train, uint64_t eval) {
  if (!ctx || (train | eval) & EVAL_STREAM) return MVAE_EINVAL;
  ctx->rng_counter = train; ctx->rng_eval = eval;
  return MVAE_OK;
}

int mvae_set_shard(mvae_ctx* ctx, int64_t row_offset) {
  if (!ctx) return MVAE_EINVAL;
  if (row_offset < 0 || row_offset + ctx->B > ctx->cfg.global_batch)
    return fail(ctx, MVAE_EINVAL, "row_offset outside [0, global_batch - batch]");
  ctx->row_off = (int)row_offset;
  return MVAE_OK;
}

int mvae_sync_params(mvae_ctx* ctx, void* stream) {
  if (!ctx) return MVAE_EINVAL;
  MV_CHECK(launch_split_planes(ctx->theta, ctx->n_all, planes_of(ctx, ctx->theta), (hipStream_t)stream));
  return MVAE_OK;
}

// ------------------------------------------------------------------ phases
static int run(mvae_ctx* ctx, const GemmDesc& d, hipStream_t st, int r = -1) {
  TimeScope ts(ctx, r < 0 ? region(ctx, "other_gemm") : r, st);
  const bool sd = st == ctx->side && ctx->side;
  float* ws = sd ? ctx->ws_side : ctx->ws;
  // descriptors name the pixel flag by its first slot; the last de-interleave raised dyn_cur
  if (ctx->dyn_cur && ctx->dyn_cur != ctx->dyn &&
      (d.dynA == ctx->dyn || d.epi.xdyn == ctx->dyn || d.anb == ctx->dyn + 2)) {
    GemmDesc dd = d;
    if (dd.dynA == ctx->dyn) dd.dynA = ctx->dyn_cur;
    if (dd.epi.xdyn == ctx->dyn) dd.epi.xdyn = ctx->dyn_cur;
    if (dd.epi.xnb == ctx->dyn + 2) dd.epi.xnb = ctx->dyn_cur + 2;
    if (dd.anb == ctx->dyn + 2) dd.anb = ctx->dyn_cur + 2;
    dd.prio = ctx->e8_prio;
    MV_CHECK(gemm_run(dd, ws, ctx->ws_elems, st));
    return MVAE_OK;
  }
  if (ctx->e8_prio) {
    GemmDesc dd = d;
    dd.prio = ctx->e8_prio;
    MV_CHECK(gemm_run(dd, ws, ctx->ws_elems, st));
    return MVAE_OK;
  }
  MV_CHECK(gemm_run(d, ws, ctx->ws_elems, st));
  return MVAE_OK;
}

// `to` waits for the work enqueued on `from` so far
static int stream_wait(mvae_ctx* ctx, hipStream_t from, hipStream_t to) {
  hipEvent_t ev = ctx->sync_ev[ctx->sync_next++ % ctx->sync_ev.size()];
  MV_CHECK(hipEventRecord(ev, from));
  MV_CHECK(hipStreamWaitEvent(to, ev, 0));
  return MVAE_OK;
}
#define TIMED(name) TimeScope ts_##__LINE__(ctx, region(ctx, name), st)

// Encoder pass over the stacked [rot | lock | key] rows. draw: ENC_TRAIN samples eps from the
// training counter when eps == NULL, ENC_EVAL from the inference counter; ENC_MEAN computes the
// latent mean/log-sigma heads only (transform: no eps, no z, no column statistics).
enum { ENC_TRAIN = 0, ENC_EVAL = 1, ENC_MEAN = 2 };

static int shadow_deint(mvae_ctx* ctx, hipStream_t st);

static int encode(mvae_ctx* ctx, const float* x, const float* eps, hipStream_t st, int draw = ENC_TRAIN) {
  auto c = ctx;
  c->last_x = x;
  if (c->side && c->side_pending) {  // an early-Adam backward whose mvae_adam never came
    c->side_pending = false;
    c->early_fork = false;
    MV_CHECK(hipEventRecord(c->sync_ev[c->sync_next % c->sync_ev.size()], c->side));
    MV_CHECK(hipStreamWaitEvent(st, c->sync_ev[c->sync_next++ % c->sync_ev.size()], 0));
  }
  if (c->xbw_pending) {  // the last transpose read the forward BitMat this pass rewrites
    c->xbw_pending = false;
    MV_CHECK(hipStreamWaitEvent(st, c->xbw_ev, 0));
  }
  if (c->stage_pending) {  // (diagnostics) the last shadow pass ends before this step
    c->stage_pending = false;
    MV_CHECK(hipEventRecord(c->sync_ev[c->sync_next % c->sync_ev.size()], c->stage));
    MV_CHECK(hipStreamWaitEvent(st, c->sync_ev[c->sync_next++ % c->sync_ev.size()], 0));
  }
  bool f0_done = false;  // the layer-0 forward ran with the fused de-interleave
  if (c->fuse && !c->diag_skip_deint && !c->diag_shadow && (reinterpret_cast<uintptr_t>(x) % 16) == 0) {
    // one launch: the de-interleave's workers beside the forward GEMM's tiles (DeintJob); then the
    // grey pass (zeroing the chunk counters) and the forward on the planes, both returning at once
    // for a 0/1 batch
    int* prev = c->dyn_cur ? c->dyn_cur : c->dyn;
    int* cur = prev == c->dyn ? c->dyn + 1 : c->dyn;
    {
      TIMED("deint_fwd0");
      GemmDesc f = c->f0f;
      f.dj.x = x;
      f.dj.dyn = cur;
      f.dj.dyn_next = prev;
      if (f.dynA == c->dyn) f.dynA = cur;
      MV_CHECK(gemm_run(f, c->ws, c->ws_elems, st));
    }
    {
      TIMED("deint_grey");
      MV_CHECK(launch_deint_grey(x, c->B, c->D, cur, c->xs, planes_of(c, c->xs), c->ldx, c->x32dyn, c->fuse_buf,
                                 c->fuse_nchunks, st));
      GemmDesc fb = c->f0fb;
      if (fb.dynA == c->dyn) fb.dynA = cur;
      fb.anb = cur + 2;
      fb.epi.only_if = cur + 2;
      MV_CHECK(gemm_run(fb, c->ws, c->ws_elems, st));
    }
    c->dyn_cur = cur;
    f0_done = true;
  } else if (!(c->diag_skip_deint && c->dyn_cur)) {  // (diagnostics: the stale image of the last pass)
    TIMED("deinterleave");
    // the flag's slots alternate: this pass raises the one the previous pass zeroed and zeroes
    // the previous one (its readers are all behind on this stream), no memset launch per step
    int* prev = c->dyn_cur ? c->dyn_cur : c->dyn;
    int* cur = c->dyn ? (prev == c->dyn ? c->dyn + 1 : c->dyn) : nullptr;
    if (c->bits_on) {  // the BitMats and target bits; the planes only for a batch not all 0 / 1
      const bool split = c->xbw_split && draw == ENC_TRAIN;  // (eval passes need no xbw)
      MV_CHECK(launch_deint_bits(x, c->B, c->D, c->xbf, c->kts_f, c->xbw, c->kts_w, c->xbits, c->ldbits, cur,
                                 prev, c->xs, planes_of(c, c->xs), c->ldx, c->x32dyn, st,
                                 split ? (c->deint_variant == 8 ? 9 : 7) : c->deint_variant));
      if (split) {  // xbw from xbf on the side stream, beside the layer-0 forward
        const bool two = c->use_side && c->side;
        hipStream_t sd = two ? c->side : st;
        if (two)
          if (int rc = stream_wait(c, st, sd)) return rc;
        MV_CHECK(launch_bits_transpose(c->xbf, c->kts_f, c->xbw, c->kts_w, c->B, sd));
        MV_CHECK(hipEventRecord(c->xbw_ev, sd));
        c->xbw_pending = true;
      }
    }
    else
      MV_CHECK(launch_deinterleave(x, c->xs, planes_of(c, c->xs), cur, c->dyn ? prev : nullptr, c->B,
                                   c->D, c->ldx, c->x32mask, c->x32dyn, st, c->xbits, c->ldbits));
    c->dyn_cur = cur;
  }
  if (c->diag_shadow && c->diag_shadow_at == 0 && draw == ENC_TRAIN) {
    int rc = shadow_deint(c, st);
    if (rc) return rc;
  }
  const size_t ne = (size_t)3 * c->B * c->L;
  if (draw != ENC_MEAN) {
    // eps of this forward: the caller's draws (copied: the backward needs them after the
    // caller's buffer may be gone), or the next call of the training / inference Philox
    // stream, regenerated inside the latent kernels (no eps buffer traffic)
    LatentEps le;
    le.seed = c->cfg.seed;
    le.Bg = c->cfg.global_batch;
    le.off = c->row_off;
    if (eps) {
      TIMED("eps_rng");
      MV_CHECK(hipMemcpyAsync(c->eps, eps, ne * sizeof(float), hipMemcpyDeviceToDevice, st));
      le.buf = c->eps;
    } else {
      le.counter = draw == ENC_TRAIN ? c->rng_counter++ : (EVAL_STREAM | c->rng_eval++);
    }
    c->eps_lazy = le.buf == nullptr;
    c->le = le;
  }
  if (c->conv) {  // the tower: xs pixels -> xf features (the FC layer-0 operand)
    const ConvTower& T = c->tower;
    const float* w2 = c->theta + c->cv2.off;
    const int nimg = 3 * c->B;
    {
      TIMED("conv1_fwd");
      MV_CHECK(launch_conv1_fwd(T, c->xs, c->ldx, c->theta + c->cv1.off, nimg, st));
    }
    {
      TIMED("conv2_fwd");
      if (T.mfma) MV_CHECK(launch_conv2_wprep(T, w2, st));
      MV_CHECK(launch_conv2(T, true, T.n1, T.n1b, w2, T.w2f, T.a2, nimg, st));
    }
    {
      TIMED("lrn2_pool2_fwd");
      MV_CHECK(launch_lrn2_pool2_fwd(T, nimg, c->xf, c->ldf, c->xf32, planes_of(c, c->xf), st));
    }
  }
  for (size_t i = f0_done ? 1 : 0; i < c->fwd_enc.size(); ++i) {
    if (c->chain && i == 1) {  // the hidden layers 1 .. nenc-1
      TimeScope ts(c, c->chain_r, st);
      MV_CHECK(launch_enc_chain(c->chain_args, st));
      i = c->nenc - 1;
      continue;
    }
    int rc = run(c, c->fwd_enc[i], st, c->fwd_enc_r[i]);
    if (rc) return rc;
  }
  if (draw == ENC_MEAN) return MVAE_OK;
  {
    TIMED("latent_fwd");
    MV_CHECK(launch_latent_fwd(c->ms, c->le, c->z, planes_of(c, c->z), c->zmask, c->B, c->L, c->ldz,
                               c->rowfwd, st));
  }
  if (c->cfg.metric == MVAE_METRIC_COSINE) {
    TIMED("colsq");
    MV_CHECK(launch_colstats(0, c->z, c->B, c->L, c->ldz, nullptr, nullptr, c->cspart, c->nchunk,
                             c->colsq, st, c->cscnt));
  }
  return MVAE_OK;
}

// the decoder's hidden layers: one chain launch or one GEMM each
static int decode_hidden(mvae_ctx* ctx, hipStream_t st) {
  if (ctx->dchain) {
    TimeScope ts(ctx, ctx->dchain_r, st);
    MV_CHECK(launch_enc_chain(ctx->dchain_args, st));
    return MVAE_OK;
  }
  int rc = run(ctx, ctx->f_d1, st, ctx->f_d1_r);
  return rc ? rc : run(ctx, ctx->f_d2, st, ctx->f_d2_r);
}

extern "C" int mvae_forward(mvae_ctx* ctx, const float* x, const float* eps, void* stream) {
  if (!ctx || !x) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int rc = encode(ctx, x, eps, st);
  if (rc) return rc;
  if ((rc = decode_hidden(ctx, st))) return rc;
  if (ctx->f_split && ctx->use_split) {
    if ((rc = run(ctx, ctx->f_out_a, st, ctx->f_out_r))) return rc;
    if ((rc = run(ctx, ctx->f_out_b, st, ctx->f_out_r))) return rc;
  } else if ((rc = run(ctx, ctx->f_out, st, ctx->f_out_r))) {
    return rc;
  }
  ctx->phase = 1;
  return MVAE_OK;
}

extern "C" int mvae_metric(mvae_ctx* ctx, const float* areas, void* stream) {
  if (!ctx || !areas) return MVAE_EINVAL;
  if (ctx->phase != 1) return fail(ctx, MVAE_ESTATE, "mvae_metric before mvae_forward");
  hipStream_t st = (hipStream_t)stream;
  auto c = ctx;
  {
    TIMED("metric_loss");
    MV_CHECK(launch_metric(c->z, c->ldz, c->rowfwd, c->rowpart, c->nblk, areas, c->colsq, c->B, c->L,
                           c->cfg.metric, c->cfg.reciprocal, c->cfg.deform_weight, c->inv_bg,
                           c->rowvals, c->dist, c->draw, st));
    MV_CHECK(launch_loss_reduce(c->rowvals, c->B, c->inv_bg, c->losses, st));
  }
  if (c->cfg.metric == MVAE_METRIC_COSINE) {
    TIMED("coldot");
    MV_CHECK(launch_colstats(1, c->z, c->B, c->L, c->ldz, c->colsq, c->draw, c->cspart, c->nchunk,
                             c->coldot, st, c->cscnt));
  }
  ctx->phase = 2;
  return MVAE_OK;
}

// Backward in R + 2 parts (R = the layer-0 weight-gradient chunks, option "wgrad0_chunks";
// phase 2 -> 4 ... -> 3); after part k the ranges mvae_grad_range(ctx, k, i, ...) hold final
// (rank-local) gradients on the caller's stream. Part 0: the decoder; part 1: the latent head
// backward, the encoder dgrad chain and layer-0 chunk 0; parts 2 .. R: layer-0 chunks 1 .. R-1
// (the conv tower's backward after the last chunk); part R + 1: joins the side stream.
// The dgrad chain (decoder output -> ... -> encoder layer 1) runs on the caller's stream; each
// weight gradient runs on the side stream as soon as its dZ exists, beside the chain (the
// chain's GEMMs leave CUs idle: few tiles, split-K reductions). Part 0 joins the decoder's
// weight gradients, the last part the encoder's (the layer-0 weight gradient runs on the
// caller's stream). join_dec = false (the single-call mvae_backward) leaves the decoder's
// weight gradients running beside the encoder chain too.
// layer-0 weight-gradient chunks in use: the option's R, or fewer when the block has fewer rows
// than R chunks of 256 (chunk boundaries are tile multiples)
static int w0n(const mvae_ctx* c) { return c->w0_chunks == 1 ? 1 : (int)c->w0c[c->w0_chunks].size(); }
static int nparts(const mvae_ctx* c) { return w0n(c) + 2; }

// (diagnostics) the shadow de-interleave on the stage stream, after the work on st so far
static int shadow_deint(mvae_ctx* ctx, hipStream_t st) {
  auto c = ctx;
  if (!c->last_x || !c->stage) return MVAE_OK;
  MV_CHECK(hipEventRecord(c->sync_ev[c->sync_next % c->sync_ev.size()], st));
  MV_CHECK(hipStreamWaitEvent(c->stage, c->sync_ev[c->sync_next++ % c->sync_ev.size()], 0));
  MV_CHECK(launch_deinterleave_grid(c->last_x, c->shadow, c->B, c->D, c->ldx, c->diag_shadow, c->stage));
  c->stage_pending = true;
  return MVAE_OK;
}

// Adam's arguments for this step (TF ApplyAdam: lr_t = lr * sqrt(1 - beta2_power) /
// (1 - beta1_power), all fp32), the whole index range
static AdamArgs adam_args(const mvae_ctx* c) {
  AdamArgs a;
  a.theta = c->theta; a.g1 = c->grads; a.g2 = c->grads + c->n_all;
  a.m1 = c->adam; a.v1 = c->adam + c->n_all;
  a.m2 = c->adam + 2 * c->n_all; a.v2 = c->adam + 2 * c->n_all + c->n_enc;
  a.n_all = c->n_all; a.n_enc = c->n_enc;
  a.b1 = c->cfg.beta1; a.b2 = c->cfg.beta2; a.eps = c->cfg.epsilon;
  a.lr1 = (c->cfg.lr[0] * std::sqrt(1.f - c->b2p[0])) / (1.f - c->b1p[0]);
  a.lr2 = (c->cfg.lr[1] * std::sqrt(1.f - c->b2p[1])) / (1.f - c->b1p[1]);
  a.tp = planes_of(c, c->theta);
  a.nt = c->adam_nt;
  return a;
}

static int backward_part(mvae_ctx* ctx, int part, hipStream_t st, bool join_dec) {
  auto c = ctx;
  int rc;
  if (c->diag_shadow && part == 0 && c->diag_shadow_at == 1 && (rc = shadow_deint(c, st))) return rc;
  if (c->diag_shadow && part == 1 && c->diag_shadow_at == 2 && (rc = shadow_deint(c, st))) return rc;
  const int R = w0n(c);
  const bool two = c->use_side && c->side;
  hipStream_t sd = two ? c->side : st;
  auto fork = [&]() -> int { return two ? stream_wait(c, st, sd) : MVAE_OK; };
  // join whatever the side stream still holds, even if "side_stream" was switched off after
  // the fork (the pending weight gradients would otherwise race with Adam / the all-reduce)
  auto join = [&]() -> int {
    if (!c->side || !c->side_pending) return MVAE_OK;
    c->side_pending = false;
    return stream_wait(c, c->side, st);
  };
  const int n = c->nenc;
  auto w0chunk = [&](int r) -> int {  // layer-0 weight gradient, chunk r of R
    if (c->xbw_pending) {  // its BitMat, transposed on the side stream (xbw_split)
      c->xbw_pending = false;
      MV_CHECK(hipStreamWaitEvent(st, c->xbw_ev, 0));
    }
    const GemmDesc& d = R == 1 ? c->bwd_enc[n] : c->w0c[c->w0_chunks][r];
    return run(c, d, st, c->bwd_enc_r[n]);
  };
  // early Adam with R > 1 chunks: chunk k's rows (final in g1 and g2 after its GEMM) updated on the
  // side stream beside chunk k + 1's GEMM, which reads no weights (elementwise: the same values)
  auto chunk_adam = [&](int k) -> int {
    if (!c->early_fork || !c->side || R == 1 || k >= R - 1 || c->enc[0].off != 0) return MVAE_OK;
    AdamArgs a = adam_args(c);
    a.i0 = c->adam0_from;
    a.i1 = (size_t)c->w0m[c->w0_chunks][k + 1] * c->enc[0].ld;
    if (int rc2 = stream_wait(c, st, c->side)) return rc2;
    MV_CHECK(launch_adam(a, c->side));
    c->adam0_from = a.i1;
    return MVAE_OK;
  };
  auto tower = [&]() -> int {  // back through the conv tower (its gradients final after it)
    if (!c->conv) return MVAE_OK;
    const ConvTower& T = c->tower;
    float* g1 = c->grads;
    float* g2 = c->grads + c->n_all;
    int rc2;
    if ((rc2 = run(c, c->bwd_feat, st, c->bwd_feat_r))) return rc2;
    {
      TIMED("pool2_bwd");
      MV_CHECK(launch_pool2_bwd(T, c->dxf, c->ldf, c->B, st));
    }
    {
      TIMED("conv2_wgrad");
      MV_CHECK(launch_conv2_wgrad(T, c->B, g1 + c->cv2.off, g2 + c->cv2.off, st));
    }
    {
      TIMED("conv2_dgrad");
      MV_CHECK(launch_conv2(T, false, T.da2, T.da2b, c->theta + c->cv2.off, T.w2d, T.dn1, 4 * c->B, st));
    }
    {
      TIMED("conv1_wgrad");
      MV_CHECK(launch_conv1_wgrad(T, c->xs, c->ldx, c->B, g1 + c->cv1.off, g2 + c->cv1.off, st));
    }
    return MVAE_OK;
  };
  if (part == 0) {
    // bwd_dec: W_out, D_out, W_d2, D_d2, W_d1, D_z
    if (!(c->side_mask & 1)) {  // option side_mask: the decoder's weight gradients in order here
      for (int i = 0; i < 6; ++i)
        if ((rc = run(c, c->bwd_dec[i], st, c->bwd_dec_r[i]))) return rc;
    } else {
      if ((rc = fork())) return rc;
      c->side_pending = two;
      if ((rc = run(c, c->bwd_dec[0], sd, c->bwd_dec_r[0]))) return rc;
      if ((rc = run(c, c->bwd_dec[1], st, c->bwd_dec_r[1]))) return rc;
      if ((rc = fork())) return rc;
      if ((rc = run(c, c->bwd_dec[2], sd, c->bwd_dec_r[2]))) return rc;
      if ((rc = run(c, c->bwd_dec[3], st, c->bwd_dec_r[3]))) return rc;
      if ((rc = fork())) return rc;
      if ((rc = run(c, c->bwd_dec[4], sd, c->bwd_dec_r[4]))) return rc;
      if ((rc = run(c, c->bwd_dec[5], st, c->bwd_dec_r[5]))) return rc;
    }
    if (join_dec && (rc = join())) return rc;
  } else if (part == 1) {
    {
      TIMED("latent_bwd");
      MV_CHECK(launch_latent_bwd(c->ms, c->le, c->dzdec, c->draw, c->colsq, c->coldot,
                                 c->B, c->L, c->cfg.metric, c->cfg.deform_weight, c->inv_bg,
                                 c->dhead32 ? c->dhead : nullptr,
                                 c->ld_dh, planes_of(c, c->dhead), st));
    }
    // bwd_enc: [dgrad(n) .. dgrad(1), wgrad(0) | wgrad(n), wgrad(n-1) .. wgrad(1)]; dgrad(i)
    // produces dZ_{i-1}, wgrad(i) needs dZ_i (dgrad(n) = the head's: dZ of layer n-1)
    auto wg = [&](int i) -> const GemmDesc& { return c->bwd_enc[c->enc_part1 + (n - i)]; };
    auto wr = [&](int i) { return c->bwd_enc_r[c->enc_part1 + (n - i)]; };
    const bool es = (c->side_mask & 2) != 0;  // the encoder's weight gradients on the side stream
    hipStream_t se = es ? sd : st;
    if (es) {
      if ((rc = fork())) return rc;
      c->side_pending = two;
    }
    if ((rc = run(c, wg(n), se, wr(n)))) return rc;  // head weight gradient (dhead)
    for (int j = 0; j < n; ++j) {
      const int i = n - j;  // dgrad(i) -> dZ_{i-1}
      if ((rc = run(c, c->bwd_enc[j], st, c->bwd_enc_r[j]))) return rc;
      if (i - 1 >= 1) {
        if (es && (rc = fork())) return rc;
        if ((rc = run(c, wg(i - 1), se, wr(i - 1)))) return rc;
      }
    }
    // early Adam: the side stream's Adam of the blocks after layer 0 (mvae_adam) may start once
    // the dgrad chain -- the last reader of their weights -- is done, beside the layer-0
    // weight gradient. Only in the single-call mvae_backward (join_dec false): a caller of
    // mvae_backward_part all-reduces the gradients between the parts and mvae_adam, and the side
    // stream is not ordered after those collectives
    c->early_fork = false;
    c->adam0_from = 0;
    if (c->early_adam && two && !join_dec) {
      if ((rc = fork())) return rc;
      c->early_fork = true;
      c->side_pending = true;  // (if mvae_adam never comes, the next encode() joins the side stream)
    }
    if ((rc = w0chunk(0))) return rc;
    if ((rc = chunk_adam(0))) return rc;
    if (R == 1 && (rc = tower())) return rc;
  } else if (part <= R) {
    if ((rc = w0chunk(part - 1))) return rc;
    if ((rc = chunk_adam(part - 1))) return rc;
    if (part == R && (rc = tower())) return rc;
  } else if (!c->early_fork) {
    if ((rc = join())) return rc;
  }
  // (early Adam: mvae_adam joins the side stream after its last launch there -- one cross-stream
  // wait per step instead of two, each ~10 us of idle GPU at the end of the step, r5y)
  c->bpart = part + 1;
  ctx->phase = part == R + 1 ? 3 : 4;
  return MVAE_OK;
}

extern "C" int mvae_backward_nparts(mvae_ctx* ctx) { return ctx ? nparts(ctx) : MVAE_EINVAL; }

extern "C" int mvae_backward_part(mvae_ctx* ctx, int part, void* stream) {
  if (!ctx) return MVAE_EINVAL;
  if (part < 0 || part >= nparts(ctx))
    return fail(ctx, MVAE_EINVAL, "backward part must be in [0, mvae_backward_nparts)");
  const bool ok = part == 0 ? ctx->phase == 2 : (ctx->phase == 4 && ctx->bpart == part);
  if (!ok) return fail(ctx, MVAE_ESTATE, "mvae_backward_part out of order");
  return backward_part(ctx, part, (hipStream_t)stream, true);
}

extern "C" int mvae_backward(mvae_ctx* ctx, void* stream) {
  if (!ctx) return MVAE_EINVAL;
  if (ctx->phase != 2) return fail(ctx, MVAE_ESTATE, "mvae_backward before mvae_metric");
  // early Adam: the layer-0 weight gradient in early_chunks chunks (default 1), Adam of each chunk
  // but the last beside the next chunk's GEMM (r5zw: -0.003 to -0.034 ms at 2 chunks with the
  // chunks' own plans; with the one-GEMM plan pinned, 2 chunks cost +1-2.5 %, r6l)
  const int w0 = ctx->w0_chunks;
  if (ctx->early_adam && ctx->use_side && ctx->side && w0 == 1 && ctx->early_chunks > 1 && !ctx->conv &&
      ctx->enc[0].off == 0)
    ctx->w0_chunks = ctx->early_chunks;
  int rc = MVAE_OK;
  for (int part = 0; part < nparts(ctx) && !rc; ++part) rc = backward_part(ctx, part, (hipStream_t)stream, false);
  ctx->w0_chunks = w0;
  return rc;
}

extern "C" int mvae_set_option(mvae_ctx* ctx, const char* name, int value) {
  if (!ctx || !name) return MVAE_EINVAL;
  const std::string k(name);
  if (k == "side_stream") {
    // not while forked weight gradients are still un-joined (mid-backward)
    if (ctx->side_pending)
      return fail(ctx, MVAE_ESTATE, "side_stream cannot change while side-stream work is pending");
    ctx->use_side = value != 0;
    return MVAE_OK;
  }
  if (k == "bce_split") {
    ctx->use_split = value != 0;
    return MVAE_OK;
  }
  if (k == "side_mask") {
    if (value < 0 || value > 3) return fail(ctx, MVAE_EINVAL, "side_mask must be in [0, 3]");
    if (ctx->phase == 4) return fail(ctx, MVAE_ESTATE, "side_mask cannot change mid-backward");
    ctx->side_mask = value;
    return MVAE_OK;
  }
  if (k == "early_adam") {
    // only for callers that do not touch the gradients between mvae_backward and mvae_adam (no
    // all-reduce): the side stream reads them as soon as the backward has written them. Taken by
    // mvae_backward only; the per-part API (mvae_backward_part, the all-reduce path) ignores it
    if (ctx->phase == 4) return fail(ctx, MVAE_ESTATE, "early_adam cannot change mid-backward");
    ctx->early_adam = value != 0;
    return MVAE_OK;
  }
  if (k == "early_chunks") {
    if (value != 1 && value != 2 && value != 4 && value != 8)
      return fail(ctx, MVAE_EINVAL, "early_chunks must be 1, 2, 4 or 8");
    if (ctx->phase == 4) return fail(ctx, MVAE_ESTATE, "early_chunks cannot change mid-backward");
    ctx->early_chunks = value;
    return MVAE_OK;
  }
  if (k == "wgrad0_chunks") {
    if (value != 1 && value != 2 && value != 4 && value != 8)
      return fail(ctx, MVAE_EINVAL, "wgrad0_chunks must be 1, 2, 4 or 8");
    if (ctx->phase == 4) return fail(ctx, MVAE_ESTATE, "wgrad0_chunks cannot change mid-backward");
    ctx->w0_chunks = value;
    return MVAE_OK;
  }
  return fail(ctx, MVAE_EINVAL, "unknown option " + k);
}

// The ranges of grads [g1 (n_all) | g2 (n_enc)] that part `part` finishes: part 0 the decoder
// slice of g1; parts 1 .. R the layer-0 rows of chunk part-1 in g1 and in g2 (the last chunk up
// to the end of the layer-0 block, plus the conv-tower blocks in front of it); part R + 1 the
// rest of the encoder slice in g1 and g2. Together they cover grads exactly once.
extern "C" int mvae_grad_range(mvae_ctx* ctx, int part, int index, float** ptr, size_t* count) {
  if (!ctx || !ptr || !count) return MVAE_EINVAL;
  const int R = w0n(ctx);
  const Block& b0 = ctx->enc[0];
  const size_t l1 = ctx->nenc > 1 ? ctx->enc[1].off : ctx->head.off;  // end of the layer-0 block
  float* g1 = ctx->grads;
  float* g2 = ctx->grads + ctx->n_all;
  std::vector<std::pair<float*, size_t>> r;
  if (part == 0) {
    r.push_back({g1 + ctx->n_enc, ctx->n_all - ctx->n_enc});
  } else if (part >= 1 && part <= R) {
    const int m0 = R == 1 ? 0 : ctx->w0m[ctx->w0_chunks][part - 1];
    const int m1 = R == 1 ? b0.K + 1 : ctx->w0m[ctx->w0_chunks][part];
    const size_t a = b0.off + (size_t)m0 * b0.ld;
    const size_t e = part == R ? l1 : b0.off + (size_t)m1 * b0.ld;
    for (float* g : {g1, g2}) r.push_back({g + a, e - a});
    if (part == R && b0.off > 0)  // conv-tower blocks / leading alignment
      for (float* g : {g1, g2}) r.push_back({g, b0.off});
  } else if (part == R + 1) {
    for (float* g : {g1, g2}) r.push_back({g + l1, ctx->n_enc - l1});
  }
  if (index < 0 || index >= (int)r.size()) return MVAE_EINVAL;
  *ptr = r[index].first;
  *count = r[index].second;
  return MVAE_OK;
}

extern "C" int mvae_adam(mvae_ctx* ctx, void* stream) {
  if (!ctx) return MVAE_EINVAL;
  if (ctx->phase != 3) return fail(ctx, MVAE_ESTATE, "mvae_adam before mvae_backward");
  auto c = ctx;
  const AdamArgs a = adam_args(c);
  hipStream_t st = (hipStream_t)stream;
  if (c->early_fork && c->side) {
    // the blocks after layer 0 on the side stream (already past the dgrad chain), layer 0 and the
    // conv-tower blocks in front of it here; the caller's stream then waits for the side stream
    c->early_fork = false;
    const size_t l1 = c->nenc > 1 ? c->enc[1].off : c->head.off;
    AdamArgs a1 = a, a0 = a;
    a1.i0 = l1;
    a0.i0 = c->adam0_from;  // (the layer-0 chunks before the last: updated in the backward)
    a0.i1 = l1;
    c->adam0_from = 0;
    MV_CHECK(launch_adam(a1, c->side));
    {
      TIMED("adam");
      MV_CHECK(launch_adam(a0, st));
    }
    if (int rc = stream_wait(c, c->side, st)) return rc;
    c->side_pending = false;
  } else {
    TIMED("adam");
    MV_CHECK(launch_adam(a, st));
  }
  for (int o = 0; o < 2; ++o) { c->b1p[o] *= c->cfg.beta1; c->b2p[o] *= c->cfg.beta2; }
  c->t1++; c->t2++;
  ctx->phase = 0;
  return MVAE_OK;
}

extern "C" int mvae_train_step(mvae_ctx* ctx, const float* x, const float* areas, const float* eps,
                               float* losses_out, float* dist_out, void* stream) {
  if (!ctx || !x || !areas) return MVAE_EINVAL;
  int rc;
  if ((rc = mvae_forward(ctx, x, eps, stream))) return rc;
  if ((rc = mvae_metric(ctx, areas, stream))) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (losses_out) MV_CHECK(hipMemcpyAsync(losses_out, ctx->losses, 5 * sizeof(float), hipMemcpyDeviceToDevice, st));
  if (dist_out) MV_CHECK(hipMemcpyAsync(dist_out, ctx->dist, ctx->B * sizeof(float), hipMemcpyDeviceToDevice, st));
  // nothing touches the gradients between the two: Adam of the blocks after layer 0 may run
  // beside the layer-0 weight gradient (option "early_adam"; f32x since profiles/r4/
  // r4ae_early_adam.txt, bf16 since the round-5 kernels: C3 1.837 vs 1.844 ms, r5m / r5n)
  const bool ea = ctx->early_adam;
  ctx->early_adam = ea || ctx->np != 0;
  rc = mvae_backward(ctx, stream);
  ctx->early_adam = ea;
  if (rc) return rc;
  return mvae_adam(ctx, stream);
}

// get_predictions in two phases (a data-parallel host all-reduces MVAE_BUF_COLSQ between them:
// the cosine distance normalises over the GLOBAL batch, 8c/vae.py:449-450)
extern "C" int mvae_predict_encode(mvae_ctx* ctx, const float* x, const float* eps, void* stream) {
  if (!ctx || !x) return MVAE_EINVAL;
  int rc = encode(ctx, x, eps, (hipStream_t)stream, ENC_EVAL);
  if (rc) return rc;
  ctx->phase = 6;
  return MVAE_OK;
}

extern "C" int mvae_predict_finish(mvae_ctx* ctx, float* dist_out, void* stream) {
  if (!ctx || !dist_out) return MVAE_EINVAL;
  if (ctx->phase != 6) return fail(ctx, MVAE_ESTATE, "mvae_predict_finish before mvae_predict_encode");
  hipStream_t st = (hipStream_t)stream;
  auto c = ctx;
  MV_CHECK(launch_metric(c->z, c->ldz, c->rowfwd, c->rowpart, c->nblk, nullptr, c->colsq, c->B, c->L,
                         c->cfg.metric, c->cfg.reciprocal, c->cfg.deform_weight, c->inv_bg,
                         c->rowvals, dist_out, c->draw, st));
  ctx->phase = 0;
  return MVAE_OK;
}

extern "C" int mvae_predict(mvae_ctx* ctx, const float* x, const float* eps, float* dist_out, void* stream) {
  if (!ctx || !x || !dist_out) return MVAE_EINVAL;
  int rc = mvae_predict_encode(ctx, x, eps, stream);
  return rc ? rc : mvae_predict_finish(ctx, dist_out, stream);
}

extern "C" int mvae_transform(mvae_ctx* ctx, const float* x, float* zmean_out, void* stream) {
  if (!ctx || !x || !zmean_out) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int rc = encode(ctx, x, nullptr, st, ENC_MEAN);
  if (rc) return rc;
  MV_CHECK(launch_copy2d(ctx->ms + (size_t)ctx->B * 2 * ctx->L, 2 * ctx->L, zmean_out, ctx->L,
                         ctx->B, ctx->L, st));
  ctx->phase = 0;
  return MVAE_OK;
}

extern "C" int mvae_reconstruct(mvae_ctx* ctx, const float* x, const float* eps, float* y_out, void* stream) {
  if (!ctx || !x || !y_out) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int rc = encode(ctx, x, eps, st, ENC_EVAL);
  if (rc) return rc;
  if ((rc = decode_hidden(ctx, st))) return rc;
  GemmDesc d = ctx->f_out;
  d.epi.y = y_out;
  d.epi.ldy = ctx->D;
  if ((rc = run(ctx, d, st))) return rc;
  ctx->phase = 0;
  return MVAE_OK;
}

extern "C" int mvae_generate(mvae_ctx* ctx, const float* zin, int n, float* y_out, void* stream) {
  if (!ctx || !zin || !y_out || n <= 0 || n > ctx->B) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  auto c = ctx;
  MV_CHECK(launch_copy2d(zin, c->L, c->zgen, c->ldz, n, c->L, st));
  MV_CHECK(launch_split_planes(c->zgen, (size_t)n * c->ldz, planes_of(c, c->zgen), st));
  // the decoder's first GEMM re-pointed at zgen: fp32 rows and (plane modes) zgen's own plane
  // images, whose plane stride is B*ldz (z's is 3*B*ldz)
  GemmDesc d1 = c->f_d1; d1.M = n; d1.A = c->zgen; d1.dynA = nullptr;
  { const Planes zp = planes_of(c, c->zgen); d1.Ap = zp.p; d1.pA = zp.stride; }
  GemmDesc d2 = c->f_d2; d2.M = n;
  GemmDesc d3 = c->f_out;
  d3.M = n; d3.C = y_out; d3.ldc = c->D; d3.epi = GemmEpi(); d3.epi.mode = EPI_SIGMOID;
  int rc;
  if ((rc = run(c, d1, st))) return rc;
  if ((rc = run(c, d2, st))) return rc;
  if ((rc = run(c, d3, st))) return rc;
  ctx->phase = 0;
  return MVAE_OK;
}

}  // extern "C"

extern "C" int mvae_debug_gemm(int M, int N, int K, const float* A, int lda, int at, const float* Bm,
                               int ldb, int bt, float* Cm, int ldc, int epi, int act, const float* aux,
                               int ld_aux, void* stream) {
  if ((epi & 15) == EPI_BCE || epi < 0 || (epi & 15) > EPI_SIGMOID || ((epi >> 4) & 15) > 2)
    return fail(nullptr, MVAE_EINVAL, "bad epilogue");
  hipStream_t st = (hipStream_t)stream;
  GemmDesc d = gd(M, N, K, A, lda, at != 0, Bm, ldb, bt != 0, Cm, ldc, epi & 15);
  d.prec = (epi >> 4) & 15;  // 0 fp32, 1 bf16, 2 fp32-accurate bf16 split
  d.variant = (epi >> 8) & 15;
  if (d.variant == 9) { d.valu = 1; d.prec = GEMM_F32; d.variant = 0; }  // the fp32 VALU kernel
  if ((epi >> 13) & 1) d.tm = 192;  // epi bit 13: the ring kernel's 192-row tiles where eligible
  d.x3 = (epi >> 16) & 3;           // epi bits 16-17: f32x ring plans on the plane-stacked kernels (x3 option)
  d.epi.act = act;
  d.epi.aux = aux;
  d.epi.ld_aux = ld_aux;
  std::vector<void*> tmp;
  hipError_t e = hipSuccess;
  if (d.prec != GEMM_F32) {  // plane images of the operands (the step's producers write these)
    const int np = d.prec == GEMM_BF16 ? 1 : 3;
    const size_t na = (size_t)(at ? K : M) * lda, nb = (size_t)(bt ? N : K) * ldb;
    void *pa = nullptr, *pb = nullptr;
    e = hipMalloc(&pa, np * na * 2);
    if (e == hipSuccess) e = hipMalloc(&pb, np * nb * 2);
    tmp = {pa, pb};
    Planes A_{(unsigned short*)pa, (long long)na, np}, B_{(unsigned short*)pb, (long long)nb, np};
    if (e == hipSuccess) e = launch_split_planes(A, na, A_, st);
    if (e == hipSuccess) e = launch_split_planes(Bm, nb, B_, st);
    d.Ap = A_.p; d.pA = A_.stride; d.nA = np;
    d.Bp = B_.p; d.pB = B_.stride; d.nB = np;
  }
  // epi bit 14 (plane modes, A of 0/1 values): A also as a BitMat, the eight-phase kernel's bits path
  if (e == hipSuccess && ((epi >> 14) & 1) && d.prec != GEMM_F32) {
    void *pbits = nullptr, *pnb = nullptr;
    const int kts = bitmat_kts(K);
    e = hipMalloc(&pbits, bitmat_words(M, K) * 4);
    if (e == hipSuccess) e = hipMalloc(&pnb, 16);
    if (e == hipSuccess) tmp.push_back(pbits), tmp.push_back(pnb);
    if (e == hipSuccess) e = hipMemsetAsync(pnb, 0, 16, st);
    if (e == hipSuccess) e = launch_bits_from_plane(d.Ap, lda, at != 0, M, K, (unsigned*)pbits, kts, (int*)pnb, st);
    d.Abits = (const unsigned*)pbits; d.abits_kts = kts; d.anb = (const int*)pnb;
    d.bits_reg = (epi >> 15) & 1;  // epi bit 15: its words loaded to registers (E8 BITS 2)
  }
  // epi bit 12 (plane modes): the output as bf16 planes only (no fp32 store), as the step's
  // producers write their operand images; C then receives the planes' sum (host side)
  const bool planes_out = ((epi >> 12) & 1) && d.prec != GEMM_F32;
  const int npc = d.prec == GEMM_BF16 ? 1 : 3;
  const size_t nc = (size_t)M * ldc;
  unsigned short* cpl = nullptr;
  if (e == hipSuccess && planes_out) {
    e = hipMalloc(&cpl, npc * nc * 2);
    if (e == hipSuccess) e = hipMemsetAsync(cpl, 0, npc * nc * 2, st);
    d.epi.cp = cpl; d.epi.pc = (long long)nc; d.epi.ncp = npc; d.epi.c32 = 0;
  }
  const size_t ws_n = gemm_workspace_elems(d);
  float* ws = nullptr;
  if (e == hipSuccess && ws_n) e = hipMalloc(&ws, ws_n * sizeof(float));
  if (e == hipSuccess) e = gemm_run(d, ws, ws_n, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess && planes_out) {
    std::vector<unsigned short> h(npc * nc);
    std::vector<float> c(nc);
    e = hipMemcpy(h.data(), cpl, h.size() * 2, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(c.data(), Cm, nc * 4, hipMemcpyDeviceToHost);
    for (int r = 0; e == hipSuccess && r < M; ++r)
      for (int j = 0; j < N; ++j) {
        const size_t o = (size_t)r * ldc + j;
        float v = 0.f;
        for (int t = npc - 1; t >= 0; --t) {
          uint32_t u = (uint32_t)h[t * nc + o] << 16;
          float f;
          std::memcpy(&f, &u, 4);
          v += f;
        }
        c[o] = v;
      }
    if (e == hipSuccess) e = hipMemcpy(Cm, c.data(), nc * 4, hipMemcpyHostToDevice);
  }
  if (cpl) (void)hipFree(cpl);
  if (ws) (void)hipFree(ws);
  for (void* q : tmp) if (q) (void)hipFree(q);
  if (e != hipSuccess) { g_create_err = hipGetErrorString(e); return (int)e; }
  return MVAE_OK;
}

extern "C" int mvae_timing_enable(mvae_ctx* ctx, int on) {
  if (!ctx) return MVAE_EINVAL;
  ctx->timing = on != 0;
  return MVAE_OK;
}

extern "C" int mvae_timing_select(mvae_ctx* ctx, int region) {
  if (!ctx || region < -1 || region >= (int)ctx->region_names.size()) return MVAE_EINVAL;
  ctx->timing_sel = region;
  return MVAE_OK;
}

extern "C" int mvae_timing_marker(mvae_ctx* ctx, int region, int on) {
  if (!ctx || region < 0 || region >= (int)ctx->region_names.size()) return MVAE_EINVAL;
  if ((int)ctx->marker.size() < (int)ctx->region_names.size()) ctx->marker.resize(ctx->region_names.size(), 0);
  ctx->marker[region] = on != 0;
  return MVAE_OK;
}

extern "C" int mvae_timing_regions(mvae_ctx* ctx) {
  return ctx ? (int)ctx->region_names.size() : MVAE_EINVAL;
}

extern "C" const char* mvae_timing_name(mvae_ctx* ctx, int r) {
  if (!ctx || r < 0 || r >= (int)ctx->region_names.size()) return nullptr;
  return ctx->region_names[r].c_str();
}

static int collect(mvae_ctx* ctx) {
  for (auto& pd : ctx->pending) {
    MV_CHECK(hipEventSynchronize(pd.b));
    float ms = 0.f;
    MV_CHECK(hipEventElapsedTime(&ms, pd.a, pd.b));
    ctx->region_ms[pd.region] += ms;
    ctx->region_n[pd.region] += 1;
    ctx->event_pool.push_back(pd.a);
    ctx->event_pool.push_back(pd.b);
  }
  ctx->pending.clear();
  return MVAE_OK;
}

extern "C" int mvae_timing_read(mvae_ctx* ctx, int r, double* total_ms, int64_t* count) {
  if (!ctx || !total_ms || !count || r < 0 || r >= (int)ctx->region_names.size()) return MVAE_EINVAL;
  int rc = collect(ctx);
  if (rc) return rc;
  *total_ms = ctx->region_ms[r];
  *count = ctx->region_n[r];
  return MVAE_OK;
}

extern "C" int mvae_timing_reset(mvae_ctx* ctx) {
  if (!ctx) return MVAE_EINVAL;
  int rc = collect(ctx);
  if (rc) return rc;
  std::fill(ctx->region_ms.begin(), ctx->region_ms.end(), 0.0);
  std::fill(ctx->region_n.begin(), ctx->region_n.end(), 0);
  return MVAE_OK;
}

// Time one GEMM shape of the step's kernel family (diagnostics): operands are allocated
// and filled with uniform [-1,1) values inside, `iters` launches are timed with HIP events
// on `stream` after 3 warm-ups. variant selects a kernel variant (0 = default).
// (diagnostics) the de-interleave of a [B][3D] batch of random 0/1 pixels (density 0.1), iters
// launches on the stream: variant 0-4 the bits forms (launch_deint_bits), 100 the bf16-plane pass
extern "C" int mvae_bench_deint(int B, int D, int variant, int iters, void* stream, float* avg_ms) {
  if (B <= 0 || D <= 0 || B % 64 || D % 8 || iters <= 0 || !avg_ms) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int ldx = (D + 1 + 7) / 8 * 8, ldbits = (D / 8 + 15) & ~15;
  const int kf = bitmat_kts(D + 1), kw = bitmat_kts(3 * B);
  std::vector<void*> m;
  auto al = [&](size_t bytes) -> void* {
    void* q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) return nullptr;
    (void)hipMemsetAsync(q, 0, bytes, st);
    m.push_back(q);
    return q;
  };
  // variant + 1000: four X images in turn (none of the next launch's X left in the 256 MB
  // last-level cache, as in the step, where the rest of the step's traffic evicts it)
  // variant + 2000 / + 4000: before every timed launch (each timed alone by its own events) a
  // heater -- a bf16 8192^3 GEMM (~1 ms of MFMA load, as the step's layer-0 weight gradient
  // precedes the next step's pass) / a 1 GB device memset (dirty lines)
  const int heat = variant >= 4000 ? 2 : (variant >= 2000 ? 1 : 0);
  variant %= 2000;
  const int nx = variant >= 1000 ? 4 : 1;
  variant %= 1000;
  float* xr[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < nx; ++i) xr[i] = (float*)al((size_t)B * 3 * D * 4);
  float* x = xr[0];
  float* xs = (float*)al((size_t)3 * B * ldx * 4);
  unsigned short* xp = (unsigned short*)al((size_t)3 * B * ldx * 2);
  unsigned* xbf = (unsigned*)al(bitmat_words(3 * B, D + 1) * 4);
  unsigned* xbw = (unsigned*)al(bitmat_words(D + 1, 3 * B) * 4);
  unsigned char* xb = (unsigned char*)al((size_t)B * ldbits);
  int* dyn = (int*)al(64);
  hipError_t e = (x && xs && xp && xbf && xbw && xb && dyn) ? hipSuccess : hipErrorOutOfMemory;
  for (int i = 0; i < nx; ++i) {
    if (e == hipSuccess && !xr[i]) e = hipErrorOutOfMemory;
    if (e == hipSuccess) e = launch_normal(xr[i], 1, 1, B * 3 * D, 1, 0, 5 + i, 0, st);
    if (e == hipSuccess) e = launch_binarize(xr[i], (size_t)B * 3 * D, st);  // x > 0: half the pixels 1
  }
  int it = 0;
  const Planes pl{xp, (long long)3 * B * ldx, 1};
  auto one = [&]() -> hipError_t {
    x = xr[it++ % nx];
    if (variant == 100) return launch_deinterleave(x, xs, pl, dyn, dyn + 4, B, D, ldx, 0, 2, st, xb, ldbits);
    return launch_deint_bits(x, B, D, xbf, kf, xbw, kw, xb, ldbits, dyn, dyn + 4, xs, pl, ldx, 2, st, variant);
  };
  hipEvent_t t0 = nullptr, t1 = nullptr;
  if (e == hipSuccess) e = hipEventCreate(&t0);
  if (e == hipSuccess) e = hipEventCreate(&t1);
  for (int i = 0; e == hipSuccess && i < 3; ++i) e = one();
  float ms = 0.f;
  if (heat) {
    const int G = 8192;
    unsigned short* ga = (unsigned short*)al((size_t)G * G * 2);
    unsigned short* gb = (unsigned short*)al((size_t)G * G * 2);
    float* gc = (float*)al((size_t)G * G * 4);
    void* junk = heat == 2 ? al((size_t)1 << 30) : nullptr;
    if (e == hipSuccess && (!ga || !gb || !gc || (heat == 2 && !junk))) e = hipErrorOutOfMemory;
    // random operands (a GEMM on zeros draws less power and holds a higher clock)
    if (e == hipSuccess) e = launch_normal(gc, 1, 1, G * G, 1, 0, 11, 0, st);
    if (e == hipSuccess) e = launch_split_planes(gc, (size_t)G * G, Planes{ga, (long long)G * G, 1}, st);
    if (e == hipSuccess) e = launch_normal(gc, 1, 1, G * G, 1, 0, 12, 0, st);
    if (e == hipSuccess) e = launch_split_planes(gc, (size_t)G * G, Planes{gb, (long long)G * G, 1}, st);
    GemmDesc d = gd(G, G, G, nullptr, G, false, nullptr, G, false, gc, G);
    d.prec = GEMM_BF16; d.Ap = ga; d.pA = (long long)G * G; d.nA = 1; d.Bp = gb; d.pB = (long long)G * G; d.nB = 1;
    for (int i = 0; e == hipSuccess && i < iters; ++i) {
      e = heat == 1 ? gemm_run(d, nullptr, 0, st) : hipMemsetAsync(junk, i & 0xff, (size_t)1 << 30, st);
      if (e == hipSuccess) e = hipEventRecord(t0, st);
      if (e == hipSuccess) e = one();
      if (e == hipSuccess) e = hipEventRecord(t1, st);
      if (e == hipSuccess) e = hipEventSynchronize(t1);
      float m1 = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&m1, t0, t1);
      ms += m1;
    }
  } else {
    if (e == hipSuccess) e = hipEventRecord(t0, st);
    for (int i = 0; e == hipSuccess && i < iters; ++i) e = one();
    if (e == hipSuccess) e = hipEventRecord(t1, st);
    if (e == hipSuccess) e = hipEventSynchronize(t1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
  }
  *avg_ms = ms / iters;
  if (t0) (void)hipEventDestroy(t0);
  if (t1) (void)hipEventDestroy(t1);
  for (void* q : m) (void)hipFree(q);
  if (e != hipSuccess) { g_create_err = hipGetErrorString(e); return (int)e; }
  return MVAE_OK;
}

extern "C" int mvae_bench_gemm(int M, int N, int K, int at, int bt, int batch, int variant, int iters,
                               void* stream, float* avg_ms) {
  if (M <= 0 || N <= 0 || K <= 0 || iters <= 0 || !avg_ms || batch <= 0) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  // operand rows padded to 8 elements (16 B), as the step's buffers are
  // MVAE_BENCH_LDPAD (diagnostics): row strides rounded to this many elements (default 8)
  int pad = 8;
  if (const char* lp = std::getenv("MVAE_BENCH_LDPAD"); lp && std::atoi(lp) >= 8) pad = std::atoi(lp) & ~7;
  auto rnd = [&](int v) { return (v + pad - 1) / pad * pad; };
  const int lda = rnd(at ? M : K), ldb = rnd(bt ? K : N);
  const size_t sa = (size_t)(at ? K : M) * lda, sb = (size_t)(bt ? N : K) * ldb;
  const int ldc = rnd(N);  // output rows padded to 16 B as well (the 16-B epilogue stores)
  const size_t na = sa * batch, nb = sb * batch, nc = (size_t)M * ldc * batch;
  float *A = nullptr, *Bm = nullptr, *Cm = nullptr, *ws = nullptr;
  GemmDesc d = gd(M, N, K, nullptr, lda, at != 0, nullptr, ldb, bt != 0, nullptr, ldc);
  d.batch = batch; d.sA = (long long)sa; d.sB = (long long)sb; d.sC = (long long)M * ldc;
  d.variant = variant & 15;
  d.prec = (variant >> 4) & 15;  // 0 fp32, 1 bf16, 2 fp32-accurate bf16 split
  if (d.variant == 9) { d.valu = 1; d.prec = GEMM_F32; d.variant = 0; }  // the fp32 VALU kernel
  d.diag = (variant >> 12) & 255; // kernel timing diagnostics (results meaningless; 32: A/B switch)
  // MVAE_BENCH_SPLIT (diagnostics): split-K forced (0 / unset: the planner's)
  if (const char* sp = std::getenv("MVAE_BENCH_SPLIT"); sp && std::atoi(sp) > 0) d.split = std::atoi(sp);
  // MVAE_BENCH_TILE_GROUP (diagnostics): the bf16 DMA kernels' tile order (m-tiles per band)
  if (const char* tg = std::getenv("MVAE_BENCH_TILE_GROUP"); tg && std::atoi(tg) >= 0) d.group = std::atoi(tg);
  unsigned short* planes = nullptr;
  const int np = d.prec == GEMM_F32 ? 0 : (d.prec == GEMM_BF16 ? 1 : 3);
  hipError_t e = hipMalloc(&A, na * 4);
  if (e == hipSuccess) e = hipMalloc(&Bm, nb * 4);
  if (e == hipSuccess) e = hipMalloc(&Cm, nc * 4);
  if (e == hipSuccess) e = launch_normal(A, 1, 1, (int)na, 1, 0, 1, 0, st);
  if (e == hipSuccess) e = launch_normal(Bm, 1, 1, (int)nb, 1, 0, 2, 0, st);
  d.A = A; d.B = Bm; d.C = Cm;
  // variant bit 20: A of 0/1 values (the layer-0 pixels; in f32x its residual planes then zero);
  // bit 21: ... and also as a BitMat per batch (the eight-phase kernel's bits path)
  const bool bin = (variant >> 20) & 1, use_bits = bin && ((variant >> 21) & 1);
  unsigned* bits = nullptr;
  int* bnb = nullptr;
  if (e == hipSuccess && bin) e = launch_binarize(A, na, st);
  if (e == hipSuccess && np) {
    e = hipMalloc(&planes, (size_t)np * (na + nb) * 2);
    Planes A_{planes, (long long)na, np}, B_{planes + np * na, (long long)nb, np};
    if (e == hipSuccess) e = launch_split_planes(A, na, A_, st);
    if (e == hipSuccess) e = launch_split_planes(Bm, nb, B_, st);
    d.Ap = A_.p; d.pA = A_.stride; d.nA = np;
    d.Bp = B_.p; d.pB = B_.stride; d.nB = np;
    if (bin && np == 3) {  // the step's pixel operand: residual planes zero, read from a zero flag
      if (e == hipSuccess) e = hipMalloc(&bnb, 16);
      if (e == hipSuccess) e = hipMemsetAsync(bnb, 0, 16, st);
      d.dynA = bnb;
    }
    if (e == hipSuccess && use_bits) {
      const int kts = bitmat_kts(K);
      const size_t bw = bitmat_words(M, K);
      if (!bnb) {
        e = hipMalloc(&bnb, 16);
        if (e == hipSuccess) e = hipMemsetAsync(bnb, 0, 16, st);
      }
      if (e == hipSuccess) e = hipMalloc(&bits, bw * batch * 4);
      for (int b = 0; e == hipSuccess && b < batch; ++b)
        e = launch_bits_from_plane(A_.p + (size_t)b * sa, lda, at != 0, M, K, bits + b * bw, kts, bnb + 2, st);
      d.Abits = bits; d.abits_kts = kts; d.abits_sb = (long long)bw; d.anb = bnb + 2;
    }
  }
  // epilogue (variant >> 8): the step's fused epilogues with their operand reads and the
  // output planes the next GEMM would read
  const int epi = (variant >> 8) & 15;
  float *aux = nullptr, *rowpart = nullptr;
  unsigned short *cpl = nullptr, *xpl = nullptr;
  if (e == hipSuccess && epi != EPI_STORE) {
    if (epi > EPI_SIGMOID) e = hipErrorInvalidValue;
    d.epi.mode = epi;
    d.epi.act = ACT_TANH;
    if (e == hipSuccess) e = hipMalloc(&aux, (size_t)M * ldc * 4);
    if (e == hipSuccess) e = launch_normal(aux, 1, 1, M * ldc, 1, 0, 3, 0, st);
    if (e == hipSuccess && epi == EPI_BCE) e = hipMalloc(&rowpart, (size_t)M * gemm_bce_nblk(N) * 4);
    d.epi.aux = aux; d.epi.ld_aux = ldc;
    d.epi.x = aux; d.epi.ldx = ldc;
    d.epi.rowpart = rowpart;
    d.epi.scale = 1.f / M;
    if (epi == EPI_ACT || epi == EPI_DACT) d.epi.padw = 1;  // as the step's padded rows
    if (e == hipSuccess && np) {
      e = hipMalloc(&cpl, (size_t)np * nc * 2);
      d.epi.cp = cpl; d.epi.pc = (long long)nc; d.epi.ncp = np;
      // MVAE_BENCH_PLANES_ONLY=1: the output as planes only, as the step's producers write it;
      // the BCE head as in the step: binary targets read from their bf16 plane (EPI_BCEB)
      if (const char* po = std::getenv("MVAE_BENCH_PLANES_ONLY"); po && *po == '1') {
        d.epi.c32 = 0;
        if (epi == EPI_BCE && e == hipSuccess) {
          e = launch_binarize(aux, (size_t)M * ldc, st);
          if (e == hipSuccess) e = hipMalloc(&xpl, (size_t)M * ldc * 2 + 16);
          if (e == hipSuccess) e = launch_split_planes(aux, (size_t)M * ldc, Planes{xpl, 0, 1}, st);
          if (e == hipSuccess) e = hipMemsetAsync(reinterpret_cast<char*>(xpl) + (size_t)M * ldc * 2, 0, 16, st);
          d.epi.xp = xpl;
          d.epi.xdyn = reinterpret_cast<const int*>(reinterpret_cast<char*>(xpl) + (size_t)M * ldc * 2);
          d.epi.xnb = d.epi.xdyn + 2;  // (the zeroed 16 B: binarized targets)
        }
      }
    }
  }
  const size_t ws_n = gemm_workspace_elems(d);
  if (e == hipSuccess && ws_n) e = hipMalloc(&ws, ws_n * 4);
  hipEvent_t t0 = nullptr, t1 = nullptr;
  if (e == hipSuccess) e = hipEventCreate(&t0);
  if (e == hipSuccess) e = hipEventCreate(&t1);
  for (int i = 0; e == hipSuccess && i < 3; ++i) e = gemm_run(d, ws, ws_n, st);
  if (e == hipSuccess) e = hipEventRecord(t0, st);
  for (int i = 0; e == hipSuccess && i < iters; ++i) e = gemm_run(d, ws, ws_n, st);
  if (e == hipSuccess) e = hipEventRecord(t1, st);
  if (e == hipSuccess) e = hipEventSynchronize(t1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
  *avg_ms = ms / iters;
  // MVAE_STAMPS=1 (diagnostics): one more launch of the stamped ring-kernel build,
  // per-workgroup segment times (us, 100 MHz stamps) summarised on stderr
  if (const char* sp = std::getenv("MVAE_STAMPS"); e == hipSuccess && sp && *sp == '1') {
    const int nmax = 1 << 20;
    unsigned long long* sb = nullptr;
    e = hipMalloc(&sb, (size_t)8 * nmax * 8);
    if (e == hipSuccess) e = hipMemsetAsync(sb, 0, (size_t)8 * nmax * 8, st);
    GemmDesc ds = d;
    ds.stamps = sb;
    if (e == hipSuccess) e = gemm_run(ds, ws, ws_n, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    std::vector<unsigned long long> h((size_t)8 * nmax);
    if (e == hipSuccess) e = hipMemcpy(h.data(), sb, h.size() * 8, hipMemcpyDeviceToHost);
    if (sb) (void)hipFree(sb);
    int n = 0;
    unsigned long long lo = ~0ull, hi = 0;
    double seg[3] = {0, 0, 0}, iss = 0, wsum = 0, vsum = 0;
    int niss = 0;
    for (int i = 0; i < nmax && e == hipSuccess; ++i) {
      const unsigned long long* q = &h[8 * (size_t)i];
      if (!q[0]) continue;
      ++n;
      lo = std::min(lo, q[0]); hi = std::max(hi, q[3]);
      for (int k = 0; k < 3; ++k) seg[k] += (double)(q[k + 1] - q[k]) * 0.01;
      if (q[4]) { iss += (double)(q[4] - q[2]) * 0.01; ++niss; }
      wsum += (double)q[5] * 0.01;
      vsum += (double)q[6] * 0.01;
    }
    if (niss) std::fprintf(stderr, "[stamps] epilogue stores issued after %.2f us (mean of %d WGs)\n", iss / niss, niss);
    if (n) std::fprintf(stderr, "[stamps] k-loop iteration boundaries (wave 0): vmcnt wait %.2f us, barrier %.2f us per WG\n", vsum / n, wsum / n);
    if (n) {
      std::vector<double> st0s, ends;
      for (int i = 0; i < nmax; ++i) {
        const unsigned long long* q = &h[8 * (size_t)i];
        if (!q[0]) continue;
        st0s.push_back((q[0] - lo) * 0.01);
        ends.push_back((q[3] - lo) * 0.01);
      }
      std::sort(st0s.begin(), st0s.end());
      std::sort(ends.begin(), ends.end());
      std::fprintf(stderr, "[stamps] M %d N %d K %d: %d workgroups, span %.2f us; mean per WG: prologue %.2f, "
                   "k-loop %.2f, epilogue %.2f us; start p50/p90/max %.2f/%.2f/%.2f; end p10/p50/max %.2f/%.2f/%.2f\n",
                   M, N, K, n, (hi - lo) * 0.01, seg[0] / n, seg[1] / n, seg[2] / n,
                   st0s[n / 2], st0s[n * 9 / 10], st0s[n - 1], ends[n / 10], ends[n / 2], ends[n - 1]);
    }
  }
  // MVAE_STAMPS=2 (diagnostics): one more launch of the stamped eight-phase build (EPI_STORE,
  // C/D epilogue): per wave the shader cycles of each of a k-tile's 8 barrier-delimited slots,
  // summed over its k-loop; printed per k-tile for waves 0-3 and 4-7 (the half one barrier
  // behind), with the in-kernel clock (shader cycles / 100 MHz realtime)
  if (const char* sp = std::getenv("MVAE_STAMPS"); e == hipSuccess && sp && *sp == '2') {
    const size_t nmax = 1 << 16;
    unsigned long long* sb = nullptr;
    e = hipMalloc(&sb, nmax * 8 * 16 * 8);
    if (e == hipSuccess) e = hipMemsetAsync(sb, 0, nmax * 8 * 16 * 8, st);
    GemmDesc ds = d;
    ds.stamps = sb;
    if (e == hipSuccess) e = gemm_run(ds, ws, ws_n, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    std::vector<unsigned long long> h(nmax * 8 * 16);
    if (e == hipSuccess) e = hipMemcpy(h.data(), sb, h.size() * 8, hipMemcpyDeviceToHost);
    if (sb) (void)hipFree(sb);
    double slot[2][8] = {}, tot[2] = {}, tiles[2] = {}, cyc = 0, rt = 0, pro = 0, loop_us = 0, epi = 0;
    int nw = 0;
    for (size_t w = 0; w < nmax * 8 && e == hipSuccess; ++w) {
      const unsigned long long* q = &h[16 * w];
      if (!q[10]) continue;
      const int half = (int)(w % 8) / 4;
      for (int k = 0; k < 8; ++k) slot[half][k] += (double)q[k];
      tot[half] += (double)q[8];
      tiles[half] += (double)q[10];
      cyc += (double)q[8];
      rt += (double)q[9];
      pro += (double)q[11] * 0.01;
      loop_us += (double)q[9] * 0.01;
      epi += (double)q[12] * 0.01;
      ++nw;
    }
    if (nw) {
      std::fprintf(stderr, "[e8stamps] M %d N %d K %d: %d waves, clock %.3f GHz, k-loop cycles per k-tile: "
                   "waves0-3 %.0f, waves4-7 %.0f; per workgroup: prologue %.2f us, k-loop %.2f us, epilogue %.2f us\n",
                   M, N, K, nw, cyc / rt * 0.1, tot[0] / tiles[0], tot[1] / tiles[1], pro / nw, loop_us / nw, epi / nw);
      for (int hf = 0; hf < 2; ++hf) {
        std::fprintf(stderr, "[e8stamps]   waves%s slots per k-tile:", hf ? "4-7" : "0-3");
        for (int k = 0; k < 8; ++k) std::fprintf(stderr, " %.0f", slot[hf][k] / tiles[hf]);
        std::fprintf(stderr, "\n");
      }
    }
  }
  if (t0) (void)hipEventDestroy(t0);
  if (t1) (void)hipEventDestroy(t1);
  for (float* p : {A, Bm, Cm, ws, aux, rowpart}) if (p) (void)hipFree(p);
  if (planes) (void)hipFree(planes);
  if (cpl) (void)hipFree(cpl);
  if (xpl) (void)hipFree(xpl);
  if (bits) (void)hipFree(bits);
  if (bnb) (void)hipFree(bnb);
  if (e != hipSuccess) { g_create_err = hipGetErrorString(e); return (int)e; }
  return MVAE_OK;
}

extern "C" int mvae_make_batch(const unsigned char* locks, const unsigned char* keys, int height,
                               int width, const int* idx, const float* coef, int batch,
                               float divisor, float* x_out, void* stream) {
  if (!locks || !keys || !idx || !coef || !x_out || height <= 0 || width <= 0 || batch <= 0 ||
      !(divisor > 0.f))
    return fail(nullptr, MVAE_EINVAL, "mvae_make_batch: bad argument");
  if ((reinterpret_cast<uintptr_t>(coef) & 15) != 0)
    return fail(nullptr, MVAE_EINVAL, "mvae_make_batch: coef must be 16-byte aligned");
  hipError_t e = launch_make_batch(locks, keys, height, width, idx, coef, batch, divisor, x_out,
                                   (hipStream_t)stream);
  if (e != hipSuccess) { g_create_err = hipGetErrorString(e); return (int)e; }
  return MVAE_OK;
}

// One conv2 kernel of the conv tower on caller data (tests only; synchronous): S1 x S1 x 64
// images, B = batch (3B forward images, 4B backward images). mode 0: out = relu(conv(x, W) + b)
// over 3B images (y = W2 block [1601][64]); mode 1: out = data gradient conv(x, W rotated) over
// 4B images (y = W2); mode 2: out[2][1601][64] = the two weight gradients of x = n1 (3B) and
// y = d a2 (4B). mfma: the bf16 MFMA kernels (operands rounded to bf16) instead of fp32 VALU.
extern "C" int mvae_debug_conv2(int S1, int B, int mode, int mfma, const float* x, const float* y,
                                float* out, void* stream) {
  if (S1 <= 0 || S1 > 50 || B <= 0 || mode < 0 || mode > 2 || !x || !y || !out)
    return fail(nullptr, MVAE_EINVAL, "mvae_debug_conv2: bad argument");
  hipStream_t st = (hipStream_t)stream;
  ConvTower T;
  T.S1 = S1; T.S = 2 * S1; T.S2 = S1 / 2;
  // mfma bit 0: the MFMA kernels; the kernel form (the create options' conv2_*): bit 1 the
  // full-channel forward / data-gradient kernel, bits 2 / 3 its 4 / 16 waves, bit 4 two taps per
  // slot, bit 5 four M-fragments per wave, bit 6 the 4-wave weight-gradient kernel
  T.mfma = (mfma & 1) != 0;
  if (mfma & 2) T.conv2_half = false;
  if (mfma & 4) T.conv2_nw = 4;
  if (mfma & 8) T.conv2_nw = 16;
  if (mfma & 16) T.conv2_tpb = 2;
  if (mfma & 32) T.conv2_fpw = 4;
  if (mfma & 64) T.conv2_wg8 = false;
  const size_t img = (size_t)S1 * S1 * 64;
  const int B2 = 2 * B;
  T.nchunk2 = std::min(B2, 32);
  T.nchunk2m = std::min(B2, 64);
  std::vector<void*> tmp;
  hipError_t e = hipSuccess;
  auto alloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (e == hipSuccess) e = hipMalloc(&p, std::max<size_t>(bytes, 4));
    if (e == hipSuccess) tmp.push_back(p);
    return p;
  };
  auto bf16_of = [&](const float* src, size_t n) -> unsigned short* {
    unsigned short* p = static_cast<unsigned short*>(alloc(n * 2));
    if (e == hipSuccess) e = launch_split_planes(src, n, Planes{p, (long long)n, 1}, st);
    return p;
  };
  if (mode == 2) {
    T.n1 = const_cast<float*>(x);
    T.da2 = const_cast<float*>(y);
    const size_t ns = (size_t)2 * (T.mfma ? T.nchunk2m : T.nchunk2) * (25 * 64 + 1) * 64;
    T.slab = static_cast<float*>(alloc(ns * 4));
    if (T.mfma) { T.n1b = bf16_of(x, 3 * B * img); T.da2b = bf16_of(y, 4 * B * img); }
    if (e == hipSuccess) e = launch_conv2_wgrad(T, B, out, out + (size_t)(25 * 64 + 1) * 64, st);
  } else {
    const int nimg = mode == 0 ? 3 * B : 4 * B;
    const unsigned short* xb = nullptr;
    if (T.mfma) {
      xb = bf16_of(x, nimg * img);
      T.w2f = static_cast<unsigned short*>(alloc(25 * 64 * 64 * 2));
      T.w2d = static_cast<unsigned short*>(alloc(25 * 64 * 64 * 2));
      if (e == hipSuccess) e = launch_conv2_wprep(T, y, st);
    }
    if (e == hipSuccess)
      e = launch_conv2(T, mode == 0, x, xb, y, mode == 0 ? T.w2f : T.w2d, out, nimg, st);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  for (void* p : tmp) (void)hipFree(p);
  if (e != hipSuccess) { g_create_err = hipGetErrorString(e); return (int)e; }
  return MVAE_OK;
}
