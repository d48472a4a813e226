/*
 * greedymml.h - C ABI of libgreedymml_hip.so, the MI355X (gfx950) kernels of the
 * balanced multi-modal training step (MVCNN + MMTM fusion + conditional-learning-
 * speed gating) of SebastianHafner/greedy_multimodal_learning.
 *
 * Conventions (every entry point):
 *   - all pointers are caller-owned DEVICE pointers (the library never allocates,
 *     frees or synchronises); descriptor structs themselves live in host memory;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *   - returns 0 on success, a negative GM_E* code on bad arguments, or a positive
 *     hipError_t from the launch; gm_last_error() gives a thread-local message;
 *   - no C++ exceptions cross the ABI; the entry points are reentrant (no mutable
 *     globals besides the thread-local error text, the sticky device fault words and
 *     two process-wide settings - spin limit, BatchNorm concurrency - see below), so
 *     they may be called from the autograd engine's worker thread and captured into
 *     hipGraphs.
 *
 * The reference is pure Python/PyTorch; each entry point below replaces the
 * implicit PyTorch kernels of one reference call site (cited as file:line of the
 * reference repository).
 */
#ifndef GREEDYMML_H
#define GREEDYMML_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_ABI_VERSION 3

/* activation element types */
#define GM_F32  0
#define GM_BF16 1
/* activation layouts: NCHW = [B][C][H*W], NHWC = [B][H*W][C] (channels_last) */
#define GM_NCHW 0
#define GM_NHWC 1
/* error codes */
#define GM_OK          0
#define GM_E_ARG      -1
#define GM_E_SCRATCH  -2
#define GM_E_UNSUP    -3

int gm_abi_version(void);
const char* gm_last_error(void);

/* In-launch hand-off health.  The single-launch BatchNorm kernels and the split-K
 * convolution turnstile hand data between workgroups of one launch through a spin on
 * a device word, bounded by a poll budget.  A spin that runs out (a grid that was not
 * co-resident after all, or a broken hand-off) never hangs and never applies stale
 * data: it sets a bit in a sticky device fault word and poisons its output with NaN.
 * gm_device_faults() synchronises the device and returns the OR of the fault words
 * (clear != 0 resets them).  gm_set_spin_limit() sets the poll budget (0 = default
 * 1<<24; a test hook).  Not graph-capturable (gm_device_faults synchronises). */
#define GM_FAULT_BN_SPIN     1u
#define GM_FAULT_SPLITK_SPIN 2u
int gm_device_faults(unsigned* out, int clear);
int gm_set_spin_limit(unsigned polls);
/* Co-residency of the single-launch BatchNorm: at most `n` such launches are assumed
 * to run at once (one per concurrently running trunk stream, plus headroom for other
 * kernels); the fused grid is capped at CUs x (measured blocks per CU) / n, else the
 * two-launch path runs.  Default 4. */
int gm_bn_set_concurrency(int n);
/* Device residency plan for every kernel whose workgroups wait on other workgroups of
 * the same launch (single-launch BatchNorm, split-K turnstile).  Such a launch is only
 * safe while all the workgroups it waits on can be resident; what else holds CU slots
 * at the same time is declared here:
 *   streams      launches of this process that can wait at once (trunk streams; >= 1)
 *   sharers      processes sharing this GPU (ranks on one device in rehearsals; >= 1)
 *   reserved_cus CUs held by concurrently resident kernels that never yield, e.g. the
 *                RCCL all-reduce kernels that overlap backward under data parallelism
 * The BatchNorm grid is capped at (CUs - reserved) x (blocks per CU) /
 * (max(concurrency, streams) x sharers) and the waiting split-K workgroups of one launch at
 * (CUs - reserved) x 2 / (streams x sharers).  Defaults: 2, 1, 0.
 * The engine sets it per process (engine.BalancedStep).  gm_get_residency reads it. */
int gm_set_residency(int streams, int sharers, int reserved_cus);
int gm_get_residency(int* streams, int* sharers, int* reserved_cus);
/* 0: always the two-launch path; 1: single launch with register-held strips only;
 * 2 (default): also the streaming single-launch variant. */
int gm_bn_set_fused_mode(int mode);

/* ---------------------------------------------------------------------------
 * Spatial reduction per (batch, channel): the MMTM squeeze and its backward.
 *   squeeze  (dy == NULL): out[b*ld_out + c] = scale * sum_hw x[b,c,hw]
 *            replaces `torch.mean(tview, dim=-1)` (src/balanced_mmtm.py:62,67,75,84,96-97)
 *   backward (dy != NULL): g = scale * sum_hw dy[b,c,hw] * x[b,c,hw]
 *            out = e ? g*e*(1-e) : g     (sigmoid derivative fused; e[b*ld_e+c])
 *            replaces autograd of `visual * vis_out` + `self.sigmoid` (:110-111,154)
 * Up to 4 problems (e.g. both modalities) per launch; all share B, dtype, layout.
 * scratch: NHWC uses fp32 partials, at least gm_spatial_reduce_scratch() bytes.
 * ------------------------------------------------------------------------- */
typedef struct gm_spatial_reduce {
    const void* x;
    const void* dy;
    int C, HW;
    float* out;
    int ld_out;
    const float* e;
    int ld_e;
    float scale;
} gm_spatial_reduce;

size_t gm_spatial_reduce_scratch(const gm_spatial_reduce* p, int nprob, int B, int dtype, int layout);
int gm_mmtm_spatial_reduce(const gm_spatial_reduce* p, int nprob, int B, int dtype, int layout,
                           void* scratch, size_t scratch_bytes, void* stream);
/* A/B knob of the NHWC squeeze: threads per workgroup (256 or 1024; negative:
 * nontemporal loads in the bf16 forward) and
 * pixels whose 16-B loads one thread keeps in flight (4, 8 or 16).
 * Process-wide, not thread-safe. */
int gm_mmtm_set_reduce_form(int threads, int unroll);

/* ---------------------------------------------------------------------------
 * Channel re-scale: y[b,c,hw] = x[b,c,hw] * s[b*ld_s + c] (+ alpha * a[b*ld_a + c])
 *   forward  (a == NULL): `visual * vis_out` (src/balanced_mmtm.py:154), ld_s = 0
 *            broadcasts one row (curation: the running average, :141-152);
 *   backward (a = dsq):   dX = dY*e + dsq/HW (autograd of :154 and of the mean :96-97).
 * Up to 4 problems per launch.
 * ------------------------------------------------------------------------- */
typedef struct gm_channel_scale {
    const void* x;
    void* y;
    int C, HW;
    const float* s;
    int ld_s;
    const float* a;
    int ld_a;
    float alpha;
} gm_channel_scale;

int gm_mmtm_channel_scale(const gm_channel_scale* p, int nprob, int B, int dtype, int layout,
                          void* stream);

/* ---------------------------------------------------------------------------
 * Small fp32 GEMM on MFMA (v_mfma_f32_16x16x4_f32, exact f32 fma chains):
 *   C[m,n] (+)= act( sum_seg sum_k A_seg[m,k] * B_seg[k,n] + bias[n] ) * mask
 * Element (i,j) of an operand X is X.ptr[i*ld0 + j*ld1]; ld0 = 0 broadcasts a row.
 * A.ptr == NULL means A == 1 (column sums: bias gradients).
 * act: 0 none, 1 relu, 2 sigmoid.  mask: if non-NULL, multiply by (mask[m,n] > 0)
 * (relu backward).  Up to 2 K-segments (concatenated-input FCs), up to 6 problems
 * per launch.  Replaces the MMTM nn.Linear layers and their autograd
 * (src/balanced_mmtm.py:38,44-45,100,107-108; SE-only / shared / turn-off :60-91).
 * ------------------------------------------------------------------------- */
typedef struct gm_operand {
    const float* ptr;
    int ld0, ld1;
} gm_operand;

typedef struct gm_gemm {
    int M, N;
    int K[2];
    gm_operand A[2];
    gm_operand B[2];
    const float* bias;
    const float* mask;
    int ld_mask;
    float* C;
    int ld_c;
    int act;
    int accumulate;
} gm_gemm;

int gm_gemm_f32(const gm_gemm* p, int nprob, void* stream);
/* A/B knob: fp32 GEMM form, waves per workgroup x k-steps per load round:
 * 0 = 4 x 8, 1 = 4 x 16 (default), 2 = 8 x 16, 3 = 16 x 8; + 256: no float4 k-segments.
 * Process-wide. */
int gm_gemm_set_form(int form);

/* ---------------------------------------------------------------------------
 * MMTM running averages (src/balanced_mmtm.py:113-116), reference quirk kept:
 * BOTH averages are updated with the VISUAL scale's batch mean:
 *   m = mean_b e_v[b,:];  ra_X_new = (m + ra_X_old*step) / (step+1)
 * ------------------------------------------------------------------------- */
int gm_mmtm_running_avg(const float* e_v, int ld_e, int B, int C,
                        const float* ra_v_old, const float* ra_s_old,
                        float* ra_v_new, float* ra_s_new, int step, void* stream);
/* Graph-capturable form: the step counter lives in device memory (read, then
 * advanced by one if `increment`), the averages are updated IN PLACE (ra_s may
 * equal ra_v).  Same arithmetic as gm_mmtm_running_avg. */
int gm_mmtm_running_avg_dev(const float* e_v, int ld_e, int B, int C, float* ra_v, float* ra_s,
                            int* step, int increment, void* stream);

/* ---------------------------------------------------------------------------
 * Per-branch weight / gradient norms for the conditional-learning-speed gate
 * (Bias_Mitigation_Strong.compute_BDR, src/callbacks.py:199-233), optionally fused
 * with the SGD update of the same parameters (torch.optim.SGD momentum=0, wd=0;
 * train.py:48-51, src/framework.py:315):
 *   out[2*g]   = sum over tensors with bit g in group_mask of sum(param^2)
 *   out[2*g+1] = same for sum((grad*grad_scale)^2)
 *   if lr != 0: param -= lr * grad * grad_scale   (after reading param)
 * `table` is a DEVICE array of ntensors gm_tensor entries (built once by the
 * caller); `offset` = prefix sum of n (elements before this tensor).  grad may be
 * NULL (a parameter without gradient: contributes 0 and is not updated).
 * ngroups <= 32 (one bit of group_mask each; the N-branch gate uses 2N groups).
 * out: DEVICE double[2*ngroups]; scratch >= gm_group_sumsq_scratch(total) bytes.
 * Deterministic (fixed reduction order).
 * ------------------------------------------------------------------------- */
typedef struct gm_tensor {
    float* param;
    const float* grad;
    long long n;
    long long offset;
    unsigned int group_mask;
    unsigned int pad;
} gm_tensor;

size_t gm_group_sumsq_scratch(long long total_elems);
/* ---------------------------------------------------------------------------
 * On-device gate (Bias_Mitigation_Strong, reference src/callbacks.py:199-267) and the
 * MMTM curation substitution it drives (src/balanced_mmtm.py:135-152): no host sync
 * per training step.  gm_gate_state lives in device memory (caller-owned, 80 B).
 * ------------------------------------------------------------------------- */
typedef struct gm_gate_state {
    int curation_mode, caring, curation_step, unlock;   /* caring: -1 = None */
    int window, n_curated, pad0, pad1;
    double eps;
    double M[4];                                          /* bypass0, bypass1, main0, main1 */
    double d_bdr;
} gm_gate_state;
/* sums: device fp64 [8] from gm_group_sumsq (main0, main1, bypass0, bypass1: w, g) */
int gm_gate_strong_step(const double* sums, gm_gate_state* state, void* stream);
/* N-branch form (configs C4 / C5: 2 <= nb <= GM_GATE_MAX_BRANCHES).  Same 32-byte prefix as
 * gm_gate_state, so the gated MMTM kernels read either.  The host gate's N-branch rule
 * (callbacks.bdr_decision): BDR_i = log10(M_bypass_i / M_main_i), d_bdr = max - min,
 * caring = argmax (first on ties); at nb = 2 this is the reference's rule
 * (src/callbacks.py:244-252).  sums: device fp64 [4*nb] from gm_group_sumsq over the 2*nb
 * groups main0..main{nb-1}, bypass0..bypass{nb-1} (w, g per group). */
#define GM_GATE_MAX_BRANCHES 16
typedef struct gm_gate_state_n {
    int curation_mode, caring, curation_step, unlock;   /* caring: -1 = None */
    int window, n_curated, nb, pad0;
    double eps;
    double M_bypass[GM_GATE_MAX_BRANCHES];
    double M_main[GM_GATE_MAX_BRANCHES];
    double bdr[GM_GATE_MAX_BRANCHES];
    double d_bdr;
} gm_gate_state_n;
int gm_gate_strong_step_n(const double* sums, gm_gate_state_n* state, void* stream);
/* s_m = running average (broadcast over B) for the cared-for modality when curating,
 * else e_m; mask[2] = {0 or 1} per modality (0: substituted, no excitation gradient) */
int gm_mmtm_select_scale(const float* e_v, int ld_v, const float* e_s, int ld_s, const float* ra_v,
                         const float* ra_s, int B, int Cv, int Cs, const gm_gate_state* state,
                         float* s_v, float* s_s, float* mask, void* stream);
int gm_mmtm_mask_rows(float* a, long long n, const float* mask, void* stream);
/* Both modalities in one launch: a[0..na) *= mask[0], b[0..nb) *= mask[1]. */
int gm_mmtm_mask_rows2(float* a, long long na, float* b, long long nb, const float* mask, void* stream);
/* The gate folded into the MMTM launches themselves (no select / mask launch): problem 0
 * (visual) and 1 (skeleton) are the two modalities; when state says modality i is
 * substituted (curation_mode && caring == i):
 *   channel_scale_gated  - problem i scales by alt_i broadcast over the batch (its running
 *                          average; ld 0) instead of its s rows, as gm_mmtm_select_scale's
 *                          s_i would hold;
 *   spatial_reduce_gated - problem i's outputs are multiplied by 0 (gm_mmtm_mask_rows2's
 *                          factor: the substituted excitation receives no gradient).
 * Both are otherwise gm_mmtm_channel_scale / gm_mmtm_spatial_reduce. */
int gm_mmtm_channel_scale_gated(const gm_channel_scale* p, int nprob, int B, int dtype, int layout,
                                const gm_gate_state* state, const float* alt_s0, const float* alt_s1,
                                void* stream);
int gm_mmtm_spatial_reduce_gated(const gm_spatial_reduce* p, int nprob, int B, int dtype, int layout,
                                 const gm_gate_state* state, void* scratch, size_t scratch_bytes, void* stream);
/* N-modality forms (MMTM_N under the on-device gate): problem i belongs to modality
 * mods[i] (-2: never substituted) and, when that modality is substituted, scales by
 * alts[i] broadcast (channel_scale) / has its outputs multiplied by 0 (spatial_reduce).
 * `state` may point at a gm_gate_state or a gm_gate_state_n (shared prefix). */
int gm_mmtm_channel_scale_gated_n(const gm_channel_scale* p, int nprob, int B, int dtype, int layout,
                                  const gm_gate_state* state, const int* mods, const float* const* alts,
                                  void* stream);
int gm_mmtm_spatial_reduce_gated_n(const gm_spatial_reduce* p, int nprob, int B, int dtype, int layout,
                                   const gm_gate_state* state, const int* mods, void* scratch,
                                   size_t scratch_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Pixel-pair packing of the RGB stem (one launch, input and weight):
 *   xp [N][Hp][Wp/2][8] bf16: xp[n][hp][wq][4j+c] = x[n, c, hp-pad, 2wq+j-pad], 0 outside
 *                       the image or for c >= C0; x fp32/bf16 with element strides sn..sw
 *   wp [K][R][(S+1)/2][8] bf16 (if w): wp[k][r][sq][4j+c] = w[k, c, r, 2sq+j], 0 past S/C0
 * The stem convolution then runs as a C = 8, strides (2, 1) convolution on the pair
 * view (conv.py).  Replaces the reference's plain Conv2d(3, 64, 7, 2, 3) input path.
 * ------------------------------------------------------------------------- */
typedef struct gm_stem_pack {
    const void* x;
    int dtype;                 /* GM_F32 or GM_BF16 */
    int N, C0, H, W, pad;
    long long sn, sc, sh, sw;  /* element strides of x */
    int Hp, Wp;
    void* xp;
    const float* w;            /* optional fp32 [K, C0, R, S] */
    int K, R, S;
    void* wp;
    long long wk, wc, wr, ws;  /* element strides of w (all 0: contiguous [K, C0, R, S]) */
} gm_stem_pack;

int gm_stem_pack_bf16(const gm_stem_pack* p, void* stream);
/* G (<= 4) view groups sharing their geometry (N, H, W, C0, pad, Hp, Wp, K, R, S, dtype) in one
 * launch, ps[g] each with its own pointers and strides; bit-identical to G gm_stem_pack_bf16 calls */
int gm_stem_pack_grouped_bf16(const gm_stem_pack* ps, int G, void* stream);

/* ---------------------------------------------------------------------------
 * Branch-summed cross-entropy (reference train.py:22-29 blend_loss: sum over the
 * branches of nn.CrossEntropyLoss()(logits, y), batch mean) and its gradient.
 * logits: fp32 [nbranch][B][N] contiguous, labels int64 [B]; lse: fp32 [nbranch*B]
 * (written by fwd, read by bwd); loss: fp32 scalar; gout: fp32 scalar (device).
 * dlogits[r,n] = gout * (softmax(x_r)[n] - [n == y]) / B.  Deterministic.
 * ------------------------------------------------------------------------- */
int gm_xent_fwd(const float* logits, int nbranch, int B, int N, const long long* labels, float* lse,
                float* loss, void* stream);
int gm_xent_bwd(const float* logits, const float* lse, int nbranch, int B, int N, const long long* labels,
                const float* gout, float* dlogits, void* stream);

int gm_group_sumsq(const gm_tensor* table, int ntensors, long long total_elems, int ngroups,
                   float grad_scale, float lr, double* out, void* scratch, size_t scratch_bytes,
                   void* stream);
/* gm_group_sumsq + the on-device gate's step (gm_gate_strong_step / _n) in the same finalize
 * launch: gate -> gm_gate_state (gate_n 0, ngroups 4) or gm_gate_state_n (gate_n 1, ngroups 2 nb);
 * identical sums and state to the two calls */
int gm_group_sumsq_gate(const gm_tensor* table, int nt, long long total, int ngroups, float gscale, float lr,
                        double* out, void* scratch, size_t scratch_bytes, void* gate, int gate_n, void* stream);

/* ---------------------------------------------------------------------------
 * ResNet trunk convolutions (torchvision resnet18/50 Conv2d, bias=False; called
 * piecewise at reference src/model.py:65-106) as bf16 implicit GEMMs on MFMA.
 * Activations NHWC [N][H][W][C] bf16, weights KRSC [K][R][S][C] bf16 (PyTorch
 * channels_last weight order), fp32 accumulation.  Output P = (H+2pad-R)/stride+1.
 *   fwd   : y[N][P][Q][K]   = conv(x, w)
 *   dgrad : dx[N][H][W][C]  = conv_transpose(dy[N][P][Q][K], w); `wt` is the
 *           channel-transposed weight [C][R][S][K] (gm_conv_weight_transpose_bf16)
 *   wgrad : dw[K][R][S][C]  = sum over N,P,Q of dy x x-patch, fp32 output;
 *           scratch >= gm_conv2d_wgrad_scratch() bytes (split-K partials)
 * C must be a power of two >= 8 (pad 3-channel images to 8), K a multiple of 8.
 * ------------------------------------------------------------------------- */
typedef struct gm_conv_desc {
    int N, H, W, C;
    int K, R, S;
    int stride, pad;
} gm_conv_desc;

int gm_conv2d_fwd_bf16(const gm_conv_desc* d, const void* x, const void* w, void* y, void* stream);
/* Per-axis stride and padding (same kernels).  The ResNet stem runs through these on a
 * zero-bordered "pixel-pair" view of its RGB input: 4-channel pixels, two per 8-channel
 * element, so the 7x7/s2 filter becomes a 7x4 (pair) filter with strides (2, 1), K = 224
 * instead of 49 taps x 8 padded channels = 392 (conv.py, stem path). */
typedef struct gm_conv_desc_hw {
    int N, H, W, C;
    int K, R, S;
    int stride_h, stride_w, pad_h, pad_w;
} gm_conv_desc_hw;
int gm_conv2d_fwd_hw_bf16(const gm_conv_desc_hw* d, const void* x, const void* w, void* y, void* stream);
int gm_conv2d_dgrad_bf16(const gm_conv_desc* d, const void* dy, const void* wt, void* dx, void* stream);
/* Same convolutions with a caller-owned split-K workspace: when 128x128 tiles alone
 * would not fill the chip (small M, long K: ResNet layers 3/4) each tile's K range is
 * split over 2-4 workgroups that hand their fp32 accumulators on in a fixed order
 * (deterministic).  ws >= gm_conv2d_splitk_ws_bytes(d, dgrad) bytes (0 = no split for
 * this shape; ws may then be NULL), ZEROED ONCE before first use (the kernel leaves
 * its turnstile words at zero); calls sharing one ws must be stream-ordered. */
size_t gm_conv2d_splitk_ws_bytes(const gm_conv_desc* d, int dgrad);
/* Main-loop form of the implicit-GEMM kernel (process-wide): -1 (default) = 2;
 * 0 = two LDS stages drained at every barrier; 2 / 3 = a 2- / 3-stage LDS ring with one
 * barrier per k-tile and counted DMA waits (3: the next tile's DMA stays in flight). */
int gm_conv_set_pipe(int pipe);
/* 3x3 / stride-1 / pad-1 convolutions (forward and input gradient, C % 64 == 0) stage
 * the input once per 64-channel chunk as a halo instead of once per tap (default on;
 * gm_conv_set_halo(0) selects the im2col kernel for them). */
int gm_conv_set_halo(int on);
/* The halo kernel with its nine taps unrolled (k_conv_h9; default on,
 * gm_conv_set_h9(0) selects the run-time-decoded k_conv_halo, an A/B switch). */
int gm_conv_set_h9(int on);
/* Split-K target: workgroups wanted from splitting K of 128x128-tile convolutions whose
 * tiles alone do not fill the device (default 384; 0 = never). */
int gm_conv_set_splitk(int target);
/* Weight-gradient kernel choice (default 22): bit 1 = k_wgrad_halo64 (64 x 9 x 64
 * gradient blocks in one workgroup's accumulators, one input row staged per output row, dedicated
 * loader waves) for 3x3 / s1 shapes with 64 channels, bit 2 = also for 128 channels, bit 3 = up to
 * 512; bit 4 = k_wgrad_ring for the other 3x3 shapes with K % 128 == 0 and C a power of two >= 32
 * (loader waves feeding an LDS ring, one workgroup per CU); the rest take k_conv_wgrad4.  Bit 0 is
 * reserved (must be 0). */
int gm_conv_set_wgrad_loop(int mode);
/* 1x1 / stride-1 / pad-0 forward and input-gradient convolutions as plain NT GEMMs on
 * k_gemm_ring (conv1x1.hip: persistent, loader waves feeding a 4-slot LDS ring; C % 64 == 0 and
 * the output channels % 128 == 0 or == 64).  Mode 2 (default) also runs the grouped 1x1 / stride-2 /
 * pad-0 forwards (the ResNet downsamples) there, the A rows gathered at stride 2; 1 = stride-1 shapes
 * only; 0 = every 1x1 back on the im2col kernels. */
int gm_conv_set_1x1_gemm(int on);
/* Weight-gradient operand staging: 0 = LDS-DMA pieces, 1 = register-staged (global_load_dwordx4
 * two steps ahead + ds_write_b128; same LDS image and arithmetic), 2 (default) = register-staged
 * for 1x1 filters, LDS-DMA otherwise. */
int gm_conv_set_wgrad_staging(int wr);
/* Resident-weight kernel for 3x3 / stride-1 convolutions with 64 -> 64 channels (ResNet
 * layer 1, forward and input gradient; default on,
 * gm_conv_set_rw(0) selects the im2col kernel for them). */
int gm_conv_set_rw(int on);
/* Dedicated kernel for the pixel-pair stem's forward (8-channel elements -> 64 channels,
 * 7 x 4 filter, strides (2, 1), no padding: weights in VGPRs, two output rows per
 * iteration; default on, gm_conv_set_stem(0) selects the im2col
 * kernel). */
int gm_conv_set_stem(int on);
/* Dedicated kernel for the pixel-pair stem's weight gradient (k_wgrad_stem: one wave per
 * tap row, fp32 partials per workgroup + the split sum; default on,
 * gm_conv_set_wgrad_stem(0) selects k_conv_wgrad4). */
int gm_conv_set_wgrad_stem(int on);
int gm_conv2d_fwd_ex_bf16(const gm_conv_desc* d, const void* x, const void* w, void* y, void* ws,
                          size_t ws_bytes, void* stream);
int gm_conv2d_dgrad_ex_bf16(const gm_conv_desc* d, const void* dy, const void* wt, void* dx, void* ws,
                            size_t ws_bytes, void* stream);
/* dgrad fused with a gradient join: dx = conv_transpose(dy, w) + addend (bf16, dx's
 * layout; may BE dx: summed in place, pixels no parity class covers keep it) - the
 * other consumer's gradient of the same tensor, so
 * the autograd add of the two is never materialised (ResNet blocks: the identity /
 * downsample branch and the first convolution both consume the block input). */
int gm_conv2d_dgrad_add_bf16(const gm_conv_desc* d, const void* dy, const void* wt, void* dx,
                             const void* addend, void* ws, size_t ws_bytes, void* stream);
int gm_conv_weight_transpose_bf16(const void* w, void* wt, int K, int RS, int C, void* stream);
/* fp32 KRSC master weight -> bf16 [K][RS][Cp] (zero-padded channels) and, if wt != NULL,
 * the transposed bf16 [Cp][RS][K] for dgrad, in one pass */
int gm_conv_weight_prep_bf16(const float* w, int K, int RS, int C, int Cp, void* wb, void* wt, void* stream);
/* Multi-tensor form: every weight of `table` (a DEVICE array of n entries, built once
 * by the caller, tile_start = prefix sum of gm_wprep_tiles()) prepared in one launch
 * of total_tiles workgroups.  Same outputs as gm_conv_weight_prep_bf16 per entry. */
typedef struct gm_wprep {
    const float* w;   /* fp32 [K][RS][C] */
    void* wb;         /* bf16 [K][RS][Cp] */
    void* wt;         /* bf16 [Cp][RS][K], or NULL */
    int K, RS, C, Cp;
    int tile_start;
    int pad;
} gm_wprep;
int gm_wprep_tiles(int K, int RS, int Cp);
int gm_conv_weight_prep_multi_bf16(const gm_wprep* table, int n, int total_tiles, void* stream);
/* dw is fp32 [K][R][S][c_real]: the first c_real of the C (padded) input channels;
 * accumulate != 0 adds into dw (a parameter's gradient buffer written in place) */
size_t gm_conv2d_wgrad_scratch(const gm_conv_desc* d);
int gm_conv2d_wgrad_bf16(const gm_conv_desc* d, const void* dy, const void* x, float* dw, int c_real,
                         int accumulate, void* scratch, size_t scratch_bytes, void* stream);
size_t gm_conv2d_wgrad_hw_scratch(const gm_conv_desc_hw* d);
int gm_conv2d_wgrad_hw_bf16(const gm_conv_desc_hw* d, const void* dy, const void* x, float* dw, int c_real,
                            int accumulate, void* scratch, size_t scratch_bytes, void* stream);
/* View groups: G views of the multi-view trunk stacked along the batch (activations
 * [G*N][H][W][C], d->N = images per view), each with its own weight, in ONE launch per
 * pass (the views' tiles fill the chip together instead of one stream each).  Group g
 * reads x + g*N*H*W*C and the weight w + g*w_stride (bf16 elements, >= one weight),
 * writes y + g*N*P*Q*K; dgrad's addend/dx and wgrad's dy/x follow the same stacking,
 * wgrad writes dw + g*dw_stride (fp32 elements).  G = 1 is the ungrouped call.  The
 * workspaces are sized for the whole grouped launch. */
int gm_conv2d_fwd_grouped_bf16(const gm_conv_desc_hw* d, int G, const void* x, const void* w, long long w_stride,
                               void* y, void* ws, size_t ws_bytes, void* stream);
int gm_conv2d_dgrad_grouped_bf16(const gm_conv_desc* d, int G, const void* dy, const void* wt, long long wt_stride,
                                 void* dx, const void* addend, void* ws, size_t ws_bytes, void* stream);
/* The same with a MASKED addend: dx = dgrad + (addend where addend_mask's bit is set) - the
 * identity branch's gradient dz = dy . [y > 0] of a block-output ReLU (reference resnet.py
 * BasicBlock/Bottleneck `out += identity; out = relu(out)`) formed in the epilogue from that
 * ReLU's dy and the BatchNorm forward's 1-bit mask (gm_bn_fwd: relu_mask; bit e of byte i =
 * element 8 i + e, group g's at addend_mask + g*N*H*W*C/8) instead of a dres tensor the BN
 * backward would write and this launch read.  addend != dx; C a multiple of 8. */
int gm_conv2d_dgrad_grouped_masked_bf16(const gm_conv_desc* d, int G, const void* dy, const void* wt,
                                        long long wt_stride, void* dx, const void* addend, const void* addend_mask,
                                        void* ws, size_t ws_bytes, void* stream);
size_t gm_conv2d_splitk_ws_bytes_grouped(const gm_conv_desc* d, int G, int dgrad);
size_t gm_conv2d_wgrad_grouped_scratch(const gm_conv_desc_hw* d, int G);
int gm_conv2d_wgrad_grouped_bf16(const gm_conv_desc_hw* d, int G, const void* dy, const void* x, float* dw,
                                 long long dw_stride, int c_real, int accumulate, void* scratch,
                                 size_t scratch_bytes, void* stream);
/* The pixel-pair stem's weight gradient (the shape gm_conv2d_wgrad_grouped_bf16 serves with
 * k_wgrad_stem: 7 x 4 filter over 8-channel pairs, strides (2, 1), K 64, Q <= 112) with dy NOT
 * materialised: the loader forms dy = the stem BatchNorm + ReLU + max-pool backward (reference
 * src/model.py:65-106 through torchvision's conv1 -> bn1 -> relu -> maxpool) per element,
 *   d  = sum over the pool windows whose argmax is the element of dy_pool (fp32, window order),
 *        rounded to bf16, zero where y * fsc + fsh <= 0;
 *   dy = bf16(ca * d + (cb * y + cc)),
 * bit-identical to gm_bn_relu_maxpool2d_bwd_grouped_bf16's dx followed by
 * gm_conv2d_wgrad_grouped_bf16.  y: the stem output [G][N][P][Q][64] bf16 (the BatchNorm's x);
 * dy_pool / idx: the pool's gradient and argmax bytes [G][N][(P+1)/2][(Q+1)/2][64];
 * fcoef: the forward's sc[64], sh[64] of group g at fcoef + g * fcoef_gs; bcoef: ca, cb, cc
 * [3][64] of group g at bcoef + g * bcoef_gs (gm_bn_relu_maxpool2d_bwd_stats_grouped_bf16).
 * Scratch: gm_conv2d_wgrad_grouped_scratch(d, G).  GM_E_UNSUP (nothing launched) for other shapes. */
typedef struct gm_stem_bn_src {
    const void* y;
    const void* dy_pool;
    const void* idx;
    const float* fcoef;
    long long fcoef_gs;
    const float* bcoef;
    long long bcoef_gs;
} gm_stem_bn_src;
/* the pixel-pair stem's weight gradient dwp [G][K][R][Sp][2][4] fp32 (as the wgrad calls above write
 * it for the stem) into each view's [K][R][S][C0] gradient dst[g] (the channels_last [K, C0, R, S]
 * parameter's memory), += when accumulate; one launch for every view (G <= 16) */
int gm_stem_dw_crop(const float* dwp, int G, int K, int R, int S, int C0, int Sp, float* const* dst, int accumulate,
                    void* stream);
int gm_conv2d_wgrad_stem_bn_ok(const gm_conv_desc_hw* d, int G); /* 1: the call below takes this shape */
int gm_conv2d_wgrad_stem_bn_grouped_bf16(const gm_conv_desc_hw* d, int G, const gm_stem_bn_src* src, const void* x,
                                         float* dw, long long dw_stride, int accumulate, void* scratch,
                                         size_t scratch_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Reference-precision (fp32) trunk convolutions: the same three passes on the exact
 * f32 MFMA (v_mfma_f32_32x32x2_f32, one rounding per product, fp32 accumulate), the
 * reference's own arithmetic type (src/model.py:65-106 through torchvision, fp32
 * tensors, no autocast: src/framework.py:146-148).  NHWC activations, KRSC weights,
 * any C >= 1 (the RGB stem runs unpadded), K any (16-byte loads when C % 4 == 0 and
 * K % 4 == 0):
 *   GM_CONV_FWD   : out = y [N][P][Q][K]            from x, w
 *   GM_CONV_DGRAD : out = dx[N][H][W][C] (+ addend) from dy, w
 *   GM_CONV_WGRAD : out = dw[K][R][S][C]            from dy, x
 * accumulate != 0 adds into out.  scratch >= gm_conv2d_f32_scratch() bytes (split
 * reductions: fp32 slabs summed in a fixed order; 0 = none needed).  Deterministic.
 * ------------------------------------------------------------------------- */
#define GM_CONV_FWD   0
#define GM_CONV_DGRAD 1
#define GM_CONV_WGRAD 2
typedef struct gm_conv_f32 {
    int mode;
    gm_conv_desc d;
    const float* x;
    const float* w;
    const float* dy;
    float* out;
    const float* addend;
    int accumulate;
    int pad0;
} gm_conv_f32;

size_t gm_conv2d_f32_scratch(const gm_conv_f32* p);
int gm_conv2d_f32(const gm_conv_f32* p, void* scratch, size_t scratch_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * BatchNorm2d (torchvision ResNet trunk, reference src/model.py:65-106 through
 * torchvision.models.resnet18), NHWC bf16 activations x[M][C] (M = N*H*W), fp32
 * affine parameters and statistics, fused with the residual add and ReLU that
 * follow it in the blocks:
 *   y = relu?( (x - mean) * invstd * gamma + beta  (+ residual) )
 * train : batch statistics (biased variance for the normalisation; running_var
 *         gets the unbiased one, momentum update - F.batch_norm semantics);
 *         save_mean/save_invstd are written for the backward;
 * infer : running statistics (module.eval()).
 * backward: dz = dy * (y > 0) if relu else dy;  dres = dz (if non-NULL);
 *         dx = BN backward(dz); dgamma/dbeta written (or added if accumulate).
 * C must be a power of two in [8, 2048].  scratch >= gm_bn_scratch(M, C) bytes,
 * ZEROED ONCE before first use; each call leaves its ticket words at zero again.
 * Calls sharing one scratch buffer must be stream-ordered.
 * ------------------------------------------------------------------------- */
typedef struct gm_bn_fwd {
    long long M;
    int C, relu;
    const void* x;
    const void* residual;
    void* y;
    const float* gamma;
    const float* beta;
    float* running_mean;
    float* running_var;
    float momentum, eps;
    float* save_mean;
    float* save_invstd;
    long long* num_batches_tracked;  /* train: += 1 if non-NULL (nn.BatchNorm2d counter) */
    float* coef_out;                 /* train, optional: the affine coefficients sc[C], sh[C] (fp32) */
    void* relu_mask;                 /* train, relu with residual, optional (bf16): the ReLU mask, one byte
                                        per 8 channels of a pixel (bit j: channel 8v + j of y's 16-B
                                        vector v is > 0), M*C/8 bytes - for gm_bn_bwd.relu_mask */
} gm_bn_fwd;

typedef struct gm_bn_bwd {
    long long M;
    int C, relu;
    const void* dy;
    const void* y;
    const void* x;
    const float* gamma;
    const float* save_mean;
    const float* save_invstd;
    void* dx;
    void* dres;
    float* dgamma;
    float* dbeta;
    int accumulate;
    int pad;
    const float* fwd_coef;  /* relu without residual: the forward's coef_out; y may then be NULL and
                               the relu mask is recomputed from x (x*sc + sh > 0, the forward's value) */
    const void* relu_mask;  /* relu (bf16), optional: the forward's relu_mask, read in place of y by the
                               single-launch backward (1/16 of y's bytes; y is still required for the
                               two-launch fallback) */
} gm_bn_bwd;

size_t gm_bn_scratch(long long M, int C);
int gm_bn_fwd_train_bf16(const gm_bn_fwd* p, void* scratch, size_t scratch_bytes, void* stream);
int gm_bn_fwd_infer_bf16(const gm_bn_fwd* p, void* scratch, size_t scratch_bytes, void* stream);
int gm_bn_bwd_bf16(const gm_bn_bwd* p, void* scratch, size_t scratch_bytes, void* stream);
/* the statistics half of gm_bn_fwd_train_bf16 alone (y is not written; coef_out required):
 * the stem's BN + ReLU is applied inside its max-pool (gm_bn_relu_maxpool2d_fwd_bf16) */
int gm_bn_fwd_stats_bf16(const gm_bn_fwd* p, void* scratch, size_t scratch_bytes, void* stream);
/* View groups: G (<= 4) descriptors that agree on M, C and every option, differing only
 * in their pointers (the views of the multi-view trunk, each with its own parameters
 * and statistics), normalised in ONE launch.  scratch >= gm_bn_scratch_grouped(M, C, G)
 * (each group its own ticket / partial area), zeroed once like gm_bn_scratch's.  The
 * grouped forms of gm_bn_fwd_train_bf16 / gm_bn_bwd_bf16 / gm_bn_fwd_stats_bf16. */
size_t gm_bn_scratch_grouped(long long M, int C, int G);
int gm_bn_fwd_train_grouped_bf16(const gm_bn_fwd* ps, int G, void* scratch, size_t scratch_bytes, void* stream);
int gm_bn_bwd_grouped_bf16(const gm_bn_bwd* ps, int G, void* scratch, size_t scratch_bytes, void* stream);
int gm_bn_fwd_stats_grouped_bf16(const gm_bn_fwd* ps, int G, void* scratch, size_t scratch_bytes, void* stream);
/* the same three on fp32 activations (x, residual, y, dy, dx, dres fp32 NHWC): the
 * reference-precision trunk; reduce + apply launches, same statistics arithmetic */
int gm_bn_fwd_train_f32(const gm_bn_fwd* p, void* scratch, size_t scratch_bytes, void* stream);
int gm_bn_fwd_infer_f32(const gm_bn_fwd* p, void* scratch, size_t scratch_bytes, void* stream);
int gm_bn_bwd_f32(const gm_bn_bwd* p, void* scratch, size_t scratch_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * MaxPool2d of the ResNet stem (kernel k, stride, padding; dilation 1, floor
 * mode), NHWC bf16, C a multiple of 8.  Forward writes y[N][P][Q][C] and idx,
 * one byte per output element = window-relative argmax (r*k + c), PyTorch's
 * tie/NaN rule; backward scatters dy to the argmax positions as a gather (dx
 * fully written, zero elsewhere).  Replaces `net.maxpool` (src/model.py:65-106).
 * ------------------------------------------------------------------------- */
typedef struct gm_pool_desc {
    int N, H, W, C;
    int k, stride, pad;
} gm_pool_desc;

int gm_maxpool2d_fwd_bf16(const gm_pool_desc* d, const void* x, void* y, void* idx, void* stream);
int gm_maxpool2d_bwd_bf16(const gm_pool_desc* d, const void* dy, const void* idx, void* dx, void* stream);
/* The stem's BatchNorm + ReLU + max-pool backward (torchvision stem: maxpool(relu(bn1(x))),
 * reference src/model.py:65-106) in two launches without materialising the pool's input
 * gradient: every thread owns a 2 x 2 pixel block and gathers its pool gradient from the
 * <= 2 x 2 windows that can select it (k_maxpool_bwd's arithmetic: fp32 sums in window
 * order, rounded to bf16), masks it with the forward's ReLU (x*sc + sh > 0); pass 1 reduces
 * and finalizes the BN backward (dgamma, dbeta, dx coefficients), pass 2 writes dx.
 * d: ONE view group's pool (N images; k 3, stride 2, pad 1, C 64); dy_pool / idx: the G
 * groups' pooled gradient and argmax stacked ([G*N][P][Q][C], gm_bn_relu_maxpool2d_fwd_*);
 * ps[g]: group g's BN backward with relu, fwd_coef, y = dres = NULL (dy unused); scratch:
 * gm_bn_scratch_grouped(N*H*W, C, G) bytes of the grouped layout.  xsel (optional): the
 * forward's selected raw x (gm_bn_relu_maxpool2d_fwd_grouped_bf16); with it pass 1 reduces
 * over the pooled tensors alone (pool gradient + xsel, a quarter of the pixels, no x read:
 * sum over windows of dy_pool * mask and of dy_pool * mask * (xsel - mean), linear in the
 * per-pixel sums; the per-pixel bf16 rounding of the gathered gradient is skipped there). */
/* The stem's BatchNorm statistics without a pass over its output: the stem convolution
 * (gm_conv2d_fwd_grouped_stats_bf16, k_conv_stem's shapes, 64 output channels) adds every
 * workgroup's (sum, sum of squares) of its stored bf16 outputs into a partial row, and
 * gm_bn_fwd_stats_finalize_grouped combines them in fp64 and finalizes like
 * gm_bn_fwd_stats_grouped_bf16 (save_mean / save_invstd, running statistics, counter,
 * coef_out).  stats: float [G][rows + 1][128], rows = gm_conv_stem_stats_rows(d, G)
 * (0: the stem kernel does not apply). */
int gm_conv_stem_stats_rows(const gm_conv_desc_hw* d, int G);
int gm_conv2d_fwd_grouped_stats_bf16(const gm_conv_desc_hw* d, int G, const void* x, const void* w,
                                     long long w_stride, void* y, float* stats, int rows, void* stream);
int gm_bn_fwd_stats_finalize_grouped(const gm_bn_fwd* ps, int G, float* stats, int rows, void* stream);
/* The same for the view-grouped trunk convolutions (replaces the statistics read of the
 * single-launch BatchNorm forward, gm_bn_fwd_train_grouped_bf16): every kernel that stages its
 * output tile - k_conv_rw (layer 1: one partial row per persistent workgroup), k_conv_h9 and
 * k_conv_igemm_ut through their LDS-staged epilogue (one row per output tile, split-K
 * included) and the 1x1 / s1 GEMM k_gemm_ring (one per wave's 64-pixel slab) - sums its
 * stored bf16 outputs per channel (fp32), writing per group [K / 64 slices][rows][64 x (sum,
 * sum of squares)] then 2K floats of coefficient area (group g at stats + g * 2K (rows + 1)).
 * stats holds stats_floats >= gm_conv2d_fwd_bn_stats_floats(d, G) floats; *rows_out receives
 * the rows of the kernel picked.  GM_E_UNSUP (nothing launched) for G < 2, K % 64 != 0, 64-bit
 * output offsets or a kernel without the staged epilogue (k_conv_halo / k_conv_igemm).
 * Then gm_bn_fwd_stats_finalize_grouped(ps, G, stats, rows) (C = K, any multiple of 64, residual
 * allowed) and gm_bn_fwd_apply_grouped_bf16: y = relu?(x*sc + sh (+ residual)) from the
 * coefficients it left in stats, one launch for evenly strided groups.  Replaces
 * /root/reference/src/model.py:65-76's conv -> BatchNorm2d (torchvision resnet, train mode). */
size_t gm_conv2d_fwd_bn_stats_floats(const gm_conv_desc_hw* d, int G);
int gm_conv2d_fwd_grouped_bn_stats_bf16(const gm_conv_desc_hw* d, int G, const void* x, const void* w,
                                        long long w_stride, void* y, float* stats, size_t stats_floats,
                                        int* rows_out, void* ws, size_t ws_bytes, void* stream);
int gm_bn_fwd_apply_grouped_bf16(const gm_bn_fwd* ps, int G, const float* stats, int rows, void* stream);
/* The BatchNorm backward's statistics from the input-gradient convolution that produces its
 * dy (replaces the statistics pass of gm_bn_bwd_grouped_bf16 for the ReLU-after-BN of the
 * torchvision blocks, conv1 -> bn1 -> relu -> conv2: /root/reference/src/model.py:65-76 via
 * resnet.py).  gm_conv2d_dgrad_grouped_bn_stats_bf16 computes dx = dgrad(dy) like
 * gm_conv2d_dgrad_grouped_bf16 (no addend) and, in the same epilogue, per channel of dx the
 * sums of dz and dz * (x - mean) with dz = dx where x * sc + sh > 0: bn_x is the BatchNorm's
 * input (dx's layout, groups at the same stride), bn_coef its forward coef_out ([G][2C]),
 * bn_mean its save_mean ([G][C]).  stats: stats_floats >= gm_conv2d_dgrad_bn_stats_floats(d, G)
 * floats, *rows_out the partial rows per 64-channel slice.  GM_E_UNSUP (nothing launched) for
 * stride != 1, G < 2, C % 64 != 0, 1x1 shapes or 64-bit offsets.  Then
 * gm_bn_bwd_stats_finalize_grouped (dgamma / dbeta, accumulate honoured, coefficients into
 * stats) and gm_bn_bwd_apply_grouped_bf16 (dx_bn = ca dz + cb x + cc, one launch for evenly
 * strided groups); ps[g] as for gm_bn_bwd_grouped_bf16 with relu + fwd_coef (or no relu), no dres. */
size_t gm_conv2d_dgrad_bn_stats_floats(const gm_conv_desc* d, int G);
int gm_conv2d_dgrad_grouped_bn_stats_bf16(const gm_conv_desc* d, int G, const void* dy, const void* wt,
                                          long long wt_stride, void* dx, const void* bn_x, const float* bn_coef,
                                          const float* bn_mean, float* stats, size_t stats_floats, int* rows_out,
                                          void* ws, size_t ws_bytes, void* stream);
size_t gm_bn_bwd_stats_coef_offset(int C, int G, int rows);
int gm_bn_bwd_stats_finalize_grouped(const gm_bn_bwd* ps, int G, float* stats, int rows, void* stream);
int gm_bn_bwd_apply_grouped_bf16(const gm_bn_bwd* ps, int G, const float* stats, int rows, void* stream);
int gm_bn_relu_maxpool2d_bwd_grouped_bf16(const gm_pool_desc* d, int G, const void* dy_pool, const void* idx,
                                          const void* xsel, const gm_bn_bwd* ps, void* scratch, size_t scratch_bytes,
                                          void* stream);
/* its statistics pass only (dgamma / dbeta; ps[g].dx may be null): *bcoef receives group 0's
 * backward coefficients ca, cb, cc ([3][C] floats, inside scratch), *bcoef_gs the floats between
 * groups - the input of gm_conv2d_wgrad_stem_bn_grouped_bf16, which forms dx in its loader */
int gm_bn_relu_maxpool2d_bwd_stats_grouped_bf16(const gm_pool_desc* d, int G, const void* dy_pool, const void* idx,
                                                const void* xsel, const gm_bn_bwd* ps, void* scratch,
                                                size_t scratch_bytes, const float** bcoef, long long* bcoef_gs,
                                                void* stream);
/* the stem's BatchNorm + ReLU + MaxPool forward: pools relu(x*sc + sh) rounded to bf16
 * (coef = sc[C], sh[C] from gm_bn_fwd_stats_bf16), bit-identical to gm_bn_fwd_train's
 * apply followed by gm_maxpool2d_fwd_bf16, without writing the normalised activation */
int gm_bn_relu_maxpool2d_fwd_bf16(const gm_pool_desc* d, const void* x, const float* coef, void* y, void* idx,
                                  void* stream);
/* G view groups of d->N images each stacked along the batch (x [G*N][H][W][C]); group g
 * applies coef + g*2C (gm_bn_fwd_stats_grouped_bf16's coef_out of group g); xsel (optional,
 * y-shaped) receives the raw x each output selected */
int gm_bn_relu_maxpool2d_fwd_grouped_bf16(const gm_pool_desc* d, int G, const void* x, const float* coef, void* y,
                                          void* idx, void* xsel, void* stream);
/* fp32 activations (the reference-precision trunk), same index format */
int gm_maxpool2d_fwd_f32(const gm_pool_desc* d, const void* x, void* y, void* idx, void* stream);
int gm_maxpool2d_bwd_f32(const gm_pool_desc* d, const void* dy, const void* idx, void* dx, void* stream);

/* ---------------------------------------------------------------------------
 * Input pipeline (reference src/dataset.py:35-47,95-128): the multi-view batch of
 * uint8 view stacks x[B][V][H][W][C=3] (each sample's `imgs[specific_view]`) becomes
 * the network input in one launch:
 *   value = (u / 255 - mean[c]) / std[c]   (ToTensor then Normalize, fp32, each
 *                                           operation rounded as torchvision rounds it)
 *   flip[b*V + v] != 0 mirrors that view horizontally (RandomHorizontalFlip; NULL = none,
 *   the test transform)
 *   out GM_NCHW: [B][V][C][H][W] (the reference's batch tensor), GM_NHWC: [V][B][H][W][C]
 *   (view-major channels_last, the engine's layout); dtype GM_F32 or GM_BF16 (RNE).
 * W must be a multiple of 4; x 4-byte aligned; out 8 (bf16) / 16 (fp32) byte aligned.
 * ------------------------------------------------------------------------- */
typedef struct gm_views_norm {
    const uint8_t* x;
    const uint8_t* flip;
    int B, V, H, W, C;
    float mean[4], std[4];
    void* out;
    int dtype, layout;
} gm_views_norm;

int gm_views_normalize(const gm_views_norm* p, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GREEDYMML_H */
