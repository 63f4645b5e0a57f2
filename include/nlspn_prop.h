/*
 * nlspn_prop.h — C ABI of the MI355X-native NLSPN propagation hot path.
 *
 * Drop-in boundary for XJTUXYC/NLSPN_ECCV20's non-local spatial propagation
 * (src/model/nlspnmodel.py:179-381) and the DCNv2 forward it rides on
 * (src/model/deformconv/src/vision.cpp:9 -> modulated_deform_conv.h:10-44 ->
 *  cuda/modulated_deform_conv_cuda.cu:19-121).  Plain pointers and sizes only:
 * no torch types cross this boundary.  All device pointers are caller-owned
 * (allocated by the caller on the current device); nothing is allocated on the
 * hot path.  `stream` is a hipStream_t passed as void* (NULL = legacy default
 * stream).  Every call only enqueues work; none synchronises the host, so every
 * call may be captured into a hipGraph.
 *
 * Layout: NCHW with one channel per plane; a "plane" is H*W contiguous
 * elements; tensors with several planes per batch item take a batch stride in
 * ELEMENTS (so slices of a (B,3K,H,W) off_aff head output can be passed without
 * a copy, as nlspnmodel.py:304-305 slices it).
 *
 * Errors: functions return 0 on success, a positive NLSPN_E* code otherwise;
 * nlspn_last_error() gives the message (thread-local), worded like the
 * reference's AT_ASSERTM/AT_ERROR messages where one exists.
 */
#ifndef NLSPN_PROP_H
#define NLSPN_PROP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NLSPN_ABI_VERSION 3

/* element type of every tensor argument (math is always fp32) */
#define NLSPN_DTYPE_F32 0
#define NLSPN_DTYPE_F16 1
#define NLSPN_DTYPE_F64 2 /* the seam-2 DCN entry points only (nlspn_mdcn_forward/backward) */

/* affinity normalisation kinds, src/config.py:259-263 / nlspnmodel.py:179-201 */
#define NLSPN_AFF_AS 0
#define NLSPN_AFF_ASS 1
#define NLSPN_AFF_TC 2
#define NLSPN_AFF_TGASS 3

/* flags (bit set) — src/config.py:250-257 */
#define NLSPN_PRESERVE_INPUT 0x1u /* args.preserve_input, nlspnmodel.py:328-334,342-344,355-357 */
#define NLSPN_ALWAYS_CLIP 0x2u    /* args.always_clip,    nlspnmodel.py:346-348,359-361,375-377 */

/* offset plane layout for nlspn_prop_step */
#define NLSPN_OFF_INSERTED 0 /* (B, 2(K+1), H, W): tap t uses planes 2t (dh), 2t+1 (dw) — _off_insert output */
#define NLSPN_OFF_RAW 1      /* (B, 2K, H, W): the head's raw slice; the reference tap is implicit zero */

/* error codes */
#define NLSPN_OK 0
#define NLSPN_EINVAL 1       /* bad shape / argument */
#define NLSPN_EUNSUPPORTED 2 /* geometry or dtype without a kernel instantiation */
#define NLSPN_EHIP 3         /* HIP runtime / launch error */
#define NLSPN_EABORTED 4     /* a resident launch aborted (nlspn_resident_status) */
/* nlspn_time_propagate *resident: bit once set when iteration 1 ran inside the resident
 * launches (an A/B form removed in round 4; never set now, kept for ABI stability) */
#define NLSPN_RESIDENT_FIRST 0x100

/* Version of this ABI (NLSPN_ABI_VERSION). */
int nlspn_abi_version(void);

/* Message for the last error on this thread ("" if none). */
const char *nlspn_last_error(void);

/*
 * S2D sparse-depth encoder front, fused.  Replaces the pool
 * pyramid and pool_convs of S2D.forward (src/model/nlspnmodel.py:437-455) and the
 * torch.cat([dep_feat, dep], 1) that feeds S2D.conv (:459):
 *   dep  : B x H x W (sparse depth, 0 = missing)
 *   w1 b1: pool_convs[0] conv weight (8 x 6) and bias (8); w2 b2: pool_convs[1]
 *          weight (16 x 8) and bias (16); device float32
 *   out  : B x 17 x H x W: channels 0..15 = ReLU(w2 . ReLU(w1 . pyramid + b1) + b2),
 *          channel 16 = dep
 *   pyr  : B x 6 x H x W, the min pools 3/5/7/9 (zeros = missing, :441-447) and max
 *          pools 11/13 (:449-452), or NULL (written for the weight gradients)
 * float32 only.
 */
int nlspn_s2d_pyramid(int dtype, const void *dep, const float *w1, const float *b1,
                      const float *w2, const float *b2, void *out, void *pyr,
                      int B, int H, int W, void *stream);

/*
 * Head epilogue: the decoder's last three 3x3 convolutions as one
 * kernel.  Replaces src/model/nlspnmodel.py:296-315 —
 *   pred_init  = ReLU(id_dec0(cat(id_fd1, fe1)))      id_dec0      :68
 *   off_aff    = off_aff_dec0(cat(off_aff_fd1, fe1))  off_aff_dec0 :74 (or :76 without offsets)
 *   confidence = Sigmoid(cf_dec0(cat(cf_fd1, fe1)))   cf_dec0      :83-86
 * with the four C-channel sources read in place (no concatenated copies):
 *   fe1, fd_oa   : B x C x H x W (fe1 and off_aff_fd1), contiguous, device float32
 *   fd_id, fd_cf : B x C x H x W (id_fd1, cf_fd1) or NULL (that head is skipped)
 *   wm, wv, bias : the weights packed by nlspn_head_pack_weights (nlspn_head_packed_size)
 *   off_aff      : B x nout x H x W;  pred_init, conf : B x 1 x H x W (NULL with their source)
 * Arithmetic: f32 operands and products on the matrix cores, f32 accumulation; only the
 * summation order differs from a sequential f32 convolution.  C % 16 == 0; float32 only.
 */
int nlspn_head_packed_size(int C, int nout, int64_t *wm_floats, int64_t *wv_floats,
                           int64_t *bias_floats);
int nlspn_head_pack_weights(const float *w_oa, const float *b_oa, const float *w_id,
                            const float *b_id, const float *w_cf, const float *b_cf,
                            float *wm, float *wv, float *bias, int C, int nout, void *stream);
int nlspn_head_epilogue(int dtype, const void *fe1, const void *fd_oa, const void *fd_id,
                        const void *fd_cf, const float *wm, const float *wv,
                        const float *bias, void *off_aff, void *pred_init, void *conf,
                        int B, int C, int H, int W, int nout, void *stream);

/*
 * The head epilogue with the propagation prologue fused in (3x3, K = 8, offsets on):
 * instead of the raw off_aff planes the epilogue writes what step 1 of the section
 * would — off_out = _off_insert(off) (nlspnmodel.py:324, B x 18 x H x W), aff_out =
 * _affinity_normalization + _aff_insert (:325, B x 9 x H x W), conf_out = the blended
 * confidence (:328-334, NULL with fd_cf), pred_init (:297) and p0 = the blended
 * [clamped] pred_init that iteration 1 propagates (:341-348) — then
 * nlspn_propagate_normalized runs the T iterations from them.  Same IEEE sequence as
 * nlspn_propagate's step 1: bit-identical outputs given the same convolution sums.
 * gamma: device pointer (learnable aff_scale_const); kind: NLSPN_AFF_*.
 */
int nlspn_head_epilogue_prologue(int dtype, const void *fe1, const void *fd_oa, const void *fd_id,
                                 const void *fd_cf, const float *wm, const float *wv,
                                 const float *bias, const void *dep, const float *gamma,
                                 void *pred_init, void *conf_out, void *aff_out, void *off_out,
                                 void *p0, int B, int C, int H, int W, int kh, int kw, int kind,
                                 unsigned flags, void *stream);

/*
 * Affinity normalisation + reference-tap insertion.
 * Replaces NLSPNModel._affinity_normalization (src/model/nlspnmodel.py:179-201)
 * followed by _aff_insert (:261-269).
 *   aff_raw : B x K planes, batch stride aff_bstride
 *   gamma   : device pointer to ONE float32 (aff_scale_const, :93-104); read on
 *             the device so a graph replay sees the current value (learnable γ)
 *   aff_out : B x (K+1) planes, contiguous, reference tap at index K/2
 */
int nlspn_affinity_normalize(int dtype, const void *aff_raw, int64_t aff_bstride,
                             const float *gamma, void *aff_out,
                             int B, int K, int H, int W, int kind, void *stream);

/*
 * One fused propagation iteration: f = p_in * conf (conf may be NULL,
 * nlspnmodel.py:350-353), out = _propagate_once(f, offset, aff) (:203-226),
 * then the preserve-input blend (:355-357) and clamp (:359-361) per flags.
 * Replaces, per iteration, DCN.modulated_deform_conv_forward
 * (modulated_deform_conv_func.py:26; vision.cpp:9; .cu:19-121) with NLSPN's
 * all-ones 1x1xkhxkw weight and zero bias, plus ~5 elementwise torch ops.
 *   p_in, conf, dep : B planes (contiguous); dep may be NULL without PRESERVE
 *   aff     : normalised affinity, B x (K+1) planes, batch stride aff_bstride
 *             (the tap at K/2 is NOT read: it is recomputed as 1 - sum of the
 *             others, bit-identical to what nlspn_affinity_normalize wrote)
 *   off     : offsets, batch stride off_bstride, layout NLSPN_OFF_* (NULL ->
 *             the no-offset branch :209-224: 3x3 replicate padding, K must be 8)
 *   p_out   : B planes; pred_out (optional): max(out, 0) — the epilogue :375-377
 *   kh, kw  : DCN kernel geometry (odd; K = kh*kw - 1). 3x3 = prop_kernel 3.
 */
int nlspn_prop_step(int dtype, const void *p_in, const void *conf, const void *dep,
                    const void *aff, int64_t aff_bstride,
                    const void *off, int64_t off_bstride, int off_layout,
                    void *p_out, void *pred_out,
                    int B, int H, int W, int kh, int kw, unsigned flags, void *stream);

/* Bytes of device workspace nlspn_propagate uses: the resident kernel's abort word
 * (index 0) and one 128-byte line per workgroup (its placement word).  With a NULL
 * workspace nlspn_propagate runs iterations 2..T as T-1 launches instead.  The resident
 * kernel also uses pred_inter itself for its hand-offs: planes 1..T-2 hold a poison
 * value (a signalling NaN) until written, so they must not alias any input. */
size_t nlspn_workspace_bytes(int dtype, int B, int H, int W);

/*
 * The whole propagation section, src/model/nlspnmodel.py:323-381, as T launches:
 *   step 1   : the prologue fused into the first iteration — _off_insert (:324)
 *              if off_out, _affinity_normalization (:325), mask_fix / confidence
 *              blend (:328-334), first blend+clamp (:341-348), then iteration 1
 *   steps 2..T: resident launches — the invariant planes held on chip for all
 *              iterations, one launch per image group (C2: all 8 NYU images in one;
 *              C3: the 4 KITTI images as two launches of 2), per-workgroup progress
 *              words in `workspace` — when the geometry allows it (3x3 learned
 *              offsets, W % 4 == 0, 16-B aligned planes, every rectangular part fits
 *              a workgroup: nlspn_resident_config), else T-1 nlspn_prop_step
 *              launches; pred_inter[t] each, the last also pred.
 *   Every form is bit-identical.
 * Inputs : pred_init, dep (B planes), conf (B planes, or NULL = conf_prop off),
 *          aff_raw (B x K planes, stride aff_bstride), off_raw (B x 2K planes,
 *          stride off_bstride, or NULL = no-offset branch), gamma (device f32).
 * Outputs: pred_inter (T x B planes, contiguous: list_pred), pred (B planes),
 *          aff_out (B x (K+1) planes), off_out (B x 2(K+1) planes, optional),
 *          conf_out (B planes, required iff conf != NULL).
 * workspace: nlspn_workspace_bytes() bytes of device memory (may be NULL when 0).
 */
int nlspn_propagate(int dtype, const void *pred_init, const void *dep, const void *conf,
                    const void *aff_raw, int64_t aff_bstride,
                    const void *off_raw, int64_t off_bstride, const float *gamma,
                    void *pred_inter, void *pred, void *aff_out, void *off_out,
                    void *conf_out, void *workspace,
                    int B, int H, int W, int kh, int kw, int T, int kind,
                    unsigned flags, void *stream);

/*
 * Plans: nlspn_propagate captured once into a hipGraph (T kernel nodes) and
 * replayed with one hipGraphLaunch.  Pointers are baked in at creation; γ stays
 * live because it is read from device memory.  A resident plan (step 1 + the
 * resident launches) re-issues its recorded launches directly instead, which
 * costs less than a graph launch; NLSPN_PLAN_GRAPH=1 forces the graph.
 */
typedef struct nlspn_plan *nlspn_plan_t;
int nlspn_plan_create(nlspn_plan_t *plan, int dtype, const void *pred_init, const void *dep,
                      const void *conf, const void *aff_raw, int64_t aff_bstride,
                      const void *off_raw, int64_t off_bstride, const float *gamma,
                      void *pred_inter, void *pred, void *aff_out, void *off_out,
                      void *conf_out, void *workspace,
                      int B, int H, int W, int kh, int kw, int T, int kind, unsigned flags);
int nlspn_plan_launch(nlspn_plan_t plan, void *stream);
int nlspn_plan_destroy(nlspn_plan_t plan);

/*
 * Backward of nlspn_propagate (float32 storage): what autograd computes through
 * src/model/nlspnmodel.py:323-381 with the DCNv2 backward for each of the T DCN
 * calls (modulated_deform_conv_cuda.cu:124-280; vision.cpp:10 ->
 * modulated_deform_conv.h:46-86).  Takes the forward's inputs and its saved
 * outputs (pred_inter, aff_out as aff_norm, conf_out as conf_eff) and the
 * incoming gradients (grad_pred and/or grad_pred_inter, T x B planes; either may
 * be NULL).  Writes grad_pred_init (B planes), grad_conf (B planes, iff conf),
 * grad_aff_raw (B x K planes, contiguous), grad_off_raw (B x 2K planes,
 * contiguous, iff off_raw), grad_gamma (1 float, TGASS only; may be NULL).
 * grad_aff_bstride / grad_off_bstride: batch strides of grad_aff_raw / grad_off_raw
 * in elements (0 = contiguous), so both can land in ONE packed (B, 3K, H, W)
 * gradient of the head output the two slices came from (nlspnmodel.py:304-305).
 * dep receives no gradient (the reference's sparse input).  workspace:
 * nlspn_backward_workspace_bytes() bytes.  dL/df is scattered with float
 * atomics (as the reference's col2im), so its last bits depend on arrival order.
 * Scratch use: the two-pass form (3x3 with offsets, T <= 3K: the default there)
 * first stores each iteration's dL/d(output) plane in grad_aff_raw / grad_off_raw
 * (the 3K planes per item they span together) and overwrites them with the gradients
 * in its second pass.  So neither may overlap any input, pred_inter, aff_norm,
 * conf_eff, the incoming gradients or each other (beyond the packed (B, 3K, H, W)
 * layout above), and after a failed call their contents are undefined.
 */
size_t nlspn_backward_workspace_bytes(int B, int H, int W, int kh, int kw);
int nlspn_propagate_backward(int dtype, const void *pred_init, const void *dep, const void *conf,
                             const void *aff_raw, int64_t aff_bstride,
                             const void *off_raw, int64_t off_bstride, const float *gamma,
                             const void *pred_inter, const void *aff_norm, const void *conf_eff,
                             const void *grad_pred, const void *grad_pred_inter,
                             void *grad_pred_init, void *grad_conf, void *grad_aff_raw,
                             int64_t grad_aff_bstride, void *grad_off_raw,
                             int64_t grad_off_bstride, float *grad_gamma, void *workspace,
                             int B, int H, int W, int kh, int kw, int T, int kind,
                             unsigned flags, void *stream);

/*
 * Backward of nlspn_prop_step (float32, raw offsets or the no-offset branch): what
 * autograd computes through one loop iteration, src/model/nlspnmodel.py:350-361, with
 * the DCNv2 backward of its _propagate_once (modulated_deform_conv_cuda.cu:124-280).
 * Used by the ConvGRU mode, where every iteration has its own affinity (:365-373).
 * Inputs are the step's inputs (feat, conf, dep, aff with (K+1) planes, raw offsets)
 * and grad_out = dL/d(step output).  Writes grad_feat and grad_conf (iff conf),
 * grad_aff ((K+1) planes per item, contiguous; plane K/2 is 0 because the step
 * recomputes that tap as 1 - sum of the others, so chaining it into
 * nlspn_affinity_normalize_backward gives the reference's _aff_insert gradient) and
 * grad_off (2K planes per item, contiguous).  workspace:
 * nlspn_prop_step_backward_workspace_bytes() bytes.
 */
size_t nlspn_prop_step_backward_workspace_bytes(int B, int H, int W);
int nlspn_prop_step_backward(int dtype, const void *feat, const void *conf, const void *dep,
                             const void *aff, int64_t aff_bstride, const void *off_raw,
                             int64_t off_bstride, const void *grad_out, void *grad_feat,
                             void *grad_conf, void *grad_aff, void *grad_off, void *workspace,
                             int B, int H, int W, int kh, int kw, unsigned flags, void *stream);

/*
 * Backward of nlspn_affinity_normalize (_affinity_normalization + _aff_insert,
 * src/model/nlspnmodel.py:179-201, :261-269): grad_aff is dL/d(output), (K+1) planes
 * per item, contiguous; writes grad_aff_raw (K planes per item, contiguous) and, for
 * TGASS, grad_gamma (1 float, summed in a fixed order; 0 for other kinds; may be
 * NULL).  workspace: nlspn_affinity_normalize_backward_workspace_bytes() bytes.
 */
size_t nlspn_affinity_normalize_backward_workspace_bytes(int B, int K, int H, int W);
int nlspn_affinity_normalize_backward(int dtype, const void *aff_raw, int64_t aff_bstride,
                                      const float *gamma, const void *grad_aff, void *grad_aff_raw,
                                      float *grad_gamma, void *workspace, int B, int K, int H,
                                      int W, int kind, void *stream);

/*
 * Modulated DCNv2 forward, seam 2 of the drop-in (the `DCN` pybind module,
 * src/model/deformconv/src/vision.cpp:9, modulated_deform_conv.h:10-44,
 * cuda/modulated_deform_conv_cuda.cu:19-121), as one direct (GEMM-free) gather
 * kernel.  dtype: float32, float16 (float arithmetic) or float64 (double
 * arithmetic, .cu:93's AT_DISPATCH_FLOATING_TYPES).  All tensors contiguous NCHW.
 *   input (B,C,H,W), weight (Cout, C/group, kh, kw), bias (Cout) or NULL,
 *   offset (B, 2*dg*kh*kw, Ho, Wo), mask (B, dg*kh*kw, Ho, Wo),
 *   output (B, Cout, Ho, Wo) with Ho = (H + 2ph - (dh(kh-1)+1))/sh + 1 (.cu:75-76).
 * Unlike the reference there is no im2col_step batch-divisibility restriction
 * (.cu:58-60); im2col_step is accepted and ignored.
 */
int nlspn_mdcn_forward(int dtype, const void *input, const void *weight, const void *bias,
                       const void *offset, const void *mask, void *output,
                       int B, int C, int H, int W, int Cout, int kh, int kw,
                       int sh, int sw, int ph, int pw, int dh, int dw,
                       int group, int deformable_group, void *stream);

/*
 * Modulated DCNv2 backward, seam 2 (DCN.modulated_deform_conv_backward,
 * src/model/deformconv/src/vision.cpp:10, modulated_deform_conv.h:46-86,
 * cuda/modulated_deform_conv_cuda.cu:124-280), float32 or float64 (dtype
 * NLSPN_DTYPE_F64: double arithmetic throughout, as the reference's
 * AT_DISPATCH_FLOATING_TYPES at .cu:221 — what gradcheck runs in).  Same layouts as
 * nlspn_mdcn_forward; grad_output (B, Cout, Ho, Wo).  Writes grad_input (zeroed
 * here, then scattered with atomics as the reference's col2im, so its last
 * bits depend on arrival order), grad_offset, grad_mask, grad_weight and — if
 * non-NULL — grad_bias.  Reproduces the reference's col2im call passing pad_h for
 * pad_w (.cuh:371): identical results for square padding, the reference's own
 * (shifted) grad_input otherwise.  No im2col_step batch-divisibility restriction.
 */
int nlspn_mdcn_backward(int dtype, const void *input, const void *weight, const void *offset,
                        const void *mask, const void *grad_output, void *grad_input,
                        void *grad_offset, void *grad_mask, void *grad_weight, void *grad_bias,
                        int B, int C, int H, int W, int Cout, int kh, int kw,
                        int sh, int sw, int ph, int pw, int dh, int dw,
                        int group, int deformable_group, void *stream);

/*
 * Diagnostics (not part of the reference surface): enqueue `reps` back-to-back
 * nlspn_prop_step launches on `stream`, each bracketed by its own HIP event
 * pair recorded by the dispatch itself (hipExtLaunchKernelGGL start/stop
 * events), then synchronise and return the mean and min per-launch kernel
 * duration in ms.  Used by bench.py for the roofline's kernel time.
 */
int nlspn_time_prop_step(int dtype, const void *p_in, const void *conf, const void *dep,
                         const void *aff, int64_t aff_bstride,
                         const void *off, int64_t off_bstride, int off_layout,
                         void *p_out, int B, int H, int W, int kh, int kw, unsigned flags,
                         int reps, void *stream, float *mean_ms, float *min_ms);

/*
 * Diagnostics: run nlspn_propagate `reps` times with dispatch-recorded HIP events
 * around every launch, synchronise, and return the mean duration of step 1
 * (first_ms) and of iterations 2..T (rest_ms: from the start of the first
 * resident launch to the end of the last, or the sum of the T-1 step kernels);
 * *resident = the number of resident launches (image groups), 0 for step launches,
 */
int nlspn_time_propagate(int dtype, const void *pred_init, const void *dep, const void *conf,
                         const void *aff_raw, int64_t aff_bstride, const void *off_raw,
                         int64_t off_bstride, const float *gamma, void *pred_inter, void *pred,
                         void *aff_out, void *off_out, void *conf_out, void *workspace,
                         int B, int H, int W, int kh, int kw, int T, int kind, unsigned flags,
                         int reps, void *stream, float *first_ms, float *rest_ms, int *resident);

/*
 * The propagation loop (nlspnmodel.py:340-381) from already-prologued inputs: p0
 * (iteration 1's input), conf_eff (the blended confidence, or NULL), aff_norm
 * (B x (K+1) planes, normalised, reference tap inserted), off_ins (B x 2(K+1)
 * planes, _off_insert layout) — the outputs of nlspn_head_epilogue_prologue or of
 * nlspn_propagate's step 1.  Writes pred_inter (T x B planes) and pred as
 * nlspn_propagate does (same kernels: iteration 1 a plain step, 2..T resident where it
 * applies); workspace as nlspn_propagate's.
 */
int nlspn_propagate_normalized(int dtype, const void *p0, const void *dep, const void *conf_eff,
                               const void *aff_norm, const void *off_ins, void *pred_inter,
                               void *pred, void *workspace, int B, int H, int W, int kh,
                               int kw, int T, unsigned flags, void *stream);

/*
 * Diagnostics: 1 if nlspn_propagate would run iterations 2..T as the resident
 * kernel for this shape (given 16-B aligned planes and a workspace), with the
 * launch shape of its first image group; 0 otherwise.  Queries the current
 * device's CU count.
 */
int nlspn_resident_config(int dtype, int B, int H, int W, int kh, int kw, int T, int has_conf,
                          int *grid, int *block, int *lds_bytes);

/*
 * Sticky abort status of the resident path on the current device: 1 if a resident
 * launch aborted since the last clear (a part polled past its spin limit, i.e. the
 * grid was not co-resident — e.g. a concurrent resident launch from another
 * process; launches from this process are serialised per device across streams).
 * Such a launch fills the outputs it had not written with NaN.  Reads a
 * host-mapped word the kernel writes: never synchronises, so the host sees an
 * abort once the launch has finished.  Sets nlspn_last_error (NLSPN_EABORTED).
 * clear != 0 resets the word after reading it.  Replaces nothing in the
 * reference, whose kernels only printf launch errors (.cuh:348-352); the torch
 * layer raises RuntimeError on it, as c10::Error surfaces in the reference.
 */
int nlspn_resident_status(int clear);

/*
 * GRU-mode convolutions (the reference's forced default mode, src/config.py:225-228): one
 * convolution of a GRU-mode iteration, f32 NCHW, inference (nlspnmodel.py:365-373), on the
 * f32-input matrix cores with bias and activation in the epilogue (csrc/nlspn_gconv.h).
 * Replaces the torch/MIOpen module calls of
 *   encode_dep / encode_aff   (:127-138)  NLSPN_GC_S2 / NLSPN_GC_S2_C16: 3x3 stride 2 pad 1
 *   ConvGRU                   (:386-403)  NLSPN_GC_GRU1 then NLSPN_GC_GRU2
 *   decode_aff + _clip_as     (:140-143, :228-250)  NLSPN_GC_T2 / NLSPN_GC_T2_C16: 3x3
 *                                          transposed stride 2 pad 1 output pad 1
 * x0 (c0 channels) then x1 (c1 channels, may be null with c1 = 0) are the input channels
 * (torch.cat order, read in place); Hi x Wi the input size.  wpk: the weights packed by
 * nlspn_gconv_pack_layout's layout (nlspn_eccv20_amd/gru.py packs them), bias padded to
 * the co tiles.  NLSPN_GC_S2* / NLSPN_GC_T2*: y = act(conv + bias) stored as (B, cout, ohs,
 * ows) (ohs / ows <= the full output size: the crop), act NLSPN_GC_ACT_*, inputs divided by
 * in_div while read (encode_dep's new_pred / max_depth; 1: none; != 1 only with
 * NLSPN_GC_S2_SMALL, else NLSPN_EINVAL).  NLSPN_GC_GRU1 (x0 = h, x1
 * = x, cout = 3 hc): z, r*h and qx (convq's x half + bias) into zb / rhb / qxb;
 * NLSPN_GC_GRU2 (x0 = rhb, c1 = 0, cout = hc): h' = (1 - z) h + z tanh(convq's r*h half +
 * qx) into hout.  Returns NLSPN_EUNSUPPORTED when a shape's window does not fit the kernel.
 */
#define NLSPN_GC_S2 0
#define NLSPN_GC_S2_C16 1
#define NLSPN_GC_GRU1 2
#define NLSPN_GC_GRU2 3
#define NLSPN_GC_T2 4
#define NLSPN_GC_T2_C16 5
/* the narrow first encoder convs on the VALU: wpk is then the module's own (16, cin, 3, 3)
 * weight tensor (cin <= 16) and bias its own (16) */
#define NLSPN_GC_S2_SMALL 6
/* NLSPN_GC_S2 / NLSPN_GC_GRU2 on 32-pixel tiles (their co tile, hence their packed weights):
 * nlspn_gconv switches to them by itself when 64-pixel tiles would give fewer than two
 * workgroups per CU (the 1/8-scale layers at NYU B=8) */
#define NLSPN_GC_S2_N32 23
#define NLSPN_GC_GRU2_N32 24
/* NLSPN_GC_T2_C16 (its packed weights) with the affinity normalisation in its epilogue: the
 * preset of nlspn_gconv_affnorm only (nlspn_gconv refuses it) */
#define NLSPN_GC_T2_AFF 25
#define NLSPN_GC_ACT_NONE 0
#define NLSPN_GC_ACT_RELU 1
#define NLSPN_GC_ACT_TANH 2
/* the packed weight layout of a preset: *co_tile output channels per tile, *cin_chunk input
 * channels per chunk (the packed input channel count is a multiple), *transposed */
int nlspn_gconv_pack_layout(int layer, int *co_tile, int *cin_chunk, int *transposed);
int nlspn_gconv(int layer, const float *x0, int c0, const float *x1, int c1, const float *wpk,
                const float *bias, float *y, const float *h, float *zb, float *rhb, float *qxb,
                float *hout, int B, int Hi, int Wi, int cout, int ohs, int ows, int act,
                float in_div, int hc, void *stream);
/*
 * decode_aff's last layer fused with the affinity normalisation that follows it
 * (nlspnmodel.py:373 _aff_head, then :179-201 _affinity_normalization and :261-269
 * _aff_insert at the next iteration's start; replaces nlspn_gconv(NLSPN_GC_T2_C16, ...)
 * + nlspn_affinity_normalize): the K = 8 raw taps of the transposed conv (x0: (B, c0, Hi,
 * Wi), weights packed as NLSPN_GC_T2_C16, act NLSPN_GC_ACT_*) are normalised per pixel as
 * they leave the accumulators and stored as aff_out (B, K + 1, ohs, ows) with the reference
 * tap at K / 2, kind NLSPN_AFF_*, *gamma the device scalar.  Bit-equal to the two launches.
 */
int nlspn_gconv_affnorm(const float *x0, int c0, const float *wpk, const float *bias, float *aff_out,
                        const float *gamma, int kind, int B, int Hi, int Wi, int K, int ohs, int ows, int act,
                        void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NLSPN_PROP_H */
