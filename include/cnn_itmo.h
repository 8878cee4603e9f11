/*
 * cnn_itmo.h -- C ABI of libcnnitmo.so, the MI355X (gfx950) kernels behind the
 * CNN-ITMO U-Net hot path.
 *
 * The reference (LynxHack/CNN-ITMO) reaches its arithmetic through the Keras
 * functional Layer API (Conv2D, Conv2DTranspose, MaxPooling2D,
 * BatchNormalization, Activation, Dropout, concatenate) at
 * /root/reference/model.py:195-281; TensorFlow/cuDNN execute it.  Each entry
 * point below replaces one of those layer calls (forward or its gradient); the
 * Python host side (cnn_itmo_amd/) mirrors the Keras API and calls these.
 *
 * Conventions
 *   - Every function is stateless, never allocates, and enqueues work on the
 *     given HIP stream (hipStream_t passed as void*).  Scratch memory is
 *     caller-owned; size it with the *_workspace_bytes / *_rows queries.
 *   - Return value: 0 = ok, negative = error (CNNITMO_E*);
 *     cnnitmo_last_error() returns a thread-local message.
 *   - dtype: CNNITMO_F32 (fp32 storage) or CNNITMO_BF16 (bf16 storage).
 *     Accumulation is always fp32 (MFMA f32 accumulators).
 *   - Activations are NHWC.  A "view" of an activation is (ptr, ld, off):
 *     element (p, c) of a P-pixel, C-channel view lives at ptr[p*ld + off + c].
 *     This is how channel concatenation (model.py:246,251,256,261) is zero-copy:
 *     producers write channel slices of one buffer.
 *   - Weight layouts: Conv2D OHWI [Cout][kh][kw][Cin]; Conv2DTranspose
 *     [2][2][Cout][Cin] (Keras' own kernel layout, layers.txt:78).  Master
 *     weights are fp32; cnnitmo_prep_* produce the dtype copies kernels read.
 *   - Per-channel fp32 vectors (bias, BN gamma/beta/stats) are always fp32.
 */
#ifndef CNN_ITMO_H_
#define CNN_ITMO_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CNNITMO_F32 0
#define CNNITMO_BF16 1

#define CNNITMO_OK 0
#define CNNITMO_EINVAL (-1)
#define CNNITMO_EUNSUPPORTED (-2)
#define CNNITMO_ELAUNCH (-3)

/* Epilogue flags for the forward convolutions. */
#define CNNITMO_RELU 1   /* Activation('relu') after the conv (model.py:196,200) */
#define CNNITMO_STATS 2  /* write per-tile BN partial sums (sum, sum of squares) */
#define CNNITMO_AFFINE 4 /* y = v*scale[c] + shift[c] after ReLU (inference BN) */
#define CNNITMO_BIAS_PER_COL 8 /* bias indexed by GEMM column (tconv: [4*cout], folded BN) */

/* Flags for BN apply / backward. */
#define CNNITMO_DROPOUT 1 /* Dropout(0.5), model.py:226,239 (train only) */
#define CNNITMO_NO_BN 2   /* bwd: plain ReLU gradient, no BN (config-1 net)  */
#define CNNITMO_PARITY 4  /* bwd apply: bias partials split by (h&1, w&1) -> [4][c] */

/* ABI version: 2 since CNNITMO_CONSUMER_ROWS went from 16 to 64 (a caller built against the
 * old header under-allocates cnnitmo_bn_consumer_sums' part: check cnnitmo_consumer_rows()) and
 * cnnitmo_bn_apply started to require 16-byte aligned scale / shift. */
int cnnitmo_version(void);
const char* cnnitmo_last_error(void);

/* ---------------------------------------------------------------------------
 * Conv2D(f, 3, padding='same') -- replaces Conv2D at model.py:196 (via ConvBN).
 * x view: [n, h, w, cin] (ld, off); wt: [cout][3][3][cin] in dtype.
 * out view: [n, h, w, cout] (ld, off).  flags: CNNITMO_RELU|STATS|AFFINE.
 * stat_part (STATS): [rows][2][cout] fp32, rows = cnnitmo_fwd_stat_rows(...).
 * aff_scale/aff_shift (AFFINE): [cout] fp32.
 * border (nullable): [cout][8] zero-padding correction of a folded input BN
 * (cnnitmo_fold_conv3x3): when x holds r and the conv's true input is
 * y = r*s + h, pass wt/bias/border from the fold.
 * Requires cin % 32 == 0 (bf16) or % 16 == 0 (f32), cout % 32 == 0.
 */
int cnnitmo_conv3x3_fwd(int dtype, const void* x, int x_ld, int x_off, int n, int h, int w,
                        int cin, const void* wt, const float* bias, int cout, void* out,
                        int out_ld, int out_off, int flags, const float* aff_scale,
                        const float* aff_shift, float* stat_part, const float* border,
                        void* stream);

/* conv3x3_fwd with the 2x2 MaxPooling2D of its output fused into the epilogue
 * (model.py:209-210, 214-215, 219-220: ConvBN -> MaxPooling2D).  pool_out
 * [n, h/2, w/2] x pool_ld (dtype) gets the pooled stored value, pool_idx (same layout,
 * bytes) its window index (first maximum in window order (0,0),(0,1),(1,0),(1,1), the
 * cnnitmo_maxpool2x2_fwd rule).  pool_sign [cout] (nullable): per channel, pool by the
 * maximum (> 0), the minimum (< 0) or take the first element (0) of the stored values:
 * with the output stored as r and the BN folded into the consumers, sign(gamma) makes
 * s * pooled + h the max-pool of y = r * s + h (s = gamma * invstd).  Requires even h, w
 * and the halo kernel (cnnitmo_conv3x3_pool_supported). */
int cnnitmo_conv3x3_fwd_pool(int dtype, const void* x, int x_ld, int x_off, int n, int h, int w, int cin,
                             const void* wt, const float* bias, int cout, void* out, int out_ld, int out_off,
                             int flags, const float* aff_scale, const float* aff_shift, float* stat_part,
                             const float* border, void* pool_out, int pool_ld, unsigned char* pool_idx,
                             const float* pool_sign, void* stream);
/* The last 3x3 ConvBN (conv9 = ConvBN(64, 3, merge9), model.py:262) with the sigmoid head
 * (model.py:276, Conv2D(3, 1, activation='sigmoid')) in its epilogue, for inference
 * (predict.py:62): yhat [n][h_valid][w][3] fp32 = sigmoid(y . head_w[3][cout] + head_b), y = the
 * conv's epilogue output (flags/aff as cnnitmo_conv3x3_fwd: ReLU, BN affine), never stored.
 * Replaces cnnitmo_conv3x3_fwd + cnnitmo_head_fwd.  cout = 64; no BN sums. */
int cnnitmo_conv3x3_fwd_head(int dtype, const void* x, int x_ld, int x_off, int n, int h, int w, int cin,
                             const void* wt, const float* bias, int cout, int flags, const float* aff_scale,
                             const float* aff_shift, int h_valid, const float* head_w, const float* head_b,
                             float* yhat, void* stream);
int cnnitmo_conv3x3_head_supported(int dtype, int n, int h, int w, int cin, int cout);
int cnnitmo_conv3x3_pool_supported(int dtype, int n, int h, int w, int cin, int cout);

/* conv3x3_fwd over concatenate([x1, x2]) (model.py:261, Keras axis=3) read from its
 * two members, without a concat buffer: input channels [0, c1) are x1's view
 * (x1_ld, x1_off), channels [c1, cin) are x2's (x2_ld, x2_off).  bf16 only, c1 % 32 == 0,
 * an epilogue (flags / bias / stats) required; CNNITMO_EUNSUPPORTED otherwise.  Used for
 * the level-0 concat [conv1 32 | up9 64], whose members each occupy partial 128-B lines
 * of a 192-B concat row. */
int cnnitmo_conv3x3_fwd_cat(int dtype, const void* x1, int x1_ld, int x1_off, int c1, const void* x2,
                            int x2_ld, int x2_off, int n, int h, int w, int cin, const void* wt,
                            const float* bias, int cout, void* out, int out_ld, int out_off, int flags,
                            const float* aff_scale, const float* aff_shift, float* stat_part,
                            const float* border, void* stream);
/* 1 if cnnitmo_conv3x3_fwd_cat runs for these sizes in this process (dtype, the
 * channel split, CNNITMO_HALO and the device's workgroup count decide), else 0: a
 * planner must not keep a concat split into members the forward cannot read. */
int cnnitmo_conv3x3_fwd_cat_supported(int dtype, int n, int h, int w, int c1, int cin, int cout);

/* Name of the kernel conv3x3_fwd (dgrad = 0) / conv3x3_dgrad (dgrad = 1, same
 * layer cin/cout) launches for these sizes (profiling labels; no GPU needed). */
const char* cnnitmo_conv3x3_kernel_name(int dtype, int n, int h, int w, int cin, int cout,
                                        int dgrad);
/* Same for tconv2x2_fwd / _dgrad over an n x h x w input grid. */
const char* cnnitmo_tconv2x2_kernel_name(int dtype, int n, int h, int w, int cin, int cout,
                                         int dgrad);

/* Rows of the BN partial-sum buffer written by a forward conv over m output
 * pixels with ncols GEMM columns (4*cout for tconv2x2; the 1-tap first layer).
 * conv3x3: use cnnitmo_conv3x3_stat_rows (the row count depends on the frame). */
int cnnitmo_fwd_stat_rows(int dtype, long m, int ncols);
long cnnitmo_conv3x3_stat_rows(int dtype, int n, int h, int w, int cin, int cout);
/* Same for cnnitmo_tconv2x2_fwd over an n x h x w input grid (columns 4*cout). */
long cnnitmo_tconv2x2_stat_rows(int dtype, int n, int h, int w, int cin, int cout);

/* Input-gradient of conv3x3 (TF Conv2DBackpropInput).  dz: [n,h,w,cout]
 * contiguous; wt_flip: [cin][3][3][cout] = W[co][2-r][2-s][ci] (from
 * cnnitmo_prep_conv3x3_weights).  dx view [n,h,w,cin] (ld, off) is OVERWRITTEN. */
int cnnitmo_conv3x3_dgrad(int dtype, const void* dz, int n, int h, int w, int cout,
                          const void* wt_flip, int cin, void* dx, int dx_ld, int dx_off,
                          void* stream);
/* conv3x3_dgrad with the PRODUCER's BN backward fused into its store (bf16):
 * input-gradient columns [c0, c1) are the gradient g of a folded BN output
 * whose backward coefficients coef [3][c1-c0] (cnnitmo_bn_bwd_finalize) are
 * already known (consumer-derived sums); they are written as the producer's
 * dz = [r>0]*(a*g - b*r + e) to dz_out [n*h*w][c1-c0] (r: the producer's saved
 * view, element (p, j) at r[p*r_ld + r_off + j]) together with column-sum
 * partials part [rows][parity ? 4 : 1][c1-c0] (rows =
 * cnnitmo_conv3x3_dgrad_bn_rows; parity splits by (h&1, w&1) like
 * CNNITMO_PARITY).  Columns outside [c0, c1) go to dx as in conv3x3_dgrad (dx
 * may be NULL when [c0, c1) = [0, cin)).  Replaces conv3x3_dgrad +
 * cnnitmo_bn_bwd_apply.  rows = 0: not available for these sizes. */
long cnnitmo_conv3x3_dgrad_bn_rows(int dtype, int n, int h, int w, int cout, int cin, int c0, int c1);
int cnnitmo_conv3x3_dgrad_bn(int dtype, const void* dz, int n, int h, int w, int cout,
                             const void* wt_flip, int cin, void* dx, int dx_ld, int dx_off, int c0,
                             int c1, const float* coef, const void* r, int r_ld, int r_off,
                             void* dz_out, float* part, int parity, void* stream);
/* Label of the kernel cnnitmo_conv3x3_dgrad_bn launches ("" = unavailable; profiling only). */
const char* cnnitmo_conv3x3_dgrad_bn_kernel_name(int dtype, int n, int h, int w, int cout, int cin,
                                                 int c0, int c1);
/* The skip path of a concatenate whose other reader is a MaxPooling2D(2) (model.py:209-211
 * + 261: conv1 feeds pool1 and merge9): the input-gradient of the concat-consuming conv
 * for the skip member's cin channels (wt_flip: its rows [cin][3][3][cout] of the flipped
 * weights), PLUS the pool's gradient dy_pool [n,h/2,w/2,cin] (dense) routed to the window
 * position idx [n,h/2,w/2,cin] (bytes, first-max index in window order, as
 * cnnitmo_maxpool2x2_fwd / _fwd_pool write them), through the producer's BN backward:
 * dz_out [n*h*w][cin] = [r>0]*(a*(bf16(g) + routed) - b*r + e), column-sum partials part
 * [rows][cin] (rows = cnnitmo_conv3x3_dgrad_bn_pooled_rows; 0: unavailable).  h, w even.
 * Replaces conv3x3_dgrad + cnnitmo_bn_bwd_apply_pooled (the skip gradient is never
 * stored). */
long cnnitmo_conv3x3_dgrad_bn_pooled_rows(int dtype, int n, int h, int w, int cout, int cin);
int cnnitmo_conv3x3_dgrad_bn_pooled(int dtype, const void* dz, int n, int h, int w, int cout,
                                    const void* wt_flip, int cin, const float* coef, const void* r, int r_ld,
                                    int r_off, const void* dy_pool, const unsigned char* idx, void* dz_out,
                                    float* part, void* stream);
const char* cnnitmo_conv3x3_dgrad_bn_pooled_kernel_name(int dtype, int n, int h, int w, int cout, int cin);

/* Weight-gradient of conv3x3 (TF Conv2DBackpropFilter).  x view [n,h,w,cin];
 * dz [n,h,w,cout] contiguous; dw: [cout][3][3][cin] fp32, OVERWRITTEN.
 * ntaps = 9 for the 3x3 conv, 1 for a 1x1 / pre-packed (im2col) input. */
size_t cnnitmo_wgrad_workspace_bytes(int dtype, int n, int h, int w, int cin, int cout,
                                     int ntaps);
/* Label of the main kernel a weight gradient launches for these sizes (ntaps 9 /
 * 1: conv, 4: tconv2x2; profiling only, no GPU needed). */
const char* cnnitmo_wgrad_kernel_name(int dtype, int ntaps, int n, int h, int w, int cin, int cout);
int cnnitmo_conv_wgrad(int dtype, int ntaps, const void* x, int x_ld, int x_off,
                       const void* dz, int n, int h, int w, int cin, int cout, float* dw,
                       int dw_cols, const float* fold_scale, const float* fold_shift,
                       const float* fold_db, const float* fold_border, float* raw_out,
                       void* workspace, size_t ws_bytes, void* stream);
/* Folded input BN (x holds r, the conv's input is y = r*s + h, see
 * cnnitmo_fold_conv3x3): pass fold_scale = s, fold_shift = h [cin], fold_db = the
 * bias gradient [cout] and fold_border = the reduced border sums [8][cout] of dz
 * (cnnitmo_border_sums + cnnitmo_colsum); dw is then the exact gradient w.r.t. W.
 * All four NULL: plain weight gradient.  raw_out (nullable, same layout as dw):
 * the uncorrected sum dz (x) r, input of cnnitmo_bn_consumer_sums. */

/* cnnitmo_conv_wgrad (ntaps 9, bf16) over concatenate([x1, x2]) read from its members
 * (see cnnitmo_conv3x3_fwd_cat): c1 == 32, cin == 96 (merge9 -> conv9, model.py:261-262).
 * workspace: cnnitmo_wgrad_cat_workspace_bytes (0 = unsupported sizes). */
size_t cnnitmo_wgrad_cat_workspace_bytes(int n, int h, int w, int c1, int cin, int cout);
const char* cnnitmo_wgrad_cat_kernel_name(int n, int h, int w, int c1, int cin, int cout);
int cnnitmo_conv_wgrad_cat(int dtype, const void* x1, int x1_ld, int x1_off, int c1, const void* x2, int x2_ld,
                           int x2_off, const void* dz, int n, int h, int w, int cin, int cout, float* dw,
                           const float* fold_scale, const float* fold_shift, const float* fold_db,
                           const float* fold_border, float* raw_out, void* workspace, size_t ws_bytes,
                           void* stream);

/* First layer (Cin=3): pack x [n,h_valid,w,3] fp32 into [n,h,w,32] dtype
 * columns k=(r*3+s)*3+c (k<27, zero pad; rows >= h_valid are zero), so that
 * conv2d_1 runs as a 1-tap GEMM with K=32.  Fuses the /255 input's cast and
 * the pad-to-multiple-of-16 of predict.py:59 / SURVEY 8a. */
int cnnitmo_im2col_c3(int dtype, const float* x, int n, int h_valid, int h, int w, void* cols,
                      void* stream);
/* 1-tap GEMM forward over packed columns: out = cols[m][k] * wt[cout][k]. */
int cnnitmo_conv1tap_fwd(int dtype, const void* cols, int k, long m, const void* wt,
                         const float* bias, int cout, void* out, int out_ld, int out_off,
                         int flags, const float* aff_scale, const float* aff_shift,
                         float* stat_part, void* stream);

/* First layer without im2col: x [n,h_valid,w,3] fp32 -> out view [n,h,w,32] in dtype
 * (bf16 or fp32; ld, off), rows >= h_valid of the input read as zero (pad-to-16).  wt:
 * [32][32] packed columns in dtype (cnnitmo_prep_c3_weights); flags/aff as conv3x3_fwd;
 * stat_part [rows][2][32] with rows = cnnitmo_conv_c3_stat_rows.  Replaces
 * cnnitmo_im2col_c3 + cnnitmo_conv1tap_fwd for model.py:208. */
long cnnitmo_conv_c3_stat_rows(int n, int h, int w);
int cnnitmo_conv_c3_fwd(int dtype, const float* x, int n, int h_valid, int h, int w, const void* wt,
                        const float* bias, void* out, int out_ld, int out_off, int flags,
                        const float* aff_scale, const float* aff_shift, float* stat_part, void* stream);
/* dw [32][27] fp32 (OVERWRITTEN; OHWI) = sum_p dz[p][co] * patch(x, p)[k], dz [n*h*w][32]
 * in dtype (bf16 or fp32) contiguous.  Replaces cnnitmo_conv_wgrad(ntaps = 1) over im2col
 * columns. */
size_t cnnitmo_conv_c3_wgrad_workspace_bytes(int n, int h, int w);
int cnnitmo_conv_c3_wgrad(int dtype, const float* x, int n, int h_valid, int h, int w, const void* dz,
                          float* dw, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Conv2DTranspose(f, 2, strides=2, 'valid') -- replaces model.py:200
 * (ConvBNTranspose).  x [n,h,w,cin] contiguous; k: [2][2][cout][cin] dtype;
 * out view [n,2h,2w,cout] (ld, off); flags/stat_part as conv3x3 (stat_part
 * columns are [4*cout] = (tap, channel) groups; only a channel's total over the
 * four groups is defined: cnnitmo_bn_fwd_finalize with groups = 4 folds them).
 */
int cnnitmo_tconv2x2_fwd(int dtype, const void* x, int n, int h, int w, int cin, const void* k,
                         const float* bias, int cout, void* out, int out_ld, int out_off,
                         int flags, const float* aff_scale, const float* aff_shift,
                         float* stat_part, void* stream);
/* dx [n,h,w,cin] (contiguous, OVERWRITTEN) from dout [n,2h,2w,cout] and
 * kT: [cin][2][2][cout] (from cnnitmo_prep_tconv2x2_weights). */
int cnnitmo_tconv2x2_dgrad(int dtype, const void* dout, int n, int h, int w, int cout,
                           const void* kT, int cin, void* dx, void* stream);
/* tconv2x2_dgrad with the PRODUCER's BN backward fused into its store (bf16;
 * the tconv input is a folded BN output whose coefficients coef [3][cin] are
 * known): dz_out [n*h*w][cin] = [r>0]*(a*g - b*r + e) of the input gradient g,
 * r the producer's saved view (element (p, c) at r[p*r_ld + r_off + c]), and
 * column-sum partials part [rows][cin] (rows = cnnitmo_tconv2x2_dgrad_bn_rows;
 * 0 = not available for these sizes).  Replaces tconv2x2_dgrad + bn_bwd_apply. */
long cnnitmo_tconv2x2_dgrad_bn_rows(int dtype, int n, int h, int w, int cout, int cin);
int cnnitmo_tconv2x2_dgrad_bn(int dtype, const void* dout, int n, int h, int w, int cout,
                              const void* kT, int cin, const float* coef, const void* r, int r_ld,
                              int r_off, void* dz_out, float* part, void* stream);
/* Label of the kernel cnnitmo_tconv2x2_dgrad_bn launches ("" = unavailable; profiling only). */
const char* cnnitmo_tconv2x2_dgrad_bn_kernel_name(int dtype, int n, int h, int w, int cout, int cin);
/* dk [2][2][cout][cin] fp32 (OVERWRITTEN) from x [n,h,w,cin], dout [n,2h,2w,cout]. */
int cnnitmo_tconv2x2_wgrad(int dtype, const void* x, const void* dout, int n, int h, int w,
                           int cin, int cout, float* dk, const float* fold_scale,
                           const float* fold_shift, const float* fold_par, float* raw_out,
                           void* workspace, size_t ws_bytes, void* stream);
/* fold_par: per-tap sums of dout [4][cout] (cnnitmo_bn_bwd_apply with
 * CNNITMO_PARITY, reduced by cnnitmo_colsum); NULL trio = plain gradient. */
size_t cnnitmo_tconv2x2_wgrad_workspace_bytes(int dtype, int n, int h, int w, int cin, int cout);

/* Weight preparation (after every optimizer step): fp32 master -> dtype copies.
 * conv3x3: w [cout][3][3][cin] -> w_fwd (same layout), w_flip [cin][3][3][cout].
 * w_flip may be NULL (first layer).  tconv: k [2][2][cout][cin] -> k_fwd (same),
 * kT [cin][2][2][cout].  pack_c3: w [32][3][3][3] -> [32][32] zero-padded. */
int cnnitmo_prep_conv3x3_weights(int dtype, const float* w, int cout, int cin, void* w_fwd,
                                 void* w_flip, void* stream);
int cnnitmo_prep_tconv2x2_weights(int dtype, const float* k, int cout, int cin, void* k_fwd,
                                  void* kT, void* stream);
int cnnitmo_prep_c3_weights(int dtype, const float* w, int cout, void* w_packed, void* stream);

/* BN folding (training): the consumer of a BN output y = r*s + h reads the
 * stored post-ReLU r and folds the affine into its own weights instead of
 * materialising y (removes one full read+write of every activation).
 * conv3x3: w_out = W*s (dtype), bias_out[cout] = b + sum_t u_t and border[cout][8]
 *   (u_t[co] = sum_ci W[co][t][ci]*h[ci]) for cnnitmo_conv3x3_fwd's border.
 * tconv2x2: k_out = K*s, bias_out[4*cout] per (tap, co) -> CNNITMO_BIAS_PER_COL.
 * scale/shift NULL = identity. */
int cnnitmo_fold_conv3x3(int dtype, const float* w, const float* bias, const float* scale,
                         const float* shift, int cout, int cin, void* w_out, float* bias_out,
                         float* border, void* stream);
int cnnitmo_fold_tconv2x2(int dtype, const float* k, const float* bias, const float* scale,
                          const float* shift, int cout, int cin, void* k_out, float* bias_out,
                          void* stream);
/* Border partial sums of dz [n,h,w,c] (contiguous): rows cnnitmo_border_rows(n)
 * of [8][c] = {row 0, row h-1, col 0, col w-1, 4 corners}; reduce with cnnitmo_colsum. */
int cnnitmo_border_rows(int n);
int cnnitmo_border_sums(int dtype, const void* dz, int n, int h, int w, int c, float* part,
                        void* stream);

/* ---------------------------------------------------------------------------
 * MaxPooling2D(pool_size=(2,2), strides=2) -- model.py:210,215,220,227.
 * fwd: x view [n,h,w,c] -> y [n,h/2,w/2,c] contiguous + argmax idx uint8 (0..3,
 * first maximum in row-major window order).
 * bwd: dx view [n,h,w,c] += scatter of dy to the argmax (other entries untouched).
 */
int cnnitmo_maxpool2x2_fwd(int dtype, const void* x, int x_ld, int x_off, int n, int h, int w,
                           int c, void* y, uint8_t* idx, const float* scale, const float* shift,
                           void* stream);
/* scale/shift (nullable, [c]): pool over x*scale + shift (a folded BN output). */
int cnnitmo_maxpool2x2_bwd(int dtype, const void* dy, const uint8_t* idx, int n, int h, int w,
                           int c, void* dx, int dx_ld, int dx_off, void* stream);

/* ---------------------------------------------------------------------------
 * BatchNormalization() (axis=-1, eps 1e-3, momentum 0.99) -- model.py:196,200.
 * Training forward: the conv epilogue writes r = relu(conv) and partial sums;
 * cnnitmo_bn_fwd_finalize reduces them (fp64) to batch mean / biased variance,
 * produces scale = gamma*invstd, shift = beta - mean*scale, saves mean/invstd for
 * backward and updates the moving statistics (Keras-2.2: var *= n/(n-(1+eps))).
 * groups: the stat_part columns are [groups][c] (4 for a tconv, else 1).
 * workspace: cnnitmo_reduce_workspace_bytes(rows, groups*c*2).
 */
size_t cnnitmo_reduce_workspace_bytes(long rows, int cols);
int cnnitmo_bn_fwd_finalize(const float* stat_part, long rows, int c, int groups, double count,
                            const float* gamma, const float* beta, float* moving_mean,
                            float* moving_var, float momentum, float eps, float* scale,
                            float* shift, float* save_mean, float* save_invstd,
                            void* workspace, void* stream);
/* Inference-mode coefficients from the moving statistics. */
int cnnitmo_bn_infer_coeffs(int c, const float* gamma, const float* beta, const float* mmean,
                            const float* mvar, float eps, float* scale, float* shift,
                            void* stream);
/* y view = r*scale + shift (optionally Dropout(0.5): element (p,c) kept iff the
 * counter hash of (seed, layer, p*c_total + c) says so, kept values x2).  scale and shift
 * must be 16-byte aligned (CNNITMO_EINVAL otherwise; since cnnitmo_version() 2). */
int cnnitmo_bn_apply(int dtype, const void* r, long p, int c, const float* scale,
                     const float* shift, void* y, int y_ld, int y_off, int flags,
                     uint64_t drop_seed, int drop_layer, void* stream);
/* Backward.  dy view (ld, off) is the gradient w.r.t. the BN (or dropout)
 * output; r is the saved post-ReLU tensor [p][c].
 * Step 1 (reduce+finalize): dgamma, dbeta (written, fp32) and the three dz
 * coefficients.  Step 2 (apply): dz = [r>0]*(a*dy' - b*r + e) -> dz [p][c] and
 * the bias gradient db (written).  With CNNITMO_NO_BN: dz = [r>0]*dy. */
int cnnitmo_bn_bwd_rows(long p, int c);
int cnnitmo_bn_bwd_reduce(int dtype, const void* dy, int dy_ld, int dy_off, const void* r,
                          int r_ld, int r_off, long p, int c, const float* mean,
                          const float* invstd, int flags,
                          uint64_t drop_seed, int drop_layer, float* part, void* stream);
int cnnitmo_bn_bwd_finalize(const float* part, long rows, int c, double count,
                            const float* gamma, const float* mean, const float* invstd,
                            float* dgamma, float* dbeta, float* coef, void* workspace,
                            void* stream);
int cnnitmo_bn_bwd_apply(int dtype, const void* dy, int dy_ld, int dy_off, const void* r,
                         int r_ld, int r_off, long p, int c, const float* coef, int flags,
                         uint64_t drop_seed, int drop_layer, int h, int w, void* dz, float* part,
                         void* stream);
/* r view: (r_ld, r_off).  part columns: [c], or [4][c] by pixel parity with
 * CNNITMO_PARITY (h, w = the spatial size, needed only then). */
/* The same for a BN output that also feeds a MaxPooling2D whose backward was
 * deferred: dy += the pool gradient dy_pool [n][h/2][w/2][c] routed by idx to
 * this pixel (replaces cnnitmo_maxpool2x2_bwd + the dy read-modify-write). */
int cnnitmo_bn_bwd_apply_pooled(int dtype, const void* dy, int dy_ld, int dy_off, const void* r,
                                int r_ld, int r_off, int n, int h, int w, int c, const float* coef,
                                const void* dy_pool, const uint8_t* idx, void* dz, float* part,
                                void* stream);
/* The same for the BN output consumed by the sigmoid head: dy is never stored;
 * dy[p][c] = sum_o g3[p][o] * wh[o][c] is formed in fp32 from the head's per-pixel
 * output gradient g3 [p][3] (cnnitmo_head_fwd_bwd_g3) and its weights wh [3][c]
 * (12 B per pixel read instead of 2*c). */
int cnnitmo_bn_bwd_apply_g3(int dtype, const float* g3, const float* wh, const void* r, int r_ld, int r_off,
                            long p, int c, const float* coef, void* dz, float* part, void* stream);
/* BN-backward sums WITHOUT a pass over dy: for a BN output whose gradient is the
 * input-gradient of a linear consumer (mode 1 conv3x3, 2 tconv2x2, 3 the 1x1
 * head), part[2][c] = {sum dy, sum dy*rhat} over the consumer's input channels
 * [ci0, ci0+c) from its weights w, its uncorrected weight-gradient raw (raw_out of
 * the *_wgrad / head_finalize call) and V (mode 1: db[cout] + border sums
 * vtab[8][cout]; mode 2: parity sums vtab[4*cout]; mode 3: db[3]).  Exact: the
 * dgrad is the transpose of the same map.  Feed to cnnitmo_bn_bwd_finalize.
 * part has CNNITMO_CONSUMER_ROWS rows [rows][2][c].  cnnitmo_pool_bnsums adds a
 * MaxPooling2D consumer's share (dyp: the pooled gradient; r: the pool input's
 * view; rows = cnnitmo_bn_bwd_rows(n*(h/2)*(w/2), c)). */
#define CNNITMO_CONSUMER_ROWS 64
/* The row count the library was built with (== CNNITMO_CONSUMER_ROWS of this header; 16 before
 * cnnitmo_version() 2): size part from this at run time. */
int cnnitmo_consumer_rows(void);
int cnnitmo_bn_consumer_sums(int mode, const float* w, const float* raw, int cout, int cin_tot, int ci0,
                             int c, const float* db, const float* vtab, const float* mean,
                             const float* invstd, float* part, void* stream);
int cnnitmo_pool_bnsums(int dtype, const void* dyp, const uint8_t* idx, int n, int h, int w, int c,
                        const void* r, int r_ld, int r_off, const float* mean, const float* invstd,
                        float* part, void* stream);
/* The same share when the pool was fused into the producer (cnnitmo_conv3x3_fwd_pool):
 * pr [n, h/2, w/2, c] dense is r at each window's index, so no window is read. */
int cnnitmo_pool_bnsums_pooled(int dtype, const void* dyp, const void* pr, int n, int h, int w, int c,
                               const float* mean, const float* invstd, float* part, void* stream);
/* Column sums of partial rows -> out[groups-folded c] (fp32, written). */
int cnnitmo_colsum(const float* part, long rows, int cols, int groups, float* out,
                   void* workspace, void* stream);

/* ---------------------------------------------------------------------------
 * Head: Conv2D(3, 1, activation='sigmoid') + MSE loss + 'accuracy'
 * (model.py:276,281).  x [p][64-ish cin] dtype; w [3][cin] fp32, b [3].
 * fwd: yhat [n,h,w,3] fp32 for rows < h_valid (predict.py:62).
 * fwd_bwd: target [n,h_valid,w,3] fp32; writes dx [p][cin] dtype
 * (= dz * W), and partials (loss sum, correct count, dW, db) into part;
 * cnnitmo_head_finalize reduces them into loss, acc, dw, db.
 * grad_numel: the element count the MSE gradient is normalised by (<= 0: this
 * batch's n*h_valid*w*3, i.e. the gradient of its mean).  Data parallel with
 * unequal shares: global_frames*h_valid*w*3/world, so that the all-reduced mean
 * of the ranks' gradients is the gradient of the GLOBAL batch mean (the loss
 * partials are unaffected). */
int cnnitmo_head_fwd(int dtype, const void* x, int n, int h, int h_valid, int w, int cin,
                     const float* wt, const float* b, const float* scale, const float* shift,
                     float* yhat, void* stream);
int cnnitmo_head_rows(long p);
int cnnitmo_head_fwd_bwd(int dtype, const void* x, int n, int h, int h_valid, int w, int cin,
                         const float* wt, const float* b, const float* scale,
                         const float* shift, const float* target, void* dx, float* part,
                         double grad_numel, void* stream);
/* As cnnitmo_head_fwd_bwd, but the input gradient leaves as its rank-3 factor
 * g3 [p][3] fp32 = dL/dz of the head (dx = g3 * W; see cnnitmo_bn_bwd_apply_g3). */
int cnnitmo_head_fwd_bwd_g3(int dtype, const void* x, int n, int h, int h_valid, int w, int cin,
                            const float* wt, const float* b, const float* scale, const float* shift,
                            const float* target, float* g3, float* part, double grad_numel, void* stream);
int cnnitmo_head_finalize(const float* part, long rows, int cin, double numel,
                          const float* scale, const float* shift, float* loss_acc, float* dw,
                          float* db, float* raw_out, void* workspace, void* stream);
/* scale/shift (nullable, [cin]): x holds r and the head's input is r*scale +
 * shift (folded BN); dx is then d/dy and dw the gradient w.r.t. the raw W. */

/* ---------------------------------------------------------------------------
 * RMSprop (keras.optimizers.RMSprop defaults via compile('rmsprop'), model.py:281):
 *   a <- rho*a + (1-rho)*g'^2 ; p <- p - lr*g'/(sqrt(a)+eps),  g' = g*grad_scale
 * over one flat fp32 buffer holding every trainable tensor (multi-tensor apply).
 */
int cnnitmo_rmsprop(float* p, const float* g, float* a, long n, float lr, float rho, float eps,
                    float grad_scale, void* stream);

/* ---------------------------------------------------------------------------
 * Training-data augmentation -- replaces the paired keras ImageDataGenerator
 * (rescale, rotation_range, horizontal/vertical_flip, zoom_range;
 * /root/reference/main.py:71-77 -> keras_preprocessing apply_transform +
 * standardize).  src [n,h,w,c] uint8 (src_u8 = 1) or fp32; mats [n][6] fp64 =
 * (a00, a01, t0, a10, a11, t1) mapping an output (row, col) to the input
 * (row, col) (transform_matrix_offset_center(rotation @ zoom)); flips [n]
 * (bit 0 horizontal, bit 1 vertical, applied after the affine map); bilinear
 * with clamp-to-edge ('nearest' fill, scipy order 1); dst [n,h,w,c] fp32 =
 * float32(interpolated) * scale.  c = 1 or 3.
 */
int cnnitmo_augment_affine(int src_u8, const void* src, int n, int h, int w, int c, const double* mats,
                           const int* flips, float scale, float* dst, void* stream);

/* ---------------------------------------------------------------------------
 * Dataset generation / HDR reconstruction maps -- replace the reference's
 * MATLAB scripts m-files/Reinhard.m:10-24 (tone mapping of HDR crops into the
 * SDR training inputs), m-files/virtual_camera.m:10-31 (random exposure + camera
 * curve) and m-files/inverse_Reinhard.m:1-23 (SDR -> HDR), float64 arithmetic.
 * Images are NHWC RGB: HDR fp32, SDR uint8.  lum_coef: HOST pointer to the 3
 * luminance weights of RGB2Lum (not in the reference; NULL = Rec. 709).
 *   stats (device, [n][2]) = per image: sum of log(max(f, realmin)) over pixels,
 *   and the count of zero-luminance pixels; f = Y (mode 0, fp32 HDR input) or
 *   X = I/(I-1) (mode 1, uint8 SDR, inverse_Reinhard.m as written).
 *   apply: curve 0 = Reinhard, 1 = virtual camera; params (device, [n][3]) =
 *   (key*2^v, n, y) -- Reinhard uses (0.18, -, -); out fp32 or, out_u8 = 1,
 *   imwrite's uint8(255*x).  inverse: a = the key (0.18); mode 1 = the script
 *   (uint8 sdr, stats of mode 1, g unused); mode 2 = the exact inverse of
 *   Reinhard.m for a linear fp32 sdr and the HDR log-average g (stats unused).
 */
size_t cnnitmo_tonemap_workspace_bytes(int n);
int cnnitmo_tonemap_stats(int mode, const void* img, int n, int h, int w, const double* lum_coef,
                          double* stats, void* workspace, size_t ws_bytes, void* stream);
int cnnitmo_tonemap_apply(int curve, const float* hdr, int n, int h, int w, const double* lum_coef,
                          const double* params, const double* stats, int out_u8, void* out, void* stream);
int cnnitmo_inverse_reinhard_apply(int mode, const void* sdr, int n, int h, int w, const double* lum_coef,
                                   const double* stats, double a, double g, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CNN_ITMO_H_ */
