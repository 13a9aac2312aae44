/*
 * plastic_unet.h - C-ABI of libplastic_unet.so, the MI355X (gfx950) kernels of the plastic U-Net
 * training path.  Plain pointers and sizes only; no torch/HIP types in any signature.
 *
 * The reference (yaricom/Plastic-UNet) is pure Python: its "interface" for this path is the set of
 * ATen operators its nn.Modules call.  Each entry point below names the reference call site(s) it
 * replaces (paths relative to the reference repo):
 *
 *   pu_conv_igemm      nn.Conv2d(k=3,p=1)+ReLU fwd     src/unet/unet_p.py:184-201 (double_conv)
 *                      conv3x3 backward-data           (autograd of the same, train.py:110)
 *                      nn.ConvTranspose2d(2,s=2) fwd   src/unet/unet_p.py:238 (up.up)
 *                      ConvTranspose2d backward-data   (autograd, train.py:110)
 *                      torch.cat([x2,x1],1) (fused)    src/unet/unet_p.py:248
 *   pu_wgrad           conv3x3 / ConvT weight+bias gradients (autograd, train.py:110)
 *   pu_maxpool2_fwd    nn.MaxPool2d(2)                 src/unet/unet_p.py:222 (down.mpconv)
 *   pu_maxpool2_bwd    its backward (+ the ReLU mask of the pooled tensor)
 *   pu_outconv_fwd/bwd nn.Conv2d(C,1,1) (outconv)      src/unet/unet_p.py:253-260
 *   pu_plastic_fwd     activin.mm(w+alpha*hebb), sigmoid, Hebb/Oja trace update
 *                                                      src/unet/unet_p.py:69-88
 *   pu_plastic_head_fwd outconv + activin.mm(w+alpha*hebb) + sigmoid + trace update, ONE launch
 *                                                      src/unet/unet_p.py:67-88
 *   pu_trace_update    the trace update alone          src/unet/unet_p.py:81-86
 *   pu_plastic_bwd     mm/mul/sigmoid backward         (autograd, train.py:110)
 *   pu_bce_fwd/bwd     nn.BCELoss (mean, log >= -100)  src/train.py:70,101-105
 *   pu_adam_multi      torch.optim.Adam.step           src/train.py:66,111
 *   pu_bn_fwd/bwd      nn.BatchNorm2d (+ReLU)          src/unet/unet_p.py:186-193 (batch_norm=True)
 *   pu_upsample_bilinear2x_fwd/bwd  nn.Upsample(2, bilinear, align_corners) unet_p.py:235-236
 *   pu_pack_weight     (layout only) OIHW parameters -> the packed GEMM operands
 *   pu_nchw_to_nhwc    (layout only) the [B,C,H,W] model input -> NHWC
 *
 * Conventions
 *   - Activations are NHWC fp32 in device memory (HBM).  Parameters keep PyTorch's layout (OIHW,
 *     ConvT [in][out][kh][kw]) so state_dicts load both ways; pu_pack_weight makes GEMM operands.
 *   - Ownership: the caller owns every buffer.  The library never allocates or frees device
 *     memory; scratch is passed in as `workspace` (size from the *_workspace_bytes query).
 *   - Streams: `stream` is a hipStream_t (NULL = default stream).  Every call only enqueues work
 *     on that stream; none synchronises, so calls are hipGraph-capturable.
 *   - Errors: 0 on success, a negative pu_status otherwise; pu_last_error() returns a
 *     thread-local message for the last failing call on this thread.
 *   - Threading: stateless and re-entrant; safe from several host threads on different streams.
 */
#ifndef PLASTIC_UNET_H
#define PLASTIC_UNET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PU_ABI_VERSION 3

typedef enum {
    PU_OK = 0,
    PU_ERR_INVALID = -1,     /* bad argument (shape, null pointer, alignment) */
    PU_ERR_UNSUPPORTED = -2, /* valid but not implemented for this shape */
    PU_ERR_LAUNCH = -3,      /* HIP launch error */
    PU_ERR_WORKSPACE = -4    /* workspace too small */
} pu_status;

int pu_abi_version(void);
const char* pu_last_error(void);
/* build id: sha256 prefix over the library sources, this header and the compile flags
 * (plastic-unet_amd/build_native.py); bench lines and profiles/ carry it so a measurement names
 * the exact build it was taken on */
const char* pu_build_id(void);
/* number of compute units and shader clock (kHz) of `device` (for roofline peaks) */
int pu_device_info(int device, int* num_cu, int* clock_khz, long long* hbm_bytes);

/* ---------------------------------------------------------------------------------------------
 * Implicit-GEMM convolution on MFMA (v_mfma_f32_32x32x2_f32):  D[m][n] = sum_k A[m][k] W[n][k]
 *   rows m  = output pixels (batch, out_h, out_w) of the GEMM grid
 *   cols k  = (tap r*kw+s, channel c) of the input at pixel (ho*stride-pad+r, wo*stride-pad+s),
 *             channels [0,c0) read from src0 and [c0,c0+c1) from src1 (concat without a copy)
 *   weight  = packed [n][k_pad] (pu_pack_weight), k_pad >= kh*kw*(c0+c1), k_pad % 16 == 0
 *   cgroup  = K order of the packed weight: 0 -> k = tap*C + c (tap-major);  16 or 32 ->
 *             k = (g*taps + tap)*cgroup + (c % cgroup), g = c / cgroup (channel-group-major: the
 *             taps of one channel group are consecutive K stages, so their shifted re-reads of the
 *             same pixels hit L2).  Requires c0 % cgroup == 0 and c1 % cgroup == 0.
 * Epilogue per element: v = acc (+ bias) (+ resid, RESID) ; RELU: v = max(v,0) ;
 *   mask: v *= (mask > 0) ; ACCUM: dst += v else dst = v.  Columns [0,n0) go to dst0 (NHWC, n0
 *   channels), [n0,n) to dst1 (NHWC, n-n0 channels).  RESID: resid is an NHWC tensor shaped like
 *   dst0 (requires n0 == n, no SHUFFLE2) - the residual add of unet_p_res.py:188 and its backward.
 *   SHUFFLE2: n = (2i+j)*co + c is stored at pixel (2ho+i-shuf_off, 2wo+j-shuf_off) of a
 *   (shuf_h, shuf_w) NHWC grid (0 -> 2*out_h, 2*out_w), co = n/4 channels, bias[c]; pixels
 *   outside the grid are dropped.  ConvTranspose2d 2x2 s2: k=1, shuf_off=0.  ConvTranspose2d 3x3
 *   s2 p0 (+ the crop of row/col 0, unet_p_res.py:207-217): k=2, pad=1, out grid (h+1)x(w+1),
 *   weight packed PU_PACK_CONVT3_FWD, shuf_off = 1 (crop) or 0, shuf_h/w = the kept extent.
 * workspace (optional): when the M x N tile grid cannot fill the chip (small pixel grids: the
 *   8x8 / 16x16 levels of the U-Net) and ws_bytes >= pu_conv_igemm_workspace_bytes(a), K is split
 *   over ksplit blocks per tile; the partial tiles go to the workspace and a second kernel sums
 *   them in fixed split order (deterministic) and runs the epilogue above.  NULL -> no split.
 * ------------------------------------------------------------------------------------------- */
/* PU_CONV_NO_HALO: a dispatch hint, not an epilogue flag - keep a bf16 3x3/s1 layer that the halo
 * kernel would take (width 32/64/128) on the per-tap lean kernel (A/B runs and the bit-identity
 * test: both compute the same sums in the same order when the per-tap launch is not split) */
/* PU_CONV_HALO_DMA: a dispatch hint - take the DMA-ring 512-pixel halo kernel instead of the
 * register-staged 256-pixel one (the default); its sums differ from the per-tap kernel's by at most
 * one bf16 ulp of the output (A/B runs).  PU_CONV_HALO_V1 (the register-staged kernel) is the
 * default and kept as an accepted no-op flag. */
/* PU_CONV_NO_SMALLX6: a dispatch hint - keep an 8/16-channel 3x3 layer on the VALU direct kernel
 * instead of the 16x16x32 MFMA one (A/B runs) */
/* PU_EPI_OUT_BF16: the single-channel stem conv only (c0 == 1, c1 == 0, 3x3 / s1 / p1 same size,
 * n in {8, 16, 32, 64}, no mask / resid / ACCUM / SHUFFLE2 / chan_scale, n0 == n): dst0 is a bf16
 * NHWC tensor and each fp32 result (after bias and ReLU) is rounded to bf16 once, to nearest even -
 * what a separate fp32 -> bf16 conversion of the fp32 output would store (the bf16 trunk's stem,
 * config C3).  Any other call with this flag fails with PU_ERR_INVALID. */
enum { PU_EPI_RELU = 1, PU_EPI_ACCUM = 2, PU_EPI_SHUFFLE2 = 4, PU_EPI_RESID = 8, PU_CONV_NO_HALO = 16,
       PU_CONV_HALO_V1 = 32, PU_CONV_NO_SMALLX6 = 64, PU_CONV_HALO_DMA = 128, PU_EPI_OUT_BF16 = 256 };

typedef struct {
    int batch;
    int in_h, in_w;
    int out_h, out_w;
    int kh, kw, stride, pad;
    const float* src0; int c0;
    const float* src1; int c1;
    const float* weight; int k_pad; int cgroup;
    int n;
    const float* bias;
    float* dst0; int n0;
    float* dst1;
    const float* mask0;
    const float* mask1;
    int flags;
    void* workspace; size_t ws_bytes;
    const float* resid;
    int shuf_h, shuf_w, shuf_off;
    /* optional: `weight` split into bf16 planes by pu_split_weight6.  When set, the MFMA path
     * computes each fp32 product as 6 exact bf16 products (hi/mid/lo terms, fp32 accumulation;
     * dropped terms < 2^-23 relative) on v_mfma_f32_32x32x16_bf16 - 2.7x the fp32-MFMA rate.
     * Layers that take another kernel (small-channel direct, odd channel counts) use `weight`. */
    const void* weight6;
    /* optional: the Winograd F(2x2,3x3) operand U of `weight` (pu_pack_wino; fwd for a forward
     * conv, dgrad for the data gradient).  When set together with weight6, a 3x3/s1/p1 layer on an
     * even same-size grid with 16-channel chunks (c1 == 0 or c1 == c0, c0 + c1 a multiple of 32),
     * n a multiple of 64 and the float4 epilogue runs as 16 element-wise GEMMs over the transformed
     * tiles (2.25x fewer products; same 6-product fp32 arithmetic, fp32 transforms) */
    const void* wino;
    /* optional: per-(image, output channel) factors [batch][chan_scale_ld] (fp32, 16-byte aligned,
     * chan_scale_ld % 4 == 0; 0 -> n, or n/4 under SHUFFLE2).  The epilogue multiplies column n
     * (SHUFFLE2: output channel c) of image b by chan_scale[b * ld + n] after the mask and before
     * ACCUM: the Dropout2d channel scale (unet_p_res.py:62, :69; x * mask / (1 - p)) applied by
     * the conv that produces the tensor instead of a separate pass over it - the same product as
     * pu_channel_scale.  fp32 entry point only (pu_conv_igemm_bf16 rejects it). */
    const float* chan_scale; int chan_scale_ld;
} pu_conv_args;

int pu_conv_igemm(const pu_conv_args* a, void* stream);
/* Winograd operand U = G g G^T of a 3x3 conv weight w[cout][cin][3][3] (fp32, OIHW):
 *   fwd   (dgrad = 0): n = cout output channels, reduced over c = cin
 *   dgrad (dgrad = 1): n = cin, c = cout, g = the flipped kernel w[c][n][2-r][2-s]
 * formed in fp64, rounded to fp32, split exactly into hi/mid/lo bf16 planes, laid out
 * [c/16][16 positions][3 planes][n][16 channels] (pu_wino_bytes(n, c) bytes; c % 16 == 0).
 * All jobs in one launch (re-packed after every optimizer step). */
typedef struct {
    const float* w;
    void* out;
    int cout, cin;
    int dgrad;
} pu_wino_job;
size_t pu_wino_bytes(int n, int c);
int pu_pack_wino(const pu_wino_job* jobs, int n_jobs, void* stream);
/* packed fp32 weight [n][k_pad] -> bf16 planes [k_pad/16][6][n][8] (q = plane*2 + (k%16)/8; plane
 * 0/1/2 = hi/mid/lo, w == hi + mid + lo exactly); out holds n*k_pad*3 bf16 (6 bytes per weight) */
int pu_split_weight6(const float* packed, void* out, int n, int k_pad, void* stream);
/* split-K scratch pu_conv_igemm would use for these arguments (0: no split planned) */
size_t pu_conv_igemm_workspace_bytes(const pu_conv_args* a);
/* the kernel instantiation pu_conv_igemm would launch: block tile bm x bn, A-loader mode
 * (0 = 16-channel chunks, 1 = float4, 2 = scalar, 3 = small-channel direct, 4 = 16-channel
 * chunks on the 6-product bf16 kernel) and K splits (1 = none; counts a->workspace);
 * for profiling/roofline attribution */
int pu_conv_igemm_tile(const pu_conv_args* a, int* bm, int* bn, int* mode, int* ksplit);

/* ---------------------------------------------------------------------------------------------
 * Weight/bias gradient of a convolution as a split-K MFMA GEMM over the B*H*W pixel rows:
 *   dweight[n][c][r][s] = sum_m P[m][n] * X[pix(m,r,s)][c]          (+ accumulate)
 *   P = rows operand [batch*out_h*out_w][n] (conv: dZ;  ConvT: its low-res input x)
 *   X = im2col operand at the (in_h,in_w) grid, channels from src0/src1 as in pu_conv_igemm
 *       (conv: the layer input; ConvT: the high-res output gradient)
 *   bias_mode 1: dbias[n] = sum_m P[m][n]                      (conv bias)
 *   bias_mode 2: dbias[c] = sum_m sum_(r,s) X[pix(m,r,s)][c]   (ConvT bias)
 * Output layout [n][c][kh][kw] is PyTorch's: conv OIHW (n=out, c=in), ConvT [in][out][kh][kw].
 * Deterministic: per-split partials go to `workspace`, then a fixed-order reduction.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    int batch;
    int in_h, in_w;
    int out_h, out_w;
    int kh, kw, stride, pad;
    const float* rows; int n;
    const float* src0; int c0;
    const float* src1; int c1;
    int bias_mode;
    float* dweight;
    float* dbias;
    int accumulate;
    /* fp32 GEMM arithmetic: 0 = v_mfma_f32_32x32x2_f32; 1 = each product as 6 exact bf16 products
     * (hi/mid/lo split of both operands, fp32 accumulation) on v_mfma_f32_32x32x16_bf16;
     * 2 = the single-channel stem (c0 == 1, c1 == 0, 3x3 / s1 / p1 same size, n = 8, 16, 32 or 64,
     * bias_mode 1) with `rows` a bf16 NHWC tensor: each bf16 dZ is widened exactly, so the result is
     * bit-identical to math 1 on the widened fp32 copy (the bf16 trunk's stem, config C3) */
    int math;
} pu_wgrad_args;

size_t pu_wgrad_workspace_bytes(const pu_wgrad_args* a);
/* the tile (bn x bk), loader (qvec: 0 scalar, 1 float4, 2 small-channel direct kernel, 3 halo-reuse kernel,
 * 4 stem kernel, 5 Winograd-domain kernel, 6 pointwise small-channel kernel) and
 * pixel-row split count pu_wgrad would use */
int pu_wgrad_tile(const pu_wgrad_args* a, int* bn, int* bk, int* qvec, int* splits);
int pu_wgrad(const pu_wgrad_args* a, void* workspace, size_t workspace_bytes, void* stream);
/* pu_wgrad in two launches-worth of phases for per-kernel timing: phase 1 = the split-K GEMM
 * (partials into the workspace), phase 2 = the fixed-order reduction + scatter; 1 then 2 on the
 * same stream == pu_wgrad */
int pu_wgrad_phase(const pu_wgrad_args* a, void* workspace, size_t workspace_bytes, int phase, void* stream);

/* ---------------------------------------------------------------------------------------------
 * BatchNorm2d (+ ReLU) of double_conv(batch_norm=True)   src/unet/unet_p.py:186-193
 *   training: slot b is normalised by its own statistics over H x W (the reference trains with
 *   batch size 1) and the running statistics take the B per-slot updates in slot order
 *   (running = (1-m) running + m stat, unbiased variance; NULL running buffers: no update);
 *   save_mean / save_rstd [batch][c].  eval (training = 0): running statistics, save_* [c].
 *   y = relu?((z - mean) * rstd * gamma + beta [+ resid]); gamma / beta may be NULL
 *   (affine=False); resid (optional, NHWC like z): the residual_block add before the ReLU
 *   (unet_p_res.py:188).
 * pu_bn_bwd: given g = dL/dy (ReLU mask applied), dz = (BN backward [+ add]) * (mask > 0) with
 *   add / mask optional, and dgamma / dbeta [c] (NULL: skipped).
 * fp64 partial sums, fixed-order reduction (deterministic).  c % 4 == 0, NHWC, 16-B aligned.
 * ------------------------------------------------------------------------------------------- */
size_t pu_bn_workspace_bytes(int batch, long long hw, int c);
int pu_bn_fwd(const float* z, const float* gamma, const float* beta, float* running_mean, float* running_var,
              float* y, float* save_mean, float* save_rstd, int batch, long long hw, int c, float eps,
              float momentum, int training, int relu, const float* resid, void* workspace,
              size_t workspace_bytes, void* stream);
int pu_bn_bwd(const float* z, const float* g, const float* save_mean, const float* save_rstd,
              const float* gamma, float* dz, float* dgamma, float* dbeta, int batch, long long hw, int c,
              const float* add, const float* mask, void* workspace, size_t workspace_bytes, void* stream);

/* nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True) of up(bilinear=True)
 * src/unet/unet_p.py:235-236, NHWC x [batch][h][w][c] -> y [batch][2h][2w][c]; the backward
 * gathers per input pixel (deterministic) and multiplies by (mask > 0) when mask != NULL. */
int pu_upsample_bilinear2x_fwd(const float* x, float* y, int batch, int h, int w, int c, void* stream);
int pu_upsample_bilinear2x_bwd(const float* dy, const float* mask, float* dx, int batch, int h, int w, int c,
                               void* stream);

/* ---------------------------------------------------------------------------------------------
 * Layout helpers
 * ------------------------------------------------------------------------------------------- */
enum {
    PU_PACK_CONV_FWD = 0,   /* w[O][I][R][S] -> p[o][(r*S+s)*I+i]                          */
    PU_PACK_CONV_DGRAD = 1, /* w[O][I][R][S] -> p[i][((R-1-r)*S+(S-1-s))*O+o] (flipped)    */
    PU_PACK_CONVT_FWD = 2,  /* w[I][O][R][S] -> p[(r*S+s)*O+o][i]                           */
    PU_PACK_CONVT_DGRAD = 3, /* w[I][O][R][S] -> p[i][(r*S+s)*O+o]                          */
    PU_PACK_CONVT3_FWD = 4   /* w[I][O][3][3] -> p[(ph*2+pw)*O+o][(dh*2+dw)*I+i] = w[i][o][R(ph,dh)][R(pw,dw)]
                              * with R(0,1)=0, R(0,0)=2, R(1,1)=1, R(1,0)=none (0): output (2p+ph)
                              * of a 3x3 s2 transposed conv reads input (p-1+dh)               */
};
/* d0,d1 = first two dims of w; rows of p are k_pad floats wide (zero padded).  cgroup != 0 packs
 * the K axis channel-group-major (see pu_conv_args.cgroup) for the FWD/DGRAD/CONVT_DGRAD modes. */
int pu_pack_weight(const float* w, float* packed, int mode, int d0, int d1, int kh, int kw,
                   int k_pad, int cgroup, void* stream);
/* Every packed GEMM operand of a model refreshed in one launch (after an optimizer step): job j
 * packs w like pu_pack_weight(mode, cgroup) into any of packed (fp32 [rows][k_pad]), packed_bf16
 * (bf16 [rows][k_pad]) and planes (the exact 3-term bf16 split of the fp32 packed operand,
 * pu_split_weight6's [k_pad/16][6][rows][8]) - bit-identical to those calls.  k_pad a multiple of 8
 * (16 with planes); outputs 16-byte aligned. */
typedef struct {
    const float* w;
    float* packed;
    void* packed_bf16;
    void* planes;
    int mode, d0, d1, kh, kw, k_pad, cgroup;
} pu_pack_job;
int pu_pack_weights(const pu_pack_job* jobs, int n_jobs, void* stream);
int pu_nchw_to_nhwc(const float* src, float* dst, int batch, int c, int h, int w, void* stream);

/* Dropout2d application (unet_p_res.py:209,248) on NHWC: y[b][p][c] = x[b][p][c] * scale[b][c]
 * (scale 0 or 1/(1-p) per sample and channel); y may alias x.  The backward is the same call on
 * the gradient. */
int pu_channel_scale(const float* x, const float* scale, float* y, int batch, long long hw, int c,
                     void* stream);

/* AddCoords (coord_conv_script.py:69-96) fused with the NCHW -> NHWC input transpose:
 * out[b][i][j] = (x[b][0..c)[i][j], xx_j, yy_i [, rr_ij]) with xx_j = 2j/(h-1) - 1,
 * yy_i = 2i/(w-1) - 1 (the script's x_dim/y_dim roles; square images), rr = sqrt((xx-.5)^2+(yy-.5)^2).
 * out has c + 2 + with_r channels. */
int pu_add_coords(const float* x, float* out, int batch, int c, int h, int w, int with_r, void* stream);

/* Column sums of a row-major [rows][cols] matrix in fp64, fixed order (deterministic):
 * out[c] (+)= sum_r x[r][c].  (ConvTranspose2d 3x3 bias gradient.) */
size_t pu_column_sum_workspace_bytes(long long rows, int cols);
int pu_column_sum(const float* x, long long rows, int cols, float* out, int accumulate,
                  void* workspace, size_t workspace_bytes, void* stream);

/* MaxPool2d(2) on NHWC (floor for odd sizes), first-max tie rule of ATen's CPU kernel.
 * bwd: dx[argmax] (+)= dy * (relu_mask ? (x[argmax] > 0) : 1); dx elsewhere: 0 (or kept if
 * accumulate). */
int pu_maxpool2_fwd(const float* x, float* y, int batch, int h, int w, int c, void* stream);
int pu_maxpool2_bwd(const float* x, const float* dy, float* dx, int batch, int h, int w, int c,
                    int relu_mask, int accumulate, void* stream);
/* The same with the Dropout2d that follows the pool (unet_p_res.py:62, pool_drop): fwd writes
 * maxpool(x) * scale[b][c]; bwd routes dy * scale[b][c] (the dropout's backward) - the products
 * pu_channel_scale computes, without its pass over the pooled tensor.  scale: [batch][c] fp32. */
int pu_maxpool2_fwd_scaled(const float* x, const float* scale, float* y, int batch, int h, int w, int c, void* stream);
int pu_maxpool2_bwd_scaled(const float* x, const float* dy, const float* scale, float* dx, int batch, int h, int w,
                           int c, int relu_mask, int accumulate, void* stream);

/* outconv (1x1, C -> 1): y[m] = b + sum_c x[m][c]*w[c].
 * bwd: dx[m][c] = dy[m]*w[c]*(relu_mask ? x[m][c] > 0 : 1); dw[c] = sum_m dy[m]x[m][c];
 *      db = sum_m dy[m]  (workspace: pu_outconv_workspace_bytes) */
int pu_outconv_fwd(const float* x, const float* w, const float* b, float* y, long long rows, int c,
                   void* stream);
size_t pu_outconv_workspace_bytes(long long rows, int c);
int pu_outconv_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db,
                   long long rows, int c, int relu_mask, void* workspace, size_t workspace_bytes,
                   void* stream);

/* ---------------------------------------------------------------------------------------------
 * bf16 mixed precision (config C3: "same model in bf16, fp32 accumulation").  Activations,
 * gradients of activations, packed weights, masks and residuals are bf16 (void* below); bias,
 * weight gradients, logits and the plastic head stay fp32.  Same argument structs and semantics
 * as the fp32 entry points; v_mfma_f32_32x32x16_bf16 with fp32 accumulation, one rounding to
 * bf16 in each epilogue.
 *   pu_conv_igemm_bf16: channel counts multiple of 32, k_pad multiple of 32, cgroup 0 or 32,
 *                       bias 16-byte aligned fp32.
 *   pu_wgrad_bf16:      rows / src bf16 (channel counts and n multiples of 8), dweight / dbias fp32.
 * ------------------------------------------------------------------------------------------- */
int pu_conv_igemm_bf16(const pu_conv_args* a, void* stream);
size_t pu_conv_igemm_bf16_workspace_bytes(const pu_conv_args* a);
/* the bf16 kernel pu_conv_igemm_bf16 would launch: tile bm x bn, K splits, kind 0 = tile kernel,
 * 1 = lean per-tap kernel, 2 = halo kernel, 3 = row-stream kernel (kind may be NULL) */
int pu_conv_igemm_bf16_tile(const pu_conv_args* a, int* bm, int* bn, int* ksplit, int* kind);
size_t pu_wgrad_bf16_workspace_bytes(const pu_wgrad_args* a);
int pu_wgrad_bf16(const pu_wgrad_args* a, void* workspace, size_t workspace_bytes, void* stream);
int pu_wgrad_bf16_phase(const pu_wgrad_args* a, void* workspace, size_t workspace_bytes, int phase, void* stream);
/* the weight-gradient plan for these arguments: tile (bn x bk), *halo = 1 when the 3x3/s1 halo-reuse
 * kernel runs (64-channel multiples, out_w % 16 == 0), pixel-row splits */
int pu_wgrad_bf16_tile(const pu_wgrad_args* a, int* bn, int* bk, int* halo, int* splits);
int pu_pack_weight_bf16(const float* w, void* packed, int mode, int d0, int d1, int kh, int kw,
                        int k_pad, int cgroup, void* stream);
int pu_convert_f32_bf16(const float* x, void* y, long long n, void* stream);
int pu_convert_bf16_f32(const void* x, float* y, long long n, void* stream);
int pu_maxpool2_fwd_bf16(const void* x, void* y, int batch, int h, int w, int c, void* stream);
int pu_maxpool2_bwd_bf16(const void* x, const void* dy, void* dx, int batch, int h, int w, int c,
                         int relu_mask, int accumulate, void* stream);
int pu_outconv_fwd_bf16(const void* x, const float* w, const float* b, float* y, long long rows, int c,
                        void* stream);
int pu_outconv_bwd_bf16(const void* x, const float* w, const float* dy, void* dx, float* dw, float* db,
                        long long rows, int c, int relu_mask, void* workspace, size_t workspace_bytes,
                        void* stream);

/* ---------------------------------------------------------------------------------------------
 * Plastic head (unet_p.py:69-88), batched over per-slot traces:
 *   Y_b = sigmoid(X_b (w + alpha (.) H_b))
 *   hebb rule (0): H'_b = (1-eta) H_b + eta x0 y0^T ;  oja rule (1): H'_b = H_b + eta (x0 - H_b y0) y0
 *   with x0 = X_b[0,:], y0 = Y_b[0,:]; hebb_out may be NULL (eval: trace not updated).
 * eta is a device pointer (the learnable parameter).  pu_plastic_fwd is ONE launch when hebb_out
 * is a separate buffer (the trace update is fused into the GEMM's epilogue); hebb_out == hebb
 * (in place) takes a second, element-wise launch.  pu_trace_update is the update alone.
 * ------------------------------------------------------------------------------------------- */
enum { PU_RULE_HEBB = 0, PU_RULE_OJA = 1 };

typedef struct {
    int batch, nbf;
    const float* x;
    const float* hebb;
    const float* w;
    const float* alpha;
    const float* eta;
    float* y;
    float* hebb_out;
    int rule;
} pu_plastic_args;

int pu_plastic_fwd(const pu_plastic_args* a, void* stream);
int pu_trace_update(const float* hebb, const float* x, const float* y, const float* eta,
                    float* hebb_out, int batch, int nbf, int rule, void* stream);

/* The fused head of SURVEY 8(b): the 1x1 outconv (unet_p.py:67, 253-260) computed in the head's
 * prologue from the trunk's last activation feat [B][N][N][C] (NHWC, fp32 or bf16 = feat_bf16),
 *   X_b[i][k] = sum_c feat[b][i][k][c] out_w[c] + out_b[0]
 * then Y_b = sigmoid(X_b Weff_b) on v_mfma_f32_16x16x4_f32 (a k-ordered fp32 fma chain) and, when
 * hebb_out != NULL, the trace update of unet_p.py:81-86 - one launch, grid (N/16, B).  x receives
 * the logits X (kept for the backward).  Requires N % 16 == 0, C % 4 == 0, 16-byte aligned feat,
 * hebb_out not aliasing hebb. */
typedef struct {
    int batch, nbf, channels;
    const void* feat;
    int feat_bf16;
    const float* out_w;
    const float* out_b;
    const float* hebb;
    const float* w;
    const float* alpha;
    const float* eta;
    float* x;
    float* y;
    float* hebb_out;
    int rule;
} pu_plastic_head_args;

int pu_plastic_head_fwd(const pu_plastic_head_args* a, void* stream);

/* backward given dy = dL/dY:  G = dy*(1-y)*y ; dx_b = G_b Weff_b^T ;
 *   dw = sum_b X_b^T G_b ; dalpha = sum_b (X_b^T G_b) (.) H_b   (no gradient to eta: S3) */
typedef struct {
    int batch, nbf;
    const float* x;
    const float* hebb;
    const float* w;
    const float* alpha;
    const float* y;
    const float* dy;
    float* dx;
    float* dw;
    float* dalpha;
} pu_plastic_bwd_args;

size_t pu_plastic_bwd_workspace_bytes(int batch, int nbf);
int pu_plastic_bwd(const pu_plastic_bwd_args* a, void* workspace, size_t workspace_bytes,
                   void* stream);

/* BCELoss (mean): loss = mean((t-1)*max(log1p(-y),-100) - t*max(log(y),-100))
 * bwd: dy = g * (y-t) / max((1-y)*y, 1e-12) / n, g = *grad_loss (device scalar) */
size_t pu_bce_workspace_bytes(long long n);
int pu_bce_fwd(const float* y, const float* t, long long n, float* loss, void* workspace,
               size_t workspace_bytes, void* stream);
int pu_bce_bwd(const float* y, const float* t, long long n, const float* grad_loss, float* dy,
               void* stream);

/* ---------------------------------------------------------------------------------------------
 * Multi-tensor Adam (torch.optim.Adam, amsgrad=False, maximize=False):
 *   m = lerp(m, g, 1-beta1) ; v = v*beta2 + (1-beta2) g^2 ;
 *   p -= step_size * m / (sqrt(v)/bc2_sqrt + eps)      (weight_decay adds wd*p to g first)
 * step_size = lr/(1-beta1^t) and bc2_sqrt = sqrt(1-beta2^t) are computed by the caller.  The
 * hyper-parameters are the optimizer's Python doubles: 1-beta1 and 1-beta2 are formed in double and
 * then rounded to fp32, as ATen does with the Scalar arguments of lerp_/addcmul_ (forming 1-beta2
 * from an fp32-rounded beta2 = 0.999 would be 1.3e-5 off).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long long numel;
} pu_adam_tensor;

int pu_adam_multi(const pu_adam_tensor* tensors, int n_tensors, double beta1, double beta2, double eps,
                  double weight_decay, double step_size, double bc2_sqrt, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PLASTIC_UNET_H */
