// 3x3/s1/p1 convolutions with 8 or 16 input and output channels (the 8/16-channel levels of
// configs C4 / C5: coord_conv_script.py:155-192, unet_p_res.py:142-189), forward and data
// gradient, on the exact 6-product bf16 MFMA scheme of the other fp32 convolutions
// (v_mfma_f32_16x16x32_bf16: each fp32 product as hi/mid/lo bf16 terms, fp32 accumulation).
//
// The VALU direct kernel (igemm.hip smallconv_kernel) issued ~38 TFLOP/s on these layers - far
// from the HBM bound they have (18-36 FLOP/B).  Here a block stages the (16+2) x (32+2) input halo
// of a 16 x 32 output tile ONCE, split into bf16 planes in LDS (both concat sources, zero
// padding), and every tap reads its shifted 16-pixel windows from that image:
//   GEMM  D[n][pixel] = sum_k W[n][k] X[k][pixel],  k = tap * C + c (the packed weight's order)
//   A = the weights (16 rows n; rows >= N are zero), held in registers as split planes for the
//       whole block (K padded to 32: 3 k-steps for C = 8, 5 for C = 16; padded k are zero);
//   B = 16 consecutive output pixels of one row x 32 k: lane (pixel j, k-group g) reads 8 channels
//       of one tap at halo pixel (row + r, col + j + s) - one conflict-free ds_read_b128 per plane
//       (channel halves of C = 16 are separate LDS images so 16 lanes read 256 contiguous bytes);
//   D (16 x 16, 4 registers): lane holds 4 consecutive channels of one pixel -> igemm's float4
//       epilogue (bias, residual, ReLU, masks, concat split, accumulate).
// Each wave owns 4 output rows x 32 pixels = 8 groups of 16 pixels: 8 accumulators of 4 registers.
//
// Row pairs (N = 8, the default; PU_SX_PAIR=0 disables): with 8 output channels rows 8..15 of A
// were zero - half of every MFMA wasted - and K = 9C was padded to a multiple of 32.  Instead a
// group covers TWO output rows y, y+1 of 16 pixels: k runs over 12 "super-taps" (input rows
// y-1 .. y+2 x 3 columns) x C channels (96 / 192 = exactly 3 / 6 k-steps), A row n < 8 holds
// W[n][dy][dx] for super-tap (dy, dx) (zero for dy = 3), row 8 + n holds W[n][dy-1][dx] (zero
// for dy = 0), so D rows 0..7 are output row y and rows 8..15 output row y+1: the MFMAs per
// output pixel halve (C = 8) or drop 40 % (C = 16), and every lane stores in the epilogue.
#include "conv_common.h"

namespace pu {

constexpr int SX_TW = 32;                            // output tile width
// output tile height: 16 rows for C = 8 (29 KB of split halo images, 5 blocks per CU); 8 rows for
// C = 16, whose 16-row images (59 KB) held the kernel to 2 blocks per CU - at 33 KB it runs 4
// (PU_SX16_TH=16 restores the 16-row tile for A/B runs)
#ifndef PU_SX16_TH
#define PU_SX16_TH 8
#endif
#ifndef PU_SX_PAIR
#define PU_SX_PAIR 1
#endif
// stride 2 (S = 2: the 3x3 / s2 data gradient of the ConvTranspose2d of unet_p_res.py:207-217 at
// the 8-channel level): 4-row tiles, the halo spans (2 * 4 + 1) x (2 * 32 + 1) input pixels (28 KB)
// KT = 2 (2 x 2 taps, N = 32: the ConvTranspose2d 3x3 / s2 forward of the 16-channel level as its
// 2 x 2 sub-pixel conv, unet_p_res.py:207-217, stored through the SHUFFLE2 epilogue)
template <int C, int S = 1> constexpr int sx_th() { return S == 2 ? 4 : C == 8 ? 16 : PU_SX16_TH; }
template <int S, int KT = 3> constexpr int sx_hw() { return (SX_TW - 1) * S + KT; }       // halo width 34 / 65 / 33
template <int C, int S = 1, int KT = 3> constexpr int sx_hp() {                          // halo pixels
    return ((sx_th<C, S>() - 1) * S + KT) * sx_hw<S, KT>();
}

typedef __bf16 bf16x8s __attribute__((ext_vector_type(8)));
typedef float f32x4s __attribute__((ext_vector_type(4)));

// One block per tile.  LDS allows 4-5 blocks per CU (29 / 33 KB): waves_per_eu(4) lets the compiler
// use 128 registers instead of squeezing into 64 with the accumulators parked in AGPRs (320 accvgpr
// moves per wave at C = 8)
template <int C, int N, int S = 1, int KT = 3>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sx_th<C>() == 16 && C == 16 ? 2 : 4))) void smallconv_x6_kernel(const IgemmParams p) {
#pragma clang fp contract(off)
    constexpr int SX_TH = sx_th<C, S>(), SX_HP = sx_hp<C, S, KT>(), SX_HW = sx_hw<S, KT>();
    constexpr bool PAIR = PU_SX_PAIR && N == 8 && S == 1 && KT == 3;   // two output rows per group (header)
    constexpr int NB = (N + 15) / 16;               // 16-row blocks of A (N = 32: two)
    constexpr int TAPS = KT * KT;
    constexpr int RPW = SX_TH / 4;                  // output rows per wave
    constexpr int GR = PAIR ? RPW : 2 * RPW;        // groups (16 pixels x 1 or 2 rows) per wave
    constexpr int HALVES = C / 8;                   // 8-channel LDS images per plane
    constexpr int KS = PAIR ? 12 * C / 32 : (TAPS * C + 31) / 32;   // 32-wide k steps
    static_assert(!PAIR || RPW % 2 == 0, "row pairs need an even number of rows per wave");
    // [plane][half][pixel][8 channels] bf16
    __shared__ __attribute__((aligned(16))) __bf16 img[3 * HALVES * SX_HP * 8];

    const int tiles_w = (p.Wo + SX_TW - 1) / SX_TW;
    const int tiles_h = (p.Ho + SX_TH - 1) / SX_TH;
    int blk = blockIdx.x;
    const int txi = blk % tiles_w;
    blk /= tiles_w;
    const int tyi = blk % tiles_h;
    const int b = blk / tiles_h;
    const int y0 = tyi * SX_TH * S - p.pad, x0 = txi * SX_TW * S - p.pad;   // halo origin
    const long long imgpix = (long long)b * p.Hi * p.Wi;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;

    // ---- weights: lane (row n = lane & 15, k-group g = lane >> 4) holds k = 32s + 8g .. +7 of
    // every step s as hi/mid/lo planes (rows >= N and k >= 9C are zero)
    bf16x8s wa[NB][KS][3];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        const int n = 16 * nb + (lane & 15), g = lane >> 4;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            f32x4s lo = {0.f, 0.f, 0.f, 0.f}, hi = {0.f, 0.f, 0.f, 0.f};
            const int k = 32 * s + 8 * g;
            if (PAIR) {                    // super-tap (dy, dx) of output row y + (n >> 3)
                const int st = k / C, dy = st / 3 - (n >> 3), wk = (dy * 3 + st % 3) * C + k % C;
                if (dy >= 0 && dy <= 2) {
                    lo = *reinterpret_cast<const f32x4s*>(p.wt + (n & 7) * p.k_pad + wk);
                    hi = *reinterpret_cast<const f32x4s*>(p.wt + (n & 7) * p.k_pad + wk + 4);
                }
            } else if (n < N && k < TAPS * C) {   // TAPS*C is a multiple of 8: the 8 k are all real or all padding
                lo = *reinterpret_cast<const f32x4s*>(p.wt + n * p.k_pad + k);
                hi = *reinterpret_cast<const f32x4s*>(p.wt + n * p.k_pad + k + 4);
            }
            split3_pairs(lo, hi, wa[nb][s][0], wa[nb][s][1], wa[nb][s][2]);
        }
    }

    // ---- stage the halo, split once: float4 e = (pixel, channel quad) of one of the sources
    {
        constexpr int Q = C / 4;
        constexpr int NE = SX_HP * Q;
        constexpr int PT = (NE + 511) / 512;        // pairs of float4 per thread
        f32x4s v[PT][2];
#pragma unroll
        for (int it = 0; it < PT; ++it)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = (it * 2 + u) * 256 + tid;
                const int q = e % Q, pix = e / Q;
                const int hx = pix % SX_HW, hy = pix / SX_HW;
                const int gy = y0 + hy, gx = x0 + hx;
                v[it][u] = f32x4s{0.f, 0.f, 0.f, 0.f};
                if (e < NE && (unsigned)gy < (unsigned)p.Hi && (unsigned)gx < (unsigned)p.Wi) {
                    const long long px = imgpix + (long long)gy * p.Wi + gx;
                    const int c = 4 * q;
                    v[it][u] = c < p.c0 ? *reinterpret_cast<const f32x4s*>(p.src0 + px * p.c0 + c)
                                        : *reinterpret_cast<const f32x4s*>(p.src1 + px * p.c1 + (c - p.c0));
                }
            }
#pragma unroll
        for (int it = 0; it < PT; ++it) {
            bf16x8_t h, m, l;
            split3_pairs(v[it][0], v[it][1], h, m, l);
            typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
            typedef unsigned u32x2s __attribute__((ext_vector_type(2)));
            const u32x4s pv[3] = {__builtin_bit_cast(u32x4s, h), __builtin_bit_cast(u32x4s, m), __builtin_bit_cast(u32x4s, l)};
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = (it * 2 + u) * 256 + tid;
                if (e >= NE) continue;
                const int q = e % Q, pix = e / Q;
                const int half = q >> 1, sub = q & 1;
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    *reinterpret_cast<u32x2s*>(img + ((pl * HALVES + half) * SX_HP + pix) * 8 + sub * 4) =
                        u32x2s{pv[pl][2 * u], pv[pl][2 * u + 1]};
            }
        }
    }
    __syncthreads();

    // ---- MFMAs: wave w owns output rows RPW w .. RPW w + RPW-1, each 2 groups of 16 pixels
    const int j = lane & 15, g = lane >> 4;
    f32x4s acc[GR][NB];
#pragma unroll
    for (int t = 0; t < GR; ++t)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[t][nb] = f32x4s{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int k = 32 * s + 8 * g;               // this lane's 8 k: one (super-)tap, 8 channels
        const int tap = k / C, c8 = (k % C) / 8;
        const bool live = PAIR || tap < TAPS;
        const int r = live ? tap / KT : 0, sx = live ? tap % KT : 0;
#pragma unroll
        for (int t = 0; t < GR; ++t) {
            const int row = RPW * wave + (PAIR ? 2 * (t >> 1) : t >> 1), col = (t & 1) * 16 + j;
            const int hp = (row * S + r) * SX_HW + col * S + sx;
            // k past TAPS*C reads tap 0's window: finite values against zero weight planes
            bf16x8s xb[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                xb[pl] = *reinterpret_cast<const bf16x8s*>(img + ((pl * HALVES + c8) * SX_HP + hp) * 8);
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                f32x4s c = acc[t][nb];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nb][s][1], xb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nb][s][2], xb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nb][s][0], xb[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nb][s][1], xb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nb][s][0], xb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[nb][s][0], xb[0], c, 0, 0, 0);
                acc[t][nb] = c;
            }
        }
    }

    // ---- epilogue: lane holds channels 4g .. 4g+3 of pixel (row, col); row pairs: channels
    // 4 (g & 1) .. +3 of row + (g >> 1)
    if (!PAIR && 4 * g >= N) return;
#pragma unroll
    for (int t = 0; t < GR; ++t) {
        const int oy = tyi * SX_TH + RPW * wave + (PAIR ? 2 * (t >> 1) + (g >> 1) : t >> 1);
        const int ox = txi * SX_TW + (t & 1) * 16 + j;
        if (oy >= p.Ho || ox >= p.Wo) continue;
        const int m = (b * p.Ho + oy) * p.Wo + ox;
        const EpiRow er = epi_row(p, m);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) epi_store4(p, er, 16 * nb + (PAIR ? 4 * (g & 1) : 4 * g), acc[t][nb]);
    }
}

// C in {8, 16} from one source or two 8-channel-aligned ones, N in {8, 16}, 3x3 / s1 / p1 same
// size - or C = 8 from one source at stride 2, pad 0 / 1 (the ConvT data gradient) - tap-major fp32
// weight rows (k_pad = 9C rounded to 16), float4 epilogue, no ConvT shuffle; or the ConvT forward's
// 2 x 2 / p1 sub-pixel conv of 16 channels into N = 32 (4 x 8 channels, SHUFFLE2)
static bool smallx6_convt_ok(const pu_conv_args* a, bool vec_epi) {
    return !(a->flags & PU_CONV_NO_SMALLX6) && a->weight6 && a->c0 == 16 && a->c1 == 0 && a->n == 32 &&
           a->kh == 2 && a->kw == 2 && a->stride == 1 && a->pad == 1 && a->out_h == a->in_h + 1 &&
           a->out_w == a->in_w + 1 && (a->flags & PU_EPI_SHUFFLE2) && vec_epi && a->cgroup == 0 && a->k_pad == 64;
}

bool smallx6_ok(const pu_conv_args* a, bool vec_epi) {
    if (smallx6_convt_ok(a, vec_epi)) return true;
    const int C = a->c0 + a->c1;
    const bool s1 = a->stride == 1 && a->pad == 1 && a->in_h == a->out_h && a->in_w == a->out_w;
    const bool s2 = a->stride == 2 && (a->pad == 0 || a->pad == 1) && C == 8 && a->c1 == 0 &&
                    2 * (a->out_h - 1) + 3 - a->pad <= a->in_h + a->pad && 2 * (a->out_w - 1) + 3 - a->pad <= a->in_w + a->pad;
    return !(a->flags & PU_CONV_NO_SMALLX6) && a->weight6 && (C == 8 || C == 16) && (a->n == 8 || a->n == 16) && a->c0 % 8 == 0 &&
           a->c1 % 8 == 0 && a->kh == 3 && a->kw == 3 && (s1 || s2) && !(a->flags & PU_EPI_SHUFFLE2) && vec_epi &&
           (a->cgroup == 0 || a->cgroup >= C) && a->k_pad == (9 * C + 15) / 16 * 16;
}

int smallx6_launch(const pu_conv_args* a, const IgemmParams& p, hipStream_t s) {
    const int C = a->c0 + a->c1;
    const int th = a->stride == 2 ? sx_th<8, 2>() : C == 8 ? sx_th<8>() : sx_th<16>();
    const dim3 grid((unsigned)(((a->out_w + SX_TW - 1) / SX_TW) * ((a->out_h + th - 1) / th) * a->batch));
    if (a->kh == 2) {
        hipLaunchKernelGGL((smallconv_x6_kernel<16, 32, 1, 2>), grid, dim3(256), 0, s, p);
        return check_launch("pu_conv_igemm (small-channel x6, ConvT 2x2 sub-pixel)");
    }
    if (a->stride == 2) {
        if (a->n == 8) hipLaunchKernelGGL((smallconv_x6_kernel<8, 8, 2>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((smallconv_x6_kernel<8, 16, 2>), grid, dim3(256), 0, s, p);
        return check_launch("pu_conv_igemm (small-channel x6, stride 2)");
    }
    if (C == 8 && a->n == 8) hipLaunchKernelGGL((smallconv_x6_kernel<8, 8>), grid, dim3(256), 0, s, p);
    else if (C == 8) hipLaunchKernelGGL((smallconv_x6_kernel<8, 16>), grid, dim3(256), 0, s, p);
    else if (a->n == 8) hipLaunchKernelGGL((smallconv_x6_kernel<16, 8>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((smallconv_x6_kernel<16, 16>), grid, dim3(256), 0, s, p);
    return check_launch("pu_conv_igemm (small-channel x6)");
}

}  // namespace pu
