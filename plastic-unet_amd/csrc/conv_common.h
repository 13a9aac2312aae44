// Types and epilogue helpers shared by the fp32 implicit-GEMM kernels (igemm.hip) and the
// Winograd F(2x2,3x3) kernel (winograd.hip): the launch parameters, the float4 output epilogue
// (bias / residual / ReLU / mask / concat split / accumulate / ConvT shuffle) and the exact
// 3-term bf16 split of fp32 operands.  Epilogue order: bias, residual, ReLU, mask, channel scale,
// accumulate.
#pragma once
#include "common.h"

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct IgemmParams {
    int M, N, K, k_pad;
    int Hi, Wi, Ho, Wo, kh, kw, stride, pad;
    int C, c0, c1;
    const float* src0;
    const float* src1;
    const float* wt;
    const float* bias;
    float* dst0;
    float* dst1;
    const float* mask0;
    const float* mask1;
    int n0, flags;
    int cgroup, taps, gn;   // K order (0 tap-major, 16/32 channel-group-major), kh*kw, n-blocks
    int vec_epi;            // float4 epilogue (channel counts % 4 == 0, 16-byte aligned buffers)
    int ksplit, t_per;      // split-K: blocks per tile and 16-wide K stages per split
    float* part;            // split-K partial tiles [ksplit][M][N]
    const float* resid;     // RESID: NHWC tensor shaped like dst0, added before ReLU / mask
    int shuf_h, shuf_w, shuf_off;   // SHUFFLE2 output grid and crop offset
    FastDiv dWo, dHo, dC, dKw, dCo, dTaps;
    int in_pix;             // batch * Hi * Wi (lean kernel's buffer extent)
    const float* cscale;    // per-(image, channel) factors [batch][cs_ld] or null (chan_scale)
    int cs_ld;
    FastDiv dHW;            // Ho * Wo: the image of GEMM row m
};

// Output position of GEMM row m: the pixel itself, or (SHUFFLE2) the batch row base b*shuf_h and
// the top-left corner (2ho - off, 2wo - off) of its 2x2 output block; b = the image (formed only
// when a channel scale needs it).
struct EpiRow {
    long long pix;
    int oh0, ow0;
    int b;
};

__device__ __forceinline__ EpiRow epi_row(const IgemmParams& p, int m) {
    if (!(p.flags & PU_EPI_SHUFFLE2)) return {m, 0, 0, p.cscale ? (int)fdiv(m, p.dHW) : 0};
    const int t2 = fdiv(m, p.dWo);
    const int wo = m - t2 * p.Wo;
    const int bb = fdiv(t2, p.dHo);
    const int ho = t2 - bb * p.Ho;
    return {(long long)bb * p.shuf_h, 2 * ho - p.shuf_off, 2 * wo - p.shuf_off, bb};
}

// SHUFFLE2 destination element offset of channel n of row r; false if cropped away
__device__ __forceinline__ bool shuf_off(const IgemmParams& p, const EpiRow& r, int n, long long* off, int* c) {
    const int co = p.N >> 2;
    const int ij = fdiv(n, p.dCo);
    *c = n - ij * co;
    const int oh = r.oh0 + (ij >> 1), ow = r.ow0 + (ij & 1);
    if ((unsigned)oh >= (unsigned)p.shuf_h || (unsigned)ow >= (unsigned)p.shuf_w) return false;
    *off = ((r.pix + oh) * p.shuf_w + ow) * co + *c;
    return true;
}

// float4 epilogue of channels n..n+3 (n % 4 == 0, vec_epi) of row r.
__device__ __forceinline__ void epi_store4(const IgemmParams& p, const EpiRow& r, int n, f32x4 v) {
    float* dst;
    const float* msk;
    long long off;
    int nb;   // bias index of the first channel
    const long long pix = r.pix;
    if (p.flags & PU_EPI_SHUFFLE2) {
        if (!shuf_off(p, r, n, &off, &nb)) return;
        dst = p.dst0; msk = p.mask0;
    } else if (n < p.n0) {
        off = pix * p.n0 + n;
        dst = p.dst0; msk = p.mask0; nb = n;
    } else {
        off = pix * (p.N - p.n0) + (n - p.n0);
        dst = p.dst1; msk = p.mask1; nb = n;
    }
    if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + nb);
    if (p.resid) v += *reinterpret_cast<const f32x4*>(p.resid + off);
    if (p.flags & PU_EPI_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (msk) {
        const f32x4 mv = *reinterpret_cast<const f32x4*>(msk + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) if (!(mv[e] > 0.f)) v[e] = 0.f;
    }
    if (p.cscale) v *= *reinterpret_cast<const f32x4*>(p.cscale + (long long)r.b * p.cs_ld + nb);
    if (p.flags & PU_EPI_ACCUM) v += *reinterpret_cast<const f32x4*>(dst + off);
    *reinterpret_cast<f32x4*>(dst + off) = v;
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pk_bf16(f32x2 v) {
    const bf16x2_t h = __builtin_convertvector(v, bf16x2_t);
    return __builtin_bit_cast(unsigned, h);
}

// x = hi + mid + lo exactly (round-to-nearest at each step), 8 elements as 4 pairs
__device__ __forceinline__ void split3_pairs(const f32x4 lo4, const f32x4 hi4, bf16x8_t& h, bf16x8_t& m, bf16x8_t& l) {
#pragma clang fp contract(off)
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 hv, mv, lv;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f32x2 x = q < 2 ? f32x2{lo4[2 * q], lo4[2 * q + 1]} : f32x2{hi4[2 * q - 4], hi4[2 * q - 3]};
        const unsigned a = pk_bf16(x);
        const f32x2 af = {__builtin_bit_cast(float, a << 16), __builtin_bit_cast(float, a & 0xffff0000u)};
        const f32x2 r = x - af;
        const unsigned b = pk_bf16(r);
        const f32x2 bf = {__builtin_bit_cast(float, b << 16), __builtin_bit_cast(float, b & 0xffff0000u)};
        const f32x2 c = r - bf;
        hv[q] = a;
        mv[q] = b;
        lv[q] = pk_bf16(c);
    }
    h = __builtin_bit_cast(bf16x8_t, hv);
    m = __builtin_bit_cast(bf16x8_t, mv);
    l = __builtin_bit_cast(bf16x8_t, lv);
}

// Winograd F(2x2,3x3) path (winograd.hip), dispatched from pu_conv_igemm
bool wino_ok(const pu_conv_args* a, bool vec_epi);
size_t wino_workspace_bytes(const pu_conv_args* a);
int wino_launch(const pu_conv_args* a, IgemmParams p, hipStream_t s);   // returns its K splits
int wino_item_channels(const pu_conv_args* a);   // output channels per Winograd item (64 or 128)
// 8/16-channel 3x3 convolutions on 16x16x32 bf16 MFMAs (smallconv.hip)
bool smallx6_ok(const pu_conv_args* a, bool vec_epi);
int smallx6_launch(const pu_conv_args* a, const IgemmParams& p, hipStream_t s);

}  // namespace pu
