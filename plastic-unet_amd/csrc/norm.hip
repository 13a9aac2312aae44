// BatchNorm2d (+ ReLU) and the bilinear 2x upsample of the UNetp variants, NHWC fp32.
//
// Reference (yaricom/Plastic-UNet): double_conv with batch_norm=True, src/unet/unet_p.py:186-193
// (Conv2d -> BatchNorm2d -> ReLU, twice), and up with bilinear=True, unet_p.py:235-236
// (nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True)); backward = what
// loss.backward() (src/train.py:110) runs through ATen on the CPU.
//
// BatchNorm semantics of the batched build: the reference trains with batch size 1,
// so each slot b is normalised by ITS OWN statistics over H x W (what BatchNorm2d computes for a
// [1,C,H,W] input), and the running statistics receive the B per-slot updates in slot order
// (running = (1-m) running + m stat_b, unbiased variance), exactly B sequential reference steps.
// Eval mode normalises with the running statistics.  Sums are fp64 (ATen's CPU accumulation
// type for float), partial per (split, slot, channel) and reduced in fixed order: deterministic.
#include "common.h"

#include <math.h>

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BN_SPLITS_MAX = 64;

// per-(split, slot, channel) partial sums over the split's pixel range:
//   MODE 0: (sum x, sum x^2)            MODE 1: (sum g, sum (x - mean) g)
// grid (ceil(C / CC), S, B); thread = (channel lane c = t % CC, pixel lane t / CC)
template <int MODE>
__global__ __launch_bounds__(256) void bn_partial_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                         const float* __restrict__ mean, int B, long long hw, int C,
                                                         int CC, int S, double* __restrict__ part) {
    __shared__ double red[2][256];
    const int tid = threadIdx.x;
    const int PL = 256 / CC;
    const int cl = tid % CC, pl = tid / CC;
    const int c = blockIdx.x * CC + cl;
    const int s = blockIdx.y, b = blockIdx.z;
    const long long per = (hw + S - 1) / S;
    const long long p0 = s * per, p1 = min(hw, p0 + per);
    double a0 = 0.0, a1 = 0.0;
    if (pl < PL && c < C) {
        const float* xb = x + (long long)b * hw * C + c;
        const float* gb = MODE == 1 ? g + (long long)b * hw * C + c : nullptr;
        const float mu = MODE == 1 ? mean[(long long)b * C + c] : 0.f;
        for (long long p = p0 + pl; p < p1; p += PL) {
            const float v = xb[p * C];
            if (MODE == 0) {
                a0 += (double)v;
                a1 += (double)v * (double)v;
            } else {
                const float gv = gb[p * C];
                a0 += (double)gv;
                a1 += ((double)v - (double)mu) * (double)gv;
            }
        }
    }
    red[0][tid] = a0;
    red[1][tid] = a1;
    __syncthreads();
    if (pl == 0 && c < C) {
        for (int q = 1; q < PL; ++q) {
            a0 += red[0][q * CC + cl];
            a1 += red[1][q * CC + cl];
        }
        double* o = part + (((long long)s * B + b) * C + c) * 2;
        o[0] = a0;
        o[1] = a1;
    }
}

// statistics: mean / rstd per (slot, channel) and the running-statistic updates in slot order.
// one thread per channel
__global__ void bn_stats_finalize_kernel(const double* __restrict__ part, int S, int B, int C, long long hw,
                                         float eps, float momentum, float* __restrict__ save_mean,
                                         float* __restrict__ save_rstd, float* __restrict__ running_mean,
                                         float* __restrict__ running_var) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double n = (double)hw;
    double rm = running_mean ? (double)running_mean[c] : 0.0;
    double rv = running_var ? (double)running_var[c] : 0.0;
    for (int b = 0; b < B; ++b) {
        double s0 = 0.0, s1 = 0.0;
        for (int s = 0; s < S; ++s) {
            const double* o = part + (((long long)s * B + b) * C + c) * 2;
            s0 += o[0];
            s1 += o[1];
        }
        const double mu = s0 / n;
        double var = s1 / n - mu * mu;     // biased (the normalisation); fp64 sums
        if (var < 0.0) var = 0.0;
        save_mean[(long long)b * C + c] = (float)mu;
        save_rstd[(long long)b * C + c] = (float)(1.0 / sqrt(var + (double)eps));
        if (running_mean) {
            // ATen: running = momentum * stat + (1 - momentum) * running, unbiased variance
            rm = (double)(float)(momentum * mu + (1.0 - momentum) * rm);
            const double unb = hw > 1 ? var * n / (n - 1.0) : var;
            rv = (double)(float)(momentum * unb + (1.0 - momentum) * rv);
        }
    }
    if (running_mean) {
        running_mean[c] = (float)rm;
        running_var[c] = (float)rv;
    }
}

// y = relu?(z * a + b), a = rstd * gamma, b = beta - mean * a; per (slot, channel) mean/rstd
// (stat_stride = C) or per channel (eval: stat_stride = 0, from the running statistics)
__global__ void bn_apply_kernel(const float* __restrict__ z, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ resid,
                                float* __restrict__ y, long long hw, int C, int stat_stride, long long total4,
                                int relu) {
#pragma clang fp contract(off)
    const int C4 = C >> 2;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total4;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C4) * 4;
        const long long b = i / C4 / hw;
        const float* mu = mean + b * stat_stride + c;
        const float* rs = rstd + b * stat_stride + c;
        f32x4 v = reinterpret_cast<const f32x4*>(z)[i];
        const f32x4 rv = resid ? reinterpret_cast<const f32x4*>(resid)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float a = rs[e] * (gamma ? gamma[c + e] : 1.f);
            const float bb = (beta ? beta[c + e] : 0.f) - mu[e] * a;
            float o = v[e] * a + bb;
            if (resid) o = o + rv[e];         // residual_block: BN output + relu(input) (unet_p_res.py:188)
            if (relu) o = fmaxf(o, 0.f);
            v[e] = o;
        }
        reinterpret_cast<f32x4*>(y)[i] = v;
    }
}

// eval-mode statistics from the running buffers: mean = running_mean, rstd = 1/sqrt(var + eps)
__global__ void bn_eval_stats_kernel(const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                     int C, float* __restrict__ mean, float* __restrict__ rstd) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    mean[c] = rm[c];
    rstd[c] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
}

// backward coefficients per (slot, channel): gm = sum g / n, k = dotp * rstd^2 / n;
// dgamma = sum_b dotp * rstd, dbeta = sum_b sum g (slot order).  one thread per channel
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ part, int S, int B, int C, long long hw,
                                       const float* __restrict__ rstd, float* __restrict__ coef,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double n = (double)hw;
    double dg = 0.0, db = 0.0;
    for (int b = 0; b < B; ++b) {
        double s0 = 0.0, s1 = 0.0;
        for (int s = 0; s < S; ++s) {
            const double* o = part + (((long long)s * B + b) * C + c) * 2;
            s0 += o[0];
            s1 += o[1];
        }
        const double r = (double)rstd[(long long)b * C + c];
        coef[((long long)b * C + c) * 2] = (float)(s0 / n);
        coef[((long long)b * C + c) * 2 + 1] = (float)(s1 * r * r / n);
        dg += s1 * r;
        db += s0;
    }
    if (dgamma) dgamma[c] = (float)dg;
    if (dbeta) dbeta[c] = (float)db;
}

// dz = (g - gm - (z - mean) k) * rstd * gamma
__global__ void bn_bwd_apply_kernel(const float* __restrict__ z, const float* __restrict__ g,
                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                    const float* __restrict__ coef, const float* __restrict__ gamma,
                                    const float* __restrict__ add, const float* __restrict__ mask,
                                    float* __restrict__ dz, long long hw, int C, long long total4) {
#pragma clang fp contract(off)
    const int C4 = C >> 2;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total4;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C4) * 4;
        const long long b = i / C4 / hw;
        const f32x4 zv = reinterpret_cast<const f32x4*>(z)[i];
        const f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const long long bc = b * C + c + e;
            const float gm = coef[bc * 2], k = coef[bc * 2 + 1];
            const float xm = (zv[e] - mean[bc]) * k;
            o[e] = (gv[e] - gm - xm) * rstd[bc] * (gamma ? gamma[c + e] : 1.f);
        }
        if (add) {
            const f32x4 av = reinterpret_cast<const f32x4*>(add)[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = o[e] + av[e];
        }
        if (mask) {
            const f32x4 mv = reinterpret_cast<const f32x4*>(mask)[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) if (!(mv[e] > 0.f)) o[e] = 0.f;
        }
        reinterpret_cast<f32x4*>(dz)[i] = o;
    }
}

// ------------------------------------------------------------------------- bilinear upsample 2x
// align_corners=True: source coordinate of output o is o * (in - 1) / (out - 1) (ATen's
// area_pixel_compute_scale / source_index in fp32), i0 = floor, i1 = i0 + (i0 < in - 1),
// weights (1 - l, l).
struct Lin {
    int i0, i1;
    float l0, l1;
};

__device__ __forceinline__ Lin lin_src(int o, int in, int out) {
    const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
    const float real = scale * (float)o;
    const int i0 = (int)real;
    const int i1 = i0 + (i0 < in - 1 ? 1 : 0);
    const float l1 = real - (float)i0;
    return {i0, i1, 1.f - l1, l1};
}

// y[b][oh][ow][c] = l0h (l0w x[h0][w0] + l1w x[h0][w1]) + l1h (l0w x[h1][w0] + l1w x[h1][w1])
__global__ void upsample_bilinear2x_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int h, int w,
                                               int C, long long total4) {
#pragma clang fp contract(off)
    const int C4 = C >> 2, H2 = 2 * h, W2 = 2 * w;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total4;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C4) * 4;
        long long r = i / C4;
        const int ow = (int)(r % W2);
        r /= W2;
        const int oh = (int)(r % H2);
        const long long b = r / H2;
        const Lin lh = lin_src(oh, h, H2), lw = lin_src(ow, w, W2);
        const float* xb = x + b * h * w * C + c;
        const f32x4 x00 = *reinterpret_cast<const f32x4*>(xb + ((long long)lh.i0 * w + lw.i0) * C);
        const f32x4 x01 = *reinterpret_cast<const f32x4*>(xb + ((long long)lh.i0 * w + lw.i1) * C);
        const f32x4 x10 = *reinterpret_cast<const f32x4*>(xb + ((long long)lh.i1 * w + lw.i0) * C);
        const f32x4 x11 = *reinterpret_cast<const f32x4*>(xb + ((long long)lh.i1 * w + lw.i1) * C);
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            o[e] = lh.l0 * (lw.l0 * x00[e] + lw.l1 * x01[e]) + lh.l1 * (lw.l0 * x10[e] + lw.l1 * x11[e]);
        reinterpret_cast<f32x4*>(y)[i] = o;
    }
}

// weight of input index p in output o along one axis (0 if o does not read p)
__device__ __forceinline__ float lin_weight(int o, int p, int in, int out) {
    const Lin l = lin_src(o, in, out);
    float wgt = 0.f;
    if (l.i0 == p) wgt += l.l0;
    if (l.i1 == p) wgt += l.l1;
    return wgt;
}

// dx[b][p][q][c] = sum over the outputs that read (p, q) of their weights x dy, gathered per input
// pixel (deterministic, no atomics); outputs reading p lie in [2p - 2, 2p + 2] (scale < 1/2 + ...)
// clipped to the grid.  mask: dx *= (mask > 0) (the ReLU of the upsampled activation)
__global__ void upsample_bilinear2x_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ mask,
                                               float* __restrict__ dx, int h, int w, int C, long long total4) {
#pragma clang fp contract(off)
    const int C4 = C >> 2, H2 = 2 * h, W2 = 2 * w;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total4;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C4) * 4;
        long long r = i / C4;
        const int q = (int)(r % w);
        r /= w;
        const int p = (int)(r % h);
        const long long b = r / h;
        const float* db = dy + b * (long long)H2 * W2 * C + c;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int oh = max(0, 2 * p - 2); oh <= min(H2 - 1, 2 * p + 2); ++oh) {
            const float wh = lin_weight(oh, p, h, H2);
            if (wh == 0.f) continue;
            for (int ow = max(0, 2 * q - 2); ow <= min(W2 - 1, 2 * q + 2); ++ow) {
                const float ww = lin_weight(ow, q, w, W2);
                if (ww == 0.f) continue;
                const f32x4 g = *reinterpret_cast<const f32x4*>(db + ((long long)oh * W2 + ow) * C);
                const float wt = wh * ww;
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] += wt * g[e];
            }
        }
        if (mask) {
            const f32x4 m = reinterpret_cast<const f32x4*>(mask)[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) if (!(m[e] > 0.f)) acc[e] = 0.f;
        }
        reinterpret_cast<f32x4*>(dx)[i] = acc;
    }
}

static int ew_grid(long long n) {
    long long g = (n + 255) / 256;
    if (g > 16384) g = 16384;
    return g < 1 ? 1 : (int)g;
}

struct BnPlan {
    int CC, S;
};

static BnPlan bn_plan(int B, long long hw, int C) {
    BnPlan pl;
    pl.CC = C < 64 ? C : 64;
    const long long cblocks = (C + pl.CC - 1) / pl.CC;
    // enough blocks to fill the chip (>= ~1024), each split >= 256 pixels
    long long s = 1024 / (cblocks * B);
    const long long smax = hw / 256;
    if (s > smax) s = smax;
    if (s > BN_SPLITS_MAX) s = BN_SPLITS_MAX;
    pl.S = s < 1 ? 1 : (int)s;
    return pl;
}

}  // namespace pu

using namespace pu;

extern "C" size_t pu_bn_workspace_bytes(int batch, long long hw, int c) {
    if (batch <= 0 || hw <= 0 || c <= 0) return 0;
    const BnPlan pl = bn_plan(batch, hw, c);
    // partials [S][B][C][2] fp64 + backward coefficients [B][C][2] fp32
    return (size_t)pl.S * batch * c * 2 * sizeof(double) + (size_t)batch * c * 2 * sizeof(float);
}

extern "C" int pu_bn_fwd(const float* z, const float* gamma, const float* beta, float* running_mean,
                         float* running_var, float* y, float* save_mean, float* save_rstd, int batch, long long hw,
                         int c, float eps, float momentum, int training, int relu, const float* resid,
                         void* workspace, size_t ws_bytes, void* stream) {
    PU_REQUIRE(z && y && save_mean && save_rstd && batch > 0 && hw > 0 && c > 0, "pu_bn_fwd: bad args");
    PU_REQUIRE(c % 4 == 0 && (((uintptr_t)z | (uintptr_t)y | (uintptr_t)resid) & 15) == 0,
               "pu_bn_fwd: channels %% 4, 16-byte alignment");
    PU_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "pu_bn_fwd: running buffers go together");
    hipStream_t s = as_stream(stream);
    const long long total4 = (long long)batch * hw * c / 4;
    if (!training) {
        PU_REQUIRE(running_mean, "pu_bn_fwd: eval mode needs the running statistics");
        hipLaunchKernelGGL(bn_eval_stats_kernel, dim3((c + 255) / 256), dim3(256), 0, s, running_mean, running_var, eps, c,
                           save_mean, save_rstd);
        hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(total4)), dim3(256), 0, s, z, save_mean, save_rstd, gamma, beta,
                           resid, y, hw, c, 0, total4, relu);
        return check_launch("pu_bn_fwd (eval)");
    }
    const BnPlan pl = bn_plan(batch, hw, c);
    if (!workspace || ws_bytes < pu_bn_workspace_bytes(batch, hw, c))
        return fail(PU_ERR_WORKSPACE, "pu_bn_fwd: workspace %zu < %zu", ws_bytes, pu_bn_workspace_bytes(batch, hw, c));
    double* part = (double*)workspace;
    hipLaunchKernelGGL(bn_partial_kernel<0>, dim3((c + pl.CC - 1) / pl.CC, pl.S, batch), dim3(256), 0, s, z, nullptr,
                       nullptr, batch, hw, c, pl.CC, pl.S, part);
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((c + 255) / 256), dim3(256), 0, s, part, pl.S, batch, c, hw, eps,
                       momentum, save_mean, save_rstd, running_mean, running_var);
    hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(total4)), dim3(256), 0, s, z, save_mean, save_rstd, gamma, beta,
                       resid, y, hw, c, c, total4, relu);
    return check_launch("pu_bn_fwd");
}

extern "C" int pu_bn_bwd(const float* z, const float* g, const float* save_mean, const float* save_rstd,
                         const float* gamma, float* dz, float* dgamma, float* dbeta, int batch, long long hw, int c,
                         const float* add, const float* mask, void* workspace, size_t ws_bytes, void* stream) {
    PU_REQUIRE(z && g && save_mean && save_rstd && dz && batch > 0 && hw > 0 && c > 0, "pu_bn_bwd: bad args");
    PU_REQUIRE(c % 4 == 0 && (((uintptr_t)z | (uintptr_t)g | (uintptr_t)dz | (uintptr_t)add | (uintptr_t)mask) & 15) == 0,
               "pu_bn_bwd: channels %% 4, 16-byte alignment");
    if (!workspace || ws_bytes < pu_bn_workspace_bytes(batch, hw, c))
        return fail(PU_ERR_WORKSPACE, "pu_bn_bwd: workspace %zu < %zu", ws_bytes, pu_bn_workspace_bytes(batch, hw, c));
    hipStream_t s = as_stream(stream);
    const BnPlan pl = bn_plan(batch, hw, c);
    double* part = (double*)workspace;
    float* coef = (float*)(part + (size_t)pl.S * batch * c * 2);
    hipLaunchKernelGGL(bn_partial_kernel<1>, dim3((c + pl.CC - 1) / pl.CC, pl.S, batch), dim3(256), 0, s, z, g,
                       save_mean, batch, hw, c, pl.CC, pl.S, part);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((c + 255) / 256), dim3(256), 0, s, part, pl.S, batch, c, hw, save_rstd,
                       coef, dgamma, dbeta);
    const long long total4 = (long long)batch * hw * c / 4;
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_grid(total4)), dim3(256), 0, s, z, g, save_mean, save_rstd, coef,
                       gamma, add, mask, dz, hw, c, total4);
    return check_launch("pu_bn_bwd");
}

extern "C" int pu_upsample_bilinear2x_fwd(const float* x, float* y, int batch, int h, int w, int c, void* stream) {
    PU_REQUIRE(x && y && batch > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0, "pu_upsample_bilinear2x_fwd: bad args");
    PU_REQUIRE((((uintptr_t)x | (uintptr_t)y) & 15) == 0, "pu_upsample_bilinear2x_fwd: 16-byte alignment");
    const long long total4 = (long long)batch * 4 * h * w * c / 4;
    hipLaunchKernelGGL(upsample_bilinear2x_fwd_kernel, dim3(ew_grid(total4)), dim3(256), 0, as_stream(stream), x, y, h, w,
                       c, total4);
    return check_launch("pu_upsample_bilinear2x_fwd");
}

extern "C" int pu_upsample_bilinear2x_bwd(const float* dy, const float* mask, float* dx, int batch, int h, int w, int c,
                                          void* stream) {
    PU_REQUIRE(dy && dx && batch > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0, "pu_upsample_bilinear2x_bwd: bad args");
    PU_REQUIRE((((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)mask) & 15) == 0, "pu_upsample_bilinear2x_bwd: alignment");
    const long long total4 = (long long)batch * h * w * c / 4;
    hipLaunchKernelGGL(upsample_bilinear2x_bwd_kernel, dim3(ew_grid(total4)), dim3(256), 0, as_stream(stream), dy, mask,
                       dx, h, w, c, total4);
    return check_launch("pu_upsample_bilinear2x_bwd");
}
