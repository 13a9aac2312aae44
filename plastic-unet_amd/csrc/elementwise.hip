// Bandwidth-bound kernels of the trunk: parameter packing, NCHW->NHWC input, MaxPool2d(2)
// forward/backward and the 1x1 outconv (C -> 1) forward/backward.  All HBM-bound: float4 (16 B
// per lane) accesses along the contiguous NHWC channel axis.
//
// Reference call sites (yaricom/Plastic-UNet): nn.MaxPool2d(2) in down (src/unet/unet_p.py:222),
// outconv nn.Conv2d(C, n_classes, 1) (unet_p.py:253-260), and their autograd backward
// (src/train.py:110).
#include "common.h"

#include <math.h>

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// activation element access for the fp32 and bf16 (config C3) variants: compute is fp32
template <typename T> __device__ __forceinline__ f32x4 ld4(const T* p);
template <> __device__ __forceinline__ f32x4 ld4<float>(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
template <> __device__ __forceinline__ f32x4 ld4<__bf16>(const __bf16* p) {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
template <typename T> __device__ __forceinline__ void st4(T* p, f32x4 v);
template <> __device__ __forceinline__ void st4<float>(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
template <> __device__ __forceinline__ void st4<__bf16>(__bf16* p, f32x4 v) {
    *reinterpret_cast<bf16x4*>(p) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}

// K position -> tap-major index (tap*C + c) for a channel-group-major packed K axis
__device__ __forceinline__ int ungroup_k(int k, int C, int taps, int G) {
    if (G == 0 || k >= taps * C) return k;
    const int tg = k / G, cg = k - tg * G;
    const int g = tg / taps, tap = tg - g * taps;
    return tap * C + g * G + cg;
}

// packed operand element (row, column kc of the packed K axis) of the parameter w (layouts: plastic_unet.h)
__device__ __forceinline__ float pack_value(const float* __restrict__ w, int mode, int d0, int d1, int taps,
                                            int row, int kc, int G) {
    const int Ck = (mode == PU_PACK_CONV_DGRAD) ? d0 : d1;   // channels along K (taps*Ck columns)
    const int k = (mode == PU_PACK_CONVT_FWD) ? kc : ungroup_k(kc, Ck, taps, G);
    float v = 0.f;
    if (mode == PU_PACK_CONV_FWD) {          // w[O=d0][I=d1][R][S] -> [o][(r*S+s)*I+i]
        if (k < taps * d1) {
            int tap = k / d1, i = k - tap * d1;
            v = w[((long long)row * d1 + i) * taps + tap];
        }
    } else if (mode == PU_PACK_CONV_DGRAD) { // -> [i][((R-1-r)*S+(S-1-s))*O+o]
        if (k < taps * d0) {
            int tapf = k / d0, o = k - tapf * d0;
            int tap = taps - 1 - tapf;       // (R-1-r, S-1-s) flattened == taps-1-(r*S+s)
            v = w[((long long)o * d1 + row) * taps + tap];
        }
    } else if (mode == PU_PACK_CONVT_FWD) {  // w[I=d0][O=d1][R][S] -> [(r*S+s)*O+o][i]
        if (k < d0) {
            int tap = row / d1, o = row - tap * d1;
            v = w[((long long)k * d1 + o) * taps + tap];
        }
    } else if (mode == PU_PACK_CONVT_DGRAD) {  // -> [i][(r*S+s)*O+o]
        if (k < taps * d1) {
            int tap = k / d1, o = k - tap * d1;
            v = w[((long long)row * d1 + o) * taps + tap];
        }
    } else {                                 // PU_PACK_CONVT3_FWD: w[I=d0][O=d1][3][3]
        // row = (ph*2+pw)*O + o, k = (dh*2+dw)*I + i ; tap index along one axis: R(0,1)=0,
        // R(0,0)=2, R(1,1)=1, R(1,0) = none
        if (k < 4 * d0) {
            const int phw = row / d1, o = row - phw * d1;
            const int dhw = k / d0, i = k - dhw * d0;
            const int ph = phw >> 1, pw = phw & 1, dh = dhw >> 1, dw = dhw & 1;
            const int r = ph == 0 ? (dh ? 0 : 2) : (dh ? 1 : -1);
            const int q = pw == 0 ? (dw ? 0 : 2) : (dw ? 1 : -1);
            if (r >= 0 && q >= 0) v = w[(((long long)i * d1 + o) * 3 + r) * 3 + q];
        }
    }
    return v;
}

template <typename TO>
__global__ void pack_weight_kernel(const float* __restrict__ w, TO* __restrict__ p, int mode, int d0, int d1,
                                   int kh, int kw, int k_pad, int rows, int G) {
    const long long total = (long long)rows * k_pad;
    const int taps = kh * kw;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int row = int(idx / k_pad);
        p[idx] = (TO)pack_value(w, mode, d0, d1, taps, row, int(idx - (long long)row * k_pad), G);
    }
}

// Every packed operand of a model in one launch (pu_pack_weights): a lane produces 8 consecutive K
// columns of one row -> the fp32 packed row (2 x 16 B), the bf16 packed row (16 B) and/or the three
// exact bf16 split planes (3 x 16 B, [k_pad/16][6][rows][8], the split of split_weight6_kernel).
constexpr int PACK_MAX_JOBS = 32;
struct PackBatch {
    const float* w[PACK_MAX_JOBS];
    float* packed[PACK_MAX_JOBS];
    __bf16* packed_bf16[PACK_MAX_JOBS];
    __bf16* planes[PACK_MAX_JOBS];
    int mode[PACK_MAX_JOBS], d0[PACK_MAX_JOBS], d1[PACK_MAX_JOBS], taps[PACK_MAX_JOBS];
    int rows[PACK_MAX_JOBS], k_pad[PACK_MAX_JOBS], G[PACK_MAX_JOBS];
    int block_start[PACK_MAX_JOBS + 1];
    int count;
};
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void pack_multi_kernel(const PackBatch b) {
#pragma clang fp contract(off)
    int j = 0;
    while (j + 1 < b.count && (int)blockIdx.x >= b.block_start[j + 1]) ++j;
    const int k_pad = b.k_pad[j], rows = b.rows[j];
    const int chunks = k_pad >> 3;
    // a wave covers 8 rows x 8 column chunks (64 columns): the fp32 rows are written as 256 B runs
    // and each (t, half) plane segment as 8 rows x 16 B = one 128 B run
    const int cgs = (chunks + 7) >> 3;
    const long long wv = (long long)(blockIdx.x - b.block_start[j]) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long long rg = wv / cgs;
    const int row = (int)(rg * 8 + (lane >> 3));
    const int chunk = (int)(wv - rg * cgs) * 8 + (lane & 7);
    if (row >= rows || chunk >= chunks) return;
    const int k0 = chunk * 8;
    const int mode = b.mode[j], d0 = b.d0[j], d1 = b.d1[j], taps = b.taps[j], G = b.G[j];
    const float* __restrict__ w = b.w[j];
    float v[8];
    // fast path: the 8 columns are 8 consecutive channels of one tap -> one index decomposition and
    // a constant source stride (no per-element integer divisions)
    const int Ck = (mode == PU_PACK_CONV_DGRAD) ? d0 : d1;
    long long base = -1, stride = 0;
    if (mode == PU_PACK_CONVT_FWD) {
        if (k0 + 8 <= d0) {
            const int tap = row / d1, o = row - tap * d1;
            base = ((long long)k0 * d1 + o) * taps + tap;
            stride = (long long)d1 * taps;
        }
    } else if (mode != PU_PACK_CONVT3_FWD && Ck % 8 == 0 && (G == 0 || G % 8 == 0) && k0 + 8 <= taps * Ck) {
        const int kk = ungroup_k(k0, Ck, taps, G);
        const int tap = kk / Ck, c0 = kk - tap * Ck;
        if (mode == PU_PACK_CONV_DGRAD) {
            base = ((long long)c0 * d1 + row) * taps + (taps - 1 - tap);
            stride = (long long)d1 * taps;
        } else {   // CONV_FWD, CONVT_DGRAD: w[row][c][tap]
            base = ((long long)row * d1 + c0) * taps + tap;
            stride = taps;
        }
    }
    if (base >= 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = w[base + e * stride];
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = pack_value(w, mode, d0, d1, taps, row, k0 + e, G);
    }
    const long long o = (long long)row * k_pad + k0;
    if (b.packed[j]) {
        *reinterpret_cast<f32x4*>(b.packed[j] + o) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(b.packed[j] + o + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
    if (b.packed_bf16[j]) {
        bf16x8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (__bf16)v[e];
        *reinterpret_cast<bf16x8*>(b.packed_bf16[j] + o) = h;
    }
    if (b.planes[j]) {
        bf16x8 hi, mid, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const __bf16 a = (__bf16)v[e];
            const float r = v[e] - (float)a;
            const __bf16 m = (__bf16)r;
            hi[e] = a; mid[e] = m; lo[e] = (__bf16)(r - (float)m);
        }
        const int t = k0 >> 4, half = (k0 >> 3) & 1;
        __bf16* P = b.planes[j];
        *reinterpret_cast<bf16x8*>(P + (((long long)t * 6 + 0 + half) * rows + row) * 8) = hi;
        *reinterpret_cast<bf16x8*>(P + (((long long)t * 6 + 2 + half) * rows + row) * 8) = mid;
        *reinterpret_cast<bf16x8*>(P + (((long long)t * 6 + 4 + half) * rows + row) * 8) = lo;
    }
}

__global__ void nchw_to_nhwc_kernel(const float* __restrict__ s, float* __restrict__ d, int C, int HW, long long total) {
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c = int(idx % C);
        const long long bp = idx / C;
        const long long b = bp / HW;
        const int pix = int(bp - b * HW);
        d[idx] = s[(b * C + c) * HW + pix];
    }
}

// ATen CPU max-pool rule: scan the window row-major, take val if (val > max || isnan(val)).
__device__ __forceinline__ void pool_take(float v, int idx, float& best, int& arg) {
    if (v > best || isnan(v)) {
        best = v;
        arg = idx;
    }
}

template <bool VEC, typename T = float>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int H, int W, int C, int Ho,
                                   int Wo, long long total, const float* __restrict__ scale) {
    const int CV = VEC ? C / 4 : C;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int cv = int(idx % CV);
        long long t = idx / CV;
        const int wo = int(t % Wo); t /= Wo;
        const int ho = int(t % Ho);
        const long long b = t / Ho;
        const long long base = ((b * H + 2 * ho) * W + 2 * wo);
        if (VEC) {
            f32x4 best = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
            int arg[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long pix = base + (q >> 1) * W + (q & 1);
                f32x4 v = ld4(x + pix * C + cv * 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) { float bb = best[e]; pool_take(v[e], q, bb, arg[e]); best[e] = bb; }
            }
            if (scale) best *= ld4(scale + b * C + cv * 4);
            st4(y + idx * 4, best);
        } else {
            float best = -INFINITY;
            int arg = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long pix = base + (q >> 1) * W + (q & 1);
                pool_take((float)x[pix * C + cv], q, best, arg);
            }
            if (scale) best *= scale[b * C + cv];
            y[idx] = (T)best;
        }
    }
}

// One thread per INPUT element group (pixel, 4 channels): recompute the window's argmax and
// route the pooled gradient to it; every other input element gets 0 (or keeps its value).
template <bool VEC, typename T = float>
__global__ void maxpool_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx,
                                   int H, int W, int C, int Ho, int Wo, int relu_mask, int accumulate,
                                   long long total, const float* __restrict__ scale) {
    constexpr int V = VEC ? 4 : 1;
    const int CV = C / V;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int cv = int(idx % CV);
        long long t = idx / CV;
        const int wi = int(t % W); t /= W;
        const int hi = int(t % H);
        const long long b = t / H;
        const int ho = hi >> 1, wo = wi >> 1;
        float out[V];
        float old[V];
        if (accumulate) {
#pragma unroll
            for (int e = 0; e < V; ++e) old[e] = (float)dx[idx * V + e];
        }
#pragma unroll
        for (int e = 0; e < V; ++e) out[e] = 0.f;
        if (ho < Ho && wo < Wo) {
            const int me = (hi & 1) * 2 + (wi & 1);
            const long long base = ((b * H + 2 * ho) * W + 2 * wo);
            float best[V];
            int arg[V];
            float xme[V];
#pragma unroll
            for (int e = 0; e < V; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long pix = base + (q >> 1) * W + (q & 1);
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    float v = (float)x[pix * C + cv * V + e];
                    if (q == me) xme[e] = v;
                    pool_take(v, q, best[e], arg[e]);
                }
            }
            const long long oidx = ((b * Ho + ho) * Wo + wo) * C + cv * V;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                if (arg[e] == me && (!relu_mask || xme[e] > 0.f))
                    out[e] = scale ? (float)dy[oidx + e] * scale[b * C + cv * V + e] : (float)dy[oidx + e];
            }
        }
#pragma unroll
        for (int e = 0; e < V; ++e) dx[idx * V + e] = (T)(accumulate ? old[e] + out[e] : out[e]);
    }
}

// 16-byte vector of V = 16 / sizeof(T) channels as floats
template <typename T>
struct Vec16 {
    static constexpr int V = 16 / sizeof(T);
    float v[V];
};
template <typename T>
__device__ __forceinline__ Vec16<T> ld16(const T* p) {
    Vec16<T> r;
    if constexpr (sizeof(T) == 4) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
        for (int e = 0; e < 4; ++e) r.v[e] = a[e];
    } else {
        typedef __bf16 b8 __attribute__((ext_vector_type(8)));
        const b8 a = *reinterpret_cast<const b8*>(p);
#pragma unroll
        for (int e = 0; e < 8; ++e) r.v[e] = (float)a[e];
    }
    return r;
}
template <typename T>
__device__ __forceinline__ void st16(T* p, const float (&v)[Vec16<T>::V]) {
    if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    } else {
        typedef __bf16 b8 __attribute__((ext_vector_type(8)));
        b8 a;
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] = (__bf16)v[e];
        *reinterpret_cast<b8*>(p) = a;
    }
}

// One thread per (pooled pixel, 16-byte channel vector): even H and W, C % V == 0, 16-B aligned.
// fwd reads the 2x2 window once (the same pool_take scan as maxpool_fwd_kernel); bwd reads the
// window and dy once and writes all four dx pixels (zeros off the argmax / under the ReLU mask),
// instead of one thread per full-resolution pixel re-reading the whole window.
template <typename T>
__global__ void maxpool_fwd_win_kernel(const T* __restrict__ x, T* __restrict__ y, int W, int C, int Ho, int Wo,
                                       long long total, const float* __restrict__ scale) {
    constexpr int V = Vec16<T>::V;
    const int CV = C / V;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int cv = int(idx % CV);
        long long t = idx / CV;
        const int wo = int(t % Wo); t /= Wo;
        const int ho = int(t % Ho);
        const long long b = t / Ho;
        const long long base = (b * 2 * Ho + 2 * ho) * (long long)W + 2 * wo;
        float best[V];
        int arg[V];
#pragma unroll
        for (int e = 0; e < V; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const Vec16<T> v = ld16(x + (base + (q >> 1) * W + (q & 1)) * C + cv * V);
#pragma unroll
            for (int e = 0; e < V; ++e) pool_take(v.v[e], q, best[e], arg[e]);
        }
        if (scale) {            // Dropout2d after the pool (unet_p_res.py:62): the pooled value times s[b][c]
#pragma unroll
            for (int e = 0; e < V; ++e) best[e] *= scale[b * C + cv * V + e];
        }
        st16(y + idx * V, best);
    }
}

template <typename T>
__global__ void maxpool_bwd_win_kernel(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx, int W,
                                       int C, int Ho, int Wo, int relu_mask, int accumulate, long long total,
                                       const float* __restrict__ scale) {
    constexpr int V = Vec16<T>::V;
    const int CV = C / V;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int cv = int(idx % CV);
        long long t = idx / CV;
        const int wo = int(t % Wo); t /= Wo;
        const int ho = int(t % Ho);
        const long long b = t / Ho;
        const long long base = (b * 2 * Ho + 2 * ho) * (long long)W + 2 * wo;
        Vec16<T> xv[4];
        float best[V];
        int arg[V];
#pragma unroll
        for (int e = 0; e < V; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            xv[q] = ld16(x + (base + (q >> 1) * W + (q & 1)) * C + cv * V);
#pragma unroll
            for (int e = 0; e < V; ++e) pool_take(xv[q].v[e], q, best[e], arg[e]);
        }
        Vec16<T> g = ld16(dy + idx * V);
        if (scale) {            // the Dropout2d backward of the pooled gradient
#pragma unroll
            for (int e = 0; e < V; ++e) g.v[e] *= scale[b * C + cv * V + e];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            T* d = dx + (base + (q >> 1) * W + (q & 1)) * C + cv * V;
            float out[V];
#pragma unroll
            for (int e = 0; e < V; ++e) out[e] = (arg[e] == q && (!relu_mask || xv[q].v[e] > 0.f)) ? g.v[e] : 0.f;
            if (accumulate) {
                const Vec16<T> o = ld16(d);
#pragma unroll
                for (int e = 0; e < V; ++e) out[e] = o.v[e] + out[e];
            }
            st16(d, out);
        }
    }
}

// outconv forward: 16 lanes per pixel, each a float4 of channels; shuffle-reduce over the 16.
template <typename T = float>
__global__ void outconv_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                                   float* __restrict__ y, long long rows, int C) {
    const int lane16 = threadIdx.x & 15;
    const long long groups = (long long)gridDim.x * (blockDim.x >> 4);
    const float bias = b ? b[0] : 0.f;
    for (long long m = blockIdx.x * (long long)(blockDim.x >> 4) + (threadIdx.x >> 4); m < rows + 0; m += groups) {
        float s = 0.f;
        for (int c = lane16 * 4; c < C; c += 64) {
            f32x4 v = ld4(x + m * C + c);
            f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
            s += dot4_fma(v, ww);
        }
        s += __shfl_xor(s, 8, 16);
        s += __shfl_xor(s, 4, 16);
        s += __shfl_xor(s, 2, 16);
        s += __shfl_xor(s, 1, 16);
        if (lane16 == 0) y[m] = s + bias;
    }
}

__global__ void outconv_fwd_scalar_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                          const float* __restrict__ b, float* __restrict__ y, long long rows, int C) {
    for (long long m = blockIdx.x * (long long)blockDim.x + threadIdx.x; m < rows; m += (long long)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int c = 0; c < C; ++c) s += x[m * C + c] * w[c];
        y[m] = s + (b ? b[0] : 0.f);
    }
}

// outconv backward: dx = dy (x) w (masked); per-block partial sums of dw (C) and db.
// Thread layout: 16 pixel groups x 16 lanes; lane owns channels lane*4 + 64*j.
constexpr int OC_BLOCKS = 1024;

template <typename T = float>
__global__ void outconv_bwd_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ dy,
                                   T* __restrict__ dx, float* __restrict__ partial, long long rows, int C,
                                   int relu_mask) {
    __shared__ float red[16][65];
    __shared__ float redb[16];
    const int lane16 = threadIdx.x & 15;
    const int grp = threadIdx.x >> 4;
    float* out = partial + (long long)blockIdx.x * (C + 1);
    for (int j = 0; j * 64 < C; ++j) {
        const int c = lane16 * 4 + 64 * j;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, ab = 0.f;
        for (long long m = blockIdx.x * 16LL + grp; m < rows; m += (long long)gridDim.x * 16) {
            const float g = dy[m];
            ab += g;
            if (c < C) {
                f32x4 v = ld4(x + m * C + c);
                f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
                f32x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (!relu_mask || v[e] > 0.f) ? g * ww[e] : 0.f;
                st4(dx + m * C + c, o);
                a0 += g * v[0]; a1 += g * v[1]; a2 += g * v[2]; a3 += g * v[3];
            }
        }
        __syncthreads();
        red[grp][lane16 * 4 + 0] = a0;
        red[grp][lane16 * 4 + 1] = a1;
        red[grp][lane16 * 4 + 2] = a2;
        red[grp][lane16 * 4 + 3] = a3;
        if (lane16 == 0) redb[grp] = ab;
        __syncthreads();
        const int t = threadIdx.x;
        if (t < 64 && 64 * j + t < C) {
            float s = 0.f;
            for (int q = 0; q < 16; ++q) s += red[q][t];
            out[64 * j + t] = s;
        }
        if (j == 0 && t == 64) {
            float s = 0.f;
            for (int q = 0; q < 16; ++q) s += redb[q];
            out[C] = s;
        }
    }
}

// outconv backward for narrow features (C = 4L, L = 2 / 4 / 8 lanes per pixel: C4 / C5's 8-channel
// head input): the 16-lane layout above leaves 16 - L lanes of every pixel group idle and keeps
// one pixel per group in flight (0.26 ms at 1.1 TB/s on C5).  Here a block covers 256 / L pixels
// per round and every thread issues OCN_U rounds' loads before their arithmetic.  The partials keep
// the layout column_sum_kernel reads; per-thread sums run over the thread's pixels in index order.
constexpr int OCN_U = 4;
template <typename T, int L>
__global__ __launch_bounds__(256) void outconv_bwd_narrow_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                                 const float* __restrict__ dy, T* __restrict__ dx,
                                                                 float* __restrict__ partial, long long rows,
                                                                 int relu_mask) {
    constexpr int C = 4 * L, P = 256 / L;     // channels, pixel groups per block
    __shared__ float red[P][C + 1];
    __shared__ float redb[P];
    const int lane = threadIdx.x % L, grp = threadIdx.x / L;
    const int c = 4 * lane;
    const f32x4 ww = *reinterpret_cast<const f32x4*>(w + c);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, ab = 0.f;
    const long long stride = (long long)gridDim.x * P;
    for (long long m0 = blockIdx.x * (long long)P + grp; m0 < rows; m0 += OCN_U * stride) {
        f32x4 v[OCN_U];
        float g[OCN_U];
#pragma unroll
        for (int u = 0; u < OCN_U; ++u) {
            const long long m = m0 + u * stride;
            const bool ok = m < rows;
            g[u] = ok ? dy[m] : 0.f;
            v[u] = ok ? ld4(x + m * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < OCN_U; ++u) {
            const long long m = m0 + u * stride;
            if (m < rows) {
                f32x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (!relu_mask || v[u][e] > 0.f) ? g[u] * ww[e] : 0.f;
                st4(dx + m * C + c, o);
                ab += g[u];
                a0 += g[u] * v[u][0]; a1 += g[u] * v[u][1]; a2 += g[u] * v[u][2]; a3 += g[u] * v[u][3];
            }
        }
    }
    red[grp][c + 0] = a0;
    red[grp][c + 1] = a1;
    red[grp][c + 2] = a2;
    red[grp][c + 3] = a3;
    if (lane == 0) redb[grp] = ab;
    __syncthreads();
    float* out = partial + (long long)blockIdx.x * (C + 1);
    const int t = threadIdx.x;
    if (t < C) {
        float s = 0.f;
        for (int q = 0; q < P; ++q) s += red[q][t];
        out[t] = s;
    } else if (t == C) {
        float s = 0.f;
        for (int q = 0; q < P; ++q) s += redb[q];
        out[C] = s;
    }
}

// one block per column: fixed-order fp64 tree over the per-block partials
__global__ void column_sum_kernel(const float* __restrict__ partial, int nparts, int cols, float* __restrict__ dw,
                                  float* __restrict__ db) {
    __shared__ double red[256];
    const int c = blockIdx.x;
    double s = 0.0;
    for (int q = threadIdx.x; q < nparts; q += 256) s += partial[(long long)q * (cols + 1) + c];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (c < cols) dw[c] = (float)red[0];
        else db[0] = (float)red[0];
    }
}

// Dropout2d on float4 channel quads: grid row y = image b, 32-bit quad index within the image
// (the generic form below spent two 64-bit divisions per float4: 2.8 TB/s on C5's planes)
__global__ void channel_scale4_kernel(const f32x4* __restrict__ x, const float* __restrict__ scale, f32x4* y,
                                      unsigned per_img, FastDiv dcq, int c) {
    const unsigned b = blockIdx.y;
    const f32x4* xb = x + (size_t)b * per_img;
    f32x4* yb = y + (size_t)b * per_img;
    const float* sc = scale + (size_t)b * c;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < per_img; i += gridDim.x * blockDim.x) {
        const unsigned c4 = (i - fdiv(i, dcq) * dcq.d) * 4;
        f32x4 v = xb[i];
        const f32x4 s4 = *reinterpret_cast<const f32x4*>(sc + c4);
        v[0] *= s4[0]; v[1] *= s4[1]; v[2] *= s4[2]; v[3] *= s4[3];
        yb[i] = v;
    }
}

// Dropout2d: y = x * scale[b][c] over NHWC
template <bool VEC>
__global__ void channel_scale_kernel(const float* __restrict__ x, const float* __restrict__ scale, float* y,
                                     long long hw, int c, long long total) {
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        if (VEC) {
            const int cq = c >> 2;
            const long long pix = idx / cq;
            const int c4 = int(idx - pix * cq) * 4;
            const long long b = pix / hw;
            f32x4 v = reinterpret_cast<const f32x4*>(x)[idx];
            const float* sc = scale + b * c + c4;
            v[0] *= sc[0]; v[1] *= sc[1]; v[2] *= sc[2]; v[3] *= sc[3];
            reinterpret_cast<f32x4*>(y)[idx] = v;
        } else {
            const long long pix = idx / c;
            const int ch = int(idx - pix * c);
            y[idx] = x[idx] * scale[(pix / hw) * c + ch];
        }
    }
}

// AddCoords + NCHW->NHWC: one thread per output element (channel fastest); fp32 with no
// contraction so the coordinate values are those of the elementwise CPU ops
#pragma clang fp contract(off)
// c == 1 with r (the CoordConv U-Net's input): one thread per pixel, one float4 store
// {x, xx, yy, r}; the same float expressions as add_coords_kernel (bit-identical), 32-bit index math
__global__ void add_coords4_kernel(const float* __restrict__ x, float* __restrict__ out, int h, int w, int pixels) {
    for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < pixels; pix += gridDim.x * blockDim.x) {
        const int rem = pix % (h * w);
        const int i = rem / w, j = rem - i * w;
        const float xx = ((float)j / (float)(h - 1)) * 2.0f - 1.0f;
        const float yy = ((float)i / (float)(w - 1)) * 2.0f - 1.0f;
        const float dx = xx - 0.5f, dy = yy - 0.5f;
        *reinterpret_cast<f32x4*>(out + 4LL * pix) = f32x4{x[pix], xx, yy, sqrtf(dx * dx + dy * dy)};
    }
}

__global__ void add_coords_kernel(const float* __restrict__ x, float* __restrict__ out, int c, int h, int w,
                                  int with_r, long long total) {
    const int co = c + 2 + with_r;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long pix = idx / co;
        const int ch = int(idx - pix * co);
        const long long hw = (long long)h * w;
        const long long b = pix / hw;
        const int rem = int(pix - b * hw);
        const int i = rem / w, j = rem - (rem / w) * w;
        float v;
        if (ch < c) {
            v = x[(b * c + ch) * hw + rem];
        } else {
            const float xx = ((float)j / (float)(h - 1)) * 2.0f - 1.0f;
            const float yy = ((float)i / (float)(w - 1)) * 2.0f - 1.0f;
            if (ch == c) v = xx;
            else if (ch == c + 1) v = yy;
            else {
                const float dx = xx - 0.5f, dy = yy - 0.5f;
                v = sqrtf(dx * dx + dy * dy);
            }
        }
        out[idx] = v;
    }
}

// column sums, pass 1: block q sums rows [q*rpb, (q+1)*rpb) of column chunk blockIdx.y in fp64.
// cols % 4 == 0: threads = (row lane, float4 column group) over a 1024-column chunk, 4 rows in
// flight per thread (independent accumulators, fixed combine order); else scalar columns.
template <bool VEC>
__global__ void colsum_partial_kernel(const float* __restrict__ x, long long rows, int cols, long long rpb,
                                      double* __restrict__ part) {
    __shared__ double red[256 * 4];
    constexpr int W = VEC ? 4 : 1;
    const int c0 = blockIdx.y * 256 * W;
    const int cw = min(256, (cols - c0 + W - 1) / W);     // column groups in this chunk
    const int rl = 256 / cw;
    const int t = threadIdx.x;
    const int cg = t % cw, lane = t / cw;
    double s[4][W];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < W; ++k) s[u][k] = 0.0;
    const long long r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
    if (lane < rl) {
        const int col = c0 + cg * W;
        long long r = r0 + lane;
        for (; r + 3LL * rl < r1; r += 4LL * rl) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float* src = x + (r + (long long)u * rl) * cols + col;
                if (VEC) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(src);
#pragma unroll
                    for (int k = 0; k < W; ++k) s[u][k] += (double)v[k];
                } else {
                    s[u][0] += (double)src[0];
                }
            }
        }
        for (; r < r1; r += rl) {
            const float* src = x + r * cols + col;
            if (VEC) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(src);
#pragma unroll
                for (int k = 0; k < W; ++k) s[0][k] += (double)v[k];
            } else {
                s[0][0] += (double)src[0];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < W; ++k) red[t * W + k] = (s[0][k] + s[1][k]) + (s[2][k] + s[3][k]);
    __syncthreads();
    if (t < cw) {
#pragma unroll
        for (int k = 0; k < W; ++k) {
            double v = 0.0;
            for (int l = 0; l < rl; ++l) v += red[(l * cw + t) * W + k];
            const int col = c0 + t * W + k;
            if (col < cols) part[(long long)blockIdx.x * cols + col] = v;
        }
    }
}

// pass 2: out[c] (+)= sum over the partial blocks, one block per column: strided fp64 partial
// sums in a fixed thread order, then a fixed LDS tree (deterministic)
__global__ void colsum_final_kernel(const double* __restrict__ part, int nparts, int cols, float* __restrict__ out,
                                    int accumulate) {
    __shared__ double red[256];
    const int c = blockIdx.x;
    double s = 0.0;
    for (int q = threadIdx.x; q < nparts; q += 256) s += part[(long long)q * cols + c];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = accumulate ? out[c] + (float)red[0] : (float)red[0];
}

static int colsum_blocks(long long rows) {
    long long b = (rows + 1023) / 1024;
    return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

static int grid_for(long long total, int block = 256, int cap = 8192) {
    long long g = (total + block - 1) / block;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, __bf16* __restrict__ y, long long n4) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
        st4(y + 4 * i, ld4(x + 4 * i));
}

__global__ void bf16_to_f32_kernel(const __bf16* __restrict__ x, float* __restrict__ y, long long n4) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
        st4(y + 4 * i, ld4(x + 4 * i));
}

}  // namespace pu

using namespace pu;

// argument checks shared by the pack entry points; *rows = rows of the packed operand
static int pack_check(const float* w, int mode, int d0, int d1, int kh, int kw, int k_pad, int cgroup, int* rows,
                      const char* name) {
    PU_REQUIRE(w && d0 > 0 && d1 > 0 && kh > 0 && kw > 0 && k_pad > 0, "%s: bad args", name);
    PU_REQUIRE(cgroup == 0 || cgroup == 16 || cgroup == 32, "%s: cgroup %d", name, cgroup);
    if (cgroup) {
        const int Ck = (mode == PU_PACK_CONV_DGRAD) ? d0 : d1;
        PU_REQUIRE(mode == PU_PACK_CONVT_FWD || Ck % cgroup == 0, "%s: %d channels not a multiple of cgroup %d", name, Ck, cgroup);
    }
    PU_REQUIRE(mode >= 0 && mode <= 4, "%s: mode %d", name, mode);
    PU_REQUIRE(mode != PU_PACK_CONVT3_FWD || (kh == 3 && kw == 3 && cgroup == 0), "%s: CONVT3_FWD is 3x3, tap-major", name);
    const int taps = kh * kw;
    int kmin;
    switch (mode) {
        case PU_PACK_CONV_FWD: *rows = d0; kmin = taps * d1; break;
        case PU_PACK_CONV_DGRAD: *rows = d1; kmin = taps * d0; break;
        case PU_PACK_CONVT_FWD: *rows = taps * d1; kmin = d0; break;
        case PU_PACK_CONVT3_FWD: *rows = 4 * d1; kmin = 4 * d0; break;
        default: *rows = d0; kmin = taps * d1; break;
    }
    PU_REQUIRE(k_pad >= kmin, "%s: k_pad %d < %d", name, k_pad, kmin);
    return PU_OK;
}

template <typename TO>
static int pack_weight_impl(const float* w, TO* packed, int mode, int d0, int d1, int kh, int kw, int k_pad, int cgroup,
                            void* stream, const char* name) {
    PU_REQUIRE(packed, "%s: bad args", name);
    int rows = 0;
    const int st = pack_check(w, mode, d0, d1, kh, kw, k_pad, cgroup, &rows, name);
    if (st != PU_OK) return st;
    const long long total = (long long)rows * k_pad;
    hipLaunchKernelGGL(pack_weight_kernel<TO>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), w, packed, mode,
                       d0, d1, kh, kw, k_pad, rows, cgroup);
    return check_launch(name);
}

extern "C" int pu_pack_weights(const pu_pack_job* jobs, int n_jobs, void* stream) {
    PU_REQUIRE(n_jobs >= 0 && (n_jobs == 0 || jobs), "pu_pack_weights: bad job list");
    int i = 0;
    while (i < n_jobs) {
        PackBatch b;
        b.count = 0;
        int blocks = 0;
        while (i < n_jobs && b.count < PACK_MAX_JOBS) {
            const pu_pack_job& J = jobs[i++];
            int rows = 0;
            const int st = pack_check(J.w, J.mode, J.d0, J.d1, J.kh, J.kw, J.k_pad, J.cgroup, &rows, "pu_pack_weights");
            if (st != PU_OK) return st;
            PU_REQUIRE(J.packed || J.packed_bf16 || J.planes, "pu_pack_weights: job %d has no output", i - 1);
            PU_REQUIRE(J.k_pad % (J.planes ? 16 : 8) == 0, "pu_pack_weights: job %d k_pad %d", i - 1, J.k_pad);
            PU_REQUIRE(((((uintptr_t)J.packed) | ((uintptr_t)J.packed_bf16) | ((uintptr_t)J.planes)) & 15) == 0,
                       "pu_pack_weights: job %d outputs must be 16-byte aligned", i - 1);
            const int k = b.count;
            b.w[k] = J.w; b.packed[k] = J.packed; b.packed_bf16[k] = (__bf16*)J.packed_bf16; b.planes[k] = (__bf16*)J.planes;
            b.mode[k] = J.mode; b.d0[k] = J.d0; b.d1[k] = J.d1; b.taps[k] = J.kh * J.kw;
            b.rows[k] = rows; b.k_pad[k] = J.k_pad; b.G[k] = J.cgroup;
            b.block_start[k] = blocks;
            const long long waves = (long long)((rows + 7) / 8) * ((J.k_pad / 8 + 7) / 8);
            blocks += (int)((waves + 3) / 4);
            b.count++;
        }
        b.block_start[b.count] = blocks;
        if (b.count == 0) continue;
        hipLaunchKernelGGL(pack_multi_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), b);
        const int st = check_launch("pu_pack_weights");
        if (st != PU_OK) return st;
    }
    return PU_OK;
}

extern "C" int pu_pack_weight(const float* w, float* packed, int mode, int d0, int d1, int kh, int kw, int k_pad,
                              int cgroup, void* stream) {
    return pack_weight_impl(w, packed, mode, d0, d1, kh, kw, k_pad, cgroup, stream, "pu_pack_weight");
}

extern "C" int pu_pack_weight_bf16(const float* w, void* packed, int mode, int d0, int d1, int kh, int kw, int k_pad,
                                   int cgroup, void* stream) {
    return pack_weight_impl(w, (__bf16*)packed, mode, d0, d1, kh, kw, k_pad, cgroup, stream, "pu_pack_weight_bf16");
}

extern "C" int pu_nchw_to_nhwc(const float* src, float* dst, int batch, int c, int h, int w, void* stream) {
    PU_REQUIRE(src && dst && batch > 0 && c > 0 && h > 0 && w > 0, "pu_nchw_to_nhwc: bad args");
    const long long total = (long long)batch * c * h * w;
    hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), src, dst, c, h * w,
                       total);
    return check_launch("pu_nchw_to_nhwc");
}

static int maxpool2_fwd_f32(const float* x, float* y, const float* scale, int batch, int h, int w, int c, void* stream) {
    PU_REQUIRE(x && y && batch > 0 && h >= 2 && w >= 2 && c > 0, "pu_maxpool2_fwd: bad args");
    const int ho = h / 2, wo = w / 2;
    const bool vec = (c % 4 == 0) && (((uintptr_t)x | (uintptr_t)y) & 15) == 0;
    if (vec && h % 2 == 0 && w % 2 == 0) {
        const long long wt = (long long)batch * ho * wo * (c / 4);
        hipLaunchKernelGGL(maxpool_fwd_win_kernel<float>, dim3(grid_for(wt)), dim3(256), 0, as_stream(stream), x, y, w, c,
                           ho, wo, wt, scale);
        return check_launch("pu_maxpool2_fwd");
    }
    const bool vs = vec && ((uintptr_t)scale & 15) == 0;
    const long long total = (long long)batch * ho * wo * (vs ? c / 4 : c);
    if (vs)
        hipLaunchKernelGGL(maxpool_fwd_kernel<true>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x, y, h, w,
                           c, ho, wo, total, scale);
    else
        hipLaunchKernelGGL(maxpool_fwd_kernel<false>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x, y, h,
                           w, c, ho, wo, total, scale);
    return check_launch("pu_maxpool2_fwd");
}

extern "C" int pu_maxpool2_fwd(const float* x, float* y, int batch, int h, int w, int c, void* stream) {
    return maxpool2_fwd_f32(x, y, nullptr, batch, h, w, c, stream);
}

extern "C" int pu_maxpool2_fwd_scaled(const float* x, const float* scale, float* y, int batch, int h, int w, int c,
                                      void* stream) {
    PU_REQUIRE(scale, "pu_maxpool2_fwd_scaled: scale missing");
    return maxpool2_fwd_f32(x, y, scale, batch, h, w, c, stream);
}

static int maxpool2_bwd_f32(const float* x, const float* dy, const float* scale, float* dx, int batch, int h, int w,
                            int c, int relu_mask, int accumulate, void* stream) {
    PU_REQUIRE(x && dy && dx && batch > 0 && h >= 2 && w >= 2 && c > 0, "pu_maxpool2_bwd: bad args");
    const int ho = h / 2, wo = w / 2;
    const bool vec = (c % 4 == 0);
    if (vec && h % 2 == 0 && w % 2 == 0 && (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) & 15) == 0) {
        const long long wt = (long long)batch * ho * wo * (c / 4);
        hipLaunchKernelGGL(maxpool_bwd_win_kernel<float>, dim3(grid_for(wt)), dim3(256), 0, as_stream(stream), x, dy, dx,
                           w, c, ho, wo, relu_mask, accumulate, wt, scale);
        return check_launch("pu_maxpool2_bwd");
    }
    const long long total = (long long)batch * h * w * (vec ? c / 4 : c);
    if (vec)
        hipLaunchKernelGGL(maxpool_bwd_kernel<true>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x, dy, dx,
                           h, w, c, ho, wo, relu_mask, accumulate, total, scale);
    else
        hipLaunchKernelGGL(maxpool_bwd_kernel<false>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x, dy, dx,
                           h, w, c, ho, wo, relu_mask, accumulate, total, scale);
    return check_launch("pu_maxpool2_bwd");
}

extern "C" int pu_maxpool2_bwd(const float* x, const float* dy, float* dx, int batch, int h, int w, int c,
                               int relu_mask, int accumulate, void* stream) {
    return maxpool2_bwd_f32(x, dy, nullptr, dx, batch, h, w, c, relu_mask, accumulate, stream);
}

extern "C" int pu_maxpool2_bwd_scaled(const float* x, const float* dy, const float* scale, float* dx, int batch, int h,
                                      int w, int c, int relu_mask, int accumulate, void* stream) {
    PU_REQUIRE(scale, "pu_maxpool2_bwd_scaled: scale missing");
    return maxpool2_bwd_f32(x, dy, scale, dx, batch, h, w, c, relu_mask, accumulate, stream);
}

extern "C" int pu_outconv_fwd(const float* x, const float* w, const float* b, float* y, long long rows, int c,
                              void* stream) {
    PU_REQUIRE(x && w && y && rows > 0 && c > 0, "pu_outconv_fwd: bad args");
    if (c % 4 == 0 && (((uintptr_t)x | (uintptr_t)w) & 15) == 0) {
        const long long groups = (rows + 15) / 16;
        hipLaunchKernelGGL(outconv_fwd_kernel<float>, dim3(grid_for(groups, 1, 8192)), dim3(256), 0, as_stream(stream), x, w,
                           b, y, rows, c);
    } else {
        hipLaunchKernelGGL(outconv_fwd_scalar_kernel, dim3(grid_for(rows)), dim3(256), 0, as_stream(stream), x, w, b, y,
                           rows, c);
    }
    return check_launch("pu_outconv_fwd");
}

#ifndef PU_OC_NARROW
#define PU_OC_NARROW 1     // 0: every width takes the 16-lane kernel (A/B runs)
#endif
// dx + per-block partials (the narrow kernel for C = 8 / 16 / 32), then the fixed-order column sums
template <typename T>
static void launch_outconv_bwd(const T* x, const float* w, const float* dy, T* dx, float* dw, float* db, float* part,
                               long long rows, int c, int relu_mask, hipStream_t s) {
    const int L = c / 4;
    int blocks;
    if (PU_OC_NARROW && (L == 2 || L == 4 || L == 8)) {
        const long long P = 256 / L;
        blocks = (int)std::min<long long>((rows + P - 1) / P, OC_BLOCKS);
        if (L == 2)
            hipLaunchKernelGGL((outconv_bwd_narrow_kernel<T, 2>), dim3(blocks), dim3(256), 0, s, x, w, dy, dx, part, rows, relu_mask);
        else if (L == 4)
            hipLaunchKernelGGL((outconv_bwd_narrow_kernel<T, 4>), dim3(blocks), dim3(256), 0, s, x, w, dy, dx, part, rows, relu_mask);
        else
            hipLaunchKernelGGL((outconv_bwd_narrow_kernel<T, 8>), dim3(blocks), dim3(256), 0, s, x, w, dy, dx, part, rows, relu_mask);
    } else {
        blocks = (int)std::min<long long>((rows + 15) / 16, OC_BLOCKS);
        hipLaunchKernelGGL(outconv_bwd_kernel<T>, dim3(blocks), dim3(256), 0, s, x, w, dy, dx, part, rows, c, relu_mask);
    }
    hipLaunchKernelGGL(column_sum_kernel, dim3(c + 1), dim3(256), 0, s, part, blocks, c, dw, db);
}

extern "C" size_t pu_outconv_workspace_bytes(long long rows, int c) {
    (void)rows;
    return (size_t)OC_BLOCKS * (c + 1) * sizeof(float);
}

extern "C" int pu_outconv_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db,
                              long long rows, int c, int relu_mask, void* workspace, size_t ws_bytes, void* stream) {
    PU_REQUIRE(x && w && dy && dx && dw && db && rows > 0, "pu_outconv_bwd: bad args");
    PU_REQUIRE(c % 4 == 0, "pu_outconv_bwd: channels %d must be a multiple of 4", c);
    PU_REQUIRE(((((uintptr_t)x | (uintptr_t)w | (uintptr_t)dx)) & 15) == 0, "pu_outconv_bwd: 16-byte alignment");
    const size_t need = pu_outconv_workspace_bytes(rows, c);
    if (!workspace || ws_bytes < need) return fail(PU_ERR_WORKSPACE, "pu_outconv_bwd: workspace %zu < %zu", ws_bytes, need);
    launch_outconv_bwd<float>(x, w, dy, dx, dw, db, (float*)workspace, rows, c, relu_mask, as_stream(stream));
    return check_launch("pu_outconv_bwd");
}

extern "C" int pu_channel_scale(const float* x, const float* scale, float* y, int batch, long long hw, int c,
                                void* stream) {
    PU_REQUIRE(x && scale && y && batch > 0 && hw > 0 && c > 0, "pu_channel_scale: bad args");
    const bool vec = (c % 4 == 0) && (((uintptr_t)x | (uintptr_t)y | (uintptr_t)scale) & 15) == 0;
    const long long total = (long long)batch * hw * (vec ? c / 4 : c);
    if (vec && hw * (c / 4) < (1LL << 31) && batch < 65536) {
        const long long per = hw * (c / 4);
        const int gx = grid_for(per, 256, (8192 + batch - 1) / batch);
        hipLaunchKernelGGL(channel_scale4_kernel, dim3(gx, batch), dim3(256), 0, as_stream(stream),
                           reinterpret_cast<const f32x4*>(x), scale, reinterpret_cast<f32x4*>(y), (unsigned)per,
                           make_fastdiv((uint32_t)(c / 4)), c);
        return check_launch("pu_channel_scale");
    }
    if (vec)
        hipLaunchKernelGGL(channel_scale_kernel<true>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x,
                           scale, y, hw, c, total);
    else
        hipLaunchKernelGGL(channel_scale_kernel<false>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x,
                           scale, y, hw, c, total);
    return check_launch("pu_channel_scale");
}

extern "C" size_t pu_column_sum_workspace_bytes(long long rows, int cols) {
    if (rows <= 0 || cols <= 0) return 0;
    return (size_t)colsum_blocks(rows) * cols * sizeof(double);
}

extern "C" int pu_column_sum(const float* x, long long rows, int cols, float* out, int accumulate, void* workspace,
                             size_t ws_bytes, void* stream) {
    PU_REQUIRE(x && out && rows > 0 && cols > 0, "pu_column_sum: bad args");
    const size_t need = pu_column_sum_workspace_bytes(rows, cols);
    if (!workspace || ws_bytes < need) return fail(PU_ERR_WORKSPACE, "pu_column_sum: workspace %zu < %zu", ws_bytes, need);
    const int nb = colsum_blocks(rows);
    const long long rpb = (rows + nb - 1) / nb;
    double* part = (double*)workspace;
    if (cols % 4 == 0 && ((uintptr_t)x & 15) == 0)
        hipLaunchKernelGGL(colsum_partial_kernel<true>, dim3(nb, (cols + 1023) / 1024), dim3(256), 0,
                           as_stream(stream), x, rows, cols, rpb, part);
    else
        hipLaunchKernelGGL(colsum_partial_kernel<false>, dim3(nb, (cols + 255) / 256), dim3(256), 0,
                           as_stream(stream), x, rows, cols, rpb, part);
    hipLaunchKernelGGL(colsum_final_kernel, dim3(cols), dim3(256), 0, as_stream(stream), part, nb, cols, out,
                       accumulate);
    return check_launch("pu_column_sum");
}

extern "C" int pu_add_coords(const float* x, float* out, int batch, int c, int h, int w, int with_r, void* stream) {
    PU_REQUIRE(x && out && batch > 0 && c > 0 && h > 1 && w > 1 && (with_r == 0 || with_r == 1),
               "pu_add_coords: bad args");
    const long long pixels = (long long)batch * h * w;
    if (c == 1 && with_r && ((uintptr_t)out & 15) == 0 && pixels < (1LL << 31)) {
        hipLaunchKernelGGL(add_coords4_kernel, dim3(grid_for(pixels)), dim3(256), 0, as_stream(stream), x, out, h, w,
                           (int)pixels);
        return check_launch("pu_add_coords");
    }
    const long long total = pixels * (c + 2 + with_r);
    hipLaunchKernelGGL(add_coords_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x, out, c, h, w,
                       with_r, total);
    return check_launch("pu_add_coords");
}

// ------------------------------------------------------------------ bf16 variants (config C3)
extern "C" int pu_convert_f32_bf16(const float* x, void* y, long long n, void* stream) {
    PU_REQUIRE(x && y && n > 0 && n % 4 == 0, "pu_convert_f32_bf16: n %lld must be a positive multiple of 4", n);
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(stream), x, (__bf16*)y, n / 4);
    return check_launch("pu_convert_f32_bf16");
}

extern "C" int pu_convert_bf16_f32(const void* x, float* y, long long n, void* stream) {
    PU_REQUIRE(x && y && n > 0 && n % 4 == 0, "pu_convert_bf16_f32: n %lld must be a positive multiple of 4", n);
    hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(stream), (const __bf16*)x, y, n / 4);
    return check_launch("pu_convert_bf16_f32");
}

extern "C" int pu_maxpool2_fwd_bf16(const void* x, void* y, int batch, int h, int w, int c, void* stream) {
    PU_REQUIRE(x && y && batch > 0 && h >= 2 && w >= 2 && c > 0 && c % 4 == 0, "pu_maxpool2_fwd_bf16: bad args");
    const int ho = h / 2, wo = w / 2;
    if (c % 8 == 0 && h % 2 == 0 && w % 2 == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0) {
        const long long wt = (long long)batch * ho * wo * (c / 8);
        hipLaunchKernelGGL(maxpool_fwd_win_kernel<__bf16>, dim3(grid_for(wt)), dim3(256), 0, as_stream(stream),
                           (const __bf16*)x, (__bf16*)y, w, c, ho, wo, wt, nullptr);
        return check_launch("pu_maxpool2_fwd_bf16");
    }
    const long long total = (long long)batch * ho * wo * (c / 4);
    hipLaunchKernelGGL((maxpool_fwd_kernel<true, __bf16>), dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                       (const __bf16*)x, (__bf16*)y, h, w, c, ho, wo, total, nullptr);
    return check_launch("pu_maxpool2_fwd_bf16");
}

extern "C" int pu_maxpool2_bwd_bf16(const void* x, const void* dy, void* dx, int batch, int h, int w, int c,
                                    int relu_mask, int accumulate, void* stream) {
    PU_REQUIRE(x && dy && dx && batch > 0 && h >= 2 && w >= 2 && c > 0 && c % 4 == 0, "pu_maxpool2_bwd_bf16: bad args");
    const int ho = h / 2, wo = w / 2;
    if (c % 8 == 0 && h % 2 == 0 && w % 2 == 0 && (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) & 15) == 0) {
        const long long wt = (long long)batch * ho * wo * (c / 8);
        hipLaunchKernelGGL(maxpool_bwd_win_kernel<__bf16>, dim3(grid_for(wt)), dim3(256), 0, as_stream(stream),
                           (const __bf16*)x, (const __bf16*)dy, (__bf16*)dx, w, c, ho, wo, relu_mask, accumulate, wt,
                           nullptr);
        return check_launch("pu_maxpool2_bwd_bf16");
    }
    const long long total = (long long)batch * h * w * (c / 4);
    hipLaunchKernelGGL((maxpool_bwd_kernel<true, __bf16>), dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                       (const __bf16*)x, (const __bf16*)dy, (__bf16*)dx, h, w, c, ho, wo, relu_mask, accumulate, total,
                       nullptr);
    return check_launch("pu_maxpool2_bwd_bf16");
}

extern "C" int pu_outconv_fwd_bf16(const void* x, const float* w, const float* b, float* y, long long rows, int c,
                                   void* stream) {
    PU_REQUIRE(x && w && y && rows > 0 && c > 0 && c % 4 == 0, "pu_outconv_fwd_bf16: bad args");
    const long long groups = (rows + 15) / 16;
    hipLaunchKernelGGL(outconv_fwd_kernel<__bf16>, dim3(grid_for(groups, 1, 8192)), dim3(256), 0, as_stream(stream),
                       (const __bf16*)x, w, b, y, rows, c);
    return check_launch("pu_outconv_fwd_bf16");
}

extern "C" int pu_outconv_bwd_bf16(const void* x, const float* w, const float* dy, void* dx, float* dw, float* db,
                                   long long rows, int c, int relu_mask, void* workspace, size_t ws_bytes, void* stream) {
    PU_REQUIRE(x && w && dy && dx && dw && db && rows > 0 && c % 4 == 0, "pu_outconv_bwd_bf16: bad args");
    const size_t need = pu_outconv_workspace_bytes(rows, c);
    if (!workspace || ws_bytes < need) return fail(PU_ERR_WORKSPACE, "pu_outconv_bwd_bf16: workspace %zu < %zu", ws_bytes, need);
    launch_outconv_bwd<__bf16>((const __bf16*)x, w, dy, (__bf16*)dx, dw, db, (float*)workspace, rows, c, relu_mask,
                               as_stream(stream));
    return check_launch("pu_outconv_bwd_bf16");
}
