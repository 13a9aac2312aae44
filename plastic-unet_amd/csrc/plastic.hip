// The plastic head, its trace update, its backward, and BCELoss.
//
// Reference (yaricom/Plastic-UNet) src/unet/unet_p.py:69-88 (== unet_p_res.py:115-134):
//   activ    = activin.mm(w + alpha*hebb)           -> head_gemm_kernel (Weff built in the loader)
//   activout = sigmoid(activ)
//   hebb'    = Hebb (:82) or Oja (:84) from ROW 0   -> trace_kernel (elementwise, float4)
// and nn.BCELoss (src/train.py:70,101-105) + the autograd backward of all of it (train.py:110).
// Batched over per-slot traces: slot b uses X_b, H_b; w/alpha/eta are shared.
//
// Element-wise formulas keep the reference's operation order with FP contraction off, so the
// trace update is bit-identical to the ATen CPU ops for the same inputs.
#include "common.h"

#include <math.h>

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int HT = 64;   // output tile
constexpr int HK = 16;   // k chunk

// Y[b][i][j] = sigmoid( sum_k X[b][i][k] * (w[k][j] + alpha[k][j]*H[b][k][j]) )
// 256 threads, each a 4x4 micro-tile of the 64x64 block tile.
__global__ __launch_bounds__(256) void head_gemm_kernel(const float* __restrict__ X, const float* __restrict__ H,
                                                        const float* __restrict__ w, const float* __restrict__ alpha,
                                                        float* __restrict__ Y, int N) {
#pragma clang fp contract(off)
    __shared__ float xs[HK][HT + 4];   // xs[k][i]
    __shared__ float ws[HK][HT + 4];   // ws[k][j]
    const int b = blockIdx.z;
    const int i0 = blockIdx.y * HT, j0 = blockIdx.x * HT;
    const float* Xb = X + (long long)b * N * N;
    const float* Hb = H + (long long)b * N * N;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < N; k0 += HK) {
        for (int e = threadIdx.x; e < HK * HT; e += 256) {
            // X tile: row i (64) x k (16), stored transposed
            int kk = e % HK, ii = e / HK;
            int gi = i0 + ii, gk = k0 + kk;
            xs[kk][ii] = (gi < N && gk < N) ? Xb[(long long)gi * N + gk] : 0.f;
            // Weff tile: k (16) x j (64)
            int jj = e % HT, kk2 = e / HT;
            int gj = j0 + jj, gk2 = k0 + kk2;
            float v = 0.f;
            if (gj < N && gk2 < N) {
                long long o = (long long)gk2 * N + gj;
                v = w[o] + alpha[o] * Hb[o];   // torch: w + mul(alpha, hebb) - two roundings
            }
            ws[kk2][jj] = v;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < HK; ++kk) {
            float a[4], bb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { a[q] = xs[kk][ty * 4 + q]; bb[q] = ws[kk][tx * 4 + q]; }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[q][r] = fmaf(a[q], bb[r], acc[q][r]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int gi = i0 + ty * 4 + q;
        if (gi >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int gj = j0 + tx * 4 + r;
            if (gj < N) Y[((long long)b * N + gi) * N + gj] = 1.f / (1.f + expf(-acc[q][r]));
        }
    }
}

// H'[b][k][j] from x0 = X[b][0][k] and y0 = Y[b][0][j]  (unet_p.py:81-86)
__global__ void trace_kernel(const float* __restrict__ H, const float* __restrict__ X, const float* __restrict__ Y,
                             const float* __restrict__ eta_p, float* __restrict__ Hn, int N, long long total, int rule) {
#pragma clang fp contract(off)
    const float eta = eta_p[0];
    const float one_m_eta = 1.f - eta;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long nn = (long long)N * N;
        const long long b = idx / nn;
        const int rem = int(idx - b * nn);
        const int k = rem / N, j = rem - k * N;
        const float h = H[idx];
        const float x0 = X[b * nn + k];
        const float y0 = Y[b * nn + j];
        float out;
        if (rule == PU_RULE_HEBB) {
            out = one_m_eta * h + eta * (x0 * y0);
        } else {
            out = h + eta * ((x0 - h * y0) * y0);
        }
        Hn[idx] = out;
    }
}

// float4 variant for N % 4 == 0 (the bs=32 x 128^2 Oja update measured in bench.py)
__global__ void trace_kernel_v4(const float* __restrict__ H, const float* __restrict__ X, const float* __restrict__ Y,
                                const float* __restrict__ eta_p, float* __restrict__ Hn, int N, long long total4,
                                int rule) {
#pragma clang fp contract(off)
    const float eta = eta_p[0];
    const float one_m_eta = 1.f - eta;
    const int N4 = N >> 2;
    const long long nn = (long long)N * N;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total4;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long row = idx / N4;            // b*N + k
        const int j4 = int(idx - row * N4);
        const long long b = row / N;
        const int k = int(row - b * N);
        const f32x4 h = reinterpret_cast<const f32x4*>(H)[idx];
        const float x0 = X[b * nn + k];
        const f32x4 y0 = *reinterpret_cast<const f32x4*>(Y + b * nn + j4 * 4);
        f32x4 out;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (rule == PU_RULE_HEBB) out[e] = one_m_eta * h[e] + eta * (x0 * y0[e]);
            else out[e] = h[e] + eta * ((x0 - h[e] * y0[e]) * y0[e]);
        }
        reinterpret_cast<f32x4*>(Hn)[idx] = out;
    }
}

// ---------------------------------------------------------------------------------------- backward
// G = dy * (1 - y) * y   (ATen sigmoid_backward: grad * (1 - out) * out)
__device__ __forceinline__ float sig_bwd(float dy, float y) {
#pragma clang fp contract(off)
    return dy * (1.f - y) * y;
}

// dX[b][i][k] = sum_j G[b][i][j] * Weff_b[k][j]
__global__ __launch_bounds__(256) void head_dx_kernel(const float* __restrict__ Yv, const float* __restrict__ dY,
                                                      const float* __restrict__ H, const float* __restrict__ w,
                                                      const float* __restrict__ alpha, float* __restrict__ dX, int N) {
#pragma clang fp contract(off)
    __shared__ float gs[HK][HT + 4];   // gs[j][i]
    __shared__ float ws[HK][HT + 4];   // ws[j][k]
    const int b = blockIdx.z;
    const int i0 = blockIdx.y * HT, k0 = blockIdx.x * HT;
    const long long off = (long long)b * N * N;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float acc[4][4] = {};
    for (int j0 = 0; j0 < N; j0 += HK) {
        for (int e = threadIdx.x; e < HK * HT; e += 256) {
            int jj = e % HK, rr = e / HK;
            int gj = j0 + jj;
            int gi = i0 + rr;
            float g = 0.f;
            if (gi < N && gj < N) {
                long long o = off + (long long)gi * N + gj;
                g = sig_bwd(dY[o], Yv[o]);
            }
            gs[jj][rr] = g;
            int gk = k0 + rr;
            float v = 0.f;
            if (gk < N && gj < N) {
                long long o = (long long)gk * N + gj;
                v = w[o] + alpha[o] * H[off + o];
            }
            ws[jj][rr] = v;
        }
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < HK; ++jj) {
            float a[4], bb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { a[q] = gs[jj][ty * 4 + q]; bb[q] = ws[jj][tx * 4 + q]; }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[q][r] = fmaf(a[q], bb[r], acc[q][r]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int gi = i0 + ty * 4 + q;
        if (gi >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int gk = k0 + tx * 4 + r;
            if (gk < N) dX[off + (long long)gi * N + gk] = acc[q][r];
        }
    }
}

// T_b[k][j] = sum_i X[b][i][k] * G[b][i][j];  partial[z] = (sum_b T_b, sum_b T_b * H_b) over the
// block's slot range.  grid (N/64, N/64, bsplit)
__global__ __launch_bounds__(256) void head_dw_kernel(const float* __restrict__ X, const float* __restrict__ Yv,
                                                      const float* __restrict__ dY, const float* __restrict__ H,
                                                      float* __restrict__ partial, int N, int B, int per) {
#pragma clang fp contract(off)
    __shared__ float xs[HK][HT + 4];   // xs[i][k]
    __shared__ float gs[HK][HT + 4];   // gs[i][j]
    const int k0 = blockIdx.y * HT, j0 = blockIdx.x * HT;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float aw[4][4] = {}, aa[4][4] = {};
    const int b_begin = blockIdx.z * per, b_end = min(B, b_begin + per);
    for (int b = b_begin; b < b_end; ++b) {
        const long long off = (long long)b * N * N;
        float t[4][4] = {};
        for (int i0 = 0; i0 < N; i0 += HK) {
            for (int e = threadIdx.x; e < HK * HT; e += 256) {
                int cc = e % HT, ii = e / HT;
                int gi = i0 + ii;
                int gk = k0 + cc, gj = j0 + cc;
                xs[ii][cc] = (gi < N && gk < N) ? X[off + (long long)gi * N + gk] : 0.f;
                float g = 0.f;
                if (gi < N && gj < N) {
                    long long o = off + (long long)gi * N + gj;
                    g = sig_bwd(dY[o], Yv[o]);
                }
                gs[ii][cc] = g;
            }
            __syncthreads();
#pragma unroll
            for (int ii = 0; ii < HK; ++ii) {
                float a[4], bb[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) { a[q] = xs[ii][ty * 4 + q]; bb[q] = gs[ii][tx * 4 + q]; }
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[q][r] = fmaf(a[q], bb[r], t[q][r]);
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int gk = k0 + ty * 4 + q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int gj = j0 + tx * 4 + r;
                float h = (gk < N && gj < N) ? H[off + (long long)gk * N + gj] : 0.f;
                aw[q][r] = aw[q][r] + t[q][r];
                aa[q][r] = aa[q][r] + t[q][r] * h;
            }
        }
    }
    float* pw = partial + (long long)blockIdx.z * 2 * N * N;
    float* pa = pw + (long long)N * N;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int gk = k0 + ty * 4 + q;
        if (gk >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int gj = j0 + tx * 4 + r;
            if (gj < N) {
                pw[(long long)gk * N + gj] = aw[q][r];
                pa[(long long)gk * N + gj] = aa[q][r];
            }
        }
    }
}

__global__ void head_dw_reduce_kernel(const float* __restrict__ partial, int nsplit, int N, float* __restrict__ dw,
                                      float* __restrict__ da) {
    const long long nn = (long long)N * N;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < nn;
         idx += (long long)gridDim.x * blockDim.x) {
        float sw = 0.f, sa = 0.f;
        for (int z = 0; z < nsplit; ++z) {
            sw += partial[(long long)z * 2 * nn + idx];
            sa += partial[(long long)z * 2 * nn + nn + idx];
        }
        dw[idx] = sw;
        da[idx] = sa;
    }
}

// --------------------------------------------------------------------------------------------- BCE
constexpr int BCE_BLOCKS = 512;

__global__ void bce_partial_kernel(const float* __restrict__ y, const float* __restrict__ t, long long n,
                                   double* __restrict__ partial) {
#pragma clang fp contract(off)
    __shared__ double red[256];
    double s = 0.0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float yy = y[i], tt = t[i];
        // ATen: (t - 1) * max(log1p(-y), -100) - t * max(log(y), -100)
        const float l = (tt - 1.f) * fmaxf(log1pf(-yy), -100.f) - tt * fmaxf(logf(yy), -100.f);
        s += (double)l;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void bce_final_kernel(const double* __restrict__ partial, int np, long long n, float* __restrict__ loss) {
    __shared__ double red[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < np; i += blockDim.x) s += partial[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = (float)(red[0] / (double)n);
}

__global__ void bce_bwd_kernel(const float* __restrict__ y, const float* __restrict__ t, long long n,
                               const float* __restrict__ g, float* __restrict__ dy) {
#pragma clang fp contract(off)
    const float gg = g ? g[0] : 1.f;
    const float inv_n = (float)n;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float yy = y[i], tt = t[i];
        const float d = gg * (yy - tt) / fmaxf((1.f - yy) * yy, 1e-12f);
        dy[i] = d / inv_n;
    }
}

static int grid_for(long long total, int block = 256, int cap = 8192) {
    long long g = (total + block - 1) / block;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

static int head_split(int B) {
    int per = (B + 7) / 8;   // <= 8 partial slabs
    return per < 1 ? 1 : per;
}

}  // namespace pu

using namespace pu;

extern "C" int pu_trace_update(const float* hebb, const float* x, const float* y, const float* eta, float* hebb_out,
                               int batch, int nbf, int rule, void* stream) {
    PU_REQUIRE(hebb && x && y && eta && hebb_out && batch > 0 && nbf > 0, "pu_trace_update: bad args");
    PU_REQUIRE(rule == PU_RULE_HEBB || rule == PU_RULE_OJA, "Must select one learning rule ('hebb' or 'oja')");
    const long long total = (long long)batch * nbf * nbf;
    if (nbf % 4 == 0 && ((((uintptr_t)hebb) | ((uintptr_t)hebb_out) | ((uintptr_t)y)) & 15) == 0) {
        hipLaunchKernelGGL(trace_kernel_v4, dim3(grid_for(total / 4, 256, 16384)), dim3(256), 0, as_stream(stream), hebb,
                           x, y, eta, hebb_out, nbf, total / 4, rule);
    } else {
        hipLaunchKernelGGL(trace_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), hebb, x, y, eta, hebb_out,
                           nbf, total, rule);
    }
    return check_launch("pu_trace_update");
}

extern "C" int pu_plastic_fwd(const pu_plastic_args* a, void* stream) {
    PU_REQUIRE(a && a->x && a->hebb && a->w && a->alpha && a->y && a->batch > 0 && a->nbf > 0, "pu_plastic_fwd: bad args");
    PU_REQUIRE(a->rule == PU_RULE_HEBB || a->rule == PU_RULE_OJA, "Must select one learning rule ('hebb' or 'oja')");
    const int N = a->nbf;
    dim3 grid(ceil_div(N, HT), ceil_div(N, HT), a->batch);
    hipLaunchKernelGGL(head_gemm_kernel, grid, dim3(256), 0, as_stream(stream), a->x, a->hebb, a->w, a->alpha, a->y, N);
    int st = check_launch("pu_plastic_fwd (gemm)");
    if (st != PU_OK || !a->hebb_out) return st;
    PU_REQUIRE(a->eta, "pu_plastic_fwd: eta missing");
    return pu_trace_update(a->hebb, a->x, a->y, a->eta, a->hebb_out, a->batch, N, a->rule, stream);
}

extern "C" size_t pu_plastic_bwd_workspace_bytes(int batch, int nbf) {
    const int per = head_split(batch);
    const int nsplit = (batch + per - 1) / per;
    return (size_t)nsplit * 2 * nbf * nbf * sizeof(float);
}

extern "C" int pu_plastic_bwd(const pu_plastic_bwd_args* a, void* workspace, size_t ws_bytes, void* stream) {
    PU_REQUIRE(a && a->x && a->hebb && a->w && a->alpha && a->y && a->dy && a->batch > 0 && a->nbf > 0,
               "pu_plastic_bwd: bad args");
    const int N = a->nbf, B = a->batch;
    hipStream_t s = as_stream(stream);
    if (a->dx) {
        dim3 grid(ceil_div(N, HT), ceil_div(N, HT), B);
        hipLaunchKernelGGL(head_dx_kernel, grid, dim3(256), 0, s, a->y, a->dy, a->hebb, a->w, a->alpha, a->dx, N);
        int st = check_launch("pu_plastic_bwd (dx)");
        if (st != PU_OK) return st;
    }
    if (a->dw || a->dalpha) {
        PU_REQUIRE(a->dw && a->dalpha, "pu_plastic_bwd: dw and dalpha go together");
        const size_t need = pu_plastic_bwd_workspace_bytes(B, N);
        if (!workspace || ws_bytes < need) return fail(PU_ERR_WORKSPACE, "pu_plastic_bwd: workspace %zu < %zu", ws_bytes, need);
        const int per = head_split(B);
        const int nsplit = (B + per - 1) / per;
        dim3 grid(ceil_div(N, HT), ceil_div(N, HT), nsplit);
        hipLaunchKernelGGL(head_dw_kernel, grid, dim3(256), 0, s, a->x, a->y, a->dy, a->hebb, (float*)workspace, N, B, per);
        hipLaunchKernelGGL(head_dw_reduce_kernel, dim3(grid_for((long long)N * N)), dim3(256), 0, s,
                           (const float*)workspace, nsplit, N, a->dw, a->dalpha);
    }
    return check_launch("pu_plastic_bwd (dw)");
}

extern "C" size_t pu_bce_workspace_bytes(long long n) {
    (void)n;
    return BCE_BLOCKS * sizeof(double);
}

extern "C" int pu_bce_fwd(const float* y, const float* t, long long n, float* loss, void* workspace, size_t ws_bytes,
                          void* stream) {
    PU_REQUIRE(y && t && loss && n > 0, "pu_bce_fwd: bad args");
    if (!workspace || ws_bytes < pu_bce_workspace_bytes(n)) return fail(PU_ERR_WORKSPACE, "pu_bce_fwd: workspace");
    int blocks = grid_for(n, 256, BCE_BLOCKS);
    hipLaunchKernelGGL(bce_partial_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), y, t, n, (double*)workspace);
    hipLaunchKernelGGL(bce_final_kernel, dim3(1), dim3(256), 0, as_stream(stream), (const double*)workspace, blocks, n,
                       loss);
    return check_launch("pu_bce_fwd");
}

extern "C" int pu_bce_bwd(const float* y, const float* t, long long n, const float* grad_loss, float* dy, void* stream) {
    PU_REQUIRE(y && t && dy && n > 0, "pu_bce_bwd: bad args");
    hipLaunchKernelGGL(bce_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), y, t, n, grad_loss, dy);
    return check_launch("pu_bce_bwd");
}
