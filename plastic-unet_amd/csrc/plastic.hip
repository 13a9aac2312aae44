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

constexpr int HK = 16;   // k chunk staged through LDS

// Tile T x T per 256-thread block (T = 64: 4x4 per thread; T = 32: 2x2, for grids that would not
// fill the chip, e.g. bs 32 x 128^2 -> 512 blocks instead of 128).
template <int T> struct HeadTile {
    static constexpr int M = T / 16;   // micro-tile side
};

__device__ __forceinline__ float trace_rule(float h, float x0, float y0, float eta, float one_m_eta, int rule) {
#pragma clang fp contract(off)
    // unet_p.py:82 (Hebb) and :84 (Oja), in the reference's operation order
    return rule == PU_RULE_HEBB ? one_m_eta * h + eta * (x0 * y0) : h + eta * ((x0 - h * y0) * y0);
}

// Y[b][i][j] = sigmoid( sum_k X[b][i][k] * (w[k][j] + alpha[k][j]*H[b][k][j]) )     (unet_p.py:70-79)
// With Hn != nullptr the trace update is fused in: every block also accumulates row 0 of its
// column tile (y0 = Y[b][0][j0:j0+T], the same fmaf chain as the block that owns row 0, so the
// values are identical) and then writes H'[b][k][j] for its own T x T tile with k in the tile's
// row range: H is read from HBM once for Weff and re-read from L2 for the update; one launch.
// Hn must not alias H (other blocks still read H).  grid (N/T, N/T, B)
template <int T>
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ X, const float* __restrict__ H,
                                                       const float* __restrict__ w, const float* __restrict__ alpha,
                                                       float* __restrict__ Y, float* __restrict__ Hn,
                                                       const float* __restrict__ eta_p, int N, int rule) {
#pragma clang fp contract(off)
    constexpr int M = HeadTile<T>::M;
    __shared__ float xs[HK][T + 4];    // xs[k][i]
    __shared__ float ws[HK][T + 4];    // ws[k][j]
    __shared__ float x0s[HK];          // X[b][0][k]
    __shared__ float y0s[T];
    const int b = blockIdx.z;
    const int i0 = blockIdx.y * T, j0 = blockIdx.x * T;
    const float* Xb = X + (long long)b * N * N;
    const float* Hb = H + (long long)b * N * N;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const bool fuse = Hn != nullptr;
    float acc[M][M] = {};
    float acc0[M] = {};
    for (int k0 = 0; k0 < N; k0 += HK) {
        for (int e = threadIdx.x; e < HK * T; e += 256) {
            int kk = e % HK, ii = e / HK;               // X tile: row i x k, stored transposed
            int gi = i0 + ii, gk = k0 + kk;
            xs[kk][ii] = (gi < N && gk < N) ? Xb[(long long)gi * N + gk] : 0.f;
            int jj = e % T, kk2 = e / T;                // Weff tile: k x j
            int gj = j0 + jj, gk2 = k0 + kk2;
            float v = 0.f;
            if (gj < N && gk2 < N) {
                long long o = (long long)gk2 * N + gj;
                v = w[o] + alpha[o] * Hb[o];   // torch: w + mul(alpha, hebb) - two roundings
            }
            ws[kk2][jj] = v;
        }
        if (fuse && threadIdx.x < HK) x0s[threadIdx.x] = (k0 + threadIdx.x < N) ? Xb[k0 + threadIdx.x] : 0.f;
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < HK; ++kk) {
            float a[M], bb[M];
#pragma unroll
            for (int q = 0; q < M; ++q) { a[q] = xs[kk][ty * M + q]; bb[q] = ws[kk][tx * M + q]; }
#pragma unroll
            for (int q = 0; q < M; ++q)
#pragma unroll
                for (int r = 0; r < M; ++r) acc[q][r] = fmaf(a[q], bb[r], acc[q][r]);
            if (fuse && ty == 0) {
                const float a0 = x0s[kk];
#pragma unroll
                for (int r = 0; r < M; ++r) acc0[r] = fmaf(a0, bb[r], acc0[r]);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < M; ++q) {
        int gi = i0 + ty * M + q;
        if (gi >= N) continue;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            int gj = j0 + tx * M + r;
            if (gj < N) Y[((long long)b * N + gi) * N + gj] = 1.f / (1.f + expf(-acc[q][r]));
        }
    }
    if (!fuse) return;
    if (ty == 0) {
#pragma unroll
        for (int r = 0; r < M; ++r) y0s[tx * M + r] = 1.f / (1.f + expf(-acc0[r]));
    }
    __syncthreads();
    const float eta = eta_p[0];
    const float one_m_eta = 1.f - eta;
    float* Hnb = Hn + (long long)b * N * N;
    // H' rows k = i0.. (the tile's row range), columns j0..: coalesced over j
    for (int e = threadIdx.x; e < T * T; e += 256) {
        const int kk = e / T, jj = e % T;
        const int gk = i0 + kk, gj = j0 + jj;
        if (gk < N && gj < N) {
            const long long o = (long long)gk * N + gj;
            Hnb[o] = trace_rule(Hb[o], Xb[gk], y0s[jj], eta, one_m_eta, rule);
        }
    }
}

// H'[b][k][j] from x0 = X[b][0][k] and y0 = Y[b][0][j]  (unet_p.py:81-86); the stand-alone update
// (pu_trace_update).  grid (ceil(N*N/4 / 256), B): one float4 per thread, 32-bit indexing
__global__ void trace_kernel(const float* __restrict__ H, const float* __restrict__ X, const float* __restrict__ Y,
                             const float* __restrict__ eta_p, float* __restrict__ Hn, int N, int rule) {
#pragma clang fp contract(off)
    const float eta = eta_p[0];
    const float one_m_eta = 1.f - eta;
    const long long off = (long long)blockIdx.y * N * N;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= N * N) return;
    const int k = idx / N, j = idx - k * N;
    Hn[off + idx] = trace_rule(H[off + idx], X[off + k], Y[off + j], eta, one_m_eta, rule);
}

__global__ void trace_kernel_v4(const float* __restrict__ H, const float* __restrict__ X, const float* __restrict__ Y,
                                const float* __restrict__ eta_p, float* __restrict__ Hn, int N, int rule) {
#pragma clang fp contract(off)
    const float eta = eta_p[0];
    const float one_m_eta = 1.f - eta;
    const int N4 = N >> 2;
    const long long off = (long long)blockIdx.y * N * N;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;    // float4 index within the slot
    if (idx >= N * N4) return;
    const int k = idx / N4, j4 = idx - k * N4;
    const f32x4 h = reinterpret_cast<const f32x4*>(H + off)[idx];
    const float x0 = X[off + k];
    const f32x4 y0 = *reinterpret_cast<const f32x4*>(Y + off + j4 * 4);
    f32x4 out;
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = trace_rule(h[e], x0, y0[e], eta, one_m_eta, rule);
    reinterpret_cast<f32x4*>(Hn + off)[idx] = out;
}


// ------------------------------------------------------------------- fused head (outconv + head)
// One block (512 threads, two per CU at N = 128) = 16 rows i0..i0+15 of slot b, all N columns.  Phases:
//  1. outconv of the block's 16 rows and of row 0 (x0, needed by the trace update) into LDS:
//     L lanes per pixel (L = C/4 up to 16), float4 channel loads, U pixels per lane group in
//     flight, dot4_fma + xor-tree over the L lanes - the arithmetic of outconv_fwd_kernel (whose
//     idle lanes add zeros), so X is bit-identical to the two-launch path;
//  2. Weff_b = w + alpha (.) H_b in chunks of kc rows through LDS (all of it at N <= 128); Y = X Weff
//     on v_mfma_f32_16x16x4_f32 (column tile t -> wave t mod 8) and y0 = x0 Weff as a VALU fmaf
//     chain in the same k order (== the MFMA's, bitwise), so every block holds row 0's Y;
//  3. Y = sigmoid, X rows written out (the backward's input);
//  4. H'[k][j] for the block's rows k from H, x0[k], y0[j] (unet_p.py:81-86 operation order).
#ifndef PU_FH_R
#define PU_FH_R 16
#endif
constexpr int FH_R = PU_FH_R; // rows per block (8: rows 8..15 of the 16-row MFMA tiles are discarded)
static_assert(FH_R == 8 || FH_R == 16, "rows per block");
constexpr int FH_NT = 512;    // threads per block (2 blocks per CU at nbf 128: one block's feature
                               // loads overlap the other's GEMM / trace phases)
constexpr int FH_WAVES = FH_NT / 64;
constexpr int FH_LDS_W = 16384;   // floats of the Weff chunk (64 KB)
#ifndef PU_FH_ABL
#define PU_FH_ABL 0               // ablation builds only: 1 = stop after the outconv phase
#endif
#ifndef PU_FH_LDS_MIN
#define PU_FH_LDS_MIN 0           // ablation builds only: pad the LDS request (blocks per CU)
#endif
#ifndef PU_FH_U
#define PU_FH_U 8                 // pixels per lane group in flight (L >= 8)
#endif

// Weff rows per LDS chunk: all N rows when N x N fits, else the largest multiple of 4 (the MFMA's
// k step) that divides N and fits (N % 16 == 0, so 16 always qualifies: N = 144 -> 72, 192 -> 64,
// 320 -> 40, 384 -> 32, 512 -> 32).  The chunk loop steps k0 by kc up to N, so kc must divide N.
inline int fused_head_chunk(int N) {
    if (N * N <= FH_LDS_W) return N;
    int best = 16;
    for (int d = 4; d * N <= FH_LDS_W && d <= N; d += 4)
        if (N % d == 0) best = d;
    return best;
}

template <typename T>
__device__ __forceinline__ f32x4 fh_ld4(const T* p);
template <>
__device__ __forceinline__ f32x4 fh_ld4<float>(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
template <>
__device__ __forceinline__ f32x4 fh_ld4<__bf16>(const __bf16* p) {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    const b4 v = *reinterpret_cast<const b4*>(p);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
// the pipelined head's feature stream: every feature is read once (row 0 aside), so the
// nontemporal form (PU_HP_NT=1) keeps it from displacing H / w / alpha in the caches
#ifndef PU_HP_NT
#define PU_HP_NT 0
#endif
template <typename T>
__device__ __forceinline__ f32x4 fh_ld4s(const T* p) {
    if constexpr (PU_HP_NT && sizeof(T) == 4) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return fh_ld4<T>(p);
}

template <typename T, int L, int TPW, int R = FH_R>
__global__ __launch_bounds__(FH_NT) void head_fused_fwd_kernel(const T* __restrict__ feat, const float* __restrict__ wo,
                                                               const float* __restrict__ bo, int C,
                                                               const float* __restrict__ H, const float* __restrict__ w,
                                                               const float* __restrict__ alpha,
                                                               const float* __restrict__ eta_p, float* __restrict__ X,
                                                               float* __restrict__ Y, float* __restrict__ Hn, int N,
                                                               FastDiv dN, int kc, int rule) {
    constexpr int RT = (R + 15) / 16;         // 16-row MFMA tiles of the block's rows
    extern __shared__ float fh_lds[];
    float* xs = fh_lds;                       // [R + 1][N]: own rows, then row 0
    float* ws = xs + (R + 1) * N;             // [kc][N]
    float* y0s = ws + kc * N;                 // [N]
    const int b = blockIdx.y;
    const int i0 = blockIdx.x * R;
    const int tid = threadIdx.x;
    const bool fuse = Hn != nullptr;
    const long long nn = (long long)N * N;
    const T* fb = feat + (long long)b * nn * C;
    const float* Hb = H + (long long)b * nn;

    // ---- 1. outconv
    {
        constexpr int U = L >= 8 ? 8 : 4;       // pixels per lane group in flight
        const float bias = bo ? bo[0] : 0.f;
        const int lane = tid % L;
        constexpr int PPP = FH_NT / L;          // pixels per pass
        const int npix = (fuse ? R + 1 : R) * N;
        auto reduce_store = [&](int q0, float (&s)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float t = s[u];
                if (L >= 16) t += __shfl_xor(t, 8, 16);
                if (L >= 8) t += __shfl_xor(t, 4, 16);
                if (L >= 4) t += __shfl_xor(t, 2, 16);
                if (L >= 2) t += __shfl_xor(t, 1, 16);
                const int q = q0 + u * PPP;
                if (lane == 0 && q < npix) xs[q] = t + bias;
            }
        };
        auto pixel = [&](int q) -> const T* {
            q = min(q, npix - 1);
            const int r = (int)fdiv((unsigned)q, dN), k = q - r * N;
            return fb + ((long long)(r < R ? i0 + r : 0) * N + k) * C;
        };
        for (int q0 = tid / L; q0 < npix; q0 += U * PPP) {
            const T* px[U];
#pragma unroll
            for (int u = 0; u < U; ++u) px[u] = pixel(q0 + u * PPP);
            float sacc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) sacc[u] = 0.f;
            for (int c = lane * 4; c < C; c += 4 * L) {
                const f32x4 ww = *reinterpret_cast<const f32x4*>(wo + c);
                f32x4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = fh_ld4<T>(px[u] + c);
#pragma unroll
                for (int u = 0; u < U; ++u) sacc[u] += dot4_fma(v[u], ww);
            }
            reduce_store(q0, sacc);
        }
    }
    __syncthreads();
    // X rows of this block -> global (coalesced)
    for (int e = tid; e < R * N; e += FH_NT) X[(long long)b * nn + (long long)i0 * N + e] = xs[e];
    if (PU_FH_ABL == 1) return;

    // the trace update's first float4 of H (rows i0.., L2-resident after the Weff build), in
    // flight during the GEMM
    f32x4 hpre = f32x4{0.f, 0.f, 0.f, 0.f};
    if (fuse && tid < R * N / 4) hpre = reinterpret_cast<const f32x4*>(Hb + (long long)i0 * N)[tid];

    // ---- 2. GEMM
    const int wave = tid >> 6, l = tid & 63;
    const int tiles = N / 16;
    f32x4 acc[TPW][RT];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[t][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float acc0 = 0.f;                                  // y0 chain of column tid (tid < N)
    for (int k0 = 0; k0 < N; k0 += kc) {
        {
#pragma clang fp contract(off)
            // float4 pieces, 8 per array and thread in flight at once (N = 128: the whole chunk in
            // one round trip; the scalar form took four, 4.4 us of the kernel by ablation)
            const int ne4 = kc * N / 4;
            const f32x4* w4 = reinterpret_cast<const f32x4*>(w + (long long)k0 * N);
            const f32x4* a4 = reinterpret_cast<const f32x4*>(alpha + (long long)k0 * N);
            const f32x4* h4 = reinterpret_cast<const f32x4*>(Hb + (long long)k0 * N);
            for (int e0 = tid; e0 < ne4; e0 += 8 * FH_NT) {
                f32x4 wv[8], av[8], hv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int o = min(e0 + FH_NT * u, ne4 - 1);
                    wv[u] = w4[o]; av[u] = a4[o]; hv[u] = h4[o];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (e0 + FH_NT * u < ne4) {
                        f32x4 o;
#pragma unroll
                        for (int c = 0; c < 4; ++c) o[c] = wv[u][c] + av[u][c] * hv[u][c];   // torch: w + mul(alpha, hebb)
                        reinterpret_cast<f32x4*>(ws)[e0 + FH_NT * u] = o;
                    }
            }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < TPW && PU_FH_ABL != 2; ++t) {
            const int tile = wave + FH_WAVES * t;
            if (tile < tiles) {
                const float* wcol = ws + (l >> 4) * N + tile * 16 + (l & 15);
                const float* xrow = xs + (l & 15) * N + k0 + (l >> 4);   // row tile rt: + 16 rt N
                // operands of 4 k-steps read before their MFMAs (kc % 16 == 0 or kc = 4 .. 12: see
                // fused_head_chunk - the tail loop takes the rest); each W fragment feeds RT tiles
                int kk = 0;
                for (; kk + 16 <= kc; kk += 16) {
                    float xa[RT][4], wb[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        wb[j] = wcol[(kk + 4 * j) * N];
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) xa[rt][j] = xrow[16 * rt * N + kk + 4 * j];
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt)
                            acc[t][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[rt][j], wb[j], acc[t][rt], 0, 0, 0);
                }
                for (; kk < kc; kk += 4)
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt)
                        acc[t][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(xrow[16 * rt * N + kk], wcol[kk * N], acc[t][rt], 0, 0, 0);
            }
        }
        if (fuse && tid < N && PU_FH_ABL != 2) {
            // the same k-ordered fmaf chain; 8 k's operands read ahead of their fmas
            float s0 = acc0;
            int kk = 0;
            for (; kk + 8 <= kc; kk += 8) {
                float xa[8], wb[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) { xa[j] = xs[R * N + k0 + kk + j]; wb[j] = ws[(kk + j) * N + tid]; }
#pragma unroll
                for (int j = 0; j < 8; ++j) s0 = fmaf(xa[j], wb[j], s0);
            }
            for (; kk < kc; ++kk) s0 = fmaf(xs[R * N + k0 + kk], ws[kk * N + tid], s0);
            acc0 = s0;
        }
        __syncthreads();
    }

    if (PU_FH_ABL == 3) return;
    // ---- 3. sigmoid + store (C layout of 16x16: column l & 15, rows 4 (l >> 4) + reg)
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int tile = wave + FH_WAVES * t;
        if (tile < tiles) {
            const int j = tile * 16 + (l & 15);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                if (16 * rt + 4 * (l >> 4) < R) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int gi = i0 + 16 * rt + 4 * (l >> 4) + r;
                        Y[((long long)b * N + gi) * N + j] = 1.f / (1.f + expf(-acc[t][rt][r]));
                    }
                }
            }
        }
    }
    if (!fuse || PU_FH_ABL == 4) return;
    if (tid < N) y0s[tid] = 1.f / (1.f + expf(-acc0));
    __syncthreads();

    // ---- 4. trace update of rows k = i0 .. i0+15
    const float eta = eta_p[0];
    const float one_m_eta = 1.f - eta;
    // rows i0 .. i0+R-1 of H / H' are contiguous: float4 over the block's R * N elements
    const f32x4* Hr = reinterpret_cast<const f32x4*>(Hb + (long long)i0 * N);
    f32x4* Hnr = reinterpret_cast<f32x4*>(Hn + (long long)b * nn + (long long)i0 * N);
    for (int e4 = tid; e4 < R * N / 4; e4 += FH_NT) {
        const f32x4 h = e4 == tid ? hpre : Hr[e4];
        const int kk = (int)fdiv((unsigned)(4 * e4), dN), j = 4 * e4 - kk * N;
        const float x0 = xs[R * N + i0 + kk];
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = trace_rule(h[e], x0, y0s[j + e], eta, one_m_eta, rule);
        Hnr[e4] = o;
    }
}

// ------------------------------------------------------- fused head, pipelined (N = 128, L = 16)
// head_fused_fwd_kernel runs its phases one after the other on all 8 waves: the feature stream
// (outconv, 26.5 us of its 35.7 at bs 32 x 128^2 x 64 channels), then Weff / GEMM / y0 / the
// trace update (9 us of latency chains) - with one block per CU nothing overlaps that tail.  Here
// 12 waves split the roles:
//   waves 0..7 (streamers, the serial kernel's outconv configuration and per-CU stream rate): one
//     continuous stream over the 17 rows in the order row 0, i0 .. i0+15, 256 pixels per pass with
//     the next pass's loads issued before the current pass is reduced - so the block barriers
//     between phases (every 2 passes = 2 rows at U = 4) do not drain the memory pipeline;
//   waves 8..11 (workers): phase 0 builds Weff = w + alpha (.) H_b in LDS; after every phase they
//     form Y = X Weff for the rows just streamed (thread = (column j, row), one k-ordered
//     fmaf chain per row - the MFMA's chain, bit-identical), sigmoid, store; the phase after row 0's
//     y0 runs the block's trace update.
// What is left after the stream is one row's GEMM.  Arithmetic identical to head_fused_fwd_kernel
// (the same outconv lane tree, k order, sigmoid and trace expressions).
#ifndef PU_HP_SW
#define PU_HP_SW 8
#endif
#ifndef PU_HP_ROT
#define PU_HP_ROT 0        // 1: per-block column rotation of the stream start (measured 2-4 % slower at U = 4)
#endif
#ifndef PU_HP_U
#define PU_HP_U 4          // pixels in flight per streamer lane group and pass (4: one row per pass)
#endif
constexpr int HP_SW = PU_HP_SW * 64, HP_NT = HP_SW + 256, HP_U = PU_HP_U, HP_N = 128;
template <typename T>
__global__ __launch_bounds__(HP_NT) void head_pipe_fwd_kernel(const T* __restrict__ feat, const float* __restrict__ wo,
                                                              const float* __restrict__ bo, int C,
                                                              const float* __restrict__ H, const float* __restrict__ w,
                                                              const float* __restrict__ alpha,
                                                              const float* __restrict__ eta_p, float* __restrict__ X,
                                                              float* __restrict__ Y, float* __restrict__ Hn, int rule) {
#pragma clang fp contract(off)
    constexpr int N = HP_N, L = 16, R = 16;
    constexpr int PPP = HP_SW / L;            // pixels per lane-group round
    constexpr int PPI = HP_U * PPP;           // pixels per pass
    constexpr int NPIX = (R + 1) * N;         // the stream: row 0, then rows i0 .. i0+15
    constexpr int NPASS = (NPIX + PPI - 1) / PPI;
    constexpr int NPH = (NPASS + 1) / 2;      // phases (2 passes each)
    constexpr int RPP = 2 * PPI / N;          // stream rows per phase (2 with 8 streamer waves at U = 4)
    constexpr int RPT = RPP / 2;              // rows per worker thread and phase
    static_assert(PPI % N == 0 && RPT <= 3, "a pass is whole rows");
    static_assert(N / R == 8, "the XCD block order below assumes 8 row blocks per slot");
    __shared__ __attribute__((aligned(16))) float xs[(R + 1) * N];   // stream order: row 0, then own rows
    __shared__ __attribute__((aligned(16))) float ws[N * N];
    __shared__ float y0s[N];
    // XCD-aware block order: blocks are dealt round-robin over the 8 XCDs by linear id, so the
    // plain (row block, slot) grid put row block x of EVERY slot on XCD x and each XCD's L2 fetched
    // every slot's H_b (W_eff) and row-0 features - 8x per slot.  Unit u = xcd * B + (lin / 8)
    // gives each XCD a contiguous run of units: the 8 row blocks of a slot share one XCD (B % 8 ==
    // 0; otherwise at most one slot straddles two).  A bijection on [0, 8B): speed only, the
    // per-block arithmetic does not depend on the placement.
    const int nslot = gridDim.y;
    const int lin = blockIdx.x + (N / R) * blockIdx.y;
    const int unit = (lin & 7) * nslot + (lin >> 3);
    const int b = unit / (N / R);
    const int rb = unit % (N / R);
    const int i0 = rb * R;
    const int tid = threadIdx.x;
    const bool streamer = tid < HP_SW;        // wave-uniform
    const long long nn = (long long)N * N;
    const T* fb = feat + (long long)b * nn * C;
    const float* Hb = H + (long long)b * nn;

    if (streamer) {
        const float bias = bo ? bo[0] : 0.f;
        const int lane = tid % L;
        // column rotation per block: the 256 blocks' streams start at staggered addresses
        const int rot = PU_HP_ROT ? (int)((rb * 8 + b) * 37u) & (N - 1) : 0;
        f32x4 buf[2][HP_U];
        // pixels of pass k (stream order q -> image row: q / N == 0 ? 0 : i0 + q / N - 1)
        auto load = [&](int k, f32x4 (&v)[HP_U]) {
#pragma unroll
            for (int u = 0; u < HP_U; ++u) {
                const int q = min(k * PPI + tid / L + u * PPP, NPIX - 1);
                const int r = q / N, col = (q + rot) & (N - 1);
                const T* px = fb + ((long long)(r == 0 ? 0 : i0 + r - 1) * N + col) * C;
                v[u] = fh_ld4s<T>(px + lane * 4);
            }
        };
        const f32x4 ww = *reinterpret_cast<const f32x4*>(wo + lane * 4);
        // reduce pass k from registers v (the next pass's loads already in flight)
        auto reduce = [&](int k, const f32x4 (&v)[HP_U]) {
#pragma unroll
            for (int u = 0; u < HP_U; ++u) {
                const int q = k * PPI + tid / L + u * PPP;
                float sacc = 0.f;
                sacc += dot4_fma(v[u], ww);
                if (C > 4 * L) {                  // channels beyond the first 64 (not prefetched)
                    const int qc = min(q, NPIX - 1);
                    const int r = qc / N, col = (qc + rot) & (N - 1);
                    const T* px = fb + ((long long)(r == 0 ? 0 : i0 + r - 1) * N + col) * C;
                    for (int c = lane * 4 + 4 * L; c < C; c += 4 * L)
                        sacc += dot4_fma(fh_ld4<T>(px + c), *reinterpret_cast<const f32x4*>(wo + c));
                }
                float t = sacc;
                t += __shfl_xor(t, 8, 16);
                t += __shfl_xor(t, 4, 16);
                t += __shfl_xor(t, 2, 16);
                t += __shfl_xor(t, 1, 16);
                if (lane == 0 && q < NPIX) xs[(q & ~(N - 1)) + ((q + rot) & (N - 1))] = t + bias;
            }
        };
        // passes in pairs (static buffer roles): a phase = 2 passes = 2 rows, then the barrier
        load(0, buf[0]);
#pragma unroll 1
        for (int k = 0; k < NPASS; k += 2) {
            if (k + 1 < NPASS) load(k + 1, buf[1]);
            reduce(k, buf[0]);
            if (k + 1 < NPASS) {
                if (k + 2 < NPASS) load(k + 2, buf[0]);
                reduce(k + 1, buf[1]);
            }
            __syncthreads();                  // this phase's rows are in xs
        }
        // X rows out (stream rows 1 .. 16 = image rows i0 .. i0+15)
        for (int e = tid; e < R * N; e += HP_SW) X[(long long)b * nn + (long long)i0 * N + e] = xs[N + e];
    } else {
        const int tw = tid - HP_SW;           // 0 .. 255
        const int j = tw & (N - 1), rh = tw >> 7;
        // phase 0: Weff
        {
            const f32x4* w4 = reinterpret_cast<const f32x4*>(w);
            const f32x4* a4 = reinterpret_cast<const f32x4*>(alpha);
            const f32x4* h4 = reinterpret_cast<const f32x4*>(Hb);
            for (int e0 = tw; e0 < N * N / 4; e0 += 8 * 256) {
                f32x4 wv[8], av[8], hv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int o = e0 + 256 * u;
                    wv[u] = w4[o]; av[u] = a4[o]; hv[u] = h4[o];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    f32x4 o;
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[c] = wv[u][c] + av[u][c] * hv[u][c];   // torch: w + mul(alpha, hebb)
                    reinterpret_cast<f32x4*>(ws)[e0 + 256 * u] = o;
                }
            }
        }
        for (int ph = 0; ph < NPH; ++ph) {
            __syncthreads();                  // phase ph's stream rows are in xs
            // Y of stream rows RPP ph + RPT rh .. (stream row 0 = image row 0 -> y0 only)
            const int s0 = RPP * ph + RPT * rh;
            const int nrow = max(0, min(RPT, R + 1 - s0));
            if (nrow > 0) {
                float acc[RPT];
#pragma unroll
                for (int r = 0; r < RPT; ++r) acc[r] = 0.f;
                for (int k = 0; k < N; k += 4) {
                    float wk[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) wk[e] = ws[(k + e) * N + j];
#pragma unroll
                    for (int r = 0; r < RPT; ++r)
                        if (r < nrow) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) acc[r] = fmaf(xs[(s0 + r) * N + k + e], wk[e], acc[r]);
                        }
                }
#pragma unroll
                for (int r = 0; r < RPT; ++r)
                    if (r < nrow) {
                        const float y = 1.f / (1.f + expf(-acc[r]));
                        if (s0 + r == 0) y0s[j] = y;
                        else Y[((long long)b * N + i0 + s0 + r - 1) * N + j] = y;
                    }
            }
            if (ph == 1) {                    // (RPP >= 2: y0 was formed in phase 0)
                // trace update of rows i0 .. i0+15 (y0 formed in phase 0's GEMM - complete at this
                // phase's barrier -, x0 = stream row 0)
                const float eta = eta_p[0];
                const float one_m_eta = 1.f - eta;
                const f32x4* Hr = reinterpret_cast<const f32x4*>(Hb + (long long)i0 * N);
                f32x4* Hnr = reinterpret_cast<f32x4*>(Hn + (long long)b * nn + (long long)i0 * N);
                for (int e4 = tw; e4 < R * N / 4; e4 += 256) {
                    const f32x4 h = Hr[e4];
                    const int kk = (4 * e4) / N, jj = 4 * e4 - kk * N;
                    const float x0 = xs[i0 + kk];
                    f32x4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = trace_rule(h[e], x0, y0s[jj + e], eta, one_m_eta, rule);
                    Hnr[e4] = o;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------- backward
// G = dy * (1 - y) * y   (ATen sigmoid_backward: grad * (1 - out) * out)
__device__ __forceinline__ float sig_bwd(float dy, float y) {
#pragma clang fp contract(off)
    return dy * (1.f - y) * y;
}

// dX[b][i][k] = sum_j G[b][i][j] * Weff_b[k][j]      grid (N/T, N/T, B)
template <int T>
__global__ __launch_bounds__(256) void head_dx_kernel(const float* __restrict__ Yv, const float* __restrict__ dY,
                                                      const float* __restrict__ H, const float* __restrict__ w,
                                                      const float* __restrict__ alpha, float* __restrict__ dX, int N) {
#pragma clang fp contract(off)
    constexpr int M = HeadTile<T>::M;
    __shared__ float gs[HK][T + 4];   // gs[j][i]
    __shared__ float ws[HK][T + 4];   // ws[j][k]
    const int b = blockIdx.z;
    const int i0 = blockIdx.y * T, k0 = blockIdx.x * T;
    const long long off = (long long)b * N * N;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float acc[M][M] = {};
    // the next chunk's operands are loaded into registers before this chunk's FMAs (raw values;
    // out-of-range entries load as 0, which the expressions below map to the 0 the tile needs)
    constexpr int E = HK * T / 256;
    static_assert(HK * T % 256 == 0, "whole loader rounds");
    float rdy[E], ryv[E], rw[E], ra[E], rh[E];
    auto fetch = [&](int j0) {
#pragma unroll
        for (int u = 0; u < E; ++u) {
            const int e = threadIdx.x + 256 * u;
            const int jj = e % HK, rr = e / HK;
            const int gj = j0 + jj, gi = i0 + rr, gk = k0 + rr;
            rdy[u] = ryv[u] = rw[u] = ra[u] = rh[u] = 0.f;
            if (gi < N && gj < N) {
                const long long o = off + (long long)gi * N + gj;
                rdy[u] = dY[o];
                ryv[u] = Yv[o];
            }
            if (gk < N && gj < N) {
                const long long o = (long long)gk * N + gj;
                rw[u] = w[o];
                ra[u] = alpha[o];
                rh[u] = H[off + o];
            }
        }
    };
    fetch(0);
    for (int j0 = 0; j0 < N; j0 += HK) {
#pragma unroll
        for (int u = 0; u < E; ++u) {
            const int e = threadIdx.x + 256 * u;
            const int jj = e % HK, rr = e / HK;
            gs[jj][rr] = sig_bwd(rdy[u], ryv[u]);
            ws[jj][rr] = rw[u] + ra[u] * rh[u];
        }
        __syncthreads();
        if (j0 + HK < N) fetch(j0 + HK);
#pragma unroll
        for (int jj = 0; jj < HK; ++jj) {
            float a[M], bb[M];
#pragma unroll
            for (int q = 0; q < M; ++q) { a[q] = gs[jj][ty * M + q]; bb[q] = ws[jj][tx * M + q]; }
#pragma unroll
            for (int q = 0; q < M; ++q)
#pragma unroll
                for (int r = 0; r < M; ++r) acc[q][r] = fmaf(a[q], bb[r], acc[q][r]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < M; ++q) {
        int gi = i0 + ty * M + q;
        if (gi >= N) continue;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            int gk = k0 + tx * M + r;
            if (gk < N) dX[off + (long long)gi * N + gk] = acc[q][r];
        }
    }
}

// T_b[k][j] = sum_i X[b][i][k] * G[b][i][j];  per slot: partial[b] = (T_b, T_b * H_b).
// grid (N/T, N/T, B); the slot sum is a separate fixed-order pass (deterministic)
template <int T>
__global__ __launch_bounds__(256) void head_dw_kernel(const float* __restrict__ X, const float* __restrict__ Yv,
                                                      const float* __restrict__ dY, const float* __restrict__ H,
                                                      float* __restrict__ partial, int N) {
#pragma clang fp contract(off)
    constexpr int M = HeadTile<T>::M;
    __shared__ float xs[HK][T + 4];   // xs[i][k]
    __shared__ float gs[HK][T + 4];   // gs[i][j]
    const int k0 = blockIdx.y * T, j0 = blockIdx.x * T;
    const int b = blockIdx.z;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const long long off = (long long)b * N * N;
    float t[M][M] = {};
    // next chunk's raw operands in registers during this chunk's FMAs (as head_dx_kernel)
    constexpr int E = HK * T / 256;
    static_assert(HK * T % 256 == 0, "whole loader rounds");
    float rx[E], rdy[E], ryv[E];
    auto fetch = [&](int i0) {
#pragma unroll
        for (int u = 0; u < E; ++u) {
            const int e = threadIdx.x + 256 * u;
            const int cc = e % T, ii = e / T;
            const int gi = i0 + ii, gk = k0 + cc, gj = j0 + cc;
            rx[u] = (gi < N && gk < N) ? X[off + (long long)gi * N + gk] : 0.f;
            rdy[u] = ryv[u] = 0.f;
            if (gi < N && gj < N) {
                const long long o = off + (long long)gi * N + gj;
                rdy[u] = dY[o];
                ryv[u] = Yv[o];
            }
        }
    };
    fetch(0);
    for (int i0 = 0; i0 < N; i0 += HK) {
#pragma unroll
        for (int u = 0; u < E; ++u) {
            const int e = threadIdx.x + 256 * u;
            const int cc = e % T, ii = e / T;
            xs[ii][cc] = rx[u];
            gs[ii][cc] = sig_bwd(rdy[u], ryv[u]);
        }
        __syncthreads();
        if (i0 + HK < N) fetch(i0 + HK);
#pragma unroll
        for (int ii = 0; ii < HK; ++ii) {
            float a[M], bb[M];
#pragma unroll
            for (int q = 0; q < M; ++q) { a[q] = xs[ii][ty * M + q]; bb[q] = gs[ii][tx * M + q]; }
#pragma unroll
            for (int q = 0; q < M; ++q)
#pragma unroll
                for (int r = 0; r < M; ++r) t[q][r] = fmaf(a[q], bb[r], t[q][r]);
        }
        __syncthreads();
    }
    float* pw = partial + (long long)b * 2 * N * N;
    float* pa = pw + (long long)N * N;
#pragma unroll
    for (int q = 0; q < M; ++q) {
        int gk = k0 + ty * M + q;
        if (gk >= N) continue;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            int gj = j0 + tx * M + r;
            if (gj < N) {
                const long long o = (long long)gk * N + gj;
                pw[o] = t[q][r];
                pa[o] = t[q][r] * H[off + o];
            }
        }
    }
}

// dw = sum_b T_b, dalpha = sum_b T_b * H_b, slots summed in order 0..B-1
__global__ void head_dw_reduce_kernel(const float* __restrict__ partial, int B, int N, float* __restrict__ dw,
                                      float* __restrict__ da) {
#pragma clang fp contract(off)
    const long long nn = (long long)N * N;
    const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (idx >= nn) return;
    float sw = 0.f, sa = 0.f;
    for (int z = 0; z < B; ++z) {
        sw += partial[(long long)z * 2 * nn + idx];
        sa += partial[(long long)z * 2 * nn + nn + idx];
    }
    dw[idx] = sw;
    da[idx] = sa;
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

// 64-tiles when they give >= 2 blocks per CU, else 32-tiles (bs 32 x 128^2: 512 blocks)
static bool head_small_tiles(int B, int N) {
    const long long t64 = (long long)ceil_div(N, 64) * ceil_div(N, 64) * B;
    return t64 < 512;
}

template <int T>
static void launch_head_fwd(const pu_plastic_args* a, float* hn, hipStream_t s) {
    dim3 grid(ceil_div(a->nbf, T), ceil_div(a->nbf, T), a->batch);
    hipLaunchKernelGGL(head_fwd_kernel<T>, grid, dim3(256), 0, s, a->x, a->hebb, a->w, a->alpha, a->y, hn, a->eta,
                       a->nbf, a->rule);
}

template <int T>
static void launch_head_bwd(const pu_plastic_bwd_args* a, float* ws, hipStream_t s) {
    const int N = a->nbf, B = a->batch;
    dim3 grid(ceil_div(N, T), ceil_div(N, T), B);
    if (a->dx) hipLaunchKernelGGL(head_dx_kernel<T>, grid, dim3(256), 0, s, a->y, a->dy, a->hebb, a->w, a->alpha, a->dx, N);
    if (ws) hipLaunchKernelGGL(head_dw_kernel<T>, grid, dim3(256), 0, s, a->x, a->y, a->dy, a->hebb, ws, N);
}

}  // namespace pu

using namespace pu;

extern "C" int pu_trace_update(const float* hebb, const float* x, const float* y, const float* eta, float* hebb_out,
                               int batch, int nbf, int rule, void* stream) {
    PU_REQUIRE(hebb && x && y && eta && hebb_out && batch > 0 && nbf > 0, "pu_trace_update: bad args");
    PU_REQUIRE(rule == PU_RULE_HEBB || rule == PU_RULE_OJA, "Must select one learning rule ('hebb' or 'oja')");
    PU_REQUIRE((long long)nbf * nbf < (1ll << 31), "pu_trace_update: nbf too large");
    if (nbf % 4 == 0 && ((((uintptr_t)hebb) | ((uintptr_t)hebb_out) | ((uintptr_t)y)) & 15) == 0) {
        dim3 grid(ceil_div((long long)nbf * nbf / 4, 256), batch);
        hipLaunchKernelGGL(trace_kernel_v4, grid, dim3(256), 0, as_stream(stream), hebb, x, y, eta, hebb_out, nbf, rule);
    } else {
        dim3 grid(ceil_div((long long)nbf * nbf, 256), batch);
        hipLaunchKernelGGL(trace_kernel, grid, dim3(256), 0, as_stream(stream), hebb, x, y, eta, hebb_out, nbf, rule);
    }
    return check_launch("pu_trace_update");
}

extern "C" int pu_plastic_fwd(const pu_plastic_args* a, void* stream) {
    PU_REQUIRE(a && a->x && a->hebb && a->w && a->alpha && a->y && a->batch > 0 && a->nbf > 0, "pu_plastic_fwd: bad args");
    PU_REQUIRE(a->rule == PU_RULE_HEBB || a->rule == PU_RULE_OJA, "Must select one learning rule ('hebb' or 'oja')");
    PU_REQUIRE(!a->hebb_out || a->eta, "pu_plastic_fwd: eta missing");
    // the fused update writes H' while other blocks still read H: an aliased output takes the
    // two-launch path (GEMM, then the stand-alone update)
    const bool fuse = a->hebb_out && a->hebb_out != a->hebb;
    hipStream_t s = as_stream(stream);
    float* hn = fuse ? a->hebb_out : nullptr;
    if (head_small_tiles(a->batch, a->nbf)) launch_head_fwd<32>(a, hn, s);
    else launch_head_fwd<64>(a, hn, s);
    int st = check_launch("pu_plastic_fwd");
    if (st != PU_OK || !a->hebb_out || fuse) return st;
    return pu_trace_update(a->hebb, a->x, a->y, a->eta, a->hebb_out, a->batch, a->nbf, a->rule, stream);
}


extern "C" int pu_plastic_head_fwd(const pu_plastic_head_args* a, void* stream) {
    PU_REQUIRE(a && a->feat && a->out_w && a->hebb && a->w && a->alpha && a->x && a->y && a->batch > 0,
               "pu_plastic_head_fwd: bad args");
    const int N = a->nbf, C = a->channels;
    PU_REQUIRE(N >= 16 && N % 16 == 0 && N <= 512, "pu_plastic_head_fwd: nbf %d must be a multiple of 16 in [16, 512]", N);
    PU_REQUIRE(C >= 4 && C % 4 == 0, "pu_plastic_head_fwd: channels %d must be a multiple of 4", C);
    PU_REQUIRE((((uintptr_t)a->feat | (uintptr_t)a->out_w) & 15) == 0 || (a->feat_bf16 && ((uintptr_t)a->feat & 7) == 0 &&
               ((uintptr_t)a->out_w & 15) == 0), "pu_plastic_head_fwd: feat / out_w alignment");
    PU_REQUIRE(a->rule == PU_RULE_HEBB || a->rule == PU_RULE_OJA, "Must select one learning rule ('hebb' or 'oja')");
    PU_REQUIRE(!a->hebb_out || (a->eta && a->hebb_out != a->hebb), "pu_plastic_head_fwd: hebb_out needs eta and no aliasing");
    PU_REQUIRE((long long)N * N * C * a->batch < (1LL << 40), "pu_plastic_head_fwd: too large");
    PU_REQUIRE((((uintptr_t)a->hebb | (uintptr_t)a->w | (uintptr_t)a->alpha | (uintptr_t)a->hebb_out) & 15) == 0,
               "pu_plastic_head_fwd: hebb / w / alpha / hebb_out must be 16-byte aligned");
    const int q = C / 4;
    const int L = q >= 16 ? 16 : (q & (q - 1)) == 0 ? q : 16;    // lanes per pixel
    // the pipelined kernel: N = 128, L = 16 lanes per pixel, the fused trace update
    // (PU_HEAD_PIPE=0 keeps the phase-serial kernel: A/B runs)
    static const bool pipe_on = [] {
        const char* e = getenv("PU_HEAD_PIPE");
        return !(e && e[0] == '0');
    }();
    // C >= 64: every streamer lane's first float4 (channels lane*4 .. lane*4+3 of the 16 lanes)
    // and its outconv weights lie inside the pixel; C = 12, 24, 48, 60 also give L = 16 but would
    // read the next pixel's channels (and past the end of wo / feat) - they take the serial kernel
    if (pipe_on && N == HP_N && L == 16 && C >= 64 && a->hebb_out) {
        const dim3 pg(N / 16, a->batch);
        if (a->feat_bf16)
            hipLaunchKernelGGL((head_pipe_fwd_kernel<__bf16>), pg, dim3(HP_NT), 0, as_stream(stream), (const __bf16*)a->feat,
                               a->out_w, a->out_b, C, a->hebb, a->w, a->alpha, a->eta, a->x, a->y, a->hebb_out, a->rule);
        else
            hipLaunchKernelGGL((head_pipe_fwd_kernel<float>), pg, dim3(HP_NT), 0, as_stream(stream), (const float*)a->feat,
                               a->out_w, a->out_b, C, a->hebb, a->w, a->alpha, a->eta, a->x, a->y, a->hebb_out, a->rule);
        return check_launch("pu_plastic_head_fwd");
    }
    const int kc = fused_head_chunk(N);                           // Weff rows per LDS chunk
    // rows per block: every block re-forms the whole W_eff = w + alpha (.) H of its slot, so at
    // nbf >= 256 (C4 / C5) 32-row blocks halve that work and feed each W fragment to two MFMA row
    // tiles (the LDS of 16-row blocks already held them to one block per CU there)
    const int R = (N >= 256 && N % 32 == 0 && ((size_t)(32 + 1) * N + (size_t)kc * N + N) * sizeof(float) <= 160 * 1024) ? 32 : FH_R;
    size_t lds = ((size_t)(R + 1) * N + (size_t)kc * N + N) * sizeof(float);
    if (lds < (size_t)PU_FH_LDS_MIN) lds = PU_FH_LDS_MIN;
    const dim3 grid(N / R, a->batch);
    const FastDiv dN = make_fastdiv(N);
    hipStream_t s = as_stream(stream);
    const int tpw = (N / 16 + FH_WAVES - 1) / FH_WAVES;           // column tiles per wave
#define PU_FH3(T_, L_, W_, R_)                                                                                 \
    hipLaunchKernelGGL((head_fused_fwd_kernel<T_, L_, W_, R_>), grid, dim3(FH_NT), lds, s, (const T_*)a->feat, \
                       a->out_w, a->out_b, C, a->hebb, a->w, a->alpha, a->eta, a->x, a->y, a->hebb_out, N, dN, kc, \
                       a->rule)
#define PU_FH2(T_, L_, W_)                                                                                     \
    do {                                                                                                    \
        if (R == 32) PU_FH3(T_, L_, W_, 32);                                                                \
        else PU_FH3(T_, L_, W_, FH_R);                                                                      \
    } while (0)
#define PU_FH(T_, L_)                                                                                       \
    do {                                                                                                    \
        if (tpw <= 1) PU_FH2(T_, L_, 1);                                                                    \
        else if (tpw <= 2) PU_FH2(T_, L_, 2);                                                               \
        else PU_FH2(T_, L_, 4);                                                                             \
    } while (0)
#define PU_FH_L(T_)                                                                                         \
    switch (L) {                                                                                            \
        case 1: PU_FH(T_, 1); break;                                                                        \
        case 2: PU_FH(T_, 2); break;                                                                        \
        case 4: PU_FH(T_, 4); break;                                                                        \
        case 8: PU_FH(T_, 8); break;                                                                        \
        default: PU_FH(T_, 16); break;                                                                      \
    }
    if (a->feat_bf16) { PU_FH_L(__bf16) } else { PU_FH_L(float) }
#undef PU_FH_L
#undef PU_FH
#undef PU_FH2
#undef PU_FH3
    return check_launch("pu_plastic_head_fwd");
}

extern "C" size_t pu_plastic_bwd_workspace_bytes(int batch, int nbf) {
    return (size_t)batch * 2 * nbf * nbf * sizeof(float);      // per-slot (T_b, T_b * H_b)
}

extern "C" int pu_plastic_bwd(const pu_plastic_bwd_args* a, void* workspace, size_t ws_bytes, void* stream) {
    PU_REQUIRE(a && a->x && a->hebb && a->w && a->alpha && a->y && a->dy && a->batch > 0 && a->nbf > 0,
               "pu_plastic_bwd: bad args");
    const int N = a->nbf, B = a->batch;
    hipStream_t s = as_stream(stream);
    float* ws = nullptr;
    if (a->dw || a->dalpha) {
        PU_REQUIRE(a->dw && a->dalpha, "pu_plastic_bwd: dw and dalpha go together");
        const size_t need = pu_plastic_bwd_workspace_bytes(B, N);
        if (!workspace || ws_bytes < need) return fail(PU_ERR_WORKSPACE, "pu_plastic_bwd: workspace %zu < %zu", ws_bytes, need);
        ws = (float*)workspace;
    }
    if (head_small_tiles(B, N)) launch_head_bwd<32>(a, ws, s);
    else launch_head_bwd<64>(a, ws, s);
    int st = check_launch("pu_plastic_bwd");
    if (st != PU_OK || !ws) return st;
    hipLaunchKernelGGL(head_dw_reduce_kernel, dim3(ceil_div((long long)N * N, 256)), dim3(256), 0, s,
                       (const float*)ws, B, N, a->dw, a->dalpha);
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
