// Implicit-GEMM convolution on CDNA4 fp32 MFMA (v_mfma_f32_32x32x2_f32), NHWC activations.
//
// Replaces (yaricom/Plastic-UNet): nn.Conv2d(k=3,p=1)+ReLU of double_conv (src/unet/unet_p.py:
// 184-201) forward and backward-data, nn.ConvTranspose2d(2,2,s=2) of up (unet_p.py:238) forward and
// backward-data, and the skip concat torch.cat([x2,x1],1) (unet_p.py:248), which is never
// materialised: the A-tile loader reads channel range [0,c0) from src0 and [c0,c0+c1) from src1.
//
// GEMM view: D[m][n] = sum_k A[m][k] * W[n][k];  m = output pixel, k = (tap, channel), n = out ch.
// Block tile BM x BN, K staged 16 at a time through double-buffered LDS (row stride 20 floats:
// conflict-free ds_read_b128 for the MFMA operand reads).  4 waves per block; each wave owns a
// (BM/WM) x (BN/WN) sub-tile of 32x32 MFMA blocks.  Each lane reads 4 consecutive k of one row with
// a single ds_read_b128 and feeds them to 4 MFMAs: for MFMA step s, lane (i, h) supplies
// A[i][kk*8 + 4h + s] and B[kk*8 + 4h + s][j] - the same k on both operands, so the sum is exact.
#include "common.h"

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int IG_BK = 16;
constexpr int IG_LDS = IG_BK + 4;

enum { LOAD_CHUNK16 = 0, LOAD_VEC4 = 1, LOAD_SCALAR = 2 };

struct IgemmParams {
    int M, N, K, k_pad;
    int Hi, Wi, Ho, Wo, kw, stride, pad;
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
    FastDiv dWo, dHo, dC, dKw, dCo;
};

// Load 4 consecutive k values (k, k+1, k+2, k+3) of GEMM row (pb, hb, wb) into v.
template <int MODE>
__device__ __forceinline__ f32x4 load_a4(const IgemmParams& p, int pb, int hb, int wb, int k) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (MODE == LOAD_SCALAR) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            int ke = k + e;
            if (ke < p.K) {
                int tap = fdiv(ke, p.dC);
                int c = ke - tap * p.C;
                int r = fdiv(tap, p.dKw);
                int s = tap - r * p.kw;
                int hi = hb + r, wi = wb + s;
                if ((unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi) {
                    long long pix = (long long)pb + hi * p.Wi + wi;
                    v[e] = c < p.c0 ? p.src0[pix * p.c0 + c] : p.src1[pix * p.c1 + (c - p.c0)];
                }
            }
        }
        return v;
    } else {
        if (k < p.K) {
            int tap = fdiv(k, p.dC);
            int c = k - tap * p.C;
            int r = fdiv(tap, p.dKw);
            int s = tap - r * p.kw;
            int hi = hb + r, wi = wb + s;
            if ((unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi) {
                long long pix = (long long)pb + hi * p.Wi + wi;
                const float* src = c < p.c0 ? p.src0 + pix * p.c0 + c : p.src1 + pix * p.c1 + (c - p.c0);
                v = *reinterpret_cast<const f32x4*>(src);
            }
        }
        return v;
    }
}

template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(256) void igemm_kernel(const IgemmParams p) {
    constexpr int FM = BM / WM / 32;
    constexpr int FN = BN / WN / 32;
    constexpr int A_LD = BM / 64;  // float4 loads per thread for the A tile (BM x 16)
    constexpr int B_LD = BN / 64;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(FM >= 1 && FN >= 1, "wave tile >= 32x32");

    __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * IG_LDS];
    float* As = lds;
    float* Bs = lds + 2 * BM * IG_LDS;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave % WM, wn = wave / WM;
    const int lr = lane & 31, lh = lane >> 5;
    const int m_blk = blockIdx.x * BM;
    const int n_blk = blockIdx.y * BN;

    // ---- per-thread A rows: row = (tid >> 2) + 64*i, k-quad = tid & 3
    const int kq = tid & 3;
    int pb[A_LD], hb[A_LD], wb[A_LD];
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
        int m = m_blk + (tid >> 2) + 64 * i;
        if (m < p.M) {
            int t = fdiv(m, p.dWo);
            int wo = m - t * p.Wo;
            int b = fdiv(t, p.dHo);
            int ho = t - b * p.Ho;
            pb[i] = b * p.Hi * p.Wi;
            hb[i] = ho * p.stride - p.pad;
            wb[i] = wo * p.stride - p.pad;
        } else {
            pb[i] = 0;
            hb[i] = -(1 << 28);  // fails the bounds test -> zeros
            wb[i] = 0;
        }
    }
    const float* wrow[B_LD];
    bool wok[B_LD];
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
        int n = n_blk + (tid >> 2) + 64 * i;
        wok[i] = n < p.N;
        wrow[i] = p.wt + (long long)(wok[i] ? n : 0) * p.k_pad + kq * 4;
    }

    f32x4 ra[A_LD], rb[B_LD];
    auto load_stage = [&](int t) {
        const int k0 = t * IG_BK;
        if (MODE == LOAD_CHUNK16) {
            // the whole 16-wide k chunk shares one tap and one source (c0, c1 multiples of 16)
            int tap = fdiv(k0, p.dC);
            int c = k0 - tap * p.C;
            int r = fdiv(tap, p.dKw);
            int s = tap - r * p.kw;
            bool first = c < p.c0;
            const float* src = first ? p.src0 : p.src1;
            int cs = first ? p.c0 : p.c1;
            int cc = (first ? c : c - p.c0) + kq * 4;
            bool kin = k0 < p.K;
#pragma unroll
            for (int i = 0; i < A_LD; ++i) {
                int hi = hb[i] + r, wi = wb[i] + s;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (kin && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi) {
                    long long pix = (long long)pb[i] + hi * p.Wi + wi;
                    v = *reinterpret_cast<const f32x4*>(src + pix * cs + cc);
                }
                ra[i] = v;
            }
        } else {
#pragma unroll
            for (int i = 0; i < A_LD; ++i) ra[i] = load_a4<MODE>(p, pb[i], hb[i], wb[i], k0 + kq * 4);
        }
#pragma unroll
        for (int i = 0; i < B_LD; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (wok[i]) v = *reinterpret_cast<const f32x4*>(wrow[i] + k0);
            rb[i] = v;
        }
    };
    auto store_stage = [&](int buf) {
        float* a = As + buf * BM * IG_LDS;
        float* b = Bs + buf * BN * IG_LDS;
#pragma unroll
        for (int i = 0; i < A_LD; ++i)
            *reinterpret_cast<f32x4*>(a + ((tid >> 2) + 64 * i) * IG_LDS + kq * 4) = ra[i];
#pragma unroll
        for (int i = 0; i < B_LD; ++i)
            *reinterpret_cast<f32x4*>(b + ((tid >> 2) + 64 * i) * IG_LDS + kq * 4) = rb[i];
    };

    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int T = p.k_pad / IG_BK;
    const int a_row0 = wm * (BM / WM) + lr;
    const int b_row0 = wn * (BN / WN) + lr;

    load_stage(0);
    store_stage(0);
    __syncthreads();

    for (int t = 0; t < T; ++t) {
        const int buf = t & 1;
        if (t + 1 < T) load_stage(t + 1);
        const float* a = As + buf * BM * IG_LDS;
        const float* b = Bs + buf * BN * IG_LDS;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            f32x4 fa[FM], fb[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i)
                fa[i] = *reinterpret_cast<const f32x4*>(a + (a_row0 + i * 32) * IG_LDS + kk * 8 + lh * 4);
#pragma unroll
            for (int j = 0; j < FN; ++j)
                fb[j] = *reinterpret_cast<const f32x4*>(b + (b_row0 + j * 32) * IG_LDS + kk * 8 + lh * 4);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < T) store_stage(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: C/D layout of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    const bool relu = p.flags & PU_EPI_RELU;
    const bool accum = p.flags & PU_EPI_ACCUM;
    const bool shuffle = p.flags & PU_EPI_SHUFFLE2;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int n = n_blk + wn * (BN / WN) + j * 32 + lr;
        if (n >= p.N) continue;
        float* dst;
        const float* msk;
        int ld, nc;
        float bv = 0.f;
        int sh_c = 0, sh_i = 0, sh_j = 0;
        if (shuffle) {
            int ij = fdiv(n, p.dCo);
            sh_c = n - ij * (p.N >> 2);
            sh_i = ij >> 1;
            sh_j = ij & 1;
            dst = p.dst0;
            msk = p.mask0;
            ld = p.N >> 2;
            nc = sh_c;
            if (p.bias) bv = p.bias[sh_c];
        } else if (n < p.n0) {
            dst = p.dst0; msk = p.mask0; ld = p.n0; nc = n;
            if (p.bias) bv = p.bias[n];
        } else {
            dst = p.dst1; msk = p.mask1; ld = p.N - p.n0; nc = n - p.n0;
            if (p.bias) bv = p.bias[n];
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m_blk + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m >= p.M) continue;
                long long off;
                if (shuffle) {
                    int t2 = fdiv(m, p.dWo);
                    int wo = m - t2 * p.Wo;
                    int bb = fdiv(t2, p.dHo);
                    int ho = t2 - bb * p.Ho;
                    long long pix = ((long long)bb * 2 * p.Ho + 2 * ho + sh_i) * (2 * p.Wo) + 2 * wo + sh_j;
                    off = pix * ld + nc;
                } else {
                    off = (long long)m * ld + nc;
                }
                float v = acc[i][j][r] + bv;
                if (relu) v = fmaxf(v, 0.f);
                if (msk && !(msk[off] > 0.f)) v = 0.f;
                if (accum) v += dst[off];
                dst[off] = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------ host
struct TileCfg {
    int bm, bn;
};

template <int BM, int BN, int WM, int WN>
static void launch_mode(int mode, const IgemmParams& p, dim3 grid, hipStream_t s) {
    switch (mode) {
        case LOAD_CHUNK16: hipLaunchKernelGGL((igemm_kernel<BM, BN, WM, WN, LOAD_CHUNK16>), grid, dim3(256), 0, s, p); break;
        case LOAD_VEC4: hipLaunchKernelGGL((igemm_kernel<BM, BN, WM, WN, LOAD_VEC4>), grid, dim3(256), 0, s, p); break;
        default: hipLaunchKernelGGL((igemm_kernel<BM, BN, WM, WN, LOAD_SCALAR>), grid, dim3(256), 0, s, p); break;
    }
}

static int blocks_for(long long M, int N, int bm, int bn) { return ceil_div(M, bm) * ceil_div(N, bn); }

// tile choice: the largest tile that still gives >= ~2 blocks per CU (256 CUs)
static void choose_tile(long long M, int N, int* bm, int* bn) {
    const int target = 480;
    if (N <= 64) {
        if (blocks_for(M, N, 256, 64) >= target) { *bm = 256; *bn = 64; }
        else if (blocks_for(M, N, 128, 64) >= target) { *bm = 128; *bn = 64; }
        else { *bm = 64; *bn = 64; }
    } else {
        if (blocks_for(M, N, 128, 128) >= target) { *bm = 128; *bn = 128; }
        else if (blocks_for(M, N, 128, 64) >= target) { *bm = 128; *bn = 64; }
        else { *bm = 64; *bn = 64; }
    }
}

static int choose_mode(int c0, int c1) {
    if (c0 % 16 == 0 && c1 % 16 == 0) return LOAD_CHUNK16;
    if (c0 % 4 == 0 && c1 % 4 == 0) return LOAD_VEC4;
    return LOAD_SCALAR;
}

}  // namespace pu

using namespace pu;

extern "C" int pu_conv_igemm(const pu_conv_args* a, void* stream) {
    PU_REQUIRE(a != nullptr, "pu_conv_igemm: null args");
    PU_REQUIRE(a->batch > 0 && a->in_h > 0 && a->in_w > 0 && a->out_h > 0 && a->out_w > 0,
               "pu_conv_igemm: bad grid %dx%dx%d -> %dx%d", a->batch, a->in_h, a->in_w, a->out_h, a->out_w);
    PU_REQUIRE(a->kh > 0 && a->kw > 0 && a->stride > 0 && a->pad >= 0, "pu_conv_igemm: bad taps");
    PU_REQUIRE(a->src0 && a->c0 > 0, "pu_conv_igemm: src0 missing");
    PU_REQUIRE(a->c1 == 0 || a->src1, "pu_conv_igemm: src1 missing for c1=%d", a->c1);
    PU_REQUIRE(a->weight && a->dst0 && a->n > 0, "pu_conv_igemm: weight/dst0/n");
    const int C = a->c0 + a->c1;
    const int K = a->kh * a->kw * C;
    PU_REQUIRE(a->k_pad >= K && a->k_pad % IG_BK == 0, "pu_conv_igemm: k_pad %d must be >= %d and a multiple of 16", a->k_pad, K);
    const bool shuffle = a->flags & PU_EPI_SHUFFLE2;
    if (shuffle) {
        PU_REQUIRE(a->n % 4 == 0, "pu_conv_igemm: SHUFFLE2 needs n %% 4 == 0");
    } else {
        PU_REQUIRE(a->n0 > 0 && a->n0 <= a->n, "pu_conv_igemm: n0 %d out of range", a->n0);
        PU_REQUIRE(a->n0 == a->n || a->dst1, "pu_conv_igemm: dst1 missing");
    }
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    PU_REQUIRE(M < (1LL << 31) && (long long)a->batch * a->in_h * a->in_w < (1LL << 31), "pu_conv_igemm: too many pixels");

    IgemmParams p;
    p.M = (int)M; p.N = a->n; p.K = K; p.k_pad = a->k_pad;
    p.Hi = a->in_h; p.Wi = a->in_w; p.Ho = a->out_h; p.Wo = a->out_w;
    p.kw = a->kw; p.stride = a->stride; p.pad = a->pad;
    p.C = C; p.c0 = a->c0; p.c1 = a->c1;
    p.src0 = a->src0; p.src1 = a->src1; p.wt = a->weight; p.bias = a->bias;
    p.dst0 = a->dst0; p.dst1 = a->dst1; p.mask0 = a->mask0; p.mask1 = a->mask1;
    p.n0 = shuffle ? a->n : a->n0; p.flags = a->flags;
    p.dWo = make_fastdiv(a->out_w); p.dHo = make_fastdiv(a->out_h);
    p.dC = make_fastdiv(C); p.dKw = make_fastdiv(a->kw); p.dCo = make_fastdiv(shuffle ? a->n / 4 : 1);

    const int mode = choose_mode(a->c0, a->c1);
    if (mode != LOAD_SCALAR) {
        PU_REQUIRE(((uintptr_t)a->src0 & 15) == 0 && ((uintptr_t)a->src1 & 15) == 0,
                   "pu_conv_igemm: sources must be 16-byte aligned");
    }
    PU_REQUIRE(((uintptr_t)a->weight & 15) == 0, "pu_conv_igemm: weight must be 16-byte aligned");

    hipStream_t s = as_stream(stream);
    const int N = a->n;
    int bm, bn;
    choose_tile(M, N, &bm, &bn);
    const dim3 grid(ceil_div(M, bm), ceil_div(N, bn));
    if (bm == 256) launch_mode<256, 64, 4, 1>(mode, p, grid, s);
    else if (bm == 128 && bn == 128) launch_mode<128, 128, 2, 2>(mode, p, grid, s);
    else if (bm == 128) launch_mode<128, 64, 2, 2>(mode, p, grid, s);
    else launch_mode<64, 64, 2, 2>(mode, p, grid, s);
    return check_launch("pu_conv_igemm");
}

extern "C" int pu_conv_igemm_tile(const pu_conv_args* a, int* bm, int* bn, int* mode) {
    PU_REQUIRE(a && bm && bn && mode, "pu_conv_igemm_tile: null args");
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    choose_tile(M, a->n, bm, bn);
    *mode = choose_mode(a->c0, a->c1);
    return PU_OK;
}
