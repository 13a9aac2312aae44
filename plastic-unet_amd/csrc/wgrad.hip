// Weight (and bias) gradients of the convolutions as split-K fp32 MFMA GEMMs.
//
// Replaces the autograd weight/bias backward of nn.Conv2d (src/unet/unet_p.py:184-201) and
// nn.ConvTranspose2d (unet_p.py:238) that loss.backward() (src/train.py:110) runs on the CPU.
//
//   out[n][k] = sum_m P[m][n] * Q[m][k]      m = pixel rows (B*H*W), split over grid.z
//   P = rows operand (conv: dZ; ConvT: its low-res input), Q = im2col of src0|src1 at tap(k)
//   bias_mode 1 adds a ones COLUMN (k == K)  -> dbias[n]  = sum_m P[m][n]
//   bias_mode 2 adds a ones ROW    (n == N)  -> dbias[c] = sum_taps sum_m Q[m][(tap,c)]
// MFMA mapping (32x32x2): lane (i, h) supplies A[i][h] = P[m0+h][n_i] and B[h][j] = Q[m0+h][k_j],
// both read from LDS with ds_read_b32 (32 consecutive floats per half-wave: conflict-free).
// Partial tiles go to a per-split slab; wgrad_reduce sums the splits in a fixed order
// (deterministic) and writes PyTorch's [n][c][kh][kw] layout.
#include "common.h"
#include <type_traits>

#ifndef PU_NO_ILV
#define PU_NO_ILV 0   // 1: leave MFMA / VALU placement to the scheduler (A/B builds)
#endif
// wgrad_wino_x6_kernel ablations (timing only, wrong results): 1 no MFMAs, 2 no plane formation
// (VALU + LDS stores), 3 no global loads, 4 no per-sub-stage barrier
#ifndef PU_WW_ABL
#define PU_WW_ABL 0
#endif

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WG_BM = 16;  // pixel rows per LDS stage

struct WgradParams {
    int M, N, Nr, K, Kc, C, c0, c1;
    int Hi, Wi, Ho, Wo, kw, stride, pad;
    const float* P;
    const float* src0;
    const float* src1;
    int bias_mode;
    float* slab;
    int mps;  // pixel rows per split (multiple of WG_BM)
    int gx, gy;  // k-tiles, n-tiles
    int Kcp;     // slab row stride (Kc rounded up to 4)
    int batch, tiles_w, tiles_h;   // small-channel kernel: pixel tiles of 16 x 32
    FastDiv dWo, dHo, dC, dKw;
};

template <int BN, int BK, int WN, int WK, bool QVEC>
__global__ __launch_bounds__(256) void wgrad_kernel(const WgradParams p) {
    constexpr int FN = BN / WN / 32;
    constexpr int FK = BK / WK / 32;
    constexpr int P_PER_ROW = BN / 4;               // float4 per P row
    constexpr int P_LD = (WG_BM * P_PER_ROW) / 256;  // float4 loads per thread
    constexpr int Q_PER_ROW = BK / 4;
    constexpr int Q_LD = (WG_BM * Q_PER_ROW) / 256;
    static_assert(WN * WK == 4, "4 waves");
    static_assert(P_LD >= 1 && Q_LD >= 1, "tile too small for 256 threads");

    __shared__ __attribute__((aligned(16))) float lds[2 * WG_BM * (BN + BK)];
    float* Ps = lds;
    float* Qs = lds + 2 * WG_BM * BN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform -> scalar math
    const int wn = wave % WN, wk = wave / WN;
    const int lr = lane & 31, lh = lane >> 5;
    // XCD-aware order: logical tile = (split z, n-tile y, k-tile x), x fastest; each XCD walks a
    // contiguous range, so the k-tiles that re-read the same pixel rows share its L2
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % p.gx;
    const int tyz = tile / p.gx;
    const int ty = tyz % p.gy;
    const int tz = tyz / p.gy;
    const int n_blk = ty * BN;
    const int k_blk = tx * BK;
    const int m_begin = tz * p.mps;
    const int m_end = min(p.M, m_begin + p.mps);

    // ---- fixed per-thread P columns
    const int p_col = (tid % P_PER_ROW) * 4;
    const int p_row = tid / P_PER_ROW;               // + i * (256 / P_PER_ROW)
    const int pn = n_blk + p_col;
    // ---- fixed per-thread Q columns: tap offsets and channel
    const int q_col = (tid % Q_PER_ROW) * 4;
    const int q_row = tid / Q_PER_ROW;               // + i * (256 / Q_PER_ROW)
    int q_r[4], q_s[4], q_c[4];
    bool q_ok[4], q_one[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        // QVEC: the four columns share one tap (C % 4 == 0), so only element 0 is decoded
        const int k = k_blk + q_col + e;
        q_ok[e] = k < p.K;
        q_one[e] = (p.bias_mode == 1) && k == p.K;
        const int kk = q_ok[e] ? k : 0;
        const int tap = fdiv(kk, p.dC);
        q_c[e] = kk - tap * p.C;
        q_r[e] = fdiv(tap, p.dKw);
        q_s[e] = tap - q_r[e] * p.kw;
        if (QVEC) break;
    }

    f32x4 rp[P_LD], rq[Q_LD];
    auto load_stage = [&](int m0) {
#pragma unroll
        for (int i = 0; i < P_LD; ++i) {
            int m = m0 + p_row + i * (256 / P_PER_ROW);
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (m < m_end) {
                if (pn + 3 < p.N) {
                    v = *reinterpret_cast<const f32x4*>(p.P + (long long)m * p.N + pn);
                } else if (p.bias_mode == 2 && pn == p.N) {
                    v[0] = 1.f;
                }
            }
            rp[i] = v;
        }
        // Q rows: the wave's first row is uniform (decomposed on the scalar unit); lanes add a
        // small row delta (0 .. 64/Q_PER_ROW - 1) with carry into ho / b.
        constexpr int QR_PER_WAVE = 64 / Q_PER_ROW;
        const int q_delta = lane / Q_PER_ROW;
#pragma unroll
        for (int i = 0; i < Q_LD; ++i) {
            const int mu = m0 + wave * QR_PER_WAVE + i * (256 / Q_PER_ROW);
            const int tu = fdiv(mu, p.dWo);
            const int wou = mu - tu * p.Wo;
            const int bu = fdiv(tu, p.dHo);
            const int hou = tu - bu * p.Ho;
            const int m = mu + q_delta;
            int wo = wou + q_delta, ho = hou, b = bu;
            while (wo >= p.Wo) {
                wo -= p.Wo;
                if (++ho >= p.Ho) { ho = 0; ++b; }
            }
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (m < m_end) {
                long long pb = (long long)b * p.Hi * p.Wi;
                int hb = ho * p.stride - p.pad, wb = wo * p.stride - p.pad;
                if (QVEC) {
                    if (q_ok[0]) {
                        int hi = hb + q_r[0], wi = wb + q_s[0];
                        if ((unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi) {
                            long long pix = pb + hi * p.Wi + wi;
                            int c = q_c[0];
                            const float* src = c < p.c0 ? p.src0 + pix * p.c0 + c : p.src1 + pix * p.c1 + (c - p.c0);
                            v = *reinterpret_cast<const f32x4*>(src);
                        }
                    } else if (q_one[0]) {
                        v[0] = 1.f;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if (q_ok[e]) {
                            int hi = hb + q_r[e], wi = wb + q_s[e];
                            if ((unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi) {
                                long long pix = pb + hi * p.Wi + wi;
                                int c = q_c[e];
                                v[e] = c < p.c0 ? p.src0[pix * p.c0 + c] : p.src1[pix * p.c1 + (c - p.c0)];
                            }
                        } else if (q_one[e]) {
                            v[e] = 1.f;
                        }
                    }
                }
            }
            rq[i] = v;
        }
    };
    auto store_stage = [&](int buf) {
        float* ps = Ps + buf * WG_BM * BN;
        float* qs = Qs + buf * WG_BM * BK;
#pragma unroll
        for (int i = 0; i < P_LD; ++i)
            *reinterpret_cast<f32x4*>(ps + (p_row + i * (256 / P_PER_ROW)) * BN + p_col) = rp[i];
#pragma unroll
        for (int i = 0; i < Q_LD; ++i)
            *reinterpret_cast<f32x4*>(qs + (q_row + i * (256 / Q_PER_ROW)) * BK + q_col) = rq[i];
    };

    f32x16 acc[FN][FK];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int a_col0 = wn * (BN / WN) + lr;
    const int b_col0 = wk * (BK / WK) + lr;

    if (m_begin < m_end) {
        load_stage(m_begin);
        store_stage(0);
    }
    __syncthreads();
    int buf = 0;
    for (int m0 = m_begin; m0 < m_end; m0 += WG_BM) {
        const bool more = m0 + WG_BM < m_end;
        if (more) load_stage(m0 + WG_BM);
        const float* ps = Ps + buf * WG_BM * BN;
        const float* qs = Qs + buf * WG_BM * BK;
#pragma unroll
        for (int ks = 0; ks < WG_BM / 2; ++ks) {
            float fa[FN], fb[FK];
            const int row = ks * 2 + lh;
#pragma unroll
            for (int i = 0; i < FN; ++i) fa[i] = ps[row * BN + a_col0 + i * 32];
#pragma unroll
            for (int j = 0; j < FK; ++j) fb[j] = qs[row * BK + b_col0 + j * 32];
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FK; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        if (more) store_stage(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }

    // ---- partial tile -> slab[z][n][k]
    float* slab = p.slab + (long long)tz * p.Nr * p.Kcp;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
#pragma unroll
        for (int j = 0; j < FK; ++j) {
            const int k = k_blk + b_col0 + j * 32;
            if (k >= p.Kc) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n_blk + wn * (BN / WN) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (n < p.Nr) slab[(long long)n * p.Kcp + k] = acc[i][j][r];
            }
        }
    }
}

// ------------------------------------------------------------------------ direct-to-LDS variant
// C % 4 == 0: P and Q tiles are fetched with global_load_lds_dwordx4 into row-major LDS images
// ([16 rows][BN] and [16 rows][BK]); the MFMA operands are ds_read_b32 of 32 consecutive floats
// per half-wave (conflict-free).  Padding / out-of-image taps read a zero page.  Roles are
// transposed (Q as the A operand) so each lane owns 4 consecutive k of one n and the partial tile
// is stored as float4 into a Kcp-strided slab.  The bias is not an extra GEMM column/row (that
// costs a whole extra tile whenever K or N is a multiple of the tile): the k-tile-0 blocks
// (mode 1) or n-tile-0 blocks (mode 2) column-sum the staged P / Q image out of LDS on the VALU
// and write the partial into slab column K / row N.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
__device__ __attribute__((aligned(16))) float g_wg_zero16[4] = {0.f, 0.f, 0.f, 0.f};

typedef __bf16 wg_bf16x8 __attribute__((ext_vector_type(8)));

// 8 fp32 values -> their exact 3-term bf16 split (see igemm.hip, igemm_x6_kernel), pair-wise:
// v_cvt_pk_bf16_f32 rounds two values at once, the residuals are v_pk_add_f32 (4.5 VALU/element)
typedef float wg_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 wg_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned wg_pk(wg_f32x2 v) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, wg_bf16x2));
}
__device__ __forceinline__ void wg_split3(const float (&x)[8], wg_bf16x8& h, wg_bf16x8& m, wg_bf16x8& l) {
#pragma clang fp contract(off)
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 hv, mv, lv;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float x0 = x[2 * q], x1 = x[2 * q + 1];
        const unsigned a = wg_pk(wg_f32x2{x0, x1});
        const float r0 = x0 - __builtin_bit_cast(float, a << 16);
        const float r1 = x1 - __builtin_bit_cast(float, a & 0xffff0000u);
        const unsigned b = wg_pk(wg_f32x2{r0, r1});
        const float l0 = r0 - __builtin_bit_cast(float, b << 16);
        const float l1 = r1 - __builtin_bit_cast(float, b & 0xffff0000u);
        hv[q] = a;
        mv[q] = b;
        lv[q] = wg_pk(wg_f32x2{l0, l1});
    }
    h = __builtin_bit_cast(wg_bf16x8, hv);
    m = __builtin_bit_cast(wg_bf16x8, mv);
    l = __builtin_bit_cast(wg_bf16x8, lv);
}

// X6: the 16 staged pixel rows are one k-step of v_mfma_f32_32x32x16_bf16 and each fp32 product
// is 6 exact bf16 products (hi/mid/lo split, fp32 accumulation) - 6 x 32 cycles against the
// 8 x 64 of v_mfma_f32_32x32x2_f32; lane (i, h) reads rows 8h..8h+7 of its column.
// NW waves (WN x WK): 6 waves give the 64 x 576 tile of the 64-channel layers (K = 9 x 64 or
// 9 x 128 with no padding, 64 x 96 per wave: 5 operand splits per 36 MFMAs); the P pieces that do
// not divide among the waves are issued by every wave anyway (the counted wait stays uniform),
// the surplus ones reading the zero page into a 1 KB sink.
// FQ: stride 1, same-size input (Hi == Ho, Wi == Wo >= 4) - a Q lane's source row is its output
// pixel m shifted by the tap, so the per-stage address is one scalar product plus per-lane
// constants, and the lane's (ho, wo) advance by compare-and-wrap (row delta < 4 < Wo) instead of
// the per-lane divisions of the general path.
template <int BN, int BK, int WN, int WK, int NBUF, bool X6, int NW = 4, bool FQ = false>
__global__ __launch_bounds__(NW * 64) void wgrad_dma_kernel(const WgradParams p) {
    constexpr int FN = BN / WN / 32;
    constexpr int FK = BK / WK / 32;
    constexpr int P_ROWS = 256 / BN;              // rows per 1 KB glds instruction
    constexpr int P_TOT = WG_BM / P_ROWS;         // P glds per stage
    constexpr int P_LD = (P_TOT + NW - 1) / NW;   // per wave (surplus -> sink)
    constexpr int Q_LD = WG_BM * BK / 256 / NW;   // Q instructions may straddle rows (BK = 192)
    constexpr int G = P_LD + Q_LD;
    constexpr int STAGE = WG_BM * (BN + BK);
    constexpr int SINK = (P_TOT % NW) ? 256 : 0;
    static_assert(WN * WK == NW && P_LD >= 1 && Q_LD >= 1 && 256 % BN == 0 && (WG_BM * BK) % (256 * NW) == 0, "tile");

    __shared__ __attribute__((aligned(16))) float lds[NBUF * STAGE + SINK];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave % WN, wk = wave / WN;
    const int lr = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % p.gx;
    const int tyz = tile / p.gx;
    const int ty = tyz % p.gy;
    const int tz = tyz / p.gy;
    const int n_blk = ty * BN;
    const int k_blk = tx * BK;
    const int m_begin = tz * p.mps;
    const int m_end = min(p.M, m_begin + p.mps);

    // P lane geometry: column n (fixed), row delta within the instruction
    const int p_col = (lane % (BN / 4)) * 4;
    const int p_dr = lane / (BN / 4);
    const int pn = n_blk + p_col;
    const bool p_in = pn < p.N;
    // Q lane geometry per instruction j: image float offset (wave*Q_LD + j)*256 + 4*lane ->
    // (uniform first row q_row0, lane row delta, column k -> tap offsets and channel)
    int q_row0[Q_LD], q_dr[Q_LD], q_r[Q_LD], q_s[Q_LD], q_cs[Q_LD];
    const float* q_ptr[Q_LD];
#pragma unroll
    for (int j = 0; j < Q_LD; ++j) {
        const int base = (wave * Q_LD + j) * 256;
        const int off = base + 4 * lane;
        q_row0[j] = base / BK;
        q_dr[j] = off / BK - q_row0[j];
        const int qk = k_blk + off % BK;
        q_r[j] = 0; q_s[j] = 0; q_cs[j] = 0; q_ptr[j] = nullptr;
        if (qk < p.K) {
            const int tap = fdiv(qk, p.dC);
            const int c = qk - tap * p.C;
            q_r[j] = fdiv(tap, p.dKw);
            q_s[j] = tap - q_r[j] * p.kw;
            const bool first = c < p.c0;
            q_ptr[j] = first ? p.src0 + c : p.src1 + (c - p.c0);
            q_cs[j] = first ? p.c0 : p.c1;
        }
    }
    // FQ lane constants: source = q_ptr + (m + dr + (r - pad) * Wi + (s - pad)) * cs
    const float* q_fb[FQ ? Q_LD : 1];
    bool q_first[FQ ? Q_LD : 1];
    if constexpr (FQ) {
#pragma unroll
        for (int j = 0; j < Q_LD; ++j) {
            q_first[j] = q_cs[j] == p.c0;
            q_fb[j] = q_ptr[j] ? q_ptr[j] + (long long)(q_dr[j] + (q_r[j] - p.pad) * p.Wi + (q_s[j] - p.pad)) * q_cs[j]
                               : g_wg_zero16;
            q_r[j] -= p.pad;
            q_s[j] -= p.pad;
        }
    }
    const float* p_lane = p.P + (long long)p_dr * p.N + pn;

    auto issue = [&](int m0, int slot) {
        float* ps = lds + slot * STAGE;
        float* qs = ps + WG_BM * BN;
#pragma unroll
        for (int j = 0; j < P_LD; ++j) {
            const int I = (P_TOT % NW) ? wave + NW * j : wave * P_LD + j;
            const int row0 = I * P_ROWS;
            const int m = m0 + row0 + p_dr;
            const float* g = g_wg_zero16;
            float* dst = ps + row0 * BN;
            if (SINK && I >= P_TOT) dst = lds + NBUF * STAGE;
            else if (m < m_end && p_in) g = p_lane + (long long)(m0 + row0) * p.N;
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)dst, 16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < Q_LD; ++j) {
            const int mu = m0 + q_row0[j];   // wave-uniform: decomposed on the scalar unit
            const int tu = fdiv(mu, p.dWo);
            const int wou = mu - tu * p.Wo;
            const int bu = fdiv(tu, p.dHo);
            const int hou = tu - bu * p.Ho;
            if constexpr (FQ) {
                int wo = wou + q_dr[j];
                const bool cw = wo >= p.Wo;
                wo = cw ? wo - p.Wo : wo;
                int ho = hou + (cw ? 1 : 0);
                ho = ho >= p.Ho ? ho - p.Ho : ho;
                const int hi = ho + q_r[j], wi = wo + q_s[j];
                const bool ok = mu + q_dr[j] < m_end && q_ptr[j] && (unsigned)hi < (unsigned)p.Hi &&
                                (unsigned)wi < (unsigned)p.Wi;
                const long long mo = q_first[j] ? (long long)mu * p.c0 : (long long)mu * p.c1;
                const float* g = ok ? q_fb[j] + mo : g_wg_zero16;
                __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(qs + (wave * Q_LD + j) * 256), 16, 0, 0);
                continue;
            }
            // lane delta with carry, branch-free (keeps the main loop one basic block)
            int wo = wou + q_dr[j];
            const int cw = fdiv(wo, p.dWo);
            wo -= cw * p.Wo;
            int ho = hou + cw;
            const int ch = fdiv(ho, p.dHo);
            ho -= ch * p.Ho;
            const int b = bu + ch;
            const float* g = g_wg_zero16;
            if (mu + q_dr[j] < m_end && q_ptr[j]) {
                const int hi = ho * p.stride - p.pad + q_r[j], wi = wo * p.stride - p.pad + q_s[j];
                if ((unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi)
                    g = q_ptr[j] + ((long long)b * p.Hi * p.Wi + (long long)hi * p.Wi + wi) * q_cs[j];
            }
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(qs + (wave * Q_LD + j) * 256), 16, 0, 0);
        }
    };

    f32x16 acc[FK][FN];
#pragma unroll
    for (int i = 0; i < FK; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int a_col0 = wn * (BN / WN) + lr;   // n columns this lane reads from P
    const int b_col0 = wk * (BK / WK) + lr;   // k columns this lane reads from Q
    const int T = (m_end > m_begin) ? (m_end - m_begin + WG_BM - 1) / WG_BM : 0;

    // bias column sums (block-uniform role): mode 1 sums P columns in k-tile 0, mode 2 Q columns in n-tile 0
    const int bias_w = (p.bias_mode == 1 && tx == 0) ? BN : (p.bias_mode == 2 && ty == 0) ? BK : 0;
    float bsum = 0.f;

    // every iteration issues one stage (past m_end: zero page), so the counted wait is constant
#pragma unroll
    for (int s0 = 0; s0 < NBUF - 1; ++s0) issue(m_begin + s0 * WG_BM, s0);

    for (int t = 0; t < T; ++t) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 2) * G) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const float* ps = lds + (t % NBUF) * STAGE;
        const float* qs = ps + WG_BM * BN;
        if constexpr (X6) {
            float xa[FN][8], xb[FK][8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int row = 8 * lh + e;
#pragma unroll
                for (int j = 0; j < FN; ++j) xa[j][e] = ps[row * BN + a_col0 + j * 32];
#pragma unroll
                for (int i = 0; i < FK; ++i) xb[i][e] = qs[row * BK + b_col0 + i * 32];
            }
            wg_bf16x8 ph[FN], pm[FN], pl[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) wg_split3(xa[j], ph[j], pm[j], pl[j]);
#pragma unroll
            for (int i = 0; i < FK; ++i) {
                wg_bf16x8 qh, qm, ql;
                wg_split3(xb[i], qh, qm, ql);
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    f32x16 c = acc[i][j];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, pm[j], c, 0, 0, 0);   // small terms first
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ql, ph[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, pl[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, ph[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, pm[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, ph[j], c, 0, 0, 0);
                    acc[i][j] = c;
                }
                if (i == 0) issue(m_begin + (t + NBUF - 1) * WG_BM, (t + NBUF - 1) % NBUF);
            }
        } else {
        // the whole stage's operands up front ((FN+FK)*8 VGPRs): the reads of step ks+1.. land
        // under the MFMAs of step ks instead of a lgkmcnt(0) bubble before every step
        float fa[WG_BM / 2][FN], fb[WG_BM / 2][FK];
#pragma unroll
        for (int ks = 0; ks < WG_BM / 2; ++ks) {
            const int row = ks * 2 + lh;
#pragma unroll
            for (int j = 0; j < FN; ++j) fa[ks][j] = ps[row * BN + a_col0 + j * 32];
#pragma unroll
            for (int i = 0; i < FK; ++i) fb[ks][i] = qs[row * BK + b_col0 + i * 32];
        }
#pragma unroll
        for (int ks = 0; ks < WG_BM / 2; ++ks) {
#pragma unroll
            for (int i = 0; i < FK; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[ks][i], fa[ks][j], acc[i][j], 0, 0, 0);
            // next stage's loads mid-stage: address arithmetic overlaps the MFMAs
            if (ks == 1) issue(m_begin + (t + NBUF - 1) * WG_BM, (t + NBUF - 1) % NBUF);
        }
        // pin the order the default scheduler undoes (it sinks each read next to its MFMA):
        // all operand reads of the stage, then the MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, (WG_BM / 2) * (FN + FK), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, (WG_BM / 2) * FN * FK, 0);
        }
        // bias column sums after the MFMA block (a divergent branch here does not split it)
        if (tid < bias_w) {   // one column per thread, all rows of the stage
            const float* img = p.bias_mode == 1 ? ps : qs;
#pragma unroll
            for (int r = 0; r < WG_BM; ++r) bsum += img[r * bias_w + tid];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain the past-the-end zero-page loads

    // partial tile -> slab[z][n][k] (row stride Kcp, float4 over 4 consecutive k)
    float* slab = p.slab + (long long)tz * p.Nr * p.Kcp;
    if (tid < bias_w) {
        if (p.bias_mode == 1) {
            const int n = n_blk + tid;
            if (n < p.N) slab[(long long)n * p.Kcp + p.K] = bsum;
        } else {
            const int k = k_blk + tid;
            if (k < p.K) slab[(long long)p.N * p.Kcp + k] = bsum;
        }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int n = n_blk + wn * (BN / WN) + j * 32 + lr;
        if (n >= p.N) continue;
#pragma unroll
        for (int i = 0; i < FK; ++i) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = k_blk + wk * (BK / WK) + i * 32 + 8 * q + 4 * lh;
                if (k >= p.K) continue;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                *reinterpret_cast<f32x4*>(slab + (long long)n * p.Kcp + k) = v;
            }
        }
    }
}

typedef short wi16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) wi16x4 lds_i16x4_t;
// swizzle of 16-byte chunks in 256-byte rows: conflict-free ds_read_b64_tr_b16
__device__ __forceinline__ int wb_sw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// ------------------------------------------ 6-product weight gradient with halo reuse (3x3/s1)
// dW[n][tap][c] = sum_m dZ[m][n] * X[m + tap][c].  A stage is 16 consecutive output pixels of one
// image row; the 9 taps read only the 3 x 18 halo pixels around them, so the block loads and
// splits that halo ONCE (54 pixel rows x 64 channels, instead of 9 x 16 im2col rows) together
// with the 16 dZ rows (64 channels), writes the hi / mid / lo bf16 planes into LDS (row-major,
// 128-byte rows, 16-byte chunk ch of row r at ch ^ 4*((r >> 1) & 1): conflict-free transposed
// reads), and every wave reads its MFMA operands with ds_read_b64_tr_b16: tap (r, s) is the
// 16-row window starting at halo row 18 r + s.  Block tile: 64 output channels x 64 input
// channels x all 9 taps, 4 waves = (channel half, output half), each 9 accumulators (one per
// tap).  Raw fp32 rows arrive in registers one stage ahead (global_load_dwordx4; halo pixels
// outside the image are zero); the planes are double buffered, one barrier per stage.
// Requires stride 1, pad 1, 3x3, Hi == Ho, Wi == Wo, Wo % 16 == 0, c0 % 64 == c1 % 64 == 0,
// N % 64 == 0, bias_mode != 2, every source under 2^31 elements.
constexpr int HX_ROWS = 54;                   // halo pixel rows (3 x 18)
constexpr int HX_IMG = (HX_ROWS + 16) * 128;  // bytes of one plane: X rows, then 16 dZ rows
__device__ __forceinline__ int hx_off(int row, int col) {   // byte offset in a 64-column plane
    return row * 128 + 16 * ((col >> 3) ^ (((row >> 1) & 1) << 2)) + 2 * (col & 7);
}

// NT = 64-channel output tiles per block: NT = 1 is 4 waves (two blocks per CU); NT = 2 is 8 waves
// (one block per CU) sharing each loaded and split X halo between 128 output channels - half the
// X reads and splits per MFMA, 12 instead of 20 raw-row registers per thread.
template <int NT>
__global__ __launch_bounds__(256 * NT) void wgrad_halo_x6_kernel(const WgradParams p) {
    constexpr int NTH = 256 * NT;
    constexpr int RS = NTH / 16;              // halo rows per X group (16 NT: keeps the row swizzle)
    constexpr int XG = (HX_ROWS + RS - 1) / RS;   // X float4 groups per thread (864 = 3 x 256 + 96 | 512 + 352)
    constexpr int IMG = (HX_ROWS + 16 * NT) * 128;  // one plane: 54 X rows, then NT x 16 dZ rows
    __shared__ __attribute__((aligned(16))) char lds[2 * 3 * IMG];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ci = wave & 1, nj = (wave >> 1) & 1, nt = wave >> 2;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % p.gx;               // 64-channel input tile
    const int tyz = tile / p.gx;
    const int ty = tyz % p.gy;                // 64-channel output tile
    const int tz = tyz / p.gy;
    const int m_begin = tz * p.mps;
    const int m_end = min(p.M, m_begin + p.mps);
    const int T = m_end > m_begin ? (m_end - m_begin) / 16 : 0;

    // ---- thread roles in the loads: column quad cq (fixed), halo pixel rows hp_i = tid/16 + RS i
    const int cq = tid & 15;
    const int c_lo = tx * 64;                 // first input channel of the tile
    const bool first = c_lo < p.c0;
    const float* xsrc = first ? p.src0 + c_lo : p.src1 + (c_lo - p.c0);
    const int cs = first ? p.c0 : p.c1;
    const float* x_lane[XG];
    unsigned x_cls[XG];                       // edge classes: 1 top, 2 bottom, 4 left, 8 right, 16 past the halo, 32 all
#pragma unroll
    for (int i = 0; i < XG; ++i) {
        const int hp = (tid >> 4) + RS * i;
        const int rr = hp / 18, cc = hp - rr * 18;
        x_lane[i] = xsrc + (long long)((rr - 1) * p.Wi + (cc - 1)) * cs + cq * 4;
        if (hp >= HX_ROWS) x_lane[i] = g_wg_zero16;   // rows past the halo: class 16 -> zero page, never stored
        x_cls[i] = 32u | (hp >= HX_ROWS ? 16u
                                        : ((rr == 0 ? 1u : 0u) | (rr == 2 ? 2u : 0u) | (cc == 0 ? 4u : 0u) | (cc == 17 ? 8u : 0u)));
    }
    // dZ roles: row prow of the stage, channel quad pq of the block's 64 NT output channels
    const int pq = tid % (16 * NT), prow = tid / (16 * NT);
    const float* p_lane = p.P + (long long)prow * p.N + ty * 64 * NT + pq * 4;

    f32x4 rx[XG], rp;
    auto load = [&](int t) {                  // raw rows of stage t into registers (branch-free:
        const int m0 = m_begin + 16 * t;      // out-of-image halo pixels read the zero page)
        const int tu = fdiv(m0, p.dWo);
        const int wo0 = m0 - tu * p.Wo;
        const int bu = fdiv(tu, p.dHo);
        const int ho = tu - bu * p.Ho;
        const bool live = t < T;
        // a stage past the split's end (prefetch beyond T) reads the zero page in every lane
        const unsigned flags = live ? (16u | (ho == 0 ? 1u : 0u) | (ho == p.Ho - 1 ? 2u : 0u) | (wo0 == 0 ? 4u : 0u) |
                                       (wo0 + 16 == p.Wo ? 8u : 0u))
                                    : 0xffffffffu;
        const unsigned xo = __umul24((unsigned)m0, (unsigned)cs);
#pragma unroll
        for (int i = 0; i < XG; ++i) {
            const float* g = (x_cls[i] & flags) ? g_wg_zero16 : x_lane[i] + xo;
            rx[i] = *reinterpret_cast<const f32x4*>(g);
        }
        const float* gp = live ? p_lane + __umul24((unsigned)m0, (unsigned)p.N) : g_wg_zero16;
        rp = *reinterpret_cast<const f32x4*>(gp);
    };
    f32x4 bsum = {0.f, 0.f, 0.f, 0.f};
    const bool bias_blk = p.bias_mode == 1 && tx == 0;
    // plane writes: halo rows hp_i = hp_0 + RS i keep the swizzle of hp_0 (RS i = 0 mod 4), so
    // every write of a thread is one base address plus an immediate
    const int w_base = hx_off(tid >> 4, cq * 4);
    const int wp_base = hx_off(HX_ROWS + 16 * (pq >> 4) + prow, (pq & 15) * 4);
    auto split_store = [&](int buf) {         // registers -> bf16 planes of buffer buf
        char* pb = lds + buf * 3 * IMG;
        auto put = [&](char* dst, const f32x4 v) {
            unsigned h[2], m[2], l[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
#pragma clang fp contract(off)
                const float x0 = v[2 * q], x1 = v[2 * q + 1];
                const unsigned a = wg_pk(wg_f32x2{x0, x1});
                const float r0 = x0 - __builtin_bit_cast(float, a << 16);
                const float r1 = x1 - __builtin_bit_cast(float, a & 0xffff0000u);
                const unsigned b = wg_pk(wg_f32x2{r0, r1});
                const float l0 = r0 - __builtin_bit_cast(float, b << 16);
                const float l1 = r1 - __builtin_bit_cast(float, b & 0xffff0000u);
                h[q] = a;
                m[q] = b;
                l[q] = wg_pk(wg_f32x2{l0, l1});
            }
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u32x2*>(dst) = u32x2{h[0], h[1]};
            *reinterpret_cast<u32x2*>(dst + IMG) = u32x2{m[0], m[1]};
            *reinterpret_cast<u32x2*>(dst + 2 * IMG) = u32x2{l[0], l[1]};
        };
#pragma unroll
        for (int i = 0; i < XG; ++i) {
            const int hp = (tid >> 4) + RS * i;
            if (i < XG - 1 || hp < HX_ROWS) put(pb + w_base + i * RS * 128, rx[i]);
        }
        put(pb + wp_base, rp);
        if (bias_blk) bsum += rp;
    };

    f32x16 acc[9];
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t9][r] = 0.f;

    // transposed reads: group grp = lane>>4 covers columns 16 (grp&1) + 0..15, rows 8 (grp>>1) +
    // gq (+4); lane 4 gq + gp addresses row gq, columns 4 gp .. 4 gp + 3
    const int grp = lane >> 4, gq = (lane >> 2) & 3, gp = lane & 3;
    const int rsub = 8 * (grp >> 1) + gq;
    const int ccol = 16 * (grp & 1) + 4 * gp;
    // tap (r, s) reads halo rows 18 r + s + rsub (+4): rows congruent mod 4 share the swizzle, so
    // the 9 taps need 3 base addresses (18 r + s mod 4 in {0, 1, 2, 3}) plus immediates
    int xb[4];
#pragma unroll
    for (int res = 0; res < 4; ++res) xb[res] = hx_off(res + rsub, ci * 32 + ccol);
    const int pbase = hx_off(HX_ROWS + 16 * nt + rsub, nj * 32 + ccol);
    auto tr2 = [&](const char* a) {           // rows +0 / +4 of a fragment -> one MFMA operand
        const wi16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a);
        const wi16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(a + 4 * 128));
        typedef short wi16x8 __attribute__((ext_vector_type(8)));
        const wi16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        return __builtin_bit_cast(wg_bf16x8, av);
    };
    auto mfma_stage = [&](auto bufc) {
        constexpr int buf = decltype(bufc)::value;
        const char* pb = lds + buf * 3 * IMG;
        const wg_bf16x8 ph = tr2(pb + pbase), pm = tr2(pb + IMG + pbase), pl = tr2(pb + 2 * IMG + pbase);
#pragma unroll
        for (int t9 = 0; t9 < 9; ++t9) {
            const int row0 = (t9 / 3) * 18 + (t9 % 3);
            const char* xa = pb + xb[row0 & 3] + (row0 & ~3) * 128;
            const wg_bf16x8 qh = tr2(xa), qm = tr2(xa + IMG), ql = tr2(xa + 2 * IMG);
            f32x16 c = acc[t9];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, pm, c, 0, 0, 0);   // small terms first
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ql, ph, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, pl, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, ph, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, pm, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, ph, c, 0, 0, 0);
            acc[t9] = c;
        }
    };
    auto step = [&](int t, auto bufc) {       // MFMAs of stage t (buffer t & 1), split stage t+1
        constexpr int buf = decltype(bufc)::value;
        mfma_stage(bufc);
        if (t + 1 < T) {
            split_store(buf ^ 1);             // raw(t+1) has been in flight for a whole stage
            load(t + 2);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");     // s_barrier is no compiler fence: keep LDS reads behind it
    };

    if (T > 0) {
        load(0);
        split_store(0);
        load(1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");     // s_barrier is no compiler fence: keep LDS reads behind it
    }
    int t = 0;
    for (; t + 1 < T; t += 2) {
        step(t, std::integral_constant<int, 0>{});
        step(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < T) step(t, std::integral_constant<int, 0>{});

    float* slab = p.slab + (long long)tz * p.Nr * p.Kcp;
    if (bias_blk) {                           // column sums of dZ: 16 rows of partials per column
        f32x4* red = reinterpret_cast<f32x4*>(lds);
        red[tid] = bsum;
        __syncthreads();
        if (tid < 16 * NT) {
            f32x4 v = red[tid];
            for (int r = 1; r < 16; ++r) v += red[r * 16 * NT + tid];
#pragma unroll
            for (int e = 0; e < 4; ++e) slab[(long long)(ty * 64 * NT + tid * 4 + e) * p.Kcp + p.K] = v[e];
        }
    }
    const int lr = lane & 31, lh = lane >> 5;
    const int n = ty * 64 * NT + nt * 64 + nj * 32 + lr;
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = t9 * p.C + c_lo + ci * 32 + 8 * q + 4 * lh;
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[t9][4 * q + e];
            *reinterpret_cast<f32x4*>(slab + (long long)n * p.Kcp + k) = v;
        }
    }
}

// ------------------------------------------ Winograd-domain 3x3 weight gradient (F(2x2, 3x3))
// The forward of F(2x2,3x3) is y = A^T [ (G g G^T) (.) (B^T d B) ] A (winograd.hip); its
// derivative w.r.t. the kernel g, summed over the 2x2 output tiles (d = the tile's 4x4 input
// window, e = its 2x2 output gradient), is
//     dW = G^T M G,   M_xi[n][c] = sum_tiles Ehat_xi[tile][n] Dhat_xi[tile][c]  (xi = 16 positions)
// with Ehat = A e A^T and Dhat = B^T d B - both formed with +-1 adds only, so every operand is an
// fp32 value that splits exactly into hi/mid/lo bf16 and the products are the same 6-term fp32
// arithmetic as every other weight gradient here, accumulated in fp32.  16 products per tile and
// (n, c) instead of the direct 36 (9 taps x 4 pixels): 2.25x fewer MFMAs.  G^T M G (factors 1/2,
// exact scalings) runs once per block on its fp32 partial M, so the slab keeps the direct
// kernels' [split][n][tap * C + c] layout (+ the bias column) and the same fixed-order fp64
// reduction finishes it - deterministic.
//
// Block: 64 output x 64 input channels x all 16 positions over a contiguous range of tiles (one
// split), 8 waves; wave (wc, wn, wj) accumulates 32 input x 32 output channels for the 8 positions
// (i, 2 wj + jj): 128 accumulators.  A stage is 16 tiles = one k-step of v_mfma_f32_32x32x16_bf16,
// split into 4 sub-stages, one per row i of the positions (as winograd.hip).  Thread (tile pt,
// channel pair cp) keeps its tile's 4x4 window (2 input channels) and 2x2 gradient tile (2 output
// channels) in registers and forms row i of Dhat and Ehat for the next sub-stage while the MFMAs
// of the current one run; the planes go to LDS as [tile row][64 channels] bf16 images (128-byte
// rows, the halo kernel's swizzle) read back with ds_read_b64_tr_b16 (k = tile).  Each window row
// is reloaded for the next stage as soon as its last transform is formed (>= 2 sub-stages of
// cover).  Ehat is formed with the sign-normalised A' = [1 0; 1 1; 1 -1; 0 1] (A's row 3 is
// [0 -1]): M_xi = s_i s_j M'_xi, s = (1, 1, 1, -1), applied in the output transform.
constexpr int WW_IMG = 16 * 128;           // one (position, plane) image: 16 tile rows x 64 channels
constexpr int WW_SLOT = 4 * 3 * WW_IMG;    // one operand, one sub-stage: 4 positions x 3 planes

struct WinoWgradParams {
    WgradParams p;
    int tiles, tps;            // tiles (batch x Ho/2 x Wo/2); tiles per split (multiple of 16)
    FastDiv dTw, dTh;          // tile index -> (image, tile row, tile column)
    unsigned x0_bytes, x1_bytes, p_bytes;   // buffer ranges (sources shifted back by Wi + 1 pixels)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ww_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    void* ub = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(ub, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// x -> hi/mid/lo bf16 of both lanes of the pair, packed (x = hi + mid + lo exactly)
__device__ __forceinline__ void ww_split(const wg_f32x2 x, unsigned& h, unsigned& m, unsigned& l) {
#pragma clang fp contract(off)
    const unsigned a = wg_pk(x);
    const float r0 = x[0] - __builtin_bit_cast(float, a << 16);
    const float r1 = x[1] - __builtin_bit_cast(float, a & 0xffff0000u);
    const unsigned b = wg_pk(wg_f32x2{r0, r1});
    const float l0 = r0 - __builtin_bit_cast(float, b << 16);
    const float l1 = r1 - __builtin_bit_cast(float, b & 0xffff0000u);
    h = a;
    m = b;
    l = wg_pk(wg_f32x2{l0, l1});
}

__global__ __launch_bounds__(512) void wgrad_wino_x6_kernel(const WinoWgradParams w) {
#pragma clang fp contract(off)
    const WgradParams& p = w.p;
    // two sub-stage slots per operand, as separate arrays: the compiler then knows that the
    // plane stores of the next sub-stage (other slot) do not alias this sub-stage's operand reads
    // and can interleave them; after the loop lx0 / lx1 carry the output-transform exchange
    __shared__ __attribute__((aligned(16))) char lx0[WW_SLOT];
    __shared__ __attribute__((aligned(16))) char lx1[WW_SLOT];
    __shared__ __attribute__((aligned(16))) char lg0[WW_SLOT];
    __shared__ __attribute__((aligned(16))) char lg1[WW_SLOT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wc = wave & 1, wn = (wave >> 1) & 1, wj = wave >> 2;
    // logical block (split z, output block ny, input block cx), cx fastest: the blocks an XCD runs
    // together read the same tiles
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int cx = blk % p.gx;
    const int rest = blk / p.gx;
    const int ny = rest % p.gy;
    const int z = rest / p.gy;
    const int t_begin = z * w.tps;
    const int t_end = min(w.tiles, t_begin + w.tps);
    const int S = (t_end - t_begin + 15) >> 4;

    // ---- producer role: tile pt of a stage, channel pair cp of the 64 input / 64 output channels
    const int pt = tid >> 5, cp = tid & 31;
    const int c_lo = cx * 64;
    const bool first = c_lo < p.c0;
    const int cs = first ? p.c0 : p.c1;       // pixel stride of the input block's source
    const int shift = p.Wi + 1;               // window corner (2ty-1, 2tx-1) >= (-1, -1)
    const __amdgpu_buffer_rsrc_t xr = ww_rsrc((first ? p.src0 : p.src1) - (long long)shift * cs,
                                              first ? w.x0_bytes : w.x1_bytes);
    const __amdgpu_buffer_rsrc_t gr = ww_rsrc(p.P, w.p_bytes);
    const unsigned pixb = (unsigned)cs * 4u;
    const unsigned xco = (unsigned)((first ? c_lo : c_lo - p.c0) + 2 * cp) * 4u;
    const unsigned gco = (unsigned)(ny * 64 + 2 * cp) * 4u;
    const unsigned gpix = (unsigned)p.N * 4u;
    const int st_off = hx_off(pt, 2 * cp);    // the thread's 4-byte slot in every image

    // window rows of a stage as the loader sees them (byte offsets; LEAN_OOB: zeros)
    unsigned xv[4];
    bool xc0 = false, xc3 = false;
    auto decode_x = [&](int k) {
        const int m = t_begin + 16 * k + pt;
        const bool mv = m < t_end;
        int ty = 0, tx = 0, b = 0;
        if (mv) {
            const int t2 = fdiv(m, w.dTw);
            tx = m - t2 * (p.Wo >> 1);
            b = fdiv(t2, w.dTh);
            ty = t2 - b * (p.Ho >> 1);
        }
        const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
        const unsigned base = (unsigned)(((b * p.Hi + y0) * p.Wi + x0 + shift) * cs) * 4u + xco;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            xv[r] = mv && (unsigned)(y0 + r) < (unsigned)p.Hi ? base + (unsigned)(r * p.Wi) * pixb : LEAN_OOB;
        xc0 = x0 >= 0;
        xc3 = x0 + 3 < p.Wi;
    };
    unsigned gv[2];
    auto decode_g = [&](int k) {
        const int m = t_begin + 16 * k + pt;
        if (m < t_end) {
            const int t2 = fdiv(m, w.dTw);
            const int tx = m - t2 * (p.Wo >> 1);
            const int b = fdiv(t2, w.dTh);
            const int ty = t2 - b * (p.Ho >> 1);
            const unsigned base = (unsigned)((b * p.Ho + 2 * ty) * p.Wo + 2 * tx) * gpix + gco;
            gv[0] = base;
            gv[1] = base + (unsigned)p.Wo * gpix;
        } else {
            gv[0] = gv[1] = LEAN_OOB;
        }
    };
    wg_f32x2 d[4][4], e[2][2];
    auto load_x = [&](int r) {
        if (PU_WW_ABL == 3) {
#pragma unroll
            for (int s = 0; s < 4; ++s) d[r][s] = wg_f32x2{1.f + r, 2.f - s};
            return;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            unsigned vo = xv[r];
            if (s == 0) vo = xc0 ? vo : LEAN_OOB;
            if (s == 3) vo = xc3 ? vo : LEAN_OOB;
            d[r][s] = __builtin_bit_cast(wg_f32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                                       xr, vo, __builtin_amdgcn_readfirstlane(s * pixb), 0));
        }
    };
    auto load_g = [&](int a) {
        if (PU_WW_ABL == 3) {
            e[a][0] = e[a][1] = wg_f32x2{0.5f, 0.25f * a};
            return;
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
            e[a][s] = __builtin_bit_cast(wg_f32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                                       gr, gv[a], __builtin_amdgcn_readfirstlane(s * gpix), 0));
    };
    // row i of Dhat (B^T d B) and Ehat (A' e A'^T) for this thread's pairs -> bf16 planes in the
    // sub-stage slots sx / sg: image (j, plane) at (3 j + plane) * WW_IMG
    auto form = [&](auto i_c, char* sx, char* sg) {
        constexpr int i = decltype(i_c)::value;
        if (PU_WW_ABL == 2) return;
        wg_f32x2 t[4], u[2];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if constexpr (i == 0) t[s] = d[0][s] - d[2][s];
            else if constexpr (i == 1) t[s] = d[1][s] + d[2][s];
            else if constexpr (i == 2) t[s] = d[2][s] - d[1][s];
            else t[s] = d[1][s] - d[3][s];
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (i == 0) u[s] = e[0][s];
            else if constexpr (i == 1) u[s] = e[0][s] + e[1][s];
            else if constexpr (i == 2) u[s] = e[0][s] - e[1][s];
            else u[s] = e[1][s];
        }
        const wg_f32x2 dv[4] = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
        const wg_f32x2 ev[4] = {u[0], u[0] + u[1], u[0] - u[1], u[1]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            unsigned h, m, l;
            ww_split(dv[j], h, m, l);
            char* b = sx + 3 * j * WW_IMG + st_off;
            *reinterpret_cast<unsigned*>(b) = h;
            *reinterpret_cast<unsigned*>(b + WW_IMG) = m;
            *reinterpret_cast<unsigned*>(b + 2 * WW_IMG) = l;
            ww_split(ev[j], h, m, l);
            b = sg + 3 * j * WW_IMG + st_off;
            *reinterpret_cast<unsigned*>(b) = h;
            *reinterpret_cast<unsigned*>(b + WW_IMG) = m;
            *reinterpret_cast<unsigned*>(b + 2 * WW_IMG) = l;
        }
    };

    // ---- MFMA role: transposed fragment reads as in wgrad_halo_x6_kernel (k = tile row)
    const int grp = lane >> 4, gq = (lane >> 2) & 3, gp = lane & 3;
    const int rsub = 8 * (grp >> 1) + gq;
    const int ccol = 16 * (grp & 1) + 4 * gp;
    const int xa = hx_off(rsub, wc * 32 + ccol) + 2 * wj * 3 * WW_IMG;
    const int ga = hx_off(rsub, wn * 32 + ccol) + 2 * wj * 3 * WW_IMG;
    auto tr2 = [&](const char* a) {
        const wi16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a);
        const wi16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(a + 4 * 128));
        typedef short wi16x8 __attribute__((ext_vector_type(8)));
        const wi16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        return __builtin_bit_cast(wg_bf16x8, av);
    };
    f32x16 acc[8];                            // [i][jj]: position (i, 2 wj + jj)
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;
    auto mma = [&](auto x_c, const char* sx, const char* sg, int jj) {
        constexpr int x = decltype(x_c)::value;
        const char* xb = sx + xa + jj * 3 * WW_IMG;
        const char* gb = sg + ga + jj * 3 * WW_IMG;
        const wg_bf16x8 qh = tr2(xb), qm = tr2(xb + WW_IMG), ql = tr2(xb + 2 * WW_IMG);
        const wg_bf16x8 ph = tr2(gb), pm = tr2(gb + WW_IMG), pl = tr2(gb + 2 * WW_IMG);
        if (PU_WW_ABL == 1) {             // keep the operand reads alive, drop the MFMAs
            acc[x][0] += __builtin_bit_cast(float, __builtin_shufflevector(qh, qm, 0, 1)) +
                         __builtin_bit_cast(float, __builtin_shufflevector(ql, ph, 0, 1)) +
                         __builtin_bit_cast(float, __builtin_shufflevector(pm, pl, 0, 1));
            return;
        }
        f32x16 c = acc[x];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, pm, c, 0, 0, 0);   // small terms first
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ql, ph, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, pl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, ph, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, pm, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, ph, c, 0, 0, 0);
        acc[x] = c;
    };
    wg_f32x2 bsum = {0.f, 0.f};               // dbias partial of the thread's output pair

    // sub-stage (k, i): MFMAs of row i from slot i & 1, row i + 1 (or the next stage's row 0)
    // formed into the other slot, then the window / gradient rows whose last use that was are
    // reloaded for the next stage (x row 0 two stages ahead: its stage-k + 1 copy was formed in
    // the sub-stage before)
    auto sub = [&](int k, auto i_c) {
        constexpr int i = decltype(i_c)::value;
        char* sx = (i & 1) ? lx1 : lx0;
        char* sg = (i & 1) ? lg1 : lg0;
        char* nx = (i & 1) ? lx0 : lx1;
        char* ng = (i & 1) ? lg0 : lg1;
        mma(std::integral_constant<int, 2 * i>{}, sx, sg, 0);
        // (past the last stage this forms zeros into a slot no MFMA reads: the sub-stage stays
        // one basic block for the interleave below)
        form(std::integral_constant<int, (i + 1) & 3>{}, nx, ng);
        if constexpr (i == 1) {               // d row 2 and e row 0 are dead: next stage's
            load_x(2);
            bsum += e[0][0] + e[0][1];
            decode_g(k + 1);
            load_g(0);
        } else if constexpr (i == 2) {        // d rows 1, 3 and e row 1 are dead
            load_x(1);
            load_x(3);
            bsum += e[1][0] + e[1][1];
            load_g(1);
        } else if constexpr (i == 3) {        // d row 0 of stage k + 1 was used: stage k + 2's
            decode_x(k + 2);
            load_x(0);
        }
        mma(std::integral_constant<int, 2 * i + 1>{}, sx, sg, 1);
        // Interleave: the wave's 12 MFMAs spread over the forming work (~110 VALU + 24 LDS
        // stores) instead of 6 before and 6 after it - the two waves of a SIMD run the same phase
        // between barriers, so MFMAs bunched at the ends leave the matrix pipe idle during the VALU
#if !PU_NO_ILV && PU_WW_ABL == 0
        __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);       // position 0 operands
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 9, 0);     // ~1/12 of the VALU
            __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);     // ~1/12 of the plane stores
            if (q == 2) __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);   // position 1 operands
        }
#endif
        if (PU_WW_ABL != 4) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");     // s_barrier is no compiler fence: keep LDS reads behind it
        }
    };

    // prologue: stage 0 whole, sub-stage (0, 0) formed, stage 1's row 0 in flight
    decode_x(0);
    load_x(0);
    load_x(1);
    load_x(2);
    load_x(3);
    decode_g(0);
    load_g(0);
    load_g(1);
    form(std::integral_constant<int, 0>{}, lx0, lg0);
    decode_x(1);
    load_x(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int k = 0; k < S; ++k) {
        sub(k, std::integral_constant<int, 0>{});
        sub(k, std::integral_constant<int, 1>{});
        sub(k, std::integral_constant<int, 2>{});
        sub(k, std::integral_constant<int, 3>{});
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // trailing (empty-range) loads

    float* slab = p.slab + (long long)z * p.Nr * p.Kcp;
    // ---- bias: column sums of dZ over the split, fixed order (thread stages, then the 16 tiles)
    if (p.bias_mode == 1 && cx == 0) {
        wg_f32x2* red = reinterpret_cast<wg_f32x2*>(lg0);
        red[tid] = bsum;
        __syncthreads();
        if (tid < 32) {
            wg_f32x2 v = red[tid];
            for (int r = 1; r < 16; ++r) v += red[r * 32 + tid];
            slab[(long long)(ny * 64 + 2 * tid) * p.Kcp + p.K] = v[0];
            slab[(long long)(ny * 64 + 2 * tid + 1) * p.Kcp + p.K] = v[1];
        }
        __syncthreads();
    }

    // ---- output transform dW = G^T M G (G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]).  Over the rows
    // first (the wave holds all 4 rows of its 2 columns j): R[r][j] = sum_a G[a][r] M[a][j]; then
    // dW[r][s] = sum_j R[r][j] G[j][s] = P0[r][s] + P1[r][s], P0 from j = 0, 1 (wj = 0), P1 from
    // j = 2, 3 (wj = 1).  The two waves of a (wc, wn) pair swap halves through LDS: wave wj
    // finishes the channel groups q = 2 wj, 2 wj + 1 of its accumulators.  Signs: M = s_i s_j M'.
    const float sj1 = wj ? -1.f : 1.f;        // s_j of column jj = 1 (j = 3 for wj = 1)
    // 6 KB per wave: the wc = 0 pairs in lx0, the wc = 1 pairs in lx1
    float* xs = reinterpret_cast<float*>(wc ? lx1 : lx0) + (wn * 2 + wj) * 24 * 64;
    const float* xrd = reinterpret_cast<const float*>(wc ? lx1 : lx0) + (wn * 2 + (1 - wj)) * 24 * 64;
    const int lr = lane & 31, lh = lane >> 5;
    const int n = ny * 64 + wn * 32 + lr;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float mine[2][3][4], other[2][3][4];  // [q half][s][e]
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int ee = 0; ee < 4; ++ee) {
                const int idx = 4 * q + ee;
                float R[2];
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    // M[a][j] = s_a s_j M'[a][j]: s_3 = -1 on row a = 3 and on column j = 3
                    const float m0 = acc[0 * 2 + jj][idx], m1 = acc[1 * 2 + jj][idx];
                    const float m2 = acc[2 * 2 + jj][idx], m3 = -acc[3 * 2 + jj][idx];
                    float v = r == 0 ? m0 + 0.5f * (m1 + m2) : r == 1 ? 0.5f * (m1 - m2) : 0.5f * (m1 + m2) + m3;
                    R[jj] = jj == 1 ? sj1 * v : v;
                }
                // this wave's share of dW[r][s] for s = 0..2
                float P[3];
                if (wj == 0) {            // j = 0, 1: R0 G[0] + R1 G[1]
                    P[0] = R[0] + 0.5f * R[1];
                    P[1] = 0.5f * R[1];
                    P[2] = 0.5f * R[1];
                } else {                  // j = 2, 3: R2 G[2] + R3 G[3]
                    P[0] = 0.5f * R[0];
                    P[1] = -0.5f * R[0];
                    P[2] = 0.5f * R[0] + R[1];
                }
                const bool keep = (q >> 1) == wj;
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    if (keep) mine[q & 1][s][ee] = P[s];
                    else other[q & 1][s][ee] = P[s];
                }
            }
        // send the partner's half: [qh][s][e] -> 24 floats per lane
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
            for (int s = 0; s < 3; ++s)
#pragma unroll
                for (int ee = 0; ee < 4; ++ee) xs[((qh * 3 + s) * 4 + ee) * 64 + lane] = other[qh][s][ee];
        __syncthreads();
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                f32x4 v;
#pragma unroll
                for (int ee = 0; ee < 4; ++ee) {
                    const float o = xrd[((qh * 3 + s) * 4 + ee) * 64 + lane];
                    // P0 + P1 in that order on both waves of the pair
                    v[ee] = wj == 0 ? mine[qh][s][ee] + o : o + mine[qh][s][ee];
                }
                const int q = 2 * wj + qh;
                const int k = (3 * r + s) * p.C + c_lo + wc * 32 + 8 * q + 4 * lh;
                *reinterpret_cast<f32x4*>(slab + (long long)n * p.Kcp + k) = v;
            }
        __syncthreads();
    }
}

// ------------------------------------ Winograd-domain weight gradient on one wave per SIMD
// wgrad_wino_x6_kernel's arithmetic (the same Dhat / Ehat planes, the same 6 products per
// accumulator in the same order over the same 16-tile k-steps, the same G^T M G expression tree)
// on 4 waves with 256 accumulator registers each: wave wj owns position column j = wj (the 4
// positions (i, wj)) and all 2 x 2 32-channel blocks (input block cb x output block nb) of the
// block's 64 x 64 channels, so every X fragment feeds 2 MFMAs and every G fragment 2 - 12 fragment
// reads per 24 MFMAs instead of 12 per 12 (the 8-wave kernel moves 96 KB of LDS reads per
// sub-stage for 48 KB of plane stores; here 48 KB).  Producer role: thread (tile pt, channel quad
// cq) forms 4 channels with 16-byte window loads and 8-byte plane stores (the 8-wave kernel's two
// neighbouring channel-pair threads, the same bytes).  Output transform: wave wj forms
// R[r][j] = sum_a G[a][r] M[a][j] for all 4 blocks; per r one exchange round gives wave b all four
// R[r][j] of block b = (cb, nb) = (b >> 1, b & 1), which then forms dW[r][s] = P0 + P1 exactly as
// the 8-wave kernel's wave pairs do.  Bit-identical to wgrad_wino_x6_kernel.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void wgrad_wino4_x6_kernel(const WinoWgradParams w) {
#pragma clang fp contract(off)
    const WgradParams& p = w.p;
    __shared__ __attribute__((aligned(16))) char lx0[WW_SLOT];
    __shared__ __attribute__((aligned(16))) char lx1[WW_SLOT];
    __shared__ __attribute__((aligned(16))) char lg0[WW_SLOT];
    __shared__ __attribute__((aligned(16))) char lg1[WW_SLOT];
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wj = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int cx = blk % p.gx;
    const int rest = blk / p.gx;
    const int ny = rest % p.gy;
    const int z = rest / p.gy;
    const int t_begin = z * w.tps;
    const int t_end = min(w.tiles, t_begin + w.tps);
    const int S = (t_end - t_begin + 15) >> 4;

    // ---- producer role: tile pt of a stage, channel quad cq of the 64 input / 64 output channels
    const int pt = tid >> 4, cq = tid & 15;
    const int c_lo = cx * 64;
    const bool first = c_lo < p.c0;
    const int cs = first ? p.c0 : p.c1;
    const int shift = p.Wi + 1;
    const __amdgpu_buffer_rsrc_t xr = ww_rsrc((first ? p.src0 : p.src1) - (long long)shift * cs,
                                              first ? w.x0_bytes : w.x1_bytes);
    const __amdgpu_buffer_rsrc_t gr = ww_rsrc(p.P, w.p_bytes);
    const unsigned pixb = (unsigned)cs * 4u;
    const unsigned xco = (unsigned)((first ? c_lo : c_lo - p.c0) + 4 * cq) * 4u;
    const unsigned gco = (unsigned)(ny * 64 + 4 * cq) * 4u;
    const unsigned gpix = (unsigned)p.N * 4u;
    const int st_off = hx_off(pt, 4 * cq);    // the thread's 8-byte slot in every image

    unsigned xv[4];
    bool xc0 = false, xc3 = false;
    auto decode_x = [&](int k) {
        const int m = t_begin + 16 * k + pt;
        const bool mv = m < t_end;
        int ty = 0, tx = 0, b = 0;
        if (mv) {
            const int t2 = fdiv(m, w.dTw);
            tx = m - t2 * (p.Wo >> 1);
            b = fdiv(t2, w.dTh);
            ty = t2 - b * (p.Ho >> 1);
        }
        const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
        const unsigned base = (unsigned)(((b * p.Hi + y0) * p.Wi + x0 + shift) * cs) * 4u + xco;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            xv[r] = mv && (unsigned)(y0 + r) < (unsigned)p.Hi ? base + (unsigned)(r * p.Wi) * pixb : LEAN_OOB;
        xc0 = x0 >= 0;
        xc3 = x0 + 3 < p.Wi;
    };
    unsigned gv[2];
    auto decode_g = [&](int k) {
        const int m = t_begin + 16 * k + pt;
        if (m < t_end) {
            const int t2 = fdiv(m, w.dTw);
            const int tx = m - t2 * (p.Wo >> 1);
            const int b = fdiv(t2, w.dTh);
            const int ty = t2 - b * (p.Ho >> 1);
            const unsigned base = (unsigned)((b * p.Ho + 2 * ty) * p.Wo + 2 * tx) * gpix + gco;
            gv[0] = base;
            gv[1] = base + (unsigned)p.Wo * gpix;
        } else {
            gv[0] = gv[1] = LEAN_OOB;
        }
    };
    f32x4 d[4][4], e[2][2];
    auto load_x = [&](int r) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            unsigned vo = xv[r];
            if (s == 0) vo = xc0 ? vo : LEAN_OOB;
            if (s == 3) vo = xc3 ? vo : LEAN_OOB;
            d[r][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    xr, vo, __builtin_amdgcn_readfirstlane(s * pixb), 0));
        }
    };
    auto load_g = [&](int a) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
            e[a][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    gr, gv[a], __builtin_amdgcn_readfirstlane(s * gpix), 0));
    };
    // 4 fp32 values -> their hi / mid / lo bf16 planes at b (+ WW_IMG, + 2 WW_IMG), two pairs
    auto put = [&](char* b, const f32x4 v) {
        unsigned h0, m0, l0, h1, m1, l1;
        ww_split(wg_f32x2{v[0], v[1]}, h0, m0, l0);
        ww_split(wg_f32x2{v[2], v[3]}, h1, m1, l1);
        *reinterpret_cast<u32x2*>(b) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(b + WW_IMG) = u32x2{m0, m1};
        *reinterpret_cast<u32x2*>(b + 2 * WW_IMG) = u32x2{l0, l1};
    };
    // row i of Dhat and Ehat for this thread's 4 channels (wgrad_wino_x6_kernel's expressions)
    auto form = [&](auto i_c, char* sx, char* sg) {
        constexpr int i = decltype(i_c)::value;
        f32x4 t[4], u[2];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if constexpr (i == 0) t[s] = d[0][s] - d[2][s];
            else if constexpr (i == 1) t[s] = d[1][s] + d[2][s];
            else if constexpr (i == 2) t[s] = d[2][s] - d[1][s];
            else t[s] = d[1][s] - d[3][s];
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (i == 0) u[s] = e[0][s];
            else if constexpr (i == 1) u[s] = e[0][s] + e[1][s];
            else if constexpr (i == 2) u[s] = e[0][s] - e[1][s];
            else u[s] = e[1][s];
        }
        const f32x4 dv[4] = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
        const f32x4 ev[4] = {u[0], u[0] + u[1], u[0] - u[1], u[1]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            put(sx + 3 * j * WW_IMG + st_off, dv[j]);
            put(sg + 3 * j * WW_IMG + st_off, ev[j]);
        }
    };

    // ---- MFMA role: transposed fragment reads of position (i, wj), blocks cb / nb
    const int grp = lane >> 4, gq = (lane >> 2) & 3, gp = lane & 3;
    const int rsub = 8 * (grp >> 1) + gq;
    const int ccol = 16 * (grp & 1) + 4 * gp;
    const int xa0 = hx_off(rsub, ccol) + 3 * wj * WW_IMG;
    const int xa1 = hx_off(rsub, 32 + ccol) + 3 * wj * WW_IMG;
    auto tr2 = [&](const char* a) {
        const wi16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a);
        const wi16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(a + 4 * 128));
        typedef short wi16x8 __attribute__((ext_vector_type(8)));
        const wi16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        return __builtin_bit_cast(wg_bf16x8, av);
    };
    f32x16 acc[4][2][2];                      // [i][cb][nb]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][a][b][r] = 0.f;
    auto mma = [&](auto i_c, const char* sx, const char* sg) {
        constexpr int i = decltype(i_c)::value;
        wg_bf16x8 q[2][3], g[2][3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
            q[0][pl] = tr2(sx + xa0 + pl * WW_IMG);
            q[1][pl] = tr2(sx + xa1 + pl * WW_IMG);
            g[0][pl] = tr2(sg + xa0 + pl * WW_IMG);
            g[1][pl] = tr2(sg + xa1 + pl * WW_IMG);
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                f32x16 c = acc[i][cb][nb];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q[cb][1], g[nb][1], c, 0, 0, 0);   // small terms first
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q[cb][2], g[nb][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q[cb][0], g[nb][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q[cb][1], g[nb][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q[cb][0], g[nb][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q[cb][0], g[nb][0], c, 0, 0, 0);
                acc[i][cb][nb] = c;
            }
    };
    f32x4 bsum = {0.f, 0.f, 0.f, 0.f};        // dbias partial of the thread's 4 output channels

    // sub-stage (k, i): the MFMAs of row i from slot i & 1, row i + 1 (or the next stage's row 0)
    // formed into the other slot, then the reloads of wgrad_wino_x6_kernel's schedule
    auto sub = [&](int k, auto i_c) {
        constexpr int i = decltype(i_c)::value;
        char* sx = (i & 1) ? lx1 : lx0;
        char* sg = (i & 1) ? lg1 : lg0;
        char* nx = (i & 1) ? lx0 : lx1;
        char* ng = (i & 1) ? lg0 : lg1;
        mma(i_c, sx, sg);
        form(std::integral_constant<int, (i + 1) & 3>{}, nx, ng);
        if constexpr (i == 1) {               // d row 2 and e row 0 are dead: next stage's
            load_x(2);
            bsum += e[0][0] + e[0][1];
            decode_g(k + 1);
            load_g(0);
        } else if constexpr (i == 2) {        // d rows 1, 3 and e row 1 are dead
            load_x(1);
            load_x(3);
            bsum += e[1][0] + e[1][1];
            load_g(1);
        } else if constexpr (i == 3) {        // d row 0 of stage k + 1 was used: stage k + 2's
            decode_x(k + 2);
            load_x(0);
        }
#if !PU_NO_ILV
        // fragment reads first, then the 24 MFMAs with the formation (~6 VALU and one 8-byte plane
        // store per MFMA) in their shadow
        __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);
#pragma unroll
        for (int q = 0; q < 24; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
#endif
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    decode_x(0);
    load_x(0);
    load_x(1);
    load_x(2);
    load_x(3);
    decode_g(0);
    load_g(0);
    load_g(1);
    form(std::integral_constant<int, 0>{}, lx0, lg0);
    decode_x(1);
    load_x(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int k = 0; k < S; ++k) {
        sub(k, std::integral_constant<int, 0>{});
        sub(k, std::integral_constant<int, 1>{});
        sub(k, std::integral_constant<int, 2>{});
        sub(k, std::integral_constant<int, 3>{});
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    float* slab = p.slab + (long long)z * p.Nr * p.Kcp;
    // ---- bias: column sums of dZ over the split, fixed order (thread stages, then the 16 tiles)
    if (p.bias_mode == 1 && cx == 0) {
        f32x4* red = reinterpret_cast<f32x4*>(lg0);
        red[tid] = bsum;
        __syncthreads();
        if (tid < 16) {
            f32x4 v = red[tid];
            for (int r = 1; r < 16; ++r) v += red[r * 16 + tid];
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) slab[(long long)(ny * 64 + 4 * tid + e4) * p.Kcp + p.K] = v[e4];
        }
        __syncthreads();
    }

    // ---- output transform dW = G^T M G, round r: R[r][j] of all 4 blocks on wave j, blocks
    // exchanged (region (source wave, its round-slot) = 16 floats x 64 lanes, 6 regions in lx0 and
    // 6 in lg0), then wave b forms dW[r][s] = P0 + P1 of block b.  Signs: M = s_i s_j M'.
    const int cbo = wj >> 1, nbo = wj & 1;
    const int lr = lane & 31, lh = lane >> 5;
    const int n = ny * 64 + nbo * 32 + lr;
    auto region = [&](int src, int slot) -> float* {
        const int rg = src * 3 + slot;
        return reinterpret_cast<float*>(rg < 6 ? lx0 : lg0) + (rg % 6) * 16 * 64;
    };
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float Rm[2][2][16];                   // this wave's R[r][wj] of every block
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int idx = 0; idx < 16; ++idx) {
                    const float m0 = acc[0][cb][nb][idx], m1 = acc[1][cb][nb][idx];
                    const float m2 = acc[2][cb][nb][idx], m3 = -acc[3][cb][nb][idx];
                    const float v = r == 0 ? m0 + 0.5f * (m1 + m2) : r == 1 ? 0.5f * (m1 - m2) : 0.5f * (m1 + m2) + m3;
                    Rm[cb][nb][idx] = wj == 3 ? -v : v;
                }
        // send the 3 other blocks' values: block b goes to slot (b - wj - 1) & 3 ... (3 slots)
#pragma unroll
        for (int bo = 1; bo < 4; ++bo) {
            const int b = (wj + bo) & 3;
            float* dst = region(wj, bo - 1);
#pragma unroll
            for (int idx = 0; idx < 16; ++idx) {
                float v = 0.f;
#pragma unroll
                for (int bb = 0; bb < 4; ++bb)
                    if (bb == b) v = Rm[bb >> 1][bb & 1][idx];
                dst[idx * 64 + lane] = v;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // R[r][j] of block wj for j = 0..3 (own: Rm; from wave j: its slot (wj - j - 1) & 3)
        float Rj[4][16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j == wj) {
#pragma unroll
                for (int idx = 0; idx < 16; ++idx) {
                    float v = 0.f;
#pragma unroll
                    for (int bb = 0; bb < 4; ++bb)
                        if (bb == wj) v = Rm[bb >> 1][bb & 1][idx];
                    Rj[j][idx] = v;
                }
            } else {
                const float* src = region(j, ((wj - j) & 3) - 1);
#pragma unroll
                for (int idx = 0; idx < 16; ++idx) Rj[j][idx] = src[idx * 64 + lane];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                f32x4 v;
#pragma unroll
                for (int ee = 0; ee < 4; ++ee) {
                    const int idx = 4 * q + ee;
                    const float R0 = Rj[0][idx], R1 = Rj[1][idx], R2 = Rj[2][idx], R3 = Rj[3][idx];
                    // j = 0, 1: R0 G[0] + R1 G[1];  j = 2, 3: R2 G[2] + R3 G[3]
                    const float P0 = s == 0 ? R0 + 0.5f * R1 : 0.5f * R1;
                    const float P1 = s == 0 ? 0.5f * R2 : s == 1 ? -0.5f * R2 : 0.5f * R2 + R3;
                    v[ee] = P0 + P1;
                }
                const int k = (3 * r + s) * p.C + c_lo + cbo * 32 + 8 * q + 4 * lh;
                *reinterpret_cast<f32x4*>(slab + (long long)n * p.Kcp + k) = v;
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
}

// ------------------------------------------------------- single-channel stem weight gradient
// dW[n][tap] = sum_m dZ[m][n] x[m + tap] and db[n] = sum_m dZ[m][n] for the 1 -> N stem conv
// (inc.c0): the layer is the read of dZ (N channels per pixel).  Blocks sweep 16 x 64 pixel tiles
// (grid-stride) with the 1-channel halo staged in LDS; lanes in groups of N/4 per pixel, each lane
// 4 output channels x (9 taps + bias) accumulators over its pixels (dZ float4 loads: a
// wave-instruction reads 4 pixels x N channels contiguously); the block's groups are summed in
// fixed order through LDS into slab row [block][n][0..9] and the fixed-order split reduction
// finishes - deterministic like every other weight gradient.
constexpr int SWS_TH = 16, SWS_TW = 64;

// BF16ROWS (pu_wgrad_args.math == 2): dZ is a bf16 NHWC tensor, widened exactly on load (the bf16
// trunk's stem: no fp32 copy of dZ), otherwise the same fmaf chains
template <int N, bool BF16ROWS = false>
__global__ __launch_bounds__(256) void wgrad_stem_kernel(const WgradParams p) {
    constexpr int L = N / 4, PG = 256 / L;
    constexpr int HH = SWS_TH + 2, HW = SWS_TW + 2;
    constexpr int RED = PG * 10 * N;
    __shared__ __attribute__((aligned(16))) float smem[RED > HH * HW ? RED : HH * HW];
    const int tid = threadIdx.x;
    const int lane_c = tid % L, grp = tid / L;
    float acc[10][4];
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[k][e] = 0.f;
    const int ntiles = p.batch * p.tiles_h * p.tiles_w;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int txi = t % p.tiles_w;
        const int tyi = (t / p.tiles_w) % p.tiles_h;
        const int b = t / (p.tiles_w * p.tiles_h);
        const int y0 = tyi * SWS_TH - 1, x0 = txi * SWS_TW - 1;
        const long long img = (long long)b * p.Hi * p.Wi;
        __syncthreads();                       // the previous tile's readers are done
        for (int e = tid; e < HH * HW; e += 256) {
            const int hy = e / HW, hx = e - hy * HW;
            const int gy = y0 + hy, gx = x0 + hx;
            smem[e] = ((unsigned)gy < (unsigned)p.Hi && (unsigned)gx < (unsigned)p.Wi)
                          ? p.src0[img + (long long)gy * p.Wi + gx] : 0.f;
        }
        __syncthreads();
        // 4 pixels per pass, their dZ loads issued together (unconditional: a pixel past the image
        // edge loads pixel 0 and adds nothing), so the loop waits once per 4 loads
        static_assert((SWS_TH * SWS_TW) % (4 * PG) == 0, "stem wgrad pass");
        for (int q0 = grp; q0 < SWS_TH * SWS_TW; q0 += 4 * PG) {
            f32x4 dzs[4];
            bool ok[4];
            int hb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + u * PG;
                const int row = q / SWS_TW, col = q - row * SWS_TW;
                const int oy = tyi * SWS_TH + row, ox = txi * SWS_TW + col;
                ok[u] = oy < p.Ho && ox < p.Wo;
                hb[u] = row * HW + col;
                const long long m = ok[u] ? ((long long)b * p.Ho + oy) * p.Wo + ox : 0;
                if constexpr (BF16ROWS) {
                    typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
                    const bf16x4_t zb = *reinterpret_cast<const bf16x4_t*>(reinterpret_cast<const __bf16*>(p.P) + m * N + 4 * lane_c);
#pragma unroll
                    for (int e = 0; e < 4; ++e) dzs[u][e] = (float)zb[e];
                } else {
                    dzs[u] = *reinterpret_cast<const f32x4*>(p.P + m * N + 4 * lane_c);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (!ok[u]) continue;
                const f32x4 dz = dzs[u];
#pragma unroll
                for (int t9 = 0; t9 < 9; ++t9) {
                    const float a = smem[hb[u] + (t9 / 3) * HW + t9 % 3];
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[t9][e] = fmaf(a, dz[e], acc[t9][e]);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[9][e] += dz[e];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) smem[(grp * 10 + k) * N + 4 * lane_c + e] = acc[k][e];
    __syncthreads();
    float* slab = p.slab + (long long)blockIdx.x * p.Nr * p.Kcp;
    for (int idx = tid; idx < 10 * N; idx += 256) {
        const int k = idx / N, n = idx - k * N;
        float v = 0.f;
        for (int g = 0; g < PG; ++g) v += smem[(g * 10 + k) * N + n];
        slab[(long long)n * p.Kcp + k] = v;   // k = tap (C = 1); k = 9 = K: the bias column
    }
}

// ------------------------------------------------------- pointwise (1x1) small weight gradient
// dW[n][c] = sum_m dZ[m][n] X[m][c] and db[n] = sum_m dZ[m][n] for a 1x1 / s1 / p0 conv with a
// handful of channels (config C4's CoordConv 1x1: 4 -> 8 channels at 256^2, 2.1 M pixels).  As a
// GEMM it is K = 4: the tiled kernel spent 85 latency-bound 16-row stages per block on it (155 us
// for 100 MB); here a thread streams whole pixels (C + N floats, consecutive pixels on consecutive
// lanes) and keeps all N x (C + 1) sums in registers, fmaf chains in pixel order.  The block's 256
// chains reduce in a fixed butterfly (xor 32 .. 1) then wave order, one slab row per block; the
// fixed-order split reduction finishes it - deterministic.
template <int C, int N>
__global__ __launch_bounds__(256) void wgrad_pw_kernel(const WgradParams p) {
    constexpr int V = N * (C + 1);                // C weights + the bias per output channel
    __shared__ float part[4][V];
    const int tid = threadIdx.x;
    float acc[N][C + 1];
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int c = 0; c <= C; ++c) acc[n][c] = 0.f;
    const long long m0 = (long long)blockIdx.x * p.mps;
    const long long m1 = min((long long)p.M, m0 + p.mps);
    for (long long m = m0 + tid; m < m1; m += 256) {
        float x[C], g[N];
        if constexpr (C % 4 == 0) {
#pragma unroll
            for (int q = 0; q < C / 4; ++q) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(p.src0 + m * C + 4 * q);
#pragma unroll
                for (int e = 0; e < 4; ++e) x[4 * q + e] = v[e];
            }
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = p.src0[m * C + c];
        }
#pragma unroll
        for (int q = 0; q < N / 4; ++q) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(p.P + m * N + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) g[4 * q + e] = v[e];
        }
#pragma unroll
        for (int n = 0; n < N; ++n) {
#pragma unroll
            for (int c = 0; c < C; ++c) acc[n][c] = fmaf(g[n], x[c], acc[n][c]);
            acc[n][C] += g[n];
        }
    }
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int c = 0; c <= C; ++c) {
            float v = acc[n][c];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) part[wave][n * (C + 1) + c] = v;
        }
    __syncthreads();
    float* slab = p.slab + (long long)blockIdx.x * p.Nr * p.Kcp;
    for (int i = tid; i < V; i += 256) {
        const float v = ((part[0][i] + part[1][i]) + part[2][i]) + part[3][i];
        const int n = i / (C + 1), c = i - n * (C + 1);
        if (c < C) slab[(long long)n * p.Kcp + c] = v;
        else if (p.bias_mode == 1) slab[(long long)n * p.Kcp + p.K] = v;
    }
}

// ------------------------------------------------------------- small-channel weight gradient
// 3x3/s1/p1 with C <= 16 input and N <= 16 output channels (configs C4/C5's 8/16-channel levels):
// a GEMM with N, K this small wastes most of an MFMA tile, so each block sweeps 16 x 32 pixel
// tiles (grid-stride), stages the input halo and the gradient tile in LDS, and accumulates
// dW[n][tap][c] on the VALU: thread items = (tap, 4 output x 4 input channels) plus bias items
// (4 output channels), replicated over pixel groups when the items do not fill the block.  The
// block's partial goes to slab row [block][n][tap*C + c] (bias at column K) and the fixed-order
// fp64 split reduction below finishes it - deterministic like the GEMM path.
constexpr int SW_TH = 16, SW_TW = 32;
#ifndef PU_SW_ROW
#define PU_SW_ROW 1     // 1: an item is a row of 3 taps over 4-pixel quads; 0: one tap per pixel
#endif

// 4x4 outer-product accumulate of 4 output channels g (x) 4 input channels x: channel pairs on
// v_pk_fma_f32 (one rounding per element, as fmaf)
__device__ __forceinline__ void sw_fma44(wg_f32x2 (&a)[4][2], const f32x4& g, const f32x4& x) {
    const wg_f32x2 xa = {x[0], x[1]}, xb = {x[2], x[3]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const wg_f32x2 gg = {g[i], g[i]};
        a[i][0] = __builtin_elementwise_fma(gg, xa, a[i][0]);
        a[i][1] = __builtin_elementwise_fma(gg, xb, a[i][1]);
    }
}

template <int C, int N>
__global__ __launch_bounds__(256) void wgrad_small_kernel(const WgradParams p) {
    constexpr int HH = SW_TH + 2, HWD = SW_TW + 2;
    constexpr int CP = (C + 3) & ~3, C4 = CP / 4, N4 = N / 4;
    // weight items: (tap row r, 4 output x 4 input channels) with the 3 taps of the row, or
    // (tap, 4 x 4) - plus bias items (4 output channels)
    constexpr int RT = PU_SW_ROW ? 3 : 1;                 // taps per item
    constexpr int WITEMS = (9 / RT) * N4 * C4;
    constexpr int ITEMS = WITEMS + N4;
    // LDS bank conflicts (64 banks: a ds_read_b128 serves 16 lanes per cycle): a group's items
    // padded to a multiple of 16 lanes keeps each 16-lane phase inside one pixel group, and a
    // halo row pitch of HWD + 1 pixels puts the 3 tap rows x input-channel quads on distinct banks
    // (C = 8: chunk offsets {0,1,6,7,12,13}; C = 16: {0..3, 12..15, 8..11})
    constexpr int ITEMS_P = ITEMS >= 12 ? (ITEMS + 15) / 16 * 16 : ITEMS;
    constexpr int HWP = HWD + 1;
    constexpr int GROUPS = 256 / ITEMS_P;
    static_assert(GROUPS >= 1, "items");
    constexpr int ACC = RT * 16;
    constexpr int HALO = HH * HWP * CP, GT = SW_TH * SW_TW * N;
    constexpr int SMEM = (HALO + GT) > (GROUPS * ITEMS * ACC) ? (HALO + GT) : (GROUPS * ITEMS * ACC);
    __shared__ __attribute__((aligned(16))) float smem[SMEM];
    float* halo = smem;
    float* gt = smem + HALO;

    const int tid = threadIdx.x;
    const int item = tid % ITEMS_P, grp = tid / ITEMS_P;
    const bool active = grp < GROUPS && item < ITEMS;
    const bool wi = item < WITEMS;
    int tq = 0, co4 = 0, ci4 = 0;                          // tq: tap row (RT = 3) or tap
    if (wi) {
        tq = item / (N4 * C4);
        const int rem = item - tq * (N4 * C4);
        co4 = rem / C4;
        ci4 = rem - co4 * C4;
    } else {
        co4 = item - WITEMS;
    }
    const int tr = RT == 3 ? tq : tq / 3, ts = RT == 3 ? 0 : tq - tr * 3;
    wg_f32x2 acc[RT][4][2];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][i][0] = acc[t][i][1] = wg_f32x2{0.f, 0.f};

    const int ntiles = p.batch * p.tiles_h * p.tiles_w;
    // the tile's halo and gradient rows are loaded into registers one tile ahead (all loads of a
    // tile in flight at once), stored to LDS between two barriers, and the next tile's loads then
    // fly under this tile's accumulation
    constexpr int NH = HH * HWD * C4, NG = SW_TH * SW_TW * N4;
    constexpr int PH = (NH + 255) / 256, PG2 = (NG + 255) / 256;
    f32x4 rh[PH], rg[PG2];
    auto load_tile = [&](int t) {
        const int txi = t % p.tiles_w;
        const int tyi = (t / p.tiles_w) % p.tiles_h;
        const int b = t / (p.tiles_w * p.tiles_h);
        const int y0 = tyi * SW_TH, x0 = txi * SW_TW;
        const long long img = (long long)b * p.Hi * p.Wi;
#pragma unroll
        for (int it = 0; it < PH; ++it) {
            const int e = it * 256 + tid;
            const int q = e % C4, pix = e / C4;
            const int hx = pix % HWD, hy = pix / HWD;
            const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (e < NH && (unsigned)gy < (unsigned)p.Hi && (unsigned)gx < (unsigned)p.Wi) {
                const long long px = img + (long long)gy * p.Wi + gx;
                if (C % 4 == 0 && p.c0 % 4 == 0) {
                    const int c = 4 * q;
                    v = c < p.c0 ? *reinterpret_cast<const f32x4*>(p.src0 + px * p.c0 + c)
                                 : *reinterpret_cast<const f32x4*>(p.src1 + px * p.c1 + (c - p.c0));
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int c = 4 * q + k;
                        if (c < C) v[k] = c < p.c0 ? p.src0[px * p.c0 + c] : p.src1[px * p.c1 + (c - p.c0)];
                    }
                }
            }
            rh[it] = v;
        }
#pragma unroll
        for (int it = 0; it < PG2; ++it) {
            const int e = it * 256 + tid;
            const int q = e % N4, pix = e / N4;
            const int oy = y0 + pix / SW_TW, ox = x0 + pix % SW_TW;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (e < NG && oy < p.Ho && ox < p.Wo)
                v = *reinterpret_cast<const f32x4*>(p.P + ((long long)(b * p.Ho + oy) * p.Wo + ox) * N + 4 * q);
            rg[it] = v;
        }
    };
    if ((int)blockIdx.x < ntiles) load_tile(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        __syncthreads();                       // previous tile's readers are done
#pragma unroll
        for (int it = 0; it < PH; ++it) {
            const int e = it * 256 + tid;
            if (e < NH) {
                const int pix = e / C4, hy = pix / HWD, hx = pix - hy * HWD;
                *reinterpret_cast<f32x4*>(halo + (hy * HWP + hx) * CP + 4 * (e % C4)) = rh[it];
            }
        }
#pragma unroll
        for (int it = 0; it < PG2; ++it) {
            const int e = it * 256 + tid;
            if (e < NG) *reinterpret_cast<f32x4*>(gt + (e / N4) * N + 4 * (e % N4)) = rg[it];
        }
        if (t + (int)gridDim.x < ntiles) load_tile(t + gridDim.x);
        __syncthreads();
        if (active) {
            if (RT == 3) {
                // 4 consecutive output pixels x the row's 3 taps: 4 gradient + 6 halo reads per
                // 192 fmas (the per-tap form: 2 reads per 16)
                constexpr int QW = SW_TW / 4;
                for (int pq = grp; pq < SW_TH * QW; pq += GROUPS) {
                    const int row = pq / QW, col0 = (pq - row * QW) * 4;
                    f32x4 g[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        g[u] = *reinterpret_cast<const f32x4*>(gt + (row * SW_TW + col0 + u) * N + 4 * co4);
                    if (wi) {
                        f32x4 x[6];
#pragma unroll
                        for (int v = 0; v < 6; ++v)
                            x[v] = *reinterpret_cast<const f32x4*>(halo + ((row + tr) * HWP + col0 + v) * CP + 4 * ci4);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int s3 = 0; s3 < RT; ++s3) sw_fma44(acc[s3], g[u], x[u + s3]);
                    } else {
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            acc[0][0][0] += wg_f32x2{g[u][0], g[u][1]};
                            acc[0][0][1] += wg_f32x2{g[u][2], g[u][3]};
                        }
                    }
                }
            } else if (wi) {
                for (int pp = grp; pp < SW_TH * SW_TW; pp += GROUPS) {
                    const int row = pp / SW_TW, col = pp - row * SW_TW;
                    const f32x4 g4 = *reinterpret_cast<const f32x4*>(gt + pp * N + 4 * co4);
                    const f32x4 x4 = *reinterpret_cast<const f32x4*>(halo + ((row + tr) * HWP + col + ts) * CP + 4 * ci4);
                    sw_fma44(acc[0], g4, x4);
                }
            } else {
                for (int pp = grp; pp < SW_TH * SW_TW; pp += GROUPS) {
                    const f32x4 g4 = *reinterpret_cast<const f32x4*>(gt + pp * N + 4 * co4);
                    acc[0][0][0] += wg_f32x2{g4[0], g4[1]};
                    acc[0][0][1] += wg_f32x2{g4[2], g4[3]};
                }
            }
        }
    }
    // fixed-order reduction over the pixel groups, then this block's slab rows
    __syncthreads();
    if (active) {
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    smem[(grp * ITEMS + item) * ACC + t * 16 + i * 4 + 2 * h] = acc[t][i][h][0];
                    smem[(grp * ITEMS + item) * ACC + t * 16 + i * 4 + 2 * h + 1] = acc[t][i][h][1];
                }
    }
    __syncthreads();
    if (tid < ITEMS) {
        float* slab = p.slab + (long long)blockIdx.x * p.Nr * p.Kcp;
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            float v[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) v[e] = 0.f;
            for (int g = 0; g < GROUPS; ++g)
#pragma unroll
                for (int e = 0; e < 16; ++e) v[e] += smem[(g * ITEMS + tid) * ACC + t * 16 + e];
            if (tid < WITEMS) {
                const int tap = RT == 3 ? 3 * tr + t : tq;
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int c = 4 * ci4 + j;
                        if (c < C) slab[(long long)(4 * co4 + i) * p.Kcp + tap * C + c] = v[i * 4 + j];
                    }
            } else if (t == 0 && p.bias_mode == 1) {   // column K exists only with a bias (Kc = K + 1)
#pragma unroll
                for (int i = 0; i < 4; ++i) slab[(long long)(4 * co4 + i) * p.Kcp + p.K] = v[i];
            }
        }
    }
}

// Split-K reduction, pass 1: part[g][idx] = sum over splits z = g, g+G, ... of slab[z][idx]
// (fp64, 4 independent accumulators so each thread keeps several loads in flight).
__global__ void wgrad_sum_splits_kernel(const float* __restrict__ slab, int splits, long long total, int G,
                                        double* __restrict__ part) {
    const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int g = blockIdx.y;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int z = g;
    for (; z + 3 * G < splits; z += 4 * G) {
        s0 += slab[(long long)z * total + idx];
        s1 += slab[(long long)(z + G) * total + idx];
        s2 += slab[(long long)(z + 2 * G) * total + idx];
        s3 += slab[(long long)(z + 3 * G) * total + idx];
    }
    for (; z < splits; z += G) s0 += slab[(long long)z * total + idx];
    part[(long long)g * total + idx] = (s0 + s1) + (s2 + s3);
}

// pass 1 on float4 quads (total % 4 == 0): the same 4 chains per entry in the same order (so
// bit-identical to wgrad_sum_splits_kernel), with two chain rounds' 8 x 16-B loads issued before
// their adds - the scalar form kept 4 x 4 B per thread in flight and ran at ~1.3 TB/s.
__global__ __launch_bounds__(256) void wgrad_sum_splits4_kernel(const float* __restrict__ slab, int splits,
                                                                long long total, int G, double* __restrict__ part) {
    const long long idx = 4 * (blockIdx.x * (long long)blockDim.x + threadIdx.x);
    if (idx >= total) return;
    const int g = blockIdx.y;
    double s[4][4] = {};
    const float* sp = slab + idx;
    int z = g;
    for (; z + 7 * G < splits; z += 8 * G) {
        f32x4 v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = *reinterpret_cast<const f32x4*>(sp + (long long)(z + c * G) * total);
#pragma unroll
        for (int c = 0; c < 8; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) s[c & 3][e] += (double)v[c][e];
    }
    if (z + 3 * G < splits) {
        f32x4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const f32x4*>(sp + (long long)(z + c * G) * total);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) s[c][e] += (double)v[c][e];
        z += 4 * G;
    }
    for (; z < splits; z += G) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(sp + (long long)z * total);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[0][e] += (double)v[e];
    }
    double* o = part + (long long)g * total + idx;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (s[0][e] + s[1][e]) + (s[2][e] + s[3][e]);
}

// pass 2: sum the G groups (fixed order, fp64) and scatter to PyTorch's [n][c][kh][kw] + bias.
// Threads [0, total) handle slab entries; threads [total, total + C) the ConvT bias (mode 2).
// T = double: the G pass-1 partials;  T = float: the slab itself (G = splits, single pass).
template <typename T>
__global__ void wgrad_finish_kernel(const T* __restrict__ part, int G, int Nr, int Kc, int N, int K, int C,  // Kc = slab row stride
                                    int kh, int kw, int bias_mode, float* __restrict__ dw, float* __restrict__ db,
                                    int accumulate) {
    const long long total = (long long)Nr * Kc;
    const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (idx < total) {
        const int n = int(idx / Kc);
        const int k = int(idx - (long long)n * Kc);
        if (n >= N) return;
        // 4 independent fp64 chains (fixed interleave, deterministic): keeps 4 loads in flight
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int g = 0;
        for (; g + 3 < G; g += 4) {
            s0 += (double)part[(long long)g * total + idx];
            s1 += (double)part[(long long)(g + 1) * total + idx];
            s2 += (double)part[(long long)(g + 2) * total + idx];
            s3 += (double)part[(long long)(g + 3) * total + idx];
        }
        for (; g < G; ++g) s0 += (double)part[(long long)g * total + idx];
        const float v = (float)((s0 + s1) + (s2 + s3));
        if (k < K) {
            const int tap = k / C, c = k - tap * C;
            const int r = tap / kw, ss = tap - r * kw;
            float* o = dw + (((long long)n * C + c) * kh + r) * kw + ss;
            *o = accumulate ? *o + v : v;
        } else if (bias_mode == 1 && k == K) {
            db[n] = accumulate ? db[n] + v : v;
        }
    } else if (bias_mode == 2 && idx < total + C) {
        const int c = int(idx - total);
        double s = 0.0;
        for (int t = 0; t < kh * kw; ++t)
            for (int g = 0; g < G; ++g) s += (double)part[(long long)g * total + (long long)N * Kc + t * C + c];
        const float v = (float)s;
        db[c] = accumulate ? db[c] + v : v;
    }
}

// wgrad_finish_kernel on quads of 4 consecutive entries of one slab row (Kc % 4 == 0): the same
// 4 fp64 chains per entry in the same order - bit-identical to wgrad_finish_kernel for the WEIGHT
// entries (and the bias of modes 0/1), 8 partial quads in flight per thread instead of 4 scalars.
// The ConvT bias (mode 2: entries t*C + c of row N over every tap t and partial g) is NOT summed in
// the scalar kernel's order: it runs as 4 interleaved fp64 chains over the flattened (t, g)
// sequence with 8 loads in flight (the scalar form's one dependent chain of taps x G loads was a
// latency tail, 17.7 us for a 64-channel ConvT in C2), so it can differ from the scalar kernel's
// result in the last fp32 ulp.  It is deterministic run to run (fixed order; pinned by
// tests/test_kernels_gpu.py::test_convT_bias_grad_run_to_run_bitwise).
template <typename T>
__global__ __launch_bounds__(256) void wgrad_finish4_kernel(const T* __restrict__ part, int G, int Nr, int Kc, int N,
                                                            int K, int C, int kh, int kw, int bias_mode,
                                                            float* __restrict__ dw, float* __restrict__ db,
                                                            int accumulate) {
    typedef T t4 __attribute__((ext_vector_type(4)));
    const long long total = (long long)Nr * Kc;
    const long long nq = total >> 2;
    const long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (q < nq) {
        const long long idx = 4 * q;
        const int n = int(idx / Kc);
        const int k0 = int(idx - (long long)n * Kc);
        if (n >= N) return;
        const T* sp = part + idx;
        double s[4][4] = {};
        int g = 0;
        for (; g + 7 < G; g += 8) {
            t4 v[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = *reinterpret_cast<const t4*>(sp + (long long)(g + c) * total);
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e) s[c & 3][e] += (double)v[c][e];
        }
        if (g + 3 < G) {
            t4 v[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const t4*>(sp + (long long)(g + c) * total);
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e) s[c][e] += (double)v[c][e];
            g += 4;
        }
        for (; g < G; ++g) {
            const t4 v = *reinterpret_cast<const t4*>(sp + (long long)g * total);
#pragma unroll
            for (int e = 0; e < 4; ++e) s[0][e] += (double)v[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = k0 + e;
            const float v = (float)((s[0][e] + s[1][e]) + (s[2][e] + s[3][e]));
            if (k < K) {
                const int tap = k / C, c = k - tap * C;
                const int r = tap / kw, ss = tap - r * kw;
                float* o = dw + (((long long)n * C + c) * kh + r) * kw + ss;
                *o = accumulate ? *o + v : v;
            } else if (bias_mode == 1 && k == K) {
                db[n] = accumulate ? db[n] + v : v;
            }
        }
    } else if (bias_mode == 2 && q < nq + C) {
        const int c = int(q - nq);
        const int J = kh * kw * G;                       // j = t * G + g
        const T* bp = part + (long long)N * Kc + c;
        auto at = [&](int j) {
            const int t = j / G, gg = j - t * G;
            return (double)bp[(long long)gg * total + t * C];
        };
        double s[4] = {0.0, 0.0, 0.0, 0.0};
        int j = 0;
        for (; j + 7 < J; j += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = at(j + u);
#pragma unroll
            for (int u = 0; u < 8; ++u) s[u & 3] += v[u];
        }
        for (; j < J; ++j) s[0] += at(j);
        const float v = (float)((s[0] + s[1]) + (s[2] + s[3]));
        db[c] = accumulate ? db[c] + v : v;
    }
}

// pass 2 with coalesced stores: block (chunk of 256 channels, row n) sums slab[.][n][tap*C + c]
// for its channels x taps (thread = (tap, 4 channels): 1-KB float4 reads per wave and split),
// transposes through LDS and stores the contiguous [c][kh][kw] run of dweight[n] as float4 (the
// scatter above writes 4 B at a 4*taps-byte stride).  Same fixed-order fp64 chains as
// wgrad_finish_kernel, so bit-identical.  C % 4 == 0, 16-B aligned rows; bias_mode 0/1 (the ConvT
// bias, mode 2, stays on wgrad_finish_kernel).
template <typename T>
__global__ __launch_bounds__(576) void wgrad_finish_t_kernel(const T* __restrict__ part, int G, int Nr, int Kc, int K,
                                                              int C, int taps, int bias_mode, float* __restrict__ dw,
                                                              float* __restrict__ db, int accumulate) {
    __shared__ float tr[256 * 9];
    typedef T t4 __attribute__((ext_vector_type(4)));
    const long long total = (long long)Nr * Kc;
    const int n = blockIdx.y;
    const int c0 = blockIdx.x * 256;
    const int tap = threadIdx.x >> 6, cq = (threadIdx.x & 63) * 4;
    const int cn = min(256, C - c0);
    if (cq < cn) {
        const long long idx = (long long)n * Kc + tap * C + c0 + cq;
        double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};
        double s2[4] = {0.0, 0.0, 0.0, 0.0}, s3[4] = {0.0, 0.0, 0.0, 0.0};
        int g = 0;
        for (; g + 3 < G; g += 4) {
            const t4 a = *reinterpret_cast<const t4*>(part + (long long)g * total + idx);
            const t4 b = *reinterpret_cast<const t4*>(part + (long long)(g + 1) * total + idx);
            const t4 c = *reinterpret_cast<const t4*>(part + (long long)(g + 2) * total + idx);
            const t4 d = *reinterpret_cast<const t4*>(part + (long long)(g + 3) * total + idx);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                s0[e] += (double)a[e];
                s1[e] += (double)b[e];
                s2[e] += (double)c[e];
                s3[e] += (double)d[e];
            }
        }
        for (; g < G; ++g) {
            const t4 a = *reinterpret_cast<const t4*>(part + (long long)g * total + idx);
#pragma unroll
            for (int e = 0; e < 4; ++e) s0[e] += (double)a[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) tr[(cq + e) * taps + tap] = (float)((s0[e] + s1[e]) + (s2[e] + s3[e]));
    }
    if (bias_mode == 1 && blockIdx.x == 0 && threadIdx.x == 0) {
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        const long long idx = (long long)n * Kc + K;
        int g = 0;
        for (; g + 3 < G; g += 4) {
            s0 += (double)part[(long long)g * total + idx];
            s1 += (double)part[(long long)(g + 1) * total + idx];
            s2 += (double)part[(long long)(g + 2) * total + idx];
            s3 += (double)part[(long long)(g + 3) * total + idx];
        }
        for (; g < G; ++g) s0 += (double)part[(long long)g * total + idx];
        const float v = (float)((s0 + s1) + (s2 + s3));
        db[n] = accumulate ? db[n] + v : v;
    }
    __syncthreads();
    // dweight[n][c0 .. c0+cn)[taps] is cn * taps contiguous floats; 16-B aligned when C*taps and
    // c0*taps are multiples of 4 (C % 4 == 0)
    float* o = dw + ((long long)n * C + c0) * taps;
    const int run = cn * taps;
    for (int i = threadIdx.x * 4; i < run; i += blockDim.x * 4) {
        f32x4 v = {tr[i], tr[i + 1], tr[i + 2], tr[i + 3]};
        if (accumulate) v += *reinterpret_cast<const f32x4*>(o + i);
        *reinterpret_cast<f32x4*>(o + i) = v;
    }
}

struct WgradPlan {
    int BN, BK, splits, mps, Nr, Kc, Kcp, M, K, C, G, gx, gy;
    bool qvec, dma, small, halo, stem;
    bool wino = false;                        // Winograd-domain kernel (wgrad_wino_x6_kernel)
    bool pw = false;                          // pointwise small-channel kernel (wgrad_pw_kernel)
    int tiles = 0, tps = 0;
    int nt = 1;                               // halo kernel: 64-channel output tiles per block
    int tiles_w, tiles_h;
    size_t slab_bytes() const { return (size_t)splits * Nr * Kcp * sizeof(float); }
    size_t part_bytes() const { return G > 1 ? (size_t)G * Nr * Kcp * sizeof(double) : 0; }
    size_t ws_bytes() const { return ((slab_bytes() + 255) / 256) * 256 + part_bytes(); }
};

static bool stem_wgrad_ok(const pu_wgrad_args* a) {
    return a->c0 == 1 && a->c1 == 0 && (a->n == 8 || a->n == 16 || a->n == 32 || a->n == 64) && a->kh == 3 && a->kw == 3 && a->stride == 1 &&
           a->pad == 1 && a->in_h == a->out_h && a->in_w == a->out_w && a->bias_mode == 1 &&
           ((uintptr_t)a->rows & 15) == 0;
}

// 1x1 / s1 / p0 same-size conv, one source, (C, N) an instantiated wgrad_pw_kernel pair
static bool pw_wgrad_ok(const pu_wgrad_args* a) {
    const int C = a->c0, N = a->n;
    return a->c1 == 0 && a->kh == 1 && a->kw == 1 && a->stride == 1 && a->pad == 0 && a->in_h == a->out_h &&
           a->in_w == a->out_w && a->bias_mode != 2 && (C == 3 || C == 4) && (N == 4 || N == 8 || N == 16) &&
           (((uintptr_t)a->rows & 15) == 0) && (C % 4 || ((uintptr_t)a->src0 & 15) == 0);
}

static bool small_wgrad_ok(const pu_wgrad_args* a) {
    const int C = a->c0 + a->c1;
    return (C == 1 || C == 4 || C == 8 || C == 12 || C == 16) &&
           (a->n == 4 || a->n == 8 || a->n == 16) && a->kh == 3 && a->kw == 3 && a->stride == 1 && a->pad == 1 &&
           a->in_h == a->out_h && a->in_w == a->out_w && a->bias_mode != 2 &&
           (C == 1 || (a->c0 % 4 == 0 && a->c1 % 4 == 0));
}

static void plan_groups(WgradPlan* pl);

// the Winograd-domain kernel: 3x3 / s1 / p1 on an even same-size grid, 64-channel input blocks
// from one source each, 64-channel output blocks, the 6-product arithmetic, byte offsets of the
// (shifted) sources and of dZ under 2^31; PU_WINO_WGRAD=0 keeps the direct kernels (A/B runs)
// the Winograd weight gradient on one wave per SIMD (wgrad_wino4_x6_kernel, bit-identical):
// PU_WW4=1 (A/B runs)
static bool ww4_on() {
    static const bool on = [] {
        const char* e = getenv("PU_WW4");
        return e && e[0] == '1';
    }();
    return on;
}

static bool wino_wgrad_ok(const pu_wgrad_args* a, const WgradPlan* pl) {
    static const bool on = [] {
        const char* e = getenv("PU_WINO_WGRAD");
        return !(e && e[0] == '0');
    }();
    if (!on || a->math != 1 || !pl->qvec) return false;
    if (a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1) return false;
    if (a->in_h != a->out_h || a->in_w != a->out_w || (a->out_h & 1) || (a->out_w & 1)) return false;
    if (a->c0 % 64 || a->c1 % 64 || a->n % 64 || a->bias_mode == 2) return false;
    const long long px = (long long)a->batch * a->in_h * a->in_w + a->in_w + 1;
    if (px * (a->c0 > a->c1 ? a->c0 : a->c1) * 4 >= (1LL << 31)) return false;
    if ((long long)a->batch * a->out_h * a->out_w * a->n * 4 >= (1LL << 31)) return false;
    return (((uintptr_t)a->rows | (uintptr_t)a->src0 | (uintptr_t)a->src1) & 7) == 0;
}

// Measured alternatives: capping the GEMM-path split count at 2 / 4 (round 3: C2 4060 -> 2262 /
// 2968 img/s - the deep layers' slab traffic is cheaper than idle CUs); round 1: 64 x 576 6-wave tiles for the 64-channel layers (-6 %), a
// 3-wave 64 x 192 tile (-8 %), a split-once-planes kernel that still staged fp32 through LDS
// (-10...-25 %); the halo kernel below replaced all of them on 3x3/s1 layers.
static int plan_wgrad(const pu_wgrad_args* a, WgradPlan* pl) {
    PU_REQUIRE(a && a->batch > 0 && a->out_h > 0 && a->out_w > 0 && a->in_h > 0 && a->in_w > 0, "pu_wgrad: bad grid");
    PU_REQUIRE(a->kh > 0 && a->kw > 0 && a->stride > 0 && a->pad >= 0, "pu_wgrad: bad taps");
    PU_REQUIRE(a->rows && a->n > 0 && a->src0 && a->c0 > 0 && (a->c1 == 0 || a->src1), "pu_wgrad: operands");
    PU_REQUIRE(a->n % 4 == 0, "pu_wgrad: n (%d) must be a multiple of 4", a->n);
    PU_REQUIRE(a->bias_mode >= 0 && a->bias_mode <= 2, "pu_wgrad: bias_mode");
    PU_REQUIRE(a->bias_mode == 0 || a->dbias, "pu_wgrad: dbias missing");
    PU_REQUIRE(a->dweight, "pu_wgrad: dweight missing");
    PU_REQUIRE(a->math >= 0 && a->math <= 2, "pu_wgrad: math %d", a->math);
    PU_REQUIRE(a->math != 2 || stem_wgrad_ok(a), "pu_wgrad: math 2 (bf16 rows) is the single-channel stem only");
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    PU_REQUIRE(M < (1LL << 31), "pu_wgrad: too many pixels");
    pl->M = (int)M;
    pl->C = a->c0 + a->c1;
    pl->K = a->kh * a->kw * pl->C;
    pl->Nr = a->n + (a->bias_mode == 2 ? 1 : 0);
    pl->Kc = pl->K + (a->bias_mode == 1 ? 1 : 0);
    pl->Kcp = (pl->Kc + 3) / 4 * 4;
    pl->qvec = (a->c0 % 4 == 0) && (a->c1 % 4 == 0);
    pl->small = small_wgrad_ok(a);
    pl->stem = stem_wgrad_ok(a);
    pl->pw = pw_wgrad_ok(a);
    pl->halo = false;
    if (pl->qvec) {
        PU_REQUIRE(((uintptr_t)a->src0 & 15) == 0 && ((uintptr_t)a->src1 & 15) == 0, "pu_wgrad: sources must be 16-byte aligned");
    }
    PU_REQUIRE(((uintptr_t)a->rows & 15) == 0, "pu_wgrad: rows must be 16-byte aligned");
    pl->dma = pl->qvec;
    if (pl->pw) {                      // pointwise: contiguous pixel ranges, one slab row block each
        pl->splits = (int)(M / 256 < 1024 ? (M + 255) / 256 : 1024);
        pl->mps = (int)ceil_div(M, (long long)pl->splits);
        pl->splits = (int)ceil_div(M, (long long)pl->mps);
        pl->BN = a->n; pl->BK = pl->K; pl->gx = pl->gy = 1; pl->dma = false;
        pl->tiles_w = pl->tiles_h = 0;
        plan_groups(pl);
        return PU_OK;
    }
    if (pl->small || pl->stem) {       // direct kernels: one slab row block per block
        pl->tiles_w = ceil_div(a->out_w, pl->stem ? SWS_TW : SW_TW);
        pl->tiles_h = ceil_div(a->out_h, pl->stem ? SWS_TH : SW_TH);
        const long long ntiles = (long long)a->batch * pl->tiles_w * pl->tiles_h;
        pl->splits = (int)(ntiles < 1024 ? ntiles : 1024);
        pl->BN = a->n; pl->BK = pl->K; pl->gx = pl->gy = 1; pl->mps = 0; pl->dma = false;
        const long long total = (long long)pl->Nr * pl->Kcp;
        int G = (int)ceil_div(262144LL, total);
        const int by_len = ceil_div(pl->splits, 8);
        if (G > by_len) G = by_len;
        if (G > 16) G = 16;
        pl->G = G < 1 ? 1 : G;
        return PU_OK;
    }
    // the direct-to-LDS kernel tiles only the N x K GEMM (bias via LDS column sums); the
    // register-staged kernel carries the bias as an extra ones column / row
    const int ext_n = pl->dma ? a->n : pl->Nr;
    const int ext_k = pl->dma ? pl->K : pl->Kc;
    int occ;  // resident blocks per CU (LDS / VGPR limited, from the resource-usage report)
    if (ext_k <= 64) { pl->BN = 64; pl->BK = 64; occ = pl->dma ? 6 : 7; }
    else if (ext_n <= 64 && !pl->dma) { pl->BN = 64; pl->BK = 256; occ = 3; }
    else if (ext_n <= 32 && a->math == 1) { pl->BN = 32; pl->BK = 128; occ = 4; }   // 32-channel layers (C4/C5)
    else if (ext_n <= 64) {
        // BK 128 (4 resident blocks) unless 192 (3 resident) pads k less - e.g. K = 9 taps x 64
        const bool b192 = ceil_div(ext_k, 192) * 192 < ceil_div(ext_k, 128) * 128;
        pl->BN = 64; pl->BK = b192 ? 192 : 128; occ = b192 ? 3 : 4;
    }
    else { pl->BN = 128; pl->BK = 128; occ = pl->dma ? 3 : 4; }
    // 6-product path: a 128 x 256 tile (2x2 waves of 64 x 128) splits 6 operand fragments per 48
    // MFMAs instead of 4 per 24, when K pads no worse than with 128
    if (a->math == 1 && pl->dma && pl->BN == 128 &&
        ceil_div(ext_k, 256) * 256 <= ceil_div(ext_k, 128) * 128) {
        pl->BK = 256;
        occ = 2;
    }
    pl->halo = false;
    if (wino_wgrad_ok(a, pl)) {
        // one 512-thread block per CU: (C / 64) x (N / 64) channel blocks x tile splits of whole
        // 16-tile stages
        pl->wino = true;
        pl->BN = 64;
        pl->BK = 9 * 64;
        pl->gx = pl->C / 64;
        pl->gy = a->n / 64;
        pl->tiles = a->batch * (a->out_h / 2) * (a->out_w / 2);
        const int stages = ceil_div(pl->tiles, 16);
        int splits = 256 / (pl->gx * pl->gy);
        if (splits > stages) splits = stages;
        if (splits < 1) splits = 1;
        pl->tps = ceil_div(stages, splits) * 16;
        pl->splits = ceil_div(pl->tiles, pl->tps);
        pl->mps = pl->tps * 4;
        plan_groups(pl);
        return PU_OK;
    }
    if (a->math == 1 && pl->dma && a->kh == 3 && a->kw == 3 && a->stride == 1 && a->pad == 1 &&
        a->in_h == a->out_h && a->in_w == a->out_w && a->out_w % 16 == 0 && a->c0 % 64 == 0 && a->c1 % 64 == 0 &&
        a->n % 64 == 0 && a->bias_mode != 2 && (long long)a->batch * a->in_h * a->in_w * (pl->C) < (1LL << 31)) {
        pl->halo = true;
        pl->nt = a->n % 128 == 0 ? 2 : 1;    // 128 output channels per block when they divide
        pl->BN = 64 * pl->nt;
        pl->BK = 9 * 64;
        const int tiles = (pl->C / 64) * (a->n / pl->BN);
        int splits = (pl->nt == 2 ? 256 : 512) / tiles;   // one 8-wave / two 4-wave blocks per CU
        const int stages = (int)(M / 16);
        if (splits > stages) splits = stages;
        if (splits < 1) splits = 1;
        pl->mps = ceil_div(stages, splits) * 16;
        pl->splits = ceil_div((int)M, pl->mps);
        pl->gx = pl->C / 64;
        pl->gy = a->n / pl->BN;
        const long long total = (long long)pl->Nr * pl->Kcp;
        int G = (int)ceil_div(262144LL, total);
        const int by_len = ceil_div(pl->splits, 8);
        if (G > by_len) G = by_len;
        if (G > 16) G = 16;
        pl->G = G < 1 ? 1 : G;
        return PU_OK;
    }
    pl->gx = ceil_div(ext_k, pl->BK);
    pl->gy = ceil_div(ext_n, pl->BN);
    const int tiles = pl->gx * pl->gy;
    // one full round of resident blocks: a grid a few blocks past a multiple of the resident
    // slots costs a whole extra round
    const int slots = 256 * occ;
    int splits = slots / tiles;
    int max_splits = ceil_div(M, 256);
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    int mps = ceil_div(ceil_div(M, splits), WG_BM) * WG_BM;
    pl->mps = mps;
    pl->splits = ceil_div(M, mps);
    // reduction groups: one pass (G = 1, each thread sums every split of its entry) when the slab
    // has enough entries to fill the chip; otherwise G groups of >= 8 splits each, then G partials
    {
        const long long total = (long long)pl->Nr * pl->Kcp;
        int G = (int)ceil_div(262144LL, total);
        const int by_len = ceil_div(pl->splits, 8);
        if (G > by_len) G = by_len;
        if (G > 16) G = 16;
        pl->G = G < 1 ? 1 : G;
    }
    return PU_OK;
}

// ------------------------------------------------------------------ bf16 weight gradient (C3)
// dW[n][k] = sum_m P[m][n] * Q[m][k] with bf16 P (dZ or ConvT input rows) and bf16 im2col Q,
// fp32 MFMA accumulation (v_mfma_f32_32x32x16_bf16), fp32 slab partials, the same fp64 split
// reduction.  The GEMM's k dimension is the pixel index m, so each MFMA operand lane needs 8
// consecutive pixel rows of one column: the stage images are row-major [32 pixel rows][128]
// bf16 (256-byte rows) read with ds_read_b64_tr_b16 (per 16-lane group: 4 rows x 16 columns,
// delivered column-major).  The 16-byte chunk ch of row r is stored at ch ^ sw(r),
// sw(r) = ((r&3)<<2) | ((r>>2)&3) (conflict-free transposed reads on 256-byte rows); glds cannot
// permute its LDS writes, so each lane fetches the global chunk that belongs at its position.
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
__device__ __attribute__((aligned(16))) __bf16 g_wg_zero_b16[8];

constexpr int WB_ROWS = 32;   // pixel rows per stage (2 MFMA k-steps)
constexpr int WB_W = 128;     // columns per image (BN = BK = 128)


struct WgradBf16Params {
    int M, N, K, Kcp, Nr, C, c0, c1;
    int Hi, Wi, Ho, Wo, kw, stride, pad;
    const __bf16* P;
    const __bf16* src0;
    const __bf16* src1;
    int bias_mode;
    float* slab;
    int mps, gx, gy;
    FastDiv dWo, dHo, dC, dKw;
};

__global__ __launch_bounds__(256) void wgrad_bf16_kernel(const WgradBf16Params p) {
    constexpr int NBUF = 3;
    constexpr int LD = WB_ROWS * WB_W * 2 / 1024 / 4;   // glds per wave per image per stage (2)
    constexpr int G = 2 * LD;
    constexpr int IMG = WB_ROWS * WB_W;                 // bf16 elements per image
    constexpr int STAGE = 2 * IMG;
    __shared__ __attribute__((aligned(16))) __bf16 lds[NBUF * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave & 1, wk = wave >> 1;            // 2 x 2 waves, 64 x 64 each
    const int lr = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % p.gx;
    const int tyz = tile / p.gx;
    const int ty = tyz % p.gy;
    const int tz = tyz / p.gy;
    const int n_blk = ty * WB_W;
    const int k_blk = tx * WB_W;
    const int m_begin = tz * p.mps;
    const int m_end = min(p.M, m_begin + p.mps);

    // loader geometry: instruction j (= wave*LD + jj) of an image covers rows 4j .. 4j+3; lane l
    // writes physical chunk l%16 of row 4j + l/16, i.e. logical chunk (l%16) ^ sw(row)
    const int lrow = lane >> 4;                          // row within the instruction
    int p_col[LD], q_r[LD], q_s[LD], q_cs[LD];
    const __bf16* q_ptr[LD];
    bool p_in[LD];
#pragma unroll
    for (int jj = 0; jj < LD; ++jj) {
        const int j = wave * LD + jj;
        const int ch = (lane & 15) ^ ((lrow << 2) | (j & 3));
        p_col[jj] = n_blk + 8 * ch;
        p_in[jj] = p_col[jj] < p.N;
        const int qk = k_blk + 8 * ch;
        q_r[jj] = 0; q_s[jj] = 0; q_cs[jj] = 0; q_ptr[jj] = nullptr;
        if (qk < p.K) {
            const int tap = fdiv(qk, p.dC);
            const int c = qk - tap * p.C;
            q_r[jj] = fdiv(tap, p.dKw);
            q_s[jj] = tap - q_r[jj] * p.kw;
            const bool first = c < p.c0;
            q_ptr[jj] = first ? p.src0 + c : p.src1 + (c - p.c0);
            q_cs[jj] = first ? p.c0 : p.c1;
        }
    }

    auto issue = [&](int m0, int slot) {
        __bf16* ps = lds + slot * STAGE;
        __bf16* qs = ps + IMG;
#pragma unroll
        for (int jj = 0; jj < LD; ++jj) {
            const int j = wave * LD + jj;
            const int m = m0 + 4 * j + lrow;
            const __bf16* g = g_wg_zero_b16;
            if (m < m_end && p_in[jj]) g = p.P + (long long)m * p.N + p_col[jj];
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(ps + j * 512), 16, 0, 0);
        }
#pragma unroll
        for (int jj = 0; jj < LD; ++jj) {
            const int j = wave * LD + jj;
            const int mu = m0 + 4 * j;                   // wave-uniform
            const int tu = fdiv(mu, p.dWo);
            const int wou = mu - tu * p.Wo;
            const int bu = fdiv(tu, p.dHo);
            const int hou = tu - bu * p.Ho;
            int wo = wou + lrow;
            const int cw = fdiv(wo, p.dWo);
            wo -= cw * p.Wo;
            int ho = hou + cw;
            const int chh = fdiv(ho, p.dHo);
            ho -= chh * p.Ho;
            const int b = bu + chh;
            const __bf16* g = g_wg_zero_b16;
            if (mu + lrow < m_end && q_ptr[jj]) {
                const int hi = ho * p.stride - p.pad + q_r[jj], wi = wo * p.stride - p.pad + q_s[jj];
                if ((unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi)
                    g = q_ptr[jj] + ((long long)b * p.Hi * p.Wi + (long long)hi * p.Wi + wi) * q_cs[jj];
            }
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(qs + j * 512), 16, 0, 0);
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // transposed-read addressing: 16-lane group g = lane>>4 covers columns 16*(g&1) + 0..15 and
    // rows 8*(g>>1) + (0..3 | 4..7) of a k-step; lane 4q+p of the group addresses row q, columns
    // 4p..4p+3 (logical chunk (p>>1), byte half (p&1))
    const int grp = lane >> 4, gq = (lane >> 2) & 3, gp = lane & 3;
    auto tr_addr = [&](int row, int col) {   // byte offset of (row, col) in a swizzled image
        return row * (WB_W * 2) + 16 * ((col >> 3) ^ wb_sw(row)) + 2 * (col & 7);
    };
    const int T = (m_end > m_begin) ? (m_end - m_begin + WB_ROWS - 1) / WB_ROWS : 0;
    const int bias_w = (p.bias_mode == 1 && tx == 0) ? 1 : (p.bias_mode == 2 && ty == 0) ? 2 : 0;
    float bsum = 0.f;

#pragma unroll
    for (int s0 = 0; s0 < NBUF - 1; ++s0) issue(m_begin + s0 * WB_ROWS, s0);

    for (int t = 0; t < T; ++t) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* pb = reinterpret_cast<const char*>(lds + (t % NBUF) * STAGE);
        const char* qb = pb + IMG * 2;
        wbf16x8 fa[2][2], fb[2][2];   // [kstep][frag]
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int row0 = ks * 16 + 8 * (grp >> 1) + gq;
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const int ccol = 16 * (grp & 1) + 4 * gp;
                // A operand: Q^T rows = k columns of the Q image
                const int qc = wk * 64 + f * 32 + ccol;
                const wi16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(qb + tr_addr(row0, qc)));
                const wi16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(qb + tr_addr(row0 + 4, qc)));
                // B operand: P columns n
                const int pc = wn * 64 + f * 32 + ccol;
                const wi16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(pb + tr_addr(row0, pc)));
                const wi16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(pb + tr_addr(row0 + 4, pc)));
                typedef short wi16x8 __attribute__((ext_vector_type(8)));
                const wi16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                const wi16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
                fa[ks][f] = __builtin_bit_cast(wbf16x8, av);
                fb[ks][f] = __builtin_bit_cast(wbf16x8, bv);
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
            if (ks == 0) issue(m_begin + (t + NBUF - 1) * WB_ROWS, (t + NBUF - 1) % NBUF);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        if (bias_w && tid < WB_W) {           // bias column sums: P columns (mode 1) / Q (mode 2)
            const char* img = bias_w == 1 ? pb : qb;
            for (int r = 0; r < WB_ROWS; ++r)
                bsum += (float)*reinterpret_cast<const __bf16*>(img + tr_addr(r, tid));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    float* slab = p.slab + (long long)tz * p.Nr * p.Kcp;
    if (bias_w && tid < WB_W) {
        if (bias_w == 1) {
            const int n = n_blk + tid;
            if (n < p.N) slab[(long long)n * p.Kcp + p.K] = bsum;
        } else {
            const int k = k_blk + tid;
            if (k < p.K) slab[(long long)p.N * p.Kcp + k] = bsum;
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n_blk + wn * 64 + j * 32 + lr;
        if (n >= p.N) continue;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = k_blk + wk * 64 + i * 32 + 8 * q + 4 * lh;
                if (k >= p.K) continue;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                *reinterpret_cast<f32x4*>(slab + (long long)n * p.Kcp + k) = v;
            }
    }
}

// ------------------------------------------ bf16 weight gradient with halo reuse (3x3/s1, C3)
// The bf16 form of wgrad_halo_x6_kernel: the operands already are bf16, so a stage's 3 x 18 halo
// (54 pixel rows x 64 channels = 128 B per row) and its 16 dZ rows go to ONE LDS plane as they
// arrive, and each tap is one v_mfma_f32_32x32x16_bf16 per wave instead of an im2col image per
// tap (wgrad_bf16_kernel stages 9 shifted copies of every pixel).  Same swizzle (hx_off), same
// transposed reads, same 4-wave (channel half, output half) x 9-tap accumulator layout, same
// slab partials.  Two stages (32 output pixels) per barrier: the bf16 MFMA work of one stage
// (9 x 32 cycles per wave) is too short to hide a barrier.  Requirements as the x6 kernel.

template <int NT>                             // 64-channel output tiles per block (as the x6 kernel)
__global__ __launch_bounds__(256 * NT) void wgrad_halo_bf16_kernel(const WgradBf16Params p) {
    constexpr int RS = 16 * NT;               // halo rows per row group
    constexpr int XG = (HX_ROWS + RS - 1) / RS;   // halo row groups per thread (54 = 3 x 16 + 6 | 32 + 22)
    constexpr int SPB = 2;                    // stages per barrier
    constexpr int IMG = (HX_ROWS + 16 * NT) * 128;  // one stage's plane: 54 X rows, then NT x 16 dZ rows
    __shared__ __attribute__((aligned(16))) char lds[2 * SPB * IMG];
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ci = wave & 1, nj = (wave >> 1) & 1, nt = wave >> 2;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % p.gx;               // 64-channel input tile
    const int tyz = tile / p.gx;
    const int ty = tyz % p.gy;                // 64-channel output tile
    const int tz = tyz / p.gy;
    const int m_begin = tz * p.mps;
    const int m_end = min(p.M, m_begin + p.mps);
    const int T = m_end > m_begin ? (m_end - m_begin) / 16 : 0;

    const int cq = tid & 15;                  // 4-channel quad of the row this thread loads
    const int c_lo = tx * 64;
    const bool first = c_lo < p.c0;
    const __bf16* xsrc = first ? p.src0 + c_lo : p.src1 + (c_lo - p.c0);
    const int cs = first ? p.c0 : p.c1;
    const __bf16* zero = reinterpret_cast<const __bf16*>(g_wg_zero16);
    const __bf16* x_lane[XG];
    unsigned x_cls[XG];                       // edge classes: 1 top, 2 bottom, 4 left, 8 right, 16 past the halo, 32 all
#pragma unroll
    for (int i = 0; i < XG; ++i) {
        const int hp = (tid >> 4) + RS * i;
        const int rr = hp / 18, cc = hp - rr * 18;
        x_lane[i] = xsrc + (long long)((rr - 1) * p.Wi + (cc - 1)) * cs + cq * 4;
        if (hp >= HX_ROWS) x_lane[i] = zero;
        x_cls[i] = 32u | (hp >= HX_ROWS ? 16u
                                        : ((rr == 0 ? 1u : 0u) | (rr == 2 ? 2u : 0u) | (cc == 0 ? 4u : 0u) | (cc == 17 ? 8u : 0u)));
    }
    const int pq = tid % (16 * NT), prow = tid / (16 * NT);   // dZ row and channel quad
    const __bf16* p_lane = p.P + (long long)prow * p.N + ty * 64 * NT + pq * 4;

    u32x2 rx[SPB][XG], rp[SPB];
    auto load = [&](int t, int j) {           // raw bf16 rows of stage t into register set j
        const int m0 = m_begin + 16 * t;
        const int tu = fdiv(m0, p.dWo);
        const int wo0 = m0 - tu * p.Wo;
        const int bu = fdiv(tu, p.dHo);
        const int ho = tu - bu * p.Ho;
        const bool live = t < T;
        const unsigned flags = live ? (16u | (ho == 0 ? 1u : 0u) | (ho == p.Ho - 1 ? 2u : 0u) | (wo0 == 0 ? 4u : 0u) |
                                       (wo0 + 16 == p.Wo ? 8u : 0u))
                                    : 0xffffffffu;
        const unsigned xo = __umul24((unsigned)m0, (unsigned)cs);
#pragma unroll
        for (int i = 0; i < XG; ++i) {
            const __bf16* g = (x_cls[i] & flags) ? zero : x_lane[i] + xo;
            rx[j][i] = *reinterpret_cast<const u32x2*>(g);
        }
        const __bf16* gp = live ? p_lane + __umul24((unsigned)m0, (unsigned)p.N) : zero;
        rp[j] = *reinterpret_cast<const u32x2*>(gp);
    };
    f32x4 bsum = {0.f, 0.f, 0.f, 0.f};
    const bool bias_blk = p.bias_mode == 1 && tx == 0;
    const int w_base = hx_off(tid >> 4, cq * 4);
    const int wp_base = hx_off(HX_ROWS + 16 * (pq >> 4) + prow, (pq & 15) * 4);
    auto store = [&](int buf, int j, bool live) {   // register set j -> plane j of buffer buf
        char* pb = lds + (buf * SPB + j) * IMG;
#pragma unroll
        for (int i = 0; i < XG; ++i) {
            const int hp = (tid >> 4) + RS * i;
            if (i < XG - 1 || hp < HX_ROWS) *reinterpret_cast<u32x2*>(pb + w_base + i * RS * 128) = rx[j][i];
        }
        *reinterpret_cast<u32x2*>(pb + wp_base) = rp[j];
        if (bias_blk && live) {
            bsum[0] += __builtin_bit_cast(float, rp[j][0] << 16);
            bsum[1] += __builtin_bit_cast(float, rp[j][0] & 0xffff0000u);
            bsum[2] += __builtin_bit_cast(float, rp[j][1] << 16);
            bsum[3] += __builtin_bit_cast(float, rp[j][1] & 0xffff0000u);
        }
    };

    f32x16 acc[9];
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t9][r] = 0.f;

    const int grp = lane >> 4, gq = (lane >> 2) & 3, gp = lane & 3;
    const int rsub = 8 * (grp >> 1) + gq;
    const int ccol = 16 * (grp & 1) + 4 * gp;
    int xb[4];
#pragma unroll
    for (int res = 0; res < 4; ++res) xb[res] = hx_off(res + rsub, ci * 32 + ccol);
    const int pbase = hx_off(HX_ROWS + 16 * nt + rsub, nj * 32 + ccol);
    auto tr2 = [&](const char* a) {
        const wi16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)a);
        const wi16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(a + 4 * 128));
        typedef short wi16x8 __attribute__((ext_vector_type(8)));
        const wi16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        return __builtin_bit_cast(wg_bf16x8, av);
    };
    auto mfma_plane = [&](const char* pb) {
        const wg_bf16x8 ph = tr2(pb + pbase);
#pragma unroll
        for (int t9 = 0; t9 < 9; ++t9) {
            const int row0 = (t9 / 3) * 18 + (t9 % 3);
            const wg_bf16x8 qh = tr2(pb + xb[row0 & 3] + (row0 & ~3) * 128);
            acc[t9] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, ph, acc[t9], 0, 0, 0);
        }
    };
    // group g = stages SPB g .. SPB g + SPB - 1 in buffer g & 1; the loads of group g + 1 are in
    // flight while group g's MFMAs run
    const int NG = (T + SPB - 1) / SPB;
    auto group = [&](int g, auto bufc) {
        constexpr int buf = decltype(bufc)::value;
#pragma unroll
        for (int j = 0; j < SPB; ++j) mfma_plane(lds + (buf * SPB + j) * IMG);
        if (g + 1 < NG) {
#pragma unroll
            for (int j = 0; j < SPB; ++j) store(buf ^ 1, j, SPB * (g + 1) + j < T);
#pragma unroll
            for (int j = 0; j < SPB; ++j) load(SPB * (g + 2) + j, j);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    if (NG > 0) {
#pragma unroll
        for (int j = 0; j < SPB; ++j) load(j, j);
#pragma unroll
        for (int j = 0; j < SPB; ++j) store(0, j, j < T);
#pragma unroll
        for (int j = 0; j < SPB; ++j) load(SPB + j, j);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    int g = 0;
    for (; g + 1 < NG; g += 2) {
        group(g, std::integral_constant<int, 0>{});
        group(g + 1, std::integral_constant<int, 1>{});
    }
    if (g < NG) group(g, std::integral_constant<int, 0>{});

    float* slab = p.slab + (long long)tz * p.Nr * p.Kcp;
    if (bias_blk) {
        f32x4* red = reinterpret_cast<f32x4*>(lds);
        red[tid] = bsum;
        __syncthreads();
        if (tid < 16 * NT) {
            f32x4 v = red[tid];
            for (int r = 1; r < 16; ++r) v += red[r * 16 * NT + tid];
#pragma unroll
            for (int e = 0; e < 4; ++e) slab[(long long)(ty * 64 * NT + tid * 4 + e) * p.Kcp + p.K] = v[e];
        }
    }
    const int lr = lane & 31, lh = lane >> 5;
    const int n = ty * 64 * NT + nt * 64 + nj * 32 + lr;
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = t9 * p.C + c_lo + ci * 32 + 8 * q + 4 * lh;
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[t9][4 * q + e];
            *reinterpret_cast<f32x4*>(slab + (long long)n * p.Kcp + k) = v;
        }
    }
}

// One-launch reduction for the direct small-channel / stem weight gradients: up to 1024 split
// rows of a few thousand entries, where the two-pass form's per-thread chains over 64 splits were
// latency rounds, not bytes.  Block = 16 entries (4 float4 quads) x 64 split lanes: lane s sums
// splits s, s + 64, ... in 4 fp64 chains, then thread e < 16 sums the 64 lanes in order and
// scatters entry e into [n][c][kh][kw] (bias at column K) - a fixed order, deterministic.
constexpr int WR_E = 16, WR_S = 64;
__global__ __launch_bounds__(256) void wgrad_reduce_wide_kernel(const float* __restrict__ slab, int splits,
                                                                 long long total, int N, int Kcp, int K, int C,
                                                                 int kh, int kw, int bias_mode, float* __restrict__ dw,
                                                                 float* __restrict__ db, int accumulate) {
    __shared__ double part[WR_S][WR_E];
    const int quad = threadIdx.x & 3, sl = threadIdx.x >> 2;
    const long long idx0 = (long long)blockIdx.x * WR_E + 4 * quad;
    double a[4][4] = {};
    if (idx0 < total) {                               // total % 4 == 0 (Kcp % 4 == 0)
        const float* sp = slab + idx0;
        int z = sl;
        for (; z + 3 * WR_S < splits; z += 4 * WR_S) {
            f32x4 v[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const f32x4*>(sp + (long long)(z + c * WR_S) * total);
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e) a[c][e] += (double)v[c][e];
        }
        for (; z < splits; z += WR_S) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(sp + (long long)z * total);
#pragma unroll
            for (int e = 0; e < 4; ++e) a[0][e] += (double)v[e];
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) part[sl][4 * quad + e] = (a[0][e] + a[1][e]) + (a[2][e] + a[3][e]);
    __syncthreads();
    if (threadIdx.x >= WR_E) return;
    const long long idx = (long long)blockIdx.x * WR_E + threadIdx.x;
    if (idx >= total) return;
    double sum = 0.0;
    for (int l = 0; l < WR_S; ++l) sum += part[l][threadIdx.x];
    const float v = (float)sum;
    const int n = (int)(idx / Kcp), k = (int)(idx - (long long)n * Kcp);
    if (n >= N) return;
    if (k < K) {
        const int tap = k / C, ch = k - tap * C;
        const int r = tap / kw, ss = tap - r * kw;
        float* o = dw + (((long long)n * C + ch) * kh + r) * kw + ss;
        *o = accumulate ? *o + v : v;
    } else if (bias_mode == 1 && k == K) {
        db[n] = accumulate ? db[n] + v : v;
    }
}

// phase 2 of every weight-gradient path: fixed-order fp64 reduction of the split partials and
// the scatter into PyTorch's [n][c][kh][kw] (+ bias)
// The one-launch wide reduction also takes the non-Winograd plans whose slab rows are short
// (Nr x Kcp <= WR_WIDE_MAX entries: C4 / C5's 32-channel weight gradients, 9216 entries over
// hundreds of splits), where the grouped form is two latency-bound launches: C5 +0.8 %, C4 +0.7 %
// (`r06_experiments/wgrad_reduce_wide_ab.txt`).  Long rows (C2 / C3, >= 32K entries) keep the
// grouped form: the wide one took C3's bf16 reductions from 0.36 to 1.39 ms per step.
// PU_WR_WIDE (A/B runs): 0 = small / stem / pointwise plans only (the round-6 form), 2 = every plan.
// The split partials are summed in fp64 either way, in a different fixed order.
constexpr long long WR_WIDE_MAX = 16384;
static int wr_wide_mode() {
    static const int m = [] {
        const char* e = getenv("PU_WR_WIDE");
        return e ? atoi(e) : 1;
    }();
    return m;
}

static int wgrad_reduce(const WgradPlan& pl, const pu_wgrad_args* a, void* workspace, hipStream_t s) {
    const long long total = (long long)pl.Nr * pl.Kcp;
    const long long threads = total + (a->bias_mode == 2 ? pl.C : 0);
    const dim3 fgrid((unsigned)((threads + 255) / 256));
    const int taps = a->kh * a->kw;
    // one launch for up to 1024 splits of a few-thousand-entry slab (the direct small-channel /
    // stem kernels; measured slower than the two-pass grouped form on the Winograd-domain
    // kernel's 64-256 splits: 0.37 vs 0.32 ms per C2 step)
    const bool wide = pl.small || pl.stem || pl.pw || (wr_wide_mode() == 1 && !pl.wino && total <= WR_WIDE_MAX) ||
                      wr_wide_mode() == 2;
    if (wide && a->bias_mode != 2 && pl.Kcp % 4 == 0) {
        hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)ceil_div(total, (long long)WR_E)), dim3(256), 0, s,
                           (const float*)workspace, pl.splits, total, a->n, pl.Kcp, pl.K, pl.C, a->kh, a->kw,
                           a->bias_mode, a->dweight, a->dbias, a->accumulate);
        return check_launch("pu_wgrad (reduce)");
    }
    if (a->bias_mode != 2 && taps <= 9 && pl.C % 4 == 0 && pl.Kcp % 4 == 0 && ((uintptr_t)a->dweight & 15) == 0) {
        const dim3 tgrid((unsigned)ceil_div(pl.C, 256), (unsigned)a->n);
        const dim3 tblock((unsigned)(64 * taps));
        if (pl.G == 1) {
            hipLaunchKernelGGL(wgrad_finish_t_kernel<float>, tgrid, tblock, 0, s, (const float*)workspace, pl.splits,
                               pl.Nr, pl.Kcp, pl.K, pl.C, taps, a->bias_mode, a->dweight, a->dbias, a->accumulate);
        } else {
            double* part = (double*)((char*)workspace + ((pl.slab_bytes() + 255) / 256) * 256);
            hipLaunchKernelGGL(wgrad_sum_splits4_kernel, dim3((unsigned)((total / 4 + 255) / 256), pl.G), dim3(256), 0,
                               s, (const float*)workspace, pl.splits, total, pl.G, part);
            hipLaunchKernelGGL(wgrad_finish_t_kernel<double>, tgrid, tblock, 0, s, (const double*)part, pl.G, pl.Nr,
                               pl.Kcp, pl.K, pl.C, taps, a->bias_mode, a->dweight, a->dbias, a->accumulate);
        }
        return check_launch("pu_wgrad (reduce)");
    }
    if (pl.Kcp % 4 == 0) {
        const long long threads4 = total / 4 + (a->bias_mode == 2 ? pl.C : 0);
        const dim3 grid4((unsigned)((threads4 + 255) / 256));
        if (pl.G == 1) {
            hipLaunchKernelGGL(wgrad_finish4_kernel<float>, grid4, dim3(256), 0, s, (const float*)workspace,
                               pl.splits, pl.Nr, pl.Kcp, a->n, pl.K, pl.C, a->kh, a->kw, a->bias_mode, a->dweight,
                               a->dbias, a->accumulate);
        } else {
            double* part = (double*)((char*)workspace + ((pl.slab_bytes() + 255) / 256) * 256);
            hipLaunchKernelGGL(wgrad_sum_splits4_kernel, dim3((unsigned)((total / 4 + 255) / 256), pl.G), dim3(256), 0,
                               s, (const float*)workspace, pl.splits, total, pl.G, part);
            hipLaunchKernelGGL(wgrad_finish4_kernel<double>, grid4, dim3(256), 0, s, (const double*)part, pl.G,
                               pl.Nr, pl.Kcp, a->n, pl.K, pl.C, a->kh, a->kw, a->bias_mode, a->dweight, a->dbias,
                               a->accumulate);
        }
        return check_launch("pu_wgrad (reduce)");
    }
    if (pl.G == 1) {
        hipLaunchKernelGGL(wgrad_finish_kernel<float>, fgrid, dim3(256), 0, s, (const float*)workspace, pl.splits,
                           pl.Nr, pl.Kcp, a->n, pl.K, pl.C, a->kh, a->kw, a->bias_mode, a->dweight, a->dbias,
                           a->accumulate);
    } else {
        double* part = (double*)((char*)workspace + ((pl.slab_bytes() + 255) / 256) * 256);
        hipLaunchKernelGGL(wgrad_sum_splits_kernel, dim3((unsigned)((total + 255) / 256), pl.G), dim3(256), 0, s,
                           (const float*)workspace, pl.splits, total, pl.G, part);
        hipLaunchKernelGGL(wgrad_finish_kernel<double>, fgrid, dim3(256), 0, s, (const double*)part, pl.G, pl.Nr,
                           pl.Kcp, a->n, pl.K, pl.C, a->kh, a->kw, a->bias_mode, a->dweight, a->dbias,
                           a->accumulate);
    }
    return check_launch("pu_wgrad (reduce)");
}

static void plan_groups(WgradPlan* pl) {
    const long long total = (long long)pl->Nr * pl->Kcp;
    int G = (int)ceil_div(262144LL, total);
    const int by_len = ceil_div(pl->splits, 8);
    if (G > by_len) G = by_len;
    if (G > 16) G = 16;
    pl->G = G < 1 ? 1 : G;
}

// bf16 plan: 128 x 128 tiles of the N x K GEMM (bias via LDS column sums), pixel rows split so
// that one round of resident blocks (3 per CU: 48 KB ring) fills the chip
static int plan_wgrad_bf16(const pu_wgrad_args* a, WgradPlan* pl) {
    PU_REQUIRE(a && a->batch > 0 && a->out_h > 0 && a->out_w > 0 && a->in_h > 0 && a->in_w > 0, "pu_wgrad_bf16: bad grid");
    PU_REQUIRE(a->kh > 0 && a->kw > 0 && a->stride > 0 && a->pad >= 0, "pu_wgrad_bf16: bad taps");
    PU_REQUIRE(a->rows && a->n > 0 && a->src0 && a->c0 > 0 && (a->c1 == 0 || a->src1), "pu_wgrad_bf16: operands");
    PU_REQUIRE(a->n % 8 == 0 && a->c0 % 8 == 0 && a->c1 % 8 == 0,
               "pu_wgrad_bf16: n (%d) and channel counts (%d, %d) must be multiples of 8", a->n, a->c0, a->c1);
    PU_REQUIRE(a->bias_mode >= 0 && a->bias_mode <= 2 && (a->bias_mode == 0 || a->dbias) && a->dweight, "pu_wgrad_bf16: outputs");
    PU_REQUIRE((((uintptr_t)a->rows | (uintptr_t)a->src0 | (uintptr_t)a->src1) & 15) == 0, "pu_wgrad_bf16: 16-byte alignment");
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    PU_REQUIRE(M < (1LL << 31), "pu_wgrad_bf16: too many pixels");
    pl->M = (int)M;
    pl->C = a->c0 + a->c1;
    pl->K = a->kh * a->kw * pl->C;
    pl->Nr = a->n + (a->bias_mode == 2 ? 1 : 0);
    pl->Kc = pl->K + (a->bias_mode == 1 ? 1 : 0);
    pl->Kcp = (pl->Kc + 3) / 4 * 4;
    pl->qvec = true; pl->dma = true; pl->small = false; pl->stem = false;
    pl->halo = a->kh == 3 && a->kw == 3 && a->stride == 1 && a->pad == 1 && a->in_h == a->out_h &&
               a->in_w == a->out_w && a->out_w % 16 == 0 && a->c0 % 64 == 0 && a->c1 % 64 == 0 && a->n % 64 == 0 &&
               a->bias_mode != 2 && M * pl->C < (1LL << 31);
    if (pl->halo) {                   // wgrad_halo_bf16_kernel: 64 NT x 64 x 9-tap tiles, 512 NT-thread blocks
        pl->nt = a->n % 128 == 0 ? 2 : 1;
        pl->BN = 64 * pl->nt; pl->BK = 9 * 64;
        pl->gx = pl->C / 64;
        pl->gy = a->n / pl->BN;
        const int stages = (int)(M / 16);
        int splits = (pl->nt == 2 ? 256 : 512) / (pl->gx * pl->gy);   // one 8-wave / two 4-wave blocks per CU
        if (splits > stages) splits = stages;
        if (splits < 1) splits = 1;
        pl->mps = ceil_div(stages, splits) * 16;
        pl->splits = ceil_div((int)M, pl->mps);
        plan_groups(pl);
        return PU_OK;
    }
    pl->BN = WB_W; pl->BK = WB_W;
    pl->gx = ceil_div(pl->K, WB_W);
    pl->gy = ceil_div(a->n, WB_W);
    const int tiles = pl->gx * pl->gy;
    int splits = 768 / tiles;
    const int max_splits = ceil_div(M, 512);
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    pl->mps = ceil_div(ceil_div(M, splits), WB_ROWS) * WB_ROWS;
    pl->splits = ceil_div(M, pl->mps);
    plan_groups(pl);
    return PU_OK;
}

}  // namespace pu

using namespace pu;

extern "C" size_t pu_wgrad_workspace_bytes(const pu_wgrad_args* a) {
    WgradPlan pl;
    if (plan_wgrad(a, &pl) != PU_OK) return 0;
    return pl.ws_bytes();
}

extern "C" int pu_wgrad_tile(const pu_wgrad_args* a, int* bn, int* bk, int* qvec, int* splits) {
    WgradPlan pl;
    int st = plan_wgrad(a, &pl);
    if (st != PU_OK) return st;
    if (bn) *bn = pl.BN;
    if (bk) *bk = pl.BK;
    if (qvec) *qvec = pl.pw ? 6 : pl.wino ? 5 : pl.stem ? 4 : pl.small ? 2 : pl.halo ? 3 : (pl.qvec ? 1 : 0);   // 2: small-channel direct, 3: halo, 4: stem, 5: Winograd, 6: pointwise
    if (splits) *splits = pl.splits;
    return PU_OK;
}

extern "C" int pu_wgrad(const pu_wgrad_args* a, void* workspace, size_t ws_bytes, void* stream) {
    return pu_wgrad_phase(a, workspace, ws_bytes, 3, stream);
}

extern "C" int pu_wgrad_phase(const pu_wgrad_args* a, void* workspace, size_t ws_bytes, int phase, void* stream) {
    PU_REQUIRE(phase >= 1 && phase <= 3, "pu_wgrad_phase: phase %d", phase);
    WgradPlan pl;
    int st = plan_wgrad(a, &pl);
    if (st != PU_OK) return st;
    const size_t need = pl.ws_bytes();
    if (!workspace || ws_bytes < need)
        return fail(PU_ERR_WORKSPACE, "pu_wgrad: workspace %zu < %zu bytes", ws_bytes, need);

    WgradParams p;
    p.M = pl.M; p.N = a->n; p.Nr = pl.Nr; p.K = pl.K; p.Kc = pl.Kc; p.Kcp = pl.Kcp; p.C = pl.C; p.c0 = a->c0; p.c1 = a->c1;
    p.Hi = a->in_h; p.Wi = a->in_w; p.Ho = a->out_h; p.Wo = a->out_w;
    p.kw = a->kw; p.stride = a->stride; p.pad = a->pad;
    p.P = a->rows; p.src0 = a->src0; p.src1 = a->src1; p.bias_mode = a->bias_mode;
    p.slab = (float*)workspace; p.mps = pl.mps;
    p.dWo = make_fastdiv(a->out_w); p.dHo = make_fastdiv(a->out_h);
    p.dC = make_fastdiv(pl.C); p.dKw = make_fastdiv(a->kw);

    hipStream_t s = as_stream(stream);
    p.gx = pl.gx;
    p.gy = pl.gy;
    p.batch = a->batch; p.tiles_w = pl.tiles_w; p.tiles_h = pl.tiles_h;
    if (pl.stem && (phase & 1) && a->math == 2) {
        if (a->n == 64) hipLaunchKernelGGL((wgrad_stem_kernel<64, true>), dim3(pl.splits), dim3(256), 0, s, p);
        else if (a->n == 32) hipLaunchKernelGGL((wgrad_stem_kernel<32, true>), dim3(pl.splits), dim3(256), 0, s, p);
        else if (a->n == 16) hipLaunchKernelGGL((wgrad_stem_kernel<16, true>), dim3(pl.splits), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((wgrad_stem_kernel<8, true>), dim3(pl.splits), dim3(256), 0, s, p);
        st = check_launch("pu_wgrad (stem, bf16 rows)");
        if (st != PU_OK) return st;
        phase &= ~1;
    }
    if (pl.stem && (phase & 1)) {
        if (a->n == 64) hipLaunchKernelGGL(wgrad_stem_kernel<64>, dim3(pl.splits), dim3(256), 0, s, p);
        else if (a->n == 32) hipLaunchKernelGGL(wgrad_stem_kernel<32>, dim3(pl.splits), dim3(256), 0, s, p);
        else if (a->n == 16) hipLaunchKernelGGL(wgrad_stem_kernel<16>, dim3(pl.splits), dim3(256), 0, s, p);
        else hipLaunchKernelGGL(wgrad_stem_kernel<8>, dim3(pl.splits), dim3(256), 0, s, p);
        st = check_launch("pu_wgrad (stem)");
        if (st != PU_OK) return st;
        phase &= ~1;
    }
    if (pl.pw && (phase & 1)) {
        const int C = pl.C, N = a->n;
        const dim3 sg(pl.splits);
#define PU_PW(C_, N_) if (C == C_ && N == N_) hipLaunchKernelGGL((wgrad_pw_kernel<C_, N_>), sg, dim3(256), 0, s, p)
        PU_PW(3, 4); else PU_PW(3, 8); else PU_PW(3, 16); else PU_PW(4, 4); else PU_PW(4, 8); else PU_PW(4, 16);
#undef PU_PW
        st = check_launch("pu_wgrad (pointwise)");
        if (st != PU_OK) return st;
        phase &= ~1;
    }
    if (pl.small && (phase & 1)) {
        const int C = pl.C, N = a->n;
        const dim3 sg(pl.splits);
#define PU_SW(C_, N_) if (C == C_ && N == N_) hipLaunchKernelGGL((wgrad_small_kernel<C_, N_>), sg, dim3(256), 0, s, p)
        PU_SW(1, 4); else PU_SW(1, 8); else PU_SW(1, 16); else PU_SW(4, 4); else PU_SW(4, 8); else PU_SW(4, 16);
        else PU_SW(8, 4); else PU_SW(8, 8); else PU_SW(8, 16); else PU_SW(12, 4); else PU_SW(12, 8);
        else PU_SW(12, 16); else PU_SW(16, 4); else PU_SW(16, 8); else PU_SW(16, 16);
#undef PU_SW
        st = check_launch("pu_wgrad (small-channel)");
        if (st != PU_OK) return st;
        phase &= ~1;
    }
    dim3 grid(p.gx * p.gy * pl.splits);
    const bool fq = a->stride == 1 && a->in_h == a->out_h && a->in_w == a->out_w && a->out_w >= 4;
    if (phase & 1) {
#define PU_WG_DMA(BN_, BK_, WN_, WK_)                                                                    \
    do {                                                                                                     \
        if (a->math == 1 && fq) hipLaunchKernelGGL((wgrad_dma_kernel<BN_, BK_, WN_, WK_, 3, true, 4, true>), grid, dim3(256), 0, s, p); \
        else if (a->math == 1) hipLaunchKernelGGL((wgrad_dma_kernel<BN_, BK_, WN_, WK_, 3, true>), grid, dim3(256), 0, s, p); \
        else hipLaunchKernelGGL((wgrad_dma_kernel<BN_, BK_, WN_, WK_, 3, false>), grid, dim3(256), 0, s, p); \
    } while (0)
#define PU_WG_REG(BN_, BK_, WN_, WK_, Q_) hipLaunchKernelGGL((wgrad_kernel<BN_, BK_, WN_, WK_, Q_>), grid, dim3(256), 0, s, p)
        if (pl.wino) {
            WinoWgradParams ww;
            ww.p = p;
            ww.tiles = pl.tiles;
            ww.tps = pl.tps;
            ww.dTw = make_fastdiv(a->out_w / 2);
            ww.dTh = make_fastdiv(a->out_h / 2);
            const long long px = (long long)a->batch * a->in_h * a->in_w + a->in_w + 1;
            ww.x0_bytes = (unsigned)(px * a->c0 * 4);
            ww.x1_bytes = (unsigned)(px * a->c1 * 4);
            ww.p_bytes = (unsigned)((long long)pl.M * a->n * 4);
            if (ww4_on() && (((uintptr_t)a->rows | (uintptr_t)a->src0 | (uintptr_t)a->src1) & 15) == 0)
                hipLaunchKernelGGL(wgrad_wino4_x6_kernel, grid, dim3(256), 0, s, ww);
            else
                hipLaunchKernelGGL(wgrad_wino_x6_kernel, grid, dim3(512), 0, s, ww);
        } else if (pl.halo) {
            if (pl.nt == 2) hipLaunchKernelGGL(wgrad_halo_x6_kernel<2>, grid, dim3(512), 0, s, p);
            else hipLaunchKernelGGL(wgrad_halo_x6_kernel<1>, grid, dim3(256), 0, s, p);
        } else if (pl.dma) {
            if (pl.BK == 64) PU_WG_DMA(64, 64, 2, 2);
            else if (pl.BN == 64 && pl.BK == 128) PU_WG_DMA(64, 128, 2, 2);
            else if (pl.BN == 32) PU_WG_DMA(32, 128, 1, 4);
            else if (pl.BK == 192) PU_WG_DMA(64, 192, 2, 2);
            else if (pl.BK == 256 && fq) hipLaunchKernelGGL((wgrad_dma_kernel<128, 256, 2, 2, 3, true, 4, true>), grid, dim3(256), 0, s, p);
            else if (pl.BK == 256) hipLaunchKernelGGL((wgrad_dma_kernel<128, 256, 2, 2, 3, true>), grid, dim3(256), 0, s, p);
            else PU_WG_DMA(128, 128, 2, 2);
        } else if (pl.qvec) {
            if (pl.BK == 64) PU_WG_REG(64, 64, 2, 2, true);
            else if (pl.BK == 256) PU_WG_REG(64, 256, 1, 4, true);
            else PU_WG_REG(128, 128, 2, 2, true);
        } else {
            if (pl.BK == 64) PU_WG_REG(64, 64, 2, 2, false);
            else if (pl.BK == 256) PU_WG_REG(64, 256, 1, 4, false);
            else PU_WG_REG(128, 128, 2, 2, false);
        }
#undef PU_WG_DMA
#undef PU_WG_REG
        st = check_launch("pu_wgrad (gemm)");
        if (st != PU_OK) return st;
    }
    if (!(phase & 2)) return PU_OK;
    return wgrad_reduce(pl, a, workspace, s);
}

extern "C" size_t pu_wgrad_bf16_workspace_bytes(const pu_wgrad_args* a) {
    WgradPlan pl;
    if (plan_wgrad_bf16(a, &pl) != PU_OK) return 0;
    return pl.ws_bytes();
}

extern "C" int pu_wgrad_bf16_phase(const pu_wgrad_args* a, void* workspace, size_t ws_bytes, int phase, void* stream) {
    PU_REQUIRE(phase >= 1 && phase <= 3, "pu_wgrad_bf16_phase: phase %d", phase);
    WgradPlan pl;
    int st = plan_wgrad_bf16(a, &pl);
    if (st != PU_OK) return st;
    const size_t need = pl.ws_bytes();
    if (!workspace || ws_bytes < need)
        return fail(PU_ERR_WORKSPACE, "pu_wgrad_bf16: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t s = as_stream(stream);
    if (phase & 1) {
        WgradBf16Params p;
        p.M = pl.M; p.N = a->n; p.K = pl.K; p.Kcp = pl.Kcp; p.Nr = pl.Nr; p.C = pl.C; p.c0 = a->c0; p.c1 = a->c1;
        p.Hi = a->in_h; p.Wi = a->in_w; p.Ho = a->out_h; p.Wo = a->out_w;
        p.kw = a->kw; p.stride = a->stride; p.pad = a->pad;
        p.P = (const __bf16*)a->rows; p.src0 = (const __bf16*)a->src0; p.src1 = (const __bf16*)a->src1;
        p.bias_mode = a->bias_mode;
        p.slab = (float*)workspace; p.mps = pl.mps; p.gx = pl.gx; p.gy = pl.gy;
        p.dWo = make_fastdiv(a->out_w); p.dHo = make_fastdiv(a->out_h);
        p.dC = make_fastdiv(pl.C); p.dKw = make_fastdiv(a->kw);
        if (pl.halo && pl.nt == 2) hipLaunchKernelGGL(wgrad_halo_bf16_kernel<2>, dim3(pl.gx * pl.gy * pl.splits), dim3(512), 0, s, p);
        else if (pl.halo) hipLaunchKernelGGL(wgrad_halo_bf16_kernel<1>, dim3(pl.gx * pl.gy * pl.splits), dim3(256), 0, s, p);
        else hipLaunchKernelGGL(wgrad_bf16_kernel, dim3(pl.gx * pl.gy * pl.splits), dim3(256), 0, s, p);
        st = check_launch("pu_wgrad_bf16 (gemm)");
        if (st != PU_OK) return st;
    }
    if (!(phase & 2)) return PU_OK;
    return wgrad_reduce(pl, a, workspace, s);
}

extern "C" int pu_wgrad_bf16_tile(const pu_wgrad_args* a, int* bn, int* bk, int* halo, int* splits) {
    WgradPlan pl;
    int st = plan_wgrad_bf16(a, &pl);
    if (st != PU_OK) return st;
    if (bn) *bn = pl.BN;
    if (bk) *bk = pl.BK;
    if (halo) *halo = pl.halo ? 1 : 0;
    if (splits) *splits = pl.splits;
    return PU_OK;
}

extern "C" int pu_wgrad_bf16(const pu_wgrad_args* a, void* workspace, size_t ws_bytes, void* stream) {
    return pu_wgrad_bf16_phase(a, workspace, ws_bytes, 3, stream);
}
