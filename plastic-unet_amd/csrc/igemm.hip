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
#include "conv_common.h"
#include <type_traits>


#ifndef PU_EPI_BATCH
#define PU_EPI_BATCH 1   // 0: every output through epi_store4 (A/B builds)
#endif

namespace pu {


constexpr int IG_BK = 16;
constexpr int IG_LDS = IG_BK + 4;

enum { LOAD_CHUNK16 = 0, LOAD_VEC4 = 1, LOAD_SCALAR = 2 };


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


// The epilogue's two common forms - bias (+ReLU), the forward, or masks (+ReLU), the data
// gradient, into one or two NHWC destinations - with every operand load issued before the first
// store.  gfx9's vmcnt counts stores as well as loads, and epi_store4 loads each output's operand
// right before its store: the wait for that load then also waited out the round trip of every
// store before it, one store latency per output.  Operands and stores go through buffer
// descriptors with 32-bit offsets (a 32-column fragment lies in one destination: n0 % 32 == 0,
// so the descriptor is wave-uniform per fragment); lanes past M / N load zeros and drop their
// stores (out-of-range offsets), so no per-lane branch splits the batch.  The bias is per channel:
// MASK == false reads it per fragment column group.  Same operations in the same order as
// epi_store4 (bias, ReLU, mask).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t epi_rsrc(const void* base, bool on) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    void* ub = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(ub, 0, on ? 0x7fffffff : 0, 0x00020000);
}

template <bool MASK, int FM, int FN>
__device__ __forceinline__ void epilogue_batched(const IgemmParams& p, f32x16 (&acc)[FM][FN], int m0, int nc0, int lr,
                                                 int lh) {
    const bool relu = p.flags & PU_EPI_RELU;
    const int n1 = p.N - p.n0;
    unsigned orow[FM][FN];             // byte offset of (row m, fragment column 0), LEAN_OOB past M
    bool first[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) first[j] = nc0 + j * 32 < p.n0;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m0 + i * 32 + lr;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int c = nc0 + j * 32 + 4 * lh - (first[j] ? 0 : p.n0);
            orow[i][j] = m < p.M && nc0 + j * 32 < p.N ? (unsigned)(m * (first[j] ? p.n0 : n1) + c) * 4u : LEAN_OOB;
        }
    }
    f32x4 ov[FM][FN][4];               // MASK: the mask of each output; else the bias of its channels
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        if constexpr (MASK) {
            const float* mk = first[j] ? p.mask0 : p.mask1;
            const __amdgpu_buffer_rsrc_t r = epi_rsrc(mk, mk != nullptr);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    ov[i][j][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, orow[i][j], 32 * q, 0));
        } else {
            const __amdgpu_buffer_rsrc_t r = epi_rsrc(p.bias, true);
            const unsigned nb = nc0 + j * 32 < p.N ? (unsigned)(nc0 + j * 32 + 4 * lh) * 4u : LEAN_OOB;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                ov[0][j][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, nb, 32 * q, 0));
        }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const __amdgpu_buffer_rsrc_t rd = epi_rsrc(first[j] ? p.dst0 : p.dst1, true);
        const bool has_mk = (first[j] ? p.mask0 : p.mask1) != nullptr;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                if constexpr (!MASK) v += ov[0][j][q];
                if (relu) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                }
                if constexpr (MASK) {
                    if (has_mk) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) if (!(ov[i][j][q][e] > 0.f)) v[e] = 0.f;
                    }
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rd, orow[i][j], 32 * q, 0);
            }
    }
}

// The ConvTranspose2d 2x2 / s2 forward's epilogue (SHUFFLE2 without a crop: column n = ij * co + c
// goes to pixel (2ho + i, 2wo + j) of the 2H x 2W grid, + bias[c]) in the same batched form: every
// bias load before the first store.  co % 32 == 0, so a 32-column fragment lies in one (i, j).
template <int FM, int FN>
__device__ __forceinline__ void epilogue_batched_shuf(const IgemmParams& p, f32x16 (&acc)[FM][FN], int m0, int nc0,
                                                      int lr, int lh) {
    const bool relu = p.flags & PU_EPI_RELU;
    const int co = p.N >> 2;
    unsigned orow[FM][FN];
    int cj[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int nj = nc0 + j * 32;
        const int ij = nj < p.N ? nj / co : 0;
        cj[j] = nj - ij * co + 4 * lh;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int m = m0 + i * 32 + lr;
            unsigned o = LEAN_OOB;
            if (m < p.M && nj < p.N) {
                const int t2 = fdiv(m, p.dWo);
                const int wo = m - t2 * p.Wo;
                const int bb = fdiv(t2, p.dHo);
                const int ho = t2 - bb * p.Ho;
                const int pix = (bb * p.shuf_h + 2 * ho + (ij >> 1)) * p.shuf_w + 2 * wo + (ij & 1);
                o = (unsigned)(pix * co + cj[j]) * 4u;
            }
            orow[i][j] = o;
        }
    }
    f32x4 bv[FN][4];
    const __amdgpu_buffer_rsrc_t rb = epi_rsrc(p.bias, true);
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            bv[j][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rb, nc0 + j * 32 < p.N ? (unsigned)cj[j] * 4u : LEAN_OOB, 32 * q, 0));
    const __amdgpu_buffer_rsrc_t rd = epi_rsrc(p.dst0, true);
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                v += bv[j][q];
                if (relu) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rd, orow[i][j], 32 * q, 0);
            }
}

template <int BM, int BN, int WM, int WN, bool BATCH = false>
__device__ __forceinline__ void epilogue(const IgemmParams& p, f32x16 (&acc)[BM / WM / 32][BN / WN / 32], int m_blk,
                                         int n_blk, int wm, int wn, int lr, int lh) {
    constexpr int FM = BM / WM / 32;
    constexpr int FN = BN / WN / 32;
    if constexpr (BATCH && PU_EPI_BATCH) {
        // 32-column fragments never straddle n0; every destination byte offset fits 31 bits
        if (p.vec_epi && !(p.flags & (PU_EPI_SHUFFLE2 | PU_EPI_ACCUM)) && !p.resid && !p.cscale && p.n0 % 32 == 0 &&
            p.N % 32 == 0 && (long long)p.M * p.N < (1LL << 29)) {
            const int m0 = m_blk + wm * (BM / WM), nc0 = n_blk + wn * (BN / WN);
            if ((p.mask0 || p.mask1) && !p.bias) {
                epilogue_batched<true, FM, FN>(p, acc, m0, nc0, lr, lh);
                return;
            }
            if (!p.mask0 && !p.mask1 && p.bias) {
                epilogue_batched<false, FM, FN>(p, acc, m0, nc0, lr, lh);
                return;
            }
        }
        if (p.vec_epi && (p.flags & PU_EPI_SHUFFLE2) && !(p.flags & PU_EPI_ACCUM) && !p.resid && !p.cscale && p.bias &&
            !p.mask0 && p.shuf_off == 0 && p.shuf_h == 2 * p.Ho && p.shuf_w == 2 * p.Wo && (p.N / 4) % 32 == 0 &&
            p.N % 128 == 0 && (long long)p.M * p.N < (1LL << 29)) {
            epilogue_batched_shuf<FM, FN>(p, acc, m_blk + wm * (BM / WM), n_blk + wn * (BN / WN), lr, lh);
            return;
        }
    }
    // ---- epilogue.  acc[i][j] = D^T block: MFMA row = channel n = 8*(r>>2) + 4*(lane>>5) + (r&3),
    // column = pixel m = lane & 31.  Registers 4q..4q+3 are 4 consecutive channels of one pixel:
    // bias / ReLU / mask / accumulate / store run on float4 (16 B per lane).
    const bool relu = p.flags & PU_EPI_RELU;
    const bool accum = p.flags & PU_EPI_ACCUM;
    const bool shuffle = p.flags & PU_EPI_SHUFFLE2;
    const bool vec = p.vec_epi;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m_blk + wm * (BM / WM) + i * 32 + lr;
        if (m >= p.M) continue;
        const EpiRow er = epi_row(p, m);
        const long long pix = er.pix;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n_blk + wn * (BN / WN) + j * 32 + 8 * q + 4 * lh;
                if (n >= p.N) continue;
                if (vec) {
                    f32x4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                    epi_store4(p, er, n, v);
                } else {
                    // odd channel counts: per element (channel n+e may cross the n0 split)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int ne = n + e;
                        if (ne >= p.N) break;
                        float* d;
                        const float* mk;
                        long long o;
                        int bi = ne;
                        if (shuffle) {
                            if (!shuf_off(p, er, ne, &o, &bi)) continue;
                            d = p.dst0; mk = p.mask0;
                        } else if (ne < p.n0) {
                            o = pix * p.n0 + ne; d = p.dst0; mk = p.mask0;
                        } else {
                            o = pix * (p.N - p.n0) + (ne - p.n0); d = p.dst1; mk = p.mask1;
                        }
                        float v = acc[i][j][4 * q + e] + (p.bias ? p.bias[bi] : 0.f) + (p.resid ? p.resid[o] : 0.f);
                        if (relu) v = fmaxf(v, 0.f);
                        if (mk && !(mk[o] > 0.f)) v = 0.f;
                        if (p.cscale) v *= p.cscale[(long long)er.b * p.cs_ld + bi];
                        if (accum) v += d[o];
                        d[o] = v;
                    }
                }
            }
        }
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
    // XCD-aware tile order: each XCD walks a contiguous range of (m-block, all n-blocks)
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mb = tile / p.gn;
    const int m_blk = mb * BM;
    const int n_blk = (tile - mb * p.gn) * BN;

    // ---- loader mapping: lane -> row (lane & 15) + 16*wave (+ 64*i), 16-byte k-quad lane >> 4.
    // 8 consecutive lanes write one k-quad of 8 different rows (row stride 20 floats): the
    // ds_write_b128 lane groups touch 8 distinct 4-bank slots, so staging is conflict-free.
    const int kq = lane >> 4;
    const int lrow = (lane & 15) + 16 * wave;
    int pb[A_LD], hb[A_LD], wb[A_LD];
    long long rb0[A_LD], rb1[A_LD];   // element offset of the tap-(0,0) pixel in src0 / src1
    unsigned tmask[A_LD];             // bit (r*kw+s): that tap's input pixel lies inside the image
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
        int m = m_blk + lrow + 64 * i;
        pb[i] = 0; hb[i] = -(1 << 28); wb[i] = 0; tmask[i] = 0; rb0[i] = 0; rb1[i] = 0;
        if (m < p.M) {
            int t = fdiv(m, p.dWo);
            int wo = m - t * p.Wo;
            int b = fdiv(t, p.dHo);
            int ho = t - b * p.Ho;
            pb[i] = b * p.Hi * p.Wi;
            hb[i] = ho * p.stride - p.pad;
            wb[i] = wo * p.stride - p.pad;
            if (MODE == LOAD_CHUNK16) {
                long long pix0 = (long long)pb[i] + (long long)hb[i] * p.Wi + wb[i];
                rb0[i] = pix0 * p.c0;
                rb1[i] = pix0 * p.c1;
                unsigned msk = 0;
                for (int r = 0; r < p.kh; ++r)
                    for (int q = 0; q < p.kw; ++q)
                        if ((unsigned)(hb[i] + r) < (unsigned)p.Hi && (unsigned)(wb[i] + q) < (unsigned)p.Wi)
                            msk |= 1u << (r * p.kw + q);
                tmask[i] = msk;
            }
        }
    }
    const float* wrow[B_LD];
    bool wok[B_LD];
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
        int n = n_blk + lrow + 64 * i;
        wok[i] = n < p.N;
        wrow[i] = p.wt + (long long)(wok[i] ? n : 0) * p.k_pad + kq * 4;
    }

    f32x4 ra[A_LD], rb[B_LD];
    auto load_stage = [&](int t) {
        const int k0 = t * IG_BK;
        if (MODE == LOAD_CHUNK16) {
            // the whole 16-wide k chunk shares one tap and one source (c0, c1 multiples of 16):
            // tap/source/offset are wave-uniform, each row only tests its tap bit and adds its base
            int tap, c;
            if (p.cgroup) {
                // channel-group-major: stage t covers group g, tap, and 16-channel half h
                const int per = p.cgroup >> 4;                // stages per (group, tap)
                const int tg = per == 2 ? (t >> 1) : t;
                const int h = per == 2 ? (t & 1) : 0;
                const int g = fdiv(tg, p.dTaps);
                tap = tg - g * p.taps;
                c = g * p.cgroup + h * 16;
            } else {
                tap = fdiv(k0, p.dC);
                c = k0 - tap * p.C;
            }
            const int r = fdiv(tap, p.dKw);
            const int s = tap - r * p.kw;
            const bool first = c < p.c0;
            const float* src = first ? p.src0 : p.src1;
            const int cs = first ? p.c0 : p.c1;
            const long long off = (long long)(r * p.Wi + s) * cs + (first ? c : c - p.c0) + kq * 4;
            const unsigned bit = (k0 < p.K) ? (1u << tap) : 0u;
#pragma unroll
            for (int i = 0; i < A_LD; ++i) {
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (tmask[i] & bit) v = *reinterpret_cast<const f32x4*>(src + (first ? rb0[i] : rb1[i]) + off);
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
            *reinterpret_cast<f32x4*>(a + (lrow + 64 * i) * IG_LDS + kq * 4) = ra[i];
#pragma unroll
        for (int i = 0; i < B_LD; ++i)
            *reinterpret_cast<f32x4*>(b + (lrow + 64 * i) * IG_LDS + kq * 4) = rb[i];
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
                        // weights as the MFMA A operand, pixels as B: acc[i][j] holds D^T (rows =
                        // output channels), so each lane ends with 4 consecutive channels of a pixel
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[j][s], fa[i][s], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < T) store_stage(buf ^ 1);
        __syncthreads();
    }

    epilogue<BM, BN, WM, WN>(p, acc, m_blk, n_blk, wm, wn, lr, lh);
}

// ------------------------------------------------------------------------ direct-to-LDS variant
// For 16-channel-chunk loads (every conv with C % 16 == 0 - all but the 1-channel stem) the A and
// B tiles are fetched with global_load_lds_dwordx4: no VGPR staging, no ds_write, loads stay in
// flight across the barrier.  LDS image per stage: rows of 64 B (16 floats), unpadded; the
// 16-byte chunk kc of row r is stored at position kc ^ ((r >> 2) & 3) (XOR swizzle on the global
// SOURCE address, same XOR on the ds_read_b128 address) so the MFMA operand reads are
// conflict-free.  NBUF-deep ring with a counted s_waitcnt vmcnt and a raw s_barrier per stage.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
__device__ __attribute__((aligned(16))) float g_zero16[4];

template <int BM, int BN, int WM, int WN, int NBUF>
__global__ __launch_bounds__(256) void igemm_dma_kernel(const IgemmParams p) {
    constexpr int FM = BM / WM / 32;
    constexpr int FN = BN / WN / 32;
    constexpr int A_LD = BM / 64;   // glds per wave per stage (16 rows x 64 B each)
    constexpr int B_LD = BN / 64;
    constexpr int G = A_LD + B_LD;
    constexpr int STAGE = (BM + BN) * 16;   // floats per ring slot
    static_assert(WM * WN == 4, "4 waves");

    __shared__ __attribute__((aligned(16))) float lds[NBUF * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int lr = lane & 31, lh = lane >> 5;
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kz = tile / (gridDim.x / p.ksplit);   // K split (outermost: a split's blocks share its weight slice)
    tile -= kz * (gridDim.x / p.ksplit);
    const int mb = tile / p.gn;
    const int m_blk = mb * BM;
    const int n_blk = (tile - mb * p.gn) * BN;

    // loader: instruction j of this wave covers tile rows wave*(BM/4) + 16j + (lane >> 2);
    // lane stores LDS position (lane & 3) of its row, i.e. logical chunk kc (the swizzle only
    // depends on lane bits because the row bases are multiples of 16)
    const int lq = lane >> 2;
    const int kc = (lane & 3) ^ ((lane >> 4) & 3);
    long long rb0[A_LD], rb1[A_LD];
    unsigned tmask[A_LD];
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
        const int m = m_blk + wave * (BM / 4) + 16 * j + lq;
        rb0[j] = 0; rb1[j] = 0; tmask[j] = 0;
        if (m < p.M) {
            const int t = fdiv(m, p.dWo);
            const int wo = m - t * p.Wo;
            const int b = fdiv(t, p.dHo);
            const int ho = t - b * p.Ho;
            const int hb = ho * p.stride - p.pad, wb = wo * p.stride - p.pad;
            const long long pix0 = (long long)b * p.Hi * p.Wi + (long long)hb * p.Wi + wb;
            rb0[j] = pix0 * p.c0 + kc * 4;
            rb1[j] = pix0 * p.c1 + kc * 4;
            unsigned msk = 0;
            for (int r = 0; r < p.kh; ++r)
                for (int q = 0; q < p.kw; ++q)
                    if ((unsigned)(hb + r) < (unsigned)p.Hi && (unsigned)(wb + q) < (unsigned)p.Wi)
                        msk |= 1u << (r * p.kw + q);
            tmask[j] = msk;
        }
    }
    const float* wrow[B_LD];
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
        const int n = n_blk + wave * (BN / 4) + 16 * j + lq;
        wrow[j] = n < p.N ? p.wt + (long long)n * p.k_pad + kc * 4 : nullptr;
    }

    const int t0 = kz * p.t_per;
    const int T = min(p.k_pad / IG_BK - t0, p.t_per);
    // issue(tl): loads of local stage tl into ring slot `slot`.  Branch-free (selects only) so the
    // main loop stays one basic block; stages tl >= T load the zero page (never read).
    auto issue = [&](int tl, int slot) {
        const bool live = tl < T;
        const int t = t0 + (live ? tl : 0);
        const int k0 = t * IG_BK;
        const bool two = p.cgroup == 32;
        const int tg = two ? (t >> 1) : t;
        const int g = fdiv(tg, p.dTaps);
        const int tap_n = fdiv(k0, p.dC);
        const int tap = p.cgroup ? tg - g * p.taps : tap_n;
        const int c = p.cgroup ? g * p.cgroup + (two ? (t & 1) * 16 : 0) : k0 - tap_n * p.C;
        const int r = fdiv(tap, p.dKw);
        const int s = tap - r * p.kw;
        const bool first = c < p.c0;
        const float* src = first ? p.src0 : p.src1;
        const int cs = first ? p.c0 : p.c1;
        const long long off = (long long)(r * p.Wi + s) * cs + (first ? c : c - p.c0);
        const unsigned bit = (live && k0 < p.K) ? (1u << tap) : 0u;
        float* a_slot = lds + slot * STAGE;
        float* b_slot = a_slot + BM * 16;
#pragma unroll
        for (int j = 0; j < A_LD; ++j) {
            const float* g = (tmask[j] & bit) ? src + (first ? rb0[j] : rb1[j]) + off : g_zero16;
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(a_slot + (wave * (BM / 4) + 16 * j) * 16),
                                             16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < B_LD; ++j) {
            const float* g = (live && wrow[j]) ? wrow[j] + k0 : g_zero16;
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(b_slot + (wave * (BN / 4) + 16 * j) * 16),
                                             16, 0, 0);
        }
    };

    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int a_row0 = wm * (BM / WM) + lr;
    const int b_row0 = wn * (BN / WN) + lr;
    const int swz = (lr >> 2) & 3;   // ((row >> 2) & 3) of every row this lane reads

#pragma unroll
    for (int s0 = 0; s0 < NBUF - 1; ++s0) issue(s0, s0);

    for (int t = 0; t < T; ++t) {
        // stage t has landed (own loads) when at most the younger stages' G loads are pending
        // (every iteration issues one stage, past the end too, so the count is constant)
        if (NBUF == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G) : "memory");
        __builtin_amdgcn_s_barrier();   // everyone's stage-t loads landed; slot (t-1) is free
        const float* a = lds + (t % NBUF) * STAGE;
        const float* b = a + BM * 16;
        // both k-halves' operands up front (the second half's reads land under the first
        // half's MFMAs); the next stage's loads are issued between the halves so their address
        // arithmetic overlaps MFMA execution instead of delaying the first MFMA of the stage
        f32x4 fa[2][FM], fb[2][FN];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int pos = ((kk * 2 + lh) ^ swz) * 4;
#pragma unroll
            for (int i = 0; i < FM; ++i) fa[kk][i] = *reinterpret_cast<const f32x4*>(a + (a_row0 + i * 32) * 16 + pos);
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[kk][j] = *reinterpret_cast<const f32x4*>(b + (b_row0 + j * 32) * 16 + pos);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[kk][j][s], fa[kk][i][s], acc[i][j], 0, 0, 0);
            if (kk == 0) issue(t + NBUF - 1, (t + NBUF - 1) % NBUF);
        }
        // keep all operand reads ahead of the MFMAs (the default scheduler sinks the second
        // half's reads behind the first half's MFMAs, exposing their latency)
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * (FM + FN), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8 * FM * FN, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain the past-the-end zero-page loads
    if (p.ksplit == 1) {
        epilogue<BM, BN, WM, WN>(p, acc, m_blk, n_blk, wm, wn, lr, lh);
        return;
    }
    // split-K: raw partial tile -> part[kz][m][n] (float4 over 4 consecutive n; N % 4 == 0)
    float* part = p.part + (long long)kz * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m_blk + wm * (BM / WM) + i * 32 + lr;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n_blk + wn * (BN / WN) + j * 32 + 8 * q + 4 * lh;
                if (n >= p.N) continue;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                *reinterpret_cast<f32x4*>(part + (long long)m * p.N + n) = v;
            }
    }
}

// ------------------------------------------------------------- fp32 GEMM as 6 bf16 MFMA products
// gfx950 has one fp32 matrix op, v_mfma_f32_32x32x2_f32 (64 cycles per 32x32x2), 1/16 of the bf16
// rate.  An fp32 value splits EXACTLY into three bf16 terms x = x_hi + x_mid + x_lo (round to
// nearest at each step: |x_mid| <= 2^-8 |x|, |x_lo| <= 2^-16 |x|, and the last residual has at
// most 8 significant bits), so
//   x*y = x_hi y_hi + (x_hi y_mid + x_mid y_hi) + (x_hi y_lo + x_lo y_hi + x_mid y_mid) + O(2^-24 xy)
// takes 6 v_mfma_f32_32x32x16_bf16 (exact bf16 products, fp32 accumulation) per 16 k: 192
// cycles against the 512 of eight f32 MFMAs - the fp32 path on the bf16 pipe, with the error of
// an fp32 product (the dropped terms are below 2^-23 relative).
// Weights come pre-split (pu_split_weight6: [k/16][q = plane*2 + half][n][8 bf16]); pixel rows
// are staged as fp32 exactly like igemm_dma_kernel and split after the LDS read (VALU work that
// co-issues with the MFMAs).  Same loader, ring, swizzle, epilogue and split-K as the fp32 kernel.

__device__ __forceinline__ void split3_bf16(const f32x4 lo4, const f32x4 hi4, bf16x8_t& h, bf16x8_t& m, bf16x8_t& l) {
#pragma clang fp contract(off)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float x = e < 4 ? lo4[e] : hi4[e - 4];
        const __bf16 a = (__bf16)x;
        const float r = x - (float)a;
        const __bf16 b = (__bf16)r;
        const float q = r - (float)b;
        h[e] = a;
        m[e] = b;
        l[e] = (__bf16)q;
    }
}

// 3-deep ring of 16-k stages, one barrier per stage; the loads of stage t+2 are issued after the
// first pixel fragment's MFMAs of stage t (they then overlap the rest of the stage).
template <int BM, int BN, int WM, int WN, int NW = 4>
__global__ __launch_bounds__(NW * 64) void igemm_x6_kernel(const IgemmParams p) {
    constexpr int NBUF = 3;
    constexpr int FM = BM / WM / 32;
    constexpr int FN = BN / WN / 32;
    constexpr int A_LD = BM / (16 * NW);      // pixel rows: glds per wave per stage (16 rows x 64 B)
    constexpr int W_TOT = 6 * BN / 64;        // weight planes: glds per block per stage (64 x 16 B)
    constexpr int W_LD = (W_TOT + NW - 1) / NW;   // per wave (surplus ones load the zero page into a sink)
    constexpr bool SINK = (W_TOT % NW) != 0;
    constexpr int G = A_LD + W_LD;            // loads per wave per ring slot
    constexpr int A_FL = BM * 16;             // floats of one stage's pixel image
    constexpr int W_FL = BN * 6 * 4;          // float-sized slots of one stage's weight planes
    constexpr int STAGE = A_FL + W_FL;
    static_assert(WM * WN == NW && A_LD >= 1, "wave grid");

    __shared__ __attribute__((aligned(16))) float lds[NBUF * STAGE + (SINK ? 256 : 0)];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int lr = lane & 31, lh = lane >> 5;
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kz = tile / (gridDim.x / p.ksplit);
    tile -= kz * (gridDim.x / p.ksplit);
    const int mb = tile / p.gn;
    const int m_blk = mb * BM;
    const int n_blk = (tile - mb * p.gn) * BN;

    const int lq = lane >> 2;
    const int kc = (lane & 3) ^ ((lane >> 4) & 3);
    long long rb0[A_LD], rb1[A_LD];
    unsigned tmask[A_LD];
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
        const int m = m_blk + wave * (BM / NW) + 16 * j + lq;
        rb0[j] = 0; rb1[j] = 0; tmask[j] = 0;
        if (m < p.M) {
            const int t = fdiv(m, p.dWo);
            const int wo = m - t * p.Wo;
            const int b = fdiv(t, p.dHo);
            const int ho = t - b * p.Ho;
            const int hb = ho * p.stride - p.pad, wb = wo * p.stride - p.pad;
            const long long pix0 = (long long)b * p.Hi * p.Wi + (long long)hb * p.Wi + wb;
            rb0[j] = pix0 * p.c0 + kc * 4;
            rb1[j] = pix0 * p.c1 + kc * 4;
            unsigned msk = 0;
            for (int r = 0; r < p.kh; ++r)
                for (int q = 0; q < p.kw; ++q)
                    if ((unsigned)(hb + r) < (unsigned)p.Hi && (unsigned)(wb + q) < (unsigned)p.Wi)
                        msk |= 1u << (r * p.kw + q);
            tmask[j] = msk;
        }
    }
    // weight-plane loads: block instruction I = wave + 4j covers entries [64 I, 64 I + 64) of the
    // stage's [q][BN] image (one plane-half q, contiguous rows -> one coalesced 1 KB read)
    const __bf16* w6 = reinterpret_cast<const __bf16*>(p.wt);
    const __bf16* wrow[W_LD];
#pragma unroll
    for (int j = 0; j < W_LD; ++j) {
        const int I = wave + NW * j;
        const int e = I * 64 + lane;
        const int q = e / BN, row = e - q * BN;
        const int n = n_blk + row;
        wrow[j] = (I < W_TOT && n < p.N) ? w6 + ((long long)q * p.N + n) * 8 : nullptr;
    }
    const long long w_stage = 6LL * p.N * 8;   // bf16 elements per 16-k stage

    const int t0 = kz * p.t_per;
    const int T = min(p.k_pad / IG_BK - t0, p.t_per);     // 16-k stages of this split
    auto issue = [&](int tl, int slot) {
        float* a_slot = lds + slot * STAGE;
        const bool live = tl < T;
        const int t = t0 + (live ? tl : 0);
        const int k0 = t * IG_BK;
        const bool two = p.cgroup == 32;
        const int tg = two ? (t >> 1) : t;
        const int g = fdiv(tg, p.dTaps);
        const int tap_n = fdiv(k0, p.dC);
        const int tap = p.cgroup ? tg - g * p.taps : tap_n;
        const int c = p.cgroup ? g * p.cgroup + (two ? (t & 1) * 16 : 0) : k0 - tap_n * p.C;
        const int r = fdiv(tap, p.dKw);
        const int s = tap - r * p.kw;
        const bool first = c < p.c0;
        const float* src = first ? p.src0 : p.src1;
        const int cs = first ? p.c0 : p.c1;
        const long long off = (long long)(r * p.Wi + s) * cs + (first ? c : c - p.c0);
        const unsigned bit = (live && k0 < p.K) ? (1u << tap) : 0u;
        const long long wo = (long long)t * w_stage;
        float* w_slot = a_slot + A_FL;
#pragma unroll
        for (int j = 0; j < A_LD; ++j) {
            const float* g = (tmask[j] & bit) ? src + (first ? rb0[j] : rb1[j]) + off : g_zero16;
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(a_slot + (wave * (BM / NW) + 16 * j) * 16),
                                             16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < W_LD; ++j) {
            const int I = wave + NW * j;
            const void* g = (live && wrow[j]) ? (const void*)(wrow[j] + wo) : (const void*)g_zero16;
            float* dst = (!SINK || I < W_TOT) ? w_slot + I * 256 : lds + NBUF * STAGE;   // 64 lanes x 16 B
            __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)dst, 16, 0, 0);
        }
    };

    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int a_row0 = wm * (BM / WM) + lr;
    const int b_row0 = wn * (BN / WN) + lr;
    const int swz = (lr >> 2) & 3;
    const int pos0 = ((2 * lh) ^ swz) * 4, pos1 = ((2 * lh + 1) ^ swz) * 4;

#pragma unroll
    for (int s0 = 0; s0 < NBUF - 1; ++s0) issue(s0, s0);

    for (int ts = 0; ts < T; ++ts) {
        // ring slot ts landed when only the younger slot's loads are pending
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const float* a = lds + (ts % NBUF) * STAGE;
        const float* wp = a + A_FL;
        f32x4 xa[FM], xb[FM];
        bf16x8_t fw[3][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            xa[i] = *reinterpret_cast<const f32x4*>(a + (a_row0 + i * 32) * 16 + pos0);
            xb[i] = *reinterpret_cast<const f32x4*>(a + (a_row0 + i * 32) * 16 + pos1);
        }
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int j = 0; j < FN; ++j)
                fw[pl][j] = *reinterpret_cast<const bf16x8_t*>(wp + ((pl * 2 + lh) * BN + b_row0 + j * 32) * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            bf16x8_t xh, xm, xl;
            split3_bf16(xa[i], xb[i], xh, xm, xl);
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                f32x16 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[1][j], xm, c, 0, 0, 0);   // small terms first
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[2][j], xh, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[0][j], xl, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[1][j], xh, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[0][j], xm, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[0][j], xh, c, 0, 0, 0);
                acc[i][j] = c;
            }
            if (i == 0) issue(ts + NBUF - 1, (ts + NBUF - 1) % NBUF);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (p.ksplit == 1) {
        epilogue<BM, BN, WM, WN, true>(p, acc, m_blk, n_blk, wm, wn, lr, lh);
        return;
    }
    float* part = p.part + (long long)kz * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m_blk + wm * (BM / WM) + i * 32 + lr;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n_blk + wn * (BN / WN) + j * 32 + 8 * q + 4 * lh;
                if (n >= p.N) continue;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                *reinterpret_cast<f32x4*>(part + (long long)m * p.N + n) = v;
            }
    }
}

// ---------------------------------------------------------------- lean 6-product kernel
// The same GEMM, tiles, LDS images, MFMA sequence and epilogue as igemm_x6_kernel, re-shaped to
// issue few instructions per K stage (PMC on the top 64-channel layer: ~130 VALU + ~95 SALU per
// 24 MFMAs per wave - the waves were issue-bound, MFMA busy 0.43):
//   * loads are buffer_load ... lds through buffer descriptors: per-lane byte offsets are
//     precomputed once per block for every tap (an out-of-image tap gets an out-of-range offset:
//     the range check writes zeros into LDS - probed, tools/probes/oob_lds.hip), the stage's
//     (tap, channel) offset is one scalar soffset;
//   * the 9 taps x CG channel halves of a channel group are unrolled, so the tap, the ring slot
//     and every LDS address are compile-time constants;
//   * the 3-term split is written pair-wise (v_cvt_pk_bf16_f32 + v_pk_add_f32: 4.5 VALU/element).
// Requirements (host: lean_ok): 3x3 taps, K order cgroup 16 (CG 1) or 32 (CG 2), c1 == 0 or
// c1 == c0 (one pixel stride for both sources), K == k_pad, split-K on group boundaries,
// every tensor under 2 GB.

template <int BM, int BN, int WM, int WN, int NW, int CG>
__global__ __launch_bounds__(NW * 64) void igemm_x6_lean_kernel(const IgemmParams p) {
    constexpr int FM = BM / WM / 32;
    constexpr int FN = BN / WN / 32;
    constexpr int A_LD = BM / (16 * NW);
    constexpr int W_TOT = 6 * BN / 64;
    constexpr int W_LD = (W_TOT + NW - 1) / NW;
    constexpr bool SINK = (W_TOT % NW) != 0;
    constexpr int G = A_LD + W_LD;
    constexpr int A_FL = BM * 16;
    constexpr int W_FL = BN * 6 * 4;
    constexpr int STAGE = A_FL + W_FL;
    constexpr int SPG = 9 * CG;               // stages per channel group (taps x 16-channel halves)
    static_assert(WM * WN == NW && A_LD >= 1 && SPG % 3 == 0, "lean tile");

    __shared__ __attribute__((aligned(16))) float lds[3 * STAGE + (SINK ? 256 : 0)];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int lr = lane & 31, lh = lane >> 5;
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kz = tile / (gridDim.x / p.ksplit);
    tile -= kz * (gridDim.x / p.ksplit);
    const int mb = tile / p.gn;
    const int m_blk = mb * BM;
    const int n_blk = (tile - mb * p.gn) * BN;

    // pixel operand: shifted base so every in-image source offset is >= 0
    const int cs = p.c0;                                      // == c1 when c1 != 0
    const int shift = p.pad * p.Wi + p.pad;
    const unsigned a_bytes0 = (unsigned)(((long long)p.in_pix + shift) * cs * 4);
    const float* a0p = p.src0 - (long long)shift * cs;
    const float* a1p = (p.c1 ? p.src1 : p.src0) - (long long)shift * cs;
    const unsigned w_bytes = (unsigned)((long long)p.k_pad * p.N * 12);

    const int lq = lane >> 2;
    const int kc = (lane & 3) ^ ((lane >> 4) & 3);
    unsigned vo[A_LD][9];
#pragma unroll
    for (int j = 0; j < A_LD; ++j) {
        const int m = m_blk + wave * (BM / NW) + 16 * j + lq;
        int hb = 0, wb = 0, pix = 0;
        const bool mv = m < p.M;
        if (mv) {
            const int t = fdiv(m, p.dWo);
            const int wo = m - t * p.Wo;
            const int b = fdiv(t, p.dHo);
            const int ho = t - b * p.Ho;
            hb = ho * p.stride - p.pad;
            wb = wo * p.stride - p.pad;
            pix = (b * p.Hi + hb) * p.Wi + wb + shift;
        }
        const unsigned base = (unsigned)pix * (unsigned)(cs * 4) + kc * 16;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const bool ok = mv && (unsigned)(hb + r) < (unsigned)p.Hi && (unsigned)(wb + q) < (unsigned)p.Wi;
                vo[j][r * 3 + q] = ok ? base : LEAN_OOB;
            }
    }
    unsigned tapoff[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) tapoff[r * 3 + q] = (unsigned)((r * p.Wi + q) * cs * 4);
    unsigned wv[W_LD];
#pragma unroll
    for (int j = 0; j < W_LD; ++j) {
        const int I = wave + NW * j;
        const int e = I * 64 + lane;
        const int q = e / BN, row = e - q * BN;
        const int n = n_blk + row;
        wv[j] = (I < W_TOT && n < p.N) ? (unsigned)((q * p.N + n) * 16) : LEAN_OOB;
    }
    const unsigned w_stage = (unsigned)p.N * 96u;   // bytes of one 16-k stage's six planes

    const int groups = p.k_pad / (16 * SPG);
    const int gps = p.t_per / SPG;                  // groups per split
    const int g0 = kz * gps;
    const int g1 = min(groups, g0 + gps);

    // loads of stage u (compile-time position in its group) of group g into ring slot u % 3
    auto issue = [&](int g, auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int tap = u / CG, h = u % CG;
        const bool live = g < g1;
        const int c = g * (16 * CG) + h * 16;                     // K-order channel of this stage
        const bool second = c >= p.c0;
        const float* abase = second ? a1p : a0p;
        const unsigned abytes = live ? a_bytes0 : 0u;
        const unsigned soff = tapoff[tap] + (unsigned)((second ? c - p.c0 : c) * 4);
        float* a_slot = lds + (u % 3) * STAGE;
#pragma unroll
        for (int j = 0; j < A_LD; ++j)
            lean_load(abase, abytes, a_slot + (wave * (BM / NW) + 16 * j) * 16, vo[j][tap], soff);
        const unsigned wbytes = live ? w_bytes : 0u;
        const unsigned wsoff = (unsigned)(g * SPG + u) * w_stage;
        float* w_slot = a_slot + A_FL;
#pragma unroll
        for (int j = 0; j < W_LD; ++j) {
            const int I = wave + NW * j;
            float* dst = (!SINK || I < W_TOT) ? w_slot + I * 256 : lds + 3 * STAGE;
            lean_load(p.wt, wbytes, dst, wv[j], wsoff);
        }
    };

    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int a_row0 = wm * (BM / WM) + lr;
    const int b_row0 = wn * (BN / WN) + lr;
    const int swz = (lr >> 2) & 3;
    const int pos0 = ((2 * lh) ^ swz) * 4, pos1 = ((2 * lh + 1) ^ swz) * 4;

    if (g0 < g1) {
        issue(g0, std::integral_constant<int, 0>{});
        issue(g0, std::integral_constant<int, 1>{});
    }
    for (int g = g0; g < g1; ++g) {
        static_for<SPG>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const float* a = lds + (u % 3) * STAGE;
            const float* wp = a + A_FL;
            f32x4 xa[FM], xb[FM];
            bf16x8_t fw[3][FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                xa[i] = *reinterpret_cast<const f32x4*>(a + (a_row0 + i * 32) * 16 + pos0);
                xb[i] = *reinterpret_cast<const f32x4*>(a + (a_row0 + i * 32) * 16 + pos1);
            }
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    fw[pl][j] = *reinterpret_cast<const bf16x8_t*>(wp + ((pl * 2 + lh) * BN + b_row0 + j * 32) * 4);
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                bf16x8_t xh, xm, xl;
                split3_pairs(xa[i], xb[i], xh, xm, xl);
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    f32x16 c = acc[i][j];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[1][j], xm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[2][j], xh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[0][j], xl, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[1][j], xh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[0][j], xm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[0][j], xh, c, 0, 0, 0);
                    acc[i][j] = c;
                }
                if (i == 0) {
                    if constexpr (u + 2 < SPG) issue(g, std::integral_constant<int, u + 2>{});
                    else issue(g + 1, std::integral_constant<int, u + 2 - SPG>{});
                }
            }
        });
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (p.ksplit == 1) {
        epilogue<BM, BN, WM, WN, true>(p, acc, m_blk, n_blk, wm, wn, lr, lh);
        return;
    }
    float* part = p.part + (long long)kz * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m_blk + wm * (BM / WM) + i * 32 + lr;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n_blk + wn * (BN / WN) + j * 32 + 8 * q + 4 * lh;
                if (n >= p.N) continue;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                *reinterpret_cast<f32x4*>(part + (long long)m * p.N + n) = v;
            }
    }
}

// packed fp32 weight [n][k_pad] -> [k_pad/16][q][n][8] bf16 planes, q = plane*2 + (k%16)/8,
// plane 0/1/2 = hi/mid/lo of the round-to-nearest split (exact: hi + mid + lo == w)
__global__ void split_weight6_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int n, int k_pad) {
#pragma clang fp contract(off)
    const long long total = (long long)n * k_pad;
    for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
        const int row = (int)(idx / k_pad);
        const int k = (int)(idx - (long long)row * k_pad);
        const float x = w[idx];
        const __bf16 a = (__bf16)x;
        const float r = x - (float)a;
        const __bf16 b = (__bf16)r;
        const __bf16 c = (__bf16)(r - (float)b);
        const int t = k >> 4, half = (k >> 3) & 1, e = k & 7;
        const __bf16 v[3] = {a, b, c};
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
            out[(((long long)t * 6 + pl * 2 + half) * n + row) * 8 + e] = v[pl];
    }
}

// split-K second pass: sum the partial tiles in split order (deterministic) + the fused epilogue
__global__ __launch_bounds__(256) void igemm_splitk_epilogue_kernel(const IgemmParams p) {
    const int nq = p.N >> 2;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)p.M * nq) return;
    const int m = (int)(idx / nq);
    const int n = (int)(idx - (long long)m * nq) * 4;
    const long long mn = (long long)p.M * p.N;
    const float* src = p.part + (long long)m * p.N + n;
    f32x4 v = *reinterpret_cast<const f32x4*>(src);
    for (int z = 1; z < p.ksplit; ++z) v += *reinterpret_cast<const f32x4*>(src + z * mn);
    epi_store4(p, epi_row(p, m), n, v);
}

// ---------------------------------------------------------------- small-channel direct conv
// For 3x3/s1/p1 convolutions with C <= 16 input and N <= 16 output channels (the 8/16-channel
// levels of configs C4/C5) a GEMM tile is mostly padding: N = 8 fills 1/8 of a 64-wide MFMA
// tile and K = 72 leaves the per-block setup dominant.  These layers are HBM-bound (~18-36
// FLOP/B), so they run as a direct convolution on the VALU: a block stages the (16+2) x (32+2)
// input halo of a 16 x 32 output tile in LDS (both concat sources, zero padding), each thread
// computes 2 adjacent pixels x all N channels with fmaf chains over (tap, channel) - the same
// k order as the MFMA path - reading the packed weight rows with wave-uniform (scalar) loads, and
// the float4 epilogue above applies bias / residual / ReLU / mask / split / accumulate.
constexpr int SC_TH = 16, SC_TW = 32;

template <int C, int N, int KP = (9 * C + 15) / 16 * 16>
__global__ __launch_bounds__(256) void smallconv_kernel(const IgemmParams p) {
    constexpr int HH = SC_TH + 2, HWD = SC_TW + 2;
    constexpr int CP = (C + 3) & ~3;     // LDS channel stride (float4 reads when C % 4 == 0)
    __shared__ __attribute__((aligned(16))) float tile[HH * HWD * CP];
    const int tiles_w = (p.Wo + SC_TW - 1) / SC_TW;
    const int tiles_h = (p.Ho + SC_TH - 1) / SC_TH;
    int blk = blockIdx.x;
    const int txi = blk % tiles_w;
    blk /= tiles_w;
    const int tyi = blk % tiles_h;
    const int b = blk / tiles_h;
    const int y0 = tyi * SC_TH - 1, x0 = txi * SC_TW - 1;   // halo origin (pad 1)
    const long long img = (long long)b * p.Hi * p.Wi;

    // stage the halo: element (hy, hx, c) from src0 (c < c0) or src1
    if (C % 4 == 0 && p.c0 % 4 == 0) {
        // every float4 of the halo a thread stages is loaded before any is stored (one round trip
        // per block instead of one per float4: 5 for C = 8, 10 for C = 16)
        constexpr int Q = C / 4 > 0 ? C / 4 : 1;     // (C == 1 never takes this branch)
        constexpr int NE = HH * HWD * Q;
        constexpr int PT = (NE + 255) / 256;
        f32x4 v[PT];
#pragma unroll
        for (int it = 0; it < PT; ++it) {
            const int e = it * 256 + threadIdx.x;
            const int q = e % Q, pix = e / Q;
            const int hx = pix % HWD, hy = pix / HWD;
            const int gy = y0 + hy, gx = x0 + hx;
            v[it] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (e < NE && (unsigned)gy < (unsigned)p.Hi && (unsigned)gx < (unsigned)p.Wi) {
                const long long px = img + (long long)gy * p.Wi + gx;
                const int c = 4 * q;
                v[it] = c < p.c0 ? *reinterpret_cast<const f32x4*>(p.src0 + px * p.c0 + c)
                                 : *reinterpret_cast<const f32x4*>(p.src1 + px * p.c1 + (c - p.c0));
            }
        }
#pragma unroll
        for (int it = 0; it < PT; ++it) {
            const int e = it * 256 + threadIdx.x;
            if (e < NE) *reinterpret_cast<f32x4*>(tile + (e / Q) * CP + 4 * (e % Q)) = v[it];
        }
    } else {
        for (int e = threadIdx.x; e < HH * HWD * CP; e += 256) {
            const int c = e % CP, pix = e / CP;
            const int hx = pix % HWD, hy = pix / HWD;
            const int gy = y0 + hy, gx = x0 + hx;
            float v = 0.f;
            if (c < C && (unsigned)gy < (unsigned)p.Hi && (unsigned)gx < (unsigned)p.Wi) {
                const long long px = img + (long long)gy * p.Wi + gx;
                v = c < p.c0 ? p.src0[px * p.c0 + c] : p.src1[px * p.c1 + (c - p.c0)];
            }
            tile[pix * CP + c] = v;
        }
    }
    __syncthreads();

    const int row = threadIdx.x / (SC_TW / 2);
    const int col = (threadIdx.x % (SC_TW / 2)) * 2;
    // accumulators packed over the thread's two pixels: one v_pk_fma_f32 per (channel, k) with the
    // activation pair {x(col), x(col+1)} and the weight broadcast from a scalar register; the
    // weight rows are KP floats apart (compile time), so the scalar loads take immediate offsets
    // and need no scalar address arithmetic per step (the fmaf form spent ~50 SALU per step)
    f32x2 acc[N];
#pragma unroll
    for (int n = 0; n < N; ++n) acc[n] = f32x2{0.f, 0.f};
    constexpr int Q4 = CP / 4;
#pragma unroll 1
    for (int step = 0; step < 9 * Q4; ++step) {
        const int tap = step / Q4, c4 = (step - tap * Q4) * 4;
        const int r = tap / 3, sx = tap - r * 3;
        const float* t0 = tile + ((row + r) * HWD + col + sx) * CP + c4;
        const float* wt = p.wt + (C % 4 == 0 ? 4 * step : step);   // tap * C + c4 (C % 4 == 0, or C == 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (e >= C) break;
            const f32x2 a = {t0[e], t0[CP + e]};
#pragma unroll
            for (int n = 0; n < N; ++n) {
                const float w = wt[n * KP + e];
                acc[n] = __builtin_elementwise_fma(a, f32x2{w, w}, acc[n]);
            }
        }
    }
    const int oy = tyi * SC_TH + row, ox = txi * SC_TW + col;
    if (oy >= p.Ho) return;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        if (ox + q >= p.Wo) break;
        const int m = (b * p.Ho + oy) * p.Wo + ox + q;
        const EpiRow er = epi_row(p, m);
#pragma unroll
        for (int n = 0; n < N; n += 4) {
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[n + e][q];
            epi_store4(p, er, n, v);
        }
    }
}


// 1x1 convolution with few channels (the CoordConv stem: AddCoords' 4 channels -> base_ch,
// coord_conv_script.py:61-85): one thread per pixel, its C input channels as float4 loads, N
// outputs as an fma chain over c in order (weights [n][k_pad] from the scalar cache), the shared
// float4 epilogue.  HBM-bound: (C + N) * 4 bytes per pixel; the MFMA tile path pads K to 16 and
// N to 64 (1/32 of the tile used).
template <int C, int N>
__global__ __launch_bounds__(256) void conv1x1_small_kernel(const IgemmParams p) {
    for (long long m = blockIdx.x * 256LL + threadIdx.x; m < p.M; m += (long long)gridDim.x * 256) {
        float x[C];
#pragma unroll
        for (int c = 0; c < C; c += 4) {
            const f32x4 v = c < p.c0 ? *reinterpret_cast<const f32x4*>(p.src0 + m * p.c0 + c)
                                     : *reinterpret_cast<const f32x4*>(p.src1 + m * p.c1 + (c - p.c0));
#pragma unroll
            for (int e = 0; e < 4; ++e) x[c + e] = v[e];
        }
        const EpiRow er = epi_row(p, (int)m);
#pragma unroll
        for (int n = 0; n < N; n += 4) {
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float* w = p.wt + (n + e) * p.k_pad;
                float acc = x[0] * w[0];
#pragma unroll
                for (int c = 1; c < C; ++c) acc = fmaf(x[c], w[c], acc);
                v[e] = acc;
            }
            epi_store4(p, er, n, v);
        }
    }
}

// ---------------------------------------------------------------- single-channel stem (C = 1)
// The first 3x3 conv (inc.c0: 1 -> N channels, N in {8, 16, 32, 64}; unet_p.py:208-215, the
// 8/16-channel stems of C4/C5) is a K = 9 GEMM: nothing for
// an MFMA tile to do, the layer is the write of its N-channel output.  A block stages the 1-channel
// halo of a 16 x 64 pixel tile in LDS; lanes work in groups of L = N/4 per pixel, each lane 4
// output channels (36 weights in registers), so every wave-instruction of the shared float4
// epilogue (bias, ReLU, masks, ...) stores 4 pixels x N channels contiguously.
constexpr int ST_TH = 16, ST_TW = 64;

// BF16OUT (PU_EPI_OUT_BF16): bias + ReLU, then one round-to-nearest-even to bf16 and an 8-byte store
// into a bf16 NHWC dst0 (the bf16 trunk's stem: no separate fp32 tensor and conversion pass)
template <int N, bool BF16OUT = false>
__global__ __launch_bounds__(256) void stem_conv_kernel(const IgemmParams p) {
    constexpr int L = N / 4;                  // lanes per pixel
    constexpr int PG = 256 / L;               // pixels per block pass
    constexpr int HH = ST_TH + 2, HW = ST_TW + 2;
    __shared__ float tile[HH * HW];
    const int tiles_w = (p.Wo + ST_TW - 1) / ST_TW;
    const int tiles_h = (p.Ho + ST_TH - 1) / ST_TH;
    int blk = blockIdx.x;
    const int txi = blk % tiles_w;
    blk /= tiles_w;
    const int tyi = blk % tiles_h;
    const int b = blk / tiles_h;
    const int y0 = tyi * ST_TH - 1, x0 = txi * ST_TW - 1;
    const long long img = (long long)b * p.Hi * p.Wi;
    for (int e = threadIdx.x; e < HH * HW; e += 256) {
        const int hy = e / HW, hx = e - hy * HW;
        const int gy = y0 + hy, gx = x0 + hx;
        tile[e] = ((unsigned)gy < (unsigned)p.Hi && (unsigned)gx < (unsigned)p.Wi) ? p.src0[img + (long long)gy * p.Wi + gx]
                                                                                  : 0.f;
    }
    const int lane_c = threadIdx.x % L;       // channels 4 lane_c .. 4 lane_c + 3
    float w[9][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t][e] = p.wt[(long long)(4 * lane_c + e) * p.k_pad + t];
    // bias (+ReLU) into one destination, the forward's form: the bias loaded once, ahead of the
    // stores (epi_store4 reloads it per pixel, after the previous pixel's store - and vmcnt counts
    // that store too)
    const bool plain = !(p.flags & (PU_EPI_SHUFFLE2 | PU_EPI_ACCUM)) && !p.mask0 && !p.resid && !p.cscale && p.n0 == N;
    const f32x4 bias4 = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + 4 * lane_c) : f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    for (int q = threadIdx.x / L; q < ST_TH * ST_TW; q += PG) {
        const int row = q / ST_TW, col = q - row * ST_TW;
        const int oy = tyi * ST_TH + row, ox = txi * ST_TW + col;
        if (oy >= p.Ho || ox >= p.Wo) continue;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const float a = tile[(row + t / 3) * HW + col + t % 3];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaf(a, w[t][e], v[e]);
        }
        const int m = (b * p.Ho + oy) * p.Wo + ox;
        if constexpr (BF16OUT) {
            if (p.bias) v += bias4;
            if (p.flags & PU_EPI_RELU) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            }
            typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
            bf16x4_t o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (__bf16)v[e];
            *reinterpret_cast<bf16x4_t*>(reinterpret_cast<__bf16*>(p.dst0) + (long long)m * N + 4 * lane_c) = o;
        } else if (plain) {
            if (p.bias) v += bias4;
            if (p.flags & PU_EPI_RELU) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            }
            *reinterpret_cast<f32x4*>(p.dst0 + (long long)m * N + 4 * lane_c) = v;
        } else {
            epi_store4(p, epi_row(p, m), 4 * lane_c, v);
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

static bool vec_epilogue(const pu_conv_args* a) {
    const bool shuffle = a->flags & PU_EPI_SHUFFLE2;
    const int n0 = shuffle ? a->n : a->n0;
    const uintptr_t al = (uintptr_t)a->dst0 | (uintptr_t)a->dst1 | (uintptr_t)a->mask0 | (uintptr_t)a->mask1 |
                         (uintptr_t)a->bias | ((a->flags & PU_EPI_RESID) ? (uintptr_t)a->resid : 0);
    // SHUFFLE2: 4 consecutive n stay inside one (i,j) block only when co = n/4 is a multiple of 4
    return (a->n % 4 == 0) && (n0 % 4 == 0) && (al & 15) == 0 && (!shuffle || (a->n / 4) % 4 == 0);
}

// Split-K plan: when the M x N tile grid fills fewer than the resident block slots of the chip
// (256 CUs x blocks per CU of the tile), split the K stages so that it does, keeping >= 8 stages
// (128 k) per split.  Only the direct-to-LDS kernel splits.
static void plan_split(const pu_conv_args* a, long long M, int bm, int bn, int* ksplit, int* t_per) {
    const int T = a->k_pad / IG_BK;
    *ksplit = 1;
    *t_per = T;
    if (choose_mode(a->c0, a->c1) != LOAD_CHUNK16 || !vec_epilogue(a)) return;
    const int occ = (bm == 256) ? 2 : (bm == 128 && bn == 128) ? 3 : 4;   // LDS-limited (3-deep ring)
    const int blocks = blocks_for(M, a->n, bm, bn);
    int ks = (256 * occ) / blocks;
    if (ks > T / 8) ks = T / 8;
    if (ks < 2) return;
    *t_per = ceil_div(T, ks);
    *ksplit = ceil_div(T, *t_per);
}

// Tile / split plan of one call.  The 6-product kernel does 6x the MFMA work per K stage of the
// fp32 one for the same loads, so its per-stage fixed cost matters less and its per-block
// setup/epilogue more: small pixel grids (the 8x8 / 16x16 levels) take the large tiles and split
// K until ~2 blocks per CU, instead of shrinking the tile to 64x64 (6 MFMAs per wave per stage).
// Measured alternatives (round 1, tools/conv_bench.py): 512x64 8-wave and 128x64 4x1 tiles for
// the 64-channel layers (-4...-9 %), 256x256 8-wave tiles for N >= 256 (-5 %).
static bool uses_x6(const pu_conv_args* a);
static bool lean_ok(const pu_conv_args* a) {
    if (!uses_x6(a)) return false;
    const int C = a->c0 + a->c1;
    if (a->kh != 3 || a->kw != 3 || !(a->cgroup == 16 || a->cgroup == 32)) return false;
    if (a->c1 != 0 && a->c1 != a->c0) return false;
    if (a->k_pad != 9 * C) return false;
    const long long shift = (long long)a->pad * a->in_w + a->pad;
    if (((long long)a->batch * a->in_h * a->in_w + shift) * a->c0 * 4 >= (1LL << 31)) return false;
    if ((long long)a->k_pad * a->n * 12 >= (1LL << 31)) return false;
    return true;
}
static void plan_tiles(const pu_conv_args* a, long long M, int* bm, int* bn, int* ksplit, int* t_per) {
    if (!uses_x6(a)) {
        choose_tile(M, a->n, bm, bn);
        plan_split(a, M, *bm, *bn, ksplit, t_per);
        return;
    }
    const int N = a->n;
    const int T = a->k_pad / IG_BK;
    int target = 512;                 // ~2 resident blocks per CU (4-wave tiles)
    if (N <= 32 && lean_ok(a)) {      // 32-channel layers (C4/C5 levels): no half-empty 64-wide tiles
        *bn = 32;
        *bm = blocks_for(M, N, 256, 32) >= 480 ? 256 : 128;
    } else if (N <= 64) {
        *bn = 64;
        *bm = blocks_for(M, N, 256, 64) >= 480 ? 256 : 128;
    } else if (a->k_pad >= 2048) {
        // 8 waves, one block per CU (85 KB of LDS), each wave 32 pixels x 128 channels: fewer
        // LDS-DMA pieces and global bytes per MFMA than two 128 x 128 blocks; +2-4% on the
        // long-K layers (16x16 / 32x32 levels), a loss on short-K ones (K = 576: l2_cat dgrad)
        *bn = 128;
        *bm = 256;
        target = 256;
    } else {
        *bn = 128;
        *bm = 128;
    }
    *ksplit = 1;
    *t_per = T;
    const int tiles = blocks_for(M, N, *bm, *bn);
    if (tiles >= target - target / 16 || !vec_epilogue(a)) return;
    int ks = ceil_div(target, tiles);
    if (ks > T / 8) ks = T / 8;
    if (ks < 2) return;
    *t_per = ceil_div(T, ks);
    if (lean_ok(a)) {                  // the lean kernel splits K on channel-group boundaries
        const int spg = 9 * (a->cgroup / 16);
        *t_per = ceil_div(*t_per, spg) * spg;
    }
    *ksplit = ceil_div(T, *t_per);
}

// the small-channel direct convolution handles: 3x3 / s1 / p1 (same size), C in {1,4,8,12,16},
// N in {4,8,16}, tap-major weight rows, float4 epilogue
// the direct 1x1 kernel: k 1 / s1 / p0 (same size), C in {4, 8}, N in {8, 16}, plain float4 epilogue
static bool conv1x1_small_ok(const pu_conv_args* a) {
    const int C = a->c0 + a->c1;
    return (C == 4 || C == 8) && (a->n == 8 || a->n == 16) && a->kh == 1 && a->kw == 1 && a->stride == 1 &&
           a->pad == 0 && a->in_h == a->out_h && a->in_w == a->out_w && !(a->flags & PU_EPI_SHUFFLE2) &&
           vec_epilogue(a) && a->c0 % 4 == 0 && a->c1 % 4 == 0 && (a->cgroup == 0 || a->cgroup >= C);
}

static bool small_conv_ok(const pu_conv_args* a) {
    const int C = a->c0 + a->c1;
    const bool cset = C == 1 || C == 4 || C == 8 || C == 12 || C == 16;
    const bool nset = a->n == 4 || a->n == 8 || a->n == 16;
    const bool nc = (a->n == 4) ? (C == 4 || C == 8 || C == 16) : true;
    return cset && nset && nc && a->kh == 3 && a->kw == 3 && a->stride == 1 && a->pad == 1 &&
           a->in_h == a->out_h && a->in_w == a->out_w && !(a->flags & PU_EPI_SHUFFLE2) && vec_epilogue(a) &&
           (a->cgroup == 0 || a->cgroup >= C) && (C == 1 || (a->c0 % 4 == 0 && a->c1 % 4 == 0)) &&
           a->k_pad == (9 * C + 15) / 16 * 16;   // the kernel's compile-time weight row stride
}

// the single-channel stem: 3x3 / s1 / p1 (same size), C = 1, N in {32, 48, 64} (4-channel lane
// groups that divide a wave), plain (non-SHUFFLE2) float4 epilogue
static bool stem_conv_ok(const pu_conv_args* a) {
    const int C = a->c0 + a->c1;
    return C == 1 && a->c1 == 0 && (a->n == 8 || a->n == 16 || a->n == 32 || a->n == 64) && a->kh == 3 && a->kw == 3 && a->stride == 1 &&
           a->pad == 1 && a->in_h == a->out_h && a->in_w == a->out_w && !(a->flags & PU_EPI_SHUFFLE2) &&
           vec_epilogue(a) && (a->cgroup == 0 || a->cgroup >= C);
}

static bool uses_x6(const pu_conv_args* a) {
    return a->weight6 && choose_mode(a->c0, a->c1) == LOAD_CHUNK16 && !small_conv_ok(a);
}

static size_t split_bytes(long long M, int n, int ksplit) {
    return ksplit > 1 ? (size_t)ksplit * (size_t)M * (size_t)n * sizeof(float) : 0;
}

}  // namespace pu

using namespace pu;

extern "C" int pu_conv_igemm(const pu_conv_args* a, void* stream) {
    PU_REQUIRE(a != nullptr, "pu_conv_igemm: null args");
    PU_REQUIRE(a->batch > 0 && a->in_h > 0 && a->in_w > 0 && a->out_h > 0 && a->out_w > 0,
               "pu_conv_igemm: bad grid %dx%dx%d -> %dx%d", a->batch, a->in_h, a->in_w, a->out_h, a->out_w);
    PU_REQUIRE(a->kh > 0 && a->kw > 0 && a->stride > 0 && a->pad >= 0, "pu_conv_igemm: bad taps");
    PU_REQUIRE(a->kh * a->kw <= 32, "pu_conv_igemm: at most 32 taps");
    PU_REQUIRE(a->src0 && a->c0 > 0, "pu_conv_igemm: src0 missing");
    PU_REQUIRE(a->c1 == 0 || a->src1, "pu_conv_igemm: src1 missing for c1=%d", a->c1);
    PU_REQUIRE(a->weight && a->dst0 && a->n > 0, "pu_conv_igemm: weight/dst0/n");
    const int C = a->c0 + a->c1;
    const int K = a->kh * a->kw * C;
    PU_REQUIRE(a->k_pad >= K && a->k_pad % IG_BK == 0, "pu_conv_igemm: k_pad %d must be >= %d and a multiple of 16", a->k_pad, K);
    const bool shuffle = a->flags & PU_EPI_SHUFFLE2;
    if (a->flags & PU_EPI_RESID) {
        PU_REQUIRE(a->resid && !shuffle && (a->n0 == a->n), "pu_conv_igemm: RESID needs resid, a single destination, no SHUFFLE2");
    }
    if (shuffle) {
        PU_REQUIRE(a->n % 4 == 0, "pu_conv_igemm: SHUFFLE2 needs n %% 4 == 0");
        PU_REQUIRE(a->shuf_off >= 0 && a->shuf_h >= 0 && a->shuf_w >= 0, "pu_conv_igemm: shuffle geometry");
    } else {
        PU_REQUIRE(a->n0 > 0 && a->n0 <= a->n, "pu_conv_igemm: n0 %d out of range", a->n0);
        PU_REQUIRE(a->n0 == a->n || a->dst1, "pu_conv_igemm: dst1 missing");
    }
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    PU_REQUIRE(M < (1LL << 31) && (long long)a->batch * a->in_h * a->in_w < (1LL << 31), "pu_conv_igemm: too many pixels");

    IgemmParams p;
    p.M = (int)M; p.N = a->n; p.K = K; p.k_pad = a->k_pad;
    p.Hi = a->in_h; p.Wi = a->in_w; p.Ho = a->out_h; p.Wo = a->out_w;
    p.kh = a->kh; p.kw = a->kw; p.stride = a->stride; p.pad = a->pad;
    p.C = C; p.c0 = a->c0; p.c1 = a->c1;
    p.src0 = a->src0; p.src1 = a->src1; p.wt = a->weight; p.bias = a->bias;
    p.dst0 = a->dst0; p.dst1 = a->dst1; p.mask0 = a->mask0; p.mask1 = a->mask1;
    p.n0 = shuffle ? a->n : a->n0; p.flags = a->flags;
    p.resid = (a->flags & PU_EPI_RESID) ? a->resid : nullptr;
    p.shuf_h = a->shuf_h ? a->shuf_h : 2 * a->out_h;
    p.shuf_w = a->shuf_w ? a->shuf_w : 2 * a->out_w;
    p.shuf_off = a->shuf_off;
    p.dWo = make_fastdiv(a->out_w); p.dHo = make_fastdiv(a->out_h);
    p.dC = make_fastdiv(C); p.dKw = make_fastdiv(a->kw); p.dCo = make_fastdiv(shuffle ? a->n / 4 : 1);
    p.taps = a->kh * a->kw;
    p.dTaps = make_fastdiv(p.taps);
    p.cgroup = a->cgroup;
    p.vec_epi = vec_epilogue(a);
    p.in_pix = a->batch * a->in_h * a->in_w;
    p.cscale = a->chan_scale;
    p.cs_ld = a->chan_scale_ld ? a->chan_scale_ld : (shuffle ? a->n / 4 : a->n);
    p.dHW = make_fastdiv(a->out_h * a->out_w);
    if (a->chan_scale) {
        PU_REQUIRE(((uintptr_t)a->chan_scale & 15) == 0 && p.cs_ld % 4 == 0 && p.cs_ld >= (shuffle ? a->n / 4 : a->n),
                   "pu_conv_igemm: chan_scale must be 16-byte aligned with a row stride >= its channels and %% 4 == 0 (ld %d)", p.cs_ld);
    }

    const int mode = choose_mode(a->c0, a->c1);
    PU_REQUIRE(a->cgroup == 0 || a->cgroup == 16 || a->cgroup == 32, "pu_conv_igemm: cgroup %d", a->cgroup);
    PU_REQUIRE(a->cgroup == 0 || (mode == LOAD_CHUNK16 && a->c0 % a->cgroup == 0 && a->c1 % a->cgroup == 0),
               "pu_conv_igemm: cgroup %d needs channel counts (%d, %d) that are multiples of it", a->cgroup, a->c0, a->c1);
    if (mode != LOAD_SCALAR) {
        PU_REQUIRE(((uintptr_t)a->src0 & 15) == 0 && ((uintptr_t)a->src1 & 15) == 0,
                   "pu_conv_igemm: sources must be 16-byte aligned");
    }
    PU_REQUIRE(((uintptr_t)a->weight & 15) == 0, "pu_conv_igemm: weight must be 16-byte aligned");

    hipStream_t s = as_stream(stream);
    const int N = a->n;
    if (a->flags & PU_EPI_OUT_BF16) {
        PU_REQUIRE(stem_conv_ok(a) && !a->mask0 && !a->mask1 && !a->resid && !a->chan_scale && a->n0 == a->n &&
                       !(a->flags & (PU_EPI_ACCUM | PU_EPI_SHUFFLE2)) && ((uintptr_t)a->dst0 & 7) == 0,
                   "pu_conv_igemm: PU_EPI_OUT_BF16 is the single-channel stem conv only (c0 1, 3x3/s1/p1, n 8/16/32/64, "
                   "no mask/resid/accum/shuffle/chan_scale, 8-byte aligned dst0)");
        p.ksplit = 1;
        const dim3 sgrid((unsigned)(((a->out_w + ST_TW - 1) / ST_TW) * ((a->out_h + ST_TH - 1) / ST_TH) * a->batch));
        if (N == 64) hipLaunchKernelGGL((stem_conv_kernel<64, true>), sgrid, dim3(256), 0, s, p);
        else if (N == 32) hipLaunchKernelGGL((stem_conv_kernel<32, true>), sgrid, dim3(256), 0, s, p);
        else if (N == 16) hipLaunchKernelGGL((stem_conv_kernel<16, true>), sgrid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((stem_conv_kernel<8, true>), sgrid, dim3(256), 0, s, p);
        return check_launch("pu_conv_igemm (stem, bf16 out)");
    }
    if (stem_conv_ok(a)) {
        p.ksplit = 1;
        const dim3 sgrid((unsigned)(((a->out_w + ST_TW - 1) / ST_TW) * ((a->out_h + ST_TH - 1) / ST_TH) * a->batch));
        if (N == 64) hipLaunchKernelGGL((stem_conv_kernel<64>), sgrid, dim3(256), 0, s, p);
        else if (N == 32) hipLaunchKernelGGL((stem_conv_kernel<32>), sgrid, dim3(256), 0, s, p);
        else if (N == 16) hipLaunchKernelGGL((stem_conv_kernel<16>), sgrid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((stem_conv_kernel<8>), sgrid, dim3(256), 0, s, p);
        return check_launch("pu_conv_igemm (stem)");
    }
    if (conv1x1_small_ok(a)) {
        p.ksplit = 1;
        const dim3 g1((unsigned)(M / 256 + 1 < 8192 ? M / 256 + 1 : 8192));
        if (C == 4 && N == 8) hipLaunchKernelGGL((conv1x1_small_kernel<4, 8>), g1, dim3(256), 0, s, p);
        else if (C == 4) hipLaunchKernelGGL((conv1x1_small_kernel<4, 16>), g1, dim3(256), 0, s, p);
        else if (N == 8) hipLaunchKernelGGL((conv1x1_small_kernel<8, 8>), g1, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((conv1x1_small_kernel<8, 16>), g1, dim3(256), 0, s, p);
        return check_launch("pu_conv_igemm (1x1 small-channel)");
    }
    if (smallx6_ok(a, p.vec_epi)) {
        p.ksplit = 1;
        return smallx6_launch(a, p, s);
    }
    if (small_conv_ok(a)) {
        p.ksplit = 1;
        const dim3 sgrid((unsigned)(((a->out_w + SC_TW - 1) / SC_TW) * ((a->out_h + SC_TH - 1) / SC_TH) * a->batch));
#define PU_SC(C_, N_) if (C == C_ && N == N_) hipLaunchKernelGGL((smallconv_kernel<C_, N_>), sgrid, dim3(256), 0, s, p)
        PU_SC(1, 8); else PU_SC(1, 16); else PU_SC(4, 8); else PU_SC(4, 16); else PU_SC(8, 8); else PU_SC(8, 16);
        else PU_SC(12, 8); else PU_SC(12, 16); else PU_SC(16, 8); else PU_SC(16, 16);
        else PU_SC(4, 4); else PU_SC(8, 4); else PU_SC(16, 4);
#undef PU_SC
        return check_launch("pu_conv_igemm (small-channel)");
    }
    if (wino_ok(a, p.vec_epi)) {
        PU_REQUIRE(((uintptr_t)a->weight6 & 15) == 0, "pu_conv_igemm: weight6 must be 16-byte aligned");
        p.gn = N / 64;
        p.part = (float*)a->workspace;
        p.ksplit = wino_launch(a, p, s);
        if (p.ksplit > 1) {
            const long long tot = M * (N / 4);
            hipLaunchKernelGGL(igemm_splitk_epilogue_kernel, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0, s, p);
        }
        return check_launch("pu_conv_igemm (winograd x6)");
    }
    int bm, bn;
    plan_tiles(a, M, &bm, &bn, &p.ksplit, &p.t_per);
    p.gn = ceil_div(N, bn);
    if (p.ksplit > 1 && (!a->workspace || a->ws_bytes < split_bytes(M, N, p.ksplit))) {
        p.ksplit = 1;                       // no scratch: unsplit
        p.t_per = a->k_pad / IG_BK;
    }
    p.part = (float*)a->workspace;
    const dim3 grid(ceil_div(M, bm) * p.gn * p.ksplit);
    if (a->weight6 && mode == LOAD_CHUNK16) {
        p.wt = reinterpret_cast<const float*>(a->weight6);
        PU_REQUIRE(((uintptr_t)a->weight6 & 15) == 0, "pu_conv_igemm: weight6 must be 16-byte aligned");
        if (lean_ok(a)) {
            const int cg = a->cgroup / 16;
            bool done = true;
#define PU_XL(BM_, BN_, WM_, WN_, NW_)                                                                          \
    do {                                                                                                        \
        if (cg == 2) hipLaunchKernelGGL((igemm_x6_lean_kernel<BM_, BN_, WM_, WN_, NW_, 2>), grid, dim3(NW_ * 64), 0, s, p); \
        else hipLaunchKernelGGL((igemm_x6_lean_kernel<BM_, BN_, WM_, WN_, NW_, 1>), grid, dim3(NW_ * 64), 0, s, p); \
    } while (0)
            if (bm == 256 && bn == 128) PU_XL(256, 128, 8, 1, 8);
            else if (bm == 256 && bn == 64) PU_XL(256, 64, 8, 1, 8);   // 8 x 1 waves: fwd +3-4 % over 4 x 1
            else if (bm == 128 && bn == 128) PU_XL(128, 128, 4, 1, 4);
            else if (bm == 128 && bn == 64) PU_XL(128, 64, 2, 2, 4);
            else if (bm == 256 && bn == 32) PU_XL(256, 32, 4, 1, 4);
            else if (bm == 128 && bn == 32) PU_XL(128, 32, 4, 1, 4);
            else done = false;
#undef PU_XL
            if (done) {
                if (p.ksplit > 1) {
                    const long long tot = M * (N / 4);
                    hipLaunchKernelGGL(igemm_splitk_epilogue_kernel, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0, s, p);
                }
                return check_launch("pu_conv_igemm (x6 lean)");
            }
        }
#define PU_X6(BM_, BN_, WM_, WN_) hipLaunchKernelGGL((igemm_x6_kernel<BM_, BN_, WM_, WN_>), grid, dim3(256), 0, s, p)
        if (bm == 256 && bn == 128)
            hipLaunchKernelGGL((igemm_x6_kernel<256, 128, 8, 1, 8>), grid, dim3(512), 0, s, p);
        else if (bm == 256) PU_X6(256, 64, 4, 1);
        else if (bm == 128 && bn == 128) PU_X6(128, 128, 4, 1);
        else PU_X6(128, 64, 2, 2);
#undef PU_X6
    } else if (mode == LOAD_CHUNK16) {
        if (bm == 256) hipLaunchKernelGGL((igemm_dma_kernel<256, 64, 4, 1, 3>), grid, dim3(256), 0, s, p);
        else if (bm == 128 && bn == 128) hipLaunchKernelGGL((igemm_dma_kernel<128, 128, 2, 2, 3>), grid, dim3(256), 0, s, p);
        else if (bm == 128) hipLaunchKernelGGL((igemm_dma_kernel<128, 64, 2, 2, 3>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((igemm_dma_kernel<64, 64, 2, 2, 3>), grid, dim3(256), 0, s, p);
    } else if (bm == 256) launch_mode<256, 64, 4, 1>(mode, p, grid, s);
    else if (bm == 128 && bn == 128) launch_mode<128, 128, 2, 2>(mode, p, grid, s);
    else if (bm == 128) launch_mode<128, 64, 2, 2>(mode, p, grid, s);
    else launch_mode<64, 64, 2, 2>(mode, p, grid, s);
    if (p.ksplit > 1) {
        const long long threads = M * (N / 4);
        hipLaunchKernelGGL(igemm_splitk_epilogue_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, p);
    }
    return check_launch("pu_conv_igemm");
}

extern "C" int pu_split_weight6(const float* packed, void* out, int n, int k_pad, void* stream) {
    PU_REQUIRE(packed && out && n > 0 && k_pad > 0 && k_pad % IG_BK == 0, "pu_split_weight6: bad args");
    const long long total = (long long)n * k_pad;
    long long blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(split_weight6_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), packed,
                       (__bf16*)out, n, k_pad);
    return check_launch("pu_split_weight6");
}

extern "C" size_t pu_conv_igemm_workspace_bytes(const pu_conv_args* a) {
    if (!a || a->batch <= 0 || a->out_h <= 0 || a->out_w <= 0 || a->n <= 0 || a->k_pad <= 0) return 0;
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    if (small_conv_ok(a) || stem_conv_ok(a) || conv1x1_small_ok(a) || smallx6_ok(a, vec_epilogue(a))) return 0;
    if (wino_ok(a, vec_epilogue(a))) return wino_workspace_bytes(a);
    int bm, bn, ks, tp;
    plan_tiles(a, M, &bm, &bn, &ks, &tp);
    return split_bytes(M, a->n, ks);
}

extern "C" int pu_conv_igemm_tile(const pu_conv_args* a, int* bm, int* bn, int* mode, int* ksplit) {
    PU_REQUIRE(a && bm && bn && mode, "pu_conv_igemm_tile: null args");
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    int ks, tp;
    plan_tiles(a, M, bm, bn, &ks, &tp);
    *mode = choose_mode(a->c0, a->c1);
    if (uses_x6(a)) *mode = 4;   // 6-product bf16
    if (stem_conv_ok(a)) {           // reported as mode 5 ("stem"), tile ST_TH x ST_TW pixels
        *bm = ST_TH * ST_TW;
        *bn = a->n;
        *mode = 5;
        if (ksplit) *ksplit = 1;
        return PU_OK;
    }
    if (conv1x1_small_ok(a)) {       // reported as mode 3 ("direct"), one pixel per thread
        *bm = 256;
        *bn = a->n;
        *mode = 3;
        if (ksplit) *ksplit = 1;
        return PU_OK;
    }
    if (smallx6_ok(a, vec_epilogue(a))) {   // reported as mode 7 ("x6s"), 16 x 32 pixels x n (stride 2: 4 x 32)
        *bm = a->stride == 2 ? 128 : a->kh == 2 ? 256 : 512;
        *bn = a->n;
        *mode = 7;
        if (ksplit) *ksplit = 1;
        return PU_OK;
    }
    if (small_conv_ok(a)) {          // reported as mode 3 ("direct"), tile SC_TH x SC_TW pixels
        *bm = SC_TH * SC_TW;
        *bn = a->n;
        *mode = 3;
        if (ksplit) *ksplit = 1;
        return PU_OK;
    }
    if (wino_ok(a, vec_epilogue(a))) {  // reported as mode 6 ("wino"): 64 tiles (256 pixels) x 64 channels,
        const int wc = wino_item_channels(a);      // or 32 tiles (128 pixels) x 128 channels
        *bm = wc == 64 ? 256 : 128;
        *bn = wc;
        *mode = 6;
        if (ksplit) {
            const size_t need = wino_workspace_bytes(a);
            *ksplit = need && a->workspace && a->ws_bytes >= need ? (int)(need / ((size_t)M * a->n * 4)) : 1;
        }
        return PU_OK;
    }
    if (ksplit) *ksplit = (ks > 1 && a->workspace && a->ws_bytes >= split_bytes(M, a->n, ks)) ? ks : 1;
    return PU_OK;
}
