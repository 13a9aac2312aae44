// bf16 mixed-precision implicit-GEMM convolution (config C3: "same model in bf16, fp32
// accumulation").  Activations, weights, masks and residuals are bf16 in HBM;
// v_mfma_f32_32x32x16_bf16 accumulates in fp32; bias is fp32; outputs are rounded to bf16 once, in
// the epilogue.
//
// Same machinery as igemm.hip's direct-to-LDS kernel, byte for byte: a stage is 64-byte LDS rows
// filled by global_load_lds_dwordx4 with the XOR swizzle kc ^ ((r>>2)&3), a 3-deep ring, counted
// vmcnt + raw barrier, branch-free loader.  A 64-byte row now holds 32 bf16 k-values (BK = 32) and
// a lane's 16-byte chunk is exactly one 32x32x16 operand fragment (8 consecutive k of its row:
// A[row l&31][k = 8h + j], B[k = 8h + j][col l&31]), so each (i, j) sub-tile takes 2 MFMAs per
// stage.  Weights are the A operand, pixels the B operand: each lane owns 4 consecutive output
// channels of one pixel, stored as 8 bytes.
#include "common.h"

#ifndef PU_EPI_BATCH
#define PU_EPI_BATCH 1   // 0: every output through epi_store4_b (A/B builds)
#endif

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BK16 = 32;   // k per stage (64 B of bf16)

struct IgemmBf16Params {
    int M, N, K, k_pad;
    int Hi, Wi, Ho, Wo, kh, kw, stride, pad;
    int C, c0, c1;
    const __bf16* src0;
    const __bf16* src1;
    const __bf16* wt;
    const float* bias;
    __bf16* dst0;
    __bf16* dst1;
    const __bf16* mask0;
    const __bf16* mask1;
    const __bf16* resid;
    int n0, flags;
    int cgroup, taps, gn;
    int ksplit, t_per;
    float* part;
    int shuf_h, shuf_w, shuf_off;
    FastDiv dWo, dHo, dC, dKw, dCo, dTaps;
    int in_pix;             // batch * Hi * Wi (the lean kernel's buffer extent)
};

struct EpiRowB {
    long long pix;
    int oh0, ow0;
};

__device__ __forceinline__ EpiRowB epi_row_b(const IgemmBf16Params& p, int m) {
    if (!(p.flags & PU_EPI_SHUFFLE2)) return {m, 0, 0};
    const int t2 = fdiv(m, p.dWo);
    const int wo = m - t2 * p.Wo;
    const int bb = fdiv(t2, p.dHo);
    const int ho = t2 - bb * p.Ho;
    return {(long long)bb * p.shuf_h, 2 * ho - p.shuf_off, 2 * wo - p.shuf_off};
}

__device__ __forceinline__ f32x4 ld4(const __bf16* p) {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

// epilogue of output channels n..n+3 (n % 4 == 0, N % 4 == 0, n0 % 4 == 0) of row r
__device__ __forceinline__ void epi_store4_b(const IgemmBf16Params& p, const EpiRowB& r, int n, f32x4 v) {
    __bf16* dst;
    const __bf16* msk;
    long long off;
    int nb;
    if (p.flags & PU_EPI_SHUFFLE2) {
        const int co = p.N >> 2;
        const int ij = fdiv(n, p.dCo);
        nb = n - ij * co;
        const int oh = r.oh0 + (ij >> 1), ow = r.ow0 + (ij & 1);
        if ((unsigned)oh >= (unsigned)p.shuf_h || (unsigned)ow >= (unsigned)p.shuf_w) return;
        off = ((r.pix + oh) * p.shuf_w + ow) * co + nb;
        dst = p.dst0; msk = p.mask0;
    } else if (n < p.n0) {
        off = r.pix * p.n0 + n;
        dst = p.dst0; msk = p.mask0; nb = n;
    } else {
        off = r.pix * (p.N - p.n0) + (n - p.n0);
        dst = p.dst1; msk = p.mask1; nb = n;
    }
    if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + nb);
    if (p.resid) v += ld4(p.resid + off);
    if (p.flags & PU_EPI_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (msk) {
        const f32x4 mv = ld4(msk + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) if (!(mv[e] > 0.f)) v[e] = 0.f;
    }
    if (p.flags & PU_EPI_ACCUM) v += ld4(dst + off);
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (__bf16)v[e];
    *reinterpret_cast<bf16x4*>(dst + off) = o;
}

// The two common epilogue forms - bias (+ReLU), the forward, or masks (+ReLU), the data gradient -
// for an [NI][NJ] grid of 32 x 32 accumulator fragments, with every operand load issued before the
// first store: gfx9's vmcnt counts stores too, so epi_store4_b's load-then-store per output made
// each output wait out the previous stores' round trips (in the persistent halo kernel, right
// before the next tile's first group).  Buffer descriptors with 32-bit offsets, wave-uniform per
// 32-column fragment (n0 % 32 == 0); lanes past M / N load zeros and drop their stores.  Same
// operations and rounding as epi_store4_b.  epi_batch_b_ok: the launch takes this form.
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t epi_rsrc_b(const void* base, bool on) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    void* ub = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(ub, 0, on ? 0x7fffffff : 0, 0x00020000);
}

__device__ __forceinline__ int epi_batch_b_ok(const IgemmBf16Params& p) {
    if (PU_EPI_BATCH == 0 || (p.flags & (PU_EPI_SHUFFLE2 | PU_EPI_ACCUM)) || p.resid || p.n0 % 32 || p.N % 32 ||
        (long long)p.M * p.N >= (1LL << 29))
        return 0;
    const bool mk = p.mask0 || p.mask1;
    return mk && !p.bias ? 1 : (!mk && p.bias ? 2 : 0);     // 1 masks, 2 bias
}

template <bool MASK, int NI, int NJ>
__device__ __forceinline__ void epilogue_batched_b(const IgemmBf16Params& p, f32x16 (&acc)[NI][NJ], int m0, int nc0,
                                                   int lr, int lh) {
    const bool relu = p.flags & PU_EPI_RELU;
    const int n1 = p.N - p.n0;
    unsigned orow[NI][NJ];             // byte offset of (row m, fragment column 0), LEAN_OOB past M / N
    bool first[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) first[j] = nc0 + j * 32 < p.n0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int m = m0 + i * 32 + lr;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int c = nc0 + j * 32 + 4 * lh - (first[j] ? 0 : p.n0);
            orow[i][j] = m < p.M && nc0 + j * 32 < p.N ? (unsigned)(m * (first[j] ? p.n0 : n1) + c) * 2u : LEAN_OOB;
        }
    }
    u32x2_t mv[NI][NJ][4];             // MASK: 4 bf16 mask values per output
    f32x4 bv[NJ][4];                   // !MASK: the bias of the output's channels
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        if constexpr (MASK) {
            const __bf16* mk = first[j] ? p.mask0 : p.mask1;
            const __amdgpu_buffer_rsrc_t r = epi_rsrc_b(mk, mk != nullptr);
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q) mv[i][j][q] = __builtin_amdgcn_raw_buffer_load_b64(r, orow[i][j], 16 * q, 0);
        } else {
            const __amdgpu_buffer_rsrc_t r = epi_rsrc_b(p.bias, true);
            const unsigned nb = nc0 + j * 32 < p.N ? (unsigned)(nc0 + j * 32 + 4 * lh) * 4u : LEAN_OOB;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                bv[j][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, nb, 32 * q, 0));
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const __amdgpu_buffer_rsrc_t rd = epi_rsrc_b(first[j] ? p.dst0 : p.dst1, true);
        const bool has_mk = (first[j] ? p.mask0 : p.mask1) != nullptr;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                if constexpr (!MASK) v += bv[j][q];
                if (relu) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                }
                if constexpr (MASK) {
                    if (has_mk) {
                        const bf16x4 mb = __builtin_bit_cast(bf16x4, mv[i][j][q]);
#pragma unroll
                        for (int e = 0; e < 4; ++e) if (!((float)mb[e] > 0.f)) v[e] = 0.f;
                    }
                }
                bf16x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (__bf16)v[e];
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, o), rd, orow[i][j], 16 * q, 0);
            }
    }
}

// The ConvTranspose2d 2x2 / s2 forward (SHUFFLE2, no crop, bias, co % 32 == 0) in the batched form:
// every bias load before the first store (the per-output epi_store4_b waited out each previous
// store's round trip before its bias load).  Same operations and rounding as epi_store4_b.
__device__ __forceinline__ bool epi_shuf_b_ok(const IgemmBf16Params& p) {
    return PU_EPI_BATCH && (p.flags & PU_EPI_SHUFFLE2) && !(p.flags & PU_EPI_ACCUM) && !p.resid && p.bias && !p.mask0 &&
           p.shuf_off == 0 && p.shuf_h == 2 * p.Ho && p.shuf_w == 2 * p.Wo && (p.N / 4) % 32 == 0 && p.N % 128 == 0 &&
           (long long)p.M * p.N < (1LL << 29);
}

template <int NI, int NJ>
__device__ __forceinline__ void epilogue_batched_shuf_b(const IgemmBf16Params& p, f32x16 (&acc)[NI][NJ], int m0,
                                                        int nc0, int lr, int lh) {
    const bool relu = p.flags & PU_EPI_RELU;
    const int co = p.N >> 2;
    unsigned orow[NI][NJ];
    int cj[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int nj = nc0 + j * 32;
        const int ij = nj < p.N ? nj / co : 0;
        cj[j] = nj - ij * co + 4 * lh;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int m = m0 + i * 32 + lr;
            unsigned o = LEAN_OOB;
            if (m < p.M && nj < p.N) {
                const int t2 = fdiv(m, p.dWo);
                const int wo = m - t2 * p.Wo;
                const int bb = fdiv(t2, p.dHo);
                const int ho = t2 - bb * p.Ho;
                const int pix = (bb * p.shuf_h + 2 * ho + (ij >> 1)) * p.shuf_w + 2 * wo + (ij & 1);
                o = (unsigned)(pix * co + cj[j]) * 2u;
            }
            orow[i][j] = o;
        }
    }
    f32x4 bv[NJ][4];
    const __amdgpu_buffer_rsrc_t rb = epi_rsrc_b(p.bias, true);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            bv[j][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rb, nc0 + j * 32 < p.N ? (unsigned)cj[j] * 4u : LEAN_OOB, 32 * q, 0));
    const __amdgpu_buffer_rsrc_t rd = epi_rsrc_b(p.dst0, true);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < NI; ++i)
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
                bf16x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (__bf16)v[e];
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, o), rd, orow[i][j], 16 * q, 0);
            }
}

// the same epilogue for channels n..n+7 of pixel m (non-SHUFFLE2, n0 % 8 == 0): 16-byte loads and
// stores, so 8 lanes cover a 64-channel pixel row of 128 contiguous bytes.  bias: preloaded.
// Every lane issues the same memory operations (a lane whose destination has no mask still loads,
// from a valid address, and ignores it), so the caller can count them for s_waitcnt: 1 store +
// one load each for resid / mask / accumulate when the launch uses them (epi8_ops).
__device__ __forceinline__ int epi8_ops(const IgemmBf16Params& p) {
    return 1 + (p.resid ? 1 : 0) + ((p.mask0 || p.mask1) ? 1 : 0) + ((p.flags & PU_EPI_ACCUM) ? 1 : 0);
}

__device__ __forceinline__ void epi_store8_b(const IgemmBf16Params& p, long long m, int n, f32x4 v0, f32x4 v1,
                                             f32x4 b0, f32x4 b1) {
    __bf16* dst;
    const __bf16* msk;
    long long off;
    if (n < p.n0) {
        off = m * p.n0 + n;
        dst = p.dst0; msk = p.mask0;
    } else {
        off = m * (p.N - p.n0) + (n - p.n0);
        dst = p.dst1; msk = p.mask1;
    }
    v0 += b0;
    v1 += b1;
    if (p.resid) {
        const bf16x8 r = *reinterpret_cast<const bf16x8*>(p.resid + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v0[e] += (float)r[e]; v1[e] += (float)r[4 + e]; }
    }
    if (p.flags & PU_EPI_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { v0[e] = fmaxf(v0[e], 0.f); v1[e] = fmaxf(v1[e], 0.f); }
    }
    if (p.mask0 || p.mask1) {
        const __bf16* mp = msk ? msk + off : (p.mask0 ? p.mask0 : p.mask1);
        const bf16x8 mv = *reinterpret_cast<const bf16x8*>(mp);
        if (msk) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!((float)mv[e] > 0.f)) v0[e] = 0.f;
                if (!((float)mv[4 + e] > 0.f)) v1[e] = 0.f;
            }
        }
    }
    if (p.flags & PU_EPI_ACCUM) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(dst + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v0[e] += (float)a[e]; v1[e] += (float)a[4 + e]; }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) { o[e] = (__bf16)v0[e]; o[4 + e] = (__bf16)v1[e]; }
    *reinterpret_cast<bf16x8*>(dst + off) = o;
}

// s_waitcnt vmcnt(base + extra) for a run-time extra in {0, 2, ..., 62 - base} (wave-uniform);
// anything else waits for vmcnt(base) (more than needed: always safe)
template <int BASE, int X = 0>
__device__ __forceinline__ void wait_vm_plus(int extra) {
    if constexpr (BASE + X <= 63) {
        if (extra == X) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BASE + X) : "memory");
            return;
        }
        wait_vm_plus<BASE, X + 2>(extra);
    } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BASE) : "memory");
    }
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
__device__ __attribute__((aligned(16))) __bf16 g_zero_b16[8];

template <int BM, int BN, int WM, int WN, int NBUF>
__global__ __launch_bounds__(256) void igemm_bf16_kernel(const IgemmBf16Params p) {
    constexpr int FM = BM / WM / 32;
    constexpr int FN = BN / WN / 32;
    constexpr int A_LD = BM / 64;
    constexpr int B_LD = BN / 64;
    constexpr int G = A_LD + B_LD;
    constexpr int STAGE = (BM + BN) * BK16;   // bf16 elements per ring slot (64 B per row)
    static_assert(WM * WN == 4, "4 waves");

    __shared__ __attribute__((aligned(16))) __bf16 lds[NBUF * STAGE];

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
    const int kc = (lane & 3) ^ ((lane >> 4) & 3);   // logical 16-B chunk this lane fetches
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
            rb0[j] = pix0 * p.c0 + kc * 8;
            rb1[j] = pix0 * p.c1 + kc * 8;
            unsigned msk = 0;
            for (int r = 0; r < p.kh; ++r)
                for (int q = 0; q < p.kw; ++q)
                    if ((unsigned)(hb + r) < (unsigned)p.Hi && (unsigned)(wb + q) < (unsigned)p.Wi)
                        msk |= 1u << (r * p.kw + q);
            tmask[j] = msk;
        }
    }
    const __bf16* wrow[B_LD];
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
        const int n = n_blk + wave * (BN / 4) + 16 * j + lq;
        wrow[j] = n < p.N ? p.wt + (long long)n * p.k_pad + kc * 8 : nullptr;
    }

    const int t0 = kz * p.t_per;
    const int T = min(p.k_pad / BK16 - t0, p.t_per);
    auto issue = [&](int tl, int slot) {
        const bool live = tl < T;
        const int t = t0 + (live ? tl : 0);
        const int k0 = t * BK16;
        // one stage = 32 consecutive channels of one tap (C % 32 == 0): tap-major, or 32-channel
        // groups (cgroup 32: k = (g*taps + tap)*32 + c%32)
        const int g = fdiv(t, p.dTaps);
        const int tap_n = fdiv(k0, p.dC);
        const int tap = p.cgroup ? t - g * p.taps : tap_n;
        const int c = p.cgroup ? g * 32 : k0 - tap_n * p.C;
        const int r = fdiv(tap, p.dKw);
        const int s = tap - r * p.kw;
        const bool first = c < p.c0;
        const __bf16* src = first ? p.src0 : p.src1;
        const int cs = first ? p.c0 : p.c1;
        const long long off = (long long)(r * p.Wi + s) * cs + (first ? c : c - p.c0);
        const unsigned bit = (live && k0 < p.K) ? (1u << tap) : 0u;
        __bf16* a_slot = lds + slot * STAGE;
        __bf16* b_slot = a_slot + BM * BK16;
#pragma unroll
        for (int j = 0; j < A_LD; ++j) {
            const __bf16* gp = (tmask[j] & bit) ? src + (first ? rb0[j] : rb1[j]) + off : g_zero_b16;
            __builtin_amdgcn_global_load_lds((gbl_void_t*)gp, (lds_void_t*)(a_slot + (wave * (BM / 4) + 16 * j) * BK16),
                                             16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < B_LD; ++j) {
            const __bf16* gp = (live && wrow[j]) ? wrow[j] + k0 : g_zero_b16;
            __builtin_amdgcn_global_load_lds((gbl_void_t*)gp, (lds_void_t*)(b_slot + (wave * (BN / 4) + 16 * j) * BK16),
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
    const int swz = (lr >> 2) & 3;

#pragma unroll
    for (int s0 = 0; s0 < NBUF - 1; ++s0) issue(s0, s0);

    for (int t = 0; t < T; ++t) {
        if (NBUF == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const __bf16* a = lds + (t % NBUF) * STAGE;
        const __bf16* b = a + BM * BK16;
        bf16x8 fa[2][FM], fb[2][FN];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int pos = ((kk * 2 + lh) ^ swz) * 8;
#pragma unroll
            for (int i = 0; i < FM; ++i) fa[kk][i] = *reinterpret_cast<const bf16x8*>(a + (a_row0 + i * 32) * BK16 + pos);
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[kk][j] = *reinterpret_cast<const bf16x8*>(b + (b_row0 + j * 32) * BK16 + pos);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[kk][j], fa[kk][i], acc[i][j], 0, 0, 0);
            if (kk == 0) issue(t + NBUF - 1, (t + NBUF - 1) % NBUF);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * (FM + FN), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * FM * FN, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    if (p.ksplit > 1) {
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
        return;
    }
    if (epi_shuf_b_ok(p)) {
        epilogue_batched_shuf_b(p, acc, m_blk + wm * (BM / WM), n_blk + wn * (BN / WN), lr, lh);
        return;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m_blk + wm * (BM / WM) + i * 32 + lr;
        if (m >= p.M) continue;
        const EpiRowB er = epi_row_b(p, m);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n_blk + wn * (BN / WN) + j * 32 + 8 * q + 4 * lh;
                if (n >= p.N) continue;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                epi_store4_b(p, er, n, v);
            }
    }
}

// ---------------------------------------------------------------- lean bf16 kernel
// The loader of igemm.hip's lean x6 kernel on bf16 operands: buffer_load ... lds through buffer
// descriptors, per-lane byte offsets precomputed once per block for all 9 taps (an out-of-image
// tap gets LEAN_OOB and lands as zeros), the stage's (tap, channel) offset one scalar soffset, the
// 9 taps of a 32-channel group unrolled (ring slots and LDS addresses are immediates).  A stage is
// one (tap, 32-channel) K slice in 64-B LDS rows with igemm_bf16_kernel's swizzle; 2 x FM x FN
// MFMAs per wave per stage, one barrier per stage.  Tiles 256 x 128 (2 x 2 waves, 16 MFMAs per
// stage) and 256 x 64 (4 x 1).  Requirements (host: lean_ok_b): 3x3, cgroup 32, c1 == 0 or
// c1 == c0, K == k_pad, split-K on group boundaries, every tensor under 2 GB.
template <int BM, int BN, int WM, int WN, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void igemm_bf16_lean_kernel(const IgemmBf16Params p) {
    constexpr int FM = BM / WM / 32;
    constexpr int FN = BN / WN / 32;
    constexpr int A_LD = BM / (16 * NW);
    constexpr int B_LD = BN / (16 * NW);
    constexpr int G = A_LD + B_LD;
    constexpr int STAGE = (BM + BN) * BK16;   // bf16 elements per ring slot
    constexpr int SPG = 9;                     // stages per 32-channel group (taps)
    static_assert(WM * WN == NW && A_LD >= 1 && B_LD >= 1, "lean bf16 tile");

    __shared__ __attribute__((aligned(16))) __bf16 lds[3 * STAGE];

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

    const int cs = p.c0;                                      // == c1 when c1 != 0
    const int shift = p.pad * p.Wi + p.pad;
    const unsigned a_bytes0 = (unsigned)(((long long)p.in_pix + shift) * cs * 2);
    const __bf16* a0p = p.src0 - (long long)shift * cs;
    const __bf16* a1p = (p.c1 ? p.src1 : p.src0) - (long long)shift * cs;
    const unsigned w_bytes = (unsigned)((long long)p.k_pad * p.N * 2);

    const int lq = lane >> 2;
    const int kc = (lane & 3) ^ ((lane >> 4) & 3);   // logical 16-B chunk this lane fetches
    unsigned vbase[A_LD], vmask[A_LD];               // row byte offset, in-image taps (bit r*3+q)
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
        vbase[j] = (unsigned)pix * (unsigned)(cs * 2) + kc * 16;
        unsigned msk = 0;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (mv && (unsigned)(hb + r) < (unsigned)p.Hi && (unsigned)(wb + q) < (unsigned)p.Wi) msk |= 1u << (r * 3 + q);
        vmask[j] = msk;
    }
    unsigned tapoff[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q) tapoff[r * 3 + q] = (unsigned)((r * p.Wi + q) * cs * 2);
    unsigned wv[B_LD];
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
        const int n = n_blk + wave * (BN / NW) + 16 * j + lq;
        wv[j] = n < p.N ? (unsigned)(n * p.k_pad * 2 + kc * 16) : LEAN_OOB;
    }

    const int groups = p.k_pad / (BK16 * SPG);
    const int gps = p.t_per / SPG;                  // groups per split
    const int g0 = kz * gps;
    const int g1 = min(groups, g0 + gps);

    auto issue = [&](int g, auto uc) {
        constexpr int u = decltype(uc)::value;      // tap
        const bool live = g < g1;
        const int c = g * BK16;
        const bool second = c >= p.c0;
        const __bf16* abase = second ? a1p : a0p;
        const unsigned soff = tapoff[u] + (unsigned)((second ? c - p.c0 : c) * 2);
        __bf16* a_slot = lds + (u % 3) * STAGE;
        __bf16* b_slot = a_slot + BM * BK16;
#pragma unroll
        for (int j = 0; j < A_LD; ++j)
            lean_load(abase, live ? a_bytes0 : 0u, a_slot + (wave * (BM / NW) + 16 * j) * BK16,
                      ((vmask[j] >> u) & 1u) ? vbase[j] : LEAN_OOB, soff);
        const unsigned wsoff = (unsigned)(g * SPG + u) * (BK16 * 2);
#pragma unroll
        for (int j = 0; j < B_LD; ++j)
            lean_load(p.wt, live ? w_bytes : 0u, b_slot + (wave * (BN / NW) + 16 * j) * BK16, wv[j], wsoff);
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
            const __bf16* a = lds + (u % 3) * STAGE;
            const __bf16* b = a + BM * BK16;
            bf16x8 fa[2][FM], fb[2][FN];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int pos = ((kk * 2 + lh) ^ swz) * 8;
#pragma unroll
                for (int i = 0; i < FM; ++i) fa[kk][i] = *reinterpret_cast<const bf16x8*>(a + (a_row0 + i * 32) * BK16 + pos);
#pragma unroll
                for (int j = 0; j < FN; ++j) fb[kk][j] = *reinterpret_cast<const bf16x8*>(b + (b_row0 + j * 32) * BK16 + pos);
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[kk][j], fa[kk][i], acc[i][j], 0, 0, 0);
                if (kk == 0) {
                    if constexpr (u + 2 < SPG) issue(g, std::integral_constant<int, u + 2>{});
                    else issue(g + 1, std::integral_constant<int, u + 2 - SPG>{});
                }
            }
        });
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    if (p.ksplit > 1) {
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
        return;
    }
    if (const int eb = epi_batch_b_ok(p)) {
        if (eb == 1) epilogue_batched_b<true>(p, acc, m_blk + wm * (BM / WM), n_blk + wn * (BN / WN), lr, lh);
        else epilogue_batched_b<false>(p, acc, m_blk + wm * (BM / WM), n_blk + wn * (BN / WN), lr, lh);
        return;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m_blk + wm * (BM / WM) + i * 32 + lr;
        if (m >= p.M) continue;
        const EpiRowB er = epi_row_b(p, m);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n_blk + wn * (BN / WN) + j * 32 + 8 * q + 4 * lh;
                if (n >= p.N) continue;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                epi_store4_b(p, er, n, v);
            }
    }
}

// ---------------------------------------------------------------- halo bf16 kernel
// 3x3 / stride 1 / pad 1 convolutions (fwd and dgrad) of width W = 32, 64 or 128: the lean
// kernel re-reads every input pixel from L2 once per tap (9 x 64 B per pixel and 32-channel group,
// ~2x the L2->LDS rate the MFMAs could consume at bf16); this one loads the (R+2) x (W+2) halo of
// R = 256 / W output rows once per group and serves all 9 taps from LDS.
//   block: 256 output pixels (R whole rows of one image) x 64 output channels, 4 waves of 64 x 64
//   (2 x 2 fragments, 72 MFMAs per wave per group); persistent over an XCD-contiguous tile range;
//   LDS (single image, 2 blocks per CU): the halo as [pixel][32 channels] with an 80-B pixel
//   stride (5 bank quads: conflict-free 16-B fragment reads at every tap shift, every address one
//   base register + an immediate) and the group's 9 tap slices of the weights [tap][n][64 B]
//   (16-B chunks swizzled by n bits 2-3); the next group's halo and weights are loaded into
//   registers under the current group's MFMAs and stored between two barriers.
// K order (cgroup 32) and the MFMA order per accumulator are igemm_bf16_lean_kernel's, so the
// two are bit-identical.  Requirements (host: halo_ok_b).
constexpr int HB_NT = 256;
constexpr int HB_BN = 64;
constexpr int HB_PX = 80;

template <int W>
__global__ __launch_bounds__(HB_NT) __attribute__((amdgpu_waves_per_eu(2))) void igemm_bf16_halo_kernel(const IgemmBf16Params p) {
    constexpr int R = 256 / W;
    constexpr int HW = W + 2;
    constexpr int HP = (R + 2) * HW;                  // halo pixels
    constexpr int XB = HP * HB_PX;
    constexpr int WB = 9 * HB_BN * 64;
    constexpr int ITEMS = 4 * HP;                     // (pixel, 16-B chunk) pieces
    constexpr int IT = (ITEMS + HB_NT - 1) / HB_NT;
    constexpr int WPC = 9 * HB_BN * 4;                // 16-B weight pieces per group
    constexpr int WIT = (WPC + HB_NT - 1) / HB_NT;
    static_assert(R * W == 256 && W % 32 == 0, "halo tile");

    __shared__ __attribute__((aligned(16))) char lds[XB + WB];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;

    const int ntiles = p.M / 256 * p.gn;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;
    const int tq = (ntiles + 7) >> 3;
    const int t_end = min(ntiles, (xcd + 1) * tq);
    int tile = xcd * tq + (int)(blockIdx.x >> 3);
    if (tile >= t_end) return;                        // uniform per block
    const int rb = p.Ho / R;

    int xsrc[IT];                                     // source element offset (-1: padding)
    auto setup = [&](int t) {
        const int mt = t / p.gn;
        const int b = mt / rb;
        const int r0 = (mt - b * rb) * R;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int e = it * HB_NT + tid;
            const int hp = e >> 2;
            const int hr = hp / HW, hc = hp - hr * HW;
            const int ir = r0 - 1 + hr, ic = hc - 1;
            const bool ok = e < ITEMS && (unsigned)ir < (unsigned)p.Hi && (unsigned)ic < (unsigned)W;
            xsrc[it] = ok ? ((b * p.Hi + ir) * W + ic) : -1;
        }
    };

    f32x4 xr[IT], wr[WIT];
    auto load = [&](int g, int n_blk) {
        const int c = g * 32;
        const bool second = c >= p.c0;
        const __bf16* src = second ? p.src1 : p.src0;
        const int cs = second ? p.c1 : p.c0;
        const int cc = (second ? c - p.c0 : c) + (tid & 3) * 8;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            xr[it] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (xsrc[it] >= 0) xr[it] = *reinterpret_cast<const f32x4*>(src + xsrc[it] * cs + cc);
        }
        const __bf16* wsrc = p.wt + (long long)n_blk * p.k_pad + g * 9 * 32;
#pragma unroll
        for (int w = 0; w < WIT; ++w) {
            const int e = w * HB_NT + tid;
            if (e < WPC) {
                const int ch = e & 3, n = (e >> 2) & 63, tap = e >> 8;
                wr[w] = *reinterpret_cast<const f32x4*>(wsrc + n * p.k_pad + tap * 32 + ch * 8);
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int e = it * HB_NT + tid;
            if (e < ITEMS) *reinterpret_cast<f32x4*>(lds + (e >> 2) * HB_PX + (e & 3) * 16) = xr[it];
        }
#pragma unroll
        for (int w = 0; w < WIT; ++w) {
            const int e = w * HB_NT + tid;
            if (e < WPC) {
                const int ch = e & 3, n = (e >> 2) & 63, tap = e >> 8;
                *reinterpret_cast<f32x4*>(lds + XB + (tap * HB_BN + n) * 64 + ((ch ^ ((n >> 2) & 3)) << 4)) = wr[w];
            }
        }
    };

    // wave = 64 output pixels (fragments i = 0, 1 of 32) x 64 channels (fragments j = 0, 1)
    const int p0 = wave * 64;
    const int orow = p0 / W, ocol = p0 - orow * W;
    const unsigned xa = (unsigned)((orow * HW + ocol + lr) * HB_PX);
    constexpr int FRAG1 = (32 / W) * HW + (32 % W);   // halo pixels from fragment 0 to 1
    const unsigned wa = (unsigned)(XB + lr * 64);
    const int wsw = (lr >> 2) & 3;

    f32x16 acc[2][2];
    const int chunks = p.C / 32;
    setup(tile);
    load(0, (tile % p.gn) * HB_BN);
    for (;;) {
        const int m_blk = tile / p.gn * 256;
        const int n_blk = (tile % p.gn) * HB_BN;
        const int next = tile + per_xcd;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        for (int g = 0; g < chunks; ++g) {
            __builtin_amdgcn_s_barrier();             // every wave is done reading group g-1
            asm volatile("" ::: "memory");
            store();
            if (g + 1 < chunks) {
                load(g + 1, n_blk);
            } else if (next < t_end) {                // the next tile's first group flies over
                setup(next);                          // this group's MFMAs and the epilogue
                load(0, (next % p.gn) * HB_BN);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int toff = ((t / 3) * HW + (t % 3)) * HB_PX;
                bf16x8 fx[2][2], fw[2][2];
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    const int chk = kk * 2 + lh;
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        fx[kk][i] = *reinterpret_cast<const bf16x8*>(lds + xa + toff + i * FRAG1 * HB_PX + chk * 16);
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        fw[kk][j] = *reinterpret_cast<const bf16x8*>(lds + wa + (t * HB_BN + j * 32) * 64 + ((chk ^ wsw) << 4));
                }
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[kk][j], fx[kk][i], acc[i][j], 0, 0, 0);
            }
        }
        const int eb = epi_batch_b_ok(p);
        if (eb == 1) {
            epilogue_batched_b<true>(p, acc, m_blk + p0, n_blk, lr, lh);
        } else if (eb == 2) {
            epilogue_batched_b<false>(p, acc, m_blk + p0, n_blk, lr, lh);
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int m = m_blk + p0 + i * 32 + lr;
                const EpiRowB er = epi_row_b(p, m);
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int n = n_blk + j * 32 + 8 * q + 4 * lh;
                        f32x4 v;
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                        epi_store4_b(p, er, n, v);
                    }
            }
        }
        if (next >= t_end) break;
        tile = next;
    }
}

// ---------------------------------------------------------------- halo bf16 kernel, DMA ring
// The same convolutions as igemm_bf16_halo_kernel (3x3 / s1 / p1, width 32 / 64 / 128), restaged so
// that nothing waits on HBM: PMC on the register-staged kernel showed MFMA busy 0.21 and waves
// parked on s_waitcnt / barriers 49 % of their cycles - its next group's halo was loaded one group
// ahead through registers, then stored to LDS between two barriers.
//   block: 4 waves (one per SIMD), one block per CU, persistent over an XCD-contiguous tile range;
//     tile = 512 output pixels (R = 512 / W whole rows of one image) x 64 output channels;
//     wave = 128 pixels x 64 channels (4 x 2 fragments: 6 fragment reads per 8 MFMAs);
//   stage = 16 input channels: the (R+2) x (W+2) halo [pixel][16 ch] (32 B per pixel: a 32-pixel
//     fragment is one contiguous 1 KB run at every tap shift - conflict-free) and the 9 tap slices
//     of the weights [tap][n][16 k], both written straight into LDS by buffer_load ... lds (32-bit
//     offsets: per-lane pixel index x the source's pixel stride + a scalar channel offset; padding
//     and out-of-image pixels get an out-of-range offset and land as zeros);
//   3-slot ring, loads issued two stages ahead (the next tile's first stages fly over this tile's
//     last MFMAs and its epilogue), one counted vmcnt + one barrier per stage.
// K order: group g (32 channels), half h, tap t - a different summation order from the per-tap
// kernels (fp32 accumulation of exact bf16 products either way).  Host: halo2_ok_b.
constexpr int H2_NT = 256;
constexpr int H2_BN = 64;
#ifndef PU_H2_ABL
#define PU_H2_ABL 0     // ablation builds only (timing): 1 no halo loads, 2 no weight loads, 3 neither
#endif

template <int W>
__global__ __launch_bounds__(H2_NT) void igemm_bf16_halo2_kernel(const IgemmBf16Params p) {
    constexpr int R = 512 / W;
    constexpr int HW = W + 2;
    constexpr int HP = (R + 2) * HW;                  // halo pixels
    constexpr int HI = (HP * 2 + 63) / 64;            // 1 KB DMA instructions for the halo
    constexpr int XB = HI * 1024;                     // halo bytes (padded to whole instructions)
    constexpr int WI = 9 * H2_BN * 2 / 64;            // weight instructions: 18
    constexpr int STAGE = XB + WI * 1024;
    constexpr int HPW = (HI + 3) / 4;                 // per wave
    constexpr int WPW = (WI + 3) / 4;
    constexpr int LPW = HPW + WPW;                    // loads per wave per stage (dummies included)
    constexpr int FRAGS = 4;                          // 32-pixel fragments per wave
    static_assert(R * W == 512 && W % 32 == 0 && 3 * STAGE + 1024 <= 160 * 1024, "halo2 tile");

    extern __shared__ __attribute__((aligned(1024))) char h2_lds[];
    char* sink = h2_lds + 3 * STAGE;                  // dummy DMA target

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;

    const int ntiles = p.M / 512 * p.gn;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;
    const int tq = (ntiles + 7) >> 3;
    const int t_end = min(ntiles, (xcd + 1) * tq);
    const int t_first = xcd * tq + (int)(blockIdx.x >> 3);
    if (t_first >= t_end) return;                      // uniform per block
    const int rb = p.Ho / R;
    const int S = p.C / 16;                            // stages per tile
    const unsigned wbytes = (unsigned)p.N * (unsigned)p.k_pad * 2u;
    const unsigned x0bytes = (unsigned)p.in_pix * (unsigned)p.c0 * 2u;
    const unsigned x1bytes = (unsigned)p.in_pix * (unsigned)p.c1 * 2u;

    // ---- loader state (the stage being issued may belong to the next tile)
    int ld_tile = t_first, ld_s = 0;
    int hpix[HPW];                                     // image pixel of this lane's halo piece, -1: zero
    unsigned hchunk[HPW];
    unsigned wvo[WPW];                                 // weight byte offset (without the stage's k)
    auto setup = [&](int t) {
        const int mt = t / p.gn;
        const int b = mt / rb;
        const int r0 = (mt - b * rb) * R;
#pragma unroll
        for (int j = 0; j < HPW; ++j) {
            const int I = wave + 4 * j;
            const int e = I * 64 + lane;
            const int hp = e >> 1;
            const int hr = hp / HW, hc = hp - hr * HW;
            const int ir = r0 - 1 + hr, ic = hc - 1;
            const bool ok = I < HI && hp < HP && (unsigned)ir < (unsigned)p.Hi && (unsigned)ic < (unsigned)W;
            hpix[j] = ok ? (b * p.Hi + ir) * W + ic : -1;
            hchunk[j] = (unsigned)(e & 1) * 16u;
        }
        const int n_blk = (t - mt * p.gn) * H2_BN;
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            const int I = wave + 4 * j;
            const int e = I * 64 + lane;
            const int tap = e >> 7, n = (e >> 1) & 63, ch = e & 1;
            wvo[j] = I < WI ? (unsigned)((n_blk + n) * p.k_pad + tap * 32 + ch * 8) * 2u : LEAN_OOB;
        }
    };
    auto issue = [&](int slot) {
        const bool live = ld_tile < t_end;
        char* base = h2_lds + slot * STAGE;
        const int g = ld_s >> 1, h = ld_s & 1;
        const int c = g * 32 + h * 16;
        const bool second = c >= p.c0;
        const __bf16* src = second ? p.src1 : p.src0;
        const unsigned cs2 = (unsigned)(second ? p.c1 : p.c0) * 2u;
        const unsigned xbytes = live ? (second ? x1bytes : x0bytes) : 0u;
        const unsigned soff = (unsigned)(second ? c - p.c0 : c) * 2u;
#pragma unroll
        for (int j = 0; j < HPW; ++j) {
            const int I = wave + 4 * j;
            const unsigned vo = hpix[j] >= 0 ? (unsigned)hpix[j] * cs2 + hchunk[j] : LEAN_OOB;
            if (PU_H2_ABL != 1 && PU_H2_ABL != 3) lean_load(src, xbytes, I < HI ? base + I * 1024 : sink, vo, soff);
        }
        const unsigned wsoff = (unsigned)(g * 288 + h * 16) * 2u;
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            const int I = wave + 4 * j;
            if (PU_H2_ABL != 2 && PU_H2_ABL != 3)
                lean_load(p.wt, live ? wbytes : 0u, I < WI ? base + XB + I * 1024 : sink, wvo[j], wsoff);
        }
        if (++ld_s == S) {                             // the next stage opens the next tile
            ld_s = 0;
            ld_tile += per_xcd;
            if (ld_tile < t_end) setup(ld_tile);
        }
    };

    // ---- fragment addresses: fragment i = pixels wave*128 + 32 i .. +31 (one image row each)
    unsigned xa[FRAGS];
#pragma unroll
    for (int i = 0; i < FRAGS; ++i) {
        const int p0 = wave * 128 + 32 * i;
        const int orow = p0 / W, ocol = p0 - orow * W;
        xa[i] = (unsigned)((orow * HW + ocol + lr) * 32 + lh * 16);
    }
    const unsigned wa = (unsigned)(XB + lr * 32 + lh * 16);

    // memory operations per wave of one tile's epilogue: 4 fragments x 4 pixel passes x epi8_ops,
    // plus the two bias loads
    const int EOPS = 16 * epi8_ops(p) + (p.bias ? 2 : 0);
    setup(t_first);
    issue(0);
    issue(1);
    int tile = t_first;
    int u = 0;                                         // stage counter (ring position)
    for (;;) {
        const int mt = tile / p.gn;
        const int m_blk = mt * 512;
        const int n_blk = (tile - mt * p.gn) * H2_BN;
        f32x16 acc[FRAGS][2];
#pragma unroll
        for (int i = 0; i < FRAGS; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        for (int s = 0; s < S; ++s, ++u) {
            // stage u landed.  In a tile's first two stages the previous tile's epilogue (EOPS
            // memory operations, issued after stage u+1's loads) is still in flight: count it
            // instead of draining it, so its stores overlap this tile's MFMAs
            if (s < 2 && tile != t_first) wait_vm_plus<LPW>(EOPS);
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPW) : "memory");
            __builtin_amdgcn_s_barrier();              // ... for every wave; slot (u+2)%3 is free
            asm volatile("" ::: "memory");
            const int slot = u % 3;
            issue(slot == 0 ? 2 : slot - 1);
            const char* a = h2_lds + slot * STAGE;
            // fragments double-buffered one tap ahead; the scheduling barriers keep tap t+1's six
            // reads ahead of tap t's eight MFMAs (left alone, the scheduler interleaved each read
            // with its consumer: one wave per SIMD then waits out every LDS latency)
            bf16x8 fx[2][FRAGS], fw[2][2];
            auto frag = [&](int t, int bsel) {
                const int toff = ((t / 3) * HW + (t % 3)) * 32;
#pragma unroll
                for (int i = 0; i < FRAGS; ++i) fx[bsel][i] = *reinterpret_cast<const bf16x8*>(a + xa[i] + toff);
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    fw[bsel][j] = *reinterpret_cast<const bf16x8*>(a + wa + (t * H2_BN + j * 32) * 32);
            };
            frag(0, 0);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                if (t + 1 < 9) frag(t + 1, (t + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < FRAGS; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[t & 1][j], fx[t & 1][i], acc[i][j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // epilogue through the ring slot this stage just consumed (free until the next stage's
        // issue, which follows a barrier): per 32-pixel fragment, the wave's 32 x 64 fp32 tile
        // goes to LDS [pixel][68 floats] (conflict-free b128 writes), and comes back as 8
        // channels of one pixel per lane - every store is a full 128-byte pixel row segment
        // (the MFMA layout would store 8 bytes per lane and 64 pieces per instruction)
        __builtin_amdgcn_s_barrier();                  // every wave is done reading the slot
        asm volatile("" ::: "memory");
        float* ep = reinterpret_cast<float*>(h2_lds + ((u - 1) % 3) * STAGE) + wave * (32 * 68);
        const int rp = lane >> 3, c8 = (lane & 7) * 8;  // read-back: pixel rp (+8 per pass), channels c8..
        f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
        if (p.bias) {
            b0 = *reinterpret_cast<const f32x4*>(p.bias + n_blk + c8);
            b1 = *reinterpret_cast<const f32x4*>(p.bias + n_blk + c8 + 4);
        }
#pragma unroll
        for (int i = 0; i < FRAGS; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f32x4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                    *reinterpret_cast<f32x4*>(ep + lr * 68 + j * 32 + 8 * q + 4 * lh) = v;
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own wave's tile only: no barrier
#pragma unroll
            for (int ps = 0; ps < 4; ++ps) {
                const int px = ps * 8 + rp;
                const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + px * 68 + c8);
                const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + px * 68 + c8 + 4);
                epi_store8_b(p, (long long)(m_blk + wave * 128 + i * 32 + px), n_blk + c8, v0, v1, b0, b1);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next fragment's writes
        }
        tile += per_xcd;
        if (tile >= t_end) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing (dead) loads drain before exit
}

// ---------------------------------------------------------------- row-stream bf16 kernel
// The 128-wide, 64 -> 64 channel 3x3 convolutions of config C3's top level (inc.conv2 and
// up4.conv2, fwd and dgrad: 4 of the 6 top-level launches, ~77 us each on the halo kernel at 0.2 of
// the MFMA peak).  The halo kernel re-loads the 36.9 KB of a 32-channel group's weights for every
// 256-pixel tile and its (R+2)/R = 2x halo; here a block keeps ALL 9 x 64 x 64 weights resident in
// LDS (72 KB, loaded once) and walks a strip of 16 output rows of one image, one row per step:
// input rows stream through a 5-row LDS ring by LDS-DMA (16 KB per row, issued two steps ahead),
// so each input byte is fetched once per strip and the per-row work is 72 MFMAs per wave.
//   block: 4 waves (one per SIMD, one block per CU: 153 KB of LDS), wave = 32 pixels x 64 output
//     channels (2 fragments; 1 pixel + 2 weight fragment reads per 2 MFMAs), fragment reads two
//     k-steps ahead;
//   LDS images: 128-byte rows (64 bf16 channels) with 16-byte chunk c stored at c ^ ((row >> 1) & 7)
//     (conflict-free ds_read_b128 for 32 consecutive rows at any shift; the DMA lanes pick their
//     source chunk accordingly), ring rows of 130 pixels whose two padding pixels stay zero;
//   epilogue: bias preloaded once, mask / residual / accumulate operands of the row loaded at the
//     start of its step (they land under its MFMAs), 8-byte stores.
// K order (32-channel group, tap, 16-channel half) and the MFMA sequence per accumulator are
// igemm_bf16_halo_kernel's, so the two are bit-identical.  Host: rows_ok_b.
#ifndef PU_RS_PD
#define PU_RS_PD 4      // k-steps of fragment reads in flight (A/B builds: 2, 3, 4)
#endif
#ifndef PU_RS_ABL
#define PU_RS_ABL 0     // ablation builds only (timing): 1 no output stores, 2 no MFMAs, 3 no per-row wait/barrier,
// 4 in-loop row loads with an empty range (no HBM reads), 5 weights with an empty range
#endif
constexpr int RS_W = 128, RS_ROWS = 16, RS_RING = 5;
constexpr int RS_ROWB = (RS_W + 2) * 128;                        // 16640 B per ring row
constexpr int RS_WB = 9 * 64 * 128;                              // 73728 B of weights
constexpr int RS_LDS = RS_RING * RS_ROWB + RS_WB;                // 156928 B

__global__ __launch_bounds__(256) void igemm_bf16_rows_kernel(const IgemmBf16Params p) {
    extern __shared__ __attribute__((aligned(1024))) char rs_lds[];
    char* const wl = rs_lds + RS_RING * RS_ROWB;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;
    const int strips = p.Ho / RS_ROWS;
    const int b = blockIdx.x / strips;
    const int r0 = (blockIdx.x - b * strips) * RS_ROWS;
    const unsigned xbytes = (unsigned)p.in_pix * 128u;           // 64 bf16 channels per pixel
    const unsigned wbytes = (unsigned)(64 * p.k_pad * 2);

    // padding pixels 0 and 129 of every ring row: zero, never written by the DMA
    if (tid < RS_RING * 2 * 8) {
        const int row = tid >> 4, side = (tid >> 3) & 1, ch = tid & 7;
        *reinterpret_cast<f32x4*>(rs_lds + row * RS_ROWB + side * (RS_W + 1) * 128 + ch * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // weights [tap][n][64 channels] (chunk-swizzled by n), 72 x 1 KB, 18 per wave
#pragma unroll
    for (int j = 0; j < 18; ++j) {
        const int I = wave + 4 * j;
        const int row = I * 8 + (lane >> 3);
        const int tap = row >> 6, n = row & 63;
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        const unsigned vo = (unsigned)(n * p.k_pad + (c >> 2) * 288 + tap * 32 + (c & 3) * 8) * 2u;
        lean_load(p.wt, PU_RS_ABL == 5 ? 0u : wbytes, wl + I * 1024, vo, 0u);
    }
    // input row ir of image b -> ring slot (ir + 1) % RS_RING, pixels 1 .. 128 (4 x 1 KB per wave)
    unsigned xvo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int I = wave + 4 * j;
        const int col = I * 8 + (lane >> 3);
        const int c = (lane & 7) ^ (((col + 1) >> 1) & 7);
        xvo[j] = (unsigned)(col * 64 + c * 8) * 2u;
    }
    auto load_row = [&](int ir) {
        const bool ok = ir >= r0 - 1 && ir <= r0 + RS_ROWS && (unsigned)ir < (unsigned)p.Hi;
        char* base = rs_lds + ((ir + 1) % RS_RING) * RS_ROWB + 128;
        const unsigned soff = ok ? (unsigned)((b * p.Hi + ir) * RS_W) * 128u : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            lean_load(p.src0, ok && !(PU_RS_ABL == 4 && ir > r0 + 2) ? xbytes : 0u, base + (wave + 4 * j) * 1024, xvo[j], soff);
    };
    load_row(r0 - 1);
    load_row(r0);
    load_row(r0 + 1);
    load_row(r0 + 2);

    // per-lane fragment offsets: pixel fragment (tap column ts, 16-channel step u), weight (u)
    const int q0 = wave * 32;
    unsigned xoff[3][4], woff[4];
#pragma unroll
    for (int ts = 0; ts < 3; ++ts) {
        const int pl = q0 + lr + ts;                              // ring pixel (col + 1)
#pragma unroll
        for (int u = 0; u < 4; ++u) xoff[ts][u] = (unsigned)(pl * 128 + (((2 * u + lh) ^ ((pl >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) woff[u] = (unsigned)(lr * 128 + (((2 * u + lh) ^ ((lr >> 1) & 7)) << 4));

    // bias of this lane's 8 channel quads (n = j*32 + 8q + 4lh)
    f32x4 bias4[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            bias4[j][q] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + j * 32 + 8 * q + 4 * lh) : f32x4{0.f, 0.f, 0.f, 0.f};
    const bool has_m = p.mask0 != nullptr, has_r = p.resid != nullptr, has_a = (p.flags & PU_EPI_ACCUM) != 0;
    const int E = 8 * ((has_m ? 1 : 0) + (has_r ? 1 : 0) + (has_a ? 1 : 0));
    // epilogue operands of row rr, loaded after the previous row's stores: they land during row
    // rr's MFMAs, and waiting for them does not wait for the row loads issued later
    bf16x4 mv[2][4], rv[2][4], av[2][4];
    auto prefetch = [&](int rr) {
        const long long mm = (long long)(b * p.Ho + rr) * RS_W + q0 + lr;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long off = mm * 64 + j * 32 + 8 * q + 4 * lh;
                if (has_m) mv[j][q] = *reinterpret_cast<const bf16x4*>(p.mask0 + off);
                if (has_r) rv[j][q] = *reinterpret_cast<const bf16x4*>(p.resid + off);
                if (has_a) av[j][q] = *reinterpret_cast<const bf16x4*>(p.dst0 + off);
            }
    };
    if (E) prefetch(r0);

    for (int r = r0; r < r0 + RS_ROWS; ++r) {
        // input row r+1 landed (issued two steps ago; issued after it: stores (8), epilogue loads (E),
        // one row (4), stores, epilogue loads - over-waiting where the count is not exact)
        if (r == r0) {
            wait_vm_plus<4>(E);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // + the padding zeros
        } else if (PU_RS_ABL == 3) asm volatile("" ::: "memory");
        else if (r == r0 + 1) wait_vm_plus<12>(2 * E);
        else wait_vm_plus<20>(2 * E);
        if (PU_RS_ABL != 3 || r == r0) __builtin_amdgcn_s_barrier();   // ... for every wave; slot of row r-2 free
        asm volatile("" ::: "memory");
        const long long m = (long long)(b * p.Ho + r) * RS_W + q0 + lr;
        load_row(r + 3);

        const int sb[3] = {(r % RS_RING) * RS_ROWB, ((r + 1) % RS_RING) * RS_ROWB, ((r + 2) % RS_RING) * RS_ROWB};
        f32x16 acc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
        // fragment reads RS_PD k-steps ahead (3 x 16 B per step; 12 in flight at RS_PD = 4 - one wave
        // per SIMD has no partner wave to cover the LDS latency: at 2 steps ahead the loop ran at the
        // read latency, 3.4 us per row with or without its MFMAs)
        constexpr int RS_PD = PU_RS_PD, NB = RS_PD + 1;
        bf16x8 fx[NB], fw[NB][2];
        auto rd = [&](auto S) {
            constexpr int s = decltype(S)::value;
            constexpr int g = s / 18, t = (s % 18) / 2, kk = s % 2, u = g * 2 + kk;
            fx[s % NB] = *reinterpret_cast<const bf16x8*>(rs_lds + sb[t / 3] + xoff[t % 3][u]);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                fw[s % NB][j] = *reinterpret_cast<const bf16x8*>(wl + (t * 64 + j * 32) * 128 + woff[u]);
        };
        static_for<RS_PD>([&](auto S) { rd(S); });
        static_for<36>([&](auto S) {
            constexpr int s = decltype(S)::value;
            if constexpr (s + RS_PD < 36) rd(std::integral_constant<int, s + RS_PD>{});
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (PU_RS_ABL == 2) acc[j][s & 15] += __builtin_bit_cast(float, __builtin_shufflevector(fw[s % NB][j], fx[s % NB], 0, 9));
                else acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[s % NB][j], fx[s % NB], acc[j], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        });

        if (E) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // this row's epilogue operands
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[j][4 * q + e];
                if (p.bias) v += bias4[j][q];
                if (has_r) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += (float)rv[j][q][e];
                }
                if (p.flags & PU_EPI_RELU) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                }
                if (has_m) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) if (!((float)mv[j][q][e] > 0.f)) v[e] = 0.f;
                }
                if (has_a) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += (float)av[j][q][e];
                }
                bf16x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (__bf16)v[e];
                if (PU_RS_ABL != 1 || (p.flags & (1 << 30))) *reinterpret_cast<bf16x4*>(p.dst0 + m * 64 + j * 32 + 8 * q + 4 * lh) = o;
            }
        if (E && r + 1 < r0 + RS_ROWS) prefetch(r + 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");             // the trailing (empty) row loads drain
}

__global__ __launch_bounds__(256) void igemm_bf16_splitk_epilogue_kernel(const IgemmBf16Params p) {
    const int nq = p.N >> 2;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)p.M * nq) return;
    const int m = (int)(idx / nq);
    const int n = (int)(idx - (long long)m * nq) * 4;
    const long long mn = (long long)p.M * p.N;
    const float* src = p.part + (long long)m * p.N + n;
    f32x4 v = *reinterpret_cast<const f32x4*>(src);
    for (int z = 1; z < p.ksplit; ++z) v += *reinterpret_cast<const f32x4*>(src + z * mn);
    epi_store4_b(p, epi_row_b(p, m), n, v);
}

static int blocks_for_b(long long M, int N, int bm, int bn) { return ceil_div(M, bm) * ceil_div(N, bn); }

static void choose_tile_b(long long M, int N, int* bm, int* bn) {
    const int target = 480;
    if (N <= 64) {
        if (blocks_for_b(M, N, 256, 64) >= target) { *bm = 256; *bn = 64; }
        else if (blocks_for_b(M, N, 128, 64) >= target) { *bm = 128; *bn = 64; }
        else { *bm = 64; *bn = 64; }
    } else {
        if (blocks_for_b(M, N, 128, 128) >= target) { *bm = 128; *bn = 128; }
        else if (blocks_for_b(M, N, 128, 64) >= target) { *bm = 128; *bn = 64; }
        else { *bm = 64; *bn = 64; }
    }
}

static void plan_split_b(const pu_conv_args* a, long long M, int bm, int bn, int* ksplit, int* t_per) {
    const int T = a->k_pad / BK16;
    *ksplit = 1;
    *t_per = T;
    const int occ = (bm == 256) ? 2 : (bm == 128 && bn == 128) ? 3 : 4;
    const int blocks = blocks_for_b(M, a->n, bm, bn);
    int ks = (256 * occ) / blocks;
    if (ks > T / 4) ks = T / 4;
    if (ks < 2) return;
    *t_per = ceil_div(T, ks);
    *ksplit = ceil_div(T, *t_per);
}

// the halo kernel: 3x3 / s1 / p1 same-size, width 32 / 64 / 128, whole 256-pixel row blocks,
// 32-channel groups, 64-channel output tiles, plain (non-SHUFFLE2) epilogue
static bool halo_ok_b(const pu_conv_args* a) {
    const int C = a->c0 + a->c1;
    if (a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1 || a->cgroup != 32) return false;
    if (a->in_h != a->out_h || a->in_w != a->out_w || (a->flags & (PU_EPI_SHUFFLE2 | PU_CONV_NO_HALO))) return false;
    if (!(a->out_w == 32 || a->out_w == 64 || a->out_w == 128) || a->out_h % (256 / a->out_w)) return false;
    if (a->k_pad != 9 * C || a->n % HB_BN) return false;
    if ((long long)a->batch * a->in_h * a->in_w * (a->c0 > a->c1 ? a->c0 : a->c1) >= (1LL << 31)) return false;
    if ((long long)a->k_pad * a->n >= (1LL << 31)) return false;
    return true;
}

static int device_cus_b() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        cus[dev] = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n >= 8) ? n : 256;
    }
    return cus[dev];
}

// the DMA-ring halo kernel: the halo kernel's shapes with 512-pixel row blocks (R = 512 / W rows);
// opt-in with PU_CONV_HALO_DMA (A/B runs, its bit-identity test); the default is the register-staged
// kernel, which the Python host runs too
static bool halo2_ok_b(const pu_conv_args* a) {
    // its epilogue stores 8 channels (16 B) per lane: 8-channel split point, 16-byte-aligned tensors
    const uintptr_t ae = (uintptr_t)a->dst0 | (uintptr_t)a->dst1 | (uintptr_t)a->mask0 | (uintptr_t)a->mask1 |
                         (uintptr_t)a->resid;
    return halo_ok_b(a) && (a->flags & PU_CONV_HALO_DMA) && a->out_h % (512 / a->out_w) == 0 && a->n0 % 8 == 0 &&
           (ae & 15) == 0;
}

// the row-stream kernel: the halo kernel's 3x3 / s1 / p1 shapes restricted to width 128, one
// 64-channel source, 64 output channels into one destination, 16-row strips; PU_BF16_ROWS=0 keeps
// the halo kernel (A/B runs)
static bool rows_ok_b(const pu_conv_args* a) {
    static const bool on = [] {
        const char* e = getenv("PU_BF16_ROWS");
        return !(e && e[0] == '0');
    }();
    if (!on || !halo_ok_b(a) || (a->flags & PU_CONV_HALO_DMA)) return false;   // the DMA ring when opted in
    if (a->out_w != RS_W || a->out_h % RS_ROWS || a->c0 != 64 || a->c1 != 0 || a->n != 64) return false;
    if (a->n0 != 0 && a->n0 != 64) return false;
    return (long long)a->batch * a->in_h * a->in_w * 128 < (1LL << 31);
}

template <int W>
static size_t halo2_lds_bytes() {
    constexpr int HP = (512 / W + 2) * (W + 2);
    constexpr int STAGE = (HP * 2 + 63) / 64 * 1024 + 18 * 1024;
    return 3 * STAGE + 1024;
}

// the lean kernel: 3x3, 32-channel K groups, one pixel stride for both sources, K == k_pad,
// byte offsets within 2 GB
static bool lean_ok_b(const pu_conv_args* a) {
    const int C = a->c0 + a->c1;
    if (a->kh != 3 || a->kw != 3 || a->cgroup != 32) return false;
    if (a->c1 != 0 && a->c1 != a->c0) return false;
    if (a->k_pad != 9 * C || (a->flags & PU_EPI_SHUFFLE2)) return false;
    const long long shift = (long long)a->pad * a->in_w + a->pad;
    if (((long long)a->batch * a->in_h * a->in_w + shift) * a->c0 * 2 >= (1LL << 31)) return false;
    if ((long long)a->k_pad * a->n * 2 >= (1LL << 31)) return false;
    return true;
}

// lean tiles: 256 x 128 (N > 64) or 256 x 64, 4 waves, ~2 resident blocks per CU (72 / 61 KB of
// LDS); small pixel grids split K on group boundaries until ~2 blocks per CU
// 128 x 128 tiles instead of a K split when they alone give a round of blocks (C3's 16^2 level:
// 256 tiles; the split's fp32 partials cost 2 x 67 MB per layer there): l4 fwd / dgrad 65 / 70 ->
// 56 / 56 us, C3 +0.8 %; PU_BF16_LEAN128=0 keeps the split (A/B runs)
static bool lean128_on() {
    static const bool on = [] {
        const char* e = getenv("PU_BF16_LEAN128");
        return !(e && e[0] == '0');
    }();
    return on;
}

static bool smallm_on() {             // PU_BF16_SMALLM=0: the 256 x 128 split (A/B runs)
    static const bool on = [] {
        const char* e = getenv("PU_BF16_SMALLM");
        return !(e && e[0] == '0');
    }();
    return on;
}

static void plan_lean_b(const pu_conv_args* a, long long M, int* bm, int* bn, int* ksplit, int* t_per) {
    *bm = 256;
    *bn = a->n > 64 ? 128 : 64;
    const int T = a->k_pad / BK16;
    *ksplit = 1;
    *t_per = T;
    const int tiles = blocks_for_b(M, a->n, *bm, *bn);
    const int target = 512;
    if (tiles >= target - target / 16) return;
    const int t128 = blocks_for_b(M, a->n, 128, 128);
    if (lean128_on() && a->n > 64 && t128 >= 240) {
        *bm = 128;
        return;
    }
    // small pixel grids (the 8^2 / 16^2 levels): 128 x 128 tiles split to ~2 blocks per CU.  The
    // 256 x 128 tiles split 8 / 16 ways wrote 8 - 16 fp32 partial tiles per output (67 MB per 8^2
    // layer, read back by the split epilogue) for blocks that ran 1 - 2 channel groups each
    // (PU_BF16_LEAN128=0 with t128 >= 240 keeps the old 256 x 128 split: the A/B switch above)
    if (smallm_on() && a->n > 64 && (lean128_on() || t128 < 240)) {
        int k2 = ceil_div(target, t128);
        if (k2 > T / 9) k2 = T / 9;
        *bm = 128;
        if (k2 >= 2) {
            *t_per = ceil_div(ceil_div(T, k2), 9) * 9;
            *ksplit = ceil_div(T, *t_per);
        }
        return;
    }
    int ks = ceil_div(target, tiles);
    if (ks > T / 9) ks = T / 9;
    if (ks < 2) return;
    *t_per = ceil_div(ceil_div(T, ks), 9) * 9;
    *ksplit = ceil_div(T, *t_per);
}

static int setup_bf16(const pu_conv_args* a, IgemmBf16Params* pp, long long* Mout) {
    PU_REQUIRE(a != nullptr, "pu_conv_igemm_bf16: null args");
    PU_REQUIRE(a->batch > 0 && a->in_h > 0 && a->in_w > 0 && a->out_h > 0 && a->out_w > 0, "pu_conv_igemm_bf16: bad grid");
    PU_REQUIRE(a->kh > 0 && a->kw > 0 && a->stride > 0 && a->pad >= 0 && a->kh * a->kw <= 32, "pu_conv_igemm_bf16: bad taps");
    PU_REQUIRE(a->src0 && a->weight && a->dst0 && a->n > 0, "pu_conv_igemm_bf16: operands");
    PU_REQUIRE(a->chan_scale == nullptr, "pu_conv_igemm_bf16: chan_scale is an fp32-path epilogue");
    PU_REQUIRE(!(a->flags & PU_EPI_OUT_BF16), "pu_conv_igemm_bf16: PU_EPI_OUT_BF16 is pu_conv_igemm's stem flag");
    PU_REQUIRE(a->c0 % 32 == 0 && a->c1 % 32 == 0 && a->c0 > 0 && (a->c1 == 0 || a->src1),
               "pu_conv_igemm_bf16: channel counts (%d, %d) must be multiples of 32", a->c0, a->c1);
    PU_REQUIRE(a->cgroup == 0 || a->cgroup == 32, "pu_conv_igemm_bf16: cgroup must be 0 or 32");
    const int C = a->c0 + a->c1;
    const int K = a->kh * a->kw * C;
    PU_REQUIRE(a->k_pad >= K && a->k_pad % BK16 == 0, "pu_conv_igemm_bf16: k_pad %d (K %d) must be a multiple of 32", a->k_pad, K);
    const bool shuffle = a->flags & PU_EPI_SHUFFLE2;
    const int n0 = shuffle ? a->n : a->n0;
    PU_REQUIRE(a->n % 4 == 0 && n0 % 4 == 0 && (!shuffle || (a->n / 4) % 4 == 0), "pu_conv_igemm_bf16: channel alignment");
    PU_REQUIRE(shuffle || (n0 > 0 && n0 <= a->n && (n0 == a->n || a->dst1)), "pu_conv_igemm_bf16: n0 / dst1");
    PU_REQUIRE(!(a->flags & PU_EPI_RESID) || (a->resid && !shuffle && n0 == a->n), "pu_conv_igemm_bf16: RESID");
    const uintptr_t al = (uintptr_t)a->src0 | (uintptr_t)a->src1 | (uintptr_t)a->weight;
    PU_REQUIRE((al & 15) == 0, "pu_conv_igemm_bf16: sources / weight must be 16-byte aligned");
    const uintptr_t ae = (uintptr_t)a->dst0 | (uintptr_t)a->dst1 | (uintptr_t)a->mask0 | (uintptr_t)a->mask1 |
                         (uintptr_t)a->resid;
    PU_REQUIRE((ae & 7) == 0 && ((uintptr_t)a->bias & 15) == 0, "pu_conv_igemm_bf16: epilogue alignment");
    const long long M = (long long)a->batch * a->out_h * a->out_w;
    PU_REQUIRE(M < (1LL << 31), "pu_conv_igemm_bf16: too many pixels");
    IgemmBf16Params& p = *pp;
    p.M = (int)M; p.N = a->n; p.K = K; p.k_pad = a->k_pad;
    p.Hi = a->in_h; p.Wi = a->in_w; p.Ho = a->out_h; p.Wo = a->out_w;
    p.kh = a->kh; p.kw = a->kw; p.stride = a->stride; p.pad = a->pad;
    p.C = C; p.c0 = a->c0; p.c1 = a->c1;
    p.src0 = (const __bf16*)a->src0; p.src1 = (const __bf16*)a->src1; p.wt = (const __bf16*)a->weight;
    p.bias = a->bias;
    p.dst0 = (__bf16*)a->dst0; p.dst1 = (__bf16*)a->dst1;
    p.mask0 = (const __bf16*)a->mask0; p.mask1 = (const __bf16*)a->mask1;
    p.resid = (a->flags & PU_EPI_RESID) ? (const __bf16*)a->resid : nullptr;
    p.n0 = n0; p.flags = a->flags;
    p.cgroup = a->cgroup; p.taps = a->kh * a->kw;
    p.shuf_h = a->shuf_h ? a->shuf_h : 2 * a->out_h;
    p.shuf_w = a->shuf_w ? a->shuf_w : 2 * a->out_w;
    p.shuf_off = a->shuf_off;
    p.dWo = make_fastdiv(a->out_w); p.dHo = make_fastdiv(a->out_h);
    p.dC = make_fastdiv(C); p.dKw = make_fastdiv(a->kw); p.dCo = make_fastdiv(shuffle ? a->n / 4 : 1);
    p.dTaps = make_fastdiv(p.taps);
    p.in_pix = a->batch * a->in_h * a->in_w;
    *Mout = M;
    return PU_OK;
}

}  // namespace pu

using namespace pu;

extern "C" size_t pu_conv_igemm_bf16_workspace_bytes(const pu_conv_args* a) {
    IgemmBf16Params p;
    long long M;
    if (setup_bf16(a, &p, &M) != PU_OK) return 0;
    int bm, bn, ks, tp;
    if (halo_ok_b(a)) return 0;
    if (lean_ok_b(a)) {
        plan_lean_b(a, M, &bm, &bn, &ks, &tp);
    } else {
        choose_tile_b(M, a->n, &bm, &bn);
        plan_split_b(a, M, bm, bn, &ks, &tp);
    }
    return ks > 1 ? (size_t)ks * (size_t)M * (size_t)a->n * sizeof(float) : 0;
}

extern "C" int pu_conv_igemm_bf16(const pu_conv_args* a, void* stream) {
    IgemmBf16Params p;
    long long M;
    int st = setup_bf16(a, &p, &M);
    if (st != PU_OK) return st;
    const int N = a->n;
    hipStream_t s = as_stream(stream);
    if (rows_ok_b(a)) {
        p.ksplit = 1;
        p.gn = 1;
        const dim3 rgrid((unsigned)(a->batch * (a->out_h / RS_ROWS)));
        hipLaunchKernelGGL(igemm_bf16_rows_kernel, rgrid, dim3(256), RS_LDS, s, p);
        return check_launch("pu_conv_igemm_bf16 (rows)");
    }
    if (halo2_ok_b(a)) {
        p.ksplit = 1;
        p.gn = N / H2_BN;
        const long long tiles = M / 512 * p.gn;
        const long long per_xcd = ceil_div(tiles, 8LL);
        const int blocks_per_xcd = device_cus_b() / 8;        // one block per CU
        const dim3 hgrid((unsigned)(8 * (per_xcd < blocks_per_xcd ? per_xcd : blocks_per_xcd)));
        if (a->out_w == 128)
            hipLaunchKernelGGL((igemm_bf16_halo2_kernel<128>), hgrid, dim3(H2_NT), halo2_lds_bytes<128>(), s, p);
        else if (a->out_w == 64)
            hipLaunchKernelGGL((igemm_bf16_halo2_kernel<64>), hgrid, dim3(H2_NT), halo2_lds_bytes<64>(), s, p);
        else
            hipLaunchKernelGGL((igemm_bf16_halo2_kernel<32>), hgrid, dim3(H2_NT), halo2_lds_bytes<32>(), s, p);
        return check_launch("pu_conv_igemm_bf16 (halo2)");
    }
    if (halo_ok_b(a)) {
        p.ksplit = 1;
        p.gn = N / HB_BN;
        const long long tiles = M / 256 * p.gn;
        const long long per_xcd = ceil_div(tiles, 8LL);
        const int blocks_per_xcd = 2 * device_cus_b() / 8;   // 2 resident blocks per CU
        const dim3 hgrid((unsigned)(8 * (per_xcd < blocks_per_xcd ? per_xcd : blocks_per_xcd)));
        if (a->out_w == 128) hipLaunchKernelGGL((igemm_bf16_halo_kernel<128>), hgrid, dim3(HB_NT), 0, s, p);
        else if (a->out_w == 64) hipLaunchKernelGGL((igemm_bf16_halo_kernel<64>), hgrid, dim3(HB_NT), 0, s, p);
        else hipLaunchKernelGGL((igemm_bf16_halo_kernel<32>), hgrid, dim3(HB_NT), 0, s, p);
        return check_launch("pu_conv_igemm_bf16 (halo)");
    }
    int bm, bn;
    const bool lean = lean_ok_b(a);
    if (lean) {
        plan_lean_b(a, M, &bm, &bn, &p.ksplit, &p.t_per);
    } else {
        choose_tile_b(M, N, &bm, &bn);
        plan_split_b(a, M, bm, bn, &p.ksplit, &p.t_per);
    }
    p.gn = ceil_div(N, bn);
    if (p.ksplit > 1 && (!a->workspace || a->ws_bytes < (size_t)p.ksplit * M * N * sizeof(float))) {
        p.ksplit = 1;
        p.t_per = a->k_pad / BK16;
    }
    p.part = (float*)a->workspace;
    const dim3 grid(ceil_div(M, bm) * p.gn * p.ksplit);
    if (lean && bm == 128) hipLaunchKernelGGL((igemm_bf16_lean_kernel<128, 128, 2, 2, 4>), grid, dim3(256), 0, s, p);
    else if (lean && bn == 128) hipLaunchKernelGGL((igemm_bf16_lean_kernel<256, 128, 2, 2, 4>), grid, dim3(256), 0, s, p);
    else if (lean) hipLaunchKernelGGL((igemm_bf16_lean_kernel<256, 64, 4, 1, 4>), grid, dim3(256), 0, s, p);
    else if (bm == 256) hipLaunchKernelGGL((igemm_bf16_kernel<256, 64, 4, 1, 3>), grid, dim3(256), 0, s, p);
    else if (bm == 128 && bn == 128) hipLaunchKernelGGL((igemm_bf16_kernel<128, 128, 2, 2, 3>), grid, dim3(256), 0, s, p);
    else if (bm == 128) hipLaunchKernelGGL((igemm_bf16_kernel<128, 64, 2, 2, 3>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((igemm_bf16_kernel<64, 64, 2, 2, 3>), grid, dim3(256), 0, s, p);
    if (p.ksplit > 1) {
        const long long threads = M * (N / 4);
        hipLaunchKernelGGL(igemm_bf16_splitk_epilogue_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, p);
    }
    return check_launch("pu_conv_igemm_bf16");
}

extern "C" int pu_conv_igemm_bf16_tile(const pu_conv_args* a, int* bm, int* bn, int* ksplit, int* kind) {
    IgemmBf16Params p;
    long long M;
    int st = setup_bf16(a, &p, &M);
    if (st != PU_OK) return st;
    int ks, tp;
    if (rows_ok_b(a)) {               // the row-stream kernel: one 128-pixel row x 64 channels per step
        *bm = 128;
        *bn = 64;
        if (ksplit) *ksplit = 1;
        if (kind) *kind = 3;
        return PU_OK;
    }
    if (halo2_ok_b(a)) {              // the DMA-ring halo kernel: 512 pixels x 64 channels
        *bm = 512;
        *bn = H2_BN;
        if (ksplit) *ksplit = 1;
        if (kind) *kind = 2;
        return PU_OK;
    }
    if (halo_ok_b(a)) {               // the halo kernel: 256 pixels x 64 channels, no split
        *bm = 256;
        *bn = HB_BN;
        if (ksplit) *ksplit = 1;
        if (kind) *kind = 2;
        return PU_OK;
    }
    if (kind) *kind = lean_ok_b(a) ? 1 : 0;
    if (lean_ok_b(a)) {
        plan_lean_b(a, M, bm, bn, &ks, &tp);
    } else {
        choose_tile_b(M, a->n, bm, bn);
        plan_split_b(a, M, *bm, *bn, &ks, &tp);
    }
    if (ksplit) *ksplit = (ks > 1 && a->workspace && a->ws_bytes >= (size_t)ks * M * a->n * sizeof(float)) ? ks : 1;
    return PU_OK;
}
