// Winograd F(2x2, 3x3) convolution for the fp32 3x3/s1/p1 layers, on the exact 6-product bf16
// MFMA scheme of igemm.hip (each fp32 product as hi/mid/lo bf16 terms, fp32 accumulation).
//
// Replaces (yaricom/Plastic-UNet): the nn.Conv2d(k=3, p=1) of double_conv (src/unet/unet_p.py:
// 184-201) forward and backward-data, over the skip concat torch.cat([x2, x1], 1) (unet_p.py:248)
// without materialising it - the same layers igemm_x6_lean_kernel computes directly.
//
// Arithmetic (Lavin & Gray's F(2x2,3x3)): a 2x2 output tile y of one (image, channel n) is
//   y = A^T [ sum_c (G g_nc G^T) (.) (B^T d_c B) ] A
// with d_c the 4x4 input window of channel c, g_nc the 3x3 kernel, (.) the element-wise product
// over the 16 positions xi = (i, j), and
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],  G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1],
//   A^T = [1 1 1 0; 0 1 -1 -1].
// So each xi is an independent GEMM  M_xi[n][tile] = sum_c U_xi[n][c] V_xi[c][tile]  with K = C
// instead of 9C: 16 products per 4 outputs instead of 36 (2.25x fewer MFMAs).  U = G g G^T is
// formed in fp64 once per weight update (pu_pack_wino) and rounded to fp32; V = B^T d B and the
// output transform are fp32 adds/subtracts (no multiplications: the transforms only scale by +-1).
// The numerics are fp32 arithmetic throughout (tests/test_precision_gpu.py bounds vs fp64).
//
// Kernel (one block = 64 tiles x 64 output channels, 4 waves as 2 x 2, each wave a 32 x 32 MFMA
// tile for all 16 xi: 16 accumulators of 16 fp32 = 256 AGPRs, one wave per SIMD):
//   * a 16-channel chunk is split into 4 sub-stages, one per row i of B^T (xi = 4i .. 4i+3);
//   * a sub-stage's LDS slot holds V_xi (4 xi x 3 planes x 64 tiles x 16 channels, bf16) and
//     U_xi (4 xi x 3 planes x 64 channels x 16), 24 KB each; 2 slots, one barrier per sub-stage;
//   * thread (tile tt, channel quad q) keeps the 4x4 window of its 4 channels in registers (16
//     buffer_load_dwordx4, out-of-image pixels fall outside the buffer range and read 0), two
//     chunks in flight (two register banks), and during sub-stage s forms V of sub-stage s+1 -
//     8 adds and one exact 3-term split per (xi row, 4 channels) - while the MFMAs of s run;
//   * U comes pre-split from HBM/L2 by buffer_load ... lds (6 x 1 KB pieces per wave per
//     sub-stage); 32-byte LDS rows with the 16-byte halves swapped on rows 8..15 mod 16 make
//     every ds_read_b128 operand read and ds_write_b64 V store conflict-free;
//   * epilogue: the output transform is lane-local (a lane holds all 16 xi of the same (tile,
//     4 channels)), then igemm's float4 epilogue (bias, ReLU, residual, masks, concat split,
//     accumulate) per output pixel; split-K writes pre-bias partial tiles for
//     igemm_splitk_epilogue_kernel.
#include "conv_common.h"

#ifndef PU_NO_ILV
#define PU_NO_ILV 0   // 1: leave MFMA / VALU placement to the scheduler (A/B builds)
#endif
// wino_x6_kernel ablations (timing only, wrong results): 1 no MFMAs, 2 no V formation (VALU + LDS
// stores), 3 no window loads, 4 no per-sub-stage barrier (the waits stay), 5 no U DMA, 6 no output
// stores, 7 no bias loads
#ifndef PU_WF_ABL
#define PU_WF_ABL 0
#endif


namespace pu {

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

constexpr int WG_BM = 64;                      // tiles per block
constexpr int WG_BN = 64;                      // output channels per block
constexpr int WG_HALF = 4 * 3 * 64 * 32;       // bytes of V (or U) in one sub-stage slot
constexpr int WG_SLOT = 2 * WG_HALF;

struct WinoParams {
    IgemmParams p;        // grid (Ho == Hi, Wo == Wi), sources, epilogue, split-K partials
    const __bf16* U;      // [C/16][16 xi][3 planes][N][16] (pu_pack_wino)
    int tiles;            // batch * Ho/2 * Wo/2
    int kc_per;           // 16-channel chunks per K split (even)
    int gm;               // tile blocks
    FastDiv dTw, dTh;     // tile index -> (image, tile row, tile column)
    unsigned a_bytes;     // extent of the shifted pixel buffers
    unsigned u_bytes;     // extent of U
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    void* ub = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(ub, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// epilogue operand load / store through a buffer descriptor (out-of-range offsets: zeros / dropped)
__device__ __forceinline__ f32x4 epi_ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void epi_st4(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

// One block walks work items (tile block x channel block x K split): PERSIST - one block per CU,
// each XCD a contiguous range of items, channel block slowest (the items an XCD runs at once share
// one U slice in its L2); otherwise one item per block (XCD-aware order).
//
// The chunks of consecutive items form one stream: the loads a chunk issues for "the next chunk"
// (its window rows, the first U pieces) target the next item's first chunk at an item's end, so
// the next item's first sub-stages are in flight during this item's last chunk and epilogue
// instead of waiting out a cold HBM round trip per item.
//
// Sub-stage s (chunk kc, row i): V of s was formed during s-1 (V slots i & 1), U of s was issued
// three sub-stages earlier (U slots i: a 4-slot ring).  Every load is issued unconditionally
// (past the last item the buffer range is empty and zeros land), so the wait counts are
// compile-time exact: issued after U(s) are the window rows of s-3, s-2, s-1 (4 / 4 / 8 / 0 row
// loads in sub-stages i = 0 / 1 / 2 / 3) and U(s+1), U(s+2) (3 pieces each).
#ifndef PU_WPP_STAMP
#define PU_WPP_STAMP 0     // diagnostic build: block 0's per-wave s_memtime before / after every barrier
#endif
#if PU_WPP_STAMP
constexpr int PU_WPP_NSTAMP = 512;
__device__ unsigned long long pu_wpp_stamp_buf[8 * PU_WPP_NSTAMP];
// lane 0 of block 0's waves: shader-clock stamp k of wave w (diagnostic builds only; the stamp
// stores are vector-memory ops and shift the kernel's counted vmcnt waits - timing only)
__device__ __forceinline__ void wpp_stamp_at(int wave, int& n) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && n < PU_WPP_NSTAMP) pu_wpp_stamp_buf[wave * PU_WPP_NSTAMP + n] = t;
    ++n;
}
#define WPP_STAMP(w, n) wpp_stamp_at(w, n)
#else
#define WPP_STAMP(w, n) ((void)0)
#endif
template <bool PERSIST>
__global__ __launch_bounds__(512) void wino_x6_kernel(const WinoParams w) {
#pragma clang fp contract(off)
    const IgemmParams& p = w.p;
    // V slots (VALU-stored) and U slots (LDS-DMA) as separate arrays: the compiler then knows the
    // V stores / operand reads do not alias the DMA in flight (no vmcnt(0) before LDS accesses)
    __shared__ __attribute__((aligned(16))) unsigned char ldv0[WG_HALF];
    __shared__ __attribute__((aligned(16))) unsigned char ldv1[WG_HALF];
    __shared__ __attribute__((aligned(16))) unsigned char ldu0[WG_HALF];
    __shared__ __attribute__((aligned(16))) unsigned char ldu1[WG_HALF];
    __shared__ __attribute__((aligned(16))) unsigned char ldu2[WG_HALF];
    __shared__ __attribute__((aligned(16))) unsigned char ldu3[WG_HALF];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, wn = (wave >> 1) & 1, wx = wave >> 2;
    int nst = 0;
    const int per_split = w.gm * p.gn;
    const int total = per_split * p.ksplit;

    // work items of this block: [it, end) with stride step
    int it, end, step;
    if (PERSIST) {
        const int xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
        const int q8 = total >> 3, r8 = total & 7;
        const int start = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
        end = start + q8 + (xcd < r8 ? 1 : 0);
        it = start + local;
        step = (int)(gridDim.x >> 3);
    } else {
        it = xcd_remap(blockIdx.x, gridDim.x);
        end = it + 1;
        step = 1;
    }
    if (it >= end) return;

    // ---- producer role: tile tt of the block, channels 2q, 2q+1 of each 16-channel chunk.
    const int tt = tid >> 3, q = tid & 7;
    const int cs = p.c0;                       // pixel stride (== c1 when c1 != 0)
    const int shift = p.Wi + 1;                // window corner (2ty-1, 2tx-1) >= (-1, -1)
    const unsigned pixb = (unsigned)cs * 4u;
    const float* a0 = p.src0 - (long long)shift * cs;
    const float* a1 = (p.c1 ? p.src1 : p.src0) - (long long)shift * cs;
    // V store address of this thread inside a slot (row tt, its 4-byte pair, swizzled half)
    const int v_st = tt * 32 + (((q >> 2) ^ ((tt >> 3) & 1)) * 16) + (q & 3) * 4;

    // ---- U loader: wave w fills pieces 3w .. 3w+2 (piece P = (j*3 + plane)*2 + row half)
    const unsigned u_lane = (unsigned)((lane >> 1) * 32 + (((lane & 1) ^ ((lane >> 4) & 1)) * 16));
    const unsigned u_row = (unsigned)p.N * 32u;                  // bytes per (xi, plane) block
    unsigned poff[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const int P = wave * 3 + e;
        poff[e] = (unsigned)(P >> 1) * u_row + (unsigned)((P & 1) * 1024);
    }

    // ---- MFMA role: positions j = 2wx, 2wx+1 of every row i; operand rows 32*wn + (lane&31)
    // of U and 32*wm + (lane&31) of V
    const int rd_sw = (((lane >> 5) ^ ((lane >> 3) & 1)) * 16);
    const int u_rd = (32 * wn + (lane & 31)) * 32 + rd_sw + 2 * wx * 3 * 2048;
    const int v_rd = (32 * wm + (lane & 31)) * 32 + rd_sw + 2 * wx * 3 * 2048;

    // an item as the loaders see it: its chunk range, channel block and this thread's window rows
    struct Item {
        int kz, m_blk, n_blk, kc0, kc1;
        unsigned vrow[4];
        bool c0ok, c3ok, live;
    };
    auto decode = [&](int item, Item& I) {
        I.live = item < end;
        I.kz = item / per_split;
        const int rest = item - I.kz * per_split;
        const int nb = rest / w.gm;          // channel block slowest (U slice shared in L2)
        I.m_blk = (rest - nb * w.gm) * WG_BM;
        I.n_blk = nb * WG_BN;
        I.kc0 = I.kz * w.kc_per;
        I.kc1 = min(p.C / 16, I.kc0 + w.kc_per);
        const int m = I.m_blk + tt;
        int ty = 0, tx = 0, b = 0;
        const bool mv = I.live && m < w.tiles;
        if (mv) {
            const int t2 = fdiv(m, w.dTw);
            tx = m - t2 * (p.Wo >> 1);
            b = fdiv(t2, w.dTh);
            ty = t2 - b * (p.Ho >> 1);
        }
        const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
        const unsigned base = (unsigned)(((b * p.Hi + y0) * p.Wi + x0 + shift) * cs * 4 + q * 8);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            I.vrow[r] = mv && (unsigned)(y0 + r) < (unsigned)p.Hi ? base + (unsigned)(r * p.Wi * cs * 4) : LEAN_OOB;
        I.c0ok = x0 >= 0;
        I.c3ok = x0 + 3 < p.Wi;
    };
    Item cur, nxt;
    decode(it, cur);
    decode(it + step, nxt);

    typedef float f32x2v __attribute__((ext_vector_type(2)));
    f32x2v d[16];
    f32x16 acc[8];                            // [i][jj]

    // window row rr (4 pixels x 2 channels) of chunk kc of item I (zeros past its chunks)
    auto load_row = [&](const Item& I, int kc, int rr) {
        if (PU_WF_ABL == 3) {
#pragma unroll
            for (int ss = 0; ss < 4; ++ss) d[rr * 4 + ss] = f32x2v{1.f + rr, 0.5f * ss};
            return;
        }
        const int c = kc * 16;
        const bool second = c >= p.c0;
        const bool ok = I.live && kc < I.kc1;
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(second ? a1 : a0, ok ? w.a_bytes : 0u);
        const unsigned cb = (unsigned)((second ? c - p.c0 : c) * 4);
#pragma unroll
        for (int ss = 0; ss < 4; ++ss) {
            unsigned vo = I.vrow[rr];
            if (ss == 0) vo = I.c0ok ? vo : LEAN_OOB;
            if (ss == 3) vo = I.c3ok ? vo : LEAN_OOB;
            const unsigned soff = __builtin_amdgcn_readfirstlane(cb + ss * pixb);
            d[rr * 4 + ss] = __builtin_bit_cast(f32x2v, __builtin_amdgcn_raw_buffer_load_b64(r, vo, soff, 0));
        }
    };
    // U pieces of sub-stage (chunk kc, row i) of item I into U slot base (zeros past its chunks)
    auto load_u = [&](const Item& I, int kc, int i, unsigned char* base) {
        if (PU_WF_ABL == 5) return;
        const unsigned bytes = I.live && kc < I.kc1 ? w.u_bytes : 0u;
        const unsigned sb = (unsigned)((kc * 16 + 4 * i) * 3) * u_row + (unsigned)(I.n_blk * 32);
#pragma unroll
        for (int e = 0; e < 3; ++e) lean_load(w.U, bytes, base + (wave * 3 + e) * 1024, u_lane, sb + poff[e]);
    };
    // V = row i of B^T d B for this thread's 2 channels -> hi/mid/lo planes in V slot sb
    auto make_v = [&](auto i_c, unsigned char* sb) {
        constexpr int i = decltype(i_c)::value;
        if (PU_WF_ABL == 2) return;
        f32x2v t[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            if constexpr (i == 0) t[s2] = d[s2] - d[8 + s2];
            else if constexpr (i == 1) t[s2] = d[4 + s2] + d[8 + s2];
            else if constexpr (i == 2) t[s2] = d[8 + s2] - d[4 + s2];
            else t[s2] = d[4 + s2] - d[12 + s2];
        }
        const f32x2v v0 = t[0] - t[2], v1 = t[1] + t[2], v2 = t[2] - t[1], v3 = t[1] - t[3];
        bf16x8_t h, m, l;
        split3_pairs(f32x4{v0[0], v0[1], v1[0], v1[1]}, f32x4{v2[0], v2[1], v3[0], v3[1]}, h, m, l);
        const u32x4 pv[3] = {__builtin_bit_cast(u32x4, h), __builtin_bit_cast(u32x4, m), __builtin_bit_cast(u32x4, l)};
        unsigned char* base = sb + v_st;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int j = 0; j < 4; ++j) *reinterpret_cast<unsigned*>(base + (j * 3 + pl) * 2048) = pv[pl][j];
    };
    // the 6 MFMAs of position (i, 2wx + jj) from V slot sv / U slot su
    auto mma = [&](auto x_c, const unsigned char* sv, const unsigned char* su, int jj) {
        constexpr int x = decltype(x_c)::value;
        const unsigned char* ub = su + u_rd + jj * 3 * 2048;
        const unsigned char* vb = sv + v_rd + jj * 3 * 2048;
        bf16x8_t fu[3], fv[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
            fu[pl] = *reinterpret_cast<const bf16x8_t*>(ub + pl * 2048);
            fv[pl] = *reinterpret_cast<const bf16x8_t*>(vb + pl * 2048);
        }
        if (PU_WF_ABL == 1) {
            acc[x][0] += __builtin_bit_cast(float, __builtin_shufflevector(fu[0], fu[1], 0, 1)) +
                         __builtin_bit_cast(float, __builtin_shufflevector(fu[2], fv[0], 0, 1)) +
                         __builtin_bit_cast(float, __builtin_shufflevector(fv[1], fv[2], 0, 1));
            return;
        }
        f32x16 c = acc[x];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[1], fv[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[2], fv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[0], fv[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[1], fv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[0], fv[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[0], fv[0], c, 0, 0, 0);
        acc[x] = c;
    };
    using I0 = std::integral_constant<int, 0>;
    auto uslot = [&](int k) -> unsigned char* { return k == 0 ? ldu0 : k == 1 ? ldu1 : k == 2 ? ldu2 : ldu3; };

    // sub-stage (kc, i) of the current item; T / tkc = the stream's next chunk (this item's kc+1,
    // or the next item's first chunk).  Issues U(s+3) into slot (i+3) & 3 (the slot sub-stage
    // s-1 read) and the window rows of the next chunk that chunk kc no longer reads (row 0 in
    // i = 0, row 2 in i = 1, rows 1 and 3 in i = 2).
    auto sub = [&](int kc, const Item& T, int tkc, auto i_c) {
        constexpr int i = decltype(i_c)::value;
        unsigned char* cv = (i & 1) ? ldv1 : ldv0;
        unsigned char* nv = (i & 1) ? ldv0 : ldv1;
        unsigned char* cu = uslot(i);
        unsigned char* fu = uslot((i + 3) & 3);
        if constexpr (i == 0) asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)" ::: "memory");
        else if constexpr (i == 1) asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)" ::: "memory");
        else if constexpr (i == 2) asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(22) lgkmcnt(0)" ::: "memory");
        WPP_STAMP(wave, nst);
        if (PU_WF_ABL != 4) __builtin_amdgcn_s_barrier();
        WPP_STAMP(wave, nst);
        asm volatile("" ::: "memory");
        if constexpr (i == 0) load_u(cur, kc, 3, fu);
        else load_u(T, tkc, i - 1, fu);
        asm volatile("" ::: "memory");                  // the wait counts assume U is issued first
        if constexpr (i == 0) load_row(T, tkc, 0);
        mma(std::integral_constant<int, 2 * i>{}, cv, cu, 0);
        if constexpr (i < 3) make_v(std::integral_constant<int, i + 1>{}, nv);
        else make_v(I0{}, nv);
        if constexpr (i == 1) load_row(T, tkc, 2);
        if constexpr (i == 2) {
            load_row(T, tkc, 1);
            load_row(T, tkc, 3);
        }
        mma(std::integral_constant<int, 2 * i + 1>{}, cv, cu, 1);
#if !PU_NO_ILV && PU_WF_ABL == 0
        // Interleave the 12 MFMAs with the V formation (~55 VALU, 12 plane stores): left to
        // itself the scheduler bunches 6 MFMAs before and 6 after it, and the two waves of a SIMD,
        // in the same phase between barriers, leave the matrix pipe idle during the VALU
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);        // position 2i operands
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            if (q == 2) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);   // position 2i + 1 operands
        }
#endif
    };

    // stream prologue: the first item's whole first window, U of sub-stages 0..2, V of 0
    load_row(cur, cur.kc0, 0);
    load_row(cur, cur.kc0, 1);
    load_row(cur, cur.kc0, 2);
    load_row(cur, cur.kc0, 3);
    load_u(cur, cur.kc0, 0, ldu0);
    load_u(cur, cur.kc0, 1, ldu1);
    load_u(cur, cur.kc0, 2, ldu2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    make_v(I0{}, ldv0);

    // output-transform exchange through V slot 1 (free at an item boundary: the last sub-stage
    // read it, the next item's first V is in slot 0), 4 registers per round:
    // [wm][wn][wx][2][4][64] floats = 16 KB
    float* xs = reinterpret_cast<float*>(ldv1) + ((wm * 2 + wn) * 2 + wx) * 512;
    const float* xr = reinterpret_cast<const float*>(ldv1) + ((wm * 2 + wn) * 2 + (1 - wx)) * 512;

    while (true) {
#pragma unroll
        for (int x = 0; x < 8; ++x)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;
        for (int kc = cur.kc0; kc < cur.kc1; ++kc) {
            const bool last = kc + 1 >= cur.kc1;
            const Item& T = last ? nxt : cur;
            const int tkc = last ? nxt.kc0 : kc + 1;
            sub(kc, T, tkc, std::integral_constant<int, 0>{});
            sub(kc, T, tkc, std::integral_constant<int, 1>{});
            sub(kc, T, tkc, std::integral_constant<int, 2>{});
            sub(kc, T, tkc, std::integral_constant<int, 3>{});
        }
        // every wave is past the last sub-stage's reads of V slot 1 and its V stores are done
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        WPP_STAMP(wave, nst);
        __builtin_amdgcn_s_barrier();
        WPP_STAMP(wave, nst);
        asm volatile("" ::: "memory");

        // ---- output transform Y = A^T M A.  Wave wx holds positions j = 2wx, 2wx+1 of every
        // row i for its (32 tiles x 32 channels); per element s_py[j] = sum_i A^T[py][i] M[i][j].
        // Wave wx finishes output row py = wx of the tile: Y[py][0] = (s[0] + s[1]) + s[2],
        // Y[py][1] = s[1] - (s[2] + s[3]); the partner wave (same wm, wn) supplies the other half.
        float y0v[16], y1v[16];
#pragma unroll
        for (int rd = 0; rd < 4; ++rd) {
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const int r = rd * 4 + r4;
                float sp[2][2];                          // [py][jj]
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    sp[0][jj] = acc[0 * 2 + jj][r] + acc[1 * 2 + jj][r] + acc[2 * 2 + jj][r];
                    sp[1][jj] = acc[1 * 2 + jj][r] - acc[2 * 2 + jj][r] - acc[3 * 2 + jj][r];
                }
                if (wx == 0) {   // j = 0, 1: keeps row 0 as (s0 + s1, s1), sends row 1 likewise
                    y0v[r] = sp[0][0] + sp[0][1];
                    y1v[r] = sp[0][1];
                    xs[r4 * 64 + lane] = sp[1][0] + sp[1][1];
                    xs[(4 + r4) * 64 + lane] = sp[1][1];
                } else {         // j = 2, 3: keeps row 1 as (s2, s2 + s3), sends row 0 likewise
                    y0v[r] = sp[1][0];
                    y1v[r] = sp[1][0] + sp[1][1];
                    xs[r4 * 64 + lane] = sp[0][0];
                    xs[(4 + r4) * 64 + lane] = sp[0][0] + sp[0][1];
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            WPP_STAMP(wave, nst);
            __builtin_amdgcn_s_barrier();
            WPP_STAMP(wave, nst);
            asm volatile("" ::: "memory");
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const int r = rd * 4 + r4;
                const float o0 = xr[r4 * 64 + lane], o1 = xr[(4 + r4) * 64 + lane];
                if (wx == 0) {
                    y0v[r] = y0v[r] + o0;
                    y1v[r] = y1v[r] - o1;
                } else {
                    y0v[r] = o0 + y0v[r];
                    y1v[r] = o1 - y1v[r];
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            WPP_STAMP(wave, nst);
            __builtin_amdgcn_s_barrier();
            WPP_STAMP(wave, nst);
            asm volatile("" ::: "memory");
        }
        const int e_m = cur.m_blk + 32 * wm + (lane & 31), e_n = cur.n_blk + 32 * wn + 4 * (lane >> 5);
        const bool e_ok = e_m < w.tiles;
        const int em = e_ok ? e_m : 0;
        const int t2 = fdiv(em, w.dTw);
        const int tx = em - t2 * (p.Wo >> 1);
        const int b = fdiv(t2, w.dTh);
        const int ty = t2 - b * (p.Ho >> 1);
        const long long pix0 = ((long long)b * p.Ho + 2 * ty + wx) * p.Wo + 2 * tx;
        if (p.ksplit == 1) {
            // igemm's float4 epilogue (bias, residual, ReLU, mask, channel scale, accumulate) for
            // the lane's two pixels.  Every operand load is issued, unconditionally and back to
            // back, before the first store: gfx9's vmcnt counts stores too, so a load issued after
            // a store (and waited for) waits out that store's round trip - with the loads inside
            // the per-flag branches each of the 8 stores was followed by a vmcnt(0).  Absent
            // operands read through an empty buffer range (no memory traffic); lanes past the
            // last tile load and store out of range.  A 64-channel item lies in one destination
            // (wino_ok: n0 % 64 == 0), so the destination is item-uniform.
            const bool first = cur.n_blk < p.n0;
            const int ld = first ? p.n0 : p.N - p.n0;
            float* dst = first ? p.dst0 : p.dst1;
            const float* msk = first ? p.mask0 : p.mask1;
            const bool relu = p.flags & PU_EPI_RELU, accum = p.flags & PU_EPI_ACCUM;
            constexpr unsigned FULL = 0x7fffffffu;
            const __amdgpu_buffer_rsrc_t r_dst = uniform_rsrc(dst, FULL);
            const __amdgpu_buffer_rsrc_t r_acc = uniform_rsrc(dst, accum ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_res = uniform_rsrc(p.resid, p.resid ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_msk = uniform_rsrc(msk, msk ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_bias = uniform_rsrc(p.bias, p.bias && PU_WF_ABL != 7 ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_cs = uniform_rsrc(p.cscale, p.cscale ? FULL : 0u);
            const unsigned o_px = e_ok ? (unsigned)(pix0 * ld + e_n - (first ? 0 : p.n0)) * 4u : LEAN_OOB;
            const unsigned o_row = (unsigned)ld * 4u;
            const unsigned o_cs = (unsigned)(b * p.cs_ld + e_n) * 4u;
            f32x4 bv[4], sv[4], rv[4][2], mv[4][2], av[4][2];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bv[g] = epi_ld4(r_bias, (unsigned)(e_n + 8 * g) * 4u);
                sv[g] = epi_ld4(r_cs, o_cs + 32u * g);
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    const unsigned off = o_px + o * o_row + 32u * g;
                    rv[g][o] = epi_ld4(r_res, off);
                    mv[g][o] = epi_ld4(r_msk, off);
                    av[g][o] = epi_ld4(r_acc, off);
                }
            }
            // pin every load here, ahead of the stores (the flag branches below would otherwise
            // take them in, each load then waited for behind the stores before it)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                asm volatile("" :: "v"(bv[g]), "v"(sv[g]));
#pragma unroll
                for (int o = 0; o < 2; ++o) asm volatile("" :: "v"(rv[g][o]), "v"(mv[g][o]), "v"(av[g][o]));
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 y[2] = {{y0v[4 * g], y0v[4 * g + 1], y0v[4 * g + 2], y0v[4 * g + 3]},
                                    {y1v[4 * g], y1v[4 * g + 1], y1v[4 * g + 2], y1v[4 * g + 3]}};
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    f32x4 v = y[o];
                    if (p.bias) v += bv[g];
                    if (p.resid) v += rv[g][o];
                    if (relu) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                    }
                    if (msk) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) if (!(mv[g][o][e] > 0.f)) v[e] = 0.f;
                    }
                    if (p.cscale) v *= sv[g];
                    if (accum) v += av[g][o];
                    const unsigned off = o_px + o * o_row + 32u * g;
                    if (PU_WF_ABL == 6) {      // no output stores (timing only): keep v alive
                        if (v[0] == 1.2345e-30f) epi_st4(r_dst, off, v);
                    } else {
                        epi_st4(r_dst, off, v);
                    }
                }
            }
        } else if (e_ok) {
            float* part = p.part + (long long)cur.kz * p.M * p.N + pix0 * p.N + e_n;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                *reinterpret_cast<f32x4*>(part + 8 * g) = f32x4{y0v[4 * g], y0v[4 * g + 1], y0v[4 * g + 2], y0v[4 * g + 3]};
                *reinterpret_cast<f32x4*>(part + p.N + 8 * g) = f32x4{y1v[4 * g], y1v[4 * g + 1], y1v[4 * g + 2], y1v[4 * g + 3]};
            }
        }
        if (!nxt.live) break;
        it += step;
        cur = nxt;
        decode(it + step, nxt);
    }
    // the stream's trailing (empty-range) LDS-DMA lands before the block's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------ one wave per SIMD: wino4_x6_kernel
// The same F(2x2,3x3) items (64 tiles x 64 output channels x a K range), products, U / V planes
// and output-transform expression tree as wino_x6_kernel - bit-identical results - re-tiled for
// one wave per SIMD: 4 waves, wave j owns position column j of every row i for the WHOLE 64 x 64
// item (2 x 2 MFMA blocks per position: 4 rows x 4 blocks = 256 accumulators, AGPRs), one item
// per block.
// Why: wino_x6_kernel's 8 waves each run a 32 x 32 block per position, so every MFMA needs its
// own U and V fragment (1 KB of LDS reads per MFMA; 96 KB per sub-stage on top of the 48 KB of U
// DMA and V stores), and after each sub-stage barrier both waves of a SIMD first wait for their
// LDS fragment reads.  Here a U fragment feeds 2 MFMAs and a V fragment 2 (24 KB of V reads per
// sub-stage), U goes straight from L2 into registers one sub-stage ahead (no LDS-DMA), and the
// sub-stages are software-pipelined so the matrix pipe does not wait for LDS after a barrier:
//   * V is formed TWO sub-stages ahead into a 3-slot ring (3 x 24 KB): during sub-stage s the
//     producer role (thread = tile tt, channel quad qq; its 4x4 window of 4 channels in 16 x f32x4)
//     forms V(s+2), and every wave pre-reads its 6 fragments of V(s+1) - complete at barrier(s) -
//     so the MFMAs of s+1 start right after barrier(s+1);
//   * window rows of a chunk are reloaded as soon as the formation no longer reads them (row 2 of
//     the next chunk in i = 0, rows 1 and 3 in i = 1, row 0 of the chunk after next in i = 2);
//   * item end: s_py[j] = sum_i A^T[py][i] M[i][j] is lane-local; wave b then owns block b
//     = (channel half b >> 1, tile half b & 1) and receives the other three columns' sums
//     through the (then idle) V ring (3 rounds), forms Y = (s0 + s1) + s2, s1 - (s2 + s3) for
//     both output rows and runs the batched float4 epilogue.
#ifndef PU_W4_ABL
#define PU_W4_ABL 0     // ablations (timing only, wrong results): 1 no MFMAs, 2 no V formation,
                        // 4 no window loads, 5 no U loads, 6 no sub-stage barrier, 7 no V plane stores
#endif
#ifndef PU_W4_VA
#define PU_W4_VA 2      // V formed PU_W4_VA sub-stages ahead into a (PU_W4_VA + 1)-slot ring (2 or 3)
#endif
#ifndef PU_W4_ITEM_STAMP
#define PU_W4_ITEM_STAMP 0  // diagnostic build: per-block s_memtime at entry / prologue / loop end / exchange / exit
#endif
#if PU_W4_ITEM_STAMP
constexpr int PU_W4_NBLK = 4096;
__device__ unsigned long long pu_w4_item_buf[PU_W4_NBLK * 8];
// lane 0 of wave 0, blocks < PU_W4_NBLK: stamp k (vector stores; timing only, tools/w4_items.py)
__device__ __forceinline__ void w4_item_stamp(int k, unsigned long long v) {
    if (threadIdx.x == 0 && blockIdx.x < PU_W4_NBLK) pu_w4_item_buf[blockIdx.x * 8 + k] = v;
}
#define W4S(k) w4_item_stamp(k, __builtin_amdgcn_s_memtime())
#else
#define W4S(k) ((void)0)
#endif
constexpr int W4_VH = 4 * 3 * 64 * 32;         // 24 KB: V of one sub-stage (4 xi x 3 planes x 64 tiles x 16)
constexpr int W4_XF = 4 * 2 * 16 * 64;         // floats in one exchange round (32 KB, inside the V ring)
#ifndef PU_W4_XCH1
#define PU_W4_XCH1 1    // 1: the output exchange in one round (96 KB: every wave's 3 outbound blocks at
                        // once, 16-byte LDS accesses, one barrier); 0: 3 rounds through the V ring
#endif
constexpr int W4_X1 = 4 * 3 * 32 * 64;         // floats of the one-round exchange (4 waves x 3 blocks)

template <bool FULL, int NCB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void wino4_x6_kernel(const WinoParams w) {
#pragma clang fp contract(off)
    const IgemmParams& p = w.p;
    // item shape: NCB 32-channel blocks x NTB 32-tile blocks (2 x 2: 64 x 64, or 4 x 1: 128
    // channels x 32 tiles - half the V formation and window loads per MFMA, twice the U)
    constexpr int NTB = 4 / NCB, BM = 32 * NTB, BN = 32 * NCB;
    constexpr int TPT = 256 / BM, CPT = 16 / TPT;       // producer threads per tile, channels per thread
    constexpr int PS = BM * 32;                          // bytes per (position, plane) block of a V slot
    constexpr int VS = 12 * PS;                          // one V slot
    typedef float wv_t __attribute__((ext_vector_type(CPT)));
    // U fragments UA sub-stages ahead in a USL-slot register ring (2 ahead for 64-channel items;
    // the 128-channel items' 12 fragments per sub-stage only fit one ahead)
    constexpr int UA = NCB == 2 ? 2 : 1, USL = 2 * UA;
    constexpr int VA = PU_W4_VA, NVS = VA + 1;
    static_assert(VA == 2 || VA == 3, "V lead");
    // one-round exchange except in the wide items' general epilogue (its operands leave no room)
    constexpr bool XCH1 = PU_W4_XCH1 && !(FULL && NCB == 4);
    constexpr int LDV = XCH1 && W4_X1 * 4 > NVS * W4_VH ? W4_X1 * 4 : NVS * W4_VH;
    __shared__ __attribute__((aligned(16))) unsigned char ldv[LDV];
    float* const xch = reinterpret_cast<float*>(ldv);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wj = __builtin_amdgcn_readfirstlane(tid >> 6);   // position column j of this wave
    W4S(0);
#if PU_W4_ITEM_STAMP
    w4_item_stamp(6, (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)));    // HW_ID
    w4_item_stamp(7, (unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)));   // XCC_ID
#endif

    // ---- the item (one per block, XCD-aware order)
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    const int per_split = w.gm * p.gn;
    const int kz = item / per_split;
    const int rest = item - kz * per_split;
    const int nbk = rest / w.gm;
    const int m_blk = (rest - nbk * w.gm) * BM;
    const int n_blk = nbk * BN;
    const int kc0 = kz * w.kc_per;
    const int kc1 = min(p.C / 16, kc0 + w.kc_per);

    // ---- producer role: tile tt of the item, channels CPT qq .. CPT qq + CPT-1 of each 16-channel chunk
    const int tt = tid / TPT, qq = tid % TPT;
    const int cs = p.c0;
    const int shift = p.Wi + 1;
    const unsigned pixb = (unsigned)cs * 4u;
    const float* a0 = p.src0 - (long long)shift * cs;
    const float* a1 = (p.c1 ? p.src1 : p.src0) - (long long)shift * cs;
    const int v_st = tt * 32 + ((((CPT * qq * 2) >> 4) ^ ((tt >> 3) & 1)) * 16) + ((CPT * qq * 2) & 15);
    unsigned vrow[4];
    bool c0ok, c3ok;
    {
        const int m = m_blk + tt;
        int ty = 0, tx = 0, b = 0;
        const bool mv = m < w.tiles;
        if (mv) {
            const int t2 = fdiv(m, w.dTw);
            tx = m - t2 * (p.Wo >> 1);
            b = fdiv(t2, w.dTh);
            ty = t2 - b * (p.Ho >> 1);
        }
        const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
        const unsigned base = (unsigned)(((b * p.Hi + y0) * p.Wi + x0 + shift) * cs * 4 + qq * CPT * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            vrow[r] = mv && (unsigned)(y0 + r) < (unsigned)p.Hi ? base + (unsigned)(r * p.Wi * cs * 4) : LEAN_OOB;
        c0ok = x0 >= 0;
        c3ok = x0 + 3 < p.Wi;
    }

    // ---- MFMA role: V rows 32 tb + (lane & 31) of position j, swizzled half (as wino_x6_kernel)
    const int rd_sw = (((lane >> 5) ^ ((lane >> 3) & 1)) * 16);
    const int v_rd = (lane & 31) * 32 + rd_sw + wj * 3 * PS;
    // U fragment (n = 32 cb + (lane & 31), k half lane >> 5) of (chunk, xi, plane): 1 KB per wave
    const unsigned u_row = (unsigned)p.N * 32u;
    const unsigned u_lane = (unsigned)(lane & 31) * 32u + (unsigned)(lane >> 5) * 16u;

    wv_t d[16];                  // window [row][col] of CPT channels
    f32x16 acc[4][NCB][NTB];     // [i][cb][tb]
    bf16x8_t fu[USL][NCB][3];    // U fragments [slot][cb][plane], UA sub-stages ahead
    bf16x8_t fv[2][NTB][3];      // V fragments [slot][tb][plane], one sub-stage ahead

    auto load_row = [&](int kc, int rr) {
        if (PU_W4_ABL == 4) {
#pragma unroll
            for (int ss = 0; ss < 4; ++ss) d[rr * 4 + ss] = wv_t(1.f + rr + 0.5f * ss + 0.25f * kc);
            return;
        }
        const int c = kc * 16;
        const bool second = c >= p.c0;
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(second ? a1 : a0, kc < kc1 ? w.a_bytes : 0u);
        const unsigned cb = (unsigned)((second ? c - p.c0 : c) * 4);
#pragma unroll
        for (int ss = 0; ss < 4; ++ss) {
            unsigned vo = vrow[rr];
            if (ss == 0) vo = c0ok ? vo : LEAN_OOB;
            if (ss == 3) vo = c3ok ? vo : LEAN_OOB;
            const unsigned soff = __builtin_amdgcn_readfirstlane(cb + ss * pixb);
            if constexpr (CPT == 4)
                d[rr * 4 + ss] = __builtin_bit_cast(wv_t, __builtin_amdgcn_raw_buffer_load_b128(r, vo, soff, 0));
            else
                d[rr * 4 + ss] = __builtin_bit_cast(wv_t, __builtin_amdgcn_raw_buffer_load_b64(r, vo, soff, 0));
        }
    };
    // U fragments of position (i, wj) of chunk kc into register slot sl (zeros past the item's chunks)
    auto load_u = [&](int kc, int i, auto sl_c) {
        constexpr int sl = decltype(sl_c)::value;
        if (PU_W4_ABL == 5) {
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) fu[sl][cb][pl] = __builtin_bit_cast(bf16x8_t, u32x4{(unsigned)kc, (unsigned)i, 0u, 1u});
            return;
        }
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(w.U, kc < kc1 ? w.u_bytes : 0u);
        const unsigned sb = (unsigned)((kc * 16 + 4 * i + wj) * 3) * u_row + (unsigned)(n_blk * 32);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                fu[sl][cb][pl] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                    r, u_lane + (unsigned)cb * 1024u, __builtin_amdgcn_readfirstlane(sb + pl * u_row), 0));
    };
    // this wave's V fragments (position wj, 2 tile halves x 3 planes) of the V slot at byte offset so
    auto read_v = [&](unsigned so, auto sl_c) {
        constexpr int sl = decltype(sl_c)::value;
        const unsigned char* vb = ldv + so + v_rd;
#pragma unroll
        for (int tb = 0; tb < NTB; ++tb)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                fv[sl][tb][pl] = *reinterpret_cast<const bf16x8_t*>(vb + tb * 1024 + pl * PS);
    };
    // V of row f (4 positions) for this thread's tile and 4 channels -> hi / mid / lo planes
    auto make_v = [&](auto f_c, unsigned so) {
        constexpr int f = decltype(f_c)::value;
        if (PU_W4_ABL == 2) return;
        wv_t t[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            if constexpr (f == 0) t[s2] = d[s2] - d[8 + s2];
            else if constexpr (f == 1) t[s2] = d[4 + s2] + d[8 + s2];
            else if constexpr (f == 2) t[s2] = d[8 + s2] - d[4 + s2];
            else t[s2] = d[4 + s2] - d[12 + s2];
        }
        const wv_t v[4] = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
        unsigned char* base = ldv + so + v_st;
        if constexpr (CPT == 4) {
#pragma unroll
            for (int jp = 0; jp < 2; ++jp) {
                bf16x8_t h, m, l;
                split3_pairs(v[2 * jp], v[2 * jp + 1], h, m, l);
                const u32x4 pv[3] = {__builtin_bit_cast(u32x4, h), __builtin_bit_cast(u32x4, m), __builtin_bit_cast(u32x4, l)};
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    if (PU_W4_ABL == 7) {      // formation without its plane stores (timing only)
                        asm volatile("" :: "v"(pv[pl]));
                        continue;
                    }
                    *reinterpret_cast<u32x2*>(base + ((2 * jp) * 3 + pl) * PS) = u32x2{pv[pl][0], pv[pl][1]};
                    *reinterpret_cast<u32x2*>(base + ((2 * jp + 1) * 3 + pl) * PS) = u32x2{pv[pl][2], pv[pl][3]};
                }
            }
        } else {
            bf16x8_t h, m, l;
            split3_pairs(f32x4{v[0][0], v[0][1], v[1][0], v[1][1]}, f32x4{v[2][0], v[2][1], v[3][0], v[3][1]}, h, m, l);
            const u32x4 pv[3] = {__builtin_bit_cast(u32x4, h), __builtin_bit_cast(u32x4, m), __builtin_bit_cast(u32x4, l)};
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int j = 0; j < 4; ++j) *reinterpret_cast<unsigned*>(base + (j * 3 + pl) * PS) = pv[pl][j];
        }
    };
    // the 24 MFMAs of position (i, wj): U slot su x V slot sv, the 6 products of each of the
    // 4 blocks in wino_x6_kernel's order; the item's first chunk starts from C = 0
    auto mma = [&](auto i_c, auto su_c, auto sl_c, auto first_c) {
        constexpr int i = decltype(i_c)::value;
        constexpr int su = decltype(su_c)::value;     // U slot
        constexpr int sl = decltype(sl_c)::value;     // V fragment slot
        constexpr bool FIRST = decltype(first_c)::value;
        if (PU_W4_ABL == 1) {
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                for (int tb = 0; tb < NTB; ++tb)
                    acc[i][cb][tb][0] += __builtin_bit_cast(float, __builtin_shufflevector(fu[su][cb][0], fv[sl][tb][1], 0, 9));
            return;
        }
        constexpr int PU[6] = {1, 2, 0, 1, 0, 0}, PV[6] = {1, 0, 2, 0, 1, 0};
#pragma unroll
        for (int e = 0; e < 6; ++e)
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                for (int tb = 0; tb < NTB; ++tb)
                    acc[i][cb][tb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        fu[su][cb][PU[e]], fv[sl][tb][PV[e]], (FIRST && e == 0) ? f32x16{} : acc[i][cb][tb], 0, 0, 0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;

    // V ring: V(s) in slot s % NVS (byte offset sv), V(s+1) .. V(s+VA) in the next VA
    unsigned sv = 0;
    auto slot_after = [](unsigned so, int k) -> unsigned {
        unsigned r = so + (unsigned)k * VS;
        return r >= (unsigned)(NVS * VS) ? r - (unsigned)(NVS * VS) : r;
    };

    // sub-stage (kc, i) = s.  At barrier(s) every wave has finished s-1, so V(s+1) (formed during
    // s-1) is complete and V(s-1)'s slot - its fragments were pre-read during s-2 - is free for
    // V(s+2).  The MFMAs use the V fragments read during s-1 and the U fragments issued during s-1.
    auto sub = [&](int kc, auto i_c, auto first_c) {
        constexpr int i = decltype(i_c)::value;
        constexpr int F = (i + VA) & 3;                // the row formed now (chunk kc, or kc+1 for i >= 4 - VA)
        if (PU_W4_ABL != 6) {
            // VA = 3: V(s+1) was stored during s-2, older than every LDS op of s-1 (3 NTB
            // fragment reads, then >= 3 NTB plane stores); LDS ops complete in order, so <= 3 NTB
            // outstanding means only s-1's youngest stores are in flight across the barrier
            if constexpr (VA == 3) asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(3 * NTB) : "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        // pin this sub-stage's fragments (U issued and V read during s-1) here: the MFMAs would
        // otherwise be hoisted across barrier(s) into sub-stage s-1
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
            for (int k = 0; k < NCB; ++k) asm volatile("" : "+v"(fu[i & (USL - 1)][k][pl]));
#pragma unroll
            for (int k = 0; k < NTB; ++k) asm volatile("" : "+v"(fv[i & 1][k][pl]));
        }
        // pin the window rows this formation reads (F = 2: rows 1, 2; 3: 1, 3; 0: 0, 2; 1: 1, 2):
        // the formation is pure VALU and would otherwise be hoisted across the barriers
        constexpr int RA = F == 0 ? 0 : 1, RB = F == 3 ? 3 : 2;
#pragma unroll
        for (int ss = 0; ss < 4; ++ss) asm volatile("" : "+v"(d[RA * 4 + ss]), "+v"(d[RB * 4 + ss]));
        read_v(slot_after(sv, 1), std::integral_constant<int, (i + 1) & 1>{});
        if constexpr (i + UA < 4) load_u(kc, i + UA, std::integral_constant<int, (i + UA) & (USL - 1)>{});
        else load_u(kc + 1, i + UA - 4, std::integral_constant<int, (i + UA) & (USL - 1)>{});
        mma(i_c, std::integral_constant<int, i & (USL - 1)>{}, std::integral_constant<int, i & 1>{}, first_c);
        // pin this sub-stage's MFMAs here: they are pure, and the selection DAG of the unrolled
        // chunk would otherwise float them past the following barriers
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int tb = 0; tb < NTB; ++tb) asm volatile("" : "+a"(acc[i][cb][tb]));
        make_v(std::integral_constant<int, F>{}, slot_after(sv, VA));
        if constexpr (VA == 2) {
            if constexpr (i == 0) load_row(kc + 1, 2);
            if constexpr (i == 1) {
                load_row(kc + 1, 1);
                load_row(kc + 1, 3);
            }
            if constexpr (i == 2) load_row(kc + 2, 0);
        } else {
            // rows 1 / 3 of chunk kc are dead after row 3's formation (i = 0), row 0 of kc+1
            // after its row 0 (i = 1), row 2 of kc+1 after its row 2 (i = 3)
            if constexpr (i == 0) {
                load_row(kc + 1, 1);
                load_row(kc + 1, 3);
            }
            if constexpr (i == 1) load_row(kc + 2, 0);
            if constexpr (i == 3) load_row(kc + 2, 2);
        }
        sv = slot_after(sv, 1);
#if PU_W4_ABL == 0 && !PU_NO_ILV
        // issue order: V(s+1) fragment reads, U(s+1), then the 24 MFMAs with the formation of
        // V(s+2) in their shadow (~4 VALU per MFMA, a plane store every other one)
        // (the 12 plane stores are merged into 6 ds_write2st64 before scheduling)
        __builtin_amdgcn_sched_group_barrier(0x100, 3 * NTB, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 3 * NCB, 0);     // U(s+UA)
#pragma unroll
        for (int q = 0; q < 24; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, CPT == 4 ? 5 : 3, 0);
            if ((q & 3) == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);
#endif
    };

    // prologue: the first chunk's window, U of sub-stage 0, V(0) and V(1) into slots 0 / 1, the
    // next chunk's row 0 (row 0 of the first chunk is dead after V(0)), V(0)'s fragments
    load_row(kc0, 0);
    load_row(kc0, 1);
    load_row(kc0, 2);
    load_row(kc0, 3);
    load_u(kc0, 0, I0{});
    if constexpr (UA == 2) load_u(kc0, 1, I1{});
    make_v(I0{}, 0u);
    make_v(I1{}, (unsigned)VS);
    if constexpr (VA == 3) make_v(std::integral_constant<int, 2>{}, (unsigned)(2 * VS));
    load_row(kc0 + 1, 0);
    if constexpr (VA == 3) load_row(kc0 + 1, 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read_v(0u, I0{});
    W4S(1);

    using BT = std::true_type;
    using BF = std::false_type;
    // the item's first chunk starts every accumulator from C = 0 (no zeroing pass); every item
    // has >= 2 chunks (wino_ok: C % 32 == 0, even chunks per K split)
    sub(kc0, std::integral_constant<int, 0>{}, BT{});
    sub(kc0, std::integral_constant<int, 1>{}, BT{});
    sub(kc0, std::integral_constant<int, 2>{}, BT{});
    sub(kc0, std::integral_constant<int, 3>{}, BT{});
    for (int kc = kc0 + 1; kc < kc1; ++kc) {
        sub(kc, std::integral_constant<int, 0>{}, BF{});
        sub(kc, std::integral_constant<int, 1>{}, BF{});
        sub(kc, std::integral_constant<int, 2>{}, BF{});
        sub(kc, std::integral_constant<int, 3>{}, BF{});
    }
    // every wave is done reading the V ring (the exchange reuses it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    W4S(2);

    // ---- output transform.  Column sums s_py[j] (lane-local, wino_x6_kernel's order):
    // s_0 = (M0 + M1) + M2, s_1 = (M1 - M2) - M3.  Wave b owns block b = (cb, tb) = (b >> 1,
    // b & 1); in round r wave j sends block (j + r) & 3 and receives block b from wave (b - r) & 3.
    // Specialised per wave (a uniform switch) so every register index is static; the column sums
    // live in accumulator registers whose products are consumed (the own column in acc[0 / 1][J],
    // the column received in round r in acc[0 / 1][block sent in round r]); Y in acc[3][py][px].
    auto xform = [&](auto j_c) {
        constexpr int J = decltype(j_c)::value;
#define W4A(i, b) acc[i][(b) / NTB][(b) % NTB]
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const float s0 = W4A(0, J)[e] + W4A(1, J)[e] + W4A(2, J)[e];
            const float s1 = W4A(1, J)[e] - W4A(2, J)[e] - W4A(3, J)[e];
            W4A(0, J)[e] = s0;
            W4A(1, J)[e] = s1;
        }
        if constexpr (XCH1) {
        // region (source wave w, round r) = 8 float4 chunks x 64 lanes: the 32 column sums of the
        // block wave w sends in round r (s_0[16], s_1[16]); chunk c holds values 4c .. 4c+3
        auto region = [&](int wsrc, int r) { return reinterpret_cast<f32x4*>(xch) + (wsrc * 3 + r - 1) * 8 * 64; };
        auto send = [&](auto r_c) {
            constexpr int R = decltype(r_c)::value;
            constexpr int SB = (J + R) & 3;
            f32x4* dst = region(J, R);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                f32x4 v;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int e = (4 * c + q) & 15;
                    v[q] = c < 4 ? W4A(0, SB)[e] + W4A(1, SB)[e] + W4A(2, SB)[e]
                                 : W4A(1, SB)[e] - W4A(2, SB)[e] - W4A(3, SB)[e];
                }
                dst[c * 64 + lane] = v;
                if (c == 3) asm volatile("" ::: "memory");
            }
        };
        auto recv = [&](auto r_c) {
            constexpr int R = decltype(r_c)::value;
            constexpr int SB = (J + R) & 3, FROM = (J - R) & 3;
            const f32x4* src = region(FROM, R);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const f32x4 v = src[c * 64 + lane];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int e = (4 * c + q) & 15;
                    if (c < 4) W4A(0, SB)[e] = v[q];
                    else W4A(1, SB)[e] = v[q];
                }
                if (c == 3) asm volatile("" ::: "memory");
            }
        };
        // (compiler fences between the blocks: one block's 32 values in registers at a time)
        send(std::integral_constant<int, 1>{});
        asm volatile("" ::: "memory");
        send(std::integral_constant<int, 2>{});
        asm volatile("" ::: "memory");
        send(std::integral_constant<int, 3>{});
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        recv(std::integral_constant<int, 1>{});
        asm volatile("" ::: "memory");
        recv(std::integral_constant<int, 2>{});
        asm volatile("" ::: "memory");
        recv(std::integral_constant<int, 3>{});
        } else {
        float* xs = xch + J * (2 * 16 * 64);
        auto round = [&](auto r_c) {
            constexpr int R = decltype(r_c)::value;
            constexpr int SB = (J + R) & 3, FROM = (J - R) & 3;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                xs[e * 64 + lane] = W4A(0, SB)[e] + W4A(1, SB)[e] + W4A(2, SB)[e];
                xs[(16 + e) * 64 + lane] = W4A(1, SB)[e] - W4A(2, SB)[e] - W4A(3, SB)[e];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const float* xr = xch + FROM * (2 * 16 * 64);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                W4A(0, SB)[e] = xr[e * 64 + lane];
                W4A(1, SB)[e] = xr[(16 + e) * 64 + lane];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        round(std::integral_constant<int, 1>{});
        round(std::integral_constant<int, 2>{});
        round(std::integral_constant<int, 3>{});
        }
        // column j was received in round r = (J - j) & 3 and sits in block (J + r) & 3 (r = 0: own)
        constexpr int B0 = (J + ((J - 0) & 3)) & 3, B1 = (J + ((J - 1) & 3)) & 3;
        constexpr int B2 = (J + ((J - 2) & 3)) & 3, B3 = (J + ((J - 3) & 3)) & 3;
#pragma unroll
        for (int py = 0; py < 2; ++py)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const float c0 = W4A(py, B0)[e], c1 = W4A(py, B1)[e], c2 = W4A(py, B2)[e], c3 = W4A(py, B3)[e];
                W4A(3, 2 * py)[e] = (c0 + c1) + c2;      // Y[py][0] = (s0 + s1) + s2
                W4A(3, 2 * py + 1)[e] = c1 - (c2 + c3);  // Y[py][1] = s1 - (s2 + s3)
            }
#undef W4A
    };
    switch (wj) {
        case 0: xform(std::integral_constant<int, 0>{}); break;
        case 1: xform(std::integral_constant<int, 1>{}); break;
        case 2: xform(std::integral_constant<int, 2>{}); break;
        default: xform(std::integral_constant<int, 3>{}); break;
    }

    W4S(3);
    const int cbo = wj / NTB, tbo = wj % NTB;
    const int e_m = m_blk + 32 * tbo + (lane & 31), e_n = n_blk + 32 * cbo + 4 * (lane >> 5);
    const bool e_ok = e_m < w.tiles;
    const int em = e_ok ? e_m : 0;
    const int t2 = fdiv(em, w.dTw);
    const int tx = em - t2 * (p.Wo >> 1);
    const int b = fdiv(t2, w.dTh);
    const int ty = t2 - b * (p.Ho >> 1);
    const long long pix00 = ((long long)b * p.Ho + 2 * ty) * p.Wo + 2 * tx;
    auto yv = [&](int py, int o, int g) {
        const int b2 = 2 * py + o;
        const f32x16& a3 = acc[3][b2 / NTB][b2 % NTB];
        return f32x4{a3[4 * g], a3[4 * g + 1], a3[4 * g + 2], a3[4 * g + 3]};
    };
    if (p.ksplit == 1) {
        // wino_x6_kernel's batched float4 epilogue for both output rows: operand loads first,
        // then the stores
        const bool first = n_blk + 32 * cbo < p.n0;     // a 32-channel block lies in one destination
        const int ld = first ? p.n0 : p.N - p.n0;
        float* dst = first ? p.dst0 : p.dst1;
        const float* msk = first ? p.mask0 : p.mask1;
        const bool relu = p.flags & PU_EPI_RELU, accum = p.flags & PU_EPI_ACCUM;
        constexpr unsigned RANGE = 0x7fffffffu;
        const __amdgpu_buffer_rsrc_t r_dst = uniform_rsrc(dst, RANGE);
        const __amdgpu_buffer_rsrc_t r_msk = uniform_rsrc(msk, msk ? RANGE : 0u);
        const __amdgpu_buffer_rsrc_t r_bias = uniform_rsrc(p.bias, p.bias ? RANGE : 0u);
        const unsigned o_px = e_ok ? (unsigned)(pix00 * ld + e_n - (first ? 0 : p.n0)) * 4u : LEAN_OOB;
        const unsigned o_col = (unsigned)ld * 4u;                  // next pixel in x
        const unsigned o_row = (unsigned)p.Wo * (unsigned)ld * 4u;  // next pixel row
        if constexpr (!FULL) {
            // bias (+ ReLU) and / or a ReLU mask (the UNetp layers): the bias and the first output
            // row's masks, that row's stores, then the second row
            f32x4 bv[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) bv[g] = epi_ld4(r_bias, (unsigned)(e_n + 8 * g) * 4u);
#pragma unroll
            for (int py = 0; py < 2; ++py) {
                f32x4 mv[4][2];
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int o = 0; o < 2; ++o) mv[g][o] = epi_ld4(r_msk, o_px + py * o_row + o * o_col + 32u * g);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    asm volatile("" :: "v"(bv[g]));
#pragma unroll
                    for (int o = 0; o < 2; ++o) asm volatile("" :: "v"(mv[g][o]));
                }
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int o = 0; o < 2; ++o) {
                        f32x4 v = yv(py, o, g);
                        if (p.bias) v += bv[g];
                        if (relu) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                        }
                        if (msk) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) if (!(mv[g][o][e] > 0.f)) v[e] = 0.f;
                        }
                        epi_st4(r_dst, o_px + py * o_row + o * o_col + 32u * g, v);
                    }
            }
        } else {
            // every epilogue operand (residual, channel scale, accumulate), one output row at a time
            const __amdgpu_buffer_rsrc_t r_acc = uniform_rsrc(dst, accum ? RANGE : 0u);
            const __amdgpu_buffer_rsrc_t r_res = uniform_rsrc(p.resid, p.resid ? RANGE : 0u);
            const __amdgpu_buffer_rsrc_t r_cs = uniform_rsrc(p.cscale, p.cscale ? RANGE : 0u);
            const unsigned o_cs = (unsigned)(b * p.cs_ld + e_n) * 4u;
#pragma unroll
            for (int py = 0; py < 2; ++py) {
                f32x4 bv[4], sv4[4], rv[4][2], mv[4][2], av[4][2];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    bv[g] = epi_ld4(r_bias, (unsigned)(e_n + 8 * g) * 4u);
                    sv4[g] = epi_ld4(r_cs, o_cs + 32u * g);
#pragma unroll
                    for (int o = 0; o < 2; ++o) {
                        const unsigned off = o_px + py * o_row + o * o_col + 32u * g;
                        rv[g][o] = epi_ld4(r_res, off);
                        mv[g][o] = epi_ld4(r_msk, off);
                        av[g][o] = epi_ld4(r_acc, off);
                    }
                }
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    asm volatile("" :: "v"(bv[g]), "v"(sv4[g]));
#pragma unroll
                    for (int o = 0; o < 2; ++o) asm volatile("" :: "v"(rv[g][o]), "v"(mv[g][o]), "v"(av[g][o]));
                }
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int o = 0; o < 2; ++o) {
                        f32x4 v = yv(py, o, g);
                        if (p.bias) v += bv[g];
                        if (p.resid) v += rv[g][o];
                        if (relu) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                        }
                        if (msk) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) if (!(mv[g][o][e] > 0.f)) v[e] = 0.f;
                        }
                        if (p.cscale) v *= sv4[g];
                        if (accum) v += av[g][o];
                        epi_st4(r_dst, o_px + py * o_row + o * o_col + 32u * g, v);
                    }
            }
        }
    } else if (e_ok) {
        float* part = p.part + (long long)kz * p.M * p.N + pix00 * p.N + e_n;
#pragma unroll
        for (int py = 0; py < 2; ++py)
#pragma unroll
            for (int o = 0; o < 2; ++o)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *reinterpret_cast<f32x4*>(part + ((long long)py * p.Wo + o) * p.N + 8 * g) = yv(py, o, g);
    }
    W4S(4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W4S(5);
}

// ------------------------------------------------------------------ 128-channel Winograd items
// wino128_x6_kernel: the same F(2x2,3x3) arithmetic, products and output transform as
// wino_x6_kernel, with items of 32 tiles x 128 output channels instead of 64 x 64, so each V
// element formed feeds 128 outputs instead of 64 (half the formation work per MFMA; a layer's V is
// formed once per 128 channels) at the price of twice the U bytes per MFMA (a 48 KB U slice per
// sub-stage).  8 waves (wn, wx): 32 tiles x 32 channels (32 wn ..) x the 8 positions of j = 2wx,
// 2wx+1 - 128 accumulators, as in wino_x6_kernel.  Thread (tile tt, channel q) holds the 4x4
// window of one channel and forms its V row per sub-stage (4 values, exact 3-term split, 12
// 2-byte plane stores).  LDS: V 2 x 12 KB, U 2 x 48 KB (U issued one sub-stage ahead; the slice is
// L2-resident - every item of an XCD shares it, channel block slowest), 120 KB.
#ifndef PU_W2_ABL
#define PU_W2_ABL 0     // wino128_x6_kernel ablations (timing only, wrong results): 1 no U DMA, 2 no V formation
#endif
constexpr int W2_BM = 32;
constexpr int W2_BN = 128;
constexpr int W2_VH = 4 * 3 * W2_BM * 32;      // 12 KB
constexpr int W2_UH = 4 * 3 * W2_BN * 32;      // 48 KB

__device__ __forceinline__ void split3_quad(const f32x4 x, bf16x4_t& h, bf16x4_t& m, bf16x4_t& l) {
#pragma clang fp contract(off)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const __bf16 a = (__bf16)x[e];
        const float r = x[e] - (float)a;
        const __bf16 b = (__bf16)r;
        h[e] = a;
        m[e] = b;
        l[e] = (__bf16)(r - (float)b);
    }
}

template <bool PERSIST>
__global__ __launch_bounds__(512) void wino128_x6_kernel(const WinoParams w) {
#pragma clang fp contract(off)
    const IgemmParams& p = w.p;
    __shared__ __attribute__((aligned(16))) unsigned char ldv0[W2_VH];
    __shared__ __attribute__((aligned(16))) unsigned char ldv1[W2_VH];
    __shared__ __attribute__((aligned(16))) unsigned char ldu0[W2_UH];
    __shared__ __attribute__((aligned(16))) unsigned char ldu1[W2_UH];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave & 3, wx = wave >> 2;
    const int per_split = w.gm * p.gn;
    const int total = per_split * p.ksplit;

    int it, end, step;
    if (PERSIST) {
        const int xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
        const int q8 = total >> 3, r8 = total & 7;
        const int start = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
        end = start + q8 + (xcd < r8 ? 1 : 0);
        it = start + local;
        step = (int)(gridDim.x >> 3);
    } else {
        it = xcd_remap(blockIdx.x, gridDim.x);
        end = it + 1;
        step = 1;
    }
    if (it >= end) return;

    // ---- producer role: tile tt of the item, channel q of each 16-channel chunk
    const int tt = tid >> 4, q = tid & 15;
    const int cs = p.c0;
    const int shift = p.Wi + 1;
    const unsigned pixb = (unsigned)cs * 4u;
    const float* a0 = p.src0 - (long long)shift * cs;
    const float* a1 = (p.c1 ? p.src1 : p.src0) - (long long)shift * cs;
    const int v_st = tt * 32 + (((q >> 3) ^ ((tt >> 3) & 1)) * 16) + (q & 7) * 2;

    // ---- U loader: wave w fills pieces 6w .. 6w+5 (piece P = (j*3 + plane)*4 + row quarter)
    const unsigned u_lane = (unsigned)((lane >> 1) * 32 + (((lane & 1) ^ ((lane >> 4) & 1)) * 16));
    const unsigned u_row = (unsigned)p.N * 32u;
    unsigned poff[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
        const int P = wave * 6 + e;
        poff[e] = (unsigned)(P >> 2) * u_row + (unsigned)((P & 3) * 1024);
    }

    // ---- MFMA role: positions j = 2wx, 2wx+1; U rows 32*wn + (lane&31), V rows lane&31
    const int rd_sw = (((lane >> 5) ^ ((lane >> 3) & 1)) * 16);
    const int u_rd = (32 * wn + (lane & 31)) * 32 + rd_sw + 2 * wx * 3 * 4096;
    const int v_rd = (lane & 31) * 32 + rd_sw + 2 * wx * 3 * 1024;

    struct Item {
        int kz, m_blk, n_blk, kc0, kc1;
        unsigned vrow[4];
        bool c0ok, c3ok, live;
    };
    auto decode = [&](int item, Item& I) {
        I.live = item < end;
        I.kz = item / per_split;
        const int rest = item - I.kz * per_split;
        const int nb = rest / w.gm;
        I.m_blk = (rest - nb * w.gm) * W2_BM;
        I.n_blk = nb * W2_BN;
        I.kc0 = I.kz * w.kc_per;
        I.kc1 = min(p.C / 16, I.kc0 + w.kc_per);
        const int m = I.m_blk + tt;
        int ty = 0, tx = 0, b = 0;
        const bool mv = I.live && m < w.tiles;
        if (mv) {
            const int t2 = fdiv(m, w.dTw);
            tx = m - t2 * (p.Wo >> 1);
            b = fdiv(t2, w.dTh);
            ty = t2 - b * (p.Ho >> 1);
        }
        const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
        const unsigned base = (unsigned)(((b * p.Hi + y0) * p.Wi + x0 + shift) * cs * 4 + q * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            I.vrow[r] = mv && (unsigned)(y0 + r) < (unsigned)p.Hi ? base + (unsigned)(r * p.Wi * cs * 4) : LEAN_OOB;
        I.c0ok = x0 >= 0;
        I.c3ok = x0 + 3 < p.Wi;
    };
    Item cur, nxt;
    decode(it, cur);
    decode(it + step, nxt);

    float d[16];
    f32x16 acc[8];

    auto load_row = [&](const Item& I, int kc, int rr) {
        const int c = kc * 16;
        const bool second = c >= p.c0;
        const bool ok = I.live && kc < I.kc1;
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(second ? a1 : a0, ok ? w.a_bytes : 0u);
        const unsigned cb = (unsigned)((second ? c - p.c0 : c) * 4);
#pragma unroll
        for (int ss = 0; ss < 4; ++ss) {
            unsigned vo = I.vrow[rr];
            if (ss == 0) vo = I.c0ok ? vo : LEAN_OOB;
            if (ss == 3) vo = I.c3ok ? vo : LEAN_OOB;
            const unsigned soff = __builtin_amdgcn_readfirstlane(cb + ss * pixb);
            d[rr * 4 + ss] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, soff, 0));
        }
    };
    auto load_u = [&](const Item& I, int kc, int i, unsigned char* base) {
        if (PU_W2_ABL == 1) return;
        const unsigned bytes = I.live && kc < I.kc1 ? w.u_bytes : 0u;
        const unsigned sb = (unsigned)((kc * 16 + 4 * i) * 3) * u_row + (unsigned)(I.n_blk * 32);
#pragma unroll
        for (int e = 0; e < 6; ++e) lean_load(w.U, bytes, base + (wave * 6 + e) * 1024, u_lane, sb + poff[e]);
    };
    // V = row i of B^T d B for this thread's channel -> hi/mid/lo planes in V slot sb
    auto make_v = [&](auto i_c, unsigned char* sb) {
        constexpr int i = decltype(i_c)::value;
        if (PU_W2_ABL == 2) return;
        float t[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            if constexpr (i == 0) t[s2] = d[s2] - d[8 + s2];
            else if constexpr (i == 1) t[s2] = d[4 + s2] + d[8 + s2];
            else if constexpr (i == 2) t[s2] = d[8 + s2] - d[4 + s2];
            else t[s2] = d[4 + s2] - d[12 + s2];
        }
        const f32x4 v = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
        bf16x4_t h, m, l;
        split3_quad(v, h, m, l);
        unsigned char* base = sb + v_st;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            *reinterpret_cast<__bf16*>(base + (j * 3 + 0) * 1024) = h[j];
            *reinterpret_cast<__bf16*>(base + (j * 3 + 1) * 1024) = m[j];
            *reinterpret_cast<__bf16*>(base + (j * 3 + 2) * 1024) = l[j];
        }
    };
    auto mma = [&](auto x_c, const unsigned char* sv, const unsigned char* su, int jj) {
        constexpr int x = decltype(x_c)::value;
        const unsigned char* ub = su + u_rd + jj * 3 * 4096;
        const unsigned char* vb = sv + v_rd + jj * 3 * 1024;
        bf16x8_t fu[3], fv[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
            fu[pl] = *reinterpret_cast<const bf16x8_t*>(ub + pl * 4096);
            fv[pl] = *reinterpret_cast<const bf16x8_t*>(vb + pl * 1024);
        }
        f32x16 c = acc[x];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[1], fv[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[2], fv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[0], fv[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[1], fv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[0], fv[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fu[0], fv[0], c, 0, 0, 0);
        acc[x] = c;
    };
    using I0 = std::integral_constant<int, 0>;

    // sub-stage (kc, i): V slot i & 1 (formed during the previous sub-stage), U slot i & 1 (issued
    // during the previous sub-stage).  Issues U of the stream's next sub-stage into the other slot
    // (read by the previous sub-stage, which every wave has left at the barrier) and the window
    // rows of the next chunk that this chunk no longer reads (row 0 in i = 0, row 2 in i = 1, rows
    // 1 and 3 in i = 2).  Wait counts: the rows issued after U in the previous sub-stage.
    auto sub = [&](int kc, const Item& T, int tkc, auto i_c) {
        constexpr int i = decltype(i_c)::value;
        unsigned char* cv = (i & 1) ? ldv1 : ldv0;
        unsigned char* nv = (i & 1) ? ldv0 : ldv1;
        unsigned char* cu = (i & 1) ? ldu1 : ldu0;
        unsigned char* fu = (i & 1) ? ldu0 : ldu1;
        if constexpr (i == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else if constexpr (i == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
        else if constexpr (i == 2) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if constexpr (i < 3) load_u(cur, kc, i + 1, fu);
        else load_u(T, tkc, 0, fu);
        asm volatile("" ::: "memory");                  // the wait counts assume U is issued first
        if constexpr (i == 0) load_row(T, tkc, 0);
        mma(std::integral_constant<int, 2 * i>{}, cv, cu, 0);
        if constexpr (i < 3) make_v(std::integral_constant<int, i + 1>{}, nv);
        else make_v(I0{}, nv);
        if constexpr (i == 1) load_row(T, tkc, 2);
        if constexpr (i == 2) {
            load_row(T, tkc, 1);
            load_row(T, tkc, 3);
        }
        mma(std::integral_constant<int, 2 * i + 1>{}, cv, cu, 1);
    };

    // stream prologue: the first item's whole first window and U of its sub-stage 0, V of 0
    load_row(cur, cur.kc0, 0);
    load_row(cur, cur.kc0, 1);
    load_row(cur, cur.kc0, 2);
    load_row(cur, cur.kc0, 3);
    load_u(cur, cur.kc0, 0, ldu0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    make_v(I0{}, ldv0);

    // output-transform exchange through U slot 1 (free at an item boundary: the last sub-stage
    // read it; the next item's U(0) is in slot 0): [wn][wx][2][4][64] floats = 16 KB per round
    float* xs = reinterpret_cast<float*>(ldu1) + (wn * 2 + wx) * 512;
    const float* xr = reinterpret_cast<const float*>(ldu1) + (wn * 2 + (1 - wx)) * 512;

    while (true) {
#pragma unroll
        for (int x = 0; x < 8; ++x)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;
        for (int kc = cur.kc0; kc < cur.kc1; ++kc) {
            const bool last = kc + 1 >= cur.kc1;
            const Item& T = last ? nxt : cur;
            const int tkc = last ? nxt.kc0 : kc + 1;
            sub(kc, T, tkc, std::integral_constant<int, 0>{});
            sub(kc, T, tkc, std::integral_constant<int, 1>{});
            sub(kc, T, tkc, std::integral_constant<int, 2>{});
            sub(kc, T, tkc, std::integral_constant<int, 3>{});
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");

        // output transform, as wino_x6_kernel (wave wx finishes output row py = wx of the tile)
        float y0v[16], y1v[16];
#pragma unroll
        for (int rd = 0; rd < 4; ++rd) {
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const int r = rd * 4 + r4;
                float sp[2][2];
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    sp[0][jj] = acc[0 * 2 + jj][r] + acc[1 * 2 + jj][r] + acc[2 * 2 + jj][r];
                    sp[1][jj] = acc[1 * 2 + jj][r] - acc[2 * 2 + jj][r] - acc[3 * 2 + jj][r];
                }
                if (wx == 0) {
                    y0v[r] = sp[0][0] + sp[0][1];
                    y1v[r] = sp[0][1];
                    xs[r4 * 64 + lane] = sp[1][0] + sp[1][1];
                    xs[(4 + r4) * 64 + lane] = sp[1][1];
                } else {
                    y0v[r] = sp[1][0];
                    y1v[r] = sp[1][0] + sp[1][1];
                    xs[r4 * 64 + lane] = sp[0][0];
                    xs[(4 + r4) * 64 + lane] = sp[0][0] + sp[0][1];
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const int r = rd * 4 + r4;
                const float o0 = xr[r4 * 64 + lane], o1 = xr[(4 + r4) * 64 + lane];
                if (wx == 0) {
                    y0v[r] = y0v[r] + o0;
                    y1v[r] = y1v[r] - o1;
                } else {
                    y0v[r] = o0 + y0v[r];
                    y1v[r] = o1 - y1v[r];
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        const int e_m = cur.m_blk + (lane & 31), e_n = cur.n_blk + 32 * wn + 4 * (lane >> 5);
        const bool e_ok = e_m < w.tiles;
        const int em = e_ok ? e_m : 0;
        const int t2 = fdiv(em, w.dTw);
        const int tx = em - t2 * (p.Wo >> 1);
        const int b = fdiv(t2, w.dTh);
        const int ty = t2 - b * (p.Ho >> 1);
        const long long pix0 = ((long long)b * p.Ho + 2 * ty + wx) * p.Wo + 2 * tx;
        if (p.ksplit == 1) {
            // the batched float4 epilogue of wino_x6_kernel; a wave's 32 channels lie in one
            // destination (n0 % 32 == 0, host)
            const bool first = cur.n_blk + 32 * wn < p.n0;
            const int ld = first ? p.n0 : p.N - p.n0;
            float* dst = first ? p.dst0 : p.dst1;
            const float* msk = first ? p.mask0 : p.mask1;
            const bool relu = p.flags & PU_EPI_RELU, accum = p.flags & PU_EPI_ACCUM;
            constexpr unsigned FULL = 0x7fffffffu;
            const __amdgpu_buffer_rsrc_t r_dst = uniform_rsrc(dst, FULL);
            const __amdgpu_buffer_rsrc_t r_acc = uniform_rsrc(dst, accum ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_res = uniform_rsrc(p.resid, p.resid ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_msk = uniform_rsrc(msk, msk ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_bias = uniform_rsrc(p.bias, p.bias ? FULL : 0u);
            const __amdgpu_buffer_rsrc_t r_cs = uniform_rsrc(p.cscale, p.cscale ? FULL : 0u);
            const unsigned o_px = e_ok ? (unsigned)(pix0 * ld + e_n - (first ? 0 : p.n0)) * 4u : LEAN_OOB;
            const unsigned o_row = (unsigned)ld * 4u;
            const unsigned o_cs = (unsigned)(b * p.cs_ld + e_n) * 4u;
            f32x4 bv[4], sv[4], rv[4][2], mv[4][2], av[4][2];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bv[g] = epi_ld4(r_bias, (unsigned)(e_n + 8 * g) * 4u);
                sv[g] = epi_ld4(r_cs, o_cs + 32u * g);
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    const unsigned off = o_px + o * o_row + 32u * g;
                    rv[g][o] = epi_ld4(r_res, off);
                    mv[g][o] = epi_ld4(r_msk, off);
                    av[g][o] = epi_ld4(r_acc, off);
                }
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                asm volatile("" :: "v"(bv[g]), "v"(sv[g]));
#pragma unroll
                for (int o = 0; o < 2; ++o) asm volatile("" :: "v"(rv[g][o]), "v"(mv[g][o]), "v"(av[g][o]));
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 y[2] = {{y0v[4 * g], y0v[4 * g + 1], y0v[4 * g + 2], y0v[4 * g + 3]},
                                    {y1v[4 * g], y1v[4 * g + 1], y1v[4 * g + 2], y1v[4 * g + 3]}};
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    f32x4 v = y[o];
                    if (p.bias) v += bv[g];
                    if (p.resid) v += rv[g][o];
                    if (relu) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                    }
                    if (msk) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) if (!(mv[g][o][e] > 0.f)) v[e] = 0.f;
                    }
                    if (p.cscale) v *= sv[g];
                    if (accum) v += av[g][o];
                    epi_st4(r_dst, o_px + o * o_row + 32u * g, v);
                }
            }
        } else if (e_ok) {
            float* part = p.part + (long long)cur.kz * p.M * p.N + pix0 * p.N + e_n;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                *reinterpret_cast<f32x4*>(part + 8 * g) = f32x4{y0v[4 * g], y0v[4 * g + 1], y0v[4 * g + 2], y0v[4 * g + 3]};
                *reinterpret_cast<f32x4*>(part + p.N + 8 * g) = f32x4{y1v[4 * g], y1v[4 * g + 1], y1v[4 * g + 2], y1v[4 * g + 3]};
            }
        }
        if (!nxt.live) break;
        it += step;
        cur = nxt;
        decode(it + step, nxt);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// U = G g G^T per (n, 8 consecutive c), fp64 then rounded to fp32 and split into hi/mid/lo bf16:
// out[((c/16*16 + xi)*3 + plane)*N + n][c % 16].  Forward: g = w[n][c]; dgrad (the transposed,
// flipped kernel of the data gradient): output channel n = input channel of w, c = its output
// channel, g[r][s] = w[c][n][2-r][2-s].
struct WinoPackJob {
    const float* w;
    __bf16* out;
    int n, c, dgrad, blocks;
};
constexpr int WINO_MAX_JOBS = 64;
struct WinoPackBatch {
    WinoPackJob job[WINO_MAX_JOBS];
    int count;
};

// Block = 32 output rows n x 64 reduced channels c (4 chunks) of one job.  The weights of the tile
// are staged through LDS with coalesced reads (fwd: 32 rows of 64 x 9 contiguous floats; dgrad:
// 64 rows of 32 x 9), so the thread that forms (n, 8 channels) reads its 72 values from LDS rather
// than 288 scattered bytes of global memory; thread = (chunk, n, half): a wave's 16-byte stores of
// one (chunk, position, plane) cover 32 n x 32 B = 1 KB contiguous.
constexpr int WP_N = 32, WP_C = 64;
constexpr int WP_LD = WP_C * 9 + 1;     // LDS floats per n row (+1: rows on distinct banks)
__global__ __launch_bounds__(256) void wino_pack_kernel(const WinoPackBatch bt) {
#pragma clang fp contract(off)
    __shared__ float gw[WP_N * WP_LD];
    int j = 0, b0 = 0;
    while (j + 1 < bt.count && (int)blockIdx.x >= b0 + bt.job[j].blocks) b0 += bt.job[j++].blocks;
    const WinoPackJob J = bt.job[j];
    const int blk = (int)blockIdx.x - b0;
    const int nblks = (J.n + WP_N - 1) / WP_N;
    const int n0 = (blk % nblks) * WP_N, c0 = (blk / nblks) * WP_C;
    const int nn = min(WP_N, J.n - n0), cc = min(WP_C, J.c - c0);
    const int tid = threadIdx.x;
    // stage g[n][c][3][3] (dgrad: g[r][s] = w[c][n][2-r][2-s], flipped when read below).  A thread
    // stages 72 floats in 3 groups of 24 loads issued back to back (out-of-tile lanes load element 0
    // and drop it), so the tile costs 3 memory round trips rather than one per element.
    constexpr int PER = WP_N * WP_C * 9 / 256, GRP = 24;
    static_assert(PER % GRP == 0, "staging groups");
#pragma unroll
    for (int g0 = 0; g0 < PER; g0 += GRP) {
        float v[GRP];
        int dst[GRP];
#pragma unroll
        for (int u = 0; u < GRP; ++u) {
            const int e = tid + (g0 + u) * 256;
            long long src;
            bool ok;
            if (!J.dgrad) {
                const int nl = e / (WP_C * 9), rest = e - nl * WP_C * 9;
                ok = nl < nn && rest < cc * 9;
                src = ((long long)(n0 + nl) * J.c + c0) * 9 + rest;
                dst[u] = ok ? nl * WP_LD + rest : -1;
            } else {
                const int cl = e / (WP_N * 9), rest = e - cl * WP_N * 9;
                const int nl = rest / 9, k = rest - nl * 9;
                ok = cl < cc && nl < nn;
                src = ((long long)(c0 + cl) * J.n + n0) * 9 + rest;
                dst[u] = ok ? nl * WP_LD + cl * 9 + k : -1;
            }
            v[u] = J.w[ok ? src : 0];
        }
#pragma unroll
        for (int u = 0; u < GRP; ++u)
            if (dst[u] >= 0) gw[dst[u]] = v[u];
    }
    __syncthreads();
    const int half = tid & 1, nl = (tid >> 1) & 31, ch = tid >> 6;
    const int c8 = (c0 >> 3) + ch * 2 + half;
    if (nl >= nn || ch * 16 + half * 8 >= cc) return;
    const int n = n0 + nl;
    const int chunk = c8 >> 1;
    typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
    const float* gr = gw + nl * WP_LD + (ch * 16 + half * 8) * 9;
    // one row a of G g G^T at a time (12 output vectors live)
#pragma unroll 1
    for (int a = 0; a < 4; ++a) {
        asm volatile("" ::: "memory");        // re-read g from LDS per row (no 72 hoisted doubles)
        bf16x8v o[4][3];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            double g[3][3];
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int s = 0; s < 3; ++s)
                    g[r][s] = J.dgrad ? (double)gr[e * 9 + (2 - r) * 3 + (2 - s)] : (double)gr[e * 9 + r * 3 + s];
            double t[3];   // row a of G g
#pragma unroll
            for (int s = 0; s < 3; ++s)
                t[s] = a == 0 ? g[0][s] : a == 1 ? 0.5 * (g[0][s] + g[1][s] + g[2][s])
                     : a == 2 ? 0.5 * (g[0][s] - g[1][s] + g[2][s]) : g[2][s];
            const double u[4] = {t[0], 0.5 * (t[0] + t[1] + t[2]), 0.5 * (t[0] - t[1] + t[2]), t[2]};
#pragma unroll
            for (int bc = 0; bc < 4; ++bc) {
                const float x = (float)u[bc];
                const __bf16 h = (__bf16)x;
                const float rr = x - (float)h;
                const __bf16 mm = (__bf16)rr;
                o[bc][0][e] = h;
                o[bc][1][e] = mm;
                o[bc][2][e] = (__bf16)(rr - (float)mm);
            }
        }
#pragma unroll
        for (int bc = 0; bc < 4; ++bc)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                *reinterpret_cast<bf16x8v*>(J.out + ((((long long)chunk * 16 + a * 4 + bc) * 3 + pl) * J.n + n) * 16 + half * 8) = o[bc][pl];
    }
}

// host side -------------------------------------------------------------------------------------

// the layers the Winograd kernel takes (the caller passed U): 3x3 / s1 / p1, same-size even grid,
// 16-channel chunks from one source each with one pixel stride (c1 == 0 or c1 == c0), an even
// number of chunks, 64-channel output blocks, the float4 epilogue, no ConvT shuffle, buffers
// addressable with 32-bit offsets
// 128-channel items (wino128_x6_kernel) for layers with n % 128 == 0: opt-in, PU_WINO128=1 - they
// measured slower than the 64 x 64 items on every C2 layer (profiles/r05_experiments/wino128_ab.txt)
static bool wino128_on() {
    static const bool on = [] {
        const char* e = getenv("PU_WINO128");
        return e && e[0] == '1';
    }();
    return on;
}

static bool wino4_on();
// 32-tile x 128-channel items: the 8-wave wino128_x6_kernel (PU_WINO128=1 with PU_WINO4=0), or the
// one-wave-per-SIMD kernel's wide items (PU_WINO4_WIDE=1)
static int wino4_wide_mode();
static bool wino128_use(const pu_conv_args* a) {
    const int C = a->c0 + a->c1;
    const int wm = wino4_wide_mode();
    const bool on = wino4_on() ? (wm == 1 || (wm == 2 && C < 128 && a->n > WG_BN)) : wino128_on();
    return on && a->n % W2_BN == 0 && (a->n0 == a->n || a->n0 % 32 == 0);
}

bool wino_ok(const pu_conv_args* a, bool vec_epi) {
    const int C = a->c0 + a->c1;
    if (!a->wino || !a->weight6) return false;
    if (a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1) return false;
    if (a->in_h != a->out_h || a->in_w != a->out_w || (a->out_h & 1) || (a->out_w & 1)) return false;
    if (a->c0 % 16 || (a->c1 != 0 && a->c1 != a->c0) || C % 32) return false;
    if (a->n % WG_BN || !vec_epi || (a->flags & PU_EPI_SHUFFLE2)) return false;
    // a short reduction (4 chunks) over several 64-channel output blocks re-forms the same V once
    // per block for little MFMA work: the concat layers' data gradients (64 -> 128 / 256) stay
    // on the direct kernel (measured: top_cat dgrad 0.43 vs 0.41 ms, l2_cat 0.21 vs 0.20)
    if (C < 128 && a->n > WG_BN && !wino128_use(a)) return false;
    const long long px = (long long)a->batch * a->in_h * a->in_w + a->in_w + 1;
    if (px * a->c0 * 4 >= (1LL << 31)) return false;
    if ((long long)C * a->n * 96 >= (1LL << 31)) return false;
    // the epilogue's 32-bit destination offsets and item-uniform destination (64-channel items
    // never straddle the split column n0)
    if ((long long)a->batch * a->out_h * a->out_w * a->n * 4 >= (1LL << 31) - 64) return false;
    if (a->n0 != a->n && a->n0 % (wino128_use(a) ? 32 : WG_BN)) return false;
    return ((uintptr_t)a->wino & 15) == 0;
}

// K split so that small tile grids (8x8 / 16x16 levels) still give ~1 block per CU: even chunk
// counts per split, >= 8 chunks (128 channels) each
void wino_plan(const pu_conv_args* a, int* ksplit, int* kc_per) {
    const int C = a->c0 + a->c1;
    const long long tiles = (long long)a->batch * (a->out_h / 2) * (a->out_w / 2);
    const bool w128 = wino128_use(a);
    const int blocks = ceil_div(tiles, w128 ? W2_BM : WG_BM) * (a->n / (w128 ? W2_BN : WG_BN));
    const int chunks = C / 16;
    *ksplit = 1;
    *kc_per = chunks;
    if (blocks >= 240) return;
    int ks = ceil_div(256, blocks);
    if (ks > chunks / 8) ks = chunks / 8;
    if (ks < 2) return;
    int per = ceil_div(chunks, ks);
    per += per & 1;
    *kc_per = per;
    *ksplit = ceil_div(chunks, per);
}

// persistent blocks (default) or one block per item: PU_WINO_PERSIST=0 (A/B runs)
static bool wino_persist() {
    static const bool on = [] {
        const char* e = getenv("PU_WINO_PERSIST");
        return !(e && e[0] == '0');
    }();
    return on;
}

// 64 x 64 items on one wave per SIMD (wino4_x6_kernel, bit-identical to wino_x6_kernel; default):
// PU_WINO4=0 keeps the 8-wave kernel (A/B runs, profiles/r06_experiments/wino4_ab.txt)
static bool wino4_on() {
    static const bool on = [] {
        const char* e = getenv("PU_WINO4");
        return !(e && e[0] == '0');
    }();
    return on;
}

// the one-wave-per-SIMD kernel's 32-tile x 128-channel items: PU_WINO4_WIDE=1 for every layer with
// n % 128 == 0 (bit-identical, measured no faster than the 64 x 64 items,
// profiles/r06_experiments/wino4_ab.txt); =2 (default) only for the short reductions (C < 128)
// into several 64-channel blocks, which the 64 x 64 items leave to the direct kernel (the concat
// data gradients: top 0.426 -> 0.409 ms, l2 0.200 -> 0.195); =0 none
static int wino4_wide_mode() {
    static const int m = [] {
        const char* e = getenv("PU_WINO4_WIDE");
        return !e ? 2 : e[0] == '1' ? 1 : e[0] == '2' ? 2 : 0;
    }();
    return m;
}

int wino_launch(const pu_conv_args* a, IgemmParams p, hipStream_t s) {
    WinoParams w;
    w.p = p;
    w.U = reinterpret_cast<const __bf16*>(a->wino);
    w.tiles = a->batch * (a->out_h / 2) * (a->out_w / 2);
    const bool w128 = wino128_use(a);
    w.gm = ceil_div(w.tiles, w128 ? W2_BM : WG_BM);
    w.p.gn = a->n / (w128 ? W2_BN : WG_BN);
    w.dTw = make_fastdiv(a->out_w / 2);
    w.dTh = make_fastdiv(a->out_h / 2);
    w.a_bytes = (unsigned)(((long long)a->batch * a->in_h * a->in_w + a->in_w + 1) * a->c0 * 4);
    w.u_bytes = (unsigned)((long long)(a->c0 + a->c1) * a->n * 96);
    int ks, per;
    wino_plan(a, &ks, &per);
    if (ks > 1 && (!a->workspace || a->ws_bytes < (size_t)ks * p.M * p.N * sizeof(float))) {
        ks = 1;
        per = (a->c0 + a->c1) / 16;
    }
    w.p.ksplit = ks;
    w.p.part = (float*)a->workspace;
    w.kc_per = per;
    const int items = w.gm * w.p.gn * ks;
    if (w128 && !wino4_on()) {
        if (wino_persist() && items > 256)
            hipLaunchKernelGGL(wino128_x6_kernel<true>, dim3(256), dim3(512), 0, s, w);
        else
            hipLaunchKernelGGL(wino128_x6_kernel<false>, dim3((unsigned)items), dim3(512), 0, s, w);
        return ks;
    }
    if (wino4_on()) {
        // one item per block (the pipelined kernel keeps the next chunks' rows in flight per item)
        const bool full = p.resid || p.cscale || (p.flags & PU_EPI_ACCUM);
        const dim3 g((unsigned)items);
        if (w128) {
            if (full) hipLaunchKernelGGL((wino4_x6_kernel<true, 4>), g, dim3(256), 0, s, w);
            else hipLaunchKernelGGL((wino4_x6_kernel<false, 4>), g, dim3(256), 0, s, w);
        } else {
            if (full) hipLaunchKernelGGL((wino4_x6_kernel<true, 2>), g, dim3(256), 0, s, w);
            else hipLaunchKernelGGL((wino4_x6_kernel<false, 2>), g, dim3(256), 0, s, w);
        }
        return ks;
    }
    if (wino_persist() && items > 256)
        hipLaunchKernelGGL(wino_x6_kernel<true>, dim3(256), dim3(512), 0, s, w);
    else
        hipLaunchKernelGGL(wino_x6_kernel<false>, dim3((unsigned)items), dim3(512), 0, s, w);
    return ks;
}

int wino_item_channels(const pu_conv_args* a) { return wino128_use(a) ? W2_BN : WG_BN; }

size_t wino_workspace_bytes(const pu_conv_args* a) {
    int ks, per;
    wino_plan(a, &ks, &per);
    return ks > 1 ? (size_t)ks * a->batch * a->out_h * a->out_w * a->n * sizeof(float) : 0;
}

}  // namespace pu

using namespace pu;

#if PU_WPP_STAMP
// diagnostic build only: copy block 0's barrier stamps ([8 waves][PU_WPP_NSTAMP] shader cycles)
extern "C" int pu_wpp_stamps(unsigned long long* dst, int n) {
    if (n > 8 * PU_WPP_NSTAMP) n = 8 * PU_WPP_NSTAMP;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(pu_wpp_stamp_buf), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? n : -1;
}
#endif

#if PU_W4_ITEM_STAMP
// diagnostic build only: per-block item stamps of the last wino4 launch ([block][8]: entry,
// prologue done, loop done, exchange done, stores issued, stores drained, HW_ID, XCC_ID)
extern "C" int pu_w4_item_stamps(unsigned long long* dst, int n) {
    if (n > 8 * PU_W4_NBLK) n = 8 * PU_W4_NBLK;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(pu_w4_item_buf), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? n : -1;
}
#endif

extern "C" size_t pu_wino_bytes(int n, int c) {
    return (n > 0 && c > 0 && c % 16 == 0) ? (size_t)n * c * 96 : 0;
}

extern "C" int pu_pack_wino(const pu_wino_job* jobs, int n_jobs, void* stream) {
    PU_REQUIRE(n_jobs >= 0 && (n_jobs == 0 || jobs), "pu_pack_wino: bad job list");
    for (int i0 = 0; i0 < n_jobs; i0 += WINO_MAX_JOBS) {
        WinoPackBatch b;
        b.count = 0;
        int total = 0;
        for (int i = i0; i < n_jobs && i < i0 + WINO_MAX_JOBS; ++i) {
            const pu_wino_job& J = jobs[i];
            PU_REQUIRE(J.w && J.out && J.cout > 0 && J.cin > 0, "pu_pack_wino: job %d incomplete", i);
            const int n = J.dgrad ? J.cin : J.cout, c = J.dgrad ? J.cout : J.cin;
            PU_REQUIRE(c % 16 == 0, "pu_pack_wino: job %d reduces over %d channels (need a multiple of 16)", i, c);
            PU_REQUIRE(((uintptr_t)J.out & 15) == 0, "pu_pack_wino: job %d output must be 16-byte aligned", i);
            WinoPackJob& o = b.job[b.count++];
            o.w = J.w;
            o.out = (__bf16*)J.out;
            o.n = n;
            o.c = c;
            o.dgrad = J.dgrad != 0;
            o.blocks = ceil_div(n, WP_N) * ceil_div(c, WP_C);   // 32 n x 64 c tiles
            total += o.blocks;
        }
        hipLaunchKernelGGL(wino_pack_kernel, dim3((unsigned)total), dim3(256), 0, as_stream(stream), b);
        const int st = check_launch("pu_pack_wino");
        if (st != PU_OK) return st;
    }
    return PU_OK;
}
