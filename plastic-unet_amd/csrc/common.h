// Shared helpers of libplastic_unet.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <type_traits>

#include "plastic_unet.h"

namespace pu {

// ------------------------------------------------------------------------------ error reporting
extern thread_local char g_last_error[512];

inline int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
    return code;
}

// PU_DEBUG builds (build_native.py --variant debug -> lib/libplastic_unet_debug.so) synchronise
// after every launch, so an asynchronous fault is reported by the entry point that caused it
// (the HIP_LAUNCH_BLOCKING / AMD_SERIALIZE_KERNEL discipline, per call instead of per process).
inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(PU_ERR_LAUNCH, "%s: %s", what, hipGetErrorString(e));
#ifdef PU_DEBUG
    e = hipDeviceSynchronize();
    if (e != hipSuccess) return fail(PU_ERR_LAUNCH, "%s (PU_DEBUG synchronous check): %s", what, hipGetErrorString(e));
#endif
    return PU_OK;
}

#define PU_REQUIRE(cond, ...)                                          \
    do {                                                               \
        if (!(cond)) return ::pu::fail(PU_ERR_INVALID, __VA_ARGS__);   \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ----------------------------------------------------------- integer division by a runtime divisor
// q = umulhi(x, mul) >> shift  for 0 <= x < 2^31, d >= 1 (Granlund-Montgomery round-up method)
struct FastDiv {
    uint32_t d, mul, shift;
};

inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    if (d == 1) {
        f.mul = 0;
        f.shift = 0;
        return f;
    }
    uint32_t l = 0;
    while ((1u << l) < d) ++l;
    // mul = ceil(2^(32+l) / d) - 2^32 ... use the simpler 64-bit form
    uint64_t m = ((uint64_t(1) << (32 + l)) + d - 1) / d;
    f.mul = uint32_t(m);  // m < 2^33; keep the low 32 bits, add x back (see div())
    f.shift = l;
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
    // q = (x + umulhi(x, mul_lo)) >> l  where mul = 2^32 + mul_lo ;  x < 2^31 so no overflow.
    // Branch-free: d == 1 has mul_lo = 0, l = 0 (keeps hot loops one basic block).
    uint32_t hi = __umulhi(x, f.mul);
    return (hi + x) >> f.shift;
}

inline int ceil_div(long long a, long long b) { return int((a + b - 1) / b); }

// 4-term dot product as an explicit fma chain (v0 w0 first): the 1x1 outconv's per-lane sum, shared
// by outconv_fwd_kernel and the fused head so both produce bit-identical logits
template <typename V>
__device__ __forceinline__ float dot4_fma(const V v, const V w) {
    return fmaf(v[3], w[3], fmaf(v[2], w[2], fmaf(v[1], w[1], v[0] * w[0])));
}

// XCD-aware block order: the dispatcher deals blocks round-robin over the 8 XCDs (block b runs on
// XCD b % 8).  Map hardware block b to a logical tile so that each XCD gets one CONTIGUOUS range
// of logical tiles (neighbouring tiles share input rows/halos -> reuse in that XCD's L2).
// Bijective for any total (the ragged variant of cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int xcd = b & 7, local = b >> 3;
    const int q = total >> 3, r = total & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}


// compile-time loop: f(integral_constant<int, I>) for I = 0 .. N-1 (unrolled; I usable as a constant)
template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, F, I + 1>(static_cast<F&&>(f));
    }
}
// lean implicit-GEMM loaders: an out-of-image tap gets this byte offset, outside every buffer
// descriptor's range, so the range check writes zeros into LDS (probed: tools/probes/oob_lds.hip)
constexpr unsigned LEAN_OOB = 0x80000000u;
typedef __attribute__((address_space(3))) void lds_void_t;

// buffer_load_dwordx4 ... lds of 16 B per lane through a descriptor built from wave-uniform
// inputs, made provably uniform (no waterfall loops around the loads); bytes == 0 drops every
// lane (zeros land in LDS).  Kept out of the kernel template so the host pass never sees the
// descriptor type.
__device__ __forceinline__ void lean_load(const void* base, unsigned bytes, void* lds_dst, unsigned voff, unsigned soff) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    void* ub = (void*)(((unsigned long long)hi << 32) | lo);
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(ub, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_dst, 16, voff, __builtin_amdgcn_readfirstlane(soff), 0, 0);
}

}  // namespace pu
