// Probe: cost of the Winograd item epilogue's store pattern (8 dwordx4 stores per lane, 8 waves,
// 64 KB per block per item, every CU storing at once) vs the same bytes with whole 128-B lines per
// 8 lanes and with 1 KB contiguous per instruction.  Each "item" = a fixed compute delay
// (s_sleep) + the stores; the next item's first wait is vmcnt(0) (the kernel's counted waits on
// loads issued after the stores behave the same: vmcnt retires in issue order).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int PAT>
__global__ __launch_bounds__(512) void probe(float* out, int items, int sleep_iters) {
    __shared__ float pad[24 * 1024];            // 96 KB: one block per CU, as the kernel
    if (sleep_iters < 0) pad[threadIdx.x] = 0.f;
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w & 1, wn = (w >> 1) & 1, wx = w >> 2;
    for (int it = 0; it < items; ++it) {
        for (int s = 0; s < sleep_iters; ++s) __builtin_amdgcn_s_sleep(127);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        float* base = out + ((long long)blockIdx.x * items + it) * 16384;
        const f32x4 v = {1.f + it, 2.f, 3.f, (float)l};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            long long off;
            if (PAT == 0) {          // wino_x6_kernel: lane = tile, 16 B of 4 channels, g = k>>1, o = k&1
                const int g = k >> 1, o = k & 1;
                const int x = 2 * (32 * wm + (l & 31)) + o, ch = 32 * wn + 4 * (l >> 5) + 8 * g;
                off = ((long long)(wx * 128 + x) * 64 + ch);
            } else if (PAT == 1) {   // 8 lanes = one pixel's 128 B (32 channels)
                const int x = 64 * wm + 8 * k + (l >> 3);
                off = ((long long)(wx * 128 + x) * 64 + 32 * wn) + (l & 7) * 4;
            } else {                 // 1 KB contiguous per instruction
                off = (long long)w * 2048 + k * 256 + l * 4;
            }
            if (PAT < 3) *reinterpret_cast<f32x4*>(base + off) = v;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
    const int blocks = 256, items = 8;
    float* d;
    hipMalloc(&d, (size_t)blocks * items * 65536);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int sl : {0, 2, 4}) {
        for (int pat = 0; pat < 4; ++pat) {
            float best = 1e9f;
            for (int rep = 0; rep < 7; ++rep) {
                hipEventRecord(e0);
                if (pat == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(512), 0, 0, d, items, sl);
                if (pat == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(512), 0, 0, d, items, sl);
                if (pat == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(512), 0, 0, d, items, sl);
                if (pat == 3) hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(512), 0, 0, d, items, sl);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep > 0 && ms < best) best = ms;
            }
            printf("sleep %d pattern %d: %.1f us (%.2f us per item, %.1f GB/s)\n", sl, pat, best * 1e3,
                   best * 1e3 / items, blocks * items * 65536.0 / (best * 1e-3) / 1e9);
        }
    }
    printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
