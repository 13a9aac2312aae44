// Bare bf16 MFMA loops on random operands held in registers: v_mfma_f32_32x32x16_bf16 vs
// v_mfma_f32_16x16x32_bf16 at the same FLOPs per wave (one accumulator set of 16 floats per lane
// = one 32x32 tile or four 16x16 tiles), 2 waves per SIMD.  Prints TFLOP/s and the kernel time.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/mfma_shape.cpp -o /tmp/mfma_shape && /tmp/mfma_shape
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k32(const bf16x8* in, float* out) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    bf16x8 a[3], b[3];
    for (int i = 0; i < 3; ++i) { a[i] = in[(t * 6 + i) & 65535]; b[i] = in[(t * 6 + 3 + i) & 65535]; }
    f32x16 c[4] = {};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[j % 3], b[(j + 1) % 3], c[j], 0, 0, 0);
            c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[(j + 1) % 3], b[j % 3], c[j], 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int j = 0; j < 4; ++j) for (int r = 0; r < 16; ++r) s += c[j][r];
    out[t] = s;
}

__global__ __launch_bounds__(256) void k16(const bf16x8* in, float* out) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    bf16x8 a[3], b[3];
    for (int i = 0; i < 3; ++i) { a[i] = in[(t * 6 + i) & 65535]; b[i] = in[(t * 6 + 3 + i) & 65535]; }
    f32x4 c[16] = {};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j % 3], b[(j + 1) % 3], c[j], 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int j = 0; j < 16; ++j) for (int r = 0; r < 4; ++r) s += c[j][r];
    out[t] = s;
}

int main() {
    const int n = 65536;
    bf16x8* h = (bf16x8*)malloc(n * sizeof(bf16x8));
    srand(1);
    for (int i = 0; i < n; ++i) for (int e = 0; e < 8; ++e) h[i][e] = (__bf16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
    bf16x8* d; float* o;
    hipMalloc(&d, n * sizeof(bf16x8));
    hipMemcpy(d, h, n * sizeof(bf16x8), hipMemcpyHostToDevice);
    const int blocks = 256 * 2;          // 2 blocks of 4 waves per CU = 2 waves per SIMD
    hipMalloc(&o, blocks * 256 * sizeof(float));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        for (int which = 0; which < 2; ++which) {
            for (int w = 0; w < 3; ++w) {
                if (which == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, d, o);
                else hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, d, o);
            }
            hipEventRecord(e0);
            const int R = 10;
            for (int r = 0; r < R; ++r) {
                if (which == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, d, o);
                else hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, d, o);
            }
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double flop = (double)R * blocks * 4 /*waves*/ * ITERS * 8 * 32768.0;   // 8 x 32x32x16 (or 16 x 16x16x32)
            printf("%s: %.3f ms/launch  %.1f TFLOP/s\n", which ? "16x16x32" : "32x32x16", ms / R, flop / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
