// Probe: vector L1 / L2 read bandwidth per CU on gfx950 for global_load_dwordx4 (the question
// behind putting the Winograd weight operand U straight into registers: can the vL1D serve
// ~190 KB per 16-channel chunk per CU next to the MFMAs?).  Each block re-reads a FOOT-byte
// window (per block: L1-resident for FOOT <= 16 KB; shared by all blocks: L2) REPS times.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/l1_bw.hip -o /tmp/l1_bw && /tmp/l1_bw
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int THREADS>
__global__ __launch_bounds__(THREADS) void rd(const f4* __restrict__ src, int foot_f4, int per_block, int reps, float* out) {
    const f4* base = src + (per_block ? (long long)blockIdx.x * foot_f4 : 0);
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    int idx = threadIdx.x;
    for (int r = 0; r < reps; ++r) {
#pragma unroll 8
        for (int i = 0; i < 8; ++i) {
            acc += base[idx];
            idx += THREADS;
            if (idx >= foot_f4) idx -= foot_f4;
        }
    }
    if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

int main() {
    int dev = 0, cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    const size_t big = (size_t)1 << 30;
    f4* src;
    float* out;
    hipMalloc(&src, big);
    hipMemset(src, 0, big);
    hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct C { int foot_kb, per_block, blocks_per_cu; };
    C cases[] = {{8, 1, 1}, {16, 1, 1}, {16, 1, 2}, {32, 1, 1}, {64, 1, 1}, {256, 0, 1}, {1024, 0, 1}, {2048, 0, 2}};
    for (const C& c : cases) {
        const int foot = c.foot_kb * 1024 / 16;
        const int blocks = cus * c.blocks_per_cu;
        const int reps = 2000;
        for (int w = 0; w < 2; ++w) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(rd<512>, dim3(blocks), dim3(512), 0, 0, src, foot, c.per_block, reps, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = (double)blocks * 512 * 16 * 8 * reps;
        const double per_cu_clk = bytes / (ms * 1e-3) / cus / (clk * 1e3);
        printf("foot %5d KB %s, %d blocks/CU: %.1f TB/s  %.1f B/clk/CU (at %d MHz)\n", c.foot_kb,
               c.per_block ? "per block" : "shared   ", c.blocks_per_cu, bytes / (ms * 1e-3) / 1e12, per_cu_clk, clk / 1000);
    }
    return 0;
}
