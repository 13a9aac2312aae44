// Probe: what buffer_load_dwordx4 ... lds writes to LDS for out-of-range lanes (gfx950), and
// whether the SGPR offset takes part in the range check.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void_t;

__global__ void probe(const float* src, int nbytes, unsigned soff, unsigned sent, float* out) {
    __shared__ __attribute__((aligned(16))) float lds[256];
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = -1.f;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nbytes, 0x00020000);
    const unsigned vo = (threadIdx.x & 1) ? sent : threadIdx.x * 16u;   // odd lanes out of range
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, vo, soff, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}

int main() {
    float h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = (float)(i + 1);
    float *d, *o;
    hipMalloc(&d, 4096); hipMalloc(&o, 1024);
    hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    float r[256];
    // case 1: soff 0, sentinel 0x80000000, records 1024 B
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 1024, 0u, 0x80000000u, o);
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    printf("case1 lane0 %g %g lane1 %g %g lane2 %g\n", r[0], r[3], r[4], r[7], r[8]);
    // case 2: records 512 B, soff 512: lane 0 voffset 0 -> address 512 in range of the 4 KB alloc,
    // beyond records if soffset counts
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 512, 512u, 0x80000000u, o);
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    printf("case2 (records 512, soff 512) lane0 %g lane2 %g lane30 %g\n", r[0], r[8], r[120]);
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
