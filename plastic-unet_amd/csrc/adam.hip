// Multi-tensor Adam: one launch for every parameter tensor of the model.
//
// Replaces torch.optim.Adam(net.parameters(), lr).step() (yaricom/Plastic-UNet src/train.py:66,111),
// whose single-tensor update is, per element (amsgrad=False, maximize=False):
//   g += wd * p (if weight_decay) ; m = lerp(m, g, 1-beta1) ; v = v*beta2 + (1-beta2)*g*g
//   p = p - step_size * m / (sqrt(v)/bc2_sqrt + eps),  step_size = lr/(1-beta1^t), bc2_sqrt = sqrt(1-beta2^t)
// HBM-bound: 4 reads + 3 writes of 4 bytes per element, float4 per lane.
#include "common.h"

#include <math.h>

namespace pu {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ADAM_MAX_T = 32;
constexpr int ADAM_CHUNK = 256 * 4 * 4;   // elements per block (256 threads x 4 float4)

struct AdamBatch {
    float* p[ADAM_MAX_T];
    const float* g[ADAM_MAX_T];
    float* m[ADAM_MAX_T];
    float* v[ADAM_MAX_T];
    long long n[ADAM_MAX_T];
    int block_start[ADAM_MAX_T + 1];
    int count;
};

__device__ __forceinline__ float adam_one(float& p, float g, float& m, float& v, float omb1, float b2, float omb2,
                                          float eps, float wd, float step_size, float bc2s) {
#pragma clang fp contract(off)
    if (wd != 0.f) g = g + wd * p;
    // ATen lerp (weight < 0.5): self + weight * (end - self)
    m = m + omb1 * (g - m);
    v = v * b2 + omb2 * g * g;
    const float denom = sqrtf(v) / bc2s + eps;
    p = p + (-step_size) * (m / denom);
    return p;
}

__global__ __launch_bounds__(256) void adam_kernel(const AdamBatch batch, float omb1, float b2, float omb2, float eps, float wd,
                                                   float step_size, float bc2s) {
    // locate this block's tensor (count <= 32: linear scan of the prefix table)
    int t = 0;
    while (t + 1 < batch.count && (int)blockIdx.x >= batch.block_start[t + 1]) ++t;
    const long long n = batch.n[t];
    const long long base = (long long)(blockIdx.x - batch.block_start[t]) * ADAM_CHUNK;
    float* P = batch.p[t];
    const float* G = batch.g[t];
    float* M = batch.m[t];
    float* V = batch.v[t];
    const bool aligned = ((((uintptr_t)P) | ((uintptr_t)G) | ((uintptr_t)M) | ((uintptr_t)V)) & 15) == 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const long long i = base + ((long long)it * 256 + threadIdx.x) * 4;
        if (i >= n) break;
        if (aligned && i + 3 < n) {
            f32x4 p = *reinterpret_cast<f32x4*>(P + i);
            f32x4 g = *reinterpret_cast<const f32x4*>(G + i);
            f32x4 m = *reinterpret_cast<f32x4*>(M + i);
            f32x4 v = *reinterpret_cast<f32x4*>(V + i);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float pe = p[e], me = m[e], ve = v[e];
                adam_one(pe, g[e], me, ve, omb1, b2, omb2, eps, wd, step_size, bc2s);
                p[e] = pe; m[e] = me; v[e] = ve;
            }
            *reinterpret_cast<f32x4*>(P + i) = p;
            *reinterpret_cast<f32x4*>(M + i) = m;
            *reinterpret_cast<f32x4*>(V + i) = v;
        } else {
            for (long long e = i; e < i + 4 && e < n; ++e) adam_one(P[e], G[e], M[e], V[e], omb1, b2, omb2, eps, wd, step_size, bc2s);
        }
    }
}

}  // namespace pu

using namespace pu;

extern "C" int pu_adam_multi(const pu_adam_tensor* tensors, int n_tensors, double beta1, double beta2, double eps,
                             double weight_decay, double step_size, double bc2_sqrt, void* stream) {
    PU_REQUIRE(n_tensors >= 0 && (n_tensors == 0 || tensors), "pu_adam_multi: bad tensor list");
    int i = 0;
    while (i < n_tensors) {
        AdamBatch b;
        b.count = 0;
        int blocks = 0;
        while (i < n_tensors && b.count < ADAM_MAX_T) {
            const pu_adam_tensor& t = tensors[i++];
            PU_REQUIRE(t.param && t.grad && t.exp_avg && t.exp_avg_sq && t.numel >= 0, "pu_adam_multi: tensor %d", i - 1);
            if (t.numel == 0) continue;
            b.p[b.count] = t.param; b.g[b.count] = t.grad; b.m[b.count] = t.exp_avg; b.v[b.count] = t.exp_avg_sq;
            b.n[b.count] = t.numel;
            b.block_start[b.count] = blocks;
            blocks += (int)((t.numel + ADAM_CHUNK - 1) / ADAM_CHUNK);
            b.count++;
        }
        b.block_start[b.count] = blocks;
        if (b.count == 0) continue;
        hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), b, (float)(1.0 - beta1),
                           (float)beta2, (float)(1.0 - beta2), (float)eps, (float)weight_decay, (float)step_size,
                           (float)bc2_sqrt);
        int st = check_launch("pu_adam_multi");
        if (st != PU_OK) return st;
    }
    return PU_OK;
}
