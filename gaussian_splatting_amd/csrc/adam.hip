// adam.hip -- the sparse Adam step of SparseGaussianAdam (include/gsr_adam.h).
//
// Semantics: the 3DGS-accel rasterizer's adamUpdate (not vendored by the reference;
// SURVEY.md section 8f row 3).  Per element i < N*M of a parameter tensor, if Gaussian
// i / M is visible: m = b1 m + (1-b1) g; v = b2 v + (1-b2) g g; p += -lr m / (sqrt(v) + eps).
//
// MI355X structure: the step is a pure stream over param, grad, exp_avg and exp_avg_sq
// (16 B read + 12 B written per visible element, nothing for an invisible one), so it is
// HBM-bound and the kernel is organised for that alone:
//  * all parameter groups of one optimizer step (xyz, f_dc, f_rest, opacity, scaling,
//    rotation: scene/gaussian_model.py:235-242) in ONE launch -- each group owns a
//    contiguous range of workgroups, found by a wave-uniform scan of <= 8 bounds;
//  * 16-byte loads and stores of four consecutive elements; a float4 whose four
//    Gaussians are all invisible issues no memory access at all;
//  * element -> Gaussian by a multiply-shift division (exact for i < 2^31, magic number
//    from the host), so the per-element visibility lookup costs a v_mad_u64_u32.
#include "kernels.h"

namespace gsr {

__device__ __forceinline__ uint32_t gauss_of(uint32_t i, const AdamGroupDev& G) {
    return (uint32_t)(((unsigned long long)i * G.magic) >> G.shift);
}

// One element, in the reference's operation order, without contraction into FMAs.
__device__ __forceinline__ float adam_elem(float p, float g, float& m, float& v, float lr, float b1, float b2,
                                           float eps) {
#pragma clang fp contract(off)
    m = b1 * m + (1.0f - b1) * g;
    v = b2 * v + (1.0f - b2) * g * g;
    const float step = -lr * m / (sqrtf(v) + eps);
    return p + step;
}

__global__ void __launch_bounds__(kAdamThreads) adam_kernel(AdamArgs a) {
    int k = 0;
    while (k + 1 < a.n_groups && blockIdx.x >= a.grp[k + 1].first_block) k++;  // wave-uniform
    const AdamGroupDev& G = a.grp[k];
    const uint32_t base = (blockIdx.x - G.first_block) * kAdamBlockElems;
    if (G.vec) {
#pragma unroll
        for (int u = 0; u < kAdamUnroll; u++) {
            const uint32_t e = base + (u * kAdamThreads + threadIdx.x) * 4;
            if (e + 3 < G.n) {
                bool vis[4];
                bool any = false;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    vis[c] = a.vis[gauss_of(e + c, G)] != 0;
                    any |= vis[c];
                }
                if (!any) continue;
                float4 p = *reinterpret_cast<const float4*>(G.p + e);
                const float4 g = *reinterpret_cast<const float4*>(G.g + e);
                float4 m = *reinterpret_cast<const float4*>(G.m + e);
                float4 v = *reinterpret_cast<const float4*>(G.v + e);
                if (vis[0]) p.x = adam_elem(p.x, g.x, m.x, v.x, G.lr, a.b1, a.b2, G.eps);
                if (vis[1]) p.y = adam_elem(p.y, g.y, m.y, v.y, G.lr, a.b1, a.b2, G.eps);
                if (vis[2]) p.z = adam_elem(p.z, g.z, m.z, v.z, G.lr, a.b1, a.b2, G.eps);
                if (vis[3]) p.w = adam_elem(p.w, g.w, m.w, v.w, G.lr, a.b1, a.b2, G.eps);
                *reinterpret_cast<float4*>(G.p + e) = p;
                *reinterpret_cast<float4*>(G.m + e) = m;
                *reinterpret_cast<float4*>(G.v + e) = v;
            } else {
                for (uint32_t i = e; i < G.n && i < e + 4; i++) {  // the group's last 1-3 elements
                    if (!a.vis[gauss_of(i, G)]) continue;
                    float m = G.m[i], v = G.v[i];
                    G.p[i] = adam_elem(G.p[i], G.g[i], m, v, G.lr, a.b1, a.b2, G.eps);
                    G.m[i] = m;
                    G.v[i] = v;
                }
            }
        }
    } else {
        for (uint32_t j = threadIdx.x; j < kAdamBlockElems; j += kAdamThreads) {
            const uint32_t i = base + j;
            if (i >= G.n || !a.vis[gauss_of(i, G)]) continue;
            float m = G.m[i], v = G.v[i];
            G.p[i] = adam_elem(G.p[i], G.g[i], m, v, G.lr, a.b1, a.b2, G.eps);
            G.m[i] = m;
            G.v[i] = v;
        }
    }
}

hipError_t launch_adam(const AdamArgs& a, uint32_t blocks, hipStream_t stream) {
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(kAdamThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
