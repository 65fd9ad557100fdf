// valu_rate.hip -- microbenchmark: wave64 VALU issue rate on gfx950 for plain and packed fp32
// and for the transcendentals the render kernels use (development tool).
//
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o tools/valu_rate && tools/valu_rate
//
// Each lane runs 8 independent dependency chains (so one wave alone is not latency-bound)
// for ITERS iterations; the grid puts WAVES waves on every SIMD.  Reported: cycles per
// wave64 instruction per SIMD, from hipEvent time at the nominal 2.4 GHz clock.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 4096;

__global__ void __launch_bounds__(256) k_fma(float* out, float a, float b) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_pkfma(float* out, float a, float b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 x[8];
    const f2 va = {a, a}, vb = {b, b};
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = f2{threadIdx.x * 0.001f + i, (float)i};
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(va), "v"(vb));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_exp(float* out, float a, float b) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = -(threadIdx.x * 0.001f + i);
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mix(float* out, float a, float b) {
    // 3 plain fma : 1 exp, the render kernels' rough mix
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (i % 4 == 3)
                asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
            else
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char* name, K kern, int waves_per_simd, float* out) {
    const int blocks = 256 * waves_per_simd;  // 256 threads = 4 waves = one per SIMD of a CU
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double insts_per_simd = 5.0 * waves_per_simd * ITERS * 8;  // wave64 instructions per SIMD
    const double cycles = ms * 1e-3 / 5.0 * 2.4e9 * 5.0;
    printf("%-8s waves/SIMD %d: %.2f cycles per wave64 instruction per SIMD (%.3f ms)\n", name, waves_per_simd,
           cycles / insts_per_simd, ms);
}

int main() {
    float* out;
    hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
    for (int w : {1, 2, 4, 8}) {
        run("fma", k_fma, w, out);
        run("pk_fma", k_pkfma, w, out);
        run("exp", k_exp, w, out);
        run("3fma+exp", k_mix, w, out);
    }
    hipFree(out);
    return 0;
}
