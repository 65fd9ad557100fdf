// Launch-floor probe: how long rocprofv3's kernel trace says a kernel that does (almost) nothing
// runs, by grid size and static LDS, so the per-kernel floor inside a rasterizer step is known
// (which kernel fusions could pay).  Each kernel writes one word from
// workgroup 0 so it is not empty.  Build: hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip
// -o tools/launch_floor; run under rocprofv3 --kernel-trace --stats.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LDS_WORDS>
__global__ void __launch_bounds__(256) floor_kernel(unsigned* out, unsigned n) {
    __shared__ unsigned s[LDS_WORDS];
    s[threadIdx.x % LDS_WORDS] = threadIdx.x;
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0 && n == 0xffffffffu) out[0] = s[1];
    if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = n;
}

__global__ void __launch_bounds__(64) floor64_kernel(unsigned* out, unsigned n) {
    if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = n;
}

int main() {
    unsigned* d = nullptr;
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 1;
    const unsigned grids[] = {1u, 64u, 256u, 2048u, 16384u};
    for (int rep = 0; rep < 200; ++rep) {
        for (unsigned g : grids) {
            hipLaunchKernelGGL(floor64_kernel, dim3(g), dim3(64), 0, st, d, g);
            hipLaunchKernelGGL(floor_kernel<64>, dim3(g), dim3(256), 0, st, d, g);
            hipLaunchKernelGGL(floor_kernel<20480>, dim3(g), dim3(256), 0, st, d, g);  // 80 KiB
        }
    }
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    unsigned h[2] = {0, 0};
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    std::printf("launch_floor ok last=%u\n", h[1]);
    hipFree(d);
    hipStreamDestroy(st);
    return h[1] == 16384u ? 0 : 1;
}
