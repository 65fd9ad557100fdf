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

// A kernel that leaves many dirty lines behind (one 4-byte store per thread, 64 B apart, like a sort's
// scattered list writes), followed back to back by an empty one: does the empty kernel's traced duration
// grow with what its predecessor wrote (the end-of-kernel write-back)?  (round 6: the class-1 sort kernel
// costs 4.6 us with nothing to sort, 2.7 over the floor above.)
__global__ void __launch_bounds__(256) dirty_kernel(unsigned* buf, unsigned n) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) buf[(size_t)i * 16u] = i;
}
__global__ void __launch_bounds__(256) after_dirty_kernel(unsigned* out, unsigned n) {
    if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = n;
}
__global__ void __launch_bounds__(256) after_clean_kernel(unsigned* out, unsigned n) {
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
    // dirty lines: 2M stores 64 B apart (128 MB of lines touched), then an empty kernel at once; and the
    // same empty kernel after an empty one (clean)
    unsigned* big = nullptr;
    const unsigned nd = 1u << 21;
    if (hipMalloc(&big, (size_t)nd * 64) != hipSuccess) return 1;
    for (int rep = 0; rep < 100; ++rep) {
        hipLaunchKernelGGL(dirty_kernel, dim3(nd / 256), dim3(256), 0, st, big, nd);
        hipLaunchKernelGGL(after_dirty_kernel, dim3(64), dim3(256), 0, st, d, 64u);
        hipLaunchKernelGGL(floor64_kernel, dim3(1), dim3(64), 0, st, d, 1u);
        hipLaunchKernelGGL(after_clean_kernel, dim3(64), dim3(256), 0, st, d, 64u);
    }
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    hipFree(big);
    // the last kernel of the loop above wrote 64; the floor loop's last value is checked below
    hipLaunchKernelGGL(floor64_kernel, dim3(1), dim3(64), 0, st, d, 16384u);
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    unsigned h[2] = {0, 0};
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    std::printf("launch_floor ok last=%u\n", h[1]);
    hipFree(d);
    hipStreamDestroy(st);
    return h[1] == 16384u ? 0 : 1;
}
