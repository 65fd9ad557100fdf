// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte counts, for
// the access shapes the rasterizer's kernels use (development tool, DESIGN.md section 4 "Counters").
//
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d OUT -o run -- tools/fetch_calib      (and a second pass with WRITE_SIZE)
//   python tools/fetch_calib.py OUT_fetch OUT_write calib.log
//
// MI355X_MICROARCH.md ("HBM") measured FETCH_SIZE at exactly half the bytes of a wide coalesced
// streaming read and WRITE_SIZE exact for 16-B-per-lane streaming stores and float atomics; other shapes
// are uncalibrated.  render_bwd's reads are mostly per-lane gathers of 48 or 64 bytes of a 64-byte splat
// record and 4-byte gathers, so each shape below moves a KNOWN number of distinct bytes of a table far
// larger than the 256 MiB Infinity Cache, every byte exactly once (a random permutation of the record
// indices), and the tool prints that count per kernel for the counters to be divided by.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                        \
        }                                                                                        \
    } while (0)

constexpr size_t kRecs = size_t(1) << 24;  // 16M records of 64 B = 1 GiB
constexpr int kBlock = 256;

// 16 B per lane, consecutive lanes consecutive (a wide coalesced streaming read): n float4
__global__ void __launch_bounds__(kBlock) calib_stream16_read(const float4* __restrict__ src, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const float4 v = src[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;  // keeps the loads
}

// one whole 64-B record per lane (4 x 16 B), records in a random order: render's splat-record gather shape
__global__ void __launch_bounds__(kBlock) calib_gather64(const float4* __restrict__ rec, const uint32_t* __restrict__ perm,
                                                         size_t n, float* out) {
    const size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (i >= n) return;
    const float4* r = rec + 4 * (size_t)perm[i];
    const float4 a = r[0], b = r[1], c = r[2], d = r[3];
    const float s = a.x + b.y + c.z + d.w;
    if (s == 12345.f) out[0] = s;
}

// rows 0-2 (48 B) of a 64-B record per lane: render_fwd's staging shape
__global__ void __launch_bounds__(kBlock) calib_gather48(const float4* __restrict__ rec, const uint32_t* __restrict__ perm,
                                                         size_t n, float* out) {
    const size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (i >= n) return;
    const float4* r = rec + 4 * (size_t)perm[i];
    const float4 a = r[0], b = r[1], c = r[2];
    const float s = a.x + b.y + c.z;
    if (s == 12345.f) out[0] = s;
}

// 4 B per lane at a random index (render_bwd's record-start gather, the tile-list entries of other waves)
__global__ void __launch_bounds__(kBlock) calib_gather4(const uint32_t* __restrict__ src, const uint32_t* __restrict__ perm,
                                                        size_t n, float* out) {
    const size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = src[16 * (size_t)perm[i]];  // one dword of each 64-B line
    if (v == 12345u) out[0] = 1.f;
}

// 16 B per lane streaming stores (exact per the guide: the reference point of the write side)
__global__ void __launch_bounds__(kBlock) calib_stream16_write(float4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        dst[i] = make_float4((float)i, 0.f, 1.f, 2.f);
}

// one 48-B record per lane at a random 64-B slot (render_bwd's gradient-record shape; 48 of every 64 B)
__global__ void __launch_bounds__(kBlock) calib_scatter48(float4* __restrict__ dst, const uint32_t* __restrict__ perm,
                                                          size_t n) {
    const size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x;
    if (i >= n) return;
    float4* r = dst + 4 * (size_t)perm[i];
    r[0] = make_float4(1.f, 2.f, 3.f, 4.f);
    r[1] = make_float4(5.f, 6.f, 7.f, 8.f);
    r[2] = make_float4(9.f, 10.f, 0.f, 0.f);
}

int main() {
    float4 *tab = nullptr, *wtab = nullptr;
    uint32_t* perm = nullptr;
    float* out = nullptr;
    CK(hipMalloc(&tab, kRecs * 64));
    CK(hipMalloc(&wtab, kRecs * 64));
    CK(hipMalloc(&perm, kRecs * 4));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(tab, 0, kRecs * 64));
    CK(hipMemset(wtab, 0, kRecs * 64));
    std::vector<uint32_t> h(kRecs);
    std::iota(h.begin(), h.end(), 0u);
    std::shuffle(h.begin(), h.end(), std::mt19937(7));
    CK(hipMemcpy(perm, h.data(), kRecs * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    const dim3 gs(4096), gg((unsigned)(kRecs / kBlock));
    // each kernel twice (the summary takes the mean per dispatch); the perm array (64 MB) is read by the
    // gather kernels too: its 4-B-per-lane coalesced reads are part of their counts (printed separately)
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(calib_stream16_read, gs, dim3(kBlock), 0, 0, tab, kRecs * 4, out);
        hipLaunchKernelGGL(calib_gather64, gg, dim3(kBlock), 0, 0, tab, perm, kRecs, out);
        hipLaunchKernelGGL(calib_gather48, gg, dim3(kBlock), 0, 0, tab, perm, kRecs, out);
        hipLaunchKernelGGL(calib_gather4, gg, dim3(kBlock), 0, 0, (const uint32_t*)tab, perm, kRecs, out);
        hipLaunchKernelGGL(calib_stream16_write, gs, dim3(kBlock), 0, 0, wtab, kRecs * 4);
        hipLaunchKernelGGL(calib_scatter48, gg, dim3(kBlock), 0, 0, wtab, perm, kRecs);
    }
    CK(hipDeviceSynchronize());
    const double R = (double)kRecs;
    // known distinct bytes per dispatch: table part, index part (perm: 4 B per record, coalesced)
    std::printf("known calib_stream16_read read_table %.0f read_index 0 write 0\n", R * 64);
    std::printf("known calib_gather64 read_table %.0f read_index %.0f write 0\n", R * 64, R * 4);
    std::printf("known calib_gather48 read_table %.0f read_index %.0f write 0\n", R * 48, R * 4);
    std::printf("known calib_gather4 read_table %.0f read_index %.0f write 0\n", R * 4, R * 4);
    std::printf("known calib_stream16_write read_table 0 read_index 0 write %.0f\n", R * 64);
    std::printf("known calib_scatter48 read_table 0 read_index %.0f write %.0f\n", R * 4, R * 48);
    CK(hipFree(tab));
    CK(hipFree(wtab));
    CK(hipFree(perm));
    CK(hipFree(out));
    return 0;
}
