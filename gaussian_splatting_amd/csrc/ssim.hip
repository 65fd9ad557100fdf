// ssim.hip -- fused SSIM forward / backward: the reference's fused-ssim
// (submodules/fused-ssim/ssim.cu:210-444, API ssim.h:8-27) rebuilt for gfx950.
//
// Semantics (kept exactly): 11x11 Gaussian window (sigma 1.5, the G_00..G_10 taps of
// ssim.cu:10-20), zero padding outside the image, per (batch, channel, pixel)
//   mu1 = G*img1, mu2 = G*img2, s11 = G*img1^2 - mu1^2, s22 = G*img2^2 - mu2^2,
//   s12 = G*(img1 img2) - mu1 mu2,
//   map = (2 mu1 mu2 + C1)(2 s12 + C2) / ((mu1^2 + mu2^2 + C1)(s11 + s22 + C2)),
// the three partial derivatives the backward needs (ssim.cu:303-311), and
//   dL/dimg1 = G*(dL dm/dmu1) + 2 img1 G*(dL dm/ds11) + img2 G*(dL dm/ds12)
// (ssim.cu:329-402).  Each separable pass accumulates its 11 taps in the
// reference's order (outermost tap first).
//
// Layout for a wave64 machine: a 256-thread workgroup owns a 64 x 64 output tile of
// one plane.  The (64 + 10)^2 input patch is staged once in LDS; lane l of wave w
// owns output column l and rows [16 w, 16 w + 16).  Walking down its 26 input rows, a
// lane filters each row horizontally from LDS (all five products at once, where the
// reference makes five passes with a barrier each) and keeps the last 11 filtered
// rows in registers, so the vertical filter never touches LDS.  The image is read
// once per tile (plus the halo) and every output is written once: the kernels are
// HBM-streaming.
#include "kernels.h"

namespace gsr {

constexpr int kSsimTile = 64;                 // output tile edge
constexpr int kSsimHalo = 5;                  // 11-tap window
constexpr int kSsimPatch = kSsimTile + 2 * kSsimHalo;  // 74
constexpr int kSsimStride = kSsimPatch + 1;   // LDS row stride (odd: conflict-free column walks)
constexpr int kSsimRowsPerWave = 16;
constexpr int kSsimThreads = 256;

__constant__ float kG[11] = {0.001028380123898387f,  0.0075987582094967365f, 0.036000773310661316f,
                             0.10936068743467331f,   0.21300552785396576f,   0.26601171493530273f,
                             0.21300552785396576f,   0.10936068743467331f,   0.036000773310661316f,
                             0.0075987582094967365f, 0.001028380123898387f};

// Stage the zero-padded (74 x 74) patch of `n` planes' worth of inputs at (x0, y0) - 5.
// The loop has a compile-time trip count and is fully unrolled, so all of a thread's loads
// are in flight together before the first LDS store (one memory latency per tile).
constexpr int kSsimStageIters = (kSsimPatch * kSsimPatch + kSsimThreads - 1) / kSsimThreads;

template <int N>
__device__ __forceinline__ void stage_patch(float (*s)[kSsimPatch][kSsimStride], const float* const* src, int H,
                                            int W, int x0, int y0) {
    float v[kSsimStageIters][N];
#pragma unroll
    for (int it = 0; it < kSsimStageIters; it++) {
        const int i = it * kSsimThreads + threadIdx.x;
        const int ly = i / kSsimPatch, lx = i - ly * kSsimPatch;
        const int y = y0 - kSsimHalo + ly, x = x0 - kSsimHalo + lx;
        const bool in = i < kSsimPatch * kSsimPatch && x >= 0 && x < W && y >= 0 && y < H;
#pragma unroll
        for (int k = 0; k < N; k++) v[it][k] = in ? src[k][(size_t)y * W + x] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < kSsimStageIters; it++) {
        const int i = it * kSsimThreads + threadIdx.x;
        if (i >= kSsimPatch * kSsimPatch) break;
        const int ly = i / kSsimPatch, lx = i - ly * kSsimPatch;
#pragma unroll
        for (int k = 0; k < N; k++) s[k][ly][lx] = v[it][k];
    }
}

// ---- forward -------------------------------------------------------------------
template <bool TRAIN>
__global__ void __launch_bounds__(kSsimThreads) ssim_fwd_kernel(int H, int W, float C1, float C2,
                                                                const float* __restrict__ img1,
                                                                const float* __restrict__ img2,
                                                                float* __restrict__ map, float* __restrict__ dm_dmu1,
                                                                float* __restrict__ dm_ds11,
                                                                float* __restrict__ dm_ds12) {
    __shared__ float s[2][kSsimPatch][kSsimStride];
    const size_t plane = (size_t)blockIdx.z * H * W;
    const int x0 = blockIdx.x * kSsimTile, y0 = blockIdx.y * kSsimTile;
    const float* srcs[2] = {img1 + plane, img2 + plane};
    stage_patch<2>(s, srcs, H, W, x0, y0);
    __syncthreads();

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int x = x0 + lane;
    // filtered rows (five products) of the last 11 input rows, indexed by row % 11
    float h1[11], h2[11], h11[11], h22[11], h12[11];
#pragma unroll
    for (int r = 0; r < kSsimRowsPerWave + 2 * kSsimHalo; r++) {
        const int ly = w * kSsimRowsPerWave + r;  // patch row
        float a1 = 0.f, a2 = 0.f, a11 = 0.f, a22 = 0.f, a12 = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            const float p = s[0][ly][lane + k], q = s[1][ly][lane + k];
            a1 += kG[k] * p;
            a11 += kG[k] * (p * p);
            a2 += kG[k] * q;
            a22 += kG[k] * (q * q);
            a12 += kG[k] * (p * q);
        }
        h1[r % 11] = a1;
        h2[r % 11] = a2;
        h11[r % 11] = a11;
        h22[r % 11] = a22;
        h12[r % 11] = a12;
        if (r < 2 * kSsimHalo) continue;
        const int y = y0 + w * kSsimRowsPerWave + r - 2 * kSsimHalo;
        float mu1 = 0.f, mu2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            const int j = (r - 10 + k) % 11;
            mu1 += kG[k] * h1[j];
            e11 += kG[k] * h11[j];
            mu2 += kG[k] * h2[j];
            e22 += kG[k] * h22[j];
            e12 += kG[k] * h12[j];
        }
        if (x >= W || y >= H) continue;
        const float sigma1_sq = e11 - mu1 * mu1, sigma2_sq = e22 - mu2 * mu2, sigma12 = e12 - mu1 * mu2;
        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
        const float C = (2.0f * mu1_mu2 + C1);
        const float D = (2.0f * sigma12 + C2);
        const float A = (mu1_sq + mu2_sq + C1);
        const float B = (sigma1_sq + sigma2_sq + C2);
        const size_t o = plane + (size_t)y * W + x;
        map[o] = (C * D) / (A * B);
        if (TRAIN) {  // ssim.cu:303-311
            dm_dmu1[o] = ((mu2 * 2.0f * D) / (A * B) - (mu2 * 2.0f * C) / (A * B) - (mu1 * 2.0f * C * D) / (A * A * B) +
                          (mu1 * 2.0f * C * D) / (A * B * B));
            dm_ds11[o] = ((-C * D) / (A * B * B));
            dm_ds12[o] = ((2 * C) / (A * B));
        }
    }
}

// ---- backward ------------------------------------------------------------------
__global__ void __launch_bounds__(kSsimThreads) ssim_bwd_kernel(int H, int W, const float* __restrict__ img1,
                                                                const float* __restrict__ img2,
                                                                const float* __restrict__ dL_dmap,
                                                                const float* __restrict__ dm_dmu1,
                                                                const float* __restrict__ dm_ds11,
                                                                const float* __restrict__ dm_ds12,
                                                                float* __restrict__ dL_dimg1) {
    __shared__ float s[3][kSsimPatch][kSsimStride];
    const size_t plane = (size_t)blockIdx.z * H * W;
    const int x0 = blockIdx.x * kSsimTile, y0 = blockIdx.y * kSsimTile;
    // the three products dL/dmap * dm/d(.) (ssim.cu:350, 366, 382), zero outside the image
    {
        const float* srcs[4] = {dL_dmap + plane, dm_dmu1 + plane, dm_ds11 + plane, dm_ds12 + plane};
        float v[kSsimStageIters][4];
#pragma unroll
        for (int it = 0; it < kSsimStageIters; it++) {
            const int i = it * kSsimThreads + threadIdx.x;
            const int ly = i / kSsimPatch, lx = i - ly * kSsimPatch;
            const int y = y0 - kSsimHalo + ly, xx = x0 - kSsimHalo + lx;
            const bool in = i < kSsimPatch * kSsimPatch && xx >= 0 && xx < W && y >= 0 && y < H;
#pragma unroll
            for (int k = 0; k < 4; k++) v[it][k] = in ? srcs[k][(size_t)y * W + xx] : 0.f;
        }
#pragma unroll
        for (int it = 0; it < kSsimStageIters; it++) {
            const int i = it * kSsimThreads + threadIdx.x;
            if (i >= kSsimPatch * kSsimPatch) break;
            const int ly = i / kSsimPatch, lx = i - ly * kSsimPatch;
            s[0][ly][lx] = v[it][1] * v[it][0];
            s[1][ly][lx] = v[it][2] * v[it][0];
            s[2][ly][lx] = v[it][3] * v[it][0];
        }
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int x = x0 + lane;
    float h0[11], h1[11], h2[11];
#pragma unroll
    for (int r = 0; r < kSsimRowsPerWave + 2 * kSsimHalo; r++) {
        const int ly = w * kSsimRowsPerWave + r;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            a0 += kG[k] * s[0][ly][lane + k];
            a1 += kG[k] * s[1][ly][lane + k];
            a2 += kG[k] * s[2][ly][lane + k];
        }
        h0[r % 11] = a0;
        h1[r % 11] = a1;
        h2[r % 11] = a2;
        if (r < 2 * kSsimHalo) continue;
        const int y = y0 + w * kSsimRowsPerWave + r - 2 * kSsimHalo;
        float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            const int j = (r - 10 + k) % 11;
            t0 += kG[k] * h0[j];
            t1 += kG[k] * h1[j];
            t2 += kG[k] * h2[j];
        }
        if (x >= W || y >= H) continue;
        const size_t o = plane + (size_t)y * W + x;
        float d = 0.f;
        d += t0;                     // from mu1
        d += img1[o] * 2.0f * t1;    // from sigma1_sq
        d += img2[o] * t2;           // from sigma12
        dL_dimg1[o] = d;
    }
}

hipError_t launch_ssim_fwd(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* map, float* dm_dmu1, float* dm_ds11, float* dm_ds12, hipStream_t stream) {
    if (planes <= 0 || H <= 0 || W <= 0) return hipSuccess;
    const dim3 grid((W + kSsimTile - 1) / kSsimTile, (H + kSsimTile - 1) / kSsimTile, planes);
    if (dm_dmu1)
        hipLaunchKernelGGL(ssim_fwd_kernel<true>, grid, dim3(kSsimThreads), 0, stream, H, W, C1, C2, img1, img2, map,
                           dm_dmu1, dm_ds11, dm_ds12);
    else
        hipLaunchKernelGGL(ssim_fwd_kernel<false>, grid, dim3(kSsimThreads), 0, stream, H, W, C1, C2, img1, img2, map,
                           nullptr, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_ssim_bwd(int planes, int H, int W, const float* img1, const float* img2, const float* dL_dmap,
                           const float* dm_dmu1, const float* dm_ds11, const float* dm_ds12, float* dL_dimg1,
                           hipStream_t stream) {
    if (planes <= 0 || H <= 0 || W <= 0) return hipSuccess;
    const dim3 grid((W + kSsimTile - 1) / kSsimTile, (H + kSsimTile - 1) / kSsimTile, planes);
    hipLaunchKernelGGL(ssim_bwd_kernel, grid, dim3(kSsimThreads), 0, stream, H, W, img1, img2, dL_dmap, dm_dmu1,
                       dm_ds11, dm_ds12, dL_dimg1);
    return hipGetLastError();
}

}  // namespace gsr
