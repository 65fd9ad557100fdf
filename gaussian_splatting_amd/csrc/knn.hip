// knn.hip -- mean squared distance to the 3 nearest neighbours of every point: the
// reference's simple-knn (submodules/simple-knn/simple_knn.cu:172-221, distCUDA2 in
// spatial.cu:14-25), rebuilt for gfx950.
//
// Same structure as the reference -- points in Morton order, boxes of 1024
// consecutive sorted points, a first bound from the 3 sorted-order neighbours on each
// side, then every box whose distance can beat the bound is scanned -- but laid out
// for a wave64 machine:
//  * the bounding box is reduced on the device (the reference copies min and max
//    back to the host twice); the reference's reduction starts from {0,0,0}, which
//    clamps min <= 0 <= max, and this one does the same (it only shapes the Morton
//    grid);
//  * the (Morton, index) pairs are sorted with rocPRIM's radix sort over the 30
//    code bits;
//  * the sorted points are gathered once into float4 rows, so the scans read
//    contiguous memory;
//  * the query runs one lane per sorted point.  64 consecutive Morton points are
//    close together, so the wave walks the boxes in lockstep: a box is scanned when
//    any lane needs it (the lanes that do not are masked), and the scanned points
//    are wave-uniform loads.
// The per-lane candidate test and update are the reference's (strict '>' insertion,
// simple_knn.cu:121-134), and every candidate whose distance could enter the best
// three is visited, so the result is the exact 3-NN mean whatever the traversal order.
#include <cfloat>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "kernels.h"

namespace gsr {

constexpr int kKnnBox = 1024;  // points per box (the reference's BOX_SIZE)
constexpr int kKnnThreads = 256;

struct Box {
    float4 mn, mx;
};

__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {  // simple_knn.cu:46-53
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}

// Per-block partial min / max, then one block folds them (starting from {0,0,0}).
__global__ void __launch_bounds__(kKnnThreads) knn_bounds_partial(int P, const float* __restrict__ pts,
                                                                   float4* __restrict__ partial) {
    __shared__ float s[6][kKnnThreads / 64];
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * kKnnThreads + threadIdx.x; i < P; i += gridDim.x * kKnnThreads) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float v = pts[3 * i + k];
            mn[k] = fminf(mn[k], v);
            mx[k] = fmaxf(mx[k], v);
        }
    }
#pragma unroll
    for (int k = 0; k < 3; k++)
        for (int off = 32; off > 0; off >>= 1) {
            mn[k] = fminf(mn[k], __shfl_xor(mn[k], off));
            mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], off));
        }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; k++) {
            s[k][w] = mn[k];
            s[3 + k][w] = mx[k];
        }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < kKnnThreads / 64; i++)
            for (int k = 0; k < 3; k++) {
                s[k][0] = fminf(s[k][0], s[k][i]);
                s[3 + k][0] = fmaxf(s[3 + k][0], s[3 + k][i]);
            }
        partial[2 * blockIdx.x] = make_float4(s[0][0], s[1][0], s[2][0], 0.f);
        partial[2 * blockIdx.x + 1] = make_float4(s[3][0], s[4][0], s[5][0], 0.f);
    }
}

__global__ void __launch_bounds__(64) knn_bounds_final(int nparts, float4* __restrict__ partial) {
    // cub::DeviceReduce with init {0,0,0} (simple_knn.cu:179-189)
    float4 mn = make_float4(0.f, 0.f, 0.f, 0.f), mx = mn;
    for (int i = threadIdx.x; i < nparts; i += 64) {
        const float4 a = partial[2 * i], b = partial[2 * i + 1];
        mn = make_float4(fminf(mn.x, a.x), fminf(mn.y, a.y), fminf(mn.z, a.z), 0.f);
        mx = make_float4(fmaxf(mx.x, b.x), fmaxf(mx.y, b.y), fmaxf(mx.z, b.z), 0.f);
    }
    for (int off = 32; off > 0; off >>= 1) {
        mn.x = fminf(mn.x, __shfl_xor(mn.x, off));
        mn.y = fminf(mn.y, __shfl_xor(mn.y, off));
        mn.z = fminf(mn.z, __shfl_xor(mn.z, off));
        mx.x = fmaxf(mx.x, __shfl_xor(mx.x, off));
        mx.y = fmaxf(mx.y, __shfl_xor(mx.y, off));
        mx.z = fmaxf(mx.z, __shfl_xor(mx.z, off));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[0] = mn;
        partial[1] = mx;
    }
}

// coord2Morton (simple_knn.cu:55-72): 10 bits per axis over the (clamped) bounding box.
__global__ void __launch_bounds__(kKnnThreads) knn_morton(int P, const float* __restrict__ pts,
                                                          const float4* __restrict__ bounds,
                                                          uint32_t* __restrict__ code, uint32_t* __restrict__ idx) {
    const int i = blockIdx.x * kKnnThreads + threadIdx.x;
    if (i >= P) return;
    const float4 mn = bounds[0], mx = bounds[1];
    const uint32_t x = prep_morton((uint32_t)(((pts[3 * i] - mn.x) / (mx.x - mn.x)) * ((1 << 10) - 1)));
    const uint32_t y = prep_morton((uint32_t)(((pts[3 * i + 1] - mn.y) / (mx.y - mn.y)) * ((1 << 10) - 1)));
    const uint32_t z = prep_morton((uint32_t)(((pts[3 * i + 2] - mn.z) / (mx.z - mn.z)) * ((1 << 10) - 1)));
    code[i] = x | (y << 1) | (z << 2);
    idx[i] = (uint32_t)i;
}

// Sorted points as float4 rows, and the min / max of every box of kKnnBox of them.
__global__ void __launch_bounds__(kKnnThreads) knn_boxes(int P, const float* __restrict__ pts,
                                                         const uint32_t* __restrict__ idx_sorted,
                                                         float4* __restrict__ sp, Box* __restrict__ boxes) {
    __shared__ float s[6][kKnnThreads / 64];
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    const int b0 = blockIdx.x * kKnnBox;
    for (int i = b0 + threadIdx.x; i < min(P, b0 + kKnnBox); i += kKnnThreads) {
        const uint32_t g = idx_sorted[i];
        const float4 p = make_float4(pts[3 * g], pts[3 * g + 1], pts[3 * g + 2], 0.f);
        sp[i] = p;
        mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
        mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
    }
#pragma unroll
    for (int k = 0; k < 3; k++)
        for (int off = 32; off > 0; off >>= 1) {
            mn[k] = fminf(mn[k], __shfl_xor(mn[k], off));
            mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], off));
        }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; k++) {
            s[k][w] = mn[k];
            s[3 + k][w] = mx[k];
        }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < kKnnThreads / 64; i++)
            for (int k = 0; k < 3; k++) {
                s[k][0] = fminf(s[k][0], s[k][i]);
                s[3 + k][0] = fmaxf(s[3 + k][0], s[3 + k][i]);
            }
        boxes[blockIdx.x] = Box{make_float4(s[0][0], s[1][0], s[2][0], 0.f), make_float4(s[3][0], s[4][0], s[5][0], 0.f)};
    }
}

// distBoxPoint (simple_knn.cu:108-118)
__device__ __forceinline__ float dist_box_point(const Box& b, float3 p) {
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (p.x < b.mn.x || p.x > b.mx.x) dx = fminf(fabsf(p.x - b.mn.x), fabsf(p.x - b.mx.x));
    if (p.y < b.mn.y || p.y > b.mx.y) dy = fminf(fabsf(p.y - b.mn.y), fabsf(p.y - b.mx.y));
    if (p.z < b.mn.z || p.z > b.mx.z) dz = fminf(fabsf(p.z - b.mn.z), fabsf(p.z - b.mx.z));
    return dx * dx + dy * dy + dz * dz;
}

// updateKBest<3> (simple_knn.cu:120-135): insertion with strict '>'.
__device__ __forceinline__ void update3(float3 ref, float4 q, float* best) {
    const float dx = q.x - ref.x, dy = q.y - ref.y, dz = q.z - ref.z;
    float d = dx * dx + dy * dy + dz * dz;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        if (best[j] > d) {
            const float t = best[j];
            best[j] = d;
            d = t;
        }
    }
}

// boxMeanDist (simple_knn.cu:137-170), one lane per sorted point.
__global__ void __launch_bounds__(kKnnThreads) knn_query(int P, const float4* __restrict__ sp,
                                                         const uint32_t* __restrict__ idx_sorted,
                                                         const Box* __restrict__ boxes, int nboxes,
                                                         float* __restrict__ out) {
    const int pos = blockIdx.x * kKnnThreads + threadIdx.x;
    const bool valid = pos < P;
    const float4 p4 = valid ? sp[pos] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float3 p = make_float3(p4.x, p4.y, p4.z);
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    if (valid)
        for (int i = max(0, pos - 3); i <= min(P - 1, pos + 3); i++)
            if (i != pos) update3(p, sp[i], best);
    const float reject = best[2];
    best[0] = best[1] = best[2] = FLT_MAX;
    for (int b = 0; b < nboxes; b++) {  // wave-uniform
        const Box box = boxes[b];
        const float d = dist_box_point(box, p);
        const bool need = valid && !(d > reject || d > best[2]);
        if (!__any(need)) continue;
        const int lo = b * kKnnBox, hi = min(P, lo + kKnnBox);
        for (int i = lo; i < hi; i++) {  // uniform loads of the box's points
            const float4 q = sp[i];
            if (need && i != pos) update3(p, q, best);
        }
    }
    if (valid) out[idx_sorted[pos]] = (best[0] + best[1] + best[2]) / 3.0f;
}

// ---- host side ------------------------------------------------------------------
namespace {
struct KnnCarve {
    uint32_t *code, *code_sorted, *idx, *idx_sorted;
    float4* bounds;  // [2 * nparts]
    float4* sp;
    Box* boxes;
    void* temp;
    size_t temp_bytes;
};

int knn_parts(int P) {
    int n = (P + kKnnThreads - 1) / kKnnThreads;
    return n < 1024 ? (n < 1 ? 1 : n) : 1024;
}

KnnCarve carve_knn(char* base, int P, size_t temp_bytes, size_t* total) {
    Carver c{base, 0};
    KnnCarve k{};
    k.code = c.take<uint32_t>(P);
    k.code_sorted = c.take<uint32_t>(P);
    k.idx = c.take<uint32_t>(P);
    k.idx_sorted = c.take<uint32_t>(P);
    k.bounds = c.take<float4>(2 * (size_t)knn_parts(P));
    k.sp = c.take<float4>(P);
    k.boxes = c.take<Box>((P + kKnnBox - 1) / kKnnBox);
    k.temp = c.take<char>(temp_bytes);
    k.temp_bytes = temp_bytes;
    *total = align_up(c.off);
    return k;
}
}  // namespace

size_t knn_scratch_bytes(int P) {
    size_t temp = 0;
    (void)rocprim::radix_sort_pairs(nullptr, temp, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                    (uint32_t*)nullptr, (size_t)P, 0, 30);
    size_t total = 0;
    carve_knn(nullptr, P, temp, &total);
    return total;
}

hipError_t launch_knn(int P, const float* pts, float* out, void* scratch, hipStream_t stream) {
    if (P <= 0) return hipSuccess;
    size_t temp = 0, total = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, temp, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)P, 0, 30);
    if (e != hipSuccess) return e;
    KnnCarve k = carve_knn((char*)scratch, P, temp, &total);
    const int parts = knn_parts(P);
    hipLaunchKernelGGL(knn_bounds_partial, dim3(parts), dim3(kKnnThreads), 0, stream, P, pts, k.bounds);
    hipLaunchKernelGGL(knn_bounds_final, dim3(1), dim3(64), 0, stream, parts, k.bounds);
    hipLaunchKernelGGL(knn_morton, dim3((P + kKnnThreads - 1) / kKnnThreads), dim3(kKnnThreads), 0, stream, P, pts,
                       k.bounds, k.code, k.idx);
    e = rocprim::radix_sort_pairs(k.temp, temp, k.code, k.code_sorted, k.idx, k.idx_sorted, (size_t)P, 0, 30, stream);
    if (e != hipSuccess) return e;
    const int nboxes = (P + kKnnBox - 1) / kKnnBox;
    hipLaunchKernelGGL(knn_boxes, dim3(nboxes), dim3(kKnnThreads), 0, stream, P, pts, k.idx_sorted, k.sp, k.boxes);
    hipLaunchKernelGGL(knn_query, dim3((P + kKnnThreads - 1) / kKnnThreads), dim3(kKnnThreads), 0, stream, P, k.sp,
                       k.idx_sorted, k.boxes, nboxes, out);
    return hipGetLastError();
}

}  // namespace gsr
