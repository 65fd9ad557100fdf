// densify.hip -- adaptive density control (include/gsr_densify.h).
//
// The reference does this in torch: boolean masks, a dozen index/cat/repeat ops per parameter
// group, fresh allocations for every intermediate, and a host sync per boolean index
// (scene/gaussian_model.py:400-654).  Here it is three passes over the Gaussians:
//
//   plan  (one thread per Gaussian)  decisions -> flag byte, per-block counts of the four
//                                    output sections (kept originals, clones, children, splits)
//   scan  (one workgroup)            exclusive scan of the block counts, section totals
//   index (one thread per Gaussian)  block-local ranks by wave ballots -> each Gaussian's rows
//                                    in the new arrays (int4: kept row, clone row, first child
//                                    row, split rank), or -1
//   apply (one thread per float of a group)  the copies: coalesced reads of the old rows, runs
//                                    of consecutive writes for kept rows; children's xyz and
//                                    scaling computed in flight; new rows' Adam moments zeroed
//
// plan, scan and index are HBM-light (24 B read, 17 B written per Gaussian); apply moves each
// parameter and moment once (HBM-bound).  No atomics: the output order is the reference's
// exactly and the result is bitwise reproducible.
#include "kernels.h"

namespace gsr {

constexpr int kDenThreads = 256;
constexpr int kDenWaves = kDenThreads / 64;

enum : uint8_t { kKeepA = 1, kKeepB = 2, kKeepC = 4, kSplit = 8 };

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.f / (1.f + expf(-x)); }

// ---- train.py:212-215 ---------------------------------------------------------------
__global__ void __launch_bounds__(kDenThreads) densify_stats_kernel(int P, const float* __restrict__ vgrad,
                                                                    const int* __restrict__ radii,
                                                                    const uint8_t* __restrict__ visible,
                                                                    float* __restrict__ accum, float* __restrict__ denom,
                                                                    float* __restrict__ max_r) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * kDenThreads + threadIdx.x;
    if (i >= P) return;
    const int r = radii ? radii[i] : 0;
    const bool vis = visible ? visible[i] != 0 : r > 0;
    if (!vis) return;
    if (vgrad) {
        const float gx = vgrad[3 * (size_t)i], gy = vgrad[3 * (size_t)i + 1];
        accum[i] += sqrtf(gx * gx + gy * gy);
        denom[i] += 1.f;
    }
    if (radii && max_r) max_r[i] = fmaxf(max_r[i], (float)r);
}

// ---- plan ---------------------------------------------------------------------------
// The four section flags of one Gaussian (gaussian_model.py:508-640).  A clone has its
// parent's opacity and scaling, and both children of a split share theirs, so one prune test
// each covers every copy.
__device__ __forceinline__ uint8_t densify_flags(float accum, float denom, float opacity, const float* s,
                                                 const DensifyArgs& a) {
#pragma clang fp contract(off)
    float g = accum / denom;
    if (g != g) g = 0.f;  // grads[grads.isnan()] = 0.0
    const float e0 = expf(s[0]), e1 = expf(s[1]), e2 = expf(s[2]);
    const float ms = fmaxf(fmaxf(e0, e1), e2);
    const bool sel = g >= a.grad_threshold;
    const bool clone = sel && ms <= a.clone_extent;
    const bool split = sel && ms > a.clone_extent;
    const bool low_op = sigmoidf_ref(opacity) < a.min_opacity;
    const bool prune_parent = low_op || (a.use_screen_size && ms > a.big_extent);
    bool prune_child = low_op;
    if (a.use_screen_size) {  // the child's scale as the reference re-reads it: exp(log(exp(s) / div))
        const float c0 = expf(logf(e0 / a.split_div)), c1 = expf(logf(e1 / a.split_div)),
                    c2 = expf(logf(e2 / a.split_div));
        prune_child = prune_child || fmaxf(fmaxf(c0, c1), c2) > a.big_extent;
    }
    uint8_t f = 0;
    if (!split && !prune_parent) f |= kKeepA;
    if (clone && !prune_parent) f |= kKeepB;
    if (split && !prune_child) f |= kKeepC;
    if (split) f |= kSplit;
    return f;
}

// Block-wide counts (and exclusive ranks) of the four flag bits: wave ballots, then a scan
// over the block's four waves in LDS.
struct BlockRanks {
    uint32_t rank[4];   // this thread's exclusive rank among the block's set bits
    uint32_t total[4];  // the block's counts
};

__device__ __forceinline__ BlockRanks block_ranks(uint8_t f) {
    __shared__ uint32_t s_cnt[kDenWaves][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    BlockRanks r;
    uint32_t in_wave[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const unsigned long long b = __ballot((f >> k) & 1);
        in_wave[k] = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) s_cnt[w][k] = (uint32_t)__popcll(b);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t before = 0, tot = 0;
        for (int v = 0; v < kDenWaves; v++) {
            const uint32_t c = s_cnt[v][k];
            before += v < w ? c : 0u;
            tot += c;
        }
        r.rank[k] = before + in_wave[k];
        r.total[k] = tot;
    }
    return r;
}

__global__ void __launch_bounds__(kDenThreads) densify_plan_kernel(DensifyArgs a) {
    const int i = blockIdx.x * kDenThreads + threadIdx.x;
    uint8_t f = 0;
    if (i < a.P) {
        f = densify_flags(a.accum[i], a.denom[i], a.opacity[i], a.scaling + 3 * (size_t)i, a);
        a.flags[i] = f;
        if (a.split_mask) a.split_mask[i] = (f & kSplit) ? 1 : 0;
    }
    const BlockRanks r = block_ranks(f);
    if (threadIdx.x < 4) a.blk[(size_t)blockIdx.x * 4 + threadIdx.x] = r.total[threadIdx.x];
}

// One workgroup: exclusive scan of the per-block counts (in place), then the section totals.
__global__ void __launch_bounds__(1024) densify_scan_kernel(uint32_t nblk, uint32_t* __restrict__ blk,
                                                            uint32_t* __restrict__ totals) {
    __shared__ uint32_t s_w[16][4];
    __shared__ uint32_t s_carry[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 4) s_carry[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nblk; base += 1024) {
        const uint32_t b = base + threadIdx.x;
        uint32_t v[4], incl[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = b < nblk ? blk[(size_t)b * 4 + k] : 0u;
            incl[k] = v[k];
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t u = __shfl_up(incl[k], off);
                if (lane >= off) incl[k] += u;
            }
            if (lane == 63) s_w[w][k] = incl[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t before = s_carry[k];
            for (int x = 0; x < w; x++) before += s_w[x][k];
            if (b < nblk) blk[(size_t)b * 4 + k] = before + incl[k] - v[k];
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            uint32_t t = 0;
            for (int x = 0; x < 16; x++) t += s_w[x][threadIdx.x];
            s_carry[threadIdx.x] += t;
        }
        __syncthreads();
    }
    if (threadIdx.x < 4) totals[threadIdx.x] = s_carry[threadIdx.x];
}

__global__ void __launch_bounds__(kDenThreads) densify_index_kernel(DensifyArgs a) {
    const int i = blockIdx.x * kDenThreads + threadIdx.x;
    const uint8_t f = i < a.P ? a.flags[i] : (uint8_t)0;
    const BlockRanks r = block_ranks(f);
    if (i >= a.P) return;
    const uint32_t* off = a.blk + (size_t)blockIdx.x * 4;
    const uint32_t nA = a.totals[0], nB = a.totals[1];
    int4 o;
    o.x = (f & kKeepA) ? (int)(off[0] + r.rank[0]) : -1;
    o.y = (f & kKeepB) ? (int)(nA + off[1] + r.rank[1]) : -1;
    o.z = (f & kKeepC) ? (int)(nA + nB + off[2] + r.rank[2]) : -1;  // first split copy; copy k adds k * nC
    o.w = (f & kSplit) ? (int)(off[3] + r.rank[3]) : -1;           // row of this parent's samples
    a.rows[i] = o;
}

// ---- apply --------------------------------------------------------------------------
// Row c of R(q) (utils/general_utils.py:78-99: q normalised, then the reference's element
// formulas) applied to the sample, plus the parent's coordinate: bmm(R, sample) + xyz
// (gaussian_model.py:530).
__device__ __forceinline__ float child_xyz(const float* q4, const float* smp, float xyz, int c) {
#pragma clang fp contract(off)
    const float nrm = sqrtf(q4[0] * q4[0] + q4[1] * q4[1] + q4[2] * q4[2] + q4[3] * q4[3]);
    const float r = q4[0] / nrm, x = q4[1] / nrm, y = q4[2] / nrm, z = q4[3] / nrm;
    float R0, R1, R2;
    if (c == 0) {
        R0 = 1.f - 2.f * (y * y + z * z); R1 = 2.f * (x * y - r * z); R2 = 2.f * (x * z + r * y);
    } else if (c == 1) {
        R0 = 2.f * (x * y + r * z); R1 = 1.f - 2.f * (x * x + z * z); R2 = 2.f * (y * z - r * x);
    } else {
        R0 = 2.f * (x * z - r * y); R1 = 2.f * (y * z + r * x); R2 = 1.f - 2.f * (x * x + y * y);
    }
    const float d = fmaf(R2, smp[2], fmaf(R1, smp[1], R0 * smp[0]));
    return d + xyz;
}

__global__ void __launch_bounds__(kDenThreads) densify_apply_kernel(DensifyApplyArgs a) {
    const uint32_t t = blockIdx.x * kDenThreads + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t i = (uint32_t)(((unsigned long long)t * a.magic) >> a.shift);  // t / width
    const uint32_t c = t - i * a.width;
    const int4 o = a.rows[i];
    const uint32_t v = a.src[t];  // bit copies: int tmp_radii move through here too
    if (o.x >= 0) {
        a.dst[(size_t)o.x * a.width + c] = v;
        if (a.dst_m) {
            a.dst_m[(size_t)o.x * a.width + c] = a.src_m[t];
            a.dst_v[(size_t)o.x * a.width + c] = a.src_v[t];
        }
    }
    if (o.y >= 0) {
        a.dst[(size_t)o.y * a.width + c] = v;
        if (a.dst_m) {
            a.dst_m[(size_t)o.y * a.width + c] = 0u;
            a.dst_v[(size_t)o.y * a.width + c] = 0u;
        }
    }
    if (o.z >= 0) {
        for (int k = 0; k < a.split_n; k++) {
            const size_t row = (size_t)o.z + (size_t)k * a.n_children;
            uint32_t out = v;
            if (a.role == GSR_DENSIFY_XYZ) {
                const float* smp = a.samples + 3 * ((size_t)k * a.n_split + (size_t)o.w);
                out = __float_as_uint(child_xyz(a.rotation + 4 * (size_t)i, smp, __uint_as_float(v), (int)c));
            } else if (a.role == GSR_DENSIFY_SCALING) {
#pragma clang fp contract(off)
                out = __float_as_uint(logf(expf(__uint_as_float(v)) / a.split_div));
            }
            a.dst[row * a.width + c] = out;
            if (a.dst_m) {
                a.dst_m[row * a.width + c] = 0u;
                a.dst_v[row * a.width + c] = 0u;
            }
        }
    }
}

// ---- launchers ----------------------------------------------------------------------
size_t densify_scratch_bytes(int P) {
    const size_t nblk = ((size_t)P + kDenThreads - 1) / kDenThreads;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return al((size_t)P * sizeof(int4)) + al((size_t)P) + al(nblk * 4 * sizeof(uint32_t)) + al(4 * sizeof(uint32_t));
}

void densify_carve(void* scratch, int P, DensifyArgs& a) {
    const size_t nblk = ((size_t)P + kDenThreads - 1) / kDenThreads;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char* p = (char*)scratch;
    a.rows = (int4*)p;
    p += al((size_t)P * sizeof(int4));
    a.flags = (uint8_t*)p;
    p += al((size_t)P);
    a.blk = (uint32_t*)p;
    p += al(nblk * 4 * sizeof(uint32_t));
    a.totals = (uint32_t*)p;
}

hipError_t launch_densify_stats(int P, const float* vgrad, const int* radii, const uint8_t* visible, float* accum,
                                float* denom, float* max_r, hipStream_t stream) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(densify_stats_kernel, dim3((P + kDenThreads - 1) / kDenThreads), dim3(kDenThreads), 0, stream,
                       P, vgrad, radii, visible, accum, denom, max_r);
    return hipGetLastError();
}

hipError_t launch_densify_plan(const DensifyArgs& a, hipStream_t stream) {
    if (a.P <= 0) return hipSuccess;
    const uint32_t nblk = (uint32_t)((a.P + kDenThreads - 1) / kDenThreads);
    hipLaunchKernelGGL(densify_plan_kernel, dim3(nblk), dim3(kDenThreads), 0, stream, a);
    hipLaunchKernelGGL(densify_scan_kernel, dim3(1), dim3(1024), 0, stream, nblk, a.blk, a.totals);
    hipLaunchKernelGGL(densify_index_kernel, dim3(nblk), dim3(kDenThreads), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_densify_apply(const DensifyApplyArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(densify_apply_kernel, dim3((a.n + kDenThreads - 1) / kDenThreads), dim3(kDenThreads), 0,
                       stream, a);
    return hipGetLastError();
}

}  // namespace gsr
