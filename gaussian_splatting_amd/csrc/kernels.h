// kernels.h -- launch arguments and entry points shared by the .hip translation units.
#pragma once

#include "gsr_common.h"
#include "../../include/gsr_densify.h"

namespace gsr {

struct PreprocessArgs {
    int P, D, M, W, H;
    const float* means3D;
    const float* scales;
    float scale_modifier;
    const float* rotations;
    const float* opacities;
    const float* shs;  // combined [P,M,3], or the rest [P,M-1,3] when dc is set (ShAddr)
    const float* dc;   // [P,1,3] or null
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    uint32_t gx, gy;
    int prefiltered, antialiasing, footprint_cull;
    int* radii;
    GeomState geom;
    uint32_t* zero;   // counters the binning accumulates into, zeroed here (no memset launch)
    uint32_t zero_n;
};

// Zero-fill of up to kFillSegs float ranges (the backward's dense outputs), zeroed beside render_bwd
// (VALU-bound, it leaves HBM bandwidth idle): "zero_fill" option, api.hip; and the atomic backward's
// accumulators, zeroed beside render_fwd.
constexpr int kFillSegs = 12;
struct FillArgs {
    float* ptr[kFillSegs];
    unsigned long long n[kFillSegs];  // floats
    int count;
};

struct RenderFwdArgs {
    int W, H;
    uint32_t gx, gy;
    const uint2* ranges;
    uint32_t* gid_sorted;  // the forward writes each staged entry's quadrant mask into its low bits
    const float4* rec;
    const float* bg;
    float* out_color;
    float* out_invdepth;
    float* ckpt;           // blend checkpoints (BinningState::ckpt)
    ImageState img;
    // the backward's work list, appended per tile (GeomState::unit_cnt / unit_part, BinningState::unit_full)
    uint32_t* unit_cnt;
    uint2* unit_part;
    uint2* unit_full;
    uint32_t full_cap;     // unit_full_cap(binning capacity): stride of unit_full's shards
    unsigned long long* tile_join;  // GeomState::tile_join
    int seg_ck;
    uint32_t* seg_ck_out;           // GeomState::fwd_seg_ck: seg_ck recorded for the backward
    uint32_t* fault;                // GeomState::status + 1: bit 0 = a shared-staging wait gave up (never expected)
    uint32_t half_tiles;            // hybrid grid (render.hip kFwdTailQuadsPct): tiles done as half-tile units
    unsigned long long* census;     // diagnostic pair counts (gsr_census_set) or null
    // reachable-prefix sort (GeomState): entries in order per tile, and the redo filing
    const uint32_t* sorted_len;
    uint32_t* redo_flag;
    uint32_t* redo_list;
    uint32_t* redo_cnt;
    // the first fill_blocks blocks of the launch zero the atomic backward's accumulators beside the VALU-bound
    // render waves, which leave HBM mostly idle: every touched word, and the row of every Gaussian that can
    // reach a list the render walks -- visible and (near-first binning) in front of the cut; the rows of far
    // Gaussians in redone tiles are zeroed by the far fill
    uint32_t fill_blocks;
    float4* acc;
    uint32_t* touched;
    const uint32_t* depth_key;
    const uint32_t* zcut;
    uint32_t n_gauss;
};

struct RenderBwdArgs {
    int W, H;
    uint32_t gx, gy;
    const uint2* ranges;
    const uint32_t* gid_sorted;
    const float4* rec;
    const float* bg;
    const float* dL_dpix;       // [3,H,W]
    const float* dL_dinvdepth;  // [H,W] or null
    ImageState img;
    GradRecs recs;
    const float* ckpt;                  // blend checkpoints written by the forward
    // work list: (tile, first checkpoint index) of each wave, written by the forward render
    const uint32_t* unit_cnt;
    const uint2* unit_part;
    const uint2* unit_full;
    uint32_t full_cap;
    const uint32_t* rec_start;          // GeomState::rec_start (record path: each Gaussian's first emission index)
    const uint32_t* seg_ck;             // GeomState::fwd_seg_ck: checkpoints per backward segment as the
                                        // forward that built the work list used it (segment = seg_ck * kCkStride)
    unsigned long long* census;         // diagnostic pair counts (gsr_census_set) or null
    uint32_t* live_count;               // the live list's shard counters, zeroed here, or null
    // "zero_fill" = 3: the first fill_blocks blocks of the launch zero the backward's dense outputs
    // (one wave each, beside the render waves) instead of a side-stream kernel forked and joined by
    // events -- each event left the GPU idle for 6-7 us (r4a trace)
    uint32_t fill_blocks;
    FillArgs fill;
    // atomic backward ("bwd_atomic"): the per-Gaussian accumulator rows and touched bits (GeomState),
    // or null for the per-instance gradient records + gauss_reduce
    float* acc;
    uint32_t* touched;
};

struct GaussBwdArgs {
    int P, D, M, W, H;
    const float* means3D;
    const float* shs;  // as PreprocessArgs::shs
    const float* dc;   // [P,1,3] or null
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    float scale_modifier;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    int antialiasing;
    const int* radii;
    GeomState geom;
    GradRecs sums;  // per Gaussian: summed render gradients (gauss_reduce_kernel; the record path)
    int have_invdepth;
    float* dL_dmean2D;    // [P,3]
    float* dL_dconic;     // [P,4] or null
    float* dL_dopacity;   // [P]
    float* dL_dcolor;     // [P,3]
    float* dL_dinvdepth;  // [P] or null
    float* dL_dmean3D;    // [P,3]
    float* dL_dcov3D;     // [P,6]
    float* dL_dsh;        // [P,M,3] or null (M == 0); the rest [P,M-1,3] when dL_ddc is set
    float* dL_ddc;        // [P,1,3] when the forward took dc, else null
    float* dL_dscale;     // [P,3] or null
    float* dL_drot;       // [P,4] or null
    int sparse;           // outputs already zero (zero_fill on the side stream): write only non-zero rows
    const uint32_t* live;        // sparse: the Gaussians with a gradient (gauss_reduce), or null
    const uint32_t* live_count;  // per shard: its length (device), kLiveCntStride apart
    uint32_t live_cap;           // entries per shard (live_list_cap)
    uint32_t* touched;           // atomic backward (sparse): the touched bits render_bwd set, or null; cleared here
    float4* acc;                 // with touched: the accumulator rows (the sums), zeroed after reading
    uint32_t touched_shift;      // with touched: a workgroup lists 128 << touched_shift Gaussians ("touched_run")
};

hipError_t launch_zero_fill(const FillArgs& f, hipStream_t stream);

// The fill's body, shared by zero_fill_kernel and the fill blocks fused into render_bwd's launch
// ("zero_fill" = 3): thread `tid` of `stride` zeroes its share of every range -- 16-byte stores over
// each range's aligned body (non-temporal: 236 MB of zeros written through the caches evicted the
// records and pixel state render_bwd and gauss_reduce re-read, r2zv), dwords for the unaligned head
// and tail.
__device__ __forceinline__ void zero_fill_part(const FillArgs& f, unsigned long long tid, unsigned long long stride) {
    for (int s = 0; s < f.count; s++) {
        float* p = f.ptr[s];
        const unsigned long long n = f.n[s];
        const unsigned long long head = ((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) / 4;
        const unsigned long long h = head < n ? head : n;
        const unsigned long long n4 = (n - h) / 4;
        float4* body = reinterpret_cast<float4*>(p + h);
        for (unsigned long long i = tid; i < n4; i += stride) {
            typedef float v4f __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store((v4f){0.f, 0.f, 0.f, 0.f}, reinterpret_cast<v4f*>(body + i));
        }
        if (tid < h) p[tid] = 0.f;
        const unsigned long long t0 = h + 4 * n4;
        if (tid < n - t0) p[t0 + tid] = 0.f;
    }
}

// ---- SH rows through LDS (preprocess and gauss_bwd, M = 16) -----------------------
// LDS row r holds the 48 floats [coefficient 0..15][3] of Gaussian r0 + r at
// lds[r * stride].  Combined layout: the block is one contiguous range of 48-float rows,
// moved with 16-byte loads and 16-byte LDS stores.  Split layout (dc given): the rest
// block is one contiguous range of 45-float rows, moved 16 bytes at a time and scattered
// to LDS as scalars behind each row's 3 dc floats (the dc block is 3 floats a row).
// Requires 16-byte aligned shs / dsh and r0 a multiple of 16.
constexpr int kShRowF = 48;     // floats per staged SH row (M = 16)
constexpr int kShRestF = 45;    // floats per rest row in the split layout

// SH rows are read once per pass (preprocess: 192 MB at 1M): non-temporal loads keep them from
// displacing the lines the next kernels re-read (r2zx: preprocess 69.5 -> 62.7 us, bin_count
// 45.6 -> 43.3, step -8 us).  Streaming stores of render_fwd's image outputs and streaming loads
// of render_bwd's dL/dpixel measured no gain.
template <int ROWS, int THREADS, bool SPLIT>
// rowmask: bit r set = stage row r (rows left out are not read; their LDS contents are undefined).
__device__ __forceinline__ void sh_stage_in(const ShAddr& sa, int r0, int rows, float* lds, int stride, int tid,
                                            unsigned long long rowmask = ~0ull) {
    if constexpr (!SPLIT) {
        const float4* src = reinterpret_cast<const float4*>(sa.shs + (size_t)r0 * kShRowF);
        const int n4 = rows * (kShRowF / 4);
#pragma unroll
        for (int k = 0; k < ROWS * kShRowF / 4 / THREADS; k++) {
            const int i4 = k * THREADS + tid;
            const int d = i4 * 4, row = d / kShRowF, col = d - row * kShRowF;
            if (i4 < n4 && ((rowmask >> row) & 1ull)) {
                typedef float v4f __attribute__((ext_vector_type(4)));
                *reinterpret_cast<v4f*>(&lds[row * stride + col]) =
                    __builtin_nontemporal_load(reinterpret_cast<const v4f*>(src) + i4);
            }
        }
        return;
    } else {
    const float* rest = sa.shs + (size_t)r0 * kShRestF;
    const int nf = rows * kShRestF, n4 = nf >> 2;
#pragma unroll
    for (int k = 0; k < (ROWS * kShRestF / 4 + THREADS - 1) / THREADS; k++) {
        const int i4 = k * THREADS + tid;
        // a 16-byte piece may straddle two rows (45-float rows): read it when either is wanted
        const int ra = (i4 * 4) / kShRestF, rb = (i4 * 4 + 3) / kShRestF;
        if (i4 < n4 && (((rowmask >> ra) | (rowmask >> rb)) & 1ull)) {
            const float4 v = reinterpret_cast<const float4*>(rest)[i4];
            const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int d = i4 * 4 + c, row = d / kShRestF;
                lds[row * stride + 3 + d - row * kShRestF] = f[c];
            }
        }
    }
    if (tid < (nf & 3)) {
        const int d = n4 * 4 + tid, row = d / kShRestF;
        lds[row * stride + 3 + d - row * kShRestF] = rest[d];
    }
    const float* dc = sa.dc + (size_t)r0 * 3;
    for (int i = tid; i < rows * 3; i += THREADS)
        if ((rowmask >> (i / 3)) & 1ull) lds[(i / 3) * stride + i % 3] = dc[i];
    }
}

// SH rows are read once per pass (preprocess: 192 MB at 1M): non-temporal loads keep them from
// displacing the lines the next kernels re-read (r2zx: preprocess 69.5 -> 62.7 us, bin_count
// 45.6 -> 43.3, step -8 us).  Streaming stores of render_fwd's image outputs and streaming loads
// of render_bwd's dL/dpixel measured no gain.
template <int ROWS, int THREADS, bool SPLIT>
// rowmask: bit r set = write row r (rows left out are not written).
__device__ __forceinline__ void sh_stage_out(const ShGradAddr& ga, int r0, int rows, const float* lds, int stride,
                                             int tid, unsigned long long rowmask = ~0ull) {
    if constexpr (!SPLIT) {
        float4* dst = reinterpret_cast<float4*>(ga.dsh + (size_t)r0 * kShRowF);
        const int n4 = rows * (kShRowF / 4);
#pragma unroll
        for (int k = 0; k < ROWS * kShRowF / 4 / THREADS; k++) {
            const int i4 = k * THREADS + tid;
            const int d = i4 * 4, row = d / kShRowF, col = d - row * kShRowF;
            if (i4 < n4 && ((rowmask >> row) & 1ull))
                dst[i4] = *reinterpret_cast<const float4*>(&lds[row * stride + col]);
        }
        return;
    } else {
    float* rest = ga.dsh + (size_t)r0 * kShRestF;
    const int nf = rows * kShRestF, n4 = nf >> 2;
#pragma unroll
    for (int k = 0; k < (ROWS * kShRestF / 4 + THREADS - 1) / THREADS; k++) {
        const int i4 = k * THREADS + tid;
        // a piece straddling two rows is written when either is wanted: the caller keeps the LDS
        // rows it does not want zero, which is what they hold in the output already
        const int ra = (i4 * 4) / kShRestF, rb = (i4 * 4 + 3) / kShRestF;
        if (i4 < n4 && (((rowmask >> ra) | (rowmask >> rb)) & 1ull)) {
            float f[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int d = i4 * 4 + c, row = d / kShRestF;
                f[c] = lds[row * stride + 3 + d - row * kShRestF];
            }
            reinterpret_cast<float4*>(rest)[i4] = make_float4(f[0], f[1], f[2], f[3]);
        }
    }
    if (tid < (nf & 3)) {
        const int d = n4 * 4 + tid, row = d / kShRestF;
        if ((rowmask >> row) & 1ull) rest[d] = lds[row * stride + 3 + d - row * kShRestF];
    }
    float* dc = ga.ddc + (size_t)r0 * 3;
    for (int i = tid; i < rows * 3; i += THREADS)
        if ((rowmask >> (i / 3)) & 1ull) dc[i] = lds[(i / 3) * stride + i % 3];
    }
}

// Gathered forms of sh_stage_in / sh_stage_out: row r of the staged block belongs to the Gaussian
// held by lane row0 + r of the wave in `g` (negative: row not read / not written), in any order --
// the live-list backward's rows.  Combined layout: 16-byte pieces (12 per row, rows are 16-byte
// aligned); split layout: dwords (45-float rest rows are only 4-byte aligned) plus the dc triple.
// All lanes must call them (the row owners' indices travel by shuffle).
// Split layout: a row's floats are copied by the lanes that own the row (immediate offsets from one
// address).  (Striped over the wave -- one dword of the block per lane and iteration -- the
// fully unrolled loop kept ~23 iterations' addresses live across the kernel: 308 VGPRs, one wave
// per SIMD; one iteration at a time serialised the loads.)
template <int ROWS, int THREADS, bool SPLIT>
__device__ __forceinline__ void sh_gather_in(const ShAddr& sa, int g, int row0, float* lds, int stride, int tid) {
    if constexpr (!SPLIT) {
        // every piece loaded before any is stored (a row not wanted loads row 0's piece, which the
        // caller's tensor always has): one memory latency for the block, where a load inside the
        // per-lane branch made each piece wait for its own (six dependent round trips per 32 rows)
        typedef float v4f __attribute__((ext_vector_type(4)));
        constexpr int K = ROWS * (kShRowF / 4) / THREADS;
        static_assert(K <= 12, "pieces per lane held in registers");
        v4f v[K];
        int gk[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int i4 = k * THREADS + tid, row = i4 / (kShRowF / 4), c4 = i4 - row * (kShRowF / 4);
            gk[k] = __shfl(g, row0 + row);
            v[k] = reinterpret_cast<const v4f*>(sa.shs + (size_t)max(gk[k], 0) * kShRowF)[c4];
        }
        __builtin_amdgcn_sched_barrier(0);  // (left alone, the scheduler sinks each load to its store)
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int i4 = k * THREADS + tid, row = i4 / (kShRowF / 4), c4 = i4 - row * (kShRowF / 4);
            if (gk[k] >= 0) *reinterpret_cast<v4f*>(&lds[row * stride + 4 * c4]) = v[k];
        }
    } else {
        // THREADS / ROWS lanes per row, each copying its share of the row's 45 rest floats (one base
        // address, immediate offsets, every load independent) and the last of them the dc triple
        static_assert(THREADS % ROWS == 0, "whole lanes per row");
        constexpr int L = THREADS / ROWS, PER = (kShRestF + L - 1) / L;
        const int row = tid / L, part = tid % L;
        const int gr = __shfl(g, row0 + row);
        if (gr >= 0) {
            const float* src = sa.shs + (size_t)gr * kShRestF + part * PER;
            float* dst = lds + row * stride + 3 + part * PER;
            const int n = kShRestF - part * PER;  // >= PER except for the last part
            float v[PER];
#pragma unroll
            for (int c = 0; c < PER; c++) v[c] = c < n ? src[c] : 0.f;
#pragma unroll
            for (int c = 0; c < PER; c++)
                if (c < n) dst[c] = v[c];
            if (part == L - 1) {
                const float* d3 = sa.dc + (size_t)gr * 3;
                const float x = d3[0], y = d3[1], z = d3[2];
                lds[row * stride] = x;
                lds[row * stride + 1] = y;
                lds[row * stride + 2] = z;
            }
        }
    }
}

template <int ROWS, int THREADS, bool SPLIT>
__device__ __forceinline__ void sh_gather_out(const ShGradAddr& ga, int g, int row0, const float* lds, int stride,
                                              int tid) {
    if constexpr (!SPLIT) {
#pragma unroll 12
        for (int k = 0; k < ROWS * (kShRowF / 4) / THREADS; k++) {
            const int i4 = k * THREADS + tid, row = i4 / (kShRowF / 4), c4 = i4 - row * (kShRowF / 4);
            const int gr = __shfl(g, row0 + row);
            if (gr >= 0)
                reinterpret_cast<float4*>(ga.dsh + (size_t)gr * kShRowF)[c4] =
                    *reinterpret_cast<const float4*>(&lds[row * stride + 4 * c4]);
        }
    } else {
        static_assert(THREADS % ROWS == 0, "whole lanes per row");
        constexpr int L = THREADS / ROWS, PER = (kShRestF + L - 1) / L;
        const int row = tid / L, part = tid % L;
        const int gr = __shfl(g, row0 + row);
        if (gr >= 0) {
            const float* src = lds + row * stride + 3 + part * PER;
            float* dst = ga.dsh + (size_t)gr * kShRestF + part * PER;
            const int n = kShRestF - part * PER;
#pragma unroll
            for (int c = 0; c < PER; c++)
                if (c < n) dst[c] = src[c];
            if (part == L - 1) {
                float* d3 = ga.ddc + (size_t)gr * 3;
                d3[0] = lds[row * stride];
                d3[1] = lds[row * stride + 1];
                d3[2] = lds[row * stride + 2];
            }
        }
    }
}
// SH path of preprocess / gauss_bwd: per-lane global loads, or LDS staging of either layout
enum ShMode { kShGlobal = 0, kShLdsCombined = 1, kShLdsSplit = 2 };

// ---- sparse Adam (adam.hip) --------------------------------------------------------
constexpr int kAdamMaxGroups = 8;  // GSR_ADAM_MAX_GROUPS
struct AdamGroupDev {
    float* p;
    const float* g;
    float* m;
    float* v;
    uint32_t n;                // N * M
    uint32_t M;
    unsigned long long magic;  // i / M == (i * magic) >> shift for i < 2^31
    uint32_t shift;
    float lr, eps;
    uint32_t first_block;      // first workgroup of this group
    int vec;                   // all four arrays 16-byte aligned
};
struct AdamArgs {
    AdamGroupDev grp[kAdamMaxGroups];
    int n_groups;
    const uint8_t* vis;
    float b1, b2;
};
constexpr int kAdamThreads = 256;
constexpr int kAdamUnroll = 2;  // float4s per thread
constexpr uint32_t kAdamBlockElems = kAdamThreads * kAdamUnroll * 4;
hipError_t launch_adam(const AdamArgs& a, uint32_t blocks, hipStream_t stream);

// ---- adaptive density control (densify.hip) ------------------------------------------
struct DensifyArgs {
    int P;
    const float* accum;
    const float* denom;
    const float* opacity;
    const float* scaling;
    float grad_threshold, clone_extent, min_opacity, big_extent, split_div;
    int use_screen_size;
    uint8_t* split_mask;  // may be null
    // scratch (densify_carve)
    int4* rows;           // [P] kept row, clone row, first child row, split rank (-1: none)
    uint8_t* flags;       // [P]
    uint32_t* blk;        // [blocks][4] counts, then exclusive offsets
    uint32_t* totals;     // [4] kept, clones, children per copy, splits
};
struct DensifyApplyArgs {
    const uint32_t* src;
    uint32_t* dst;
    const uint32_t* src_m;
    const uint32_t* src_v;
    uint32_t* dst_m;  // null: the group has no Adam state
    uint32_t* dst_v;
    uint32_t n;       // P * width
    uint32_t width;
    unsigned long long magic;  // t / width == (t * magic) >> shift for t < 2^31
    uint32_t shift;
    int role;
    const int4* rows;
    const float* rotation;
    const float* samples;
    uint32_t n_split, n_children;
    int split_n;
    float split_div;
};
size_t densify_scratch_bytes(int P);
void densify_carve(void* scratch, int P, DensifyArgs& a);
hipError_t launch_densify_stats(int P, const float* vgrad, const int* radii, const uint8_t* visible, float* accum,
                                float* denom, float* max_r, hipStream_t stream);
hipError_t launch_densify_plan(const DensifyArgs& a, hipStream_t stream);
hipError_t launch_densify_apply(const DensifyApplyArgs& a, hipStream_t stream);

// preprocess.hip
hipError_t launch_preprocess(const PreprocessArgs& a, hipStream_t stream);
hipError_t launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t stream);
// binning.hip
size_t bin_chunk_count(int P);
size_t bin_cell_count(uint32_t gx, uint32_t gy);
// u32 words of the counters preprocess zeroes (GeomState::tile_cnt on): tile, cell and near counts, the
// depth-mass histogram
inline size_t bin_zero_words(size_t tiles, size_t cells) { return ((2 * tiles + cells + 1) & ~(size_t)1) + 2 * kZBins; }
// host_total: mapped coherent host memory K2 (or the fused K3) also writes the instance count to, or
// null.  fused (capacity mode, LDS cursors): K2 is folded into K3 -- launch_bin_count runs K0 + K1
// only, launch_bin_scatter scans the counts and publishes ranges / classes / the count, and
// launch_tile_sort re-zeroes the tile and cell counters.
// near_target > 0 (fused only): near-first binning (binning.hip) with that depth-cut target (fixed-point
// mass over the image: kMassScale x W x H x mean mass); launch_bin_scatter's near_first must agree.
hipError_t launch_bin_count(int P, const GeomState& g, uint32_t gx, uint32_t gy, uint2* ranges, size_t cap,
                            unsigned long long* host_total, hipStream_t stream, bool fused = false,
                            unsigned long long near_target = 0);
hipError_t launch_bin_scatter(int P, const GeomState& g, uint32_t gx, uint32_t gy, const BinningState& b, size_t cap,
                              hipStream_t stream, uint2* ranges = nullptr, unsigned long long* host_total = nullptr,
                              bool fused = false, bool near_first = false, bool recs = true);
// The record path's inputs (record starts, zeroed content bits) after a forward whose K3 skipped them
hipError_t launch_rec_prep(int P, const GeomState& g, const BinningState& b, size_t cap, hipStream_t stream);
// the far instances of the tiles the forward filed for a redo (redo), behind their near entries
// acc (atomic backward, redo only): the accumulator rows of the far Gaussians filled in are zeroed too
hipError_t launch_far_fill(int P, const GeomState& g, uint32_t gx, uint32_t tiles, const uint2* ranges,
                           const BinningState& b, size_t cap, bool redo, hipStream_t stream, float4* acc = nullptr);
bool bin_near_ok(uint32_t tiles);  // near-first binning applies (fused scan, K1 by rectangles)
// prefix: sort only the first `prefix` (+ the rest of an LDS bin) entries of the lists longer than
// one wave's sort (0: whole lists); GeomState::sorted_len records each list's sorted length.
hipError_t launch_tile_sort(uint32_t tiles, const uint2* ranges, const GeomState& g, const BinningState& b,
                            size_t cap, hipStream_t stream, bool zero_counts = false, uint32_t cells = 0,
                            uint32_t prefix = 0);
// The forward's redo of tiles whose walk passed their sorted prefix: whole-list sort of the filed
// tiles (before launch_render_fwd_redo).
hipError_t launch_tile_sort_redo(uint32_t tiles, const uint2* ranges, const GeomState& g, const BinningState& b,
                                 size_t cap, hipStream_t stream);
// Inspection: every tile's whole sorted list into `out` (the product's sorted entries, the rest
// sorted here), without writing the forward's buffers.
hipError_t launch_sorted_lists_copy(uint32_t tiles, const uint2* ranges, const GeomState& g, const BinningState& b,
                                    size_t cap, uint32_t* out, hipStream_t stream, int P = 0, uint32_t gx = 0,
                                    bool near_first = false);
bool bin_fused_ok(uint32_t tiles);  // the fused form applies (LDS cursors)
// render.hip
// quads: 8x8 quadrants per wave, 2 (half tiles) or 4 (whole tiles; the "fwd_quads" option)
hipError_t launch_render_fwd(const RenderFwdArgs& a, hipStream_t stream, int quads = 2);
// the tiles filed for a redo (GeomState::redo_list), after launch_tile_sort_redo; exits at once if none
hipError_t launch_render_fwd_redo(const RenderFwdArgs& a, hipStream_t stream, int quads = 2);
// a tile-major pixel plane (tile_px) -> image order [H][W], 4-byte elements (inspection only)
hipError_t launch_untile(const uint32_t* src, uint32_t* dst, int W, int H, uint32_t gx, hipStream_t stream);
// grid_mode ("bwd_grid" option): 0 = strided when the worst-case grid is far larger than the tiles,
// 1 = one block per possible unit, 2 = strided
hipError_t launch_render_bwd(const RenderBwdArgs& a, size_t max_units, hipStream_t stream, int grid_mode = 0);
// backward work list: one unit per (tile, segment of seg_ck * kCkStride entries below the tile's limit),
// written by the forward render; at most R / (seg_ck kCkStride) + tiles of them
size_t bwd_max_units(size_t R, uint32_t tiles, int seg_ck);
// Longest reachable prefix K4 sorts ("sort_prefix" option range; binning.hip kPrefixBuf holds twice it).
constexpr uint32_t kSortPrefixMax = 1024;
// knn.hip
size_t knn_scratch_bytes(int P);
hipError_t launch_knn(int P, const float* pts, float* out, void* scratch, hipStream_t stream);
// ssim.hip
hipError_t launch_ssim_fwd(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* map, float* dm_dmu1, float* dm_ds11, float* dm_ds12, hipStream_t stream);
hipError_t launch_ssim_bwd(int planes, int H, int W, const float* img1, const float* img2, const float* dL_dmap,
                           const float* dm_dmu1, const float* dm_ds11, const float* dm_ds12, float* dL_dimg1,
                           hipStream_t stream);
// backward.hip
hipError_t launch_gauss_reduce(int P, const GeomState& g, const GradRecs& recs, const GradRecs& sums,
                               uint32_t* flags, const int* radii, uint32_t* live, uint32_t* live_count,
                               hipStream_t stream);
// atomic screen-space backward: the view block's dense sums (a touched Gaussian's row, zeroed after; zeros
// otherwise) and flag words (visible, SH clamp bits) from the touched bits (re-zeroed) -- gauss_reduce's view
// block output without records
hipError_t launch_gauss_live_views(int P, uint32_t* touched, float4* acc, const int* radii, const uint8_t* clamped,
                                   const GradRecs& sums, uint32_t* flags, hipStream_t stream);
// multi-view backward over gathered view blocks (backward.hip section 4)
struct ViewsBwdArgs {
    int P, D, M;
    const float* means3D;
    const float* shs;
    const float* dc;
    const float* opacities;
    const float* scales;
    const float* rotations;
    float scale_modifier;
    int n_views;
    const float* blocks;  // [n_views][block_floats]: view blocks, or packed blocks when `flags` is set
    size_t block_floats;
    // Packed mode (gsr_view_block_index): the flag word of Gaussian g in view v is flags[v * P + g],
    // its entry index in view v's packed block << 4 | the block's flag bits; the sums are read from
    // that packed entry, the camera from the packed block's header.  Null: dense view blocks.
    const uint32_t* flags;
    // with flags: the live list of Gaussians some view flags (launch_views_live), or null; with it
    // the kernel runs a lane per listed Gaussian and the outputs must be zero beforehand
    const uint32_t* live;
    const uint32_t* live_count;
    uint32_t live_cap;
    float* dL_dmean3D;
    float* dL_dsh;
    float* dL_ddc;
    float* dL_dopacity;
    float* dL_dscale;
    float* dL_drot;
};
hipError_t launch_gauss_bwd_views(const ViewsBwdArgs& a, hipStream_t stream);
// (g0, g1): the Gaussian range of one chunk of a chunked exchange; (0, P) for the whole block
hipError_t launch_view_pack(uint32_t P, uint32_t g0, uint32_t g1, const float* block, float* packed,
                            unsigned long long cap, uint32_t* scratch, uint32_t* count, hipStream_t stream);
hipError_t launch_views_live(uint32_t P, uint32_t g0, uint32_t g1, int n_views, const uint32_t* flags, uint32_t* live,
                             uint32_t* live_count, hipStream_t stream);
hipError_t launch_view_index(uint32_t P, uint32_t g0, uint32_t g1, int n_views, const float* packed,
                             unsigned long long packed_floats, uint32_t* flags, unsigned long long cap,
                             hipStream_t stream);
hipError_t launch_view_unpack(uint32_t P, int n_views, const float* packed, unsigned long long packed_floats,
                              float* blocks, unsigned long long cap, hipStream_t stream);
hipError_t launch_view_header(float* blk, const float* view, const float* proj, const float* campos, float tan_fovx,
                              float tan_fovy, float focal_x, float focal_y, int antialiasing, int have_invdepth,
                              hipStream_t stream);
hipError_t launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t stream);

}  // namespace gsr
