// gsr_common.h -- shared definitions for the gfx950 Gaussian tile rasterizer.
//
// Everything here is written for CDNA4 (wave64, 160 KiB LDS per CU).  The
// algorithm it implements is the reference's tile rasterizer
// (submodules/diff-gaussian-rasterization/cuda_rasterizer, "CR" below); the
// data layout and the kernel decomposition are this project's own.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace gsr {

constexpr int kTile = 16;                 // tile edge in pixels (CR/config.h:16-17)
constexpr int kTilePix = kTile * kTile;   // 256 pixels = 256 threads = 4 waves
constexpr int kWave = 64;
constexpr int kChannels = 3;              // CR/config.h:15
constexpr size_t kAlign = 256;            // sub-array alignment inside the scratch buffers

// Spherical-harmonics constants (CR/auxiliary.h:23-40).
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f, SH_C2_2 = 0.31539156525252005f,
                SH_C2_3 = -1.0925484305920792f, SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f, SH_C3_2 = -0.4570457994644658f,
                SH_C3_3 = 0.3731763325901154f, SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                SH_C3_6 = -0.5900435899266435f;

// ---------------------------------------------------------------------------
// Per-Gaussian splat record written by preprocess, gathered by both render
// passes: one 64-byte, 64-byte-aligned block, so a gather touches one cache line.
//   row 0 = (x_pix, y_pix, conic.a, conic.b)
//   row 1 = (conic.c, opacity_eff, 1/depth, bbox_x packed)
//   row 2 = (r, g, b, bbox_y packed)
//   row 3 = (rect_min.x, rect_min.y, rect width, unused) as u32 bits
// bbox_* are the conservative pixel bounds of the alpha >= 1/255 footprint
// (int16 lo | int16 hi << 16), used to skip whole waves (DESIGN.md "footprint
// culling"); lo > hi means "never contributes".  Row 3 is the tile rectangle of
// getRect.  The Gaussian's first emission index e0 is in the record-start array
// (GeomState::rec_start), which only the record-path backward reads: K3 writes it after a
// bwd_atomic=0 forward, rec_prep_kernel on demand otherwise.  The instance of this Gaussian
// in tile (tx, ty) has emission index e0 + (ty - min.y) * width + (tx - min.x), the row-major
// order of duplicateWithKeys (CR/rasterizer_impl.cu:108-124).
// ---------------------------------------------------------------------------
constexpr int kRecRows = 4;

// Tile-list entries (BinningState::gid_sorted) are Gaussian << 4 | quadrant mask: bit k set
// when the splat's alpha >= 1/255 footprint reaches a pixel centre of the tile's 8x8
// quadrant k (footprint.h).  Binning writes the mask bits as 0; the forward render writes
// back, for each entry it stages, the quadrants in which some pixel blended it
// (the blend mask, a subset of the footprint's), and the backward, which only visits
// entries the forward staged, skips entries whose mask is 0.  Hence P < 2^28.
constexpr int kEntryMaskBits = 4;
constexpr uint32_t kEntryMask = 0xfu;
constexpr int kMaxGaussians = 1 << (32 - kEntryMaskBits);

__host__ __device__ inline size_t align_up(size_t x, size_t a = kAlign) { return (x + a - 1) / a * a; }

// LDS hand-off between the lanes of ONE wave (a one-wave workgroup, or the lanes of one wave of a
// larger one): a wave's LDS accesses complete in order, so no s_barrier and no wait for the wave's
// outstanding global stores (which __syncthreads' workgroup fence adds) is needed.  The wavefront-scope
// release / acquire fences emit no instructions; they give the IR the ordering of one lane's LDS store
// before another lane's load, which wave_barrier alone (IntrNoMem: a scheduling barrier only) does not
// (the form rocPRIM's wave_barrier uses).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Bump allocator over a caller-provided chunk (the three opaque uint8 tensors of
// the reference, CR/rasterizer_impl.h:26-90; contents are private to us).
struct Carver {
    char* base;
    size_t off;
    template <typename T>
    T* take(size_t count) {
        off = align_up(off);
        T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
        off += count * sizeof(T);
        return p;
    }
};

// Geometry state: per Gaussian (P).
struct GeomState {
    float4* rec;                // [P][kRecRows] splat records
    uint32_t* depth_key;        // float bits of view-space z, 0xffffffff if culled
    uint32_t* tiles_touched;    // per Gaussian (CR/forward.cu:350)
    uint2* rect;                // getRect, packed: (min.x | min.y << 16, max.x | max.y << 16)
    uint32_t* rec_start;        // first gradient-record index (exclusive scan of tiles_touched)
    uint8_t* clamped;           // SH clamp mask, 3 bits (CR/forward.cu:74-76)
    uint32_t* status;           // device status words: [0] prefiltered violation, [2] fwd_seg_ck
    uint32_t* fwd_seg_ck;       // status + 2: checkpoints per backward segment of the forward's work list
                                // (render_fwd writes it, render_bwd reads it: the two always agree)
    // binning scratch (binning.hip)
    uint32_t* tile_cnt;         // [tiles] instances per tile; cell_cnt follows it (one memset)
    uint32_t* cell_cnt;         // [cells] visible Gaussians per screen cell (spatial order, binning.hip K0)
    uint32_t* cell_off;         // [chunks][cells] each chunk's offset inside each cell's block
    uint4* order;               // [P] visible Gaussians grouped by screen cell: (index, rect, depth key)
    uint32_t* n_visible;        // [1] entries of order
    uint32_t* tile_base;        // [tiles] first instance of each tile (scatter cursors without LDS)
    uint32_t* chunk_off;        // [chunks][tiles] each chunk's offset inside each tile's block
    uint32_t* cls_list;         // [2][tiles] tiles whose lists are too long for one wave's sort, by class
    uint32_t* cls_count;        // [2] entries of each class list
    unsigned long long* chunk_total;  // [chunks] tiles_touched per Gaussian chunk
    unsigned long long* total;        // [1] number of instances (num_rendered)
    // backward work list (render.hip, see kUnitLists): counters [list][shard] one per 128-B line,
    // zeroed by K2 before each forward render; the partial-segment lists, [4][shard][unit_part_cap]
    uint32_t* unit_cnt;
    uint2* unit_part;
    unsigned long long* tile_join;  // [tiles] the forward's half-tile waves combine their limits here (K2 zeroes)
    // Reachable-prefix sort (binning.hip K4, the "sort_prefix" option): entries [0, sorted_len[t]) of
    // tile t's list are in final order, the rest unsorted.  A forward wave that reaches sorted_len
    // with pixels still blending files the tile for a redo (flag + list + count; K4 zeroes them):
    // the tail is sorted and the tile rendered again (render.hip).
    uint32_t* sorted_len;       // [tiles]
    uint32_t* redo_flag;        // [tiles]
    uint32_t* redo_list;        // [tiles]
    uint32_t* redo_cnt;         // [1]
    // Atomic backward ("bwd_atomic" option, gsr_common.h "Per-Gaussian accumulators"): the render
    // backward adds each (tile, Gaussian) instance's ten reduced sums straight into the Gaussian's row
    // and sets its bit in `touched`.  Both are zeroed by the forward (fill blocks in render_fwd's launch)
    // and restored to zero by the backward that consumed them (gauss_bwd_touched_kernel, or
    // gauss_live_views for a view block), so any number of backwards of one forward start from zero.
    float4* acc;                // [P][kAccRow4]: (dcolour, dinvdepth), (dmean2D, dopacity, dconic.b), (dconic.a, .c, 0, 0), pad
    uint32_t* touched;          // [touched_words(P)] bit g: Gaussian g has a gradient term
    // Near-first binning ("near_mass" option, binning.hip "Near-first binning"): only the Gaussians in
    // front of a frame-wide depth cut enter the keys and the sort; the rest are emitted for a tile only
    // if its forward walk passes its near entries (the redo).
    uint32_t* mass;             // [P] opacity mass of each Gaussian's footprint, x kMassScale (preprocess)
    uint32_t* near_cnt;         // [tiles] near instances per tile (K1; zeroed with tile_cnt)
    unsigned long long* zhist;  // [kZBins] opacity mass by depth bin (K0a; zeroed with tile_cnt)
    uint32_t* zcut;             // [1] the depth bin of the cut (K1 block 0): near iff zbin(depth) <= zcut
    uint2* sranges;             // [tiles] each tile's near entries [start, start + near) (K3): K4's lists
    uint32_t* far_cur;          // [tiles] far-fill cursors (zeroed by K4)
};
constexpr int kAccRow4 = 4;     // float4 per accumulator row: 64 bytes, one line (one memory-side atomic request)
__host__ __device__ inline size_t touched_words(size_t P) { return (P + 31) / 32; }
// Depth bins of the near-first cut: 16 per octave of view-space z from the near plane (0.2) on, by the
// float bits (monotonic for z > 0): bin = (bits >> 19) - (bits(0.2f) >> 19), clamped to [0, kZBins).
constexpr int kZBins = 256;
constexpr uint32_t kZBinBase = 0x3E4CCCCDu >> 19;  // bits of 0.2f
__host__ __device__ inline uint32_t zbin(uint32_t depth_bits) {
    const uint32_t b = depth_bits >> 19;
    return b <= kZBinBase ? 0u : (b - kZBinBase >= (uint32_t)kZBins ? (uint32_t)kZBins - 1u : b - kZBinBase);
}
constexpr float kMassScale = 16.f;  // fixed point of GeomState::mass (per pixel of footprint)
constexpr uint32_t kZCutNone = 0xffffffffu;  // no cut: every Gaussian is near

// Image state: per pixel and per tile.  The per-pixel planes are tile-major: pixel (x, y) of
// tile t, in 8x8 quadrant q at lane l = (y & 7) * 8 + (x & 7), is element t * 256 + q * 64 + l
// (tile_px), so a wave's 64 lanes of one quadrant read / write 256 contiguous bytes per plane.
// (Image-major, each 8-pixel row was 32 B of a 128-B line whose other parts belong to other
// quadrants and tiles: render_bwd fetched 312 MB for 75 MB of pixel state, r2zp.)
__host__ __device__ inline size_t tile_px(uint32_t tile, int q, int lane) {
    return (size_t)tile * 256 + (size_t)q * 64 + (size_t)lane;
}
struct ImageState {
    float* final_T;       // [tiles * 256], tile-major (tile_px)
    uint32_t* n_contrib;  // [tiles * 256]
    float* accum;         // [4][tiles * 256]: colour r,g,b and inverse depth, without background
    uint2* ranges;        // [tiles]
};

// Binning state: per instance (R, or the capacity the buffer was requested for).
struct BinningState {
    unsigned long long* keys;  // per instance, grouped by tile: depth bits << 32 | tile-list entry
    uint32_t* gid_sorted;      // entry of each instance in (tile, depth, index) order: the tile lists
                               // (Gaussian << kEntryMaskBits | quadrant mask)
    float* ckpt;               // blend checkpoints, [C / kCkStride + 1][kCkFloats] (see below)
    uint2* unit_full;          // backward units covering full segments, [shard][unit_full_cap(C)]
    uint8_t* rec_flag;         // per emission index: the gradient record's content byte (GradRecs::flag),
                               // zeroed by K3, set by render_bwd, read by gauss_reduce; C + 16 bytes
};

// ---------------------------------------------------------------------------
// Blend checkpoints.  Every kCkStride list entries the forward render stores each
// pixel's blend state (live transmittance, accumulated colour, accumulated inverse
// depth) -- checkpoint c of a tile is the state after its first c * kCkStride entries.
// The backward then walks a tile's list in independent segments of kCkStride entries
// (one wave each) instead of one wave per tile, which bounds the work of a wave and
// removes the launch's tail.  Slot of the checkpoint at list position p (absolute,
// p = range.x + c * kCkStride, c >= 1): p / kCkStride -- unique because checkpoints of
// one tile are kCkStride apart and the next tile's first one is kCkStride past its start.
// Layout of a slot: [5 values][4 quadrant slots][64 lanes] floats, the values being
// T, C.r, C.g, C.b, invdepth.
// ---------------------------------------------------------------------------
constexpr int kCkStride = 256;  // a multiple of the render batch (64)
constexpr int kCkFloats = 5 * 4 * 64;

// ---------------------------------------------------------------------------
// The backward's work list.  The forward render appends, per tile, one unit (tile, first
// checkpoint) for each full segment below the tile's limit and one for the partial last
// segment; the backward runs one wave per unit in list order: full segments, then the
// partial ones by length quarter, longest first.  Every list is sharded by tile % 8 (the
// XCD the dispatcher deals the tile's workgroup to): appends are returning atomics, and one
// counter word shared by all tiles saturates (~88 adds/us chip-wide) and stalls the
// forward's waves at their ends.
// ---------------------------------------------------------------------------
constexpr int kUnitLists = 5;       // full, partial quarters 0..3 (longest first)
constexpr int kUnitShards = 8;
constexpr int kUnitCntStride = 32;  // counter words, one per 128-B line
__host__ __device__ inline uint32_t unit_part_cap(uint32_t tiles) { return (tiles + kUnitShards - 1) / kUnitShards; }
__host__ __device__ inline size_t unit_full_cap(size_t C) { return C / kCkStride + 1; }

// ---------------------------------------------------------------------------
// View block (multi-GPU exchange, include/gsr.h gsr_rasterize_backward_screen /
// gsr_gauss_backward_views): one view's camera and per-Gaussian render-gradient sums,
// in floats: [0, 64) header (the camera, offsets below), then sums.a [P][4], sums.b [P][4],
// sums.c [P][2] and the flag word [P] (bit 0 visible, bits 1-3 SH clamp mask); the block
// is padded to a multiple of 64 floats so the next view's block stays 256-byte aligned.
// ---------------------------------------------------------------------------
constexpr int kViewBlockHeader = 64;
constexpr int kViewCamView = 0, kViewCamProj = 16, kViewCamPos = 32, kViewCamTanX = 35, kViewCamTanY = 36,
              kViewCamFocalX = 37, kViewCamFocalY = 38, kViewCamAA = 39, kViewCamInvDepth = 40;
__host__ __device__ inline size_t view_block_floats(size_t P) {
    return (kViewBlockHeader + 11 * P + 63) / 64 * 64;
}
// Packed (sparse) view block: the header, the entry count in header float kViewPackCount, then
// kViewPackEntry floats per Gaussian with a non-zero render gradient (backward.hip view_pack).
constexpr int kViewPackCount = 63, kViewPackEntry = 12;
__host__ __device__ inline size_t view_pack_floats(size_t entries) {
    return (kViewBlockHeader + kViewPackEntry * entries + 63) / 64 * 64;
}

// Gradient records (backward scratch): the per-instance records of the record path, and the
// per-Gaussian sums (three arrays).
// The records' content flags are one BIT per emission index (render_bwd ORs it in with a global
// atomic, order-free): 5M@4K 14 MB for K3 to zero and gauss_reduce to scan, against 115 MB as bytes.
// render_bwd reads each entry's first emission index from rec_start[] (not the splat record's row 3,
// which K3 would then patch for every visible Gaussian: 160 MB of partial writes at 5M@4K).
struct GradRecs {
    float4* a;  // (dcolor.r, dcolor.g, dcolor.b, dinvdepth)
    float4* b;  // (dmean2D.x, dmean2D.y, dopacity_eff, dconic.b)
    float2* c;  // (dconic.a, dconic.c)
    uint8_t* flag;  // per-instance records only: the content bits (BinningState::rec_flag)
};
// The render backward writes a record and its content bit only for an entry with a gradient term
// (~half of the staged entries at 1M@1080p, 7.6M of 114.7M instances at 5M@4K); the content bits
// live in the binning buffer and are zeroed by the forward's K3 (each chunk clears its emission
// range with 16-byte stores, no memset launch), so gauss_reduce finds the records from the bits
// alone and skips the rest.  Whether an entry has a gradient term depends on the geometry only,
// not on the upstream gradient, so a second backward of the same forward sets the same bits.

// The live list (backward scratch): the Gaussians with a gradient, appended by gauss_reduce (record
// path) and views_live for the sparse gauss_bwd.  Sharded by the appending wave (one counter per
// 128-byte line): a single counter took 15625 returning atomics in a row at 1M Gaussians
// (gauss_reduce 62 -> 201 us).
constexpr int kLiveShards = 64;
constexpr int kLiveCntStride = 32;  // uint32 per counter line
// Entries per shard: the appenders' wave w adds at most its run of 64 consecutive Gaussians to shard
// w % kLiveShards, so a shard holds at most ceil(runs / kLiveShards) x 64.
__host__ __device__ inline uint32_t live_list_cap(uint32_t P) {
    constexpr uint32_t run = 64u;
    const uint32_t runs = (P + run - 1) / run;
    return (runs + kLiveShards - 1) / kLiveShards * run;
}
// The render backward's per-instance records (not the per-Gaussian sums, which stay three
// arrays) are interleaved as 48-byte records a, b, (c, pad), so one instance's three stores land
// in one or two cache lines instead of three.  Index strides:
constexpr int kRecAB = 3;  // float4 units between records (a, b)
constexpr int kRecC = 6;   // float2 units between records (c)

// ---------------------------------------------------------------------------
// SH coefficient addressing.  Two layouts reach the kernels:
//  * combined: shs [P, M, 3], coefficient k of Gaussian i at shs + (i M + k) 3
//    (CR/forward.cu:29, the vendored rasterizer);
//  * split (dc != nullptr): dc [P, 1, 3] holds coefficient 0 and shs [P, M-1, 3] the
//    rest -- the 3DGS-accel rasterizer's (dc, shs) arguments, i.e. GaussianModel's
//    _features_dc / _features_rest passed without a torch.cat
//    (gaussian_renderer/__init__.py:106-125).
// M is always the total coefficient count seen by the SH evaluation.
// ---------------------------------------------------------------------------
struct ShAddr {
    const float* shs;
    const float* dc;
    int M;
    __device__ __forceinline__ const float* coef(int idx, int k) const {
        if (!dc) return shs + ((size_t)idx * M + k) * 3;
        return k == 0 ? dc + (size_t)idx * 3 : shs + ((size_t)idx * (M - 1) + (k - 1)) * 3;
    }
};
struct ShGradAddr {
    float* dsh;
    float* ddc;
    int M;
    __device__ __forceinline__ float* coef(int idx, int k) const {
        if (!ddc) return dsh + ((size_t)idx * M + k) * 3;
        return k == 0 ? ddc + (size_t)idx * 3 : dsh + ((size_t)idx * (M - 1) + (k - 1)) * 3;
    }
};

// ---------------------------------------------------------------------------
// Device math helpers (CR/auxiliary.h:43-117)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float3 xform_point_4x3(const float3& p, const float* m) {
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ __forceinline__ float4 xform_point_4x4(const float3& p, const float* m) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}
// ndc2Pix: the reference's literal 1.0 makes this a double expression (CR/auxiliary.h:45).
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// getRect (CR/auxiliary.h:49-59).  float->int conversion on gfx950 saturates like CUDA's.
__device__ __forceinline__ void get_rect(float px, float py, int max_radius, uint32_t gx, uint32_t gy, uint2& rmin,
                                         uint2& rmax) {
    const float r = (float)max_radius;
    int v;
    v = max(0, (int)((px - r) / (float)kTile));
    rmin.x = min(gx, (uint32_t)v);
    v = max(0, (int)((py - r) / (float)kTile));
    rmin.y = min(gy, (uint32_t)v);
    v = max(0, (int)((((px + r) + (float)kTile) - 1.0f) / (float)kTile));
    rmax.x = min(gx, (uint32_t)v);
    v = max(0, (int)((((py + r) + (float)kTile) - 1.0f) / (float)kTile));
    rmax.y = min(gy, (uint32_t)v);
}

__device__ __forceinline__ uint32_t pack_i16x2(int lo, int hi) {
    lo = max(-32768, min(32767, lo));
    hi = max(-32768, min(32767, hi));
    return ((uint32_t)(uint16_t)(int16_t)lo) | ((uint32_t)(uint16_t)(int16_t)hi << 16);
}
__device__ __forceinline__ int unpack_lo(uint32_t v) { return (int)(int16_t)(uint16_t)(v & 0xffffu); }
__device__ __forceinline__ int unpack_hi(uint32_t v) { return (int)(int16_t)(uint16_t)(v >> 16); }

// ---------------------------------------------------------------------------
// Diagnostic timestamps (variant builds only: -DGSR_STAMPS).  Thread 0 of a
// workgroup writes s_memtime (shader clock) into a per-translation-unit device
// buffer, slot = workgroup * kStampSlots + phase; tools/stamps.py reads them back
// through gsr_diag_stamps().  Compiled out of the product library.
// ---------------------------------------------------------------------------
constexpr int kStampSlots = 8;
constexpr size_t kStampCap = (size_t)1 << 20;
#ifdef GSR_STAMPS
#define GSR_STAMP_BUFFER(name) static __device__ unsigned long long name[kStampCap]
#define GSR_STAMP(buf, wg, phase)                                                                       \
    do {                                                                                                \
        if (threadIdx.x == 0 && (size_t)(wg) * kStampSlots + (phase) < kStampCap)                      \
            buf[(size_t)(wg) * kStampSlots + (phase)] = __builtin_amdgcn_s_memtime();                   \
    } while (0)
// s_memrealtime (constant 100 MHz, one time base for the whole device; s_memtime is a
// per-CU shader-clock counter, fine for durations, not comparable across CUs)
#define GSR_STAMP_RT(buf, wg, slot)                                                                     \
    do {                                                                                                \
        if (threadIdx.x == 0 && (size_t)(wg) * kStampSlots + (slot) < kStampCap)                       \
            buf[(size_t)(wg) * kStampSlots + (slot)] = __builtin_amdgcn_s_memrealtime();                \
    } while (0)
// slot 7: hardware placement, XCC id << 32 | HW_ID (simd [5:4], cu [11:8], sh [12], se [15:13])
#define GSR_STAMP_HWID(buf, wg)                                                                         \
    do {                                                                                                \
        if (threadIdx.x == 0 && (size_t)(wg) * kStampSlots + 7 < kStampCap)                            \
            buf[(size_t)(wg) * kStampSlots + 7] =                                                       \
                ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) |                \
                (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                                     \
    } while (0)
#define GSR_STAMP_VAL(buf, wg, phase, v)                                                                \
    do {                                                                                                \
        if (threadIdx.x == 0 && (size_t)(wg) * kStampSlots + (phase) < kStampCap)                      \
            buf[(size_t)(wg) * kStampSlots + (phase)] = (unsigned long long)(v);                        \
    } while (0)
#else
#define GSR_STAMP_BUFFER(name) static_assert(true, "")
#define GSR_STAMP_HWID(buf, wg) do { } while (0)
#define GSR_STAMP_RT(buf, wg, slot) do { } while (0)
#define GSR_STAMP(buf, wg, phase) do { } while (0)
#define GSR_STAMP_VAL(buf, wg, phase, v) do { } while (0)
#endif

// Wave64 helpers.
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

template <int CTRL, int ROW_MASK, bool BOUND_ZERO>
__device__ __forceinline__ float dpp_f32(float v) {
    return __builtin_bit_cast(float,
                              __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, BOUND_ZERO));
}

template <uint32_t CTRL, uint32_t ROW_MASK, bool BOUND_ZERO>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, BOUND_ZERO);
}
// Non-temporal (streaming) loads of vector types HIP defines as structs.
__device__ __forceinline__ float4 load_nt(const float4* p) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 load_nt(const float2* p) {
    typedef float v2f __attribute__((ext_vector_type(2)));
    const v2f v = __builtin_nontemporal_load(reinterpret_cast<const v2f*>(p));
    return make_float2(v.x, v.y);
}

// Inclusive prefix sum / max over the wave: row_shr 1, 2, 4, 8 inside each 16-lane row, then
// row_bcast:15 and row_bcast:31 carry the row totals up (identity 0).  Six VALU steps, no LDS.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += dpp_u32<0x111, 0xf, true>(v);
    v += dpp_u32<0x112, 0xf, true>(v);
    v += dpp_u32<0x114, 0xf, true>(v);
    v += dpp_u32<0x118, 0xf, true>(v);
    v += dpp_u32<0x142, 0xa, false>(v);
    v += dpp_u32<0x143, 0xc, false>(v);
    return v;
}
__device__ __forceinline__ unsigned long long wave_incl_sum_u64(unsigned long long v) {
#define GSR_DPP64(CTRL, RM, BZ)                                                                      \
    v += ((unsigned long long)dpp_u32<CTRL, RM, BZ>((uint32_t)(v >> 32)) << 32) |                     \
         (unsigned long long)dpp_u32<CTRL, RM, BZ>((uint32_t)v)
    GSR_DPP64(0x111, 0xf, true);
    GSR_DPP64(0x112, 0xf, true);
    GSR_DPP64(0x114, 0xf, true);
    GSR_DPP64(0x118, 0xf, true);
    GSR_DPP64(0x142, 0xa, false);
    GSR_DPP64(0x143, 0xc, false);
#undef GSR_DPP64
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, dpp_u32<0x111, 0xf, true>(v));
    v = max(v, dpp_u32<0x112, 0xf, true>(v));
    v = max(v, dpp_u32<0x114, 0xf, true>(v));
    v = max(v, dpp_u32<0x118, 0xf, true>(v));
    v = max(v, dpp_u32<0x142, 0xa, false>(v));
    v = max(v, dpp_u32<0x143, 0xc, false>(v));
    return v;
}

// Full wave64 sum, valid in lane 63: Hillis-Steele prefix inside each 16-lane row
// (row_shr 1,2,4,8 with zero fill), then row_bcast:15 / row_bcast:31 carry the row
// totals upward.  Six VALU ops, no LDS traffic.
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
    v += dpp_f32<0x111, 0xf, true>(v);
    v += dpp_f32<0x112, 0xf, true>(v);
    v += dpp_f32<0x114, 0xf, true>(v);
    v += dpp_f32<0x118, 0xf, true>(v);
    v += dpp_f32<0x142, 0xa, false>(v);
    v += dpp_f32<0x143, 0xc, false>(v);
    return v;
}

// Sum over each 16-lane row, valid in lanes 15, 31, 47 and 63 (four DPP ops).
__device__ __forceinline__ float row_sum_to_lane15(float v) {
    v += dpp_f32<0x111, 0xf, true>(v);
    v += dpp_f32<0x112, 0xf, true>(v);
    v += dpp_f32<0x114, 0xf, true>(v);
    v += dpp_f32<0x118, 0xf, true>(v);
    return v;
}

// Reduce-scatter halving steps built on gfx950's lane-swap instructions.
// half_fold(x, y): lanes 0-31 get x[l] + x[l+32], lanes 32-63 get y[l-32] + y[l]
// (v_permlane32_swap exchanges the upper half of x with the lower half of y).
__device__ __forceinline__ float half_fold(float x, float y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// row_fold(x, y): on 16-lane rows, row 0 gets x0 + x1, row 1 y0 + y1, row 2 x2 + x3,
// row 3 y2 + y3 (v_permlane16_swap exchanges odd rows of x with even rows of y).
__device__ __forceinline__ float row_fold(float x, float y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// eight_fold(x, y, hi8) with hi8 = (lane & 8): on every 16-lane row, lanes 0-7 get x[l] + x[l+8]
// and lanes 8-15 get y[l-8] + y[l] (DPP row_ror:8; gfx950 has no 8-lane swap instruction).
__device__ __forceinline__ float eight_fold(float x, float y, bool hi8) {
    const float a = hi8 ? y : x, b = hi8 ? x : y;
    return a + dpp_f32<0x128, 0xf, true>(b);
}
// Sum over each 8-lane half row, in every lane of it: quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror (no lane shifted out, so every step folds into one v_add_f32_dpp).
__device__ __forceinline__ float half_row_allsum(float v) {
    v += dpp_f32<0xB1, 0xf, true>(v);
    v += dpp_f32<0x4E, 0xf, true>(v);
    v += dpp_f32<0x141, 0xf, true>(v);
    return v;
}
// Sum over each 16-lane row, in every lane of it (half_row_allsum, then row_mirror).
__device__ __forceinline__ float row_allsum(float v) {
    v = half_row_allsum(v);
    v += dpp_f32<0x140, 0xf, true>(v);
    return v;
}

}  // namespace gsr
