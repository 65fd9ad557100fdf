// binning.hip -- per-tile Gaussian lists in (depth, index) order, without a
// global sort.
//
// The reference emits one (tile << 32 | depth) key per (tile, Gaussian) instance
// and radix-sorts all of them over 32 + log2(tiles) bits (duplicateWithKeys and
// the CUB sort, CR/rasterizer_impl.cu:78-126, 332-340), which yields each tile's
// list in (depth, index) order.  Here the same lists are built in four passes:
//
//   K1 tile_count    every workgroup owns a contiguous chunk of Gaussians and
//                    counts its tile hits in LDS (+1/-1 at each tile rectangle's
//                    corners, then a 2-D prefix sum); the flush is one RETURNING atomic add
//                    per (chunk, tile), whose result -- the chunk's offset inside
//                    the tile's block -- is kept in chunk_off[chunk][tile];
//   K2 tile_scan     one workgroup: exclusive scan of the tile counts (-> the
//                    per-tile ranges, identifyTileRanges' output); it also
//                    lists the tiles too long for one wave's sort (two classes);
//   K3 tile_scatter  every chunk loads its cursors (tile start + chunk offset)
//                    into LDS and scatters 64-bit keys (depth bits << 32 |
//                    index << 4) with LDS atomics (the low 4 bits of a tile-list
//                    entry, its quadrant mask, are filled in by the forward
//                    render); it also writes each Gaussian's first record index
//                    (the chunk's base summed from K0a's chunk totals, then an
//                    in-order scan of tiles_touched);
//   K4 tile_sort     per tile, a bitonic network held in registers (exchanges
//                    inside a lane, across lanes by swizzle/permute, across
//                    waves through LDS), writing the Gaussian ids -- the tile
//                    lists the render passes walk.  Two waves per tile up to 1024
//                    keys; longer lists go to persistent kernels walking K2's
//                    class lists.
//
// K1 and K3 enumerate (Gaussian, tile) instances flattened over the wave: the 64
// Gaussians of a wave are scanned by tile count and every lane takes one
// instance per step, so a Gaussian covering 100 tiles costs its wave two steps,
// not 100 serial iterations of one lane (the reference's per-thread tile loop,
// CR/rasterizer_impl.cu:108-124).
//
// The order inside a tile is fully determined by the (depth bits, index) keys,
// which is exactly the reference's order (its sort is stable on index-ordered
// input), so the result is deterministic although K3's scatter order is not.
// No global sort, no memsets of lookback state, no host round trip: the
// instance count never leaves the device until the forward ends.
#include "kernels.h"

namespace gsr {

constexpr int kBinThreads = 1024;
constexpr int kBinWaves = kBinThreads / 64;
constexpr int kBinUnroll = 4;  // K0 / K1 Gaussians per thread per round (loads in flight together)
constexpr uint32_t kLdsTilesMax = 36864;  // K3 keeps one u32 per tile in LDS (144 KiB)
constexpr uint32_t kSortWaveMax = 1024;   // longest list tile_sort_kernel sorts (one workgroup of kSortT per tile)
// Longer lists go to two persistent 256-thread kernels walking K2's class lists: class 0
// (1024, 4096], class 1 (> 4096; bucket sort up to 8192 keys, a network in global memory
// beyond).
constexpr int kSortClasses = 2;
constexpr uint32_t kClass0Max = 4096;
constexpr uint32_t kBucketMax = 8192;

typedef unsigned long long u64;

GSR_STAMP_BUFFER(g_st_count);
GSR_STAMP_BUFFER(g_st_scatter);
GSR_STAMP_BUFFER(g_st_sort);

__device__ __forceinline__ void unpack_rect(uint2 r, uint32_t& x0, uint32_t& y0, uint32_t& x1, uint32_t& y1) {
    x0 = r.x & 0xffffu;
    y0 = r.x >> 16;
    x1 = r.y & 0xffffu;
    y1 = r.y >> 16;
}

// Tiles in a packed rectangle (= tiles_touched of its Gaussian).
__device__ __forceinline__ uint32_t rect_tiles(uint2 r) {
    return ((r.y & 0xffffu) - (r.x & 0xffffu)) * ((r.y >> 16) - (r.x >> 16));
}

// A workgroup barrier that orders LDS only: unlike __syncthreads, whose workgroup fence also waits for
// every global store the wave has in flight, it leaves the wave's stores draining.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
template <bool LDS_ONLY>
__device__ __forceinline__ void wg_barrier() {
    if constexpr (LDS_ONLY)
        lds_barrier();
    else
        __syncthreads();
}

// Sum over the workgroup (a multiple of 64 threads); result valid in every thread.
template <typename T, bool LDS_ONLY = false>
__device__ T block_sum(T v, T* s_tmp) {
    if constexpr (sizeof(T) == 4)
        v = (T)wave_incl_sum((uint32_t)v);  // DPP: the wave's sum lands in lane 63
    else
        v = (T)wave_incl_sum_u64((unsigned long long)v);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    wg_barrier<LDS_ONLY>();
    if ((threadIdx.x & 63) == 63) s_tmp[w] = v;
    wg_barrier<LDS_ONLY>();
    T t = 0;
    for (int i = 0; i < nw; i++) t += s_tmp[i];
    return t;
}

// Exclusive scan over the workgroup of one value per thread (thread order).
template <typename T, bool LDS_ONLY = false>
__device__ T block_exclusive_scan(T v, T* s_tmp, T* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T incl = v;
    if constexpr (sizeof(T) == 4)
        incl = (T)wave_incl_sum((uint32_t)v);  // DPP, no ds_bpermute chain
    else
        incl = (T)wave_incl_sum_u64((unsigned long long)v);
    wg_barrier<LDS_ONLY>();
    if (lane == 63) s_tmp[w] = incl;
    wg_barrier<LDS_ONLY>();
    T base = 0, all = 0;
    for (int i = 0; i < nw; i++) {
        if (i < w) base += s_tmp[i];
        all += s_tmp[i];
    }
    if (total) *total = all;
    return base + incl - v;
}

// Calls f(valid, owner, tile, tx, ty) once per step on every lane of the wave; over all
// steps, the valid calls are exactly the (Gaussian, tile) instances of the wave's 64
// Gaussians (lane l: n tiles in rectangle r), each once; `owner` is the lane of the
// instance's Gaussian, (tx, ty) the tile's column and row.  f may shuffle from `owner`
// (all lanes are active).
template <class F>
__device__ __forceinline__ void for_each_instance(uint32_t n, uint2 r, uint32_t gx, F&& f) {
    const int lane = threadIdx.x & 63;
    // Owner of slot s: the largest lane whose run starts at or before s.  Each round, the lanes
    // whose runs start inside it mark their start in the wave's LDS row (lane + 1), and an
    // inclusive max-scan over the wave spreads the marks; the previous round's last owner
    // fills the slots before the first mark.  (One wave's LDS accesses execute in order.)
    __shared__ uint32_t s_mark[kBinThreads];
    uint32_t* mark = s_mark + (threadIdx.x & ~63u);
    const uint32_t incl = wave_incl_sum(n);
    const uint32_t excl = incl - n;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t w = (r.y & 0xffffu) - (r.x & 0xffffu);
    uint32_t carry = 0;
    for (uint32_t base = 0; base < total; base += 64) {
        const uint32_t s = base + lane;
        mark[lane] = 0u;
        wave_lds_sync();
        if (n && excl >= base && excl < base + 64) mark[excl - base] = (uint32_t)lane + 1u;
        wave_lds_sync();
        const uint32_t m = max(wave_incl_max(mark[lane]), carry);
        wave_lds_sync();
        carry = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
        const int owner = (int)m - 1;
        const uint32_t k = s - __shfl(excl, owner);
        const uint32_t ow = __shfl(w, owner), org = __shfl(r.x, owner);
        const bool valid = s < total;
        // k / ow in fp32, branch-free (so the caller's shuffles from `owner` issue with these):
        // (k + 1/2) / ow is at least 1/(2 ow) from an integer, and rcp + mul err by < 2^-22
        // relative, so the floor is exact while k < 2^21 (a Gaussian touches < 2^21 tiles:
        // the forward rejects grids of 2^21 tiles or more, api.hip kMaxTiles).  Invalid lanes compute garbage that f ignores.
        const uint32_t dy = (uint32_t)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)max(ow, 1u)));
        // 24-bit multiplies (full rate; v_mul_lo_u32 / v_mad_u64_u32 are quarter rate): every
        // operand is < 2^16 (tile coordinates and widths, gx)
        const uint32_t tx = (org & 0xffffu) + (k - __umul24(dy, ow)), ty = (org >> 16) + dy;
        const uint32_t tile = __umul24(ty, gx) + tx;
        f(valid, owner, tile, tx, ty);
    }
}

// ---- K0: spatial order ------------------------------------------------------
// The visible Gaussians are counting-sorted by screen cell (kCell x kCell tiles,
// cell of the footprint rectangle's centre) into order[0, V).  K1 and K3 walk
// Gaussians in this order, so a chunk covers a compact screen region: it touches
// few tiles, with long runs per tile, and K3's key stores land in long contiguous
// runs instead of a few bytes per (chunk, tile) across the whole image.
constexpr uint32_t kCell = 4;
static_assert(kCell >= 1 && kCell <= 64 && (kCell & (kCell - 1)) == 0,
              "kCell: a power of two in [1, 64] (cells are formed by shifts; bin_cells coarsens them by powers of two)");

// Cells in Z order (Morton code of the cell column and row, over the power-of-two square that holds the
// grid), so a chunk of the order covers a square-ish block of cells rather than a strip of a cell row
// (5M@4K: 936 instead of 1062 tiles per chunk; r4c: bin_scatter 852-855 -> 827-831 us at 5M@4K).
__host__ __device__ inline uint32_t spread_bits16(uint32_t x) {
    x &= 0xffffu;
    x = (x | (x << 8)) & 0x00ff00ffu;
    x = (x | (x << 4)) & 0x0f0f0f0fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
}
// The cell grid K0 sorts by (bin_cells): cells of (1 << shift) tiles a side, numbered in Z order when the
// power-of-two square around the grid fits K0's LDS table (kLdsTilesMax words), row-major otherwise (a wide
// or tall frame: 10000 x 1000 px is 157 x 16 cells, whose Z square would be 65536); and coarser than
// kCell when even the row-major grid would not fit (> 589,824 tiles), so no image size is refused.
struct CellGrid {
    uint32_t cgx;     // cells per row (row-major numbering)
    uint32_t shift;   // log2 of the cell side in tiles
    uint32_t morton;  // 1: Z-order numbering
};
__device__ __forceinline__ uint32_t cell_of(uint2 r, CellGrid g) {
    const uint32_t cx = (((r.x & 0xffffu) + (r.y & 0xffffu)) >> 1) >> g.shift,
                   cy = (((r.x >> 16) + (r.y >> 16)) >> 1) >> g.shift;
    if (g.morton) return spread_bits16(cx) | (spread_bits16(cy) << 1);  // (uniform branch: a kernel argument)
    return cy * g.cgx + cx;
}

// K0a: per-chunk cell histogram in LDS; one returning atomic per (chunk, cell) gives the
// chunk's offset inside the cell's block (kept in cell_off[chunk][cell]).  Also the
// chunk's instance total (index order), for the record starts.
// zhist (near-first binning, null otherwise): each visible Gaussian's opacity mass (GeomState::mass) is
// added to its depth bin (LDS, then one global add per bin and chunk) -- the profile K1 cuts at.
__global__ void __launch_bounds__(kBinThreads) cell_count_kernel(int P, int chunk, const uint2* __restrict__ rect,
                                                                 const uint32_t* __restrict__ tiles_touched,
                                                                 uint32_t cells, CellGrid cgx,
                                                                 uint32_t* __restrict__ cell_cnt,
                                                                 uint32_t* __restrict__ cell_off,
                                                                 u64* __restrict__ chunk_total,
                                                                 const uint32_t* __restrict__ depth_key,
                                                                 const uint32_t* __restrict__ mass,
                                                                 u64* __restrict__ zhist) {
    extern __shared__ uint32_t s_c[];  // cells words
    __shared__ u64 s_tmp[kBinWaves];
    __shared__ u64 s_zh[kZBins];
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    for (uint32_t i = threadIdx.x; i < cells; i += blockDim.x) s_c[i] = 0;
    if (zhist && threadIdx.x < kZBins) s_zh[threadIdx.x] = 0ull;
    __syncthreads();
    u64 mine = 0;
    // kBinUnroll Gaussians per thread per round, their loads all issued before the LDS atomics
    for (int gb = g0 + (int)threadIdx.x; gb < g1; gb += kBinUnroll * kBinThreads) {
        uint32_t n[kBinUnroll], dk[kBinUnroll], ms[kBinUnroll];
        uint2 r[kBinUnroll];
#pragma unroll
        for (int u = 0; u < kBinUnroll; u++) {
            const int g = gb + u * kBinThreads;
            n[u] = g < g1 ? tiles_touched[g] : 0u;
            r[u] = g < g1 ? rect[g] : make_uint2(0u, 0u);
            dk[u] = zhist && g < g1 ? depth_key[g] : 0u;
            ms[u] = zhist && g < g1 ? mass[g] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kBinUnroll; u++) {
            mine += n[u];
            if (n[u]) {
                atomicAdd(&s_c[cell_of(r[u], cgx)], 1u);
                if (zhist && ms[u]) atomicAdd(&s_zh[zbin(dk[u])], (u64)ms[u]);
            }
        }
    }
    const u64 total = block_sum(mine, s_tmp);  // ends with a barrier: the histograms are complete
    if (threadIdx.x == 0) chunk_total[blockIdx.x] = total;
    if (zhist && threadIdx.x < kZBins && s_zh[threadIdx.x]) atomicAdd(&zhist[threadIdx.x], s_zh[threadIdx.x]);
    uint32_t* off = cell_off + (size_t)blockIdx.x * cells;
    for (uint32_t i = threadIdx.x; i < cells; i += blockDim.x) {
        const uint32_t c = s_c[i];
        if (c) off[i] = atomicAdd(&cell_cnt[i], c);
    }
}

// ---- Near-first binning ----------------------------------------------------------
// ("near_mass" option, api.hip.)  A pixel stops blending once T < 1e-4, after an opacity mass of
// -ln 1e-4 = 9.2 in front of it, so the back of a dense frame is never reached: at 5M@4K the walk reads
// 6.7% of the 114.7M instances and no tile reads past z = 2.29 of the scene's [2, 12]
// (tools/cutoff_estimate.py, profiles/r05/cutoff_estimate_5m_4k.json).  The cut: the depth bin at which
// the screen-averaged mass of the Gaussians in front (K0a's histogram over the image area) reaches the
// option's target (30 by default: 3.3x what one pixel needs -- 2.52 at 5M@4K).  Only the Gaussians at or
// in front of it get keys (K3) and are sorted (K4, over GeomState::sranges); each tile's range keeps its
// full length, the near entries at its start, so num_rendered, the ranges and the emission indices are
// the full list's.  A tile whose forward walk passes its near entries with pixels still blending is filed
// for the redo (render.hip, as for the reachable-prefix sort): tile_far_fill_kernel emits its far
// instances behind the near ones, the whole list is sorted and the tile rendered again -- so images and
// gradients are those of the full lists whatever the cut.
// The cut bin (in each K1 workgroup, one wave): the first bin whose cumulative mass reaches `target`
// (fixed point, kMassScale x pixels x mean mass), or kZCutNone.
__device__ uint32_t zcut_from_hist(const u64* __restrict__ zhist, u64 target) {
    const int lane = threadIdx.x & 63;
    constexpr int kPer = kZBins / 64;
    u64 v[kPer], run = 0;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
        v[i] = zhist[lane * kPer + i];
        run += v[i];
    }
    const u64 incl = wave_incl_sum_u64(run);
    u64 at = incl - run;
    uint32_t found = kZCutNone;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
        at += v[i];
        if (at >= target && found == kZCutNone) found = (uint32_t)(lane * kPer + i);
    }
    // the first lane with a crossing holds the smallest bin
    const unsigned long long m = __ballot(found != kZCutNone);
    return m ? (uint32_t)__builtin_amdgcn_readlane((int)found, __builtin_ctzll(m)) : kZCutNone;
}
__device__ __forceinline__ bool is_near(uint32_t depth_bits, uint32_t cut) {
    return cut == kZCutNone || zbin(depth_bits) <= cut;
}
// K1 / K3 arguments of the near-first binning (zhist null: off)
struct NearArgs {
    const u64* zhist;
    u64 target;
    uint32_t* zcut;      // written by K1 workgroup 0, read by K3 and the far fill
    uint32_t* near_cnt;  // per tile: near instances (K1's returning adds give each chunk its near offset)
    uint2* sranges;      // per tile: [start, start + near) (K3)
};

// K0c: every chunk scans the cell counts (redundantly, cells are few), then scatters its
// visible Gaussians into their cells' blocks as 16-byte binning records (index, rect,
// depth key), so that K1 and K3 read their chunk's Gaussians as one contiguous range
// instead of gathering them.  Block 0 publishes V.
__global__ void __launch_bounds__(kBinThreads) cell_scatter_kernel(int P, int chunk, const uint2* __restrict__ rect,
                                                                   const uint32_t* __restrict__ tiles_touched,
                                                                   uint32_t cells, CellGrid cgx,
                                                                   const uint32_t* __restrict__ cell_cnt,
                                                                   const uint32_t* __restrict__ cell_off,
                                                                   const uint32_t* __restrict__ depth_key,
                                                                   uint4* __restrict__ order,
                                                                   uint32_t* __restrict__ n_visible) {
    extern __shared__ uint32_t s_c[];  // cells words
    __shared__ uint32_t s_tmp[kBinWaves];
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    const uint32_t* off = cell_off + (size_t)blockIdx.x * cells;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < cells; base += kBinThreads) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t c = i < cells ? cell_cnt[i] : 0u;
        uint32_t all = 0;
        const uint32_t at = carry + block_exclusive_scan(c, s_tmp, &all);
        if (i < cells) s_c[i] = at + (c ? off[i] : 0u);  // off[] is written only where this chunk has entries
        carry += all;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) n_visible[0] = carry;
    __syncthreads();
    for (int gb = g0 + (int)threadIdx.x; gb < g1; gb += kBinUnroll * kBinThreads) {
        uint32_t n[kBinUnroll], dk[kBinUnroll];
        uint2 r[kBinUnroll];
#pragma unroll
        for (int u = 0; u < kBinUnroll; u++) {
            const int g = gb + u * kBinThreads;
            n[u] = g < g1 ? tiles_touched[g] : 0u;
            r[u] = g < g1 ? rect[g] : make_uint2(0u, 0u);
            dk[u] = g < g1 ? depth_key[g] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kBinUnroll; u++)
            if (n[u])
                order[atomicAdd(&s_c[cell_of(r[u], cgx)], 1u)] =
                    make_uint4((uint32_t)(gb + u * kBinThreads), r[u].x, r[u].y, dk[u]);
    }
}

// ---- K1 ---------------------------------------------------------------------
// FusedZero (K2 folded into K3, capacity mode): what K2 used to clear before the render, cleared
// here instead (nothing reads them between K1 and K3's end): the render work-list counters, the
// half-tile join words and the long-list class counters.
struct FusedZero {
    uint32_t* unit_cnt;            // null: not fused
    unsigned long long* tile_join;
    uint32_t* cls_count;
};

// K1 by rectangles (with LDS counters): a chunk's per-tile counts are the
// number of its Gaussians whose tile rectangle covers the tile, so each Gaussian adds +1 / -1 at its
// rectangle's four corners of a 2-D difference array in LDS (one u32 per tile; a corner on the far
// edge of the grid is dropped) and a 2-D inclusive prefix sum -- rows by DPP scans, one wave per row,
// then columns in register blocks -- turns the differences into the counts.  Four LDS atomics per
// Gaussian instead of one per instance (5M@4K: 20M instead of 114.7M) and no instance walk; the
// counts are exactly an instance walk's, so everything downstream is unchanged.  (Without LDS
// counters -- a grid over kLdsTilesMax tiles -- K1 walks the instances with global atomics.)
constexpr int kColBlock = 8;  // rows per register block of the column pass

// cut != kZCutNone (near-first binning): each Gaussian counts 1 in the low 16 bits (all instances) and,
// when near, also 1 in the high 16 (near instances) -- both fields exact after the prefix sums, since a
// chunk holds < 65536 Gaussians (bin_chunks) and the sums are exact integers modulo 2^32.
__device__ __forceinline__ void count_by_rectangles(int g0, int g1, const uint4* __restrict__ order, uint32_t tiles,
                                                    uint32_t gx, uint32_t* s_d, uint32_t cut = kZCutNone) {
    const uint32_t gy = tiles / gx;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < tiles; i += blockDim.x) s_d[i] = 0u;
    __syncthreads();
    for (int pb = g0 + (int)threadIdx.x; pb < g1; pb += kBinUnroll * kBinThreads) {
        uint2 rr[kBinUnroll];
        uint32_t wt[kBinUnroll];
#pragma unroll
        for (int u = 0; u < kBinUnroll; u++) {
            const int p = pb + u * kBinThreads;
            const uint4 o = p < g1 ? order[p] : make_uint4(0u, 0u, 0u, 0u);
            rr[u] = make_uint2(o.y, o.z);
            wt[u] = cut == kZCutNone ? 1u : (is_near(o.w, cut) ? 0x10001u : 1u);
        }
#pragma unroll
        for (int u = 0; u < kBinUnroll; u++) {
            uint32_t x0, y0, x1, y1;
            unpack_rect(rr[u], x0, y0, x1, y1);
            if (x0 < x1 && y0 < y1) {  // (K0 orders only Gaussians with tiles; padding lanes are empty)
                const uint32_t w = wt[u], nw = 0u - wt[u];
                atomicAdd(&s_d[y0 * gx + x0], w);
                if (x1 < gx) atomicAdd(&s_d[y0 * gx + x1], nw);
                if (y1 < gy) {
                    atomicAdd(&s_d[y1 * gx + x0], nw);
                    if (x1 < gx) atomicAdd(&s_d[y1 * gx + x1], w);
                }
            }
        }
    }
    __syncthreads();
    // rows (modular u32 arithmetic: every partial sum of a row is a count difference, the
    // final values are counts)
    for (uint32_t y = (uint32_t)wave; y < gy; y += kBinWaves) {
        uint32_t carry = 0u;
        for (uint32_t xb = 0; xb < gx; xb += 64) {
            const uint32_t x = xb + (uint32_t)lane;
            const uint32_t v = x < gx ? s_d[y * gx + x] : 0u;
            const uint32_t incl = wave_incl_sum(v) + carry;
            if (x < gx) s_d[y * gx + x] = incl;
            carry = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
    }
    __syncthreads();
    // columns: one thread per column, kColBlock independent loads per round trip
    for (uint32_t x = threadIdx.x; x < gx; x += blockDim.x) {
        uint32_t run = 0u;
        for (uint32_t yb = 0; yb < gy; yb += kColBlock) {
            uint32_t v[kColBlock];
#pragma unroll
            for (int i = 0; i < kColBlock; i++) v[i] = yb + i < gy ? s_d[(yb + i) * gx + x] : 0u;
#pragma unroll
            for (int i = 0; i < kColBlock; i++) {
                run += v[i];
                if (yb + i < gy) s_d[(yb + i) * gx + x] = run;
            }
        }
    }
    __syncthreads();
}

template <bool LDS>
__global__ void __launch_bounds__(kBinThreads) tile_count_kernel(int P, int chunk, const uint2* __restrict__ rect,
                                                                 const uint32_t* __restrict__ tiles_touched,
                                                                 const uint4* __restrict__ order,
                                                                 const uint32_t* __restrict__ n_visible,
                                                                 uint32_t tiles, uint32_t gx, uint32_t* __restrict__ cnt,
                                                                 uint32_t* __restrict__ chunk_off, FusedZero fz,
                                                                 NearArgs na) {
    extern __shared__ uint32_t s_hist[];  // (LDS) the 2-D difference array: tiles words
    if (fz.unit_cnt) {
        if (blockIdx.x == 0 && threadIdx.x < kUnitLists * kUnitShards) fz.unit_cnt[threadIdx.x * kUnitCntStride] = 0u;
        if (blockIdx.x == 0 && threadIdx.x < kSortClasses) fz.cls_count[threadIdx.x] = 0u;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < tiles; i += gridDim.x * blockDim.x)
            fz.tile_join[i] = 0ull;
    }
    if (!na.zhist && na.zcut && blockIdx.x == 0 && threadIdx.x == 0) *na.zcut = kZCutNone;  // (inspection, far fill)
    const int V = (int)n_visible[0];
    const int g0 = blockIdx.x * chunk, g1 = min(V, g0 + chunk);  // positions in order[]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    GSR_STAMP(g_st_count, blockIdx.x, 0);
    if (LDS) {
        uint32_t cut = kZCutNone;
        if (na.zhist) {  // near-first binning: the cut, from K0a's depth-mass histogram (each workgroup alike)
            __shared__ uint32_t s_cut;
            if (wave == 0) {
                const uint32_t c = zcut_from_hist(na.zhist, na.target);
                if (lane == 0) {
                    s_cut = c;
                    if (blockIdx.x == 0) *na.zcut = c;
                }
            }
            __syncthreads();
            cut = s_cut;
        }
        count_by_rectangles(g0, g1, order, tiles, gx, s_hist, cut);
        GSR_STAMP(g_st_count, blockIdx.x, 2);
        uint32_t* off = chunk_off + (size_t)blockIdx.x * tiles;
        if (cut != kZCutNone) {
            // all instances into the tile counts (the ranges keep the full lists); the near ones into the
            // near counts, whose returning adds give this chunk's near offsets (K3 places only those)
            for (uint32_t i = threadIdx.x; i < tiles; i += blockDim.x) {
                const uint32_t v = s_hist[i], full = v & 0xffffu, nr = v >> 16;
                if (full) atomicAdd(&cnt[i], full);
                if (nr) off[i] = atomicAdd(&na.near_cnt[i], nr);
            }
        } else {
            for (uint32_t i = threadIdx.x; i < tiles; i += blockDim.x) {
                const uint32_t c = s_hist[i];
                if (c) off[i] = atomicAdd(&cnt[i], c);
            }
        }
        GSR_STAMP(g_st_count, blockIdx.x, 3);
        return;
    }
    GSR_STAMP(g_st_count, blockIdx.x, 1);
    for (int pb = g0 + wave * 64; pb < g1; pb += kBinThreads) {
        const int p = pb + lane;
        const uint4 o = p < g1 ? order[p] : make_uint4(0u, 0u, 0u, 0u);
        const uint2 r = make_uint2(o.y, o.z);
        const uint32_t n = rect_tiles(r);
        for_each_instance(n, r, gx, [&](bool valid, int, uint32_t t, uint32_t, uint32_t) {
            if (valid) atomicAdd(&cnt[t], 1u);
        });
    }
}

// ---- K2 ---------------------------------------------------------------------
// One workgroup.  Rounds of blockDim * 8 tiles: each thread loads 8 consecutive
// counts (independent loads), then one block scan per round.
constexpr int kScanV = 8;

// v = p[b, b + 8) (zero past n): two 16-byte loads where the run is whole and aligned.  K3's prologue loads
// the per-tile words this way: the wave's lanes read consecutive 32-byte runs, and with one word per
// instruction each load touched 16 cache lines for 256 bytes (8x the requests; stamps: ~5 us per load
// at K3's start, 256 workgroups reading at once).
__device__ __forceinline__ void load_run8(const uint32_t* __restrict__ p, uint32_t b, uint32_t n, uint32_t (&v)[kScanV]) {
    static_assert(kScanV == 8, "two uint4 per run");
    if (b + kScanV <= n && ((uintptr_t)(p + b) & 15u) == 0) {
        const uint4 x = *reinterpret_cast<const uint4*>(p + b), y = *reinterpret_cast<const uint4*>(p + b + 4);
        v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w, v[4] = y.x, v[5] = y.y, v[6] = y.z, v[7] = y.w;
    } else {
#pragma unroll
        for (int i = 0; i < kScanV; i++) v[i] = b + i < n ? p[b + i] : 0u;
    }
}

__global__ void __launch_bounds__(kBinThreads) tile_scan_kernel(uint32_t tiles, uint32_t* __restrict__ cnt,
                                                                uint32_t n_counters, uint32_t* __restrict__ unit_cnt,
                                                                unsigned long long* __restrict__ tile_join,
                                                                uint2* __restrict__ ranges,
                                                                uint32_t* __restrict__ tile_base, u64* __restrict__ total,
                                                                u64* host_total, u64 cap, uint32_t* __restrict__ cls_list,
                                                                uint32_t* __restrict__ cls_count) {
    __shared__ u64 s_tmp[kBinWaves];
    __shared__ uint32_t s_cls[kSortClasses];
    GSR_STAMP(g_st_count, 1000, 0);  // K2's phases at workgroup slot 1000 of K1's buffer (tools/stamps.py)
    if (threadIdx.x < kSortClasses) s_cls[threadIdx.x] = 0;  // published by the scan's barriers
    if (threadIdx.x < kUnitLists * kUnitShards) unit_cnt[threadIdx.x * kUnitCntStride] = 0u;  // render work lists
    const uint32_t T = blockDim.x;
    u64 carry = 0;
    for (uint32_t base = 0; base < tiles; base += T * kScanV) {
        const uint32_t b = base + threadIdx.x * kScanV;
        uint32_t v[kScanV];
        load_run8(cnt, b, tiles, v);  // (as K3's prologue)
        u64 run = 0;
#pragma unroll
        for (int i = 0; i < kScanV; i++) run += v[i];
        u64 all = 0;
        u64 at = carry + block_exclusive_scan(run, s_tmp, &all);
#pragma unroll
        for (int i = 0; i < kScanV; i++) {
            if (b + i < tiles) {
                // clamped to the binning capacity: with a too-small capacity hint the lists are
                // truncated (and rebuilt after the forward reads the count), never overrun
                const u64 lo = at < cap ? at : cap, hi = at + v[i] < cap ? at + v[i] : cap;
                ranges[b + i] = make_uint2((uint32_t)lo, (uint32_t)hi);
                tile_base[b + i] = (uint32_t)at;
                // long list: one of the class kernels (K4).  Filed by the RAW count: on a truncated
                // pass (capacity hint too small) a tile whose clamped length is <= kSortWaveMax is
                // then sorted twice -- by tile_sort_kernel (which goes by the clamped length) and by
                // its class kernel -- into the same order, and the pass is rebuilt exactly anyway
                // (api.hip), so a tile may have two sorters only in a pass whose lists are discarded.
                if (v[i] > kSortWaveMax) {
                    const int c = v[i] <= kClass0Max ? 0 : 1;
                    cls_list[(size_t)c * tiles + atomicAdd(&s_cls[c], 1u)] = b + i;
                }
            }
            at += v[i];
        }
        carry += all;
    }
    GSR_STAMP(g_st_count, 1000, 1);
    if (threadIdx.x == 0) {
        total[0] = carry;
        // the host's copy (coherent pinned memory, mapped): no copy launch behind this kernel
        if (host_total) __hip_atomic_store(host_total, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    GSR_STAMP(g_st_count, 1000, 2);
    __syncthreads();
    GSR_STAMP(g_st_count, 1000, 3);
    if (threadIdx.x < kSortClasses) cls_count[threadIdx.x] = s_cls[threadIdx.x];
    // Leave the tile and cell counters zeroed (all reads of them are done): a rebuild of the
    // lists (capacity hint too small, api.hip) counts again without a memset.  preprocess
    // zeroes them for the first count of a call.
    for (uint32_t i = threadIdx.x; i < n_counters; i += T) cnt[i] = 0u;
    for (uint32_t i = threadIdx.x; i < tiles; i += T) tile_join[i] = 0ull;  // render_fwd's half-tile join
    GSR_STAMP(g_st_count, 1000, 4);
}

// ---- K3 ---------------------------------------------------------------------
// Fused (capacity mode, LDS cursors): K2's scan folded in.  Every workgroup scans the tile counts
// itself (8160 words at 1080p, read from L2) for its cursors; workgroup b also publishes the
// ranges and long-list classes of every gridDim-th group of 8 tiles, workgroup 0 the instance
// count.  A kernel boundary and K2's single-workgroup pass (13 us at 1M@1080p) disappear.
struct FusedScan {
    const uint32_t* cnt;          // null: not fused (tile_base holds K2's tile starts)
    uint2* ranges;
    u64* total;
    u64* host_total;
    uint32_t* cls_list;
    uint32_t* cls_count;
};

// The record path's inputs for chunk blockIdx.x (Gaussians [g0, g1), their instances starting at `chunk_base`):
// every Gaussian's first record index -- chunk base + in-order scan of tiles_touched -- and the zeroed content
// bits of the chunk's emission range.  The counts of up to four rounds are requested before the first scan,
// the scans' barriers are LDS-only, and the content-bit zeroing is issued last -- the memory counter is in
// order, so a load issued after a store waits for that store too.  K3 runs it when the forward's backward may
// take the record path; rec_prep_kernel when a backward takes it after a forward that skipped it.
__device__ __forceinline__ void rec_starts_chunk(int g0, int g1, u64 chunk_base, const uint32_t* __restrict__ tiles_touched,
                                                 const u64* __restrict__ chunk_total, uint32_t* __restrict__ rec_start,
                                                 float4* __restrict__ rec, uint8_t* __restrict__ rec_flag, u64 cap,
                                                 u64* s_tmp) {
    u64 carry = chunk_base;
    for (int gq = g0; gq < g1; gq += 4 * kBinThreads) {
        uint32_t nr[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int g = gq + u * kBinThreads + (int)threadIdx.x;
            nr[u] = g < g1 ? tiles_touched[g] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int gb = gq + u * kBinThreads;
            if (gb >= g1) break;  // uniform
            const int g = gb + (int)threadIdx.x;
            u64 all = 0;
            const u64 at = carry + block_exclusive_scan<u64, true>((u64)nr[u], s_tmp, &all);
            if (g < g1) rec_start[g] = (uint32_t)at;
            carry += all;
        }
    }
    if (rec_flag) {  // (content bits: 128 per 16-byte word)
        constexpr u64 kPer = 128;
        const u64 e1 = min(chunk_base + chunk_total[blockIdx.x], cap);
        uint4* w = reinterpret_cast<uint4*>(rec_flag);
        for (u64 i = chunk_base / kPer + threadIdx.x; i < (e1 + kPer - 1) / kPer; i += blockDim.x)
            w[i] = make_uint4(0u, 0u, 0u, 0u);
    }
}

template <bool LDS>
__global__ void __launch_bounds__(kBinThreads) tile_scatter_kernel(
    int P, int chunk, const uint2* __restrict__ rect, const uint32_t* __restrict__ tiles_touched,
    const uint32_t* __restrict__ depth_key, const uint4* __restrict__ order, const uint32_t* __restrict__ n_visible,
    uint32_t tiles, uint32_t gx, uint32_t* __restrict__ tile_base,
    const uint32_t* __restrict__ chunk_off, const u64* __restrict__ chunk_total, u64* __restrict__ keys, u64 cap,
    uint32_t* __restrict__ rec_start, float4* __restrict__ rec, uint8_t* __restrict__ rec_flag, FusedScan fs,
    NearArgs na) {
    extern __shared__ uint32_t s_cur[];  // tiles words
    __shared__ u64 s_tmp[kBinWaves];
    // near-first binning (fused only): the cut K1 chose; kZCutNone when off or when the frame's mass never
    // reached the target (then K1 counted as usual and the near lists are the whole lists)
    const uint32_t cut = na.zhist && fs.cnt ? *na.zcut : kZCutNone;
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    GSR_STAMP(g_st_scatter, blockIdx.x, 0);
    // this chunk's first record index: the instance totals of the chunks before it (K0a), summed
    // here (loads issued first, they land while the cursors load) instead of scanned in K2
    u64 before = 0;
    for (uint32_t c = threadIdx.x; c < blockIdx.x; c += blockDim.x) before += chunk_total[c];
    if (LDS && fs.cnt) {
        // the tile starts (K2's scan, redone by every workgroup), then this chunk's cursors
        const uint32_t* off = chunk_off + (size_t)blockIdx.x * tiles;
        u64 carry_t = 0;
        for (uint32_t base = 0; base < tiles; base += kBinThreads * kScanV) {
            const uint32_t b = base + threadIdx.x * kScanV;
            uint32_t v[kScanV], o[kScanV];
            load_run8(fs.cnt, b, tiles, v);
            u64 run = 0;
#pragma unroll
            for (int i = 0; i < kScanV; i++) run += v[i];
            u64 all = 0;
            u64 at = carry_t + block_exclusive_scan(run, s_tmp, &all);
            load_run8(off, b, tiles, o);
            const bool publish = (b / kScanV) % gridDim.x == blockIdx.x;  // this group's ranges and classes
#pragma unroll
            for (int i = 0; i < kScanV; i++) {
                if (b + i < tiles) {
                    s_cur[b + i] = (uint32_t)at + o[i];  // garbage where the chunk has no instance: unused
                    if (publish) {
                        const u64 lo = at < cap ? at : cap, hi = at + v[i] < cap ? at + v[i] : cap;
                        fs.ranges[b + i] = make_uint2((uint32_t)lo, (uint32_t)hi);
                        if (na.zhist) {  // K4's list: the near entries at the range's start
                            const uint32_t nr = cut == kZCutNone ? v[i] : na.near_cnt[b + i];
                            const u64 nh = at + nr < cap ? at + nr : cap;
                            na.sranges[b + i] = make_uint2((uint32_t)lo, (uint32_t)nh);
                        }
                    }
                }
                at += v[i];
            }
            carry_t += all;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            fs.total[0] = carry_t;
            if (fs.host_total) __hip_atomic_store(fs.host_total, carry_t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        // (classes by raw count, as K2: see the note there on truncated passes)
        // this workgroup's long-list tiles into the class lists: counted in LDS, one global atomic
        // per class reserves the workgroup's run (one global atomic per tile serialised ~30000
        // returning atomics on one counter at 4K: +340 us), then each tile takes its slot
        __shared__ uint32_t s_cls[kSortClasses], s_cbase[kSortClasses];
        const uint32_t groups = (tiles + kScanV - 1) / kScanV;
        const uint32_t my_groups = groups > blockIdx.x ? (groups - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
        if (threadIdx.x < kSortClasses) s_cls[threadIdx.x] = 0u;
        __syncthreads();
        // (the sort's list length: the near count under a cut)
        const uint32_t* scnt = cut != kZCutNone ? na.near_cnt : fs.cnt;
        for (uint32_t j = threadIdx.x; j < my_groups * kScanV; j += blockDim.x) {
            const uint32_t t = (blockIdx.x + (j / kScanV) * gridDim.x) * kScanV + j % kScanV;
            const uint32_t v = t < tiles ? scnt[t] : 0u;
            if (v > kSortWaveMax) atomicAdd(&s_cls[v <= kClass0Max ? 0 : 1], 1u);
        }
        __syncthreads();
        if (threadIdx.x < kSortClasses) {
            const uint32_t k = s_cls[threadIdx.x];
            s_cbase[threadIdx.x] = k ? atomicAdd(&fs.cls_count[threadIdx.x], k) : 0u;
            s_cls[threadIdx.x] = 0u;
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < my_groups * kScanV; j += blockDim.x) {
            const uint32_t t = (blockIdx.x + (j / kScanV) * gridDim.x) * kScanV + j % kScanV;
            const uint32_t v = t < tiles ? scnt[t] : 0u;
            if (v > kSortWaveMax) {
                const int c = v <= kClass0Max ? 0 : 1;
                fs.cls_list[(size_t)c * tiles + s_cbase[c] + atomicAdd(&s_cls[c], 1u)] = t;
            }
        }
    } else if (LDS) {
        // this chunk's cursors: tile start + the chunk's offset inside the tile (K1); entries of
        // tiles the chunk does not touch are garbage and never used
        const uint32_t* off = chunk_off + (size_t)blockIdx.x * tiles;
        for (uint32_t i = threadIdx.x; i < tiles; i += blockDim.x) s_cur[i] = tile_base[i] + off[i];
    }
    // first record index of every Gaussian: chunk base + in-order scan of tiles_touched (rec_starts_chunk)
    // (rec_start null: the forward's backward takes the atomic path, which reads neither)
    if (rec_start) {
        const u64 chunk_base = block_sum<u64, true>(before, s_tmp);
        rec_starts_chunk(g0, g1, chunk_base, tiles_touched, chunk_total, rec_start, rec, rec_flag, cap, s_tmp);
    }
    if (LDS) lds_barrier();
    GSR_STAMP(g_st_scatter, blockIdx.x, 1);
    // the keys: chunk positions [q0, q1) of the spatial order (K0), as K1 counted them
    const int V = (int)n_visible[0];
    const int q0 = blockIdx.x * chunk, q1 = min(V, q0 + chunk);
    for (int pb = q0 + wave * 64; pb < q1; pb += kBinThreads) {
        const int p = pb + lane;
        const uint4 o = p < q1 ? order[p] : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t g = o.x, dk = o.w;
        const uint2 r = make_uint2(o.y, o.z);
        const uint32_t n = is_near(dk, cut) ? rect_tiles(r) : 0u;  // (a cut: the far Gaussians get no keys)
        for_each_instance(n, r, gx, [&](bool valid, int owner, uint32_t t, uint32_t, uint32_t) {
            const uint32_t kh = __shfl(dk, owner), kg = __shfl(g, owner);
            if (!valid) return;
            const uint32_t pos = LDS ? atomicAdd(&s_cur[t], 1u) : atomicAdd(&tile_base[t], 1u);
            if (pos < cap) keys[pos] = ((u64)kh << 32) | (kg << kEntryMaskBits);  // cap: redone if exceeded
        });
    }
#ifdef GSR_STAMPS
    __syncthreads();
#endif
    GSR_STAMP(g_st_scatter, blockIdx.x, 2);
}

// ---- K4 ---------------------------------------------------------------------
// Bitonic sorting network over N2 = T * E keys, element i = thread * E + r held in
// register a[r] (keys past the list are +infinity = ~0).  Exchange distance j:
//   j < E        inside the thread (registers),
//   E <= j < 64E across lanes, lane distance j / E: DPP (1, 2, 4, 8) or the gfx950
//                lane-swap instructions (16, 32) -- VALU only, no LDS traffic,
//   j >= 64E     across waves, through LDS (T > 64 only).
// Every compare-exchange is one 64-bit compare whose result is flipped by the
// direction mask, then selects.
template <int S>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
    const int x = (int)v;
    if constexpr (S == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]
    } else if constexpr (S == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xf, 0xf, true);  // quad_perm [2,3,0,1]
    } else if constexpr (S == 4) {
        const int up = __builtin_amdgcn_mov_dpp(x, 0x104, 0xf, 0xf, true);  // row_shl:4, lane + 4
        const int dn = __builtin_amdgcn_mov_dpp(x, 0x114, 0xf, 0xf, true);  // row_shr:4, lane - 4
        return (uint32_t)((threadIdx.x & 4) ? dn : up);
    } else if constexpr (S == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x128, 0xf, 0xf, true);  // row_ror:8
    } else if constexpr (S == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // rows (0,1), (2,3) swapped
        return (threadIdx.x & 16) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // halves swapped
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
}

template <int S>
__device__ __forceinline__ u64 lane_xor_u64(u64 v) {
    return ((u64)lane_xor<S>((uint32_t)(v >> 32)) << 32) | lane_xor<S>((uint32_t)v);
}

template <int E, int S>
__device__ __forceinline__ void xlane_step(u64 (&a)[E], bool keep_min) {
#pragma unroll
    for (int r = 0; r < E; r++) {
        const u64 b = lane_xor_u64<S>(a[r]);
        a[r] = ((b < a[r]) == keep_min) ? b : a[r];
    }
}

template <int T, int E>
__device__ __forceinline__ void bitonic_regs(u64 (&a)[E], u64* s_x) {
    constexpr uint32_t N2 = (uint32_t)T * E;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
#pragma unroll
    for (uint32_t k = 2; k <= N2; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (j < (uint32_t)E) {
#pragma unroll
                for (int r = 0; r < E; r++) {
                    if (r & j) continue;
                    const int p = r | (int)j;
                    const bool desc = ((tid * E + r) & k) != 0;
                    const u64 lo = a[r], hi = a[p];
                    const bool sw = (hi < lo) != desc;
                    a[r] = sw ? hi : lo;
                    a[p] = sw ? lo : hi;
                }
            } else if (j < 64u * E) {
                const uint32_t s = j / E;
                const bool keep_min = ((lane & s) == 0) == (((tid * E) & k) == 0);
                switch (s) {  // compile-time after unrolling
                    case 1: xlane_step<E, 1>(a, keep_min); break;
                    case 2: xlane_step<E, 2>(a, keep_min); break;
                    case 4: xlane_step<E, 4>(a, keep_min); break;
                    case 8: xlane_step<E, 8>(a, keep_min); break;
                    case 16: xlane_step<E, 16>(a, keep_min); break;
                    default: xlane_step<E, 32>(a, keep_min); break;
                }
            } else {
#pragma unroll
                for (int r = 0; r < E; r++) s_x[tid * E + r] = a[r];
                __syncthreads();
                const uint32_t i0 = tid * E;  // j >= 64E: partner of i0 + r is (i0 ^ j) + r
                const bool keep_min = ((i0 & j) == 0) == ((i0 & k) == 0);
#pragma unroll
                for (int r = 0; r < E; r++) {
                    const u64 b = s_x[(i0 ^ j) + r];
                    a[r] = ((b < a[r]) == keep_min) ? b : a[r];
                }
                __syncthreads();
            }
        }
    }
}

// Sort keys[lo, lo + n) (n <= T * E, T = the workgroup size) and write the tile-list
// entries (low key halves: Gaussian << 4; the Gaussian index is unique, so the order is the
// reference's (depth, index) order).
template <int T, int E>
__device__ __forceinline__ void sort_list(const u64* __restrict__ keys, uint32_t lo, uint32_t n,
                                          uint32_t* __restrict__ gid_sorted, u64* s_x) {
    u64 a[E];
    const uint32_t i0 = threadIdx.x * E;
#pragma unroll
    for (int r = 0; r < E; r++) a[r] = i0 + r < n ? *(keys + lo + i0 + r) : ~0ull;
    bitonic_regs<T, E>(a, s_x);
#pragma unroll
    for (int r = 0; r < E; r++)
        if (i0 + r < n) gid_sorted[lo + i0 + r] = (uint32_t)a[r];
}

__device__ __forceinline__ uint32_t tile_len(uint2 r, u64 cap) {
    const u64 hi = r.y < cap ? r.y : cap;
    return hi > r.x ? (uint32_t)(hi - r.x) : 0u;
}

// Bitonic network in global memory, for lists longer than any register/LDS sort here (any
// length; slow -- real scenes rarely produce such tiles, and the bucket sort below takes every
// list up to kBucketMax).  The "flip" form: every comparator is ascending; for block size k the
// first step pairs i with i ^ (k - 1), the others with i ^ j, so keys past n behave as +infinity
// and are never touched.
__device__ void sort_list_global(u64* __restrict__ keys, uint32_t lo, uint32_t n, uint32_t* __restrict__ gid_sorted) {
    u64* k = keys + lo;
    uint32_t N2 = 1;
    while (N2 < n) N2 <<= 1;
    for (uint32_t kk = 2; kk <= N2; kk <<= 1) {
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t p = threadIdx.x; p < N2 / 2; p += blockDim.x) {
                const uint32_t a = ((p & ~(j - 1)) << 1) | (p & (j - 1));  // p-th index with bit j clear
                const uint32_t b = (j == (kk >> 1)) ? (a ^ (kk - 1)) : (a | j);
                if (b < n) {
                    const u64 x = k[a], y = k[b];
                    if (y < x) {
                        k[a] = y;
                        k[b] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) gid_sorted[lo + i] = (uint32_t)k[i];
}

// ---- bucket-rank sort ---------------------------------------------------------
// A tile's keys are unique 64-bit values (depth bits << 32 | Gaussian << 4), so a key's
// place in the sorted list is the number of smaller keys.  Two steps, all in LDS:
//  1. bucket: the tile's key range [min, max] is cut into 2^lg equal bins (the key minus min,
//     shifted right); each key takes a slot in its bin with a returning LDS atomic (the order
//     inside a bin is arbitrary), a scan of the bin counts gives the bin starts, and the keys
//     are scattered to their bins;
//  2. rank: a key's position is its bin's start plus the number of smaller keys in its bin.
//     Neighbouring lanes hold keys of the same or adjacent bins, so their LDS reads of a bin
//     are mostly broadcasts.
// The work is ~n plus the sum over bins of size^2, against ~78 compare-exchange stages per key
// for a 4096-key bitonic network (the sort this replaces).  When the bins are badly skewed --
// the tile's depths cluster in a sliver of their range, sum of squares above kSkew * n -- the
// list goes to the bitonic network instead (the caller's fallback).  The result is the
// reference's (depth, index) order exactly: keys are compared whole.
constexpr int kBinShift = 1;       // bins = pow2 >= n >> kBinShift (about two keys per bin)
constexpr uint32_t kSkew = 48;     // fallback when sum(bin size^2) > kSkew * n

template <int T, int NMAX, int NBMAX>
struct BucketLds {
    u64 buf[NMAX];
    uint32_t start[NBMAX + 1];
    u64 red[2 * (T / 64)];
    uint32_t tmp[T / 64];
    uint32_t m;   // entries sorted (prefix mode); a window's end (window modes)
    uint32_t mb;  // the first bin past a window (bucket_sort_long)
};

template <int T>
__device__ __forceinline__ void block_minmax_u64(u64& mn, u64& mx, u64* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const u64 a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if constexpr (T > 64) {
        const int w = threadIdx.x >> 6;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) {
            red[2 * w] = mn;
            red[2 * w + 1] = mx;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < T / 64; i++) {
            mn = red[2 * i] < mn ? red[2 * i] : mn;
            mx = red[2 * i + 1] > mx ? red[2 * i + 1] : mx;
        }
    }
}

// Sorts keys[lo, lo + n) (n <= T * E) into gid_sorted[lo, lo + n) (low key halves) and returns
// true, or returns false (nothing written, uniformly over the workgroup) when the bins are too
// skewed.  The keys are loaded once, striped over the workgroup (all E loads of a thread in
// flight together), and stay in registers until they are scattered to their bins.  The caller
// must barrier before reusing the LDS.
// Prefix mode (lim < n): only the bins that start below lim are scattered and ranked -- the
// smallest *sorted = lim + (the rest of the bin lim falls in) keys, in final order at
// gid_sorted[lo, lo + *sorted); the other entries are left unwritten.  The bins are the full key
// range's, so the keys kept are exactly the smallest *sorted of the list.
// Window mode (WIN, whole lists longer than the LDS buffer): the bins are scattered and ranked in
// windows of whole bins of at most NMAX keys each, in order, reusing the buffer; it fails (uniformly,
// after writing part of the list -- the caller's fallback rewrites all of it) when one bin alone
// exceeds the buffer.
template <int T, int E, int NMAX, int NBMAX, bool WIN = false>
__device__ bool bucket_sort_list(const u64* __restrict__ keys, uint32_t lo, uint32_t n,
                                 uint32_t* __restrict__ gid_sorted, BucketLds<T, NMAX, NBMAX>& s,
                                 uint32_t lim = ~0u, uint32_t* sorted = nullptr) {
    // T * E > NMAX: more keys in registers than the LDS buffer takes -- for prefix use; the sort
    // fails (uniformly) when the prefix does not fit the buffer
    const uint32_t tid = threadIdx.x;
    u64 k[E];
    uint32_t o[E];
    u64 mn = ~0ull, mx = 0ull;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)e * T + tid;
        k[e] = i < n ? *(keys + lo + i) : 0ull;
    }
#pragma unroll
    for (int e = 0; e < E; e++) {
        if ((uint32_t)e * T + tid < n) {
            mn = k[e] < mn ? k[e] : mn;
            mx = k[e] > mx ? k[e] : mx;
        }
    }
    block_minmax_u64<T>(mn, mx, s.red);
    uint32_t lg = 0;
    while ((1u << lg) < (n >> kBinShift) && (1u << lg) < (uint32_t)NBMAX) lg++;
    const u64 range = mx - mn;
    const uint32_t bits = range ? 64u - (uint32_t)__clzll((long long)range) : 0u;
    const uint32_t sh = bits > lg ? bits - lg : 0u;
    const uint32_t nb = (uint32_t)(range >> sh) + 1u;  // <= 2^lg bins
    const uint32_t per = (nb + T - 1) / T;            // bins per thread in the scan
    for (uint32_t i = tid; i < per * T + 1; i += T) s.start[i] = 0u;
    if (tid == 0) s.m = n;  // the prefix ends at n unless a bin below crosses lim
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++)
        if ((uint32_t)e * T + tid < n) o[e] = atomicAdd(&s.start[(uint32_t)((k[e] - mn) >> sh)], 1u);
    __syncthreads();
    // bin counts -> bin starts (in place), and the sum of squared bin sizes
    uint32_t run = 0, sq = 0;
    for (uint32_t c = 0; c < per; c++) {
        const uint32_t v = s.start[tid * per + c];
        run += v;
        sq += v * v;
    }
    uint32_t all = 0;
    uint32_t at = block_exclusive_scan(run, s.tmp, &all);
    const uint32_t sumsq = block_sum(sq, s.tmp);  // (ends with a barrier: every count was read)
    if (sumsq > kSkew * n) return false;  // uniform
    for (uint32_t c = 0; c < per; c++) {
        const uint32_t v = s.start[tid * per + c];
        s.start[tid * per + c] = at;
        // the prefix ends with the bin lim falls in, or right before the nonempty bin starting at
        // lim (one bin of the workgroup matches, if any)
        if ((at < lim && lim < at + v) || (at == lim && v)) s.m = at < lim ? at + v : at;
        at += v;
    }
    if (tid == 0) s.start[nb] = n;  // bins past nb are empty and never looked up
    __syncthreads();
    if constexpr (WIN) {
        for (uint32_t w0 = 0; w0 < n;) {  // uniform
            // the window [w0, w1): up to the start of the bin that straddles w0 + NMAX, if one does
            const uint32_t cut = w0 + (uint32_t)NMAX;
            if (tid == 0) s.m = cut < n ? cut : n;
            __syncthreads();
            if (cut < n)
                for (uint32_t c = 0; c < per; c++) {
                    const uint32_t b = tid * per + c;
                    if (s.start[b] < cut && cut < s.start[b + 1]) atomicMin(&s.m, s.start[b]);
                }
            __syncthreads();
            const uint32_t w1 = s.m;
            if (w1 <= w0) return false;  // uniform: one bin holds more keys than the buffer
#pragma unroll
            for (int e = 0; e < E; e++) {
                if ((uint32_t)e * T + tid < n) {
                    const uint32_t st = s.start[(uint32_t)((k[e] - mn) >> sh)];
                    if (st >= w0 && st < w1) s.buf[st - w0 + o[e]] = k[e];
                }
            }
            __syncthreads();
            for (uint32_t j = tid; j < w1 - w0; j += T) {
                const u64 kj = s.buf[j];
                const uint32_t b = (uint32_t)((kj - mn) >> sh);
                const uint32_t st = s.start[b] - w0, en = s.start[b + 1] - w0;
                uint32_t c = 0;
#pragma unroll 4
                for (uint32_t q = st; q < en; q++) c += s.buf[q] < kj ? 1u : 0u;
                gid_sorted[lo + w0 + st + c] = (uint32_t)kj;
            }
            __syncthreads();  // the buffer and s.m are reused by the next window
            w0 = w1;
        }
        if (sorted && tid == 0) *sorted = n;
        return true;
    }
    const uint32_t m = s.m;
    if (T * E > NMAX && m > (uint32_t)NMAX) return false;  // uniform: the prefix overflows the buffer
#pragma unroll
    for (int e = 0; e < E; e++) {
        if ((uint32_t)e * T + tid < n) {
            const uint32_t st = s.start[(uint32_t)((k[e] - mn) >> sh)];
            if (st < m) s.buf[st + o[e]] = k[e];
        }
    }
    __syncthreads();
    if (sorted && tid == 0) *sorted = m;
    for (uint32_t j = tid; j < m; j += T) {
        const u64 kj = s.buf[j];
        const uint32_t b = (uint32_t)((kj - mn) >> sh);
        const uint32_t st = s.start[b], en = s.start[b + 1];
        uint32_t c = 0;
#pragma unroll 4
        for (uint32_t q = st; q < en; q++) c += s.buf[q] < kj ? 1u : 0u;
        gid_sorted[lo + st + c] = (uint32_t)kj;
    }
    return true;
}

// The same bucket sort for a list longer than the workgroup holds in registers (n > T x E): the keys stay in
// global memory (a tile's list, L2-resident) and are read once for the range, once for the bin counts and
// once per window of whole bins of at most NMAX keys (the WIN mode above, with the keys re-read instead of
// held).  A key's slot in its bin comes from an LDS atomic on the bin's start, which leaves start[b] at the
// next bin's start; so after a window's scatter bin b spans [start[b - 1], start[b]) (b > 0; [0, start[0])
// for b = 0), since every bin before it is scattered or empty.  The rank inside the bin is its count of
// smaller keys, as above.  Fails (uniformly; part of the list may be written, the caller's fallback rewrites
// all of it) on skew or when one bin alone exceeds the buffer.
// Prefix mode (lim < n): the windows stop once they cover lim keys; *sorted receives the keys in order (the
// windows' end, >= lim), the rest is left unwritten -- the smallest *sorted keys of the list, as above.
template <int T, int NMAX, int NBMAX>
__device__ bool bucket_sort_long(const u64* __restrict__ keys, uint32_t lo, uint32_t n,
                                 uint32_t* __restrict__ gid_sorted, BucketLds<T, NMAX, NBMAX>& s,
                                 uint32_t lim = ~0u, uint32_t* sorted = nullptr) {
    constexpr int U = 4;  // loads in flight per thread and pass
    const uint32_t tid = threadIdx.x;
    const u64* kl = keys + lo;
    u64 mn = ~0ull, mx = 0ull;
    for (uint32_t i0 = tid; i0 < n; i0 += U * T) {
        u64 k[U];
#pragma unroll
        for (int u = 0; u < U; u++) k[u] = i0 + u * T < n ? kl[i0 + u * T] : 0ull;
#pragma unroll
        for (int u = 0; u < U; u++)
            if (i0 + u * T < n) {
                mn = k[u] < mn ? k[u] : mn;
                mx = k[u] > mx ? k[u] : mx;
            }
    }
    block_minmax_u64<T>(mn, mx, s.red);
    uint32_t lg = 0;
    while ((1u << lg) < (n >> kBinShift) && (1u << lg) < (uint32_t)NBMAX) lg++;
    const u64 range = mx - mn;
    const uint32_t bits = range ? 64u - (uint32_t)__clzll((long long)range) : 0u;
    const uint32_t sh = bits > lg ? bits - lg : 0u;
    const uint32_t nb = (uint32_t)(range >> sh) + 1u;  // <= 2^lg bins
    const uint32_t per = (nb + T - 1) / T;
    for (uint32_t i = tid; i < per * T + 1; i += T) s.start[i] = 0u;
    __syncthreads();
    for (uint32_t i0 = tid; i0 < n; i0 += U * T) {
        u64 k[U];
#pragma unroll
        for (int u = 0; u < U; u++) k[u] = i0 + u * T < n ? kl[i0 + u * T] : 0ull;
#pragma unroll
        for (int u = 0; u < U; u++)
            if (i0 + u * T < n) atomicAdd(&s.start[(uint32_t)((k[u] - mn) >> sh)], 1u);
    }
    __syncthreads();
    uint32_t run = 0, sq = 0;
    for (uint32_t c = 0; c < per; c++) {
        const uint32_t v = s.start[tid * per + c];
        run += v;
        sq += v * v;
    }
    uint32_t all = 0;
    uint32_t at = block_exclusive_scan(run, s.tmp, &all);
    const uint32_t sumsq = block_sum(sq, s.tmp);  // (ends with a barrier: every count was read)
    if (sumsq > kSkew * n) return false;  // uniform
    for (uint32_t c = 0; c < per; c++) {
        const uint32_t v = s.start[tid * per + c];
        s.start[tid * per + c] = at;
        at += v;
    }
    if (tid == 0) s.start[nb] = n;
    __syncthreads();
    // the window's bins are [bw0, bw1): the bins before bw0 are scattered (start[b] moved to the next bin's
    // start, at most w0), so they never straddle a cut
    uint32_t bw0 = 0, w0 = 0;
    while (w0 < n && w0 < lim) {  // uniform
        const uint32_t cut = w0 + (uint32_t)NMAX;
        if (tid == 0) {
            s.m = cut < n ? cut : n;
            s.mb = nb;
        }
        __syncthreads();
        if (cut < n)
            for (uint32_t c = 0; c < per; c++) {
                const uint32_t b = tid * per + c;
                if (b >= bw0 && b < nb && s.start[b] < cut && cut < s.start[b + 1]) atomicMin(&s.m, s.start[b]);
            }
        __syncthreads();
        const uint32_t w1 = s.m;
        if (w1 <= w0) return false;  // uniform: one bin holds more keys than the buffer
        for (uint32_t c = 0; c < per; c++) {  // the first bin starting at or past w1
            const uint32_t b = tid * per + c;
            if (b >= bw0 && b < nb && s.start[b] >= w1) atomicMin(&s.mb, b);
        }
        __syncthreads();
        const uint32_t bw1 = s.mb;
        for (uint32_t i0 = tid; i0 < n; i0 += U * T) {
            u64 k[U];
#pragma unroll
            for (int u = 0; u < U; u++) k[u] = i0 + u * T < n ? kl[i0 + u * T] : 0ull;
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (i0 + u * T < n) {
                    const uint32_t b = (uint32_t)((k[u] - mn) >> sh);
                    if (b >= bw0 && b < bw1) s.buf[atomicAdd(&s.start[b], 1u) - w0] = k[u];
                }
            }
        }
        __syncthreads();
        for (uint32_t j = tid; j < w1 - w0; j += T) {
            const u64 kj = s.buf[j];
            const uint32_t b = (uint32_t)((kj - mn) >> sh);
            const uint32_t st = (b ? s.start[b - 1] : 0u) - w0, en = s.start[b] - w0;
            uint32_t c = 0;
#pragma unroll 4
            for (uint32_t q = st; q < en; q++) c += s.buf[q] < kj ? 1u : 0u;
            gid_sorted[lo + w0 + st + c] = (uint32_t)kj;
        }
        __syncthreads();  // the buffer, the starts and s.m / s.mb are reused by the next window
        w0 = w1;
        bw0 = bw1;
    }
    if (sorted && tid == 0) *sorted = w0;
    return true;
}

// Lists of up to kSortWaveMax keys: one workgroup (kSortT threads) per tile.  Short lists (<= kBucketMinN) are
// sorted by a bitonic network in registers (no LDS, no barrier); longer ones by the bucket
// sort, with the register network as its skew fallback.
constexpr uint32_t kBucketMinN = 128;
// Threads per tile of the bucket sort below: 128 = two waves per tile, each holding half of the
// tile's keys (the same LDS per tile as one wave, half the serial chain per thread: tile_sort
// 66.6 -> 55.6-58.1 us at 1M@1080p against one wave, 62 us with four; r3y1).  The register
// network for short or skewed lists runs on the first wave alone.
constexpr int kSortT = 128;
static_assert(kSortT == 64 || kSortT == 128 || kSortT == 256, "tile_sort_kernel: 1, 2 or 4 waves");

__global__ void __launch_bounds__(kSortT) tile_sort_kernel(const uint2* __restrict__ ranges,
                                                       const u64* __restrict__ keys, u64 cap,
                                                       uint32_t* __restrict__ gid_sorted,
                                                       uint32_t* __restrict__ zero_cnt, uint32_t n_zero,
                                                       uint32_t* __restrict__ sorted_len,
                                                       uint32_t* __restrict__ redo_flag,
                                                       uint32_t* __restrict__ redo_cnt,
                                                       uint32_t* __restrict__ far_cur) {
    __shared__ BucketLds<kSortT, kSortWaveMax, kSortWaveMax / 2> s;
    // fused binning: K2's re-zeroing of the counters (tile, cell and near counts, the depth-mass
    // histogram: bin_zero_words), strided over the grid's threads (a tiny frame has fewer threads than words)
    if (zero_cnt)
        for (uint32_t i = blockIdx.x * kSortT + threadIdx.x; i < n_zero; i += gridDim.x * kSortT) zero_cnt[i] = 0u;
    if (far_cur && threadIdx.x == 0) far_cur[blockIdx.x] = 0u;  // (near-first binning: the redo's far fill)
    const uint2 r = ranges[blockIdx.x];
    const uint32_t n = tile_len(r, cap);
    if (threadIdx.x == 0) {  // the forward's redo state (render.hip), and this kernel's lists' lengths
        redo_flag[blockIdx.x] = 0u;
        if (blockIdx.x == 0) redo_cnt[0] = 0u;
        if (n <= kSortWaveMax) sorted_len[blockIdx.x] = n;  // (longer lists: the class kernels)
    }
    GSR_STAMP(g_st_sort, blockIdx.x, 0);
    GSR_STAMP_VAL(g_st_sort, blockIdx.x, 2, n);
    if (n <= 1) {
        if (n == 1 && threadIdx.x == 0) gid_sorted[r.x] = (uint32_t)keys[r.x];
        return;
    }
    if (n > kSortWaveMax) return;  // a class kernel's list (K2)
    if (n > kBucketMinN) {  // uniform
        const bool done = n <= 256   ? bucket_sort_list<kSortT, 256 / kSortT>(keys, r.x, n, gid_sorted, s)
                          : n <= 512 ? bucket_sort_list<kSortT, 512 / kSortT>(keys, r.x, n, gid_sorted, s)
                                     : bucket_sort_list<kSortT, 1024 / kSortT>(keys, r.x, n, gid_sorted, s);
        if (done) {
            GSR_STAMP(g_st_sort, blockIdx.x, 1);
            return;
        }
    }
    if (kSortT > 64 && threadIdx.x >= 64) return;  // (no barrier follows: the network is one wave's)
    if (n <= 64)
        sort_list<64, 1>(keys, r.x, n, gid_sorted, nullptr);
    else if (n <= 128)
        sort_list<64, 2>(keys, r.x, n, gid_sorted, nullptr);
    else if (n <= 256)
        sort_list<64, 4>(keys, r.x, n, gid_sorted, nullptr);
    else if (n <= 512)
        sort_list<64, 8>(keys, r.x, n, gid_sorted, nullptr);
    else if (n <= kSortWaveMax)
        sort_list<64, 16>(keys, r.x, n, gid_sorted, nullptr);
    GSR_STAMP(g_st_sort, blockIdx.x, 1);
}

// Persistent: 256-thread workgroups walk the class lists of long tiles (K2).  Whole-list mode:
// tile_sort_window_kernel below takes both classes.  Prefix mode: tile_sort_prefix_kernel, both classes too.
constexpr int kClassThreads = 256;

// Prefix mode (the "sort_prefix" option in force): every long list -- both class lists -- sorted
// to its reachable prefix by one kernel whose LDS holds only the prefix (kPrefixBuf keys and up to
// kPrefixBins bins: 24 KiB, twice the class-0 kernel's occupancy), the keys themselves in
// registers (up to kBucketMax per tile).  Skewed bins, a prefix over the buffer or a list over
// kBucketMax fall back to the global-memory network (whole list).
constexpr int kPrefixBuf = 2048;
static_assert(kPrefixBuf >= 2 * (int)kSortPrefixMax, "a prefix plus the rest of its bucket fits the LDS buffer");
constexpr int kPrefixBins = 2048;

// T threads x E keys per thread: 256 x 16 (<= 4096 keys: class 0's lists).  16 keys in at most 96 VGPRs: five
// workgroups per CU (the LDS would allow six; 80 VGPRs spill): tile_sort 372-373 -> 357-360 us at 5M@4K against
// four; 512 x 8 measured 450 (six waves per SIMD) and 397 us (eight) (r3y3).  Class 1's lists (longer) are
// walked first by the same kernel, their keys re-read from memory (bucket_sort_long, prefix mode) -- no launch
// of their own, and no length limit (a 256 x 32 register kernel took them up to 8192 keys before).
constexpr int kPrefixWaves = 5;
template <int T, int E>
__global__ void __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(kPrefixWaves)))
tile_sort_prefix_kernel(const uint2* __restrict__ ranges, u64* __restrict__ keys, u64 cap,
                        uint32_t* __restrict__ gid_sorted, const uint32_t* __restrict__ list0,
                        const uint32_t* __restrict__ count0, const uint32_t* __restrict__ list1,
                        const uint32_t* __restrict__ count1, uint32_t lim, uint32_t* __restrict__ sorted_len) {
    __shared__ BucketLds<T, kPrefixBuf, kPrefixBins> s;
    const uint32_t n1 = count1[0], nb = n1 + count0[0];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t t = b < n1 ? list1[b] : list0[b - n1];
        const uint2 r = ranges[t];
        const uint32_t n = tile_len(r, cap);
        if (n <= 1) {
            if (n == 1 && threadIdx.x == 0) gid_sorted[r.x] = (uint32_t)keys[r.x];
            if (threadIdx.x == 0) sorted_len[t] = n;
        } else if (n > (uint32_t)(T * E)
                       ? !bucket_sort_long<T, kPrefixBuf, kPrefixBins>(keys, r.x, n, gid_sorted, s, lim, sorted_len + t)
                       : !bucket_sort_list<T, E>(keys, r.x, n, gid_sorted, s, lim, sorted_len + t)) {
            __syncthreads();
            sort_list_global(keys, r.x, n, gid_sorted);
            if (threadIdx.x == 0) sorted_len[t] = n;
        }
        __syncthreads();  // the LDS is reused by the next tile
    }
}

// Whole-list mode, both classes: the prefix kernel's layout -- the keys in registers, an LDS buffer of
// kPrefixBuf keys (24 KiB: five workgroups per CU, against three for the 41-KiB class-0 kernel) --
// with the bins ranked in windows of at most kPrefixBuf keys; a skewed list or one bin over the
// buffer takes the global-memory network.  tile_sort 57.5-57.9 -> 52.3-52.4 us at 1M@1080p (r3y6),
// against a class-0 kernel with the whole 41-KiB list buffer in LDS.  Five waves (at four, no spill
// but slower, r6e).  Class-1 lists (> kClass0Max keys, more than the registers hold) are walked first
// (the longest work first) and bucket-sorted with the keys re-read from memory (bucket_sort_long), so
// no launch of their own is needed: a kernel queued behind another costs ~4.6 us however little it
// does (tools/launch_floor.hip, r7n), which the 82-KiB class-1 kernel paid every step at 1080p with
// nothing to sort.
__global__ void __launch_bounds__(kClassThreads) __attribute__((amdgpu_waves_per_eu(kPrefixWaves)))
tile_sort_window_kernel(const uint2* __restrict__ ranges, u64* __restrict__ keys, u64 cap,
                        uint32_t* __restrict__ gid_sorted, const uint32_t* __restrict__ list0,
                        const uint32_t* __restrict__ count0, const uint32_t* __restrict__ list1,
                        const uint32_t* __restrict__ count1, uint32_t* __restrict__ sorted_len) {
    constexpr int T = kClassThreads, E = kClass0Max / kClassThreads;
    __shared__ BucketLds<T, kPrefixBuf, kPrefixBins> s;
    const uint32_t n1 = count1[0], nb = n1 + count0[0];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t t = b < n1 ? list1[b] : list0[b - n1];
        const uint2 r = ranges[t];
        const uint32_t n = tile_len(r, cap);  // may be shorter than its class when truncated by cap
        if (n <= 1) {
            if (n == 1 && threadIdx.x == 0) gid_sorted[r.x] = (uint32_t)keys[r.x];
            if (threadIdx.x == 0) sorted_len[t] = n;
        } else if (n > (uint32_t)(T * E) ? !bucket_sort_long<T, kPrefixBuf, kPrefixBins>(keys, r.x, n, gid_sorted, s)
                                         : !bucket_sort_list<T, E, kPrefixBuf, kPrefixBins, true>(
                                               keys, r.x, n, gid_sorted, s, ~0u, sorted_len + t)) {
            __syncthreads();
            sort_list_global(keys, r.x, n, gid_sorted);
            if (threadIdx.x == 0) sorted_len[t] = n;
        } else if (n > (uint32_t)(T * E) && threadIdx.x == 0) {
            sorted_len[t] = n;
        }
        __syncthreads();  // the LDS is reused by the next tile
    }
}

// Whole-list sort of selected tiles, 256 threads per tile (any length: the bucket sort up to
// kBucketMax keys, then a register network up to 4096, a global-memory network beyond).
//  * redo (list != null): the tiles the forward filed because a wave reached the end of their
//    sorted prefix with pixels still blending (render.hip); the full list goes to `out`
//    (= gid_sorted), sorted_len becomes the whole length and the tile's half-wave join word is
//    cleared, so the redo render starts the tile afresh.  Persistent; exits at once when the list
//    is empty (the usual case).
//  * inspection (list == null): every tile whose list is only prefix-sorted gets its whole sorted
//    list in `out` (gsr_debug_forward_state's copy; the product's buffers are not written).
__global__ void __launch_bounds__(kClassThreads) tile_sort_full_kernel(const uint2* __restrict__ ranges,
                                                                      u64* __restrict__ keys, u64 cap,
                                                                      uint32_t* __restrict__ out,
                                                                      const uint32_t* __restrict__ list,
                                                                      const uint32_t* __restrict__ count,
                                                                      uint32_t tiles,
                                                                      uint32_t* __restrict__ sorted_len,
                                                                      unsigned long long* __restrict__ tile_join) {
    constexpr int T = kClassThreads;
    __shared__ BucketLds<T, kBucketMax, kBucketMax / 2> s;
    const uint32_t nb = list ? count[0] : tiles;
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t t = list ? list[b] : b;
        const uint2 r = ranges[t];
        const uint32_t n = tile_len(r, cap);
        if (!list && sorted_len[t] >= n) continue;  // uniform: a whole-sorted list
        if (n <= 1) {
            if (n == 1 && threadIdx.x == 0) out[r.x] = (uint32_t)keys[r.x];
        } else if (n > kBucketMax || !bucket_sort_list<T, kBucketMax / T>(keys, r.x, n, out, s)) {
            __syncthreads();
            if (n <= (uint32_t)T * 16)
                sort_list<T, 16>(keys, r.x, n, out, s.buf);
            else
                sort_list_global(keys, r.x, n, out);
        }
        if (list && threadIdx.x == 0) {
            sorted_len[t] = n;
            tile_join[t] = 0ull;
        }
        __syncthreads();  // the LDS is reused by the next tile
    }
}

// out[lo, lo + sorted_len) = gid_sorted[lo, ...) for every tile (gsr_debug_forward_state: the
// product's sorted entries, with the quadrant masks the forward wrote into them).
__global__ void __launch_bounds__(64) copy_sorted_prefix_kernel(const uint2* __restrict__ ranges, u64 cap,
                                                                 const uint32_t* __restrict__ gid_sorted,
                                                                 const uint32_t* __restrict__ sorted_len,
                                                                 uint32_t* __restrict__ out) {
    const uint2 r = ranges[blockIdx.x];
    const uint32_t n = min(tile_len(r, cap), sorted_len[blockIdx.x]);
    for (uint32_t i = threadIdx.x; i < n; i += 64) out[r.x + i] = gid_sorted[r.x + i];
}

// ---- launchers ----------------------------------------------------------------
constexpr int kBinChunksMax = 256;
int bin_chunks(int P, int* chunk) {
    // ~256 chunks (enough workgroups for the chip), each < 65536 Gaussians (16-bit LDS counters)
    int n = (P + 1023) / 1024;
    if (n > kBinChunksMax) n = kBinChunksMax;
    if (n < 1) n = 1;
    int c = (P + n - 1) / n;
    if (c > 65535) {
        c = 65535;
        n = (P + c - 1) / c;
    }
    *chunk = c;
    return n;
}

size_t bin_chunk_count(int P) {
    int chunk = 0;
    return (size_t)bin_chunks(P, &chunk);
}

// The cell grid of a gx x gy tile grid (CellGrid above) and its cell count, always <= kLdsTilesMax.
uint32_t bin_cells(uint32_t gx, uint32_t gy, CellGrid* cg) {
    uint32_t shift = 0;
    while ((1u << shift) < kCell) shift++;
    for (;; shift++) {
        const uint32_t cgx = (gx + (1u << shift) - 1) >> shift, cgy = (gy + (1u << shift) - 1) >> shift;
        {  // Morton codes of the cells: the power-of-two square around the grid
            uint32_t side = 1;
            while (side < cgx || side < cgy) side <<= 1;
            if ((size_t)side * side <= kLdsTilesMax) {
                *cg = CellGrid{cgx, shift, 1u};
                return side * side;
            }
        }
        if ((size_t)cgx * cgy <= kLdsTilesMax) {
            *cg = CellGrid{cgx, shift, 0u};
            return cgx * cgy;
        }
    }
}

bool bin_fused_ok(uint32_t tiles) { return tiles <= kLdsTilesMax; }
bool bin_near_ok(uint32_t tiles) { return tiles <= kLdsTilesMax; }

size_t bin_cell_count(uint32_t gx, uint32_t gy) {
    CellGrid cg{};
    return bin_cells(gx, gy, &cg);
}

// K0 + K1 + K2: spatial order, chunk instance totals, tile counts, ranges, tile starts,
// chunk offsets, the long-list class lists and the instance count (g.total).
hipError_t launch_bin_count(int P, const GeomState& g, uint32_t gx, uint32_t gy, uint2* ranges, size_t cap,
                            unsigned long long* host_total, hipStream_t stream, bool fused, unsigned long long near_target) {
    const uint32_t tiles = gx * gy;
    int chunk = 0;
    const int nchunks = bin_chunks(P, &chunk);
    CellGrid cgx{};
    const uint32_t cells = bin_cells(gx, gy, &cgx);  // (<= kLdsTilesMax for any grid)
    const bool lds = tiles <= kLdsTilesMax;
    const dim3 grid(nchunks), block(kBinThreads);
    // g.tile_cnt / g.cell_cnt are zero here: preprocess zeroes them, tile_scan_kernel re-zeroes them
    const size_t cell_bytes = cells * sizeof(uint32_t);
    // near-first binning (near_target > 0; fused, K1 by rectangles only): K0a's depth-mass histogram, K1's cut
    const bool near = near_target > 0 && fused && lds;
    const NearArgs na = near ? NearArgs{g.zhist, near_target, g.zcut, g.near_cnt, g.sranges}
                             : NearArgs{nullptr, 0ull, g.zcut, nullptr, nullptr};  // (K1 records "no cut")
    hipLaunchKernelGGL(cell_count_kernel, grid, block, cell_bytes, stream, P, chunk, g.rect, g.tiles_touched, cells,
                       cgx, g.cell_cnt, g.cell_off, g.chunk_total, g.depth_key, g.mass, near ? g.zhist : nullptr);
    hipLaunchKernelGGL(cell_scatter_kernel, grid, block, cell_bytes, stream, P, chunk, g.rect, g.tiles_touched,
                       cells, cgx, g.cell_cnt, g.cell_off, g.depth_key, g.order, g.n_visible);
    // K1's LDS: one u32 per tile (by rectangles) or two 16-bit walk counters per word
    const size_t hist_bytes = !lds ? 0 : tiles * sizeof(uint32_t);
    if (fused && !lds) return hipErrorInvalidValue;  // the fused scan needs the LDS cursors
    const FusedZero fz = fused ? FusedZero{g.unit_cnt, g.tile_join, g.cls_count} : FusedZero{nullptr, nullptr, nullptr};
    if (lds)
        hipLaunchKernelGGL(tile_count_kernel<true>, grid, block, hist_bytes, stream, P, chunk, g.rect, g.tiles_touched,
                           g.order, g.n_visible, tiles, gx, g.tile_cnt, g.chunk_off, fz, na);
    else
        hipLaunchKernelGGL(tile_count_kernel<false>, grid, block, 0, stream, P, chunk, g.rect, g.tiles_touched,
                           g.order, g.n_visible, tiles, gx, g.tile_cnt, g.chunk_off, fz, na);
    if (!fused)  // (fused: K3 scans the counts itself)
        hipLaunchKernelGGL(tile_scan_kernel, dim3(1), block, 0, stream, tiles, g.tile_cnt, tiles + cells, g.unit_cnt,
                           g.tile_join, ranges, g.tile_base, g.total, (u64*)host_total, (u64)cap, g.cls_list,
                           g.cls_count);
    return hipGetLastError();
}

// K3: scatter the keys into a binning buffer of capacity `cap` (after launch_bin_count).
hipError_t launch_bin_scatter(int P, const GeomState& g, uint32_t gx, uint32_t gy, const BinningState& b, size_t cap,
                              hipStream_t stream, uint2* ranges, unsigned long long* host_total, bool fused,
                              bool near_first, bool recs) {
    const uint32_t tiles = gx * gy;
    int chunk = 0;
    const int nchunks = bin_chunks(P, &chunk);
    const bool lds = tiles <= kLdsTilesMax;
    const dim3 grid(nchunks), block(kBinThreads);
    const size_t cur_bytes = lds ? tiles * sizeof(uint32_t) : 0;
    if (fused && !lds) return hipErrorInvalidValue;
    const FusedScan fs = fused ? FusedScan{g.tile_cnt, ranges, g.total, (u64*)host_total, g.cls_list, g.cls_count}
                               : FusedScan{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    // (as launch_bin_count decided it: the target is K1's business, K3 reads the cut)
    const NearArgs na = near_first && fused && lds
                            ? NearArgs{g.zhist, 1ull, g.zcut, g.near_cnt, g.sranges}
                            : NearArgs{nullptr, 0ull, nullptr, nullptr, nullptr};
    if (lds)
        hipLaunchKernelGGL(tile_scatter_kernel<true>, grid, block, cur_bytes, stream, P, chunk, g.rect,
                           g.tiles_touched, g.depth_key, g.order, g.n_visible, tiles, gx, g.tile_base, g.chunk_off,
                           g.chunk_total, b.keys, (u64)cap, recs ? g.rec_start : nullptr, g.rec,
                           recs ? b.rec_flag : nullptr, fs, na);
    else
        hipLaunchKernelGGL(tile_scatter_kernel<false>, grid, block, 0, stream, P, chunk, g.rect, g.tiles_touched,
                           g.depth_key, g.order, g.n_visible, tiles, gx, g.tile_base, g.chunk_off, g.chunk_total,
                           b.keys, (u64)cap, recs ? g.rec_start : nullptr, g.rec, recs ? b.rec_flag : nullptr, fs, na);
    return hipGetLastError();
}

// The record path's inputs after a forward that skipped them (launch_bin_scatter's `recs` false): K3's chunks,
// each its base from K0a's chunk totals, its record starts and its content bits.
__global__ void __launch_bounds__(kBinThreads) rec_prep_kernel(int P, int chunk, const uint32_t* __restrict__ tiles_touched,
                                                               const u64* __restrict__ chunk_total,
                                                               uint32_t* __restrict__ rec_start, float4* __restrict__ rec,
                                                               uint8_t* __restrict__ rec_flag, u64 cap) {
    __shared__ u64 s_tmp[kBinWaves];
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    u64 before = 0;
    for (uint32_t c = threadIdx.x; c < blockIdx.x; c += blockDim.x) before += chunk_total[c];
    const u64 chunk_base = block_sum<u64, true>(before, s_tmp);
    rec_starts_chunk(g0, g1, chunk_base, tiles_touched, chunk_total, rec_start, rec, rec_flag, cap, s_tmp);
}

hipError_t launch_rec_prep(int P, const GeomState& g, const BinningState& b, size_t cap, hipStream_t stream) {
    if (P <= 0) return hipSuccess;
    int chunk = 0;
    const int nchunks = bin_chunks(P, &chunk);
    hipLaunchKernelGGL(rec_prep_kernel, dim3(nchunks), dim3(kBinThreads), 0, stream, P, chunk, g.tiles_touched,
                       g.chunk_total, g.rec_start, g.rec, b.rec_flag, (u64)cap);
    return hipGetLastError();
}

hipError_t launch_tile_sort(uint32_t tiles, const uint2* ranges, const GeomState& g, const BinningState& b,
                            size_t cap, hipStream_t stream, bool zero_counts, uint32_t cells, uint32_t prefix) {
    if (tiles == 0 || cap == 0) return hipSuccess;
    const u64 c = cap;
    const uint32_t lim = prefix ? prefix : ~0u;
    const uint32_t n_zero = (uint32_t)bin_zero_words(tiles, cells);
    hipLaunchKernelGGL(tile_sort_kernel, dim3(tiles), dim3(kSortT), 0, stream, ranges, b.keys, c, b.gid_sorted,
                       zero_counts ? g.tile_cnt : nullptr, n_zero, g.sorted_len, g.redo_flag, g.redo_cnt, g.far_cur);
    // persistent class kernels: grids sized to fill the chip when their lists are long
    const auto grid = [&](uint32_t want) { return dim3(tiles < want ? tiles : want); };
    if (prefix) {
        hipLaunchKernelGGL((tile_sort_prefix_kernel<kClassThreads, kClass0Max / kClassThreads>), grid(4096),
                           dim3(kClassThreads), 0, stream, ranges, b.keys, c, b.gid_sorted, g.cls_list, g.cls_count,
                           g.cls_list + tiles, g.cls_count + 1, lim, g.sorted_len);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(tile_sort_window_kernel, grid(2048), dim3(kClassThreads), 0, stream, ranges, b.keys, c,
                       b.gid_sorted, g.cls_list, g.cls_count, g.cls_list + tiles, g.cls_count + 1, g.sorted_len);
    return hipGetLastError();
}

hipError_t launch_tile_sort_redo(uint32_t tiles, const uint2* ranges, const GeomState& g, const BinningState& b,
                                 size_t cap, hipStream_t stream) {
    if (tiles == 0 || cap == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_sort_full_kernel, dim3(tiles < 256 ? tiles : 256), dim3(kClassThreads), 0, stream, ranges,
                       b.keys, (u64)cap, b.gid_sorted, g.redo_list, g.redo_cnt, tiles, g.sorted_len, g.tile_join);
    return hipGetLastError();
}

// Near-first binning's far fill: the far instances (depth bin past the cut) of the selected tiles, keyed
// as K3 keys them, behind each tile's near entries [start + near, start + full) -- in any order (the
// whole-list sort follows).  Selected: the tiles the forward filed for a redo (redo mode; exits at once
// when none, the usual case), or every tile whose sorted entries fall short of its whole list
// (inspection, gsr_debug_forward_state).  The walk is K3's, over the spatial order, with the selected
// tiles as a bitmap in LDS; its cost is an instance walk of the far Gaussians, paid only by a frame
// with a filed tile.
__global__ void __launch_bounds__(kBinThreads) tile_far_fill_kernel(int chunk, const uint4* __restrict__ order,
                                                                    const uint32_t* __restrict__ n_visible,
                                                                    const uint32_t* __restrict__ zcut, uint32_t tiles,
                                                                    uint32_t gx, const uint2* __restrict__ ranges,
                                                                    const uint2* __restrict__ sranges,
                                                                    const uint32_t* __restrict__ redo_list,
                                                                    const uint32_t* __restrict__ redo_cnt,
                                                                    const uint32_t* __restrict__ sorted_len,
                                                                    uint32_t* __restrict__ far_cur, u64* __restrict__ keys,
                                                                    u64 cap, float4* __restrict__ acc) {
    extern __shared__ uint32_t s_sel[];  // (tiles + 31) / 32 words: selected tiles
    const uint32_t cut = *zcut;
    const uint32_t nred = redo_cnt ? redo_cnt[0] : 0u;
    if (cut == kZCutNone || (redo_cnt && nred == 0)) return;  // uniform
    const uint32_t words = (tiles + 31) / 32;
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) s_sel[i] = 0u;
    __syncthreads();
    if (redo_cnt) {
        for (uint32_t i = threadIdx.x; i < nred; i += blockDim.x) {
            const uint32_t t = redo_list[i];
            atomicOr(&s_sel[t >> 5], 1u << (t & 31u));
        }
    } else {
        for (uint32_t t = threadIdx.x; t < tiles; t += blockDim.x)
            if (sorted_len[t] < tile_len(ranges[t], cap)) atomicOr(&s_sel[t >> 5], 1u << (t & 31u));
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int V = (int)n_visible[0];
    const int q0 = blockIdx.x * chunk, q1 = min(V, q0 + chunk);
    for (int pb = q0 + wave * 64; pb < q1; pb += kBinThreads) {
        const int p = pb + lane;
        const uint4 o = p < q1 ? order[p] : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t g = o.x, dk = o.w;
        const uint2 r = make_uint2(o.y, o.z);
        const uint32_t n = p < q1 && !is_near(dk, cut) ? rect_tiles(r) : 0u;
        for_each_instance(n, r, gx, [&](bool valid, int owner, uint32_t t, uint32_t, uint32_t) {
            const uint32_t kh = __shfl(dk, owner), kg = __shfl(g, owner);
            if (!valid || !((s_sel[t >> 5] >> (t & 31u)) & 1u)) return;
            const uint2 rr = ranges[t];
            const uint32_t at = sranges[t].y + atomicAdd(&far_cur[t], 1u);
            if (at < rr.y && at < cap) keys[at] = ((u64)kh << 32) | (kg << kEntryMaskBits);
            if (acc) {  // (atomic backward: this Gaussian's row, which the forward's fill left alone, zeroed)
                float4* row = acc + (size_t)kg * kAccRow4;
#pragma unroll
                for (int k = 0; k < kAccRow4; k++) row[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        });
    }
}

hipError_t launch_far_fill(int P, const GeomState& g, uint32_t gx, uint32_t tiles, const uint2* ranges,
                           const BinningState& b, size_t cap, bool redo, hipStream_t stream, float4* acc) {
    if (tiles == 0 || cap == 0 || P == 0) return hipSuccess;
    int chunk = 0;
    const int nchunks = bin_chunks(P, &chunk);
    hipLaunchKernelGGL(tile_far_fill_kernel, dim3(nchunks), dim3(kBinThreads), ((tiles + 31) / 32) * sizeof(uint32_t),
                       stream, chunk, g.order, g.n_visible, g.zcut, tiles, gx, ranges, g.sranges,
                       redo ? g.redo_list : nullptr, redo ? g.redo_cnt : nullptr, g.sorted_len, g.far_cur, b.keys,
                       (u64)cap, redo ? acc : nullptr);
    return hipGetLastError();
}

hipError_t launch_sorted_lists_copy(uint32_t tiles, const uint2* ranges, const GeomState& g, const BinningState& b,
                                    size_t cap, uint32_t* out, hipStream_t stream, int P, uint32_t gx, bool near_first) {
    if (tiles == 0 || cap == 0) return hipSuccess;
    if (near_first) {  // the far entries of every tile not rendered from its whole list, then their cursors reset
        if (hipError_t e = launch_far_fill(P, g, gx, tiles, ranges, b, cap, false, stream)) return e;
        if (hipError_t e = hipMemsetAsync(g.far_cur, 0, sizeof(uint32_t) * tiles, stream)) return e;
    }
    hipLaunchKernelGGL(tile_sort_full_kernel, dim3(tiles < 2048 ? tiles : 2048), dim3(kClassThreads), 0, stream,
                       ranges, b.keys, (u64)cap, out, nullptr, nullptr, tiles, g.sorted_len, nullptr);
    hipLaunchKernelGGL(copy_sorted_prefix_kernel, dim3(tiles), dim3(64), 0, stream, ranges, (u64)cap, b.gid_sorted,
                       g.sorted_len, out);
    return hipGetLastError();
}

}  // namespace gsr

#ifdef GSR_STAMPS
extern "C" int gsr_diag_stamps_binning(int which, unsigned long long* out, size_t n) {
    using namespace gsr;
    if (n > kStampCap) n = kStampCap;
    const void* sym = which == 0 ? (const void*)&g_st_count : which == 1 ? (const void*)&g_st_scatter
                                                                          : (const void*)&g_st_sort;
    return (int)hipMemcpyFromSymbol(out, sym, n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost);
}
#endif
