// binning.hip -- per-tile Gaussian lists in (depth, index) order, without a
// global sort.
//
// The reference emits one (tile << 32 | depth) key per (tile, Gaussian) instance
// and radix-sorts all of them over 32 + log2(tiles) bits (duplicateWithKeys and
// the CUB sort, CR/rasterizer_impl.cu:78-126, 332-340), which yields each tile's
// list in (depth, index) order.  Here the same lists are built in four passes:
//
//   K1 tile_count    every workgroup owns a contiguous chunk of Gaussians and
//                    counts its tile hits in an LDS histogram (two 16-bit
//                    counters per word), flushed with one atomic add per tile;
//                    it also sums the chunk's tiles_touched;
//   K2 tile_scan     one workgroup: exclusive scans of the tile counts (-> the
//                    per-tile ranges, identifyTileRanges' output) and of the
//                    chunk totals (-> each chunk's first record index);
//   K3 tile_scatter  every chunk reserves a block per tile with ONE returning
//                    atomic and scatters 64-bit keys (depth bits << 32 | index)
//                    into it; it also writes each Gaussian's first record index;
//   K4 tile_sort     per tile, an in-LDS sorting network on the keys (one
//                    workgroup per tile, sized by the list length), writing the
//                    Gaussian ids -- the tile lists the render passes walk.
//
// The order inside a tile is fully determined by the (depth bits, index) keys,
// which is exactly the reference's order (its sort is stable on index-ordered
// input), so the result is deterministic although K3's scatter order is not.
// No global sort, no memsets of lookback state, no host round trip: the
// instance count never leaves the device until the forward ends.
#include "kernels.h"

namespace gsr {

constexpr int kBinThreads = 1024;
constexpr uint32_t kLdsTilesMax = 36864;  // K3 keeps one u32 per tile in LDS (144 KiB)

__device__ __forceinline__ void unpack_rect(uint2 r, uint32_t& x0, uint32_t& y0, uint32_t& x1, uint32_t& y1) {
    x0 = r.x & 0xffffu;
    y0 = r.x >> 16;
    x1 = r.y & 0xffffu;
    y1 = r.y >> 16;
}

// Sum over the workgroup (a multiple of 64 threads); result valid in every thread.
template <typename T>
__device__ T block_sum(T v, T* s_tmp) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_tmp[w] = v;
    __syncthreads();
    T t = 0;
    for (int i = 0; i < nw; i++) t += s_tmp[i];
    return t;
}

// Exclusive scan over the workgroup of one value per thread (thread order).
template <typename T>
__device__ T block_exclusive_scan(T v, T* s_tmp, T* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T incl = v;
    for (int off = 1; off < 64; off <<= 1) {
        const T u = __shfl_up(incl, off);
        if (lane >= off) incl += u;
    }
    __syncthreads();
    if (lane == 63) s_tmp[w] = incl;
    __syncthreads();
    T base = 0, all = 0;
    for (int i = 0; i < nw; i++) {
        if (i < w) base += s_tmp[i];
        all += s_tmp[i];
    }
    if (total) *total = all;
    return base + incl - v;
}

// ---- K1 ---------------------------------------------------------------------
template <bool LDS>
__global__ void __launch_bounds__(kBinThreads) tile_count_kernel(int P, int chunk, const uint2* __restrict__ rect,
                                                                 const uint32_t* __restrict__ tiles_touched,
                                                                 uint32_t tiles, uint32_t gx, uint32_t* __restrict__ cnt,
                                                                 unsigned long long* __restrict__ chunk_total) {
    extern __shared__ uint32_t s_hist[];  // (tiles + 1) / 2 words: 16-bit counters (a chunk has < 65536 Gaussians)
    __shared__ unsigned long long s_tmp[kBinThreads / 64];
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    const uint32_t words = (tiles + 1) / 2;
    if (LDS) {
        for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) s_hist[i] = 0;
        __syncthreads();
    }
    unsigned long long mine = 0;
    for (int g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
        const uint32_t n = tiles_touched[g];
        if (n == 0) continue;
        mine += n;
        uint32_t x0, y0, x1, y1;
        unpack_rect(rect[g], x0, y0, x1, y1);
        for (uint32_t y = y0; y < y1; y++)
            for (uint32_t x = x0; x < x1; x++) {
                const uint32_t t = y * gx + x;
                if (LDS)
                    atomicAdd(&s_hist[t >> 1], 1u << ((t & 1u) * 16));
                else
                    atomicAdd(&cnt[t], 1u);
            }
    }
    const unsigned long long total = block_sum(mine, s_tmp);
    if (threadIdx.x == 0) chunk_total[blockIdx.x] = total;
    if (LDS) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) {
            const uint32_t w = s_hist[i];
            if (w & 0xffffu) atomicAdd(&cnt[2 * i], w & 0xffffu);
            if ((w >> 16) && 2 * i + 1 < tiles) atomicAdd(&cnt[2 * i + 1], w >> 16);
        }
    }
}

// ---- K2 ---------------------------------------------------------------------
// One workgroup.  Thread t scans a contiguous run of tiles (then of chunks).
__global__ void __launch_bounds__(kBinThreads) tile_scan_kernel(uint32_t tiles, const uint32_t* __restrict__ cnt,
                                                                uint2* __restrict__ ranges, uint32_t* __restrict__ cursor,
                                                                int nchunks,
                                                                const unsigned long long* __restrict__ chunk_total,
                                                                unsigned long long* __restrict__ chunk_base,
                                                                unsigned long long* __restrict__ total,
                                                                unsigned long long cap) {
    __shared__ unsigned long long s_tmp[kBinThreads / 64];
    const uint32_t T = blockDim.x;
    {
        const uint32_t per = (tiles + T - 1) / T, b = threadIdx.x * per, e = min(tiles, b + per);
        unsigned long long run = 0;
        for (uint32_t t = b; t < e; t++) run += cnt[t];
        unsigned long long all = 0;
        unsigned long long at = block_exclusive_scan(run, s_tmp, &all);
        for (uint32_t t = b; t < e; t++) {
            const uint32_t c = cnt[t];
            // clamped to the binning capacity: with a too-small capacity hint the lists are
            // truncated (and rebuilt after the forward reads the count), never overrun
            const unsigned long long lo = at < cap ? at : cap, hi = at + c < cap ? at + c : cap;
            ranges[t] = make_uint2((uint32_t)lo, (uint32_t)hi);
            cursor[t] = (uint32_t)at;
            at += c;
        }
        if (threadIdx.x == 0) total[0] = all;
    }
    {
        const uint32_t n = (uint32_t)nchunks, per = (n + T - 1) / T, b = threadIdx.x * per, e = min(n, b + per);
        unsigned long long run = 0;
        for (uint32_t c = b; c < e; c++) run += chunk_total[c];
        unsigned long long at = block_exclusive_scan(run, s_tmp, (unsigned long long*)nullptr);
        for (uint32_t c = b; c < e; c++) {
            chunk_base[c] = at;
            at += chunk_total[c];
        }
    }
}

// ---- K3 ---------------------------------------------------------------------
// Thread i of a chunk owns Gaussians [g0 + i*per, g0 + (i+1)*per): contiguous runs,
// so the record offsets are an in-order block scan.
template <bool LDS>
__global__ void __launch_bounds__(kBinThreads) tile_scatter_kernel(
    int P, int chunk, const uint2* __restrict__ rect, const uint32_t* __restrict__ tiles_touched,
    const uint32_t* __restrict__ depth_key, uint32_t tiles, uint32_t gx, uint32_t* __restrict__ cursor,
    const unsigned long long* __restrict__ chunk_base, unsigned long long* __restrict__ keys, unsigned long long cap,
    uint32_t* __restrict__ rec_start, float4* __restrict__ rec) {
    extern __shared__ uint32_t s_cur[];  // tiles words
    __shared__ unsigned long long s_tmp[kBinThreads / 64];
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    const int per = (chunk + (int)blockDim.x - 1) / (int)blockDim.x;
    const int b = g0 + (int)threadIdx.x * per, e = min(g1, b + per);

    // first record index of every Gaussian: chunk base + in-order scan of tiles_touched
    unsigned long long run = 0;
    for (int g = b; g < e; g++) run += tiles_touched[g];
    unsigned long long at = chunk_base[blockIdx.x] + block_exclusive_scan(run, s_tmp, (unsigned long long*)nullptr);
    for (int g = b; g < e; g++) {
        const uint32_t n = tiles_touched[g];
        rec_start[g] = (uint32_t)at;
        if (n) reinterpret_cast<uint32_t*>(rec + (size_t)kRecRows * g + 3)[3] = (uint32_t)at;
        at += n;
    }

    if (LDS) {
        for (uint32_t i = threadIdx.x; i < tiles; i += blockDim.x) s_cur[i] = 0;
        __syncthreads();
        for (int g = b; g < e; g++) {
            if (tiles_touched[g] == 0) continue;
            uint32_t x0, y0, x1, y1;
            unpack_rect(rect[g], x0, y0, x1, y1);
            for (uint32_t y = y0; y < y1; y++)
                for (uint32_t x = x0; x < x1; x++) atomicAdd(&s_cur[y * gx + x], 1u);
        }
        __syncthreads();
        // one reservation per (chunk, tile)
        for (uint32_t i = threadIdx.x; i < tiles; i += blockDim.x) {
            const uint32_t c = s_cur[i];
            if (c) s_cur[i] = atomicAdd(&cursor[i], c);
        }
        __syncthreads();
    }
    for (int g = b; g < e; g++) {
        if (tiles_touched[g] == 0) continue;
        const unsigned long long key = ((unsigned long long)depth_key[g] << 32) | (uint32_t)g;
        uint32_t x0, y0, x1, y1;
        unpack_rect(rect[g], x0, y0, x1, y1);
        for (uint32_t y = y0; y < y1; y++)
            for (uint32_t x = x0; x < x1; x++) {
                const uint32_t t = y * gx + x;
                const uint32_t pos = LDS ? atomicAdd(&s_cur[t], 1u) : atomicAdd(&cursor[t], 1u);
                if (pos < cap) keys[pos] = key;  // cap: capacity of the binning buffer (redone if exceeded)
            }
    }
}

// ---- K4 ---------------------------------------------------------------------
// Sorting network with ascending comparators only ("flip" bitonic form): for
// k = 2, 4, .., N2 the first step pairs i with i ^ (k - 1), the others with
// i ^ j.  Every comparator puts the minimum at the lower index, so elements past
// n behave as +infinity and are never touched: any n sorts in place.
template <typename Load, typename Store>
__device__ __forceinline__ void sort_network(uint32_t n, Load ld, Store st) {
    uint32_t N2 = 1;
    while (N2 < n) N2 <<= 1;
    for (uint32_t k = 2; k <= N2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t p = threadIdx.x; p < N2 / 2; p += blockDim.x) {
                // p-th pair of this step: lo has bit j clear
                const uint32_t lo = ((p & ~(j - 1)) << 1) | (p & (j - 1));
                const uint32_t hi = (j == (k >> 1)) ? (lo ^ (k - 1)) : (lo | j);
                if (hi < n) {
                    const unsigned long long a = ld(lo), b = ld(hi);
                    if (b < a) {
                        st(lo, b);
                        st(hi, a);
                    }
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ uint32_t tile_len(uint2 r, unsigned long long cap) {
    const unsigned long long hi = r.y < cap ? r.y : cap;
    return hi > r.x ? (uint32_t)(hi - r.x) : 0u;
}

template <int T, int CAP>
__global__ void __launch_bounds__(T) tile_sort_lds_kernel(const uint2* __restrict__ ranges,
                                                         const unsigned long long* __restrict__ keys,
                                                         unsigned long long cap, uint32_t* __restrict__ gid_sorted,
                                                         uint32_t min_exclusive) {
    __shared__ unsigned long long s[CAP];
    const uint2 r = ranges[blockIdx.x];
    const uint32_t n = tile_len(r, cap);
    if (n <= min_exclusive || n > (uint32_t)CAP) return;  // another kernel's size class
    for (uint32_t i = threadIdx.x; i < n; i += T) s[i] = keys[r.x + i];
    __syncthreads();
    sort_network(
        n, [&](uint32_t i) { return s[i]; }, [&](uint32_t i, unsigned long long v) { s[i] = v; });
    for (uint32_t i = threadIdx.x; i < n; i += T) gid_sorted[r.x + i] = (uint32_t)s[i];
}

// Lists longer than the LDS classes: the same network directly on the global keys
// (one workgroup per tile; correct for any length, slow -- real scenes rarely need it).
__global__ void __launch_bounds__(kBinThreads) tile_sort_global_kernel(const uint2* __restrict__ ranges,
                                                                       unsigned long long* __restrict__ keys,
                                                                       unsigned long long cap,
                                                                       uint32_t* __restrict__ gid_sorted,
                                                                       uint32_t min_exclusive) {
    const uint2 r = ranges[blockIdx.x];
    const uint32_t n = tile_len(r, cap);
    if (n <= min_exclusive) return;
    unsigned long long* k = keys + r.x;
    sort_network(
        n, [&](uint32_t i) { return k[i]; }, [&](uint32_t i, unsigned long long v) { k[i] = v; });
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) gid_sorted[r.x + i] = (uint32_t)k[i];
}

// ---- launchers ----------------------------------------------------------------
int bin_chunks(int P, int* chunk) {
    // ~256 chunks (enough workgroups for the chip), each < 65536 Gaussians (16-bit LDS counters)
    int n = (P + 1023) / 1024;
    if (n > 256) n = 256;
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

// K1 + K2: tile counts, ranges, cursors, record bases and the instance count (g.total).
hipError_t launch_bin_count(int P, const GeomState& g, uint32_t gx, uint32_t gy, uint2* ranges, size_t cap,
                            hipStream_t stream) {
    const uint32_t tiles = gx * gy;
    int chunk = 0;
    const int nchunks = bin_chunks(P, &chunk);
    const bool lds = tiles <= kLdsTilesMax;
    const dim3 grid(nchunks), block(kBinThreads);
    hipError_t e = hipMemsetAsync(g.tile_cnt, 0, tiles * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const size_t hist_bytes = lds ? ((tiles + 1) / 2) * sizeof(uint32_t) : 0;
    if (lds)
        hipLaunchKernelGGL(tile_count_kernel<true>, grid, block, hist_bytes, stream, P, chunk, g.rect, g.tiles_touched,
                           tiles, gx, g.tile_cnt, g.chunk_total);
    else
        hipLaunchKernelGGL(tile_count_kernel<false>, grid, block, 0, stream, P, chunk, g.rect, g.tiles_touched, tiles,
                           gx, g.tile_cnt, g.chunk_total);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), block, 0, stream, tiles, g.tile_cnt, ranges, g.tile_cursor, nchunks,
                       g.chunk_total, g.chunk_base, g.total, (unsigned long long)cap);
    return hipGetLastError();
}

// K3: scatter the keys into a binning buffer of capacity `cap` (after launch_bin_count).
hipError_t launch_bin_scatter(int P, const GeomState& g, uint32_t gx, uint32_t gy, const BinningState& b, size_t cap,
                              hipStream_t stream) {
    const uint32_t tiles = gx * gy;
    int chunk = 0;
    const int nchunks = bin_chunks(P, &chunk);
    const bool lds = tiles <= kLdsTilesMax;
    const dim3 grid(nchunks), block(kBinThreads);
    const size_t cur_bytes = lds ? tiles * sizeof(uint32_t) : 0;
    if (lds)
        hipLaunchKernelGGL(tile_scatter_kernel<true>, grid, block, cur_bytes, stream, P, chunk, g.rect,
                           g.tiles_touched, g.depth_key, tiles, gx, g.tile_cursor, g.chunk_base, b.keys,
                           (unsigned long long)cap, g.rec_start, g.rec);
    else
        hipLaunchKernelGGL(tile_scatter_kernel<false>, grid, block, 0, stream, P, chunk, g.rect, g.tiles_touched,
                           g.depth_key, tiles, gx, g.tile_cursor, g.chunk_base, b.keys, (unsigned long long)cap,
                           g.rec_start, g.rec);
    return hipGetLastError();
}

hipError_t launch_tile_sort(uint32_t tiles, const uint2* ranges, const BinningState& b, size_t cap,
                            hipStream_t stream) {
    if (tiles == 0 || cap == 0) return hipSuccess;
    const unsigned long long c = cap;
    hipLaunchKernelGGL((tile_sort_lds_kernel<256, 2048>), dim3(tiles), dim3(256), 0, stream, ranges, b.keys, c,
                       b.gid_sorted, 0u);
    hipLaunchKernelGGL((tile_sort_lds_kernel<512, 8192>), dim3(tiles), dim3(512), 0, stream, ranges, b.keys, c,
                       b.gid_sorted, 2048u);
    hipLaunchKernelGGL(tile_sort_global_kernel, dim3(tiles), dim3(kBinThreads), 0, stream, ranges, b.keys, c,
                       b.gid_sorted, 8192u);
    return hipGetLastError();
}

}  // namespace gsr
