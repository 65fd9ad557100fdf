// binning.hip -- depth pre-sort, tile-touch scan, wave-cooperative instance
// emission, 16-bit tile radix sort and tile ranges.
//
// The reference sorts one 64-bit key (tile << 32 | depth bits) per instance
// with a stable radix sort over 32+log2(tiles) bits (CR/rasterizer_impl.cu:78-126,
// 332-340).  Here the same total order -- (tile, depth, Gaussian index) -- is
// produced in two cheaper sorts:
//   1. a stable 32-bit sort of the P Gaussians by depth bits (ties keep index order),
//   2. instances are emitted in that depth order and stably sorted by tile id only
//      (16 bits while tiles <= 65536: two radix passes instead of six).
// Stability of (2) keeps each tile's list in (depth, index) order, which is
// exactly the reference's order.
#include <cstring>

#include "kernels.h"

#include <rocprim/rocprim.hpp>

namespace gsr {

// Always take the onesweep radix path: rocPRIM's default switches to block sort +
// merge sort up to 2^20 items, which costs 20+ launches at P = 1M.
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 0>;

// ---- 1. depth pre-sort ------------------------------------------------------
size_t depth_sort_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs<SortConfig>(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                    rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr, (size_t)P, 0, 32);
    return bytes;
}

hipError_t depth_sort(GeomState& g, int P, hipStream_t stream) {
    size_t bytes = g.sort_temp_bytes;
    return rocprim::radix_sort_pairs<SortConfig>(g.sort_temp, bytes, g.depth_key, g.depth_key_sorted,
                                     rocprim::counting_iterator<uint32_t>(0), g.gid_by_rank, (size_t)P, 0, 32, stream);
}

// ---- 2. ranked tile counts + inverse permutation, then a 64-bit inclusive scan
__global__ void rank_prep_kernel(int P, const uint32_t* __restrict__ gid_by_rank,
                                 const uint32_t* __restrict__ tiles_touched, uint32_t* __restrict__ tiles_ranked,
                                 uint32_t* __restrict__ rank_of) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P) return;
    const uint32_t gid = gid_by_rank[r];
    tiles_ranked[r] = tiles_touched[gid];
    rank_of[gid] = (uint32_t)r;
}

size_t scan_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (unsigned long long*)nullptr, (size_t)P,
                            rocprim::plus<unsigned long long>());
    return bytes;
}

hipError_t rank_and_scan(GeomState& g, int P, hipStream_t stream) {
    hipLaunchKernelGGL(rank_prep_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, g.gid_by_rank, g.tiles_touched,
                       g.tiles_ranked, g.rank_of);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t bytes = g.scan_temp_bytes;
    return rocprim::inclusive_scan(g.scan_temp, bytes, g.tiles_ranked, g.offsets, (size_t)P,
                                   rocprim::plus<unsigned long long>(), stream);
}

// ---- 3. instance emission ----------------------------------------------------
// One thread per depth rank.  A wave's 64 Gaussians own one contiguous range of
// the emission order; the wave walks it 64 slots at a time, so every store is a
// full coalesced wave store no matter how unevenly the tile counts are spread
// (the reference's thread-per-Gaussian loop writes 1..hundreds of entries per
// thread, CR/rasterizer_impl.cu:108-124).  Each slot finds its owning lane by a
// 6-step binary search over the lanes' exclusive starts (ds_bpermute).
template <typename KeyT>
__global__ void __launch_bounds__(256) duplicate_kernel(int P, const uint32_t* __restrict__ gid_by_rank,
                                                        const unsigned long long* __restrict__ offsets,
                                                        const int* __restrict__ radii, float4* __restrict__ rec,
                                                        uint32_t gx, uint32_t gy, KeyT* __restrict__ keys,
                                                        uint32_t* __restrict__ emit_gid, unsigned long long cap) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    if (r - lane >= P) return;  // whole wave past the end (wave-uniform)
    const bool valid = r < P;
    uint32_t gid = 0, count = 0;
    uint2 rmin = make_uint2(0, 0), rmax = make_uint2(0, 0);
    unsigned long long incl = 0;
    if (valid) {
        gid = gid_by_rank[r];
        incl = offsets[r];
        const int rad = radii[gid];
        if (rad > 0) {
            const float4 v = rec[(size_t)kRecRows * gid];
            get_rect(v.x, v.y, rad, gx, gy, rmin, rmax);
            count = (rmax.y - rmin.y) * (rmax.x - rmin.x);
        }
    }
    const unsigned long long excl = incl - count;
    // first emission index of this Gaussian -> record row 3 (the render backward addresses
    // its per-instance gradient records with it)
    if (count) reinterpret_cast<uint32_t*>(rec + (size_t)kRecRows * gid + 3)[3] = (uint32_t)excl;
    // The wave's ranks are consecutive: its emissions are [E0, E1) with both ends
    // read from the scan (wave-uniform addresses -> scalar loads).
    const int r0 = r - lane;
    const int r_last = min(r0 + 63, P - 1);
    const unsigned long long E0 = r0 == 0 ? 0ull : offsets[r0 - 1];
    const unsigned long long E1 = offsets[r_last];
    const uint32_t total = (uint32_t)(E1 - E0);
    const uint32_t my_start = valid ? (uint32_t)(excl - E0) : total;  // invalid lanes start at the end
    const uint32_t w = rmax.x - rmin.x;

    for (uint32_t base = 0; base < total; base += 64) {
        const uint32_t k = base + lane;
        // largest lane whose start <= k (starts are non-decreasing across lanes)
        int lo = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const int cand = lo + step;
            const uint32_t v = __shfl(my_start, cand & 63);
            if (cand < 64 && v <= k) lo = cand;
        }
        const uint32_t o_start = __shfl(my_start, lo);
        const uint32_t o_w = __shfl(w, lo);
        const uint32_t o_x0 = __shfl(rmin.x, lo);
        const uint32_t o_y0 = __shfl(rmin.y, lo);
        const uint32_t o_gid = __shfl(gid, lo);
        if (k < total && E0 + k < cap) {  // cap: instances the binning buffer holds
            const uint32_t local = k - o_start;
            const uint32_t ty = local / o_w;
            const uint32_t tx = local - ty * o_w;
            const uint32_t tile = (o_y0 + ty) * gx + (o_x0 + tx);
            keys[E0 + k] = (KeyT)tile;
            emit_gid[E0 + k] = o_gid;
        }
    }
}

hipError_t launch_duplicate(int P, const GeomState& g, const int* radii, uint32_t gx, uint32_t gy,
                            const BinningState& b, bool key16, size_t cap, hipStream_t stream) {
    const dim3 grid((P + 255) / 256), block(256);
    if (key16)
        hipLaunchKernelGGL(duplicate_kernel<uint16_t>, grid, block, 0, stream, P, g.gid_by_rank, g.offsets, radii,
                           g.rec, gx, gy, (uint16_t*)b.keys, b.emit_gid, (unsigned long long)cap);
    else
        hipLaunchKernelGGL(duplicate_kernel<uint32_t>, grid, block, 0, stream, P, g.gid_by_rank, g.offsets, radii,
                           g.rec, gx, gy, (uint32_t*)b.keys, b.emit_gid, (unsigned long long)cap);
    return hipGetLastError();
}

// ---- 3b. capacity mode: the slots past the device-side instance count get the
// sentinel tile id `tiles` (it fits in bit_length(tiles) bits and sorts last), so
// the sort can run on a host-known capacity without a host round trip.
template <typename KeyT>
__global__ void pad_keys_kernel(const unsigned long long* __restrict__ total, unsigned long long cap,
                                KeyT* __restrict__ keys, KeyT sentinel) {
    const unsigned long long R = *total;
    for (unsigned long long i = R + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < cap;
         i += (unsigned long long)gridDim.x * blockDim.x)
        keys[i] = sentinel;
}

hipError_t launch_pad_keys(const unsigned long long* total, size_t cap, const BinningState& b, bool key16,
                           uint32_t sentinel, hipStream_t stream) {
    const dim3 grid(512), block(256);
    if (key16)
        hipLaunchKernelGGL(pad_keys_kernel<uint16_t>, grid, block, 0, stream, total, (unsigned long long)cap,
                           (uint16_t*)b.keys, (uint16_t)sentinel);
    else
        hipLaunchKernelGGL(pad_keys_kernel<uint32_t>, grid, block, 0, stream, total, (unsigned long long)cap,
                           (uint32_t*)b.keys, sentinel);
    return hipGetLastError();
}

// ---- 4. stable tile sort over bits [0, bit_length(tiles)) ---------------------
size_t tile_sort_temp_bytes(size_t R, bool key16) {
    size_t bytes = 0;
    if (key16)
        (void)rocprim::radix_sort_pairs<SortConfig>(nullptr, bytes, (const uint16_t*)nullptr, (uint16_t*)nullptr,
                                                    (const uint32_t*)nullptr, (uint32_t*)nullptr, R, 0, 16);
    else
        (void)rocprim::radix_sort_pairs<SortConfig>(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                    (const uint32_t*)nullptr, (uint32_t*)nullptr, R, 0, 32);
    return bytes;
}

hipError_t tile_sort(BinningState& b, size_t R, unsigned end_bit, bool key16, hipStream_t stream) {
    size_t bytes = b.sort_temp_bytes;
    if (key16)
        return rocprim::radix_sort_pairs<SortConfig>(b.sort_temp, bytes, (const uint16_t*)b.keys, (uint16_t*)b.keys_sorted,
                                                     (const uint32_t*)b.emit_gid, b.gid_sorted, R, 0, end_bit, stream);
    return rocprim::radix_sort_pairs<SortConfig>(b.sort_temp, bytes, (const uint32_t*)b.keys, (uint32_t*)b.keys_sorted,
                                                 (const uint32_t*)b.emit_gid, b.gid_sorted, R, 0, end_bit, stream);
}

// ---- 5. per-tile [start, end) (identifyTileRanges, CR/rasterizer_impl.cu:132-164)
// Keys >= tiles are capacity-mode padding (sorted last) and own no range.
template <typename KeyT>
__global__ void finalize_kernel(uint32_t R, uint32_t tiles, const KeyT* __restrict__ keys_sorted,
                                uint2* __restrict__ ranges) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const uint32_t cur = keys_sorted[i];
    if (cur >= tiles) {
        if (i > 0 && keys_sorted[i - 1] < tiles) ranges[keys_sorted[i - 1]].y = i;
        return;
    }
    if (i == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = keys_sorted[i - 1];
        if (cur != prev) {
            ranges[prev].y = i;
            ranges[cur].x = i;
        }
    }
    if (i == R - 1) ranges[cur].y = R;
}

hipError_t launch_finalize(size_t R, uint32_t tiles, const BinningState& b, uint2* ranges, bool key16,
                           hipStream_t stream) {
    const dim3 grid((unsigned)((R + 255) / 256)), block(256);
    if (key16)
        hipLaunchKernelGGL(finalize_kernel<uint16_t>, grid, block, 0, stream, (uint32_t)R, tiles,
                           (const uint16_t*)b.keys_sorted, ranges);
    else
        hipLaunchKernelGGL(finalize_kernel<uint32_t>, grid, block, 0, stream, (uint32_t)R, tiles,
                           (const uint32_t*)b.keys_sorted, ranges);
    return hipGetLastError();
}

}  // namespace gsr
