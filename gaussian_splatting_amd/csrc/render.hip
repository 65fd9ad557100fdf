// render.hip -- per-tile front-to-back alpha blending (forward) and its
// front-to-back gradient pass (backward).
//
// Forward semantics follow renderCUDA (CR/forward.cu:367-513) exactly: the same
// per-pixel skip tests (power > 0, alpha < 1/255), the same early termination
// (T * (1 - alpha) < 1e-4 ends the pixel without adding that Gaussian), and the
// same outputs (colour + T * bg, inverse depth, final T, last contributor).
//
// CDNA4 structure:
//  * forward: one wave64 per half tile (16x8 pixels); lane l owns pixel (l & 7, l >> 3)
//    of each of the half's two 8x8 quadrants ("slots"); the backward: one wave64 per
//    (tile, 256-entry segment) unit with all four quadrants, started from the forward's
//    blend checkpoint;
//  * list entries are staged 64 at a time (one per lane) into LDS as 48-byte
//    splat records; while loading, each entry's alpha >= 1/255 footprint (its
//    box, then the ellipse itself) is tested against the four quadrants (4-bit
//    mask, conservative);
//  * the wave walks only entries whose mask is non-zero (scalar bit scan of a
//    ballot) and, per entry, runs only the slots whose bit is set -- uniform
//    branches, no vector work for culled quadrants;
//  * record reads from LDS are wave-uniform broadcasts (no bank conflicts).
//
// The backward pass walks the list in the same (front-to-back) order,
// recomputing T exactly as the forward did instead of recovering it by division
// as the reference does (CR/backward.cu:553).  The colour "behind" an entry
// enters dL/dalpha only through the dot product with dL/dpixel, so each pixel
// keeps one running scalar gB = dL/dpix . (colour behind) + dL/dinvdepth .
// (inverse depth behind), initialised from the forward's accumulated colour.
// A slot is retired once the walk passes the last contributor of all its pixels
// (n_contrib from the forward).  Per-Gaussian sums over the tile's pixels are
// first summed over the lane's four slots in registers, then over the wave with a
// lane-swap reduce-scatter and DPP row sums -- once per (tile, Gaussian) instance.
// The atomic path (the default) adds those sums into the Gaussian's accumulator row with
// one float atomic per value and instance; the record path writes them with plain stores
// for gauss_reduce and is bitwise reproducible.  The reference issues 10 global float
// atomics per pixel-Gaussian pair (CR/backward.cu:569-609).
#include <cstdlib>

#include "footprint.h"
#include "kernels.h"

#include <algorithm>
#include <atomic>

namespace gsr {

constexpr int kBatch = 64;  // list entries staged per round (one per lane)

// Each lane's tile-list entry of the NEXT batch is loaded during the current batch's walk, so a
// batch's staging waits for one round trip (the splat records) instead of two (entry, then record).
//
// The entry mask the forward leaves for the backward is the blend mask: the quadrants in which some
// pixel blended the entry (set after the batch's walk from one wave-uniform bit per (entry, quadrant)
// evaluation that passed its any-alpha test), each half-tile part OR-ing its own quadrants' bits.  The
// backward evaluates an entry's quadrant only where a pixel can have a gradient term, and the blend mask
// is the tightest superset of those; entries with no blending pixel are neither gathered nor walked by
// the backward.  (r5u, interleaved: 1M@1080p 0.7227 -> 0.7213 ms, 5M@4K 2.222 -> 2.207; the ORs are
// issued once the next batch's loads are in flight -- before its staging they made it wait, r5t.)
// Variants measured and rejected (DESIGN.md "Measured and rejected"; git history keeps their code):
// shared two-wave staging, lane-held entries, the blend bits in one VGPR, software-pipelined LDS reads,
// non-temporal image stores / dL/dpixel loads, an occupancy cap on the backward.

GSR_STAMP_BUFFER(g_st_rfwd);
GSR_STAMP_BUFFER(g_st_rbwd);

__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Staged form of a splat's conic: the exponent is evaluated as
//   power * log2(e) = dx * (A dx + B dy) + C dy^2,  A = -a/2 log2e, B = -b log2e, C = -c/2 log2e
// so the per-pixel cost is five VALU ops and exp2 takes it directly.  The
// coefficients are computed once per list entry while staging (one lane each).
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float4 stage_conic(float4 v0, float4 v1, uint32_t qm) {
    return make_float4(-0.5f * kLog2e * v0.z, -kLog2e * v0.w, -0.5f * kLog2e * v1.x, __uint_as_float(qm));
}

// The reference's two skip tests (power > 0, alpha < 1/255; CR/forward.cu:466-472) folded into
// one value: the exponent is forced to -inf when positive so alpha becomes 0, and alpha below
// 1/255 is zeroed.  Returns alpha for a contributing pixel, 0 otherwise; G = exp(power).
__device__ __forceinline__ float splat_alpha(float p2, float opacity, float& G) {
    G = __builtin_amdgcn_exp2f(p2);  // raw v_exp_f32 (+inf for a large positive p2: masked below)
    const float alpha = fminf(0.99f, opacity * G);
    return ((p2 <= 0.f) & (alpha >= 1.0f / 255.0f)) ? alpha : 0.f;  // one mask, one select
}

// ---------------------------------------------------------------------------
// Per-pixel state is arithmetic, not boolean: Tl is the live transmittance and
// drops to 0 when the pixel terminates (CR/forward.cu:477-482); Tc is T after the
// pixel's last contributor, which is the reference's final_T whether or not the pixel
// terminated (skipped entries leave T alone).  A finished pixel therefore blends with weight 0
// without any mask bookkeeping, and the only wave-level decisions are "does any
// lane of this slot blend this splat" and "is any pixel of this slot still live".
// SGPR budget of the forward: at .sgpr_count 82-96 the hardware admits 7 one-wave workgroups per
// SIMD, at <= 80 eight (MI355X_MICROARCH.md "Residency"); the VGPRs (61) allow eight.
// (r4b: render_fwd 199-200 -> 195-197 us; 8 SGPRs spill to VGPR lanes, prologue only)
#define GSR_FWD_OCCUPANCY __attribute__((amdgpu_num_sgpr(80)))
// One wave per PART of a tile: NQ = 4 quadrants (the whole 16x16 tile) or NQ = 2 (its top or
// bottom half).  Each lane owns one pixel in each of the part's NQ quadrants ("slots").  With
// half tiles the 8160 tiles of a 1080p view become 16320 waves of half the blend work each, so
// the launch no longer ends with SIMDs finishing their second whole tile alone; the price is
// that both halves stage the same entries.  Grid: groups of 8 consecutive tiles x NPART parts,
// block b -> tile 8 (b / (8 NPART)) + b % 8, part (b / 8) % NPART: the parts of a tile sit on
// the same XCD (blocks are dealt round-robin over the 8 XCDs) and share its L2.
// CENSUS (diagnostic instantiation, gsr_census_set): counts the work the blend does -- see
// include/gsr.h "Census" for the counters -- with wave-uniform scalar counters, one atomic per wave.
// Reachable-prefix sort (binning.hip K4): only entries [0, sorted_len) of a long list are in
// order.  A part that reaches sorted_len with pixels still blending files its tile for a redo
// (one flag per tile, so a tile is listed once) and stops without writing anything: after this
// launch the tile's whole list is sorted and both parts render it again from the start
// (render_fwd_redo_kernel).  The forward walks ~7% of a 4K tile's list and ~34% of a 1080p
// one, so with a prefix of 1024 entries a redo is rare.

// The render kernels' per-batch LDS hand-offs (staged entries, the backward's reduced sums).  A render
// unit is one wave, whose LDS accesses complete in order, so the hand-off needs only the compiler kept
// from moving LDS accesses across it -- __syncthreads' workgroup fence also makes the wave wait for
// every store it has in flight (the backward's gradient records, the forward's entry masks and
// checkpoints) before the next batch's loads.
__device__ __forceinline__ void unit_sync() {
    wave_lds_sync();
}

struct FwdLds {
    float4 xy[kBatch], cq[kBatch], col[kBatch];
};
__device__ __forceinline__ FwdLds& fwd_lds() {
    __shared__ FwdLds s;
    return s;
}

template <int NQ, bool CENSUS>
__device__ __forceinline__ void render_fwd_tile(const RenderFwdArgs& a, const uint32_t tile, const int part) {
  {
    constexpr uint32_t kPartMask = (1u << NQ) - 1u;
    constexpr int NPART = 4 / NQ;
    const uint32_t tiles = a.gx * a.gy;
    const int qbase = part * NQ;  // first quadrant of this part
    const int tile_x0 = (int)(tile % a.gx) * kTile, tile_y0 = (int)(tile / a.gx) * kTile;
    const int lane = threadIdx.x & (kWave - 1);
    const int lx = lane & 7, ly = lane >> 3;
    const float pxf0 = (float)(tile_x0 + lx), pyf0 = (float)(tile_y0 + ly);  // this lane's pixel in quadrant 0
    if (part == 0) {
        GSR_STAMP(g_st_rfwd, tile, 0);
        GSR_STAMP_HWID(g_st_rfwd, tile);
        GSR_STAMP_RT(g_st_rfwd, tile, 4);
    }

    // (one LDS block whatever NQ: the hybrid launch's half-tile and quadrant units share it)
    FwdLds& L = fwd_lds();
    auto& s_xy = L.xy;  // (x, y, o, 1/z)
    auto& s_cq = L.cq;  // (A, B, C, quads)
    auto& s_col = L.col;  // rgb

    float Tl[NQ], Tc[NQ], C0[NQ], C1[NQ], C2[NQ], D[NQ];
    uint32_t last[NQ];
    uint32_t alive = 0;  // wave-uniform: slots with at least one pixel still blending
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = qbase + k;
        const int px = tile_x0 + (q & 1) * 8 + lx, py = tile_y0 + (q >> 1) * 8 + ly;
        Tl[k] = (px < a.W && py < a.H) ? 1.f : 0.f;
        Tc[k] = 1.f;
        C0[k] = C1[k] = C2[k] = D[k] = 0.f;
        last[k] = 0;
        if (__any(Tl[k] > 0.f)) alive |= 1u << k;
    }

    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    const int ns = a.sorted_len ? min(n, (int)a.sorted_len[tile]) : n;  // entries in order
    unsigned long long c_staged = 0, c_eval = 0, c_alpha = 0, c_blend = 0, c_idle = 0;  // CENSUS only
    uint32_t ent_next = lane < ns ? a.gid_sorted[range.x + lane] : 0u;  // the next batch's entry
    // the previous batch's blend bits, OR-ed into its entries once this batch's loads are in flight
    // (vmcnt counts stores too: issued before the next staging, the ORs made it wait for them)
    uint32_t pend_bq = 0;
    int pend_b0 = 0;
    for (int b0 = 0; b0 < ns && alive; b0 += kBatch) {
        if (CENSUS) c_staged += (unsigned long long)min(kBatch, ns - b0);
        uint32_t qm = 0;
        if (b0 + lane < ns) {
            // Gaussian << 4 | quadrant mask (the other part may be OR-ing its mask bits into the entry:
            // only the Gaussian bits are used)
            const uint32_t gid = ent_next >> kEntryMaskBits;
            const float4* rec = a.rec + (size_t)kRecRows * gid;
            const float4 v0 = rec[0], v1 = rec[1], v2 = rec[2];
            s_xy[lane] = make_float4(v0.x, v0.y, v1.y, v1.z);
            s_col[lane] = v2;
            // this part's quadrants only; the backward (which visits only staged entries) gets every
            // part's blend bits OR-ed into the entry K4 wrote with clear mask bits.  A part that stopped
            // before an entry leaves its bits clear there: its pixels all ended earlier, so the
            // backward has retired those slots by then (slot limits from n_contrib).
            qm = quad_bits_exact(v0, v1, v2, tile_x0, tile_y0, kPartMask << qbase);
            s_cq[lane] = stage_conic(v0, v1, qm >> qbase);
        }
        if (b0 + kBatch + lane < ns) ent_next = a.gid_sorted[range.x + b0 + kBatch + lane];
        unit_sync();
        if (pend_bq)  // (the previous batch's bits: see above)
            __hip_atomic_fetch_or(a.gid_sorted + range.x + pend_b0 + lane, pend_bq, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        // Blend checkpoint (gsr_common.h): the state before entry b0, stored after this batch's
        // loads have landed.  vmcnt counts stores too, so stores issued ahead of the loads would
        // make the staging wait for them; here they drain while the batch blends.  A part writes
        // its own quadrants' slots while it is alive: a backward slot that reaches past b0 has a
        // pixel that blended past b0, so its part was alive here.
        if (b0 > 0 && (b0 & (kCkStride - 1)) == 0) {  // uniform
            float* ck = a.ckpt + (size_t)((range.x + (uint32_t)b0) / kCkStride) * kCkFloats + lane;
#pragma unroll
            for (int k = 0; k < NQ; k++) {
                const int q = qbase + k;
                ck[(0 * 4 + q) * 64] = Tl[k];
                ck[(1 * 4 + q) * 64] = C0[k];
                ck[(2 * 4 + q) * 64] = C1[k];
                ck[(3 * 4 + q) * 64] = C2[k];
                ck[(4 * 4 + q) * 64] = D[k];
            }
        }
        unsigned long long todo = __ballot((qm >> qbase) & kPartMask);
        // bit j of blend[k]: some pixel of quadrant k blended entry j (one 64-bit mask per quadrant in
        // SGPRs; under the 80-SGPR budget those spill to VGPR lanes)
        unsigned long long blend[NQ];
#pragma unroll
        for (int k = 0; k < NQ; k++) blend[k] = 0ull;
        while (todo && alive) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const float4 xy = s_xy[j], cq = s_cq[j], col = s_col[j];
            const uint32_t m = uniform_u32(__float_as_uint(cq.w)) & alive;
            const uint32_t pos1 = (uint32_t)(b0 + j + 1);
#pragma unroll
            for (int k = 0; k < NQ; k++) {
                if (!(m & (1u << k))) continue;  // uniform: footprint misses this quadrant
                const int q = qbase + k;
                const float dx = xy.x - (pxf0 + (float)((q & 1) * 8)), dy = xy.y - (pyf0 + (float)((q >> 1) * 8));
                const float p2 = dx * (cq.x * dx + cq.y * dy) + cq.z * dy * dy;
                float G;
                const float alpha = splat_alpha(p2, xy.z, G);
                const float w0 = alpha * Tl[k];  // > 0 iff this pixel blends the splat
                if (CENSUS) {
                    c_eval++;
                    c_alpha += (unsigned long long)__popcll(__ballot(w0 > 0.f));
                    const unsigned long long bl = __ballot(w0 > 0.f && Tl[k] * (1.f - alpha) >= 0.0001f);
                    c_blend += (unsigned long long)__popcll(bl);
                    c_idle += bl ? 0ull : 1ull;
                }
                if (!__any(w0 > 0.f)) continue;  // uniform
                blend[k] |= 1ull << j;
                const float test_T = Tl[k] * (1.f - alpha);
                const bool term = test_T < 0.0001f;  // live pixel: ends it, splat not added
                const float w = term ? 0.f : w0;
                const bool blended = w > 0.f;
                Tl[k] = term ? 0.f : test_T;
                C0[k] += col.x * w;
                C1[k] += col.y * w;
                C2[k] += col.z * w;
                D[k] += xy.w * w;
                last[k] = blended ? pos1 : last[k];
                Tc[k] = blended ? test_T : Tc[k];  // T after the last contributor = final_T
                // the slot dies when its last live pixel terminated just now (one compare; guarding
                // it with "some pixel terminated here" cost two VALU to materialise the guard)
                if (!__any(Tl[k] > 0.f)) alive &= ~(1u << k);
            }
        }
        {
            // OR-ed into the entry K4 wrote with clear mask bits (the other part adds its own) during the next
            // batch, or after the walk
            uint32_t bq = 0;
#pragma unroll
            for (int k = 0; k < NQ; k++) bq |= (uint32_t)((blend[k] >> lane) & 1ull) << (qbase + k);
            pend_bq = b0 + lane < ns ? bq : 0u;
            pend_b0 = b0;
        }
        unit_sync();
#ifdef GSR_STAMPS
        if (lane == 0 && part == 0) g_st_rfwd[(size_t)tile * kStampSlots + 3] = (unsigned long long)(b0 + kBatch);
#endif
    }
    if (pend_bq)  // the last walked batch's bits
        __hip_atomic_fetch_or(a.gid_sorted + range.x + pend_b0 + lane, pend_bq, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    if (CENSUS && lane == 0) {
        atomicAdd(&a.census[0], c_staged);
        atomicAdd(&a.census[1], c_eval);
        atomicAdd(&a.census[2], c_alpha);
        atomicAdd(&a.census[3], c_blend);
        atomicAdd(&a.census[9], c_idle);
    }
    if (ns < n && alive) {  // uniform: the sorted prefix ran out with pixels still blending
        if (lane == 0 && atomicOr(&a.redo_flag[tile], 1u) == 0u) a.redo_list[atomicAdd(a.redo_cnt, 1u)] = tile;
        return;
    }
    if (part == 0) {
        GSR_STAMP(g_st_rfwd, tile, 1);
        GSR_STAMP_RT(g_st_rfwd, tile, 5);
        GSR_STAMP_VAL(g_st_rfwd, tile, 2, n);
    }
    const size_t N = (size_t)a.W * a.H, NT = (size_t)tiles * 256;
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = qbase + k;
        const int px = tile_x0 + (q & 1) * 8 + lx, py = tile_y0 + (q >> 1) * 8 + ly;
        if (px < a.W && py < a.H) {
            const size_t pix = (size_t)py * a.W + px, t = tile_px(tile, q, lane);
            // the reference's final_T is T after the pixel's last contributor: entries after it
            // either do not blend (T unchanged) or end the pixel without blending
            const float T = Tc[k];
            a.img.final_T[t] = T;
            a.img.n_contrib[t] = last[k];
            a.img.accum[t] = C0[k];
            a.img.accum[NT + t] = C1[k];
            a.img.accum[2 * NT + t] = C2[k];
            a.img.accum[3 * NT + t] = D[k];
            a.out_color[pix] = C0[k] + T * a.bg[0];
            a.out_color[N + pix] = C1[k] + T * a.bg[1];
            a.out_color[2 * N + pix] = C2[k] + T * a.bg[2];
            a.out_invdepth[pix] = D[k];
        }
    }

    // The tile's limit for the backward: its largest n_contrib.  With two parts the second part
    // to finish combines them: each adds (1 << 62) + (its limit << 31 part) to the tile's join
    // word (zeroed by K2), so the second add returns the first part's limit -- no fence needed.
    uint32_t lm = last[0];
#pragma unroll
    for (int k = 1; k < NQ; k++) lm = max(lm, last[k]);
    lm = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(lm), 63);  // DPP max, no ds_bpermute chain
    if (NPART == 2) {
        unsigned long long old = 0;
        if (lane == 0)
            old = atomicAdd(&a.tile_join[tile], (1ull << 62) + ((unsigned long long)lm << (31 * part)));
        old = __shfl(old, 0);
        if ((old >> 62) == 0) return;  // the other part finishes the tile
        lm = max(lm, (uint32_t)((old >> (31 * (part ^ 1))) & 0x7fffffffull));
    } else if (NPART == 4) {
        // quadrant units: the join word's low half is the max of the limits, its high half the count
        // of parts done.  Each part's max returns before it counts itself, so the part that counts 3
        // finds every other part's limit in the max (one L2, atomics in arrival order).
        uint32_t* jw = reinterpret_cast<uint32_t*>(&a.tile_join[tile]);
        uint32_t done = 0;
        if (lane == 0) {
            (void)atomicMax(&jw[0], lm);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the max has been performed before the count
            done = atomicAdd(&jw[1], 1u);
            if (done == 3u) lm = max(lm, atomicMax(&jw[0], 0u));
        }
        done = (uint32_t)__shfl((int)done, 0);
        if (done != 3u) return;  // another part finishes the tile
        lm = (uint32_t)__shfl((int)lm, 0);
    }
    // The backward's work list: units (tile, k * seg_ck) for the full segments of S entries below
    // the limit, then the last partial segment into one of four lists by length quarter.
    // Lanes 0 and 1 append in parallel (separate counters, gsr_common.h "work list").
    const uint32_t S = (uint32_t)a.seg_ck * kCkStride;
    const uint32_t nf = lm / S, rem = lm % S;
    const uint32_t shard = tile % kUnitShards;
    const uint32_t b = min(3u, (uint32_t)(((unsigned long long)(S - rem) * 4) / S));  // longest -> 0
    uint32_t base = 0;
    if ((lane == 0 && nf) || (lane == 1 && rem)) {
        const uint32_t list = lane == 0 ? 0u : 1u + b;
        base = atomicAdd(&a.unit_cnt[(list * kUnitShards + shard) * kUnitCntStride], lane == 0 ? nf : 1u);
    }
    const uint32_t fbase = __shfl(base, 0);
    uint2* full = a.unit_full + (size_t)shard * a.full_cap;
    for (uint32_t k = lane; k < nf; k += kWave) full[fbase + k] = make_uint2(tile, k * (uint32_t)a.seg_ck);
    if (lane == 1 && rem)
        a.unit_part[((size_t)b * kUnitShards + shard) * unit_part_cap(tiles) + base] =
            make_uint2(tile, nf * (uint32_t)a.seg_ck);
  }
}

// The forward launch's first fill_blocks blocks zero RenderFwdArgs::fill (the atomic backward's
// accumulator rows and touched bits) beside the render waves and exit; the render blocks count from
// there (fill_blocks is a multiple of 8, so a tile's blocks keep their XCD).
__device__ __forceinline__ bool fwd_fill_block(const RenderFwdArgs& a, uint32_t& bid) {
    if (blockIdx.x < a.fill_blocks) {  // uniform
        const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, stride = a.fill_blocks * blockDim.x;
        const uint32_t cut = *a.zcut, words = (uint32_t)touched_words(a.n_gauss);
        for (uint32_t i = tid; i < words; i += stride) a.touched[i] = 0u;
        typedef float v4f __attribute__((ext_vector_type(4)));
        for (uint32_t g = tid; g < a.n_gauss; g += stride) {
            const uint32_t dk = a.depth_key[g];
            if (dk != 0xffffffffu && (cut == kZCutNone || zbin(dk) <= cut)) {  // visible, in front of the cut
                v4f* row = reinterpret_cast<v4f*>(a.acc + (size_t)g * kAccRow4);
#pragma unroll
                for (int k = 0; k < kAccRow4; k++) __builtin_nontemporal_store((v4f){0.f, 0.f, 0.f, 0.f}, row + k);
            }
        }
        return true;
    }
    bid = blockIdx.x - a.fill_blocks;
    return false;
}

template <int NQ, bool CENSUS>
__global__ void __launch_bounds__(64) GSR_FWD_OCCUPANCY render_fwd_kernel(RenderFwdArgs a) {
    constexpr int NPART = 4 / NQ;
    uint32_t bid = 0;
    if (fwd_fill_block(a, bid)) return;
    const uint32_t tile = (bid / (8 * NPART)) * 8 + bid % 8;
    const int part = NPART == 1 ? 0 : (int)((bid / 8) % NPART);
    if (bid == 0 && threadIdx.x == 0) *a.seg_ck_out = (uint32_t)a.seg_ck;  // for the backward
    if (tile >= a.gx * a.gy) return;
    render_fwd_tile<NQ, CENSUS>(a, tile, part);
}

// Hybrid grid: half-tile units for the first tiles in dispatch order, quadrant units (one wave per 8x8
// quadrant, four per tile) for the last kFwdTailQuadsPct percent of the tiles.  A launch ends about
// one unit's duration after its last units start, and a half tile's cost (set by how soon its pixels
// saturate) is not known in advance, so the units dispatched last are made short instead: the tail
// shrinks, for ~2x the staging work on those tiles only.
constexpr uint32_t kFwdTailQuadsPct = 10;
__global__ void __launch_bounds__(64) GSR_FWD_OCCUPANCY render_fwd_hybrid_kernel(RenderFwdArgs a) {
    uint32_t bid = 0;
    if (fwd_fill_block(a, bid)) return;
    if (bid == 0 && threadIdx.x == 0) *a.seg_ck_out = (uint32_t)a.seg_ck;  // for the backward
    const uint32_t half_tiles = a.half_tiles;
    const uint32_t hb = 2 * half_tiles;  // blocks of the half-tile region (half_tiles: a multiple of 8)
    if (bid < hb) {
        const uint32_t tile = (bid / 16) * 8 + bid % 8;
        render_fwd_tile<2, false>(a, tile, (int)((bid / 8) % 2));
    } else {
        const uint32_t b = bid - hb;
        const uint32_t tile = half_tiles + (b / 32) * 8 + b % 8;
        if (tile >= a.gx * a.gy) return;
        render_fwd_tile<1, false>(a, tile, (int)((b / 8) % 4));
    }
}

// The redo of the tiles render_fwd_kernel filed (their whole lists sorted since, by
// tile_sort_full_kernel): NPART blocks per tile, persistent over the redo list.
template <int NQ, bool CENSUS>
__global__ void __launch_bounds__(64) GSR_FWD_OCCUPANCY render_fwd_redo_kernel(RenderFwdArgs a) {
    constexpr int NPART = 4 / NQ;
    const uint32_t cnt = a.redo_cnt[0];
    for (uint32_t i = blockIdx.x / NPART; i < cnt; i += gridDim.x / NPART)
        render_fwd_tile<NQ, CENSUS>(a, a.redo_list[i], (int)(blockIdx.x % NPART));
}

__global__ void untile_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int W, int H, uint32_t gx) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const uint32_t tile = blockIdx.y * gx + blockIdx.x;
    const int q = ((y & 15) >> 3) * 2 + ((x & 15) >> 3), lane = (y & 7) * 8 + (x & 7);
    dst[(size_t)y * W + x] = src[tile_px(tile, q, lane)];
}

hipError_t launch_untile(const uint32_t* src, uint32_t* dst, int W, int H, uint32_t gx, hipStream_t stream) {
    const uint32_t gy = (H + kTile - 1) / kTile;
    if (gx == 0 || gy == 0) return hipSuccess;
    hipLaunchKernelGGL(untile_kernel, dim3(gx, gy), dim3(256), 0, stream, src, dst, W, H, gx);
    return hipGetLastError();
}

hipError_t launch_render_fwd_redo(const RenderFwdArgs& a, hipStream_t stream, int quads) {
    if (a.gx * a.gy == 0) return hipSuccess;
    constexpr uint32_t kTilesPerPass = 256;  // persistent: each block walks the list in steps of this
    if (a.census)
        hipLaunchKernelGGL((render_fwd_redo_kernel<2, true>), dim3(2 * kTilesPerPass), dim3(kWave), 0, stream, a);
    else if (quads == 4)
        hipLaunchKernelGGL((render_fwd_redo_kernel<4, false>), dim3(kTilesPerPass), dim3(kWave), 0, stream, a);
    else
        hipLaunchKernelGGL((render_fwd_redo_kernel<2, false>), dim3(2 * kTilesPerPass), dim3(kWave), 0, stream, a);
    return hipGetLastError();
}

// Quadrants per forward wave: 2 (half tiles) or 4 (whole tiles; the "fwd_quads" option, api.hip).
hipError_t launch_render_fwd(const RenderFwdArgs& a, hipStream_t stream, int quads) {
    const uint32_t tiles = a.gx * a.gy;
    if (tiles == 0) return hipSuccess;
    const uint32_t groups = (tiles + 7) / 8;
    // the current device's CU count, read once per device (the hybrid grid below is sized by it)
    static std::atomic<uint32_t> cu_count[64];
    uint32_t cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        cus = cu_count[dev].load(std::memory_order_relaxed);
        if (cus == 0) {
            int n = 256;
            (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
            cus = (uint32_t)max(1, n);
            cu_count[dev].store(cus, std::memory_order_relaxed);
        }
    }
    const uint32_t fb = a.fill_blocks;  // (fill blocks first: a multiple of 8)
    if (quads == 2 && !a.census && tiles >= 16 && tiles <= 64 * cus) {
        // the last tiles (whole groups of 8) as quadrant units: kFwdTailQuadsPct percent of them, at most
        // ~0.4 groups per CU.  Measured (profiles/r04/r4k, r4l): 1M@1080p render_fwd 194 -> 188 us, 500k@1080p
        // 217 -> 212 us; at 5M@4K (32400 tiles, ~8 rounds of half tiles per wave slot) the tail is a smaller
        // share and the quadrants' extra staging cost more than it saves (+3..8 us), hence the tile bound.
        const uint32_t qgroups = min((cus * 2) / 5 + 1, max(1u, groups * kFwdTailQuadsPct / 100u));
        const uint32_t hgroups = groups - qgroups;
        RenderFwdArgs h = a;
        h.half_tiles = hgroups * 8;
        hipLaunchKernelGGL(render_fwd_hybrid_kernel, dim3(fb + hgroups * 16 + qgroups * 32), dim3(kWave), 0, stream, h);
    } else if (a.census)
        hipLaunchKernelGGL((render_fwd_kernel<2, true>), dim3(fb + groups * 16), dim3(kWave), 0, stream, a);
    else if (quads == 4)
        hipLaunchKernelGGL((render_fwd_kernel<4, false>), dim3(fb + groups * 8), dim3(kWave), 0, stream, a);
    else
        hipLaunchKernelGGL((render_fwd_kernel<2, false>), dim3(fb + groups * 16), dim3(kWave), 0, stream, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ATOMIC ("bwd_atomic" option): each entry's ten reduced sums are added straight into its Gaussian's
// accumulator row (GeomState::acc, 64 B) with float atomics and the Gaussian's touched bit is set,
// instead of a 48-byte record at the instance's emission index for gauss_reduce to sum: no record
// writes, no record-start gathers, no gauss_reduce.  The flush compacts the batch's written entries
// into an LDS list and issues one wave instruction per FOUR entries -- lane 16k + v adds value v
// (< 10) of listed entry k -- so an instruction touches four 64-byte rows, the shape the memory-side
// atomic units take at full rate (MI355X_MICROARCH.md "Global float atomics": 64 lanes in 64 rows
// run ~17x slower).  The summation order over a Gaussian's instances then follows the hardware, so
// the result is not bitwise reproducible; the record path (bwd_atomic=0) is.  The default since r5f:
// 1M@1080p 0.7335 -> 0.7320 ms, 5M@4K 2.328 -> 2.224 ms (gauss_reduce gone; profiles/r05/r5f).
template <bool CENSUS, bool STRIDED, bool ATOMIC>
__global__ void __launch_bounds__(64) render_bwd_kernel(RenderBwdArgs a) {
  {
    // One wave per unit = (tile, segment): the entries [start, end) of the tile's list, start a
    // multiple of the checkpoint stride.  Units come longest first (bwd_units_kernel), so the
    // dispatcher deals equal-sized pieces of work round-robin over the SIMDs and the short ones
    // fill the slots that free up last -- no tile's full list ever sits on one SIMD.
    if (blockIdx.x == 0 && threadIdx.x < kLiveShards && a.live_count)  // gauss_reduce appends
        a.live_count[threadIdx.x * kLiveCntStride] = 0u;
    if (blockIdx.x < a.fill_blocks) {  // uniform: a fill block (RenderBwdArgs::fill)
        zero_fill_part(a.fill, (unsigned long long)blockIdx.x * kWave + threadIdx.x,
                       (unsigned long long)a.fill_blocks * kWave);
        return;
    }
    static_assert(kUnitLists * kUnitShards <= kWave, "one lane per list counter");
    constexpr int nl = kUnitLists * kUnitShards;
    // All 40 list counters in one vector load and an inclusive DPP scan (once per block)
    const uint32_t incl = wave_incl_sum(threadIdx.x < nl ? a.unit_cnt[threadIdx.x * kUnitCntStride] : 0u);
    // STRIDED (launch_render_bwd picks it when the worst-case grid is far larger than the tile count):
    // kBwdGridTiles blocks per tile, each taking units i, i + G, ... -- the grid sized for the shortest
    // segments launches ~10x more blocks than there are units at 5M@4K, each a counter load before it
    // can exit (render_bwd 882 -> 803-833 us, r4ad); at 1080p (~2.5x) the one-unit grid stays.
    for (uint32_t i = blockIdx.x - a.fill_blocks;; i += gridDim.x - a.fill_blocks) {
    uint2 unit;
    {  // full segments first, then the partial ones, longest quarter first; shards in order:
        // a ballot over the scanned counters finds the list holding unit i
        const int lane = threadIdx.x;
        const int l = __popcll(__ballot(lane < nl && incl <= i));  // lists wholly before unit i
        if (l >= nl) return;  // past the lists (the grid is sized for the worst case)
        const uint32_t before = l ? (uint32_t)__builtin_amdgcn_readlane((int)incl, l - 1) : 0u;
        const uint32_t k = i - before;
        if (l < kUnitShards)
            unit = a.unit_full[(size_t)l * a.full_cap + k];
        else
            unit = a.unit_part[(size_t)(l - kUnitShards) * unit_part_cap(a.gx * a.gy) + k];
    }
    const uint32_t tile = unit.x;
    const int start = (int)unit.y * kCkStride;
    const int tile_x0 = (int)(tile % a.gx) * kTile, tile_y0 = (int)(tile / a.gx) * kTile;
    // (STRIDED: opaque to the compiler, so that lane-derived constants are formed per unit rather than
    // hoisted out of the unit loop and held in registers across it: 86 VGPRs instead of 98)
    int lane_o = threadIdx.x;
    if (STRIDED) asm volatile("" : "+v"(lane_o));
    const int lane = lane_o;
    const int lx = lane & 7, ly = lane >> 3;
    const float pxf0 = (float)(tile_x0 + lx), pyf0 = (float)(tile_y0 + ly);  // this lane's pixel in quadrant 0

    __shared__ float4 s_xy[kBatch], s_cq[kBatch], s_col[kBatch];  // as in the forward
    // per entry: the 10 reduced sums (r8, r9 in 2 parts), three float4 planes indexed by entry like the
    // staged rows, so a reduction's store address is the entry's row offset (already scalar for the
    // row reads) plus a per-lane constant (an [entry][3] layout cost a quarter-rate v_mad_u64_u32)
    __shared__ float4 s_acc[3][kBatch];
    __shared__ uint32_t s_wgid[ATOMIC ? kBatch : 1], s_wj[ATOMIC ? kBatch : 1];  // ATOMIC: written entries' Gaussian, slot
    GSR_STAMP(g_st_rbwd, blockIdx.x, 0);
    GSR_STAMP_HWID(g_st_rbwd, blockIdx.x);
    GSR_STAMP_RT(g_st_rbwd, blockIdx.x, 4);

    const uint2 range = a.ranges[tile];
    const size_t N = (size_t)a.W * a.H;
    float T[4], gB[4], g0[4], g1[4], g2[4], gi[4];
    int nc[4];
    // Every slot's pixel state is loaded with no branch in between (an outside pixel reads a
    // clamped, valid address and is zeroed afterwards), so all the loads are in flight at once.
    float c0[4], c1[4], c2[4], cd[4], fT[4], k0[4], k1[4], k2[4], k3[4], k4[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int px = min(tile_x0 + (q & 1) * 8 + lx, a.W - 1), py = min(tile_y0 + (q >> 1) * 8 + ly, a.H - 1);
        const size_t pix = (size_t)py * a.W + px, t = tile_px(tile, q, lane), NT = (size_t)a.gx * a.gy * 256;
        nc[q] = (int)a.img.n_contrib[t];
        g0[q] = a.dL_dpix[pix];
        g1[q] = a.dL_dpix[N + pix];
        g2[q] = a.dL_dpix[2 * N + pix];
        gi[q] = a.dL_dinvdepth ? a.dL_dinvdepth[pix] : 0.f;
        c0[q] = a.img.accum[t];
        c1[q] = a.img.accum[NT + t];
        c2[q] = a.img.accum[2 * NT + t];
        cd[q] = a.img.accum[3 * NT + t];
        fT[q] = a.img.final_T[t];
        // blend state at `start`: the forward's checkpoint (gsr_common.h), or the empty state
        const float* ck = a.ckpt + (size_t)((range.x + (uint32_t)start) / kCkStride) * kCkFloats + lane;
        const bool has_ck = start > 0;
        k0[q] = has_ck ? ck[(0 * 4 + q) * 64] : 1.f;
        k1[q] = has_ck ? ck[(1 * 4 + q) * 64] : 0.f;
        k2[q] = has_ck ? ck[(2 * 4 + q) * 64] : 0.f;
        k3[q] = has_ck ? ck[(3 * 4 + q) * 64] : 0.f;
        k4[q] = has_ck ? ck[(4 * 4 + q) * 64] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int px = tile_x0 + (q & 1) * 8 + lx, py = tile_y0 + (q >> 1) * 8 + ly;
        const bool in = px < a.W && py < a.H;
        nc[q] = in ? nc[q] : 0;
        g0[q] = in ? g0[q] : 0.f;
        g1[q] = in ? g1[q] : 0.f;
        g2[q] = in ? g2[q] : 0.f;
        gi[q] = in ? gi[q] : 0.f;
        T[q] = k0[q];
        // dL/dpix . (what the forward accumulated from `start` on) + the background term of
        // dL/dalpha (CR/backward.cu:587-590); shrinks to "behind this entry" as the walk proceeds
        gB[q] = in ? g0[q] * (c0[q] - k1[q]) + g1[q] * (c1[q] - k2[q]) + g2[q] * (c2[q] - k3[q]) +
                         gi[q] * (cd[q] - k4[q]) + fT[q] * (a.bg[0] * g0[q] + a.bg[1] * g1[q] + a.bg[2] * g2[q])
                   : 0.f;
    }
    // Per-slot limits: entries at positions >= slim[q] reach no pixel of slot q (the forward
    // stopped all of them earlier), so the slot is skipped from there on.
    int slim[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        slim[q] = __builtin_amdgcn_readlane((int)wave_incl_max((uint32_t)nc[q]), 63);  // DPP max over the wave
    }
    const int limit = max(max(slim[0], slim[1]), max(slim[2], slim[3]));
    const int end = min(limit, start + (int)uniform_u32(*a.seg_ck) * kCkStride);  // the forward's segments
    uint32_t live = 0;     // slots still reachable at the current position (uniform)
    int next_lim = limit;  // smallest slot limit among live slots
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (slim[q] > start) {
            live |= 1u << q;
            next_lim = min(next_lim, slim[q]);
        }
    // where this lane's part of the reduce-scatter lands in s_acc (see below): in each 16-lane
    // row, lane 0 holds a sum of w0, lane 8 one of w1, lane 15 a row partial of r8 / r9
    const int row = lane >> 4, slot_k = ((row & 1) << 1) | (row >> 1), li = lane & 15;
    const bool hi8 = (lane & 8) != 0, acc_wr = li == 0 || li == 8 || li == 15, acc_h4 = li == 15;
    const int acc_off = li == 0 ? slot_k : li == 8 ? 4 + slot_k : 8 + row;
    const int acc_lane = (acc_off >> 2) * (4 * kBatch) + (acc_off & 3);  // float offset in s_acc, entry 0

    const uint32_t ttx = tile % a.gx, tty = tile / a.gx;
    unsigned long long c_staged = 0, c_eval = 0, c_alpha = 0, c_red = 0, c_idle = 0;  // CENSUS only
    // The ten per-entry sums stay zero between entries (reset after each reduction), so an entry
    // whose first quadrants are inactive does not materialise zeros (10 VALU) before accumulating.
    uint32_t ent_next = start + lane < end ? a.gid_sorted[range.x + start + lane] : 0u;  // the next batch's entry
    for (int b0 = start; b0 < end; b0 += kBatch) {
        const bool has = b0 + lane < end;
        if (CENSUS) c_staged += (unsigned long long)min(kBatch, end - b0);
        uint32_t qm = 0, e = 0;
        float ca = 0.f, cb = 0.f, cc = 0.f, o = 0.f;  // this lane's entry: raw conic and opacity, for the flush
        if (has) {
            // Gaussian << 4 | quadrant mask (loaded during the previous batch)
            const uint32_t ent = ent_next;
          if (ent & kEntryMask) {  // (blend mask: an entry no pixel blended is not walked)
            const float4* rec = a.rec + (size_t)kRecRows * (ent >> kEntryMaskBits);
            const float4 v0 = rec[0], v1 = rec[1], v2 = rec[2];
            if (ATOMIC) {
                e = ent >> kEntryMaskBits;  // (the Gaussian: its accumulator row)
            } else {
                const float4 v3 = rec[3];
                // this instance's emission index (row 3: tile rectangle [and first emission])
                const uint32_t first = a.rec_start[ent >> kEntryMaskBits];
                e = first + (tty - __float_as_uint(v3.y)) * __float_as_uint(v3.z) + (ttx - __float_as_uint(v3.x));
            }
            s_xy[lane] = make_float4(v0.x, v0.y, v1.y, v1.z);
            s_col[lane] = v2;
            ca = v0.z;
            cb = v0.w;
            cc = v1.x;
            o = v1.y;
            qm = ent & kEntryMask;
            s_cq[lane] = stage_conic(v0, v1, qm);
          }
        }
        if (b0 + kBatch + lane < end) ent_next = a.gid_sorted[range.x + b0 + kBatch + lane];
        unit_sync();
        unsigned long long todo = __ballot(qm != 0);
        unsigned long long written = 0;
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int pos = b0 + j;
            const float4 xy = s_xy[j], cq = s_cq[j], col = s_col[j];
            if (pos >= next_lim) {  // uniform: retire the slots whose last contributor has passed
                next_lim = limit;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (pos >= slim[q]) live &= ~(1u << q);
                    else next_lim = min(next_lim, slim[q]);
                }
            }
            const uint32_t m = uniform_u32(__float_as_uint(cq.w)) & live;
            if (m == 0) continue;
            float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f, r4 = 0.f, r5 = 0.f, r6 = 0.f, r7 = 0.f, r8 = 0.f, r9 = 0.f;
            bool contrib = false;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!(m & (1u << q))) continue;  // uniform
                const float dx = xy.x - (pxf0 + (float)((q & 1) * 8)), dy = xy.y - (pyf0 + (float)((q >> 1) * 8));
                const float p2 = dx * (cq.x * dx + cq.y * dy) + cq.z * dy * dy;
                // the skip tests and "the forward stopped this pixel before `pos`" as ONE mask,
                // shared by alpha and u below (no separate alpha > 0 test)
                const float G = __builtin_amdgcn_exp2f(p2);
                const float ac = fminf(0.99f, xy.z * G);
                const bool on = (p2 <= 0.f) & (ac >= 1.0f / 255.0f) & (pos < nc[q]);
                const float alpha = on ? ac : 0.f;
                if (CENSUS) {
                    c_eval++;
                    c_alpha += (unsigned long long)__popcll(__ballot(alpha > 0.f));
                    c_idle += __any(on) ? 0ull : 1ull;
                }
                if (!__any(on)) continue;  // uniform
                contrib = true;
                const float w = alpha * T[q];
                const float sdot = g0[q] * col.x + g1[q] * col.y + g2[q] * col.z + gi[q] * xy.w;
                gB[q] -= w * sdot;  // now dL/dpix . (colour strictly behind this entry) + background term
                const float one_m_a = 1.f - alpha;
                const float dLda = T[q] * sdot - gB[q] * __builtin_amdgcn_rcpf(one_m_a);
                const float u = on ? dLda * G : 0.f;
                r0 += w * g0[q];
                r1 += w * g1[q];
                r2 += w * g2[q];
                r3 += w * gi[q];
                const float udx = u * dx, udy = u * dy;
                r4 += udx;
                r5 += udy;
                r6 += udx * dx;
                r7 += udx * dy;
                r8 += udy * dy;
                r9 += u;
                T[q] *= one_m_a;  // alpha = 0 leaves T unchanged
            }
            if (contrib) {  // uniform
                // Reduce-scatter over the wave: two lane-swap halvings take the ten sums from
                // 64 lanes to 16 (four sums per register), a DPP 8-lane fold packs w0 and w1 into
                // one register, and three DPP steps finish each 8-lane half (24 VALU; r8 / r9
                // leave as two row partials each, added by the flush).
                const float h0 = half_fold(r0, r1), h1 = half_fold(r2, r3), h2 = half_fold(r4, r5),
                            h3 = half_fold(r6, r7), h4 = half_fold(r8, r9);
                // rows of w0: r0 r2 r1 r3; w1: r4 r6 r5 r7; h4: r8 r8 r9 r9
                const float f = half_row_allsum(eight_fold(row_fold(h0, h1), row_fold(h2, h3), hi8));
                const float g4 = row_allsum(h4);
                if (acc_wr) reinterpret_cast<float*>(s_acc)[j * 4 + acc_lane] = acc_h4 ? g4 : f;
                written |= 1ull << j;
                if (CENSUS) c_red++;
            }
        }
        unit_sync();
        const bool content = (written >> lane) & 1ull;
        if (ATOMIC) {
            // this entry's sums in their final form, over its own LDS slots, and its place in the list
            if (has && content) {
                const float4 A = s_acc[0][lane], B = s_acc[1][lane], Cc = s_acc[2][lane];
                const float s8 = Cc.x + Cc.y, s9 = Cc.z + Cc.w;
                s_acc[1][lane] = make_float4(-0.5f * (float)a.W * o * (ca * B.x + cb * B.y),
                                             -0.5f * (float)a.H * o * (cc * B.y + cb * B.x), s9, -0.5f * o * B.w);
                s_acc[2][lane] = make_float4(-0.5f * o * B.z, -0.5f * o * s8, 0.f, 0.f);
                (void)A;  // (row a is stored as reduced)
                const int slot = __popcll(written & ((1ull << lane) - 1ull));
                s_wgid[slot] = e;
                s_wj[slot] = (uint32_t)lane;
                // the Gaussian has a gradient (gauss_bwd lists it); OR is order-free
                (void)atomicOr(a.touched + (e >> 5), 1u << (e & 31u));
            }
            unit_sync();
            // one wave instruction per four listed entries: lane 16 k + v adds value v of entry k
            const int nw = __popcll(written), sub = lane >> 4, v = lane & 15;
            for (int k0 = 0; k0 < nw; k0 += 4) {  // uniform
                const int k = k0 + sub;
                if (k < nw && v < 10) {
                    const int j = (int)s_wj[k];
                    const float val = reinterpret_cast<const float*>(s_acc)[(v >> 2) * (4 * kBatch) + j * 4 + (v & 3)];
                    (void)atomicAdd(a.acc + (size_t)s_wgid[k] * (4 * kAccRow4) + v, val);  // (no return: fire and forget)
                }
            }
        } else if (has && content) {
            (void)atomicOr(reinterpret_cast<uint32_t*>(a.recs.flag) + (e >> 5), 1u << (e & 31u));
            float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
            float2 rc = make_float2(0.f, 0.f);
            if (content) {
                const float4 A = s_acc[0][lane], B = s_acc[1][lane], Cc = s_acc[2][lane];
                // dL/dmean2D in NDC units (x 0.5 W, 0.5 H, CR/backward.cu:509-510,600-601);
                // dL/dconic with the reference's -0.5 factors (CR/backward.cu:604-606).  (Applying
                // these linear maps per Gaussian in gauss_reduce instead measured +10 us in all, r2o.)
                ra = A;
                const float s8 = Cc.x + Cc.y, s9 = Cc.z + Cc.w;  // r8, r9 from their row partials
                rb = make_float4(-0.5f * (float)a.W * o * (ca * B.x + cb * B.y),
                                 -0.5f * (float)a.H * o * (cc * B.y + cb * B.x), s9, -0.5f * o * B.w);
                rc = make_float2(-0.5f * o * B.z, -0.5f * o * s8);
            }
            // one 48-byte record (a, b, c + pad at recs.a + 0/1/2): one address, full-width stores
            float4* r = a.recs.a + (size_t)kRecAB * e;
            r[0] = ra;
            r[1] = rb;
            r[2] = make_float4(rc.x, rc.y, 0.f, 0.f);
        }
        unit_sync();
    }
    if (CENSUS && lane == 0) {
        atomicAdd(&a.census[4], c_staged);
        atomicAdd(&a.census[5], c_eval);
        atomicAdd(&a.census[6], c_alpha);
        atomicAdd(&a.census[7], c_red);
        atomicAdd(&a.census[8], c_idle);
    }
    GSR_STAMP(g_st_rbwd, blockIdx.x, 1);
    GSR_STAMP_RT(g_st_rbwd, blockIdx.x, 5);
    GSR_STAMP_VAL(g_st_rbwd, blockIdx.x, 2, tile);
    GSR_STAMP_VAL(g_st_rbwd, blockIdx.x, 3, end - start);
    if (!STRIDED) break;  // one unit per block
    }
  }
}

// (the backward sizes its grid with seg_ck = 1, the most units any forward can append: the forward's
// own seg_ck is on the device only; surplus blocks exit at the unit lookup)
size_t bwd_max_units(size_t R, uint32_t tiles, int seg_ck) { return R / ((size_t)seg_ck * kCkStride) + tiles; }

template <bool ATOMIC>
static void launch_render_bwd_t(const RenderBwdArgs& a, uint32_t grid, bool strided, hipStream_t stream) {
    if (a.census)
        hipLaunchKernelGGL((render_bwd_kernel<true, false, ATOMIC>), dim3(grid), dim3(kWave), 0, stream, a);
    else if (strided)
        hipLaunchKernelGGL((render_bwd_kernel<false, true, ATOMIC>), dim3(grid), dim3(kWave), 0, stream, a);
    else
        hipLaunchKernelGGL((render_bwd_kernel<false, false, ATOMIC>), dim3(grid), dim3(kWave), 0, stream, a);
}

// The strided grid: kBwdGridTiles unit blocks per tile, used when the worst-case grid (max_units) is
// more than kBwdStrideRatio times that.
constexpr uint32_t kBwdGridTiles = 2, kBwdStrideRatio = 4;
hipError_t launch_render_bwd(const RenderBwdArgs& a, size_t max_units, hipStream_t stream, int grid_mode) {
    if (max_units == 0) return hipSuccess;
    const size_t strided_units = std::min(max_units, (size_t)kBwdGridTiles * a.gx * a.gy);
    const bool strided = !a.census && (grid_mode == 2 || (grid_mode == 0 && max_units > kBwdStrideRatio * strided_units));
    const uint32_t grid = (uint32_t)(strided ? strided_units : max_units) + a.fill_blocks;  // fill blocks first
    if (a.acc)
        launch_render_bwd_t<true>(a, grid, strided, stream);
    else
        launch_render_bwd_t<false>(a, grid, strided, stream);
    return hipGetLastError();
}

}  // namespace gsr

#ifdef GSR_STAMPS
extern "C" int gsr_diag_stamps_render(int which, unsigned long long* out, size_t n) {
    using namespace gsr;
    if (n > kStampCap) n = kStampCap;
    const void* sym = which == 0 ? (const void*)&g_st_rfwd : (const void*)&g_st_rbwd;
    return (int)hipMemcpyFromSymbol(out, sym, n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost);
}
#endif
