// render.hip -- per-tile front-to-back alpha blending (forward) and its
// front-to-back gradient pass (backward).
//
// Forward semantics follow renderCUDA (CR/forward.cu:367-513) exactly: the same
// per-pixel skip tests (power > 0, alpha < 1/255), the same early termination
// (T * (1 - alpha) < 1e-4 ends the pixel without adding that Gaussian), and the
// same outputs (colour + T * bg, inverse depth, final T, last contributor).
//
// CDNA4 structure (DESIGN.md "render"):
//  * ONE wave64 per 16x16 tile.  Lane l owns pixel (l & 7, l >> 3) of each of the
//    four 8x8 quadrants ("slots" 0..3), so a lane carries four pixels' state;
//  * list entries are staged 64 at a time (one per lane) into LDS as 48-byte
//    splat records; while loading, each entry's conservative alpha >= 1/255
//    footprint box is tested against the four quadrants (4-bit mask);
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
// Per-Gaussian sums over the tile's pixels are first summed over the lane's four
// slots in registers, then over the wave with DPP reductions -- once per
// (tile, Gaussian) instance -- and written with plain stores.  There are no
// float atomics anywhere, so the result is bitwise reproducible (the reference
// issues 10 global float atomics per pixel-Gaussian pair, CR/backward.cu:569-609).
#include "kernels.h"

namespace gsr {

constexpr int kBatch = 64;  // list entries staged per round (one per lane)

#ifndef GSR_ROWRED
#define GSR_ROWRED 0
#endif

// Quadrant mask of one splat's footprint box inside the tile at (tile_x0, tile_y0).
__device__ __forceinline__ uint32_t quad_bits(float4 v1, float4 v2, int tile_x0, int tile_y0) {
    const uint32_t bx = __float_as_uint(v1.w), by = __float_as_uint(v2.w);
    const int x0 = unpack_lo(bx), x1 = unpack_hi(bx), y0 = unpack_lo(by), y1 = unpack_hi(by);
    uint32_t q = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int qx0 = tile_x0 + (k & 1) * 8, qy0 = tile_y0 + (k >> 1) * 8;
        if (x0 <= qx0 + 7 && x1 >= qx0 && y0 <= qy0 + 7 && y1 >= qy0) q |= 1u << k;
    }
    return q;
}

__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) render_fwd_kernel(RenderFwdArgs a) {
    const uint32_t tile = blockIdx.x;
    const int tile_x0 = (int)(tile % a.gx) * kTile, tile_y0 = (int)(tile / a.gx) * kTile;
    const int lane = threadIdx.x;
    const int lx = lane & 7, ly = lane >> 3;

    __shared__ float4 s_r0[kBatch], s_r1[kBatch], s_r2[kBatch];

    float T[4], C0[4], C1[4], C2[4], D[4];
    uint32_t last[4];
    bool done[4];
    uint32_t alive = 0;  // wave-uniform: slots with at least one pixel still blending
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int px = tile_x0 + (q & 1) * 8 + lx, py = tile_y0 + (q >> 1) * 8 + ly;
        done[q] = !(px < a.W && py < a.H);
        T[q] = 1.f;
        C0[q] = C1[q] = C2[q] = D[q] = 0.f;
        last[q] = 0;
        if (__any(!done[q])) alive |= 1u << q;
    }
    const float pxf0 = (float)(tile_x0 + lx), pyf0 = (float)(tile_y0 + ly);

    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int b0 = 0; b0 < n && alive; b0 += kBatch) {
        uint32_t qm = 0;
        if (b0 + lane < n) {
            const uint32_t g = a.emit_gid[a.e_sorted[range.x + b0 + lane]];
            const float4 v0 = a.rec0[g], v1 = a.rec1[g], v2 = a.rec2[g];
            qm = quad_bits(v1, v2, tile_x0, tile_y0);
            s_r0[lane] = v0;
            s_r1[lane] = make_float4(v1.x, v1.y, v1.z, __uint_as_float(qm));
            s_r2[lane] = v2;
        }
        __syncthreads();
        unsigned long long todo = __ballot(qm != 0);
        while (todo && alive) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const float4 v0 = s_r0[j], v1 = s_r1[j], v2 = s_r2[j];
            const uint32_t m = uniform_u32(__float_as_uint(v1.w)) & alive;
            const uint32_t pos1 = (uint32_t)(b0 + j + 1);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!(m & (1u << q))) continue;  // uniform: footprint misses this quadrant
                // The reference's three tests become predicates (power is clamped to <= 0 before
                // exp so skipped lanes stay finite); the update runs only if some lane passes.
                const float dx = v0.x - (pxf0 + (float)((q & 1) * 8));
                const float dy = v0.y - (pyf0 + (float)((q >> 1) * 8));
                const float power = -0.5f * (v0.z * dx * dx + v1.x * dy * dy) - v0.w * dx * dy;
                const float alpha = fminf(0.99f, v1.y * __expf(fminf(power, 0.f)));
                const bool hit = !done[q] && power <= 0.0f && alpha >= 1.0f / 255.0f;
                if (!__any(hit)) continue;  // uniform
                const float test_T = T[q] * (1.f - alpha);
                const bool term = hit && test_T < 0.0001f;  // CR/forward.cu:477-482: ends the pixel, not added
                const bool add = hit && !term;
                done[q] = done[q] || term;
                const float w = add ? alpha * T[q] : 0.f;
                C0[q] += v2.x * w;
                C1[q] += v2.y * w;
                C2[q] += v2.z * w;
                D[q] += v1.z * w;
                T[q] = add ? test_T : T[q];
                last[q] = add ? pos1 : last[q];
                if (__all(done[q])) alive &= ~(1u << q);
            }
        }
        __syncthreads();
    }
    const size_t N = (size_t)a.W * a.H;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int px = tile_x0 + (q & 1) * 8 + lx, py = tile_y0 + (q >> 1) * 8 + ly;
        if (px < a.W && py < a.H) {
            const size_t pix = (size_t)py * a.W + px;
            a.img.final_T[pix] = T[q];
            a.img.n_contrib[pix] = last[q];
            a.img.accum[pix] = C0[q];
            a.img.accum[N + pix] = C1[q];
            a.img.accum[2 * N + pix] = C2[q];
            a.img.accum[3 * N + pix] = D[q];
            a.out_color[pix] = C0[q] + T[q] * a.bg[0];
            a.out_color[N + pix] = C1[q] + T[q] * a.bg[1];
            a.out_color[2 * N + pix] = C2[q] + T[q] * a.bg[2];
            a.out_invdepth[pix] = D[q];
        }
    }
}

hipError_t launch_render_fwd(const RenderFwdArgs& a, hipStream_t stream) {
    const uint32_t tiles = a.gx * a.gy;
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(render_fwd_kernel, dim3(tiles), dim3(kWave), 0, stream, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) render_bwd_kernel(RenderBwdArgs a) {
    const uint32_t tile = blockIdx.x;
    const int tile_x0 = (int)(tile % a.gx) * kTile, tile_y0 = (int)(tile / a.gx) * kTile;
    const int lane = threadIdx.x;
    const int lx = lane & 7, ly = lane >> 3;

    __shared__ float4 s_r0[kBatch], s_r1[kBatch], s_r2[kBatch];
#if GSR_ROWRED
    // per entry: four 16-lane row partials of the 10 sums (12 floats each), padded stride
    constexpr int kPart = 52;
    __shared__ __attribute__((aligned(16))) float s_part[kBatch * kPart];
#else
    __shared__ float4 s_acc[kBatch][3];  // per entry: 10 reduced sums (+2 pad)
#endif

    const size_t N = (size_t)a.W * a.H;
    float T[4], gB[4], g0[4], g1[4], g2[4], gi[4], bgt[4];
    int nc[4];
    uint32_t wmax = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int px = tile_x0 + (q & 1) * 8 + lx, py = tile_y0 + (q >> 1) * 8 + ly;
        T[q] = 1.f;
        nc[q] = 0;
        gB[q] = g0[q] = g1[q] = g2[q] = gi[q] = bgt[q] = 0.f;
        if (px < a.W && py < a.H) {
            const size_t pix = (size_t)py * a.W + px;
            nc[q] = (int)a.img.n_contrib[pix];
            g0[q] = a.dL_dpix[pix];
            g1[q] = a.dL_dpix[N + pix];
            g2[q] = a.dL_dpix[2 * N + pix];
            if (a.dL_dinvdepth) gi[q] = a.dL_dinvdepth[pix];
            // dL/dpix . (everything the forward accumulated) -- shrinks to "behind" as we walk
            gB[q] = g0[q] * a.img.accum[pix] + g1[q] * a.img.accum[N + pix] + g2[q] * a.img.accum[2 * N + pix] +
                    gi[q] * a.img.accum[3 * N + pix];
            // background term of dL/dalpha (CR/backward.cu:587-590)
            bgt[q] = a.img.final_T[pix] * (a.bg[0] * g0[q] + a.bg[1] * g1[q] + a.bg[2] * g2[q]);
        }
        wmax = max(wmax, (uint32_t)nc[q]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, off));
    const int limit = (int)uniform_u32(wmax);  // entries at positions >= limit reach no pixel of this tile
    const float pxf0 = (float)(tile_x0 + lx), pyf0 = (float)(tile_y0 + ly);

    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int b0 = 0; b0 < n; b0 += kBatch) {
        const bool has = b0 + lane < n;
        const uint32_t e = has ? a.e_sorted[range.x + b0 + lane] : 0u;
        if (b0 >= limit) {  // uniform: zero records for entries no pixel reaches
            if (has) {
                a.recs.a[e] = make_float4(0.f, 0.f, 0.f, 0.f);
                a.recs.b[e] = make_float4(0.f, 0.f, 0.f, 0.f);
                a.recs.c[e] = make_float2(0.f, 0.f);
            }
            continue;
        }
        uint32_t qm = 0;
        if (has) {
            const uint32_t g = a.emit_gid[e];
            const float4 v0 = a.rec0[g], v1 = a.rec1[g], v2 = a.rec2[g];
            qm = quad_bits(v1, v2, tile_x0, tile_y0);
            s_r0[lane] = v0;
            s_r1[lane] = make_float4(v1.x, v1.y, v1.z, __uint_as_float(qm));
            s_r2[lane] = v2;
        }
        __syncthreads();
        unsigned long long todo = __ballot(qm != 0);
        const int span = limit - b0;  // only positions < limit matter
        if (span < 64) todo &= (1ull << span) - 1ull;
        unsigned long long written = 0;
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int pos = b0 + j;
            const float4 v0 = s_r0[j], v1 = s_r1[j], v2 = s_r2[j];
            const uint32_t m = uniform_u32(__float_as_uint(v1.w));
            float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f, r4 = 0.f, r5 = 0.f, r6 = 0.f, r7 = 0.f, r8 = 0.f, r9 = 0.f;
            bool contrib = false;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!(m & (1u << q))) continue;  // uniform
                // Same tests as the forward, as predicates; the gradient work runs only if some
                // lane of the slot passes them.
                const float dx = v0.x - (pxf0 + (float)((q & 1) * 8));
                const float dy = v0.y - (pyf0 + (float)((q >> 1) * 8));
                const float power = -0.5f * (v0.z * dx * dx + v1.x * dy * dy) - v0.w * dx * dy;
                const float G = __expf(fminf(power, 0.f));
                const float alpha = fminf(0.99f, v1.y * G);
                const bool hit = pos < nc[q] && power <= 0.0f && alpha >= 1.0f / 255.0f;
                if (!__any(hit)) continue;  // uniform
                contrib = true;
                const float w = hit ? alpha * T[q] : 0.f;
                const float sdot = g0[q] * v2.x + g1[q] * v2.y + g2[q] * v2.z + gi[q] * v1.z;
                gB[q] -= w * sdot;  // now dL/dpix . (colour strictly behind this entry)
                const float one_m_a = 1.f - alpha;
                const float dLda = T[q] * sdot - (gB[q] + bgt[q]) * __builtin_amdgcn_rcpf(one_m_a);
                const float u = hit ? dLda * G : 0.f;
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
                T[q] = hit ? T[q] * one_m_a : T[q];
            }
            if (contrib) {  // uniform
#if GSR_ROWRED
                r0 = row_sum_to_lane15(r0);
                r1 = row_sum_to_lane15(r1);
                r2 = row_sum_to_lane15(r2);
                r3 = row_sum_to_lane15(r3);
                r4 = row_sum_to_lane15(r4);
                r5 = row_sum_to_lane15(r5);
                r6 = row_sum_to_lane15(r6);
                r7 = row_sum_to_lane15(r7);
                r8 = row_sum_to_lane15(r8);
                r9 = row_sum_to_lane15(r9);
                if ((lane & 15) == 15) {
                    float4* p = reinterpret_cast<float4*>(&s_part[j * kPart + (lane >> 4) * 12]);
                    p[0] = make_float4(r0, r1, r2, r3);
                    p[1] = make_float4(r4, r5, r6, r7);
                    p[2] = make_float4(r8, r9, 0.f, 0.f);
                }
#else
                r0 = wave_sum_to_lane63(r0);
                r1 = wave_sum_to_lane63(r1);
                r2 = wave_sum_to_lane63(r2);
                r3 = wave_sum_to_lane63(r3);
                r4 = wave_sum_to_lane63(r4);
                r5 = wave_sum_to_lane63(r5);
                r6 = wave_sum_to_lane63(r6);
                r7 = wave_sum_to_lane63(r7);
                r8 = wave_sum_to_lane63(r8);
                r9 = wave_sum_to_lane63(r9);
                if (lane == 63) {
                    s_acc[j][0] = make_float4(r0, r1, r2, r3);
                    s_acc[j][1] = make_float4(r4, r5, r6, r7);
                    s_acc[j][2] = make_float4(r8, r9, 0.f, 0.f);
                }
#endif
                written |= 1ull << j;
            }
        }
        __syncthreads();
        if (has) {
            float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
            float2 rc = make_float2(0.f, 0.f);
            if ((written >> lane) & 1ull) {
#if GSR_ROWRED
                const float4* p = reinterpret_cast<const float4*>(&s_part[lane * kPart]);
                float4 A = p[0], B = p[1], Cc = p[2];
#pragma unroll
                for (int rr = 1; rr < 4; rr++) {  // fixed order: deterministic
                    const float4 a4 = p[3 * rr], b4 = p[3 * rr + 1], c4 = p[3 * rr + 2];
                    A.x += a4.x; A.y += a4.y; A.z += a4.z; A.w += a4.w;
                    B.x += b4.x; B.y += b4.y; B.z += b4.z; B.w += b4.w;
                    Cc.x += c4.x; Cc.y += c4.y;
                }
#else
                const float4 A = s_acc[lane][0], B = s_acc[lane][1], Cc = s_acc[lane][2];
#endif
                const float4 v0 = s_r0[lane], v1 = s_r1[lane];
                const float o = v1.y, ca = v0.z, cb = v0.w, cc = v1.x;
                // dL/dmean2D in NDC units (x 0.5 W, 0.5 H, CR/backward.cu:509-510,600-601);
                // dL/dconic with the reference's -0.5 factors (CR/backward.cu:604-606)
                ra = A;
                rb = make_float4(-0.5f * (float)a.W * o * (ca * B.x + cb * B.y),
                                 -0.5f * (float)a.H * o * (cc * B.y + cb * B.x), Cc.y, -0.5f * o * B.w);
                rc = make_float2(-0.5f * o * B.z, -0.5f * o * Cc.x);
            }
            a.recs.a[e] = ra;
            a.recs.b[e] = rb;
            a.recs.c[e] = rc;
        }
        __syncthreads();
    }
}

hipError_t launch_render_bwd(const RenderBwdArgs& a, hipStream_t stream) {
    const uint32_t tiles = a.gx * a.gy;
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(render_bwd_kernel, dim3(tiles), dim3(kWave), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
