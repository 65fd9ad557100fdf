// render.hip -- per-tile front-to-back alpha blending (forward) and its
// front-to-back gradient pass (backward).
//
// Forward semantics follow renderCUDA (CR/forward.cu:367-513) exactly: the same
// per-pixel skip tests (power > 0, alpha < 1/255), the same early termination
// (T * (1 - alpha) < 1e-4 ends the pixel without adding that Gaussian), and the
// same outputs (colour + T * bg, inverse depth, final T, last contributor).
//
// CDNA4 structure (DESIGN.md "render"):
//  * one 256-thread workgroup per 16x16 tile; wave w owns the 8x8 quadrant
//    (w & 1, w >> 1), so a wave's pixels are compact;
//  * a batch of 256 list entries is gathered into LDS as 48-byte splat records;
//    while loading, each entry's conservative alpha >= 1/255 footprint box is
//    tested against the four quadrants, and every wave turns its bit into a
//    64-bit ballot -- the wave then visits only the entries that can touch its
//    pixels (scalar bit scan), skipping the rest with no vector work;
//  * LDS reads of a record are wave-uniform broadcasts (no bank conflicts).
//
// The backward pass walks the list in the same (front-to-back) order, recomputing
// T exactly as the forward did instead of recovering it by division as the
// reference does (CR/backward.cu:553); the colour "behind" each Gaussian comes
// from the forward's accumulated colour.  Per-Gaussian sums over the tile's
// pixels are formed with DPP wave reductions + one LDS add per wave, and written
// once per (tile, Gaussian) instance with plain stores -- no global atomics
// (the reference issues 10 global float atomics per pixel-Gaussian pair,
// CR/backward.cu:569-609).
#include "kernels.h"

namespace gsr {


// Quadrant mask of one splat's footprint box inside tile (tx, ty).
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

__global__ void __launch_bounds__(256) render_fwd_kernel(RenderFwdArgs a) {
    const uint32_t tile = blockIdx.x;
    const int tile_x0 = (int)(tile % a.gx) * kTile, tile_y0 = (int)(tile / a.gx) * kTile;
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const int px = tile_x0 + (wv & 1) * 8 + (lane & 7);
    const int py = tile_y0 + (wv >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;

    __shared__ float4 s_r0[kTilePix], s_r1[kTilePix], s_r2[kTilePix];
    __shared__ uint32_t s_q[kTilePix];

    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    float T = 1.f, C0 = 0.f, C1 = 0.f, C2 = 0.f, D = 0.f;
    uint32_t last = 0;
    bool done = !inside;

    for (int b0 = 0; b0 < n; b0 += kTilePix) {
        // Barrier (also protects the LDS batch) + block-wide early exit (CR/forward.cu:436-438).
        if (__syncthreads_count(done) == kTilePix) break;
        if (b0 + t < n) {
            const uint32_t g = a.sorted_gid[range.x + b0 + t];
            const float4 v0 = a.rec0[g], v1 = a.rec1[g], v2 = a.rec2[g];
            s_r0[t] = v0;
            s_r1[t] = v1;
            s_r2[t] = v2;
            s_q[t] = quad_bits(v1, v2, tile_x0, tile_y0);
        } else {
            s_q[t] = 0;
        }
        __syncthreads();
        const int cnt = min(kTilePix, n - b0);
        for (int c = 0; c * 64 < cnt; c++) {
            unsigned long long m = __ballot((s_q[c * 64 + lane] >> wv) & 1u);
            while (m) {
                if (__all(done)) break;
                const int j = c * 64 + __builtin_ctzll(m);
                m &= m - 1;
                const float4 v0 = s_r0[j], v1 = s_r1[j], v2 = s_r2[j];
                if (!done) {
                    const float dx = v0.x - pxf, dy = v0.y - pyf;
                    const float power = -0.5f * (v0.z * dx * dx + v1.x * dy * dy) - v0.w * dx * dy;
                    if (power <= 0.0f) {
                        const float alpha = fminf(0.99f, v1.y * __expf(power));
                        if (alpha >= 1.0f / 255.0f) {
                            const float test_T = T * (1.f - alpha);
                            if (test_T < 0.0001f) {
                                done = true;
                            } else {
                                const float w = alpha * T;
                                C0 += v2.x * w;
                                C1 += v2.y * w;
                                C2 += v2.z * w;
                                D += v1.z * w;
                                T = test_T;
                                last = (uint32_t)(b0 + j + 1);
                            }
                        }
                    }
                }
            }
        }
    }
    if (inside) {
        const size_t N = (size_t)a.W * a.H;
        const size_t pix = (size_t)py * a.W + px;
        a.img.final_T[pix] = T;
        a.img.n_contrib[pix] = last;
        a.img.accum[pix] = C0;
        a.img.accum[N + pix] = C1;
        a.img.accum[2 * N + pix] = C2;
        a.img.accum[3 * N + pix] = D;
        a.out_color[pix] = C0 + T * a.bg[0];
        a.out_color[N + pix] = C1 + T * a.bg[1];
        a.out_color[2 * N + pix] = C2 + T * a.bg[2];
        a.out_invdepth[pix] = D;
    }
}

hipError_t launch_render_fwd(const RenderFwdArgs& a, hipStream_t stream) {
    const uint32_t tiles = a.gx * a.gy;
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(render_fwd_kernel, dim3(tiles), dim3(kTilePix), 0, stream, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) render_bwd_kernel(RenderBwdArgs a) {
    const uint32_t tile = blockIdx.x;
    const int tile_x0 = (int)(tile % a.gx) * kTile, tile_y0 = (int)(tile / a.gx) * kTile;
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const int px = tile_x0 + (wv & 1) * 8 + (lane & 7);
    const int py = tile_y0 + (wv >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;

    __shared__ float4 s_r0[kTilePix], s_r1[kTilePix], s_r2[kTilePix];
    __shared__ uint32_t s_q[kTilePix];
    __shared__ float s_acc[10][kTilePix];
    __shared__ uint32_t s_maxnc;

    const size_t N = (size_t)a.W * a.H;
    const size_t pix = inside ? (size_t)py * a.W + px : 0;
    uint32_t nc = 0;
    float T_final = 0.f, Ct0 = 0.f, Ct1 = 0.f, Ct2 = 0.f, Dt = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f, gi = 0.f;
    if (inside) {
        nc = a.img.n_contrib[pix];
        T_final = a.img.final_T[pix];
        Ct0 = a.img.accum[pix];
        Ct1 = a.img.accum[N + pix];
        Ct2 = a.img.accum[2 * N + pix];
        Dt = a.img.accum[3 * N + pix];
        g0 = a.dL_dpix[pix];
        g1 = a.dL_dpix[N + pix];
        g2 = a.dL_dpix[2 * N + pix];
        if (a.dL_dinvdepth) gi = a.dL_dinvdepth[pix];
    }
    // background term of dL/dalpha (CR/backward.cu:587-590), constant per pixel
    const float bg_term = T_final * (a.bg[0] * g0 + a.bg[1] * g1 + a.bg[2] * g2);

    // wave / block maximum of the per-pixel contributor counts
    uint32_t wmax = nc;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, off));
    if (t == 0) s_maxnc = 0;
    __syncthreads();
    if (lane == 0) atomicMax(&s_maxnc, wmax);
    __syncthreads();
    const int block_max = (int)s_maxnc;

    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    float T = 1.f, A0 = 0.f, A1 = 0.f, A2 = 0.f, AD = 0.f;

    for (int b0 = 0; b0 < n; b0 += kTilePix) {
        const bool has = b0 + t < n;
        const uint32_t e = has ? a.e_sorted[range.x + b0 + t] : 0u;
        if (b0 >= block_max) {  // block-uniform: nobody in this tile reaches these entries
            if (has) {
                a.recs.a[e] = make_float4(0.f, 0.f, 0.f, 0.f);
                a.recs.b[e] = make_float4(0.f, 0.f, 0.f, 0.f);
                a.recs.c[e] = make_float2(0.f, 0.f);
            }
            continue;
        }
        __syncthreads();  // previous batch's LDS fully consumed
        if (has) {
            const uint32_t g = a.sorted_gid[range.x + b0 + t];
            const float4 v0 = a.rec0[g], v1 = a.rec1[g], v2 = a.rec2[g];
            s_r0[t] = v0;
            s_r1[t] = v1;
            s_r2[t] = v2;
            s_q[t] = quad_bits(v1, v2, tile_x0, tile_y0);
        } else {
            s_q[t] = 0;
        }
#pragma unroll
        for (int v = 0; v < 10; v++) s_acc[v][t] = 0.f;
        __syncthreads();

        const int cnt = min(kTilePix, n - b0);
        for (int c = 0; c * 64 < cnt; c++) {
            if (b0 + c * 64 >= (int)wmax) break;  // wave-uniform: no pixel of this wave reaches here
            unsigned long long m = __ballot((s_q[c * 64 + lane] >> wv) & 1u);
            while (m) {
                const int j = c * 64 + __builtin_ctzll(m);
                m &= m - 1;
                const int pos = b0 + j;  // 0-based position in the tile list
                if (pos >= (int)wmax) break;
                const float4 v0 = s_r0[j], v1 = s_r1[j], v2 = s_r2[j];
                float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f, r4 = 0.f, r5 = 0.f, r6 = 0.f, r7 = 0.f, r8 = 0.f,
                      r9 = 0.f;
                bool contrib = false;
                if (pos < (int)nc) {
                    const float dx = v0.x - pxf, dy = v0.y - pyf;
                    const float power = -0.5f * (v0.z * dx * dx + v1.x * dy * dy) - v0.w * dx * dy;
                    if (power <= 0.0f) {
                        const float G = __expf(power);
                        const float alpha = fminf(0.99f, v1.y * G);
                        if (alpha >= 1.0f / 255.0f) {
                            contrib = true;
                            const float w = alpha * T;
                            A0 += v2.x * w;
                            A1 += v2.y * w;
                            A2 += v2.z * w;
                            AD += v1.z * w;
                            const float one_m_a = 1.f - alpha;
                            const float inv1ma = 1.f / one_m_a;
                            const float front = T * (g0 * v2.x + g1 * v2.y + g2 * v2.z + gi * v1.z);
                            const float behind = g0 * (Ct0 - A0) + g1 * (Ct1 - A1) + g2 * (Ct2 - A2) + gi * (Dt - AD);
                            const float dLda = front - (behind + bg_term) * inv1ma;
                            const float u = dLda * G;
                            r0 = w * g0;
                            r1 = w * g1;
                            r2 = w * g2;
                            r3 = w * gi;
                            const float udx = u * dx, udy = u * dy;
                            r4 = udx;
                            r5 = udy;
                            r6 = udx * dx;
                            r7 = udx * dy;
                            r8 = udy * dy;
                            r9 = u;
                            T *= one_m_a;
                        }
                    }
                }
                if (__any(contrib)) {
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
                        atomicAdd(&s_acc[0][j], r0);
                        atomicAdd(&s_acc[1][j], r1);
                        atomicAdd(&s_acc[2][j], r2);
                        atomicAdd(&s_acc[3][j], r3);
                        atomicAdd(&s_acc[4][j], r4);
                        atomicAdd(&s_acc[5][j], r5);
                        atomicAdd(&s_acc[6][j], r6);
                        atomicAdd(&s_acc[7][j], r7);
                        atomicAdd(&s_acc[8][j], r8);
                        atomicAdd(&s_acc[9][j], r9);
                    }
                }
            }
        }
        __syncthreads();
        if (has) {
            const float4 v0 = s_r0[t], v1 = s_r1[t];
            const float o = v1.y, ca = v0.z, cb = v0.w, cc = v1.x;
            const float S4 = s_acc[4][t], S5 = s_acc[5][t];
            const float m2x = -0.5f * (float)a.W * o * (ca * S4 + cb * S5);
            const float m2y = -0.5f * (float)a.H * o * (cc * S5 + cb * S4);
            a.recs.a[e] = make_float4(s_acc[0][t], s_acc[1][t], s_acc[2][t], s_acc[3][t]);
            a.recs.b[e] = make_float4(m2x, m2y, s_acc[9][t], -0.5f * o * s_acc[7][t]);
            a.recs.c[e] = make_float2(-0.5f * o * s_acc[6][t], -0.5f * o * s_acc[8][t]);
        }
    }
}

hipError_t launch_render_bwd(const RenderBwdArgs& a, hipStream_t stream) {
    const uint32_t tiles = a.gx * a.gy;
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(render_bwd_kernel, dim3(tiles), dim3(kTilePix), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
