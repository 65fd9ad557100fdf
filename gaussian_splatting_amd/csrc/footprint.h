// footprint.h -- conservative tests of a splat's alpha >= 1/255 footprint against the
// four 8x8 quadrants of a 16x16 tile.  Used when binning (binning.hip K3 stores each
// (tile, Gaussian) instance's 4-bit quadrant mask in its tile-list entry) and by the render
// kernels' consumers of that mask.  Inputs are the first three rows of the splat record
// (gsr_common.h).
#pragma once

#include "gsr_common.h"

namespace gsr {

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

// Conic quadratic form Q(d) = a dx^2 + 2 b dx dy + c dy^2 (power = -Q/2), minimised over the
// pixel-centre rectangle [x0,x1] x [y0,y1] of offsets d = p - mean.  For a positive-definite
// conic the minimum is 0 if the mean is inside, otherwise on an edge, where Q is a 1-D
// parabola minimised at the clamped vertex.
__device__ __forceinline__ float rect_min_form(float a, float b, float c, float ra, float rc, float x0, float x1,
                                               float y0, float y1) {
    if (x0 <= 0.f && x1 >= 0.f && y0 <= 0.f && y1 >= 0.f) return 0.f;
    float best = INFINITY;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const float dx = k ? x1 : x0;
        const float dy = fminf(y1, fmaxf(y0, -b * dx * rc));
        best = fminf(best, a * dx * dx + (2.f * b * dx + c * dy) * dy);
        const float ey = k ? y1 : y0;
        const float ex = fminf(x1, fmaxf(x0, -b * ey * ra));
        best = fminf(best, c * ey * ey + (2.f * b * ey + a * ex) * ex);
    }
    return best;
}

// Quadrant mask refined by the footprint ellipse itself: a quadrant the box overlaps is
// dropped when no pixel centre of it lies inside the alpha >= 1/255 ellipse
// Q <= 2 ln(255 o), with the same relative/absolute margin the box uses (preprocess.hip), so
// the test stays conservative under fp32 rounding of the per-pixel evaluation.  Degenerate
// conics keep the box result.  Runs while staging, one list entry per lane.
// `only`: the quadrants to test (the others' bits come back clear) -- a half-tile render wave
// tests its own two.
__device__ __forceinline__ uint32_t quad_bits_exact(float4 v0, float4 v1, float4 v2, int tile_x0, int tile_y0,
                                                    uint32_t only = 0xfu) {
    uint32_t q = quad_bits(v1, v2, tile_x0, tile_y0) & only;
    const float a = v0.z, b = v0.w, c = v1.x, o = v1.y;
    if (q == 0 || !(a > 0.f && c > 0.f && a * c - b * b > 0.f) || !(o > 0.f)) return q;
    const float tau = fmaxf(0.f, __logf(255.f * o)) * 1.001f + 0.01f;
    const float lim = 2.f * tau;
    const float ra = 1.f / a, rc = 1.f / c;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (!(only & (1u << k))) continue;  // (compile-time after inlining with a constant mask)
        if (!(q & (1u << k))) continue;
        const float x0 = (float)(tile_x0 + (k & 1) * 8) - v0.x, y0 = (float)(tile_y0 + (k >> 1) * 8) - v0.y;
        if (rect_min_form(a, b, c, ra, rc, x0, x0 + 7.f, y0, y0 + 7.f) > lim) q &= ~(1u << k);
    }
    return q;
}

// One quadrant's bit of quad_bits_exact: does the alpha >= 1/255 footprint (box, then
// ellipse) reach a pixel centre of the 8x8 quadrant at (qx0, qy0)?
__device__ __forceinline__ bool quad_hit(float4 v0, float4 v1, float4 v2, int qx0, int qy0) {
    const uint32_t bx = __float_as_uint(v1.w), by = __float_as_uint(v2.w);
    if (!(unpack_lo(bx) <= qx0 + 7 && unpack_hi(bx) >= qx0 && unpack_lo(by) <= qy0 + 7 && unpack_hi(by) >= qy0))
        return false;
    const float a = v0.z, b = v0.w, c = v1.x, o = v1.y;
    if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f) || !(o > 0.f)) return true;
    const float tau = fmaxf(0.f, __logf(255.f * o)) * 1.001f + 0.01f;
    const float x0 = (float)qx0 - v0.x, y0 = (float)qy0 - v0.y;
    return rect_min_form(a, b, c, 1.f / a, 1.f / c, x0, x0 + 7.f, y0, y0 + 7.f) <= 2.f * tau;
}

}  // namespace gsr
