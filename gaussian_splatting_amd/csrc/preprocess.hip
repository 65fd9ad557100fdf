// preprocess.hip -- per-Gaussian projection, culling, EWA covariance and SH colour.
//
// Semantics follow preprocessCUDA (CR/forward.cu:222-351) and its helpers
// (computeCov3D :149-190, computeCov2D :89-141, computeColorFromSH :22-80,
// in_frustum / getRect / ndc2Pix in CR/auxiliary.h).  What differs is the output
// layout: one 48-byte splat record per Gaussian (gsr_common.h), a depth sort key,
// and a conservative footprint box that lets the render kernels skip whole waves.
#include "kernels.h"

namespace gsr {

// Sigma = (S R)^T (S R) in the reference's GLM (column-major) convention, which is
// R_std S^2 R_std^T with R_std the usual rotation of quaternion (r, x, y, z).
__device__ __forceinline__ void cov3d_from_scale_rot(float3 s, float mod, float4 q, float cov[6]) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    // rows of R_std
    const float R00 = 1.f - 2.f * (y * y + z * z), R01 = 2.f * (x * y - r * z), R02 = 2.f * (x * z + r * y);
    const float R10 = 2.f * (x * y + r * z), R11 = 1.f - 2.f * (x * x + z * z), R12 = 2.f * (y * z - r * x);
    const float R20 = 2.f * (x * z - r * y), R21 = 2.f * (y * z + r * x), R22 = 1.f - 2.f * (x * x + y * y);
    const float sx = mod * s.x, sy = mod * s.y, sz = mod * s.z;
    // L = R_std * diag(s): columns scaled
    const float L00 = R00 * sx, L01 = R01 * sy, L02 = R02 * sz;
    const float L10 = R10 * sx, L11 = R11 * sy, L12 = R12 * sz;
    const float L20 = R20 * sx, L21 = R21 * sy, L22 = R22 * sz;
    cov[0] = L00 * L00 + L01 * L01 + L02 * L02;
    cov[1] = L00 * L10 + L01 * L11 + L02 * L12;
    cov[2] = L00 * L20 + L01 * L21 + L02 * L22;
    cov[3] = L10 * L10 + L11 * L11 + L12 * L12;
    cov[4] = L10 * L20 + L11 * L21 + L12 * L22;
    cov[5] = L20 * L20 + L21 * L21 + L22 * L22;
}

// EWA projection of the 3-D covariance: cov2D = A Sigma A^T with A = J(t) * Rv,
// t clamped to 1.3 x the field of view (CR/forward.cu:97-106).
__device__ __forceinline__ float3 cov2d_project(float3 t, float fx, float fy, float tanx, float tany, const float* V,
                                                const float cov[6]) {
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float j00 = fx / t.z, j02 = -(fx * t.x) / (t.z * t.z);
    const float j11 = fy / t.z, j12 = -(fy * t.y) / (t.z * t.z);
    // Rv rows: (V0, V4, V8), (V1, V5, V9), (V2, V6, V10)
    const float a0 = j00 * V[0] + j02 * V[2], a1 = j00 * V[4] + j02 * V[6], a2 = j00 * V[8] + j02 * V[10];
    const float b0 = j11 * V[1] + j12 * V[2], b1 = j11 * V[5] + j12 * V[6], b2 = j11 * V[9] + j12 * V[10];
    // Sigma * a, Sigma * b
    const float sa0 = cov[0] * a0 + cov[1] * a1 + cov[2] * a2;
    const float sa1 = cov[1] * a0 + cov[3] * a1 + cov[4] * a2;
    const float sa2 = cov[2] * a0 + cov[4] * a1 + cov[5] * a2;
    const float sb0 = cov[0] * b0 + cov[1] * b1 + cov[2] * b2;
    const float sb1 = cov[1] * b0 + cov[3] * b1 + cov[4] * b2;
    const float sb2 = cov[2] * b0 + cov[4] * b1 + cov[5] * b2;
    return make_float3(a0 * sa0 + a1 * sa1 + a2 * sa2, a0 * sb0 + a1 * sb1 + a2 * sb2, b0 * sb0 + b1 * sb1 + b2 * sb2);
}

// SH -> RGB for one channel set; sh[k] holds coefficient k (3 channels).
__device__ __forceinline__ float3 sh_to_rgb(int deg, const float3* sh, float x, float y, float z) {
    float3 res = make_float3(SH_C0 * sh[0].x, SH_C0 * sh[0].y, SH_C0 * sh[0].z);
    if (deg > 0) {
        const float c1 = -SH_C1 * y, c2 = SH_C1 * z, c3 = -SH_C1 * x;
        res.x += c1 * sh[1].x + c2 * sh[2].x + c3 * sh[3].x;
        res.y += c1 * sh[1].y + c2 * sh[2].y + c3 * sh[3].y;
        res.z += c1 * sh[1].z + c2 * sh[2].z + c3 * sh[3].z;
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            const float k4 = SH_C2_0 * xy, k5 = SH_C2_1 * yz, k6 = SH_C2_2 * (2.f * zz - xx - yy), k7 = SH_C2_3 * xz,
                        k8 = SH_C2_4 * (xx - yy);
            res.x += k4 * sh[4].x + k5 * sh[5].x + k6 * sh[6].x + k7 * sh[7].x + k8 * sh[8].x;
            res.y += k4 * sh[4].y + k5 * sh[5].y + k6 * sh[6].y + k7 * sh[7].y + k8 * sh[8].y;
            res.z += k4 * sh[4].z + k5 * sh[5].z + k6 * sh[6].z + k7 * sh[7].z + k8 * sh[8].z;
            if (deg > 2) {
                const float k9 = SH_C3_0 * y * (3.f * xx - yy), k10 = SH_C3_1 * xy * z,
                            k11 = SH_C3_2 * y * (4.f * zz - xx - yy), k12 = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy),
                            k13 = SH_C3_4 * x * (4.f * zz - xx - yy), k14 = SH_C3_5 * z * (xx - yy),
                            k15 = SH_C3_6 * x * (xx - 3.f * yy);
                res.x += k9 * sh[9].x + k10 * sh[10].x + k11 * sh[11].x + k12 * sh[12].x + k13 * sh[13].x +
                         k14 * sh[14].x + k15 * sh[15].x;
                res.y += k9 * sh[9].y + k10 * sh[10].y + k11 * sh[11].y + k12 * sh[12].y + k13 * sh[13].y +
                         k14 * sh[14].y + k15 * sh[15].y;
                res.z += k9 * sh[9].z + k10 * sh[10].z + k11 * sh[11].z + k12 * sh[12].z + k13 * sh[13].z +
                         k14 * sh[14].z + k15 * sh[15].z;
            }
        }
    }
    res.x += 0.5f;
    res.y += 0.5f;
    res.z += 0.5f;
    return res;
}

// Load the first K = (deg+1)^2 coefficients (K <= 16) of Gaussian idx, either layout.
__device__ __forceinline__ void load_sh(const ShAddr& sa, int idx, int K, float3 sh[16]) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if (k < K) {
            const float* c = sa.coef(idx, k);
            sh[k] = make_float3(c[0], c[1], c[2]);
        } else {
            sh[k] = make_float3(0.f, 0.f, 0.f);
        }
    }
}

// Stage rows [r0, r0 + rows) of the SH coefficients into LDS rows of kShRowStride floats
// laid out [coefficient 0..15][3].  Combined layout: each row is 48 contiguous floats and
// the block is one contiguous range (16-byte loads, 16-byte LDS stores).  Split layout: the
// rest block (45 floats a row) is one contiguous range too, loaded 16 bytes at a time and
// scattered to LDS as scalars behind the 3 dc floats of each row.
// One wave per 64 consecutive Gaussians.  The geometry is per lane; two data paths are
// cooperative so that every global access of the wave is a contiguous block:
//  * SH (192 B per Gaussian at M = 16, most of the kernel's bytes): the wave's rows are
//    staged through LDS in two halves of 32 rows (6 KiB each, 16-byte loads of one
//    contiguous range), and lanes 0-31 / 32-63 evaluate their colours from LDS;
//  * the 64-byte splat records are assembled in LDS and written as one 4 KiB block.
// A culled Gaussian gets the reference's zero radius / tiles_touched, a 0xffffffff depth
// key and an all-zero record (never read).
constexpr int kPreThreads = 64;  // (the SH prefetch's LDS hand-offs are wave-local: one wave)
constexpr int kShHalfRows = 32;
constexpr int kShRowStride = 52;   // padded LDS row stride (16-byte aligned, conflict-free b128)
template <int SH_MODE>
__global__ void __launch_bounds__(kPreThreads) preprocess_kernel(PreprocessArgs a) {
    __shared__ __attribute__((aligned(16))) float s_buf[SH_MODE != kShGlobal ? kShHalfRows * kShRowStride : 64 * 16];
    static_assert(kShHalfRows * kShRowStride >= 64 * 16, "the record block reuses the SH buffer");
    static_assert(kShHalfRows * kShRowStride >= kShHalfRows * (kShRestF + 3), "the split staging fits the buffer");
    const int lane = threadIdx.x;
    const int g0 = blockIdx.x * kPreThreads;
    const int idx = g0 + lane;
    const bool valid = idx < a.P;
    const int nvalid = min(kPreThreads, a.P - g0);
    for (uint32_t i = blockIdx.x * kPreThreads + lane; i < a.zero_n; i += gridDim.x * kPreThreads) a.zero[i] = 0u;
    // The wave's inputs requested up front: the scale, rotation and opacity of each lane's Gaussian and
    // the first half of the wave's SH block in registers (6 x 16 B per lane), the second half once the
    // first is in LDS -- where the geometry's loads waited for the view transform and each SH half for
    // the previous half's colours.
    typedef float v4f __attribute__((ext_vector_type(4)));
    constexpr bool kPf = SH_MODE == kShLdsCombined;
    constexpr int kPieces = kShHalfRows * (kShRowF / 4) / kPreThreads;  // 16-byte pieces per lane and half
    v4f shp[2][kPieces];
    if constexpr (kPf) {  // the first half
        const v4f* src = reinterpret_cast<const v4f*>(a.shs + (size_t)g0 * kShRowF);
        const int n4 = nvalid * (kShRowF / 4);
#pragma unroll
        for (int k = 0; k < kPieces; k++) {
            const int i4 = k * kPreThreads + lane;
            shp[0][k] = i4 < n4 ? __builtin_nontemporal_load(src + i4) : (v4f){0.f, 0.f, 0.f, 0.f};
        }
    }
    float3 pf_sc = make_float3(0.f, 0.f, 0.f);
    float4 pf_q = make_float4(1.f, 0.f, 0.f, 0.f);
    float pf_op = 0.f;
    if (valid) {
        if (a.scales && !a.cov3D_precomp) {
            pf_sc = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
            pf_q = reinterpret_cast<const float4*>(a.rotations)[idx];
        }
        pf_op = a.opacities[idx];
    }

    // ---- geometry (CR/forward.cu:255-326): `ok` replaces the reference's early returns
    bool ok = valid;
    float3 p = make_float3(0.f, 0.f, 0.f), p_view = p;
    if (valid) {
        p = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
        p_view = xform_point_4x3(p, a.viewmatrix);
        if (p_view.z <= 0.2f) {  // in_frustum (CR/auxiliary.h:180-188); the reference traps when prefiltered
            if (a.prefiltered) atomicOr(a.geom.status, 1u);
            ok = false;
        }
    }
    float px = 0.f, py = 0.f, ca = 0.f, cb = 0.f, cc = 0.f, h_scale = 1.f, det = 0.f;
    float3 cov = make_float3(0.f, 0.f, 0.f);
    int irad = 0;
    uint2 rmin = make_uint2(0u, 0u), rmax = rmin;
    uint32_t touched = 0;
    if (ok) {
        const float4 p_hom = xform_point_4x4(p, a.projmatrix);
        const float p_w = 1.0f / (p_hom.w + 0.0000001f);
        const float px_ndc = p_hom.x * p_w, py_ndc = p_hom.y * p_w;
        float cov3[6];
        if (a.cov3D_precomp) {
#pragma unroll
            for (int i = 0; i < 6; i++) cov3[i] = a.cov3D_precomp[6 * idx + i];
        } else {
            cov3d_from_scale_rot(pf_sc, a.scale_modifier, pf_q, cov3);
        }
        cov = cov2d_project(p_view, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, a.viewmatrix, cov3);
        constexpr float h_var = 0.3f;
        const float det_cov = cov.x * cov.z - cov.y * cov.y;
        cov.x += h_var;
        cov.z += h_var;
        det = cov.x * cov.z - cov.y * cov.y;
        if (a.antialiasing) h_scale = sqrtf(fmaxf(0.000025f, det_cov / det));
        if (det == 0.0f) {
            ok = false;
        } else {
            const float det_inv = 1.f / det;
            ca = cov.z * det_inv;
            cb = -cov.y * det_inv;
            cc = cov.x * det_inv;
            const float mid = 0.5f * (cov.x + cov.z);
            const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
            const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
            const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
            px = ndc2pix(px_ndc, a.W);
            py = ndc2pix(py_ndc, a.H);
            irad = (int)my_radius;
            get_rect(px, py, irad, a.gx, a.gy, rmin, rmax);
            touched = (rmax.y - rmin.y) * (rmax.x - rmin.x);
            if (touched == 0) ok = false;
        }
    }

    // ---- colour (CR/forward.cu:329-336)
    float3 rgb = make_float3(0.f, 0.f, 0.f);
    float3 dir = make_float3(0.f, 0.f, 0.f);
    if (ok && !a.colors_precomp) {
        float3 d = make_float3(p.x - a.campos[0], p.y - a.campos[1], p.z - a.campos[2]);
        const float len = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
        dir = make_float3(d.x / len, d.y / len, d.z / len);
    }
    if (a.colors_precomp) {
        if (ok) rgb = make_float3(a.colors_precomp[3 * idx], a.colors_precomp[3 * idx + 1], a.colors_precomp[3 * idx + 2]);
    } else if constexpr (SH_MODE == kShLdsCombined) {
        const ShAddr sa{a.shs, a.dc, a.M};
#pragma unroll
        for (int half = 0; half < 2; half++) {
            const int rows = min(kShHalfRows, nvalid - half * kShHalfRows);
            if (rows > 0) {  // wave-uniform
                (void)sa;
#pragma unroll
                for (int k = 0; k < kPieces; k++) {
                    const int i4 = k * kPreThreads + lane, row = i4 / (kShRowF / 4), c4 = i4 - row * (kShRowF / 4);
                    *reinterpret_cast<v4f*>(&s_buf[row * kShRowStride + 4 * c4]) = shp[half][k];
                }
                if (half == 0) {  // the second half requested now, read after this one
                    const v4f* src = reinterpret_cast<const v4f*>(a.shs + (size_t)g0 * kShRowF);
                    const int n4 = nvalid * (kShRowF / 4);
#pragma unroll
                    for (int k = 0; k < kPieces; k++) {
                        const int i4 = kShHalfRows * (kShRowF / 4) + k * kPreThreads + lane;
                        shp[1][k] = i4 < n4 ? __builtin_nontemporal_load(src + i4) : (v4f){0.f, 0.f, 0.f, 0.f};
                    }
                }
                wave_lds_sync();  // (one wave: its LDS accesses complete in order)
                if ((lane >> 5) == half && ok) {
                    const float* row = &s_buf[(lane & 31) * kShRowStride];
                    float3 sh[16];
#pragma unroll
                    for (int k = 0; k < 16; k++) sh[k] = make_float3(row[3 * k], row[3 * k + 1], row[3 * k + 2]);
                    rgb = sh_to_rgb(a.D, sh, dir.x, dir.y, dir.z);
                }
                wave_lds_sync();
            }
        }
    } else if constexpr (SH_MODE == kShLdsSplit) {
        // dc + rest (train.py's separate_sh path): the half's 32 rest rows (45 floats each) are one
        // contiguous range in global memory and are kept contiguous in LDS too (row stride 45,
        // odd: conflict-free reads), so they move as 16-byte pieces; the dc triples go to their own
        // area behind them.  (Scattering the rest floats behind each row's dc triple took scalar
        // LDS stores and per-float row divisions: 83 vs 63 us for the combined layout at 1M.)
        float* s_rest = s_buf;                         // [32][45]
        float* s_dc = s_buf + kShHalfRows * kShRestF;  // [32][3]
#pragma unroll
        for (int half = 0; half < 2; half++) {
            const int rows = min(kShHalfRows, nvalid - half * kShHalfRows);
            if (rows > 0) {  // wave-uniform
                const int r0 = g0 + half * kShHalfRows;
                typedef float v4f __attribute__((ext_vector_type(4)));
                const v4f* rest = reinterpret_cast<const v4f*>(a.shs + (size_t)r0 * kShRestF);
                const int nf = rows * kShRestF, n4 = nf >> 2;
#pragma unroll
                for (int k = 0; k < (kShHalfRows * kShRestF / 4 + kPreThreads - 1) / kPreThreads; k++) {
                    const int i4 = k * kPreThreads + lane;
                    if (i4 < n4) reinterpret_cast<v4f*>(s_rest)[i4] = __builtin_nontemporal_load(rest + i4);
                }
                if (lane < (nf & 3)) s_rest[n4 * 4 + lane] = a.shs[(size_t)r0 * kShRestF + n4 * 4 + lane];
                for (int i = lane; i < rows * 3; i += kPreThreads) s_dc[i] = __builtin_nontemporal_load(a.dc + (size_t)r0 * 3 + i);
                __syncthreads();
                if ((lane >> 5) == half && ok) {
                    const float* rr = &s_rest[(lane & 31) * kShRestF];
                    const float* dr = &s_dc[(lane & 31) * 3];
                    float3 sh[16];
                    sh[0] = make_float3(dr[0], dr[1], dr[2]);
#pragma unroll
                    for (int k = 1; k < 16; k++) sh[k] = make_float3(rr[3 * k - 3], rr[3 * k - 2], rr[3 * k - 1]);
                    rgb = sh_to_rgb(a.D, sh, dir.x, dir.y, dir.z);
                }
                __syncthreads();
            }
        }
    } else if (ok) {
        float3 sh[16];
        const int K = (a.D + 1) * (a.D + 1);
        load_sh(ShAddr{a.shs, a.dc, a.M}, idx, K, sh);
        rgb = sh_to_rgb(a.D, sh, dir.x, dir.y, dir.z);
    }
    if (ok && !a.colors_precomp) {
        a.geom.clamped[idx] = (uint8_t)((rgb.x < 0.f ? 1 : 0) | (rgb.y < 0.f ? 2 : 0) | (rgb.z < 0.f ? 4 : 0));
        rgb.x = fmaxf(rgb.x, 0.f);
        rgb.y = fmaxf(rgb.y, 0.f);
        rgb.z = fmaxf(rgb.z, 0.f);
    }

    // ---- footprint box and outputs
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0, r3 = r0;
    if (ok) {
        const float o_eff = pf_op * h_scale;
        // Conservative box of the alpha >= 1/255 footprint: o*exp(-q/2) >= 1/255 <=> q <= 2 ln(255 o).
        uint32_t bbx = pack_i16x2(-32768, 32767), bby = pack_i16x2(-32768, 32767);
        if (a.footprint_cull) {
            if (o_eff * 255.f < 0.999f) {
                bbx = pack_i16x2(1, 0);
                bby = pack_i16x2(1, 0);
            } else if (det > 0.f && cov.x > 0.f && cov.z > 0.f) {
                const float tau = fmaxf(0.f, logf(255.f * o_eff)) * 1.001f + 0.01f;
                const float ex = sqrtf(2.f * tau * cov.x) + 0.05f, ey = sqrtf(2.f * tau * cov.z) + 0.05f;
                const float x0 = floorf(px - ex), x1 = ceilf(px + ex), y0 = floorf(py - ey), y1 = ceilf(py + ey);
                if (isfinite(x0) && isfinite(x1) && isfinite(y0) && isfinite(y1)) {
                    bbx = pack_i16x2((int)fmaxf(x0, -32768.f), (int)fminf(x1, 32767.f));
                    bby = pack_i16x2((int)fmaxf(y0, -32768.f), (int)fminf(y1, 32767.f));
                }
            }
        }
        r0 = make_float4(px, py, ca, cb);
        r1 = make_float4(cc, o_eff, 1.0f / p_view.z, __uint_as_float(bbx));
        r2 = make_float4(rgb.x, rgb.y, rgb.z, __uint_as_float(bby));
        r3 = make_float4(__uint_as_float(rmin.x), __uint_as_float(rmin.y), __uint_as_float(rmax.x - rmin.x), 0.f);
    }
    if (valid) {
        a.radii[idx] = ok ? irad : 0;
        a.geom.tiles_touched[idx] = ok ? touched : 0u;
        a.geom.depth_key[idx] = ok ? __float_as_uint(p_view.z) : 0xffffffffu;
        a.geom.rect[idx] = make_uint2(rmin.x | (rmin.y << 16), rmax.x | (rmax.y << 16));
        // the footprint's opacity mass, the integral of alpha over the plane (o 2 pi sqrt(det cov2D)), for
        // the near-first binning's depth cut (binning.hip); fixed point, saturating
        float mass = 0.f;
        if (ok) {
            mass = pf_op * h_scale * 6.2831853f * sqrtf(fmaxf(det, 0.f)) * kMassScale;
        }
        a.geom.mass[idx] = (uint32_t)fminf(mass, 4.0e9f);
    }
    // the wave's 64 records as one contiguous 4 KiB store
    float4* s_rec = reinterpret_cast<float4*>(s_buf);
    s_rec[lane * kRecRows + 0] = r0;
    s_rec[lane * kRecRows + 1] = r1;
    s_rec[lane * kRecRows + 2] = r2;
    s_rec[lane * kRecRows + 3] = r3;
    wave_lds_sync();  // (not __syncthreads: its fence would wait for the stores above)
    float4* dst = a.geom.rec + (size_t)kRecRows * g0;
#pragma unroll
    for (int k = 0; k < kRecRows; k++) {
        const int i = k * kPreThreads + lane;
        if (i < nvalid * kRecRows) dst[i] = s_rec[i];
    }
}

hipError_t launch_preprocess(const PreprocessArgs& a, hipStream_t stream) {
    if (a.P == 0) return hipSuccess;
    const dim3 grid((a.P + kPreThreads - 1) / kPreThreads), block(kPreThreads);
    // LDS staging for the full SH3 row, either layout (combined [P,16,3] or dc + rest [P,15,3])
    const bool lds = a.shs && !a.colors_precomp && a.M == 16 && a.D == 3 &&
                     ((reinterpret_cast<uintptr_t>(a.shs) & 15) == 0);
    if (lds && a.dc)
        hipLaunchKernelGGL(preprocess_kernel<kShLdsSplit>, grid, block, 0, stream, a);
    else if (lds)
        hipLaunchKernelGGL(preprocess_kernel<kShLdsCombined>, grid, block, 0, stream, a);
    else
        hipLaunchKernelGGL(preprocess_kernel<kShGlobal>, grid, block, 0, stream, a);
    return hipGetLastError();
}

// checkFrustum (CR/rasterizer_impl.cu:56-73): view-space z > 0.2.
__global__ void mark_visible_kernel(int P, const float* __restrict__ means3D, const float* __restrict__ V,
                                    bool* __restrict__ present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float3 p = make_float3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
    present[idx] = xform_point_4x3(p, V).z > 0.2f;
}

hipError_t launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, means3D, view, present);
    return hipGetLastError();
}

}  // namespace gsr
