// backward.hip -- fused per-Gaussian backward.
//
// One thread per Gaussian (coalesced over the output rows):
//   1. sums the Gaussian's per-(tile) gradient records -- they are contiguous in
//      emission order, so this is a deterministic segmented sum with no atomics;
//   2. computeCov2DCUDA (CR/backward.cu:153-290) including the tail that the
//      vendored file truncates (dL/dcov3D and dL/dmean3D through the EWA
//      projection, the clamp masks and the inverse-depth term), derived in
//      DESIGN.md "Backward conventions";
//   3. preprocessCUDA (CR/backward.cu:372-429): screen-space mean -> 3-D mean,
//      SH colour backward (:12-146) and scale/rotation backward (:296-365).
// Every output row is written, zeros included, so the host never memsets the
// gradient tensors (the reference zero-fills all of them first,
// RI/rasterize_points.cu:186-195).
#include "kernels.h"

namespace gsr {


__device__ __forceinline__ void store3(float* p, int i, float x, float y, float z) {
    p[3 * i] = x;
    p[3 * i + 1] = y;
    p[3 * i + 2] = z;
}

__global__ void __launch_bounds__(256) gauss_bwd_kernel(GaussBwdArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    const int M = a.M;
    if (!(a.radii[idx] > 0)) {
        store3(a.dL_dmean2D, idx, 0.f, 0.f, 0.f);
        if (a.dL_dconic) reinterpret_cast<float4*>(a.dL_dconic)[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
        a.dL_dopacity[idx] = 0.f;
        store3(a.dL_dcolor, idx, 0.f, 0.f, 0.f);
        if (a.dL_dinvdepth) a.dL_dinvdepth[idx] = 0.f;
        store3(a.dL_dmean3D, idx, 0.f, 0.f, 0.f);
        for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * idx + k] = 0.f;
        if (a.dL_dsh)
            for (int k = 0; k < 3 * M; k++) a.dL_dsh[(size_t)idx * 3 * M + k] = 0.f;
        if (a.dL_dscale) store3(a.dL_dscale, idx, 0.f, 0.f, 0.f);
        if (a.dL_drot) reinterpret_cast<float4*>(a.dL_drot)[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }

    // ---- 1. segmented sum of this Gaussian's (tile) records
    const uint32_t r = a.geom.rank_of[idx];
    const unsigned long long e1 = a.geom.offsets[r];
    const unsigned long long e0 = r == 0 ? 0ull : a.geom.offsets[r - 1];
    float4 sa = make_float4(0.f, 0.f, 0.f, 0.f), sb = make_float4(0.f, 0.f, 0.f, 0.f);
    float2 sc = make_float2(0.f, 0.f);
    for (unsigned long long e = e0; e < e1; e++) {
        const float4 x = a.recs.a[e], y = a.recs.b[e];
        const float2 z = a.recs.c[e];
        sa.x += x.x; sa.y += x.y; sa.z += x.z; sa.w += x.w;
        sb.x += y.x; sb.y += y.y; sb.z += y.z; sb.w += y.w;
        sc.x += z.x; sc.y += z.y;
    }
    const float3 dcol = make_float3(sa.x, sa.y, sa.z);
    const float dinvd = sa.w;
    const float m2x = sb.x, m2y = sb.y;
    float dop = sb.z;
    // dL/dconic in the reference's convention: (a, b/2-weighted, c) (CR/backward.cu:604-606)
    const float dca = sc.x, dcb = sb.w, dcc = sc.y;
    store3(a.dL_dmean2D, idx, m2x, m2y, 0.f);
    store3(a.dL_dcolor, idx, dcol.x, dcol.y, dcol.z);
    if (a.dL_dconic) reinterpret_cast<float4*>(a.dL_dconic)[idx] = make_float4(dca, dcb, 0.f, dcc);
    if (a.dL_dinvdepth) a.dL_dinvdepth[idx] = dinvd;

    // ---- 2. computeCov2DCUDA
    const float* V = a.viewmatrix;
    const float3 mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
    float3 t = xform_point_4x3(mean, V);
    const float limx = 1.3f * a.tan_fovx, limy = 1.3f * a.tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0.f : 1.f;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0.f : 1.f;
    const float fx = a.focal_x, fy = a.focal_y;
    const float j00 = fx / t.z, j02 = -(fx * t.x) / (t.z * t.z);
    const float j11 = fy / t.z, j12 = -(fy * t.y) / (t.z * t.z);
    // A = J * Rv rows a (x) and b (y); Rv rows (V0,V4,V8) (V1,V5,V9) (V2,V6,V10)
    const float A0[3] = {j00 * V[0] + j02 * V[2], j00 * V[4] + j02 * V[6], j00 * V[8] + j02 * V[10]};
    const float A1[3] = {j11 * V[1] + j12 * V[2], j11 * V[5] + j12 * V[6], j11 * V[9] + j12 * V[10]};

    float cov[6];
    float3 sc3 = make_float3(0.f, 0.f, 0.f);
    float4 q = make_float4(1.f, 0.f, 0.f, 0.f);
    if (a.scales) {
        sc3 = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
        q = reinterpret_cast<const float4*>(a.rotations)[idx];
    }
    if (a.cov3D_precomp) {
        for (int k = 0; k < 6; k++) cov[k] = a.cov3D_precomp[6 * idx + k];
    } else {
        const float r_ = q.x, x = q.y, y = q.z, z = q.w;
        const float R00 = 1.f - 2.f * (y * y + z * z), R01 = 2.f * (x * y - r_ * z), R02 = 2.f * (x * z + r_ * y);
        const float R10 = 2.f * (x * y + r_ * z), R11 = 1.f - 2.f * (x * x + z * z), R12 = 2.f * (y * z - r_ * x);
        const float R20 = 2.f * (x * z - r_ * y), R21 = 2.f * (y * z + r_ * x), R22 = 1.f - 2.f * (x * x + y * y);
        const float sx = a.scale_modifier * sc3.x, sy = a.scale_modifier * sc3.y, sz = a.scale_modifier * sc3.z;
        const float L00 = R00 * sx, L01 = R01 * sy, L02 = R02 * sz, L10 = R10 * sx, L11 = R11 * sy, L12 = R12 * sz,
                    L20 = R20 * sx, L21 = R21 * sy, L22 = R22 * sz;
        cov[0] = L00 * L00 + L01 * L01 + L02 * L02;
        cov[1] = L00 * L10 + L01 * L11 + L02 * L12;
        cov[2] = L00 * L20 + L01 * L21 + L02 * L22;
        cov[3] = L10 * L10 + L11 * L11 + L12 * L12;
        cov[4] = L10 * L20 + L11 * L21 + L12 * L22;
        cov[5] = L20 * L20 + L21 * L21 + L22 * L22;
    }
    // Sigma * A0, Sigma * A1
    const float SA0[3] = {cov[0] * A0[0] + cov[1] * A0[1] + cov[2] * A0[2],
                          cov[1] * A0[0] + cov[3] * A0[1] + cov[4] * A0[2],
                          cov[2] * A0[0] + cov[4] * A0[1] + cov[5] * A0[2]};
    const float SA1[3] = {cov[0] * A1[0] + cov[1] * A1[1] + cov[2] * A1[2],
                          cov[1] * A1[0] + cov[3] * A1[1] + cov[4] * A1[2],
                          cov[2] * A1[0] + cov[4] * A1[1] + cov[5] * A1[2]};
    float c_xx = A0[0] * SA0[0] + A0[1] * SA0[1] + A0[2] * SA0[2];
    const float c_xy = A0[0] * SA1[0] + A0[1] * SA1[1] + A0[2] * SA1[2];
    float c_yy = A1[0] * SA1[0] + A1[1] * SA1[1] + A1[2] * SA1[2];

    constexpr float h_var = 0.3f;
    float d_inside_root = 0.f;
    if (a.antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
        const float h = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
        const float d_h = dop * a.opacities[idx];
        dop = dop * h;
        d_inside_root = (det_cov / det_cov_plus_h_cov) <= 0.000025f ? 0.f : d_h / (2.f * h);
    } else {
        c_xx += h_var;
        c_yy += h_var;
    }
    float dL_dc_xx = 0.f, dL_dc_xy = 0.f, dL_dc_yy = 0.f;
    if (a.antialiasing) {
        // reference formula (CR/backward.cu:256-270), evaluated at the dilated x, y as written there
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float qd = w * w + w * (x + y) + x * y - z * z;
        const float denom_f = d_inside_root / (qd * qd);
        dL_dc_xx = w * (w * y + y * y + z * z) * denom_f;
        dL_dc_yy = w * (w * x + x * x + z * z) * denom_f;
        dL_dc_xy = -2.f * w * z * (w + x + y) * denom_f;
    }
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    if (denom2inv != 0.f) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dca + 2.f * c_xy * c_yy * dcb + (denom - c_xx * c_yy) * dcc);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dcc + 2.f * c_xx * c_xy * dcb + (denom - c_xx * c_yy) * dca);
        dL_dc_xy += denom2inv * 2.f * (c_xy * c_yy * dca - (denom + 2.f * c_xy * c_xy) * dcb + c_xx * c_xy * dcc);
    }
    a.dL_dopacity[idx] = dop;

    // tail: cov2D = A Sigma A^T  ->  dL/dcov3D (6 stored entries) and dL/dA
    const float ga = dL_dc_xx, gb = dL_dc_xy, gc = dL_dc_yy;
    float dcov[6];
    dcov[0] = A0[0] * A0[0] * ga + A0[0] * A1[0] * gb + A1[0] * A1[0] * gc;
    dcov[3] = A0[1] * A0[1] * ga + A0[1] * A1[1] * gb + A1[1] * A1[1] * gc;
    dcov[5] = A0[2] * A0[2] * ga + A0[2] * A1[2] * gb + A1[2] * A1[2] * gc;
    dcov[1] = 2.f * A0[0] * A0[1] * ga + (A0[0] * A1[1] + A0[1] * A1[0]) * gb + 2.f * A1[0] * A1[1] * gc;
    dcov[2] = 2.f * A0[0] * A0[2] * ga + (A0[0] * A1[2] + A0[2] * A1[0]) * gb + 2.f * A1[0] * A1[2] * gc;
    dcov[4] = 2.f * A0[2] * A0[1] * ga + (A0[1] * A1[2] + A0[2] * A1[1]) * gb + 2.f * A1[1] * A1[2] * gc;
    for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * idx + k] = dcov[k];

    float dA0[3], dA1[3];
    for (int k = 0; k < 3; k++) {
        dA0[k] = 2.f * ga * SA0[k] + gb * SA1[k];
        dA1[k] = 2.f * gc * SA1[k] + gb * SA0[k];
    }
    const float dJ00 = dA0[0] * V[0] + dA0[1] * V[4] + dA0[2] * V[8];
    const float dJ02 = dA0[0] * V[2] + dA0[1] * V[6] + dA0[2] * V[10];
    const float dJ11 = dA1[0] * V[1] + dA1[1] * V[5] + dA1[2] * V[9];
    const float dJ12 = dA1[0] * V[2] + dA1[1] * V[6] + dA1[2] * V[10];
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -fx * tz2 * dJ02;
    const float dL_dty = y_grad_mul * -fy * tz2 * dJ12;
    float dL_dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.f * fx * t.x) * tz3 * dJ02 + (2.f * fy * t.y) * tz3 * dJ12;
    if (a.have_invdepth) dL_dtz -= dinvd / (t.z * t.z);
    // transformVec4x3Transpose (CR/auxiliary.h:109-117)
    float3 dmean = make_float3(V[0] * dL_dtx + V[1] * dL_dty + V[2] * dL_dtz, V[4] * dL_dtx + V[5] * dL_dty + V[6] * dL_dtz,
                               V[8] * dL_dtx + V[9] * dL_dty + V[10] * dL_dtz);

    // ---- 3a. screen-space mean -> 3-D mean through the projection (CR/backward.cu:403-420)
    const float* Pm = a.projmatrix;
    const float4 m_hom = xform_point_4x4(mean, Pm);
    const float m_w = 1.0f / (m_hom.w + 0.0000001f);
    const float mul1 = m_hom.x * m_w * m_w, mul2 = m_hom.y * m_w * m_w;
    dmean.x += (Pm[0] * m_w - Pm[3] * mul1) * m2x + (Pm[1] * m_w - Pm[3] * mul2) * m2y;
    dmean.y += (Pm[4] * m_w - Pm[7] * mul1) * m2x + (Pm[5] * m_w - Pm[7] * mul2) * m2y;
    dmean.z += (Pm[8] * m_w - Pm[11] * mul1) * m2x + (Pm[9] * m_w - Pm[11] * mul2) * m2y;

    // ---- 3b. SH colour backward (CR/backward.cu:12-146)
    if (a.shs) {
        const float3 dir_orig = make_float3(mean.x - a.campos[0], mean.y - a.campos[1], mean.z - a.campos[2]);
        const float len = sqrtf(dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z);
        const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
        const uint8_t cm = a.geom.clamped[idx];
        const float3 g = make_float3((cm & 1) ? 0.f : dcol.x, (cm & 2) ? 0.f : dcol.y, (cm & 4) ? 0.f : dcol.z);
        const float* sh = a.shs + (size_t)idx * M * 3;
        float* dsh = a.dL_dsh + (size_t)idx * M * 3;
        const int deg = a.D;
        float k[16];
        for (int i = 0; i < 16; i++) k[i] = 0.f;
        // d(colour)/d(dir) accumulated per channel as dot with g directly
        float ddx = 0.f, ddy = 0.f, ddz = 0.f;
        k[0] = SH_C0;
        auto dotg = [&](int c) { return sh[3 * c] * g.x + sh[3 * c + 1] * g.y + sh[3 * c + 2] * g.z; };
        if (deg > 0) {
            k[1] = -SH_C1 * y;
            k[2] = SH_C1 * z;
            k[3] = -SH_C1 * x;
            const float s1 = dotg(1), s2 = dotg(2), s3 = dotg(3);
            ddx = -SH_C1 * s3;
            ddy = -SH_C1 * s1;
            ddz = SH_C1 * s2;
            if (deg > 1) {
                const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                k[4] = SH_C2_0 * xy;
                k[5] = SH_C2_1 * yz;
                k[6] = SH_C2_2 * (2.f * zz - xx - yy);
                k[7] = SH_C2_3 * xz;
                k[8] = SH_C2_4 * (xx - yy);
                const float s4 = dotg(4), s5 = dotg(5), s6 = dotg(6), s7 = dotg(7), s8 = dotg(8);
                ddx += SH_C2_0 * y * s4 + SH_C2_2 * 2.f * -x * s6 + SH_C2_3 * z * s7 + SH_C2_4 * 2.f * x * s8;
                ddy += SH_C2_0 * x * s4 + SH_C2_1 * z * s5 + SH_C2_2 * 2.f * -y * s6 + SH_C2_4 * 2.f * -y * s8;
                ddz += SH_C2_1 * y * s5 + SH_C2_2 * 2.f * 2.f * z * s6 + SH_C2_3 * x * s7;
                if (deg > 2) {
                    k[9] = SH_C3_0 * y * (3.f * xx - yy);
                    k[10] = SH_C3_1 * xy * z;
                    k[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
                    k[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                    k[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
                    k[14] = SH_C3_5 * z * (xx - yy);
                    k[15] = SH_C3_6 * x * (xx - 3.f * yy);
                    const float s9 = dotg(9), s10 = dotg(10), s11 = dotg(11), s12 = dotg(12), s13 = dotg(13),
                                s14 = dotg(14), s15 = dotg(15);
                    ddx += SH_C3_0 * s9 * 3.f * 2.f * xy + SH_C3_1 * s10 * yz + SH_C3_2 * s11 * -2.f * xy +
                           SH_C3_3 * s12 * -3.f * 2.f * xz + SH_C3_4 * s13 * (-3.f * xx + 4.f * zz - yy) +
                           SH_C3_5 * s14 * 2.f * xz + SH_C3_6 * s15 * 3.f * (xx - yy);
                    ddy += SH_C3_0 * s9 * 3.f * (xx - yy) + SH_C3_1 * s10 * xz +
                           SH_C3_2 * s11 * (-3.f * yy + 4.f * zz - xx) + SH_C3_3 * s12 * -3.f * 2.f * yz +
                           SH_C3_4 * s13 * -2.f * xy + SH_C3_5 * s14 * -2.f * yz + SH_C3_6 * s15 * -3.f * 2.f * xy;
                    ddz += SH_C3_1 * s10 * xy + SH_C3_2 * s11 * 4.f * 2.f * yz +
                           SH_C3_3 * s12 * 3.f * (2.f * zz - xx - yy) + SH_C3_4 * s13 * 4.f * 2.f * xz +
                           SH_C3_5 * s14 * (xx - yy);
                }
            }
        }
        const int K = (deg + 1) * (deg + 1);
        for (int c = 0; c < M; c++) {
            const float kc = c < K && c < 16 ? k[c] : 0.f;
            dsh[3 * c] = kc * g.x;
            dsh[3 * c + 1] = kc * g.y;
            dsh[3 * c + 2] = kc * g.z;
        }
        // dnormvdv (CR/auxiliary.h:129-139)
        const float3 v = dir_orig;
        const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
        const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
        dmean.x += ((sum2 - v.x * v.x) * ddx - v.y * v.x * ddy - v.z * v.x * ddz) * invsum32;
        dmean.y += (-v.x * v.y * ddx + (sum2 - v.y * v.y) * ddy - v.z * v.y * ddz) * invsum32;
        dmean.z += (-v.x * v.z * ddx - v.y * v.z * ddy + (sum2 - v.z * v.z) * ddz) * invsum32;
    } else if (a.dL_dsh) {
        for (int c = 0; c < 3 * M; c++) a.dL_dsh[(size_t)idx * 3 * M + c] = 0.f;
    }
    store3(a.dL_dmean3D, idx, dmean.x, dmean.y, dmean.z);

    // ---- 3c. scale / rotation backward (CR/backward.cu:296-365)
    if (a.scales) {  // CR/backward.cu:427-428
        const float r_ = q.x, x = q.y, y = q.z, z = q.w;
        // Rg[col][row] = GLM rotation (R_std transposed)
        const float Rg[3][3] = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r_ * z), 2.f * (x * z + r_ * y)},
                                {2.f * (x * y + r_ * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r_ * x)},
                                {2.f * (x * z - r_ * y), 2.f * (y * z + r_ * x), 1.f - 2.f * (x * x + y * y)}};
        const float s[3] = {a.scale_modifier * sc3.x, a.scale_modifier * sc3.y, a.scale_modifier * sc3.z};
        float Mg[3][3];
        for (int c = 0; c < 3; c++)
            for (int rr = 0; rr < 3; rr++) Mg[c][rr] = s[rr] * Rg[c][rr];
        const float dS[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                                {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                                {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
        float dMt[3][3];  // dMt[i][k] = dL_dM[k][i]; dL_dM = 2 M dSigma (GLM product)
        for (int c = 0; c < 3; c++)
            for (int rr = 0; rr < 3; rr++)
                dMt[rr][c] = 2.f * (Mg[0][rr] * dS[c][0] + Mg[1][rr] * dS[c][1] + Mg[2][rr] * dS[c][2]);
        // dot(Rt[i], dL_dMt[i]), Rt[i][k] = Rg[k][i]; the reference leaves the scale modifier out here
        const float ds0 = Rg[0][0] * dMt[0][0] + Rg[1][0] * dMt[0][1] + Rg[2][0] * dMt[0][2];
        const float ds1 = Rg[0][1] * dMt[1][0] + Rg[1][1] * dMt[1][1] + Rg[2][1] * dMt[1][2];
        const float ds2 = Rg[0][2] * dMt[2][0] + Rg[1][2] * dMt[2][1] + Rg[2][2] * dMt[2][2];
        store3(a.dL_dscale, idx, ds0, ds1, ds2);
        for (int i = 0; i < 3; i++)
            for (int kk = 0; kk < 3; kk++) dMt[i][kk] *= s[i];
        float4 dq;
        dq.x = 2.f * z * (dMt[0][1] - dMt[1][0]) + 2.f * y * (dMt[2][0] - dMt[0][2]) + 2.f * x * (dMt[1][2] - dMt[2][1]);
        dq.y = 2.f * y * (dMt[1][0] + dMt[0][1]) + 2.f * z * (dMt[2][0] + dMt[0][2]) + 2.f * r_ * (dMt[1][2] - dMt[2][1]) -
               4.f * x * (dMt[2][2] + dMt[1][1]);
        dq.z = 2.f * x * (dMt[1][0] + dMt[0][1]) + 2.f * r_ * (dMt[2][0] - dMt[0][2]) + 2.f * z * (dMt[1][2] + dMt[2][1]) -
               4.f * y * (dMt[2][2] + dMt[0][0]);
        dq.w = 2.f * r_ * (dMt[0][1] - dMt[1][0]) + 2.f * x * (dMt[2][0] + dMt[0][2]) + 2.f * y * (dMt[1][2] + dMt[2][1]) -
               4.f * z * (dMt[1][1] + dMt[0][0]);
        reinterpret_cast<float4*>(a.dL_drot)[idx] = dq;
    } else {
        if (a.dL_dscale) store3(a.dL_dscale, idx, 0.f, 0.f, 0.f);
        if (a.dL_drot) reinterpret_cast<float4*>(a.dL_drot)[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

hipError_t launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t stream) {
    if (a.P == 0) return hipSuccess;
    hipLaunchKernelGGL(gauss_bwd_kernel, dim3((a.P + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
