/*
 * gsr_oracle.c -- CPU restatement of the reference tile rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path links or calls this
 * file: it is loaded by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, and there only as the checker / CPU baseline.
 *
 * It restates the algorithm of the reference's
 * submodules/diff-gaussian-rasterization (graphdeco `dr_aa` branch vendored at
 * /root/reference) step for step, in the reference's own order:
 *   preprocess            CR/forward.cu:222-351 (+ CR/auxiliary.h:43-190)
 *   inclusive scan        CR/rasterizer_impl.cu:309
 *   duplicateWithKeys     CR/rasterizer_impl.cu:78-126
 *   stable radix sort     CR/rasterizer_impl.cu:332-340 (bits [0, 32+msb))
 *   identifyTileRanges    CR/rasterizer_impl.cu:132-164
 *   render (fwd)          CR/forward.cu:367-513
 *   render (bwd)          CR/backward.cu:433-612 (back-to-front, T recovered
 *                         by division, exactly as the reference does)
 *   computeCov2DCUDA      CR/backward.cu:153-290 + the tail that is truncated in
 *                         the vendored file (re-derived analytically, see
 *                         DESIGN.md "Backward conventions")
 *   preprocess (bwd)      CR/backward.cu:296-429
 * (CR = submodules/diff-gaussian-rasterization/cuda_rasterizer)
 *
 * Parity pinning: the reference's own tests hold no vectors for this path
 * (SURVEY.md section 8c).  This restatement is pinned by (1) the reference's
 * importable Python (utils/sh_utils.eval_sh, utils/graphics_utils camera
 * matrices) via tests/golden fixtures made by tests/golden/make_golden.py,
 * (2) torch autograd over an independent differentiable restatement
 * (tests/torch_ref.py), (3) central finite differences in float64, and
 * (4) closed-form known-answer cases.
 *
 * Built twice: -DOR_DOUBLE=0 (float, the reference's arithmetic type; ndc2Pix in
 * double as CR/auxiliary.h:45 does) and -DOR_DOUBLE=1 (all double, used for
 * finite-difference gradient checks).  -ffp-contract=off keeps every operation
 * individually rounded.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#if OR_DOUBLE
typedef double real;
#define EXP exp
#define SQRT sqrt
#define CEIL ceil
#define FMINR fmin
#define FMAXR fmax
#define SYM(name) oracle64_##name
#else
typedef float real;
#define EXP expf
#define SQRT sqrtf
#define CEIL ceilf
#define FMINR fminf
#define FMAXR fmaxf
#define SYM(name) oracle32_##name
#endif
#define R(x) ((real)(x))

#define BLOCK_X 16
#define BLOCK_Y 16
#define BLOCK_SIZE (BLOCK_X * BLOCK_Y)
#define NUM_CHANNELS 3

/* SH constants: CR/auxiliary.h:23-40 */
static const real SH_C0 = R(0.28209479177387814);
static const real SH_C1 = R(0.4886025119029199);
static const real SH_C2[5] = {R(1.0925484305920792), R(-1.0925484305920792), R(0.31539156525252005),
                              R(-1.0925484305920792), R(0.5462742152960396)};
static const real SH_C3[7] = {R(-0.5900435899266435), R(2.890611442640554), R(-0.4570457994644658),
                              R(0.3731763325901154), R(-0.4570457994644658), R(1.445305721320277),
                              R(-0.5900435899266435)};

/* GPU float->int conversion saturates and maps NaN to 0 (cvt.rzi / v_cvt_i32_f32);
 * plain C (int) is undefined there, so restate it. */
static int f2i_sat(double f) {
    if (f != f) return 0;
    if (f >= 2147483647.0) return 2147483647;
    if (f <= -2147483648.0) return (-2147483647 - 1);
    return (int)f;
}

/* ndc2Pix, CR/auxiliary.h:43-46: the literal 1.0 makes it a double expression, rounded to float on return. */
#if OR_DOUBLE
static real ndc2pix(real v, int S) { return ((v + 1.0) * S - 1.0) * 0.5; }
#else
static real ndc2pix(real v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }
#endif

/* getRect, CR/auxiliary.h:49-59 */
static void get_rect(real px, real py, int max_radius, unsigned gx, unsigned gy, unsigned rmin[2], unsigned rmax[2]) {
    const real r = (real)max_radius;
    int v;
    v = f2i_sat((px - r) / R(BLOCK_X)); v = v > 0 ? v : 0; rmin[0] = (unsigned)v < gx ? (unsigned)v : gx;
    v = f2i_sat((py - r) / R(BLOCK_Y)); v = v > 0 ? v : 0; rmin[1] = (unsigned)v < gy ? (unsigned)v : gy;
    v = f2i_sat((((px + r) + R(BLOCK_X)) - R(1)) / R(BLOCK_X)); v = v > 0 ? v : 0; rmax[0] = (unsigned)v < gx ? (unsigned)v : gx;
    v = f2i_sat((((py + r) + R(BLOCK_Y)) - R(1)) / R(BLOCK_Y)); v = v > 0 ? v : 0; rmax[1] = (unsigned)v < gy ? (unsigned)v : gy;
}

/* transformPoint4x3 / 4x4, CR/auxiliary.h:75-95: column-major 4x4 as 16 floats. */
static void xform43(const real* p, const real* m, real* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
static void xform44(const real* p, const real* m, real* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}

/* ---- state kept between forward and backward (the reference's 3 byte buffers) ---- */
typedef struct {
    int P, D, M, W, H, antialiasing, prefiltered;
    unsigned gx, gy;
    real scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    real bg[3], view[16], proj[16], campos[3];
    /* inputs (copied) */
    real *means3D, *shs, *colors_precomp, *opacities, *scales, *rotations, *cov3D_precomp;
    /* geometry state, CR/rasterizer_impl.h GeometryState */
    real *depths, *means2D, *cov3D, *conic_opacity, *rgb;
    unsigned char* clamped;
    int* radii;
    uint32_t *tiles_touched, *point_offsets;
    /* binning state */
    int R;
    uint64_t* keys;
    uint32_t* point_list;
    /* image state */
    uint32_t* ranges; /* [tiles][2] */
    real* final_T;
    uint32_t* n_contrib;
    int prefilter_violation;
} OracleState;

static real* dup_arr(const real* src, size_t n) {
    if (!src || n == 0) return NULL;
    real* d = (real*)malloc(n * sizeof(real));
    memcpy(d, src, n * sizeof(real));
    return d;
}

/* computeColorFromSH (forward), CR/forward.cu:22-80 */
static void color_from_sh(const OracleState* s, int idx, real* out, unsigned char* clamped) {
    const real* pos = s->means3D + 3 * idx;
    real dir[3] = {pos[0] - s->campos[0], pos[1] - s->campos[1], pos[2] - s->campos[2]};
    real len = SQRT(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
    const real* sh = s->shs + (size_t)idx * s->M * 3;
    const int deg = s->D;
    unsigned char cm = 0;
    for (int c = 0; c < 3; c++) {
        real res = SH_C0 * sh[0 * 3 + c];
        if (deg > 0) {
            real x = dir[0], y = dir[1], z = dir[2];
            res = res - SH_C1 * y * sh[1 * 3 + c] + SH_C1 * z * sh[2 * 3 + c] - SH_C1 * x * sh[3 * 3 + c];
            if (deg > 1) {
                real xx = x * x, yy = y * y, zz = z * z;
                real xy = x * y, yz = y * z, xz = x * z;
                res = res + SH_C2[0] * xy * sh[4 * 3 + c] + SH_C2[1] * yz * sh[5 * 3 + c] +
                      SH_C2[2] * (R(2) * zz - xx - yy) * sh[6 * 3 + c] + SH_C2[3] * xz * sh[7 * 3 + c] +
                      SH_C2[4] * (xx - yy) * sh[8 * 3 + c];
                if (deg > 2) {
                    res = res + SH_C3[0] * y * (R(3) * xx - yy) * sh[9 * 3 + c] + SH_C3[1] * xy * z * sh[10 * 3 + c] +
                          SH_C3[2] * y * (R(4) * zz - xx - yy) * sh[11 * 3 + c] +
                          SH_C3[3] * z * (R(2) * zz - R(3) * xx - R(3) * yy) * sh[12 * 3 + c] +
                          SH_C3[4] * x * (R(4) * zz - xx - yy) * sh[13 * 3 + c] +
                          SH_C3[5] * z * (xx - yy) * sh[14 * 3 + c] + SH_C3[6] * x * (xx - R(3) * yy) * sh[15 * 3 + c];
                }
            }
        }
        res += R(0.5);
        if (res < 0) cm |= (unsigned char)(1u << c);
        out[c] = res < 0 ? R(0) : res; /* glm::max(result, 0.0f) */
    }
    *clamped = cm;
}

/* computeCov3D (forward), CR/forward.cu:149-190: Sigma = (S R)^T (S R), GLM column-major */
static void cov3d_fwd(const real* scale, real mod, const real* rot, real* cov) {
    real S[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    real r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    /* Rg[col][row] as constructed by glm::mat3(...) */
    real Rg[3][3] = {{R(1) - R(2) * (y * y + z * z), R(2) * (x * y - r * z), R(2) * (x * z + r * y)},
                     {R(2) * (x * y + r * z), R(1) - R(2) * (x * x + z * z), R(2) * (y * z - r * x)},
                     {R(2) * (x * z - r * y), R(2) * (y * z + r * x), R(1) - R(2) * (x * x + y * y)}};
    real Mg[3][3]; /* M = S * R: M[c][r] = S_r * R[c][r] */
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) Mg[c][rr] = S[rr] * Rg[c][rr];
    /* Sigma[c][r] = sum_k M[r][k] M[c][k] */
    real Sg[3][3];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) Sg[c][rr] = Mg[rr][0] * Mg[c][0] + Mg[rr][1] * Mg[c][1] + Mg[rr][2] * Mg[c][2];
    cov[0] = Sg[0][0]; cov[1] = Sg[0][1]; cov[2] = Sg[0][2];
    cov[3] = Sg[1][1]; cov[4] = Sg[1][2]; cov[5] = Sg[2][2];
}

/* The 2x3 Jacobian-times-view-rotation "T" of computeCov2D, CR/forward.cu:89-141.
 * Returns Tg[col][row] in GLM layout (col 2 is zero) and the (clamped) t. */
static void cov2d_T(const OracleState* s, const real* mean, real Tg[3][3], real t[3], real* txtz_o, real* tytz_o) {
    xform43(mean, s->view, t);
    const real limx = R(1.3) * s->tan_fovx;
    const real limy = R(1.3) * s->tan_fovy;
    const real txtz = t[0] / t[2];
    const real tytz = t[1] / t[2];
    *txtz_o = txtz; *tytz_o = tytz;
    t[0] = FMINR(limx, FMAXR(-limx, txtz)) * t[2];
    t[1] = FMINR(limy, FMAXR(-limy, tytz)) * t[2];
    const real fx = s->focal_x, fy = s->focal_y;
    real J[3][3] = {{fx / t[2], R(0), -(fx * t[0]) / (t[2] * t[2])},
                    {R(0), fy / t[2], -(fy * t[1]) / (t[2] * t[2])},
                    {R(0), R(0), R(0)}};
    const real* v = s->view;
    real Wg[3][3] = {{v[0], v[4], v[8]}, {v[1], v[5], v[9]}, {v[2], v[6], v[10]}};
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) Tg[c][rr] = Wg[0][rr] * J[c][0] + Wg[1][rr] * J[c][1] + Wg[2][rr] * J[c][2];
}

static void cov2d_fwd(const OracleState* s, const real* mean, const real* cov3D, real out[3]) {
    real Tg[3][3], t[3], a, b;
    cov2d_T(s, mean, Tg, t, &a, &b);
    real V[3][3] = {{cov3D[0], cov3D[1], cov3D[2]}, {cov3D[1], cov3D[3], cov3D[4]}, {cov3D[2], cov3D[4], cov3D[5]}};
    /* cov = T^T * V^T * T evaluated left to right */
    real X[3][3];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) X[c][rr] = Tg[rr][0] * V[c][0] + Tg[rr][1] * V[c][1] + Tg[rr][2] * V[c][2];
    real C[3][3];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) C[c][rr] = X[0][rr] * Tg[c][0] + X[1][rr] * Tg[c][1] + X[2][rr] * Tg[c][2];
    out[0] = C[0][0]; out[1] = C[0][1]; out[2] = C[1][1];
}

/* preprocessCUDA (forward), CR/forward.cu:222-351 */
static void preprocess_one(OracleState* s, int idx) {
    s->radii[idx] = 0;
    s->tiles_touched[idx] = 0;
    const real* p = s->means3D + 3 * idx;
    /* in_frustum, CR/auxiliary.h:164-190 */
    real p_view[3];
    xform43(p, s->view, p_view);
    if (p_view[2] <= R(0.2)) {
        if (s->prefiltered) s->prefilter_violation = 1; /* reference: printf + __trap() */
        return;
    }
    real p_hom[4];
    xform44(p, s->proj, p_hom);
    real p_w = R(1) / (p_hom[3] + R(0.0000001));
    real p_proj[3] = {p_hom[0] * p_w, p_hom[1] * p_w, p_hom[2] * p_w};
    const real* cov3D;
    if (s->cov3D_precomp) {
        cov3D = s->cov3D_precomp + 6 * idx;
    } else {
        cov3d_fwd(s->scales + 3 * idx, s->scale_modifier, s->rotations + 4 * idx, s->cov3D + 6 * idx);
        cov3D = s->cov3D + 6 * idx;
    }
    real cov[3];
    cov2d_fwd(s, p, cov3D, cov);
    const real h_var = R(0.3);
    const real det_cov = cov[0] * cov[2] - cov[1] * cov[1];
    cov[0] += h_var;
    cov[2] += h_var;
    const real det_cov_plus_h_cov = cov[0] * cov[2] - cov[1] * cov[1];
    real h_convolution_scaling = R(1);
    if (s->antialiasing) h_convolution_scaling = SQRT(FMAXR(R(0.000025), det_cov / det_cov_plus_h_cov));
    const real det = det_cov_plus_h_cov;
    if (det == R(0)) return;
    real det_inv = R(1) / det;
    real conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
    real mid = R(0.5) * (cov[0] + cov[2]);
    real lambda1 = mid + SQRT(FMAXR(R(0.1), mid * mid - det));
    real lambda2 = mid - SQRT(FMAXR(R(0.1), mid * mid - det));
    real my_radius = CEIL(R(3) * SQRT(FMAXR(lambda1, lambda2)));
    real px = ndc2pix(p_proj[0], s->W), py = ndc2pix(p_proj[1], s->H);
    unsigned rmin[2], rmax[2];
    get_rect(px, py, f2i_sat(my_radius), s->gx, s->gy, rmin, rmax);
    if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) return;
    if (!s->colors_precomp) color_from_sh(s, idx, s->rgb + 3 * idx, s->clamped + idx);
    s->depths[idx] = p_view[2];
    s->radii[idx] = f2i_sat(my_radius);
    s->means2D[2 * idx + 0] = px;
    s->means2D[2 * idx + 1] = py;
    s->conic_opacity[4 * idx + 0] = conic[0];
    s->conic_opacity[4 * idx + 1] = conic[1];
    s->conic_opacity[4 * idx + 2] = conic[2];
    s->conic_opacity[4 * idx + 3] = s->opacities[idx] * h_convolution_scaling;
    s->tiles_touched[idx] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
}

/* getHigherMsb, CR/rasterizer_impl.cu:36-51 == bit_length(n) */
static unsigned higher_msb(uint32_t n) {
    unsigned b = 0;
    while (b < 32 && (n >> b)) b++;
    return b;
}

/* stable LSD radix sort on bits [0, end_bit) -- cub::DeviceRadixSort::SortPairs semantics */
static void radix_sort_pairs(uint64_t* keys, uint32_t* vals, size_t n, unsigned end_bit) {
    if (n == 0) return;
    uint64_t* k2 = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint32_t* v2 = (uint32_t*)malloc(n * sizeof(uint32_t));
    for (unsigned shift = 0; shift < end_bit; shift += 8) {
        unsigned bits = end_bit - shift < 8 ? end_bit - shift : 8;
        uint64_t mask = ((uint64_t)1 << bits) - 1;
        size_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        for (size_t i = 0; i < n; i++) cnt[((keys[i] >> shift) & mask) + 1]++;
        for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
        for (size_t i = 0; i < n; i++) {
            size_t dst = cnt[(keys[i] >> shift) & mask]++;
            k2[dst] = keys[i];
            v2[dst] = vals[i];
        }
        memcpy(keys, k2, n * sizeof(uint64_t));
        memcpy(vals, v2, n * sizeof(uint32_t));
    }
    free(k2);
    free(v2);
}

static void set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

/* Rasterizer::forward, CR/rasterizer_impl.cu:227-370 */
void* SYM(forward)(int P, int D, int M, const real* bg, int W, int H, const real* means3D, const real* shs,
                   const real* colors_precomp, const real* opacities, const real* scales, real scale_modifier,
                   const real* rotations, const real* cov3D_precomp, const real* viewmatrix, const real* projmatrix,
                   const real* campos, real tan_fovx, real tan_fovy, int prefiltered, int antialiasing,
                   real* out_color, real* out_invdepth, int* radii_out, int* num_rendered_out, int nthreads) {
    set_threads(nthreads);
    OracleState* s = (OracleState*)calloc(1, sizeof(OracleState));
    s->P = P; s->D = D; s->M = M; s->W = W; s->H = H;
    s->antialiasing = antialiasing; s->prefiltered = prefiltered;
    s->scale_modifier = scale_modifier; s->tan_fovx = tan_fovx; s->tan_fovy = tan_fovy;
    s->focal_y = (real)H / (R(2) * tan_fovy);
    s->focal_x = (real)W / (R(2) * tan_fovx);
    memcpy(s->bg, bg, 3 * sizeof(real));
    memcpy(s->view, viewmatrix, 16 * sizeof(real));
    memcpy(s->proj, projmatrix, 16 * sizeof(real));
    memcpy(s->campos, campos, 3 * sizeof(real));
    s->gx = (unsigned)((W + BLOCK_X - 1) / BLOCK_X);
    s->gy = (unsigned)((H + BLOCK_Y - 1) / BLOCK_Y);
    const size_t tiles = (size_t)s->gx * s->gy;
    s->means3D = dup_arr(means3D, (size_t)P * 3);
    s->shs = dup_arr(shs, (size_t)P * M * 3);
    s->colors_precomp = dup_arr(colors_precomp, (size_t)P * 3);
    s->opacities = dup_arr(opacities, (size_t)P);
    s->scales = dup_arr(scales, (size_t)P * 3);
    s->rotations = dup_arr(rotations, (size_t)P * 4);
    s->cov3D_precomp = dup_arr(cov3D_precomp, (size_t)P * 6);
    s->depths = (real*)calloc((size_t)P + 1, sizeof(real));
    s->means2D = (real*)calloc((size_t)P * 2 + 1, sizeof(real));
    s->cov3D = (real*)calloc((size_t)P * 6 + 1, sizeof(real));
    s->conic_opacity = (real*)calloc((size_t)P * 4 + 1, sizeof(real));
    s->rgb = (real*)calloc((size_t)P * 3 + 1, sizeof(real));
    s->clamped = (unsigned char*)calloc((size_t)P + 1, 1);
    s->radii = (int*)calloc((size_t)P + 1, sizeof(int));
    s->tiles_touched = (uint32_t*)calloc((size_t)P + 1, sizeof(uint32_t));
    s->point_offsets = (uint32_t*)calloc((size_t)P + 1, sizeof(uint32_t));
    s->ranges = (uint32_t*)calloc(tiles * 2 + 2, sizeof(uint32_t));
    s->final_T = (real*)calloc((size_t)W * H + 1, sizeof(real));
    s->n_contrib = (uint32_t*)calloc((size_t)W * H + 1, sizeof(uint32_t));

    /* RasterizeGaussiansCUDA: outputs zero-filled, P == 0 skips everything (RI/rasterize_points.cu:82-108) */
    memset(out_color, 0, sizeof(real) * 3 * (size_t)W * H);
    memset(out_invdepth, 0, sizeof(real) * (size_t)W * H);
    memset(radii_out, 0, sizeof(int) * (size_t)P);
    *num_rendered_out = 0;
    if (P == 0) return s;

#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; i++) preprocess_one(s, i);

    uint64_t acc = 0;
    for (int i = 0; i < P; i++) {
        acc += s->tiles_touched[i];
        s->point_offsets[i] = (uint32_t)acc;
    }
    int num_rendered = (int)s->point_offsets[P - 1];
    s->R = num_rendered;
    s->keys = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)num_rendered + 1));
    s->point_list = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)num_rendered + 1));
    /* duplicateWithKeys, CR/rasterizer_impl.cu:78-126 */
    for (int idx = 0; idx < P; idx++) {
        if (s->radii[idx] > 0) {
            uint32_t off = idx == 0 ? 0 : s->point_offsets[idx - 1];
            unsigned rmin[2], rmax[2];
            get_rect(s->means2D[2 * idx], s->means2D[2 * idx + 1], s->radii[idx], s->gx, s->gy, rmin, rmax);
            float dz = (float)s->depths[idx];
            uint32_t dbits;
            memcpy(&dbits, &dz, 4);
            for (unsigned y = rmin[1]; y < rmax[1]; y++)
                for (unsigned x = rmin[0]; x < rmax[0]; x++) {
                    uint64_t key = (uint64_t)(y * s->gx + x);
                    key <<= 32;
                    key |= dbits;
                    s->keys[off] = key;
                    s->point_list[off] = (uint32_t)idx;
                    off++;
                }
        }
    }
    radix_sort_pairs(s->keys, s->point_list, (size_t)num_rendered, 32 + higher_msb((uint32_t)tiles));
    /* identifyTileRanges, CR/rasterizer_impl.cu:132-164 (ranges zeroed first, :342) */
    for (int i = 0; i < num_rendered; i++) {
        uint32_t cur = (uint32_t)(s->keys[i] >> 32);
        if (i == 0)
            s->ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(s->keys[i - 1] >> 32);
            if (cur != prev) {
                s->ranges[2 * prev + 1] = (uint32_t)i;
                s->ranges[2 * cur] = (uint32_t)i;
            }
        }
        if (i == num_rendered - 1) s->ranges[2 * cur + 1] = (uint32_t)num_rendered;
    }
    /* renderCUDA (forward), CR/forward.cu:367-513; feature_ptr per CR/rasterizer_impl.cu:353 */
    const real* features = s->colors_precomp ? s->colors_precomp : s->rgb;
#pragma omp parallel for schedule(dynamic, 4)
    for (long tile = 0; tile < (long)tiles; tile++) {
        const unsigned tx = (unsigned)(tile % s->gx), ty = (unsigned)(tile / s->gx);
        const uint32_t r0 = s->ranges[2 * tile], r1 = s->ranges[2 * tile + 1];
        for (int ly = 0; ly < BLOCK_Y; ly++)
            for (int lx = 0; lx < BLOCK_X; lx++) {
                unsigned pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
                if (pxi >= (unsigned)W || pyi >= (unsigned)H) continue;
                const size_t pix_id = (size_t)W * pyi + pxi;
                const real pfx = (real)pxi, pfy = (real)pyi;
                real T = R(1);
                uint32_t contributor = 0, last_contributor = 0;
                real C[3] = {0, 0, 0};
                real invd = 0;
                for (uint32_t k = r0; k < r1; k++) {
                    contributor++;
                    const uint32_t g = s->point_list[k];
                    const real* xy = s->means2D + 2 * g;
                    const real* co = s->conic_opacity + 4 * g;
                    real dx = xy[0] - pfx, dy = xy[1] - pfy;
                    real power = R(-0.5) * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > R(0)) continue;
                    real alpha = FMINR(R(0.99), co[3] * EXP(power));
                    if (alpha < R(1) / R(255)) continue;
                    real test_T = T * (R(1) - alpha);
                    if (test_T < R(0.0001)) break; /* done = true; the loop ends for this pixel */
                    for (int ch = 0; ch < 3; ch++) C[ch] += features[3 * g + ch] * alpha * T;
                    invd += (R(1) / s->depths[g]) * alpha * T;
                    T = test_T;
                    last_contributor = contributor;
                }
                s->final_T[pix_id] = T;
                s->n_contrib[pix_id] = last_contributor;
                for (int ch = 0; ch < 3; ch++) out_color[(size_t)ch * H * W + pix_id] = C[ch] + T * s->bg[ch];
                out_invdepth[pix_id] = invd;
            }
    }
    for (int i = 0; i < P; i++) radii_out[i] = s->radii[i];
    *num_rendered_out = num_rendered;
    return s;
}

int SYM(prefilter_violation)(void* h) { return ((OracleState*)h)->prefilter_violation; }
int SYM(num_rendered)(void* h) { return ((OracleState*)h)->R; }

/* Accessors for stage-level comparisons (geometry / binning / image state). */
void SYM(get_geom)(void* h, real* depths, real* means2D, real* conic_opacity, real* rgb, uint32_t* tiles_touched,
                   unsigned char* clamped) {
    OracleState* s = (OracleState*)h;
    size_t P = (size_t)s->P;
    if (depths) memcpy(depths, s->depths, P * sizeof(real));
    if (means2D) memcpy(means2D, s->means2D, 2 * P * sizeof(real));
    if (conic_opacity) memcpy(conic_opacity, s->conic_opacity, 4 * P * sizeof(real));
    if (rgb) memcpy(rgb, s->rgb, 3 * P * sizeof(real));
    if (tiles_touched) memcpy(tiles_touched, s->tiles_touched, P * sizeof(uint32_t));
    if (clamped) memcpy(clamped, s->clamped, P);
}
void SYM(get_binning)(void* h, uint32_t* point_list, uint32_t* ranges) {
    OracleState* s = (OracleState*)h;
    if (point_list && s->R) memcpy(point_list, s->point_list, (size_t)s->R * sizeof(uint32_t));
    if (ranges) memcpy(ranges, s->ranges, (size_t)s->gx * s->gy * 2 * sizeof(uint32_t));
}
void SYM(get_image)(void* h, real* final_T, uint32_t* n_contrib) {
    OracleState* s = (OracleState*)h;
    size_t N = (size_t)s->W * s->H;
    if (final_T) memcpy(final_T, s->final_T, N * sizeof(real));
    if (n_contrib) memcpy(n_contrib, s->n_contrib, N * sizeof(uint32_t));
}

/* computeCov3D (CR/forward.cu:149-190) over P Gaussians, for pinning against the reference's
 * Python covariance (scene/gaussian_model.py:32-42 via utils/general_utils.py:78-110). */
void SYM(cov3d)(int P, const real* scales, real mod, const real* rotations, real* cov3D) {
    for (int i = 0; i < P; i++) cov3d_fwd(scales + 3 * i, mod, rotations + 4 * i, cov3D + 6 * i);
}

/* Distance of every pixel's blend (CR/forward.cu:455-500, walked exactly as the forward above)
 * to the reference's discrete thresholds, for explaining fp32 disagreements between two
 * implementations: per pixel, over the entries the loop visits up to and including its
 * termination, the minimum of |power| (the power > 0 skip), |alpha * 255 - 1| (the alpha < 1/255
 * skip; alpha before that test) and |test_T * 1e4 - 1| (the T < 1e-4 termination). */
void SYM(pixel_margins)(void* h, real* m_power, real* m_alpha, real* m_T, int nthreads) {
    OracleState* s = (OracleState*)h;
    set_threads(nthreads);
    const int W = s->W, H = s->H;
    const size_t tiles = (size_t)s->gx * s->gy;
#pragma omp parallel for schedule(dynamic, 4)
    for (long tile = 0; tile < (long)tiles; tile++) {
        const unsigned tx = (unsigned)(tile % s->gx), ty = (unsigned)(tile / s->gx);
        const uint32_t r0 = s->ranges[2 * tile], r1 = s->ranges[2 * tile + 1];
        for (int ly = 0; ly < BLOCK_Y; ly++)
            for (int lx = 0; lx < BLOCK_X; lx++) {
                unsigned pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
                if (pxi >= (unsigned)W || pyi >= (unsigned)H) continue;
                const size_t pix_id = (size_t)W * pyi + pxi;
                const real pfx = (real)pxi, pfy = (real)pyi;
                real T = R(1), mp = R(1e30), ma = R(1e30), mt = R(1e30);
                for (uint32_t k = r0; k < r1; k++) {
                    const uint32_t g = s->point_list[k];
                    const real* xy = s->means2D + 2 * g;
                    const real* co = s->conic_opacity + 4 * g;
                    real dx = xy[0] - pfx, dy = xy[1] - pfy;
                    real power = R(-0.5) * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    real ap = power < 0 ? -power : power;
                    if (ap < mp) mp = ap;
                    if (power > R(0)) continue;
                    real alpha = FMINR(R(0.99), co[3] * EXP(power));
                    real da = alpha * R(255) - R(1);
                    da = da < 0 ? -da : da;
                    if (da < ma) ma = da;
                    if (alpha < R(1) / R(255)) continue;
                    real test_T = T * (R(1) - alpha);
                    real dt = test_T * R(10000) - R(1);
                    dt = dt < 0 ? -dt : dt;
                    if (dt < mt) mt = dt;
                    if (test_T < R(0.0001)) break;
                    T = test_T;
                }
                m_power[pix_id] = mp;
                m_alpha[pix_id] = ma;
                m_T[pix_id] = mt;
            }
    }
}

/* The Gaussians whose own blend, at some pixel, comes within the given margins of one of the
 * reference's discrete thresholds (same walk and measures as pixel_margins): the power > 0 or
 * alpha < 1/255 skip of that Gaussian at that pixel, or the pixel terminating at it (T < 1e-4).
 * A different fp32 evaluation order may decide such an event the other way, which moves that
 * pixel's whole term in or out of the Gaussian's gradient.  flags[g] = 1 for those. */
void SYM(threshold_gaussians)(void* h, real mp, real ma, real mt, unsigned char* flags, int nthreads) {
    OracleState* s = (OracleState*)h;
    set_threads(nthreads);
    const int W = s->W, H = s->H;
    const size_t tiles = (size_t)s->gx * s->gy;
    memset(flags, 0, (size_t)s->P);
#pragma omp parallel for schedule(dynamic, 4)
    for (long tile = 0; tile < (long)tiles; tile++) {
        const unsigned tx = (unsigned)(tile % s->gx), ty = (unsigned)(tile / s->gx);
        const uint32_t r0 = s->ranges[2 * tile], r1 = s->ranges[2 * tile + 1];
        for (int ly = 0; ly < BLOCK_Y; ly++)
            for (int lx = 0; lx < BLOCK_X; lx++) {
                unsigned pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
                if (pxi >= (unsigned)W || pyi >= (unsigned)H) continue;
                const real pfx = (real)pxi, pfy = (real)pyi;
                real T = R(1);
                for (uint32_t k = r0; k < r1; k++) {
                    const uint32_t g = s->point_list[k];
                    const real* xy = s->means2D + 2 * g;
                    const real* co = s->conic_opacity + 4 * g;
                    real dx = xy[0] - pfx, dy = xy[1] - pfy;
                    real power = R(-0.5) * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    int near = (power < 0 ? -power : power) < mp;
                    if (power <= R(0)) {
                        real alpha = FMINR(R(0.99), co[3] * EXP(power));
                        real da = alpha * R(255) - R(1);
                        near |= (da < 0 ? -da : da) < ma;
                        if (alpha >= R(1) / R(255)) {
                            real test_T = T * (R(1) - alpha);
                            real dt = test_T * R(10000) - R(1);
                            near |= (dt < 0 ? -dt : dt) < mt;
                            if (near) {
#pragma omp atomic write
                                flags[g] = 1;
                            }
                            if (test_T < R(0.0001)) break;
                            T = test_T;
                            continue;
                        }
                    }
                    if (near) {
#pragma omp atomic write
                        flags[g] = 1;
                    }
                }
            }
    }
}

#if defined(_OPENMP)
#define ATOMIC_ADD(p, v) _Pragma("omp atomic") (p) += (v)
#else
#define ATOMIC_ADD(p, v) (p) += (v)
#endif

/* computeColorFromSH (backward), CR/backward.cu:12-146 */
static void color_from_sh_bwd(const OracleState* s, int idx, const real* dL_dcolor, real* dL_dmeans, real* dL_dshs) {
    const real* pos = s->means3D + 3 * idx;
    real dir_orig[3] = {pos[0] - s->campos[0], pos[1] - s->campos[1], pos[2] - s->campos[2]};
    real len = SQRT(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
    real dir[3] = {dir_orig[0] / len, dir_orig[1] / len, dir_orig[2] / len};
    const real* sh = s->shs + (size_t)idx * s->M * 3;
    real dL_dRGB[3];
    for (int c = 0; c < 3; c++) dL_dRGB[c] = dL_dcolor[3 * idx + c] * ((s->clamped[idx] >> c) & 1 ? R(0) : R(1));
    real dRGBdx[3] = {0, 0, 0}, dRGBdy[3] = {0, 0, 0}, dRGBdz[3] = {0, 0, 0};
    real x = dir[0], y = dir[1], z = dir[2];
    real* dL_dsh = dL_dshs + (size_t)idx * s->M * 3;
    const int deg = s->D;
#define SHV(k, c) sh[(k)*3 + (c)]
#define DSH(k, coef) for (int c = 0; c < 3; c++) dL_dsh[(k)*3 + c] = (coef) * dL_dRGB[c]
    DSH(0, SH_C0);
    if (deg > 0) {
        real d1 = -SH_C1 * y, d2 = SH_C1 * z, d3 = -SH_C1 * x;
        DSH(1, d1); DSH(2, d2); DSH(3, d3);
        for (int c = 0; c < 3; c++) {
            dRGBdx[c] = -SH_C1 * SHV(3, c);
            dRGBdy[c] = -SH_C1 * SHV(1, c);
            dRGBdz[c] = SH_C1 * SHV(2, c);
        }
        if (deg > 1) {
            real xx = x * x, yy = y * y, zz = z * z;
            real xy = x * y, yz = y * z, xz = x * z;
            real d4 = SH_C2[0] * xy, d5 = SH_C2[1] * yz, d6 = SH_C2[2] * (R(2) * zz - xx - yy);
            real d7 = SH_C2[3] * xz, d8 = SH_C2[4] * (xx - yy);
            DSH(4, d4); DSH(5, d5); DSH(6, d6); DSH(7, d7); DSH(8, d8);
            for (int c = 0; c < 3; c++) {
                dRGBdx[c] += SH_C2[0] * y * SHV(4, c) + SH_C2[2] * R(2) * -x * SHV(6, c) + SH_C2[3] * z * SHV(7, c) +
                             SH_C2[4] * R(2) * x * SHV(8, c);
                dRGBdy[c] += SH_C2[0] * x * SHV(4, c) + SH_C2[1] * z * SHV(5, c) + SH_C2[2] * R(2) * -y * SHV(6, c) +
                             SH_C2[4] * R(2) * -y * SHV(8, c);
                dRGBdz[c] += SH_C2[1] * y * SHV(5, c) + SH_C2[2] * R(2) * R(2) * z * SHV(6, c) + SH_C2[3] * x * SHV(7, c);
            }
            if (deg > 2) {
                real d9 = SH_C3[0] * y * (R(3) * xx - yy);
                real d10 = SH_C3[1] * xy * z;
                real d11 = SH_C3[2] * y * (R(4) * zz - xx - yy);
                real d12 = SH_C3[3] * z * (R(2) * zz - R(3) * xx - R(3) * yy);
                real d13 = SH_C3[4] * x * (R(4) * zz - xx - yy);
                real d14 = SH_C3[5] * z * (xx - yy);
                real d15 = SH_C3[6] * x * (xx - R(3) * yy);
                DSH(9, d9); DSH(10, d10); DSH(11, d11); DSH(12, d12); DSH(13, d13); DSH(14, d14); DSH(15, d15);
                for (int c = 0; c < 3; c++) {
                    dRGBdx[c] += (SH_C3[0] * SHV(9, c) * R(3) * R(2) * xy + SH_C3[1] * SHV(10, c) * yz +
                                  SH_C3[2] * SHV(11, c) * R(-2) * xy + SH_C3[3] * SHV(12, c) * R(-3) * R(2) * xz +
                                  SH_C3[4] * SHV(13, c) * (R(-3) * xx + R(4) * zz - yy) +
                                  SH_C3[5] * SHV(14, c) * R(2) * xz + SH_C3[6] * SHV(15, c) * R(3) * (xx - yy));
                    dRGBdy[c] += (SH_C3[0] * SHV(9, c) * R(3) * (xx - yy) + SH_C3[1] * SHV(10, c) * xz +
                                  SH_C3[2] * SHV(11, c) * (R(-3) * yy + R(4) * zz - xx) +
                                  SH_C3[3] * SHV(12, c) * R(-3) * R(2) * yz + SH_C3[4] * SHV(13, c) * R(-2) * xy +
                                  SH_C3[5] * SHV(14, c) * R(-2) * yz + SH_C3[6] * SHV(15, c) * R(-3) * R(2) * xy);
                    dRGBdz[c] += (SH_C3[1] * SHV(10, c) * xy + SH_C3[2] * SHV(11, c) * R(4) * R(2) * yz +
                                  SH_C3[3] * SHV(12, c) * R(3) * (R(2) * zz - xx - yy) +
                                  SH_C3[4] * SHV(13, c) * R(4) * R(2) * xz + SH_C3[5] * SHV(14, c) * (xx - yy));
                }
            }
        }
    }
#undef SHV
#undef DSH
    real dL_ddir[3] = {0, 0, 0};
    for (int c = 0; c < 3; c++) {
        dL_ddir[0] += dRGBdx[c] * dL_dRGB[c];
        dL_ddir[1] += dRGBdy[c] * dL_dRGB[c];
        dL_ddir[2] += dRGBdz[c] * dL_dRGB[c];
    }
    /* dnormvdv, CR/auxiliary.h:129-139 */
    const real* v = dir_orig;
    real sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    real invsum32 = R(1) / SQRT(sum2 * sum2 * sum2);
    const real* dv = dL_ddir;
    dL_dmeans[3 * idx + 0] += ((+sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
    dL_dmeans[3 * idx + 1] += (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
    dL_dmeans[3 * idx + 2] += (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

/* computeCov2DCUDA, CR/backward.cu:153-290, with the truncated tail (dL_dcov3D, dL_dmean3D) re-derived:
 * cov2D = A Sigma A^T with A = J(t) Rv (Rv = view rotation); see DESIGN.md. */
static void cov2d_bwd(OracleState* s, int idx, const real* cov3D, const real* dL_dconics, real* dL_dopacity,
                      const real* dL_dinvdepth, real* dL_dmeans, real* dL_dcov) {
    const real* mean = s->means3D + 3 * idx;
    real dL_dconic[3] = {dL_dconics[4 * idx], dL_dconics[4 * idx + 1], dL_dconics[4 * idx + 3]};
    real Tg[3][3], t[3], txtz, tytz;
    cov2d_T(s, mean, Tg, t, &txtz, &tytz);
    const real limx = R(1.3) * s->tan_fovx, limy = R(1.3) * s->tan_fovy;
    const real x_grad_mul = txtz < -limx || txtz > limx ? R(0) : R(1);
    const real y_grad_mul = tytz < -limy || tytz > limy ? R(0) : R(1);
    real V[3][3] = {{cov3D[0], cov3D[1], cov3D[2]}, {cov3D[1], cov3D[3], cov3D[4]}, {cov3D[2], cov3D[4], cov3D[5]}};
    real X[3][3], C[3][3];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) X[c][rr] = Tg[rr][0] * V[c][0] + Tg[rr][1] * V[c][1] + Tg[rr][2] * V[c][2];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) C[c][rr] = X[0][rr] * Tg[c][0] + X[1][rr] * Tg[c][1] + X[2][rr] * Tg[c][2];
    real c_xx = C[0][0], c_xy = C[0][1], c_yy = C[1][1];
    const real h_var = R(0.3);
    real d_inside_root = 0;
    if (s->antialiasing) {
        const real det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const real det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
        const real h_convolution_scaling = SQRT(FMAXR(R(0.000025), det_cov / det_cov_plus_h_cov));
        const real dL_dopacity_v = dL_dopacity[idx];
        const real d_h_convolution_scaling = dL_dopacity_v * s->opacities[idx];
        dL_dopacity[idx] = dL_dopacity_v * h_convolution_scaling;
        d_inside_root = (det_cov / det_cov_plus_h_cov) <= R(0.000025) ? R(0)
                                                                       : d_h_convolution_scaling / (R(2) * h_convolution_scaling);
    } else {
        c_xx += h_var;
        c_yy += h_var;
    }
    real dL_dc_xx = 0, dL_dc_xy = 0, dL_dc_yy = 0;
    if (s->antialiasing) {
        /* reference formula (CR/backward.cu:256-270), evaluated at the dilated x, y exactly as written there */
        const real x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const real q = w * w + w * (x + y) + x * y - z * z;
        const real denom_f = d_inside_root / (q * q);
        dL_dc_xx = w * (w * y + y * y + z * z) * denom_f;
        dL_dc_yy = w * (w * x + x * x + z * z) * denom_f;
        dL_dc_xy = R(-2) * w * z * (w + x + y) * denom_f;
    }
    real denom = c_xx * c_yy - c_xy * c_xy;
    real denom2inv = R(1) / ((denom * denom) + R(0.0000001));
    if (denom2inv != R(0)) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dL_dconic[0] + R(2) * c_xy * c_yy * dL_dconic[1] +
                                 (denom - c_xx * c_yy) * dL_dconic[2]);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dL_dconic[2] + R(2) * c_xx * c_xy * dL_dconic[1] +
                                 (denom - c_xx * c_yy) * dL_dconic[0]);
        dL_dc_xy += denom2inv * R(2) *
                    (c_xy * c_yy * dL_dconic[0] - (denom + R(2) * c_xy * c_xy) * dL_dconic[1] + c_xx * c_xy * dL_dconic[2]);
    }
    /* ---- re-derived tail ----
     * A[i][k] = Tg[i][k] (row i of the 2x3 projection A = J Rv, GLM column i).
     * cov_xx = A0 S A0^T, cov_xy = A0 S A1^T, cov_yy = A1 S A1^T. */
    const real a = dL_dc_xx, b = dL_dc_xy, c = dL_dc_yy;
    real A0[3] = {Tg[0][0], Tg[0][1], Tg[0][2]};
    real A1[3] = {Tg[1][0], Tg[1][1], Tg[1][2]};
    /* gradient w.r.t. the 6 stored (upper-triangle) covariance entries */
    dL_dcov[6 * idx + 0] = A0[0] * A0[0] * a + A0[0] * A1[0] * b + A1[0] * A1[0] * c;
    dL_dcov[6 * idx + 3] = A0[1] * A0[1] * a + A0[1] * A1[1] * b + A1[1] * A1[1] * c;
    dL_dcov[6 * idx + 5] = A0[2] * A0[2] * a + A0[2] * A1[2] * b + A1[2] * A1[2] * c;
    dL_dcov[6 * idx + 1] = R(2) * A0[0] * A0[1] * a + (A0[0] * A1[1] + A0[1] * A1[0]) * b + R(2) * A1[0] * A1[1] * c;
    dL_dcov[6 * idx + 2] = R(2) * A0[0] * A0[2] * a + (A0[0] * A1[2] + A0[2] * A1[0]) * b + R(2) * A1[0] * A1[2] * c;
    dL_dcov[6 * idx + 4] = R(2) * A0[2] * A0[1] * a + (A0[1] * A1[2] + A0[2] * A1[1]) * b + R(2) * A1[1] * A1[2] * c;
    /* dL/dA0 = 2a S A0 + b S A1 ; dL/dA1 = 2c S A1 + b S A0 */
    real SA0[3], SA1[3], dA0[3], dA1[3];
    for (int k = 0; k < 3; k++) {
        SA0[k] = V[k][0] * A0[0] + V[k][1] * A0[1] + V[k][2] * A0[2];
        SA1[k] = V[k][0] * A1[0] + V[k][1] * A1[1] + V[k][2] * A1[2];
    }
    for (int k = 0; k < 3; k++) {
        dA0[k] = R(2) * a * SA0[k] + b * SA1[k];
        dA1[k] = R(2) * c * SA1[k] + b * SA0[k];
    }
    /* A = J Rv with Rv row r = (view[r], view[4+r], view[8+r]);  J = [[j00,0,j02],[0,j11,j12]] */
    const real* v = s->view;
    real Rv[3][3] = {{v[0], v[4], v[8]}, {v[1], v[5], v[9]}, {v[2], v[6], v[10]}};
    real dJ00 = dA0[0] * Rv[0][0] + dA0[1] * Rv[0][1] + dA0[2] * Rv[0][2];
    real dJ02 = dA0[0] * Rv[2][0] + dA0[1] * Rv[2][1] + dA0[2] * Rv[2][2];
    real dJ11 = dA1[0] * Rv[1][0] + dA1[1] * Rv[1][1] + dA1[2] * Rv[1][2];
    real dJ12 = dA1[0] * Rv[2][0] + dA1[1] * Rv[2][1] + dA1[2] * Rv[2][2];
    const real fx = s->focal_x, fy = s->focal_y;
    real tz = R(1) / t[2];
    real tz2 = tz * tz, tz3 = tz2 * tz;
    real dL_dtx = x_grad_mul * -fx * tz2 * dJ02;
    real dL_dty = y_grad_mul * -fy * tz2 * dJ12;
    real dL_dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (R(2) * fx * t[0]) * tz3 * dJ02 + (R(2) * fy * t[1]) * tz3 * dJ12;
    if (dL_dinvdepth) dL_dtz -= dL_dinvdepth[idx] / (t[2] * t[2]);
    /* transformVec4x3Transpose, CR/auxiliary.h:109-117 */
    dL_dmeans[3 * idx + 0] = v[0] * dL_dtx + v[1] * dL_dty + v[2] * dL_dtz;
    dL_dmeans[3 * idx + 1] = v[4] * dL_dtx + v[5] * dL_dty + v[6] * dL_dtz;
    dL_dmeans[3 * idx + 2] = v[8] * dL_dtx + v[9] * dL_dty + v[10] * dL_dtz;
}

/* computeCov3D (backward), CR/backward.cu:296-365 */
static void cov3d_bwd(const OracleState* s, int idx, const real* dL_dcov3Ds, real* dL_dscales, real* dL_drots) {
    const real* rot = s->rotations + 4 * idx;
    const real* scale = s->scales + 3 * idx;
    real r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    real Rg[3][3] = {{R(1) - R(2) * (y * y + z * z), R(2) * (x * y - r * z), R(2) * (x * z + r * y)},
                     {R(2) * (x * y + r * z), R(1) - R(2) * (x * x + z * z), R(2) * (y * z - r * x)},
                     {R(2) * (x * z - r * y), R(2) * (y * z + r * x), R(1) - R(2) * (x * x + y * y)}};
    real sv[3] = {s->scale_modifier * scale[0], s->scale_modifier * scale[1], s->scale_modifier * scale[2]};
    real Mg[3][3];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) Mg[c][rr] = sv[rr] * Rg[c][rr];
    const real* g = dL_dcov3Ds + 6 * idx;
    /* dL_dSigma (GLM, symmetric) */
    real dS[3][3] = {{g[0], R(0.5) * g[1], R(0.5) * g[2]},
                     {R(0.5) * g[1], g[3], R(0.5) * g[4]},
                     {R(0.5) * g[2], R(0.5) * g[4], g[5]}};
    /* dL_dM = 2 * M * dL_dSigma (GLM product) : P[c][r] = sum_k M[k][r] dS[c][k] */
    real dM[3][3];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) dM[c][rr] = R(2) * (Mg[0][rr] * dS[c][0] + Mg[1][rr] * dS[c][1] + Mg[2][rr] * dS[c][2]);
    /* Rt = transpose(R), dL_dMt = transpose(dL_dM) */
    real Rt[3][3], dMt[3][3];
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) {
            Rt[c][rr] = Rg[rr][c];
            dMt[c][rr] = dM[rr][c];
        }
    /* scale gradient: dot(Rt[i], dL_dMt[i]); the reference does not apply the scale modifier here */
    for (int i = 0; i < 3; i++) dL_dscales[3 * idx + i] = Rt[i][0] * dMt[i][0] + Rt[i][1] * dMt[i][1] + Rt[i][2] * dMt[i][2];
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) dMt[i][k] *= sv[i];
    real* q = dL_drots + 4 * idx;
    q[0] = R(2) * z * (dMt[0][1] - dMt[1][0]) + R(2) * y * (dMt[2][0] - dMt[0][2]) + R(2) * x * (dMt[1][2] - dMt[2][1]);
    q[1] = R(2) * y * (dMt[1][0] + dMt[0][1]) + R(2) * z * (dMt[2][0] + dMt[0][2]) + R(2) * r * (dMt[1][2] - dMt[2][1]) -
           R(4) * x * (dMt[2][2] + dMt[1][1]);
    q[2] = R(2) * x * (dMt[1][0] + dMt[0][1]) + R(2) * r * (dMt[2][0] - dMt[0][2]) + R(2) * z * (dMt[1][2] + dMt[2][1]) -
           R(4) * y * (dMt[2][2] + dMt[0][0]);
    q[3] = R(2) * r * (dMt[0][1] - dMt[1][0]) + R(2) * x * (dMt[2][0] + dMt[0][2]) + R(2) * y * (dMt[1][2] + dMt[2][1]) -
           R(4) * z * (dMt[1][1] + dMt[0][0]);
}

/* Rasterizer::backward, CR/rasterizer_impl.cu:374-479 + RasterizeGaussiansBackwardCUDA zero-init
 * (RI/rasterize_points.cu:186-204).  Output arrays are overwritten (zeroed first). */
void SYM(backward)(void* h, const real* dL_dpix, const real* dL_dinvdepths, real* dL_dmean2D /*P*3*/,
                   real* dL_dconic /*P*4*/, real* dL_dopacity /*P*/, real* dL_dcolor /*P*3*/,
                   real* dL_dinvdepth /*P, may be NULL*/, real* dL_dmean3D /*P*3*/, real* dL_dcov3D /*P*6*/,
                   real* dL_dsh /*P*M*3*/, real* dL_dscale /*P*3*/, real* dL_drot /*P*4*/, int nthreads) {
    OracleState* s = (OracleState*)h;
    set_threads(nthreads);
    const int P = s->P, W = s->W, H = s->H;
    memset(dL_dmean2D, 0, sizeof(real) * 3 * (size_t)P);
    memset(dL_dconic, 0, sizeof(real) * 4 * (size_t)P);
    memset(dL_dopacity, 0, sizeof(real) * (size_t)P);
    memset(dL_dcolor, 0, sizeof(real) * 3 * (size_t)P);
    if (dL_dinvdepth) memset(dL_dinvdepth, 0, sizeof(real) * (size_t)P);
    memset(dL_dmean3D, 0, sizeof(real) * 3 * (size_t)P);
    memset(dL_dcov3D, 0, sizeof(real) * 6 * (size_t)P);
    memset(dL_dsh, 0, sizeof(real) * 3 * (size_t)P * s->M);
    memset(dL_dscale, 0, sizeof(real) * 3 * (size_t)P);
    memset(dL_drot, 0, sizeof(real) * 4 * (size_t)P);
    if (P == 0) return;
    const real* inv_in = dL_dinvdepth ? dL_dinvdepths : NULL; /* reference: only when grad_out_depth is non-empty */
    const real* colors = s->colors_precomp ? s->colors_precomp : s->rgb;
    const size_t tiles = (size_t)s->gx * s->gy;
    const real ddelx_dx = R(0.5) * W, ddely_dy = R(0.5) * H;
    /* renderCUDA (backward), CR/backward.cu:433-612 */
#pragma omp parallel for schedule(dynamic, 4)
    for (long tile = 0; tile < (long)tiles; tile++) {
        const unsigned tx = (unsigned)(tile % s->gx), ty = (unsigned)(tile / s->gx);
        const uint32_t r0 = s->ranges[2 * tile], r1 = s->ranges[2 * tile + 1];
        for (int ly = 0; ly < BLOCK_Y; ly++)
            for (int lx = 0; lx < BLOCK_X; lx++) {
                unsigned pxi = tx * BLOCK_X + lx, pyi = ty * BLOCK_Y + ly;
                if (pxi >= (unsigned)W || pyi >= (unsigned)H) continue;
                const size_t pix_id = (size_t)W * pyi + pxi;
                const real pfx = (real)pxi, pfy = (real)pyi;
                const real T_final = s->final_T[pix_id];
                real T = T_final;
                uint32_t contributor = r1 - r0;
                const uint32_t last_contributor = s->n_contrib[pix_id];
                real accum_rec[3] = {0, 0, 0}, dL_dpixel[3], dL_invd = 0, accum_invd_rec = 0;
                for (int c = 0; c < 3; c++) dL_dpixel[c] = dL_dpix[(size_t)c * H * W + pix_id];
                if (inv_in) dL_invd = inv_in[pix_id];
                real last_alpha = 0, last_color[3] = {0, 0, 0}, last_invd = 0;
                for (uint32_t k = r1; k > r0; k--) {
                    contributor--;
                    if (contributor >= last_contributor) continue;
                    const uint32_t g = s->point_list[k - 1];
                    const real* xy = s->means2D + 2 * g;
                    const real* co = s->conic_opacity + 4 * g;
                    const real dx = xy[0] - pfx, dy = xy[1] - pfy;
                    const real power = R(-0.5) * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > R(0)) continue;
                    const real G = EXP(power);
                    const real alpha = FMINR(R(0.99), co[3] * G);
                    if (alpha < R(1) / R(255)) continue;
                    T = T / (R(1) - alpha);
                    const real dchannel_dcolor = alpha * T;
                    real dL_dalpha = 0;
                    for (int ch = 0; ch < 3; ch++) {
                        const real cc = colors[3 * g + ch];
                        accum_rec[ch] = last_alpha * last_color[ch] + (R(1) - last_alpha) * accum_rec[ch];
                        last_color[ch] = cc;
                        dL_dalpha += (cc - accum_rec[ch]) * dL_dpixel[ch];
                        ATOMIC_ADD(dL_dcolor[3 * g + ch], dchannel_dcolor * dL_dpixel[ch]);
                    }
                    if (inv_in) {
                        const real invd = R(1) / s->depths[g];
                        accum_invd_rec = last_alpha * last_invd + (R(1) - last_alpha) * accum_invd_rec;
                        last_invd = invd;
                        dL_dalpha += (invd - accum_invd_rec) * dL_invd;
                        ATOMIC_ADD(dL_dinvdepth[g], dchannel_dcolor * dL_invd);
                    }
                    dL_dalpha *= T;
                    last_alpha = alpha;
                    real bg_dot_dpixel = 0;
                    for (int c = 0; c < 3; c++) bg_dot_dpixel += s->bg[c] * dL_dpixel[c];
                    dL_dalpha += (-T_final / (R(1) - alpha)) * bg_dot_dpixel;
                    const real dL_dG = co[3] * dL_dalpha;
                    const real gdx = G * dx, gdy = G * dy;
                    const real dG_ddelx = -gdx * co[0] - gdy * co[1];
                    const real dG_ddely = -gdy * co[2] - gdx * co[1];
                    ATOMIC_ADD(dL_dmean2D[3 * g + 0], dL_dG * dG_ddelx * ddelx_dx);
                    ATOMIC_ADD(dL_dmean2D[3 * g + 1], dL_dG * dG_ddely * ddely_dy);
                    ATOMIC_ADD(dL_dconic[4 * g + 0], R(-0.5) * gdx * dx * dL_dG);
                    ATOMIC_ADD(dL_dconic[4 * g + 1], R(-0.5) * gdx * dy * dL_dG);
                    ATOMIC_ADD(dL_dconic[4 * g + 3], R(-0.5) * gdy * dy * dL_dG);
                    ATOMIC_ADD(dL_dopacity[g], G * dL_dalpha);
                }
            }
    }
    /* BACKWARD::preprocess, CR/backward.cu:614-657: computeCov2DCUDA then preprocessCUDA */
    const real* cov3D_ptr = s->cov3D_precomp ? s->cov3D_precomp : s->cov3D;
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(s->radii[idx] > 0)) continue;
        cov2d_bwd(s, idx, cov3D_ptr + 6 * (size_t)idx, dL_dconic, dL_dopacity, inv_in ? dL_dinvdepth : NULL, dL_dmean3D, dL_dcov3D);
        /* preprocessCUDA (backward), CR/backward.cu:372-429 */
        const real* m = s->means3D + 3 * idx;
        const real* proj = s->proj;
        real m_hom[4];
        xform44(m, proj, m_hom);
        real m_w = R(1) / (m_hom[3] + R(0.0000001));
        real mul1 = (proj[0] * m[0] + proj[4] * m[1] + proj[8] * m[2] + proj[12]) * m_w * m_w;
        real mul2 = (proj[1] * m[0] + proj[5] * m[1] + proj[9] * m[2] + proj[13]) * m_w * m_w;
        const real* d2 = dL_dmean2D + 3 * idx;
        dL_dmean3D[3 * idx + 0] += (proj[0] * m_w - proj[3] * mul1) * d2[0] + (proj[1] * m_w - proj[3] * mul2) * d2[1];
        dL_dmean3D[3 * idx + 1] += (proj[4] * m_w - proj[7] * mul1) * d2[0] + (proj[5] * m_w - proj[7] * mul2) * d2[1];
        dL_dmean3D[3 * idx + 2] += (proj[8] * m_w - proj[11] * mul1) * d2[0] + (proj[9] * m_w - proj[11] * mul2) * d2[1];
        if (s->shs) color_from_sh_bwd(s, idx, dL_dcolor, dL_dmean3D, dL_dsh);
        if (s->scales) cov3d_bwd(s, idx, dL_dcov3D, dL_dscale, dL_drot);
    }
}

/* markVisible / checkFrustum, CR/rasterizer_impl.cu:56-73,169-181 */
void SYM(mark_visible)(int P, const real* means3D, const real* viewmatrix, unsigned char* present) {
    for (int i = 0; i < P; i++) {
        real pv[3];
        xform43(means3D + 3 * i, viewmatrix, pv);
        present[i] = pv[2] > R(0.2) ? 1 : 0;
    }
}

void SYM(free)(void* h) {
    OracleState* s = (OracleState*)h;
    if (!s) return;
    free(s->means3D); free(s->shs); free(s->colors_precomp); free(s->opacities); free(s->scales);
    free(s->rotations); free(s->cov3D_precomp); free(s->depths); free(s->means2D); free(s->cov3D);
    free(s->conic_opacity); free(s->rgb); free(s->clamped); free(s->radii); free(s->tiles_touched);
    free(s->point_offsets); free(s->keys); free(s->point_list); free(s->ranges); free(s->final_T);
    free(s->n_contrib);
    free(s);
}
