// kernels.h -- launch arguments and entry points shared by the .hip translation units.
#pragma once

#include "gsr_common.h"

namespace gsr {

struct PreprocessArgs {
    int P, D, M, W, H;
    const float* means3D;
    const float* scales;
    float scale_modifier;
    const float* rotations;
    const float* opacities;
    const float* shs;
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    uint32_t gx, gy;
    int prefiltered, antialiasing, footprint_cull;
    int* radii;
    GeomState geom;
};

struct RenderFwdArgs {
    int W, H;
    uint32_t gx, gy;
    const uint2* ranges;
    uint32_t* gid_sorted;  // the forward writes each staged entry's quadrant mask into its low bits
    const float4* rec;
    const float* bg;
    float* out_color;
    float* out_invdepth;
    ImageState img;
};

struct RenderBwdArgs {
    int W, H;
    uint32_t gx, gy;
    const uint2* ranges;
    const uint32_t* gid_sorted;
    const float4* rec;
    const float* bg;
    const float* dL_dpix;       // [3,H,W]
    const float* dL_dinvdepth;  // [H,W] or null
    ImageState img;
    GradRecs recs;
    const uint32_t* depth_key;          // per Gaussian
    unsigned long long* lim_key;        // [tiles] out: key of the last entry that has a record (0: none)
};

struct GaussBwdArgs {
    int P, D, M, W, H;
    const float* means3D;
    const float* shs;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    float scale_modifier;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    int antialiasing;
    const int* radii;
    GeomState geom;
    GradRecs sums;  // per Gaussian: summed render gradients (gauss_reduce_kernel)
    int have_invdepth;
    float* dL_dmean2D;    // [P,3]
    float* dL_dconic;     // [P,4] or null
    float* dL_dopacity;   // [P]
    float* dL_dcolor;     // [P,3]
    float* dL_dinvdepth;  // [P] or null
    float* dL_dmean3D;    // [P,3]
    float* dL_dcov3D;     // [P,6]
    float* dL_dsh;        // [P,M,3] or null (M == 0)
    float* dL_dscale;     // [P,3] or null
    float* dL_drot;       // [P,4] or null
};

// preprocess.hip
hipError_t launch_preprocess(const PreprocessArgs& a, hipStream_t stream);
hipError_t launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t stream);
// binning.hip
size_t bin_chunk_count(int P);
size_t bin_cell_count(uint32_t gx, uint32_t gy);
hipError_t launch_bin_count(int P, const GeomState& g, uint32_t gx, uint32_t gy, uint2* ranges, size_t cap,
                            hipStream_t stream);
hipError_t launch_bin_scatter(int P, const GeomState& g, uint32_t gx, uint32_t gy, const BinningState& b, size_t cap,
                              hipStream_t stream);
hipError_t launch_tile_sort(uint32_t tiles, const uint2* ranges, const GeomState& g, const BinningState& b,
                            size_t cap, hipStream_t stream);
// render.hip
hipError_t launch_render_fwd(const RenderFwdArgs& a, hipStream_t stream);
hipError_t launch_render_bwd(const RenderBwdArgs& a, hipStream_t stream);
hipError_t launch_tile_order(uint32_t tiles, const uint32_t* cost, uint32_t* order, hipStream_t stream);
// knn.hip
size_t knn_scratch_bytes(int P);
hipError_t launch_knn(int P, const float* pts, float* out, void* scratch, hipStream_t stream);
// ssim.hip
hipError_t launch_ssim_fwd(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* map, float* dm_dmu1, float* dm_ds11, float* dm_ds12, hipStream_t stream);
hipError_t launch_ssim_bwd(int planes, int H, int W, const float* img1, const float* img2, const float* dL_dmap,
                           const float* dm_dmu1, const float* dm_ds11, const float* dm_ds12, float* dL_dimg1,
                           hipStream_t stream);
// backward.hip
hipError_t launch_gauss_reduce(int P, const GeomState& g, uint32_t gx, const unsigned long long* lim_key,
                               const GradRecs& recs, const GradRecs& sums, hipStream_t stream);
hipError_t launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t stream);

}  // namespace gsr
