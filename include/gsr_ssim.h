/*
 * gsr_ssim.h -- C ABI of the MI355X (gfx950) fused SSIM, the replacement for the
 * reference's fused-ssim extension (mango1118/gaussian_splatting, submodules/fused-ssim).
 *
 *   gsr_fused_ssim_forward   <- fusedssim (ssim.h:8-15, ssim.cu:368-404 + kernel :210-313;
 *                               pybind ext.cpp:4-7)
 *   gsr_fused_ssim_backward  <- fusedssim_backward (ssim.h:17-27, ssim.cu:406-444 + kernel
 *                               :315-366; ext.cpp:4-7)
 *
 * Images are [B][CH][H][W] contiguous fp32 device arrays (the reference takes 4-D NCHW
 * tensors).  The SSIM map uses an 11x11 Gaussian window (sigma 1.5) with zero padding
 * ("same"); the "valid" crop is done by the caller, as in the reference's Python.
 * Forward: dm_dmu1 / dm_dsigma1_sq / dm_dsigma12 are written when non-NULL (train=True);
 * pass all three or none.  Backward: dL/dimg1 from dL/dmap and those three maps.
 * Every output element is written.  Work is enqueued on `stream`.
 */
#ifndef GSR_SSIM_H_INCLUDED
#define GSR_SSIM_H_INCLUDED

#include "gsr.h"

#ifdef __cplusplus
extern "C" {
#endif

int gsr_fused_ssim_forward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, void* stream);

int gsr_fused_ssim_backward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                            const float* dL_dmap, const float* dm_dmu1, const float* dm_dsigma1_sq,
                            const float* dm_dsigma12, float* dL_dimg1, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GSR_SSIM_H_INCLUDED */
