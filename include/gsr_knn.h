/*
 * gsr_knn.h -- C ABI of the MI355X (gfx950) replacement for the reference's
 * simple-knn extension (mango1118/gaussian_splatting, submodules/simple-knn).
 *
 *   gsr_knn_mean_dist2  <- SimpleKNN::knn (simple_knn.h:14-20, simple_knn.cu:172-221)
 *                          and distCUDA2 (spatial.cu:14-25), the one function the
 *                          pybind module exports (ext.cpp:14-17).  The reference's
 *                          only caller is GaussianModel.create_from_pcd
 *                          (scene/gaussian_model.py:198), which uses it to size the
 *                          initial Gaussians.
 *
 * For each of P points, the mean of the squared distances to its 3 nearest other
 * points (indices differ; duplicates count as distance 0).  With fewer than three
 * other points the missing distances are FLT_MAX, as in the reference.  Results are
 * exact nearest neighbours: the spatial structure (Morton order, boxes) only prunes.
 *
 * Conventions as gsr.h: device pointers to contiguous fp32 data, scratch memory
 * through an allocation callback (freed by the caller after the call returns; the
 * stream is synchronised before returning), work on `stream`.
 */
#ifndef GSR_KNN_H_INCLUDED
#define GSR_KNN_H_INCLUDED

#include <stddef.h>

#include "gsr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* points: [P][3] fp32 (device); mean_dists: [P] fp32 (device), every element written. */
int gsr_knn_mean_dist2(int P, const float* points, float* mean_dists, gsr_alloc_fn scratch_alloc,
                       void* scratch_ctx, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GSR_KNN_H_INCLUDED */
