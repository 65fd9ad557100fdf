/*
 * gsr_adam.h -- C ABI of the sparse Adam step on MI355X (gfx950).
 *
 * The reference's train.py steps its optimizer with `optimizer.step(visible, N)` when
 * `--optimizer_type sparse_adam` is chosen and diff_gaussian_rasterization exports
 * SparseGaussianAdam (train.py:41-45,74,240-246; scene/gaussian_model.py:246-251).
 * That class belongs to the 3DGS-accel build of the rasterizer, which the reference
 * does not vendor.  Its per-group native call is
 *
 *     _C.adamUpdate(param, param.grad, exp_avg, exp_avg_sq, visible, lr, 0.9, 0.999, eps, N, M)
 *
 * with M = param.numel() / N values per Gaussian.  For every element i < N*M whose
 * Gaussian g = i / M is visible (visible[g] != 0):
 *
 *     m  = b1 * m + (1 - b1) * grad
 *     v  = b2 * v + (1 - b2) * grad * grad
 *     param += -lr * m / (sqrt(v) + eps)
 *
 * (no bias correction, no step counter); elements of invisible Gaussians are not
 * touched.  fp32, IEEE division and square root, no fused multiply-add contraction.
 *
 *   gsr_adam_update        <- _C.adamUpdate (one parameter tensor)
 *   gsr_adam_update_multi  <- SparseGaussianAdam.step's loop over its param groups,
 *                             fused into one launch (up to GSR_ADAM_MAX_GROUPS groups)
 *
 * Pointers are device pointers to contiguous fp32 arrays (visible: N bytes, bool);
 * work is enqueued on `stream` (hipStream_t).  Returns 0 or a GSR_ERR_* code
 * (include/gsr.h); gsr_last_error() has the message.
 */
#ifndef GSR_ADAM_H_INCLUDED
#define GSR_ADAM_H_INCLUDED

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ADAM_MAX_GROUPS 8

typedef struct gsr_adam_group {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long long numel; /* N * M */
    int M;           /* values per Gaussian */
    float lr;
    float eps;
} gsr_adam_group;

int gsr_adam_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const unsigned char* visible,
                    float lr, float b1, float b2, float eps, int N, int M, void* stream);

int gsr_adam_update_multi(const gsr_adam_group* groups, int n_groups, const unsigned char* visible, int N, float b1,
                          float b2, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GSR_ADAM_H_INCLUDED */
