/*
 * gsr_densify.h -- C ABI of adaptive density control on MI355X (gfx950).
 *
 * The reference grows and prunes its Gaussians in torch (scene/gaussian_model.py:
 * add_densification_stats :643-654, densify_and_prune :574-640 with densify_and_clone
 * :552-571, densify_and_split :508-550, prune_points :420-437, _prune_optimizer :400-418,
 * cat_tensors_to_optimizer :439-481, densification_postfix :483-506) and updates max_radii2D in train.py:212-213.
 * SURVEY.md section 8f row 4.  These entry points do the same work in three launches
 * plus one 40-byte host read, on the torch stream:
 *
 *   gsr_densify_stats   <- train.py:212-215: max_radii2D[vis] = max(max_radii2D[vis], radii[vis]);
 *                          add_densification_stats: grad_accum[vis] += ||dmeans2D[vis, :2]||,
 *                          denom[vis] += 1
 *   gsr_densify_plan    <- the decisions of densify_and_prune: grads = accum / denom (NaN -> 0);
 *                          clone: grad >= max_grad and max(exp(scaling)) <= percent_dense * extent;
 *                          split: grad >= max_grad and max(exp(scaling)) >  percent_dense * extent;
 *                          prune: sigmoid(opacity) < min_opacity, or (max_screen_size set) a
 *                          world-space scale > 0.1 * extent.  (The screen-size test of the
 *                          reference compares max_radii2D, which densification_postfix has just
 *                          zeroed, so it never prunes; that is kept.)  Writes the per-Gaussian
 *                          output rows into scratch and returns the counts to the host.
 *   gsr_densify_apply   <- the tensor surgery: the new parameter arrays and Adam states in the
 *                          reference's order: kept originals, kept clones, kept children of the
 *                          first split copy, kept children of the second; new rows get zero
 *                          Adam moments (cat_tensors_to_optimizer), kept rows keep theirs.
 *                          Children: xyz = R(q) * sample + xyz, scaling = log(exp(s) / (0.8 N)).
 *
 * The normal samples of the split are drawn by the caller exactly as the reference draws them
 * (torch.normal(mean=zeros(2 ns, 3), std=get_scaling[split].repeat(2, 1)),
 * gaussian_model.py:520-528), so a seeded run consumes the same random numbers.
 *
 * All pointers are device pointers to contiguous arrays unless stated; work is enqueued on
 * `stream` (hipStream_t).  Returns 0 or a GSR_ERR_* code (include/gsr.h).
 */
#ifndef GSR_DENSIFY_H_INCLUDED
#define GSR_DENSIFY_H_INCLUDED

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_DENSIFY_MAX_GROUPS 8

/* what a parameter group's children rows are */
#define GSR_DENSIFY_COPY 0    /* the parent's row (f_dc, f_rest, opacity, rotation) */
#define GSR_DENSIFY_XYZ 1     /* R(q) * sample + xyz (needs the rotation and the samples) */
#define GSR_DENSIFY_SCALING 2 /* log(exp(s) / split_div) */

typedef struct gsr_densify_group {
    const float* src;            /* [P][width] */
    float* dst;                  /* [P_new][width] */
    const float* src_exp_avg;    /* Adam moments [P][width], or NULL when the group has no state yet */
    const float* src_exp_avg_sq;
    float* dst_exp_avg;          /* [P_new][width]; NULL iff src_exp_avg is NULL */
    float* dst_exp_avg_sq;
    int width;                   /* floats per Gaussian */
    int role;                    /* GSR_DENSIFY_COPY / _XYZ / _SCALING */
} gsr_densify_group;

typedef struct gsr_densify_params {
    float grad_threshold;  /* max_grad */
    float clone_extent;    /* percent_dense * extent (computed in double, as torch compares) */
    float min_opacity;
    float big_extent;      /* 0.1 * extent */
    int use_screen_size;   /* max_screen_size is truthy (enables the world-space test) */
    int split_n;           /* N = 2 */
    float split_div;       /* 0.8 * N */
} gsr_densify_params;

/* counts written by gsr_densify_plan */
#define GSR_DENSIFY_KEPT 0      /* originals kept (neither split nor pruned) */
#define GSR_DENSIFY_CLONES 1    /* clones kept */
#define GSR_DENSIFY_CHILDREN 2  /* children kept per split copy */
#define GSR_DENSIFY_SPLIT 3     /* originals split (samples are drawn for split_n * this many rows) */
#define GSR_DENSIFY_TOTAL 4     /* P_new = KEPT + CLONES + split_n * CHILDREN */
#define GSR_DENSIFY_NCOUNTS 5

/* radii: [P] int (visibility = radii > 0, max_radii2D updated) or NULL with `visible` given;
   visible: [P] bytes, or NULL (then radii > 0); viewspace_grad: [P][3] (dL/dmeans2D), or NULL
   to update max_radii2D only (grad_accum / denom then unused). */
int gsr_densify_stats(int P, const float* viewspace_grad, const int* radii, const unsigned char* visible,
                      float* grad_accum, float* denom, float* max_radii2D, void* stream);

/* device scratch that gsr_densify_plan fills and gsr_densify_apply reads */
unsigned long long gsr_densify_scratch_bytes(int P);

/* grad_accum, denom: [P]; opacity: [P] raw (pre-sigmoid); scaling: [P][3] raw (log);
   split_mask: [P] bytes out (1 = split), may be NULL; counts: host array of GSR_DENSIFY_NCOUNTS.
   Synchronises with the stream once (the counts). */
int gsr_densify_plan(int P, const float* grad_accum, const float* denom, const float* opacity, const float* scaling,
                     const gsr_densify_params* prm, void* scratch, unsigned char* split_mask, long long* counts,
                     void* stream);

/* rotation: [P][4] raw quaternions (children's xyz); samples: [split_n * n_split][3];
   tmp_radii_in [P] / tmp_radii_out [P_new] int, both NULL or both set. */
int gsr_densify_apply(int P, const void* scratch, const gsr_densify_group* groups, int n_groups,
                      const float* rotation, const float* samples, const int* tmp_radii_in, int* tmp_radii_out,
                      const gsr_densify_params* prm, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GSR_DENSIFY_H_INCLUDED */
