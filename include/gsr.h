/*
 * gsr.h -- C ABI of the MI355X (gfx950) differentiable Gaussian tile rasterizer.
 *
 * This is the drop-in boundary for the reference's native rasterizer
 * (mango1118/gaussian_splatting, submodules/diff-gaussian-rasterization).  Each
 * entry point replaces one C++ interface of the reference:
 *
 *   gsr_rasterize_forward   <- CudaRasterizer::Rasterizer::forward
 *                              (cuda_rasterizer/rasterizer.h:31-58,
 *                               cuda_rasterizer/rasterizer_impl.cu:227-370)
 *   gsr_rasterize_backward  <- CudaRasterizer::Rasterizer::backward
 *                              (cuda_rasterizer/rasterizer.h:60-91,
 *                               cuda_rasterizer/rasterizer_impl.cu:374-479)
 *   gsr_mark_visible        <- CudaRasterizer::Rasterizer::markVisible
 *                              (cuda_rasterizer/rasterizer.h:23-29,
 *                               cuda_rasterizer/rasterizer_impl.cu:169-181)
 *
 * and, one layer up, the three pybind functions of ext.cpp:15-19
 * (rasterize_gaussians / rasterize_gaussians_backward / mark_visible), whose
 * tensor handling lives in the Python host layer (gaussian_splatting_amd/_C.py).
 *
 * Conventions (same as the reference):
 *  - every float array is a device pointer to contiguous fp32 data; an absent
 *    optional input is NULL (the reference's data_ptr() == nullptr test);
 *  - viewmatrix / projmatrix are 16 floats read column-major
 *    (cuda_rasterizer/auxiliary.h:75-95);
 *  - the three scratch buffers are obtained through allocation callbacks exactly
 *    like the reference's std::function<char*(size_t)> resize functors
 *    (rasterize_points.cu:29-43); their contents are private to this library and
 *    must be passed back unchanged to gsr_rasterize_backward;
 *  - all work is enqueued on `stream` (a hipStream_t; NULL = the default stream).
 *    gsr_rasterize_forward synchronises that stream once, to learn the number of
 *    tile instances (cuda_rasterizer/rasterizer_impl.cu:313).
 *
 * Every function returns 0 on success or a nonzero GSR_ERR_* code; the message
 * of the last failure on the calling thread is available from gsr_last_error().
 */
#ifndef GSR_H_INCLUDED
#define GSR_H_INCLUDED

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_OK 0
#define GSR_ERR_ARGUMENT 1      /* invalid argument (shape, size, null pointer) */
#define GSR_ERR_HIP 2           /* a HIP runtime / kernel launch error */
#define GSR_ERR_ALLOC 3         /* an allocation callback returned NULL */
#define GSR_ERR_OVERFLOW 4      /* more than INT_MAX tile instances */
#define GSR_ERR_PREFILTERED 5   /* prefiltered=1 but a point failed the frustum test */

/* Scratch allocation callback: return a device pointer to at least `nbytes`
 * bytes that stays valid until the matching backward call has returned.
 * Replaces std::function<char*(size_t)> (rasterize_points.cu:29-43). */
typedef void* (*gsr_alloc_fn)(void* ctx, size_t nbytes);

/* Forward pass (CudaRasterizer::Rasterizer::forward).
 * P Gaussians, active SH degree D, M SH coefficients per Gaussian (0 if shs is NULL).
 * out_color [3,H,W], out_invdepth [1,H,W] and radii [P] are written for every
 * element.  *num_rendered receives the number of (tile, Gaussian) instances. */
int gsr_rasterize_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                          gsr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                          int width, int height, const float* means3D, const float* shs, const float* colors_precomp,
                          const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                          const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                          const float* cam_pos, float tan_fovx, float tan_fovy, int prefiltered, float* out_color,
                          float* out_invdepth, int antialiasing, int* radii, int debug, void* stream,
                          int* num_rendered);

/* Same as gsr_rasterize_forward, without the mid-forward host synchronisation.
 * The binning buffer is requested for capacity_hint instances before the count is
 * known (typically the previous call's num_rendered plus a margin), the tile sort
 * runs on that capacity with the unused slots padded, and the stream is
 * synchronised once at the end to read num_rendered.  If num_rendered exceeds the
 * hint, the binning stage is redone exactly (the binning callback is called again
 * with a larger size).  capacity_hint <= 0 behaves like gsr_rasterize_forward.
 * *binning_capacity receives the capacity the binning buffer was laid out for;
 * pass it to gsr_rasterize_backward_ex. */
int gsr_rasterize_forward_ex(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                             int width, int height, const float* means3D, const float* shs,
                             const float* colors_precomp, const float* opacities, const float* scales,
                             float scale_modifier, const float* rotations, const float* cov3D_precomp,
                             const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                             float tan_fovy, int prefiltered, float* out_color, float* out_invdepth, int antialiasing,
                             int* radii, int debug, void* stream, int* num_rendered, int capacity_hint,
                             int* binning_capacity);

/* Backward pass (CudaRasterizer::Rasterizer::backward).
 * R = num_rendered from the forward; geom/binning/image buffers are the ones the
 * forward's callbacks returned.  dL_dinvdepths ([1,H,W]) may be NULL, in which
 * case dL_dinvdepth must be NULL too.  dL_dconic ([P,4]) may be NULL.  Every
 * element of every non-NULL output is written (no pre-zeroing needed).
 * `scratch_alloc` provides 48 bytes per tile instance for the per-instance
 * gradient records, plus 40 bytes and a live-list slot per Gaussian.  The backward
 * also sets the records' content bytes, which live in the forward's binning buffer
 * (zeroed by the forward); they depend on the geometry only, so a second backward of
 * the same forward (retain_graph) sets the same bytes. */
int gsr_rasterize_backward(int P, int D, int M, int R, const float* background, int width, int height,
                           const float* means3D, const float* shs, const float* colors_precomp,
                           const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                           const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                           const float* campos, float tan_fovx, float tan_fovy, const int* radii, void* geom_buffer,
                           void* binning_buffer, void* image_buffer, const float* dL_dpix, const float* dL_dinvdepths,
                           float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor,
                           float* dL_dinvdepth, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                           float* dL_drot, int antialiasing, int debug, gsr_alloc_fn scratch_alloc,
                           void* scratch_ctx, void* stream);

/* Backward for a forward made by gsr_rasterize_forward_ex: binning_capacity is the
 * value it returned, or 0.  With 0 and a nonzero binning_bytes (the binning buffer's
 * size) the capacity is recovered from the size: gsr_rasterize_forward_ex lays the
 * buffer out for a multiple of 256 instances, over which the size determines the layout
 * (so the buffer can travel through any tensor copy, e.g. saved-tensor hooks).  With 0
 * and 0 it is R (gsr_rasterize_forward's exact layout).  A size that matches no layout,
 * or a given capacity whose layout has another size, is GSR_ERR_ARGUMENT. */
int gsr_rasterize_backward_ex(int P, int D, int M, int R, const float* background, int width, int height,
                              const float* means3D, const float* shs, const float* colors_precomp,
                              const float* opacities, const float* scales, float scale_modifier,
                              const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                              const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                              const int* radii, void* geom_buffer, void* binning_buffer, void* image_buffer,
                              const float* dL_dpix, const float* dL_dinvdepths, float* dL_dmean2D, float* dL_dconic,
                              float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D,
                              float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot, int antialiasing,
                              int debug, gsr_alloc_fn scratch_alloc, void* scratch_ctx, void* stream,
                              int binning_capacity, size_t binning_bytes);

/* Separate-DC variants: the 3DGS-accel rasterizer's interface (the build that ships
 * SparseGaussianAdam), which the reference's callers select with separate_sh=True
 * (train.py:41-45,105,144; gaussian_renderer/__init__.py:106-125 passes dc= and
 * shs= = GaussianModel._features_dc / _features_rest).  Its _C.rasterize_gaussians /
 * _C.rasterize_gaussians_backward take `dc` right before `sh`, and the backward returns
 * dL_ddc before dL_dsh.  Here: dc is [P,1,3] (coefficient 0), shs is [P,M,3] with M
 * the number of REST coefficients (15 at SH degree 3; shs may be NULL when M == 0), and
 * the colour is the same polynomial as with one combined [P,M+1,3] array.  dL_ddc
 * ([P,1,3]) and dL_dsh ([P,M,3]) are written for every element.  Everything else is
 * gsr_rasterize_forward_ex / gsr_rasterize_backward_ex. */
int gsr_rasterize_forward_dc(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                             int width, int height, const float* means3D, const float* dc, const float* shs,
                             const float* colors_precomp, const float* opacities, const float* scales,
                             float scale_modifier, const float* rotations, const float* cov3D_precomp,
                             const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                             float tan_fovy, int prefiltered, float* out_color, float* out_invdepth, int antialiasing,
                             int* radii, int debug, void* stream, int* num_rendered, int capacity_hint,
                             int* binning_capacity);

int gsr_rasterize_backward_dc(int P, int D, int M, int R, const float* background, int width, int height,
                              const float* means3D, const float* dc, const float* shs, const float* colors_precomp,
                              const float* opacities, const float* scales, float scale_modifier,
                              const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                              const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                              const int* radii, void* geom_buffer, void* binning_buffer, void* image_buffer,
                              const float* dL_dpix, const float* dL_dinvdepths, float* dL_dmean2D, float* dL_dconic,
                              float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth, float* dL_dmean3D,
                              float* dL_dcov3D, float* dL_ddc, float* dL_dsh, float* dL_dscale, float* dL_drot,
                              int antialiasing, int debug, gsr_alloc_fn scratch_alloc, void* scratch_ctx,
                              void* stream, int binning_capacity, size_t binning_bytes);

/* Multi-GPU view exchange (gaussian_splatting_amd/distributed.py
 * ViewExchange).  The reference trains on one GPU; sharding views over N ranks needs the
 * N views' parameter gradients summed on every rank.  Instead of all-reducing the 59-float
 * parameter gradients (2 (N-1)/N x 236 B per Gaussian per rank over xGMI), each rank
 * all-gathers the other ranks' "view blocks" -- a camera header and, per Gaussian, the 10
 * summed render gradients (dL/dcolour, dL/dinvdepth, dL/dmean2D, dL/dopacity, dL/dconic)
 * plus a visibility / SH-clamp word, 44 B -- and every rank runs the per-Gaussian backward
 * over all views at once (10 (N-1) floats received per Gaussian instead of 118 (N-1)/N).
 *
 * gsr_view_block_floats(P): floats in one view block (padded to 256 B).
 * gsr_rasterize_backward_screen: the backward of gsr_rasterize_backward_dc up to the
 *   per-Gaussian sums (CR/backward.cu:433-612 = renderCUDA backward), written with the
 *   camera into view_block (device, 16-byte aligned, gsr_view_block_floats(P) floats);
 *   colours from SH (dc + shs, or shs alone with dc NULL), cov3D from scales/rotations.
 *   dL/dmeans2D of this view is the block's float pair at [64 + 4P + 2g] (densification).
 * gsr_gauss_backward_views: the rest of the backward (CR/backward.cu:153-429,
 *   computeCov2DCUDA + preprocessCUDA, as gsr_rasterize_backward_dc's last stage) for all
 *   n_views gathered blocks (blocks[v * block_floats ...]), writing the SUM over views of
 *   dL/dmeans3D, dL/ddc, dL/dsh, dL/dopacity, dL/dscales, dL/drotations.  With one view it
 *   equals the single-view backward bit for bit. */
unsigned long long gsr_view_block_floats(int P);

int gsr_rasterize_backward_screen(int P, int D, int M, int R, const float* background, int width, int height,
                                  const float* means3D, const float* dc, const float* shs, const float* opacities,
                                  const float* scales, float scale_modifier, const float* rotations,
                                  const float* viewmatrix, const float* projmatrix, const float* campos,
                                  float tan_fovx, float tan_fovy, const int* radii, void* geom_buffer,
                                  void* binning_buffer, void* image_buffer, const float* dL_dpix,
                                  const float* dL_dinvdepths, int antialiasing, int debug, gsr_alloc_fn scratch_alloc,
                                  void* scratch_ctx, void* stream, int binning_capacity, size_t binning_bytes,
                                  float* view_block);

int gsr_gauss_backward_views(int P, int D, int M, const float* means3D, const float* dc, const float* shs,
                             const float* opacities, const float* scales, const float* rotations, float scale_modifier,
                             int n_views, const float* blocks, long long block_floats, float* dL_dmean3D,
                             float* dL_ddc, float* dL_dsh, float* dL_dopacity, float* dL_dscale, float* dL_drot,
                             void* stream);

/* Sparse view blocks.  Behind saturated pixels most Gaussians get no render gradient (about
 * 14% of a 1M@1080p view have one), so a view block travels packed: its header (64 floats,
 * the entry count as uint32 bits in float 63) and, per Gaussian that is visible with a non-zero
 * sum, 12 floats (index bits, the 10 sums, the flag word), in Gaussian order.
 * gsr_view_pack_floats(n): floats of a packed block holding n entries (padded to 256 B).
 * gsr_view_pack_scratch_bytes(P): device scratch gsr_view_block_pack needs.
 * gsr_view_block_pack: view_block (gsr_view_block_floats(P) floats) -> packed
 *   (gsr_view_pack_floats(cap) floats); *count (device uint32, may be NULL) receives the entry
 *   count, which may exceed cap (then only the first cap entries are written).
 * gsr_view_block_unpack: n_views packed blocks (packed_floats apart) -> n_views dense view
 *   blocks (gsr_view_block_floats(P) apart), entries beyond cap ignored.  Only the flag words
 *   are cleared first: a Gaussian left out has flag 0 and its sums are left as they were
 *   (gsr_gauss_backward_views never reads them).  Unpacked blocks give gsr_gauss_backward_views
 *   the dense blocks' result (a Gaussian left out had all-zero sums, which add nothing). */
unsigned long long gsr_view_pack_floats(long long entries);
unsigned long long gsr_view_pack_scratch_bytes(int P);
int gsr_view_block_pack(int P, const float* view_block, float* packed, long long cap, void* scratch,
                        unsigned int* count, void* stream);
/* Chunked exchange (distributed.py ViewExchange(chunks=K), no reference counterpart): the same over the
 * Gaussians [g0, g1) only -- one chunk's packed block (entries keep their absolute index), so chunk k+1's
 * all-gather can run while the multi-view backward works on chunk k.  gsr_view_block_pack(...) is
 * gsr_view_block_pack_range(P, 0, P, ...). */
int gsr_view_block_pack_range(int P, int g0, int g1, const float* view_block, float* packed, long long cap,
                              void* scratch, unsigned int* count, void* stream);
int gsr_view_block_unpack(int P, int n_views, const float* packed, long long packed_floats, float* blocks,
                          long long cap, void* stream);

/* Packed mode of the multi-view backward (what ViewExchange uses): no dense blocks are rebuilt.
 * gsr_view_block_index: flags ([n_views][P] uint32) cleared, then for entry i of packed block v,
 *   flags[v * P + g] = i << 4 | the entry's flag bits (cap < 2^28 entries).  One 4-byte store per
 *   entry instead of the unpack's 44 bytes scattered over four arrays.
 * gsr_gauss_backward_views_packed: gsr_gauss_backward_views over the packed blocks themselves
 *   (camera from each packed header, sums from the entry its flag word indexes); the same result
 *   as over the unpacked blocks. */
int gsr_view_block_index(int P, int n_views, const float* packed, long long packed_floats, unsigned int* flags,
                         long long cap, void* stream);
/* Chunk form: clears and sets the flags of Gaussians [g0, g1) only (the packed blocks hold that chunk). */
int gsr_view_block_index_range(int P, int g0, int g1, int n_views, const float* packed, long long packed_floats,
                               unsigned int* flags, long long cap, void* stream);
int gsr_gauss_backward_views_packed(int P, int D, int M, const float* means3D, const float* dc, const float* shs,
                                    const float* opacities, const float* scales, const float* rotations,
                                    float scale_modifier, int n_views, const float* packed, long long packed_floats,
                                    const unsigned int* flags, float* dL_dmean3D, float* dL_ddc, float* dL_dsh,
                                    float* dL_dopacity, float* dL_dscale, float* dL_drot, void* stream);

/* Live-list form (sparse outputs): only the Gaussians some view flags are visited.
 * gsr_views_live_floats(P): uint32 words of the list buffer (entries + shard counters).
 * gsr_views_live_list: builds it from the flags of gsr_view_block_index.
 * gsr_gauss_backward_views_live: gsr_gauss_backward_views_packed over the listed Gaussians only,
 *   one lane each; every output row of the others is left untouched, so the caller zeroes the
 *   outputs beforehand (ViewExchange does it on a second stream while the all-gather runs). */
unsigned long long gsr_views_live_floats(int P);
int gsr_views_live_list(int P, int n_views, const unsigned int* flags, unsigned int* live, void* stream);
/* Chunk form: only Gaussians [g0, g1) are listed. */
int gsr_views_live_list_range(int P, int g0, int g1, int n_views, const unsigned int* flags, unsigned int* live,
                              void* stream);
int gsr_gauss_backward_views_live(int P, int D, int M, const float* means3D, const float* dc, const float* shs,
                                  const float* opacities, const float* scales, const float* rotations,
                                  float scale_modifier, int n_views, const float* packed, long long packed_floats,
                                  const unsigned int* flags, const unsigned int* live, float* dL_dmean3D,
                                  float* dL_ddc, float* dL_dsh, float* dL_dopacity, float* dL_dscale, float* dL_drot,
                                  void* stream);

/* Frustum test, view-space z > 0.2 (CudaRasterizer::Rasterizer::markVisible).
 * `present` is P bytes (bool). */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     unsigned char* present, void* stream);

/* Inspection of a forward's private state, for parity tests (the reference keeps the same
 * state in its binning / image buffers: BinningState::point_list and ImageState::ranges /
 * n_contrib / accum_alpha, cuda_rasterizer/rasterizer_impl.h:39-72).  Copies, on `stream`,
 * device to device, into caller-provided device arrays (any may be NULL to skip it):
 *   ranges     [tiles][2]  each tile's [start, end) in point_list (identifyTileRanges);
 *   point_list [R]         the tile lists, tile-major, each tile in (depth, index) order;
 *                          entry = Gaussian index << 4 | the forward's 4-bit quadrant mask;
 *   n_contrib  [H*W]       last contributor (1-based list position) per pixel;
 *   final_T    [H*W]       transmittance after the last contributor.
 * binning_capacity / binning_bytes as for gsr_rasterize_backward_ex. */
int gsr_debug_forward_state(int P, int width, int height, int R, int binning_capacity, size_t binning_bytes,
                            const void* geom_buffer, const void* binning_buffer, const void* image_buffer,
                            unsigned int* ranges, unsigned int* point_list, unsigned int* n_contrib, float* final_T,
                            void* stream);

/* Inspection of the reachable-prefix sort ("sort_prefix" option): copies, on `stream`, device to
 * device, the number of entries of each tile's list in final order (sorted_len [tiles]; the whole
 * length unless K4 sorted only a prefix) and the number of tiles the forward redid because a wave
 * passed the sorted prefix (redo_count [1]).  Either pointer may be NULL. */
int gsr_debug_sort_state(int P, int width, int height, const void* geom_buffer, unsigned int* sorted_len,
                         unsigned int* redo_count, void* stream);
/* Near-first binning state of a forward (the "near_mass" option; tests): the depth bin of its cut
 * (0xffffffff: none -- off, or the frame's opacity mass never reached the target) and, when there was a
 * cut, each tile's near entries [start, start + near) as K4 sorted them ([tiles][2] uint32). */
int gsr_debug_near_state(int P, int width, int height, const void* geom_buffer, unsigned int* zcut,
                         unsigned int* near_ranges, void* stream);

/* Number of forwards (process-wide) whose capacity hint was too small, so the binning stage
 * was redone with the exact count (gsr_rasterize_forward_ex). */
long long gsr_forward_rebuilds(void);

/* Host-side statistics since the last reset (reset != 0 clears after reading), for finding time
 * the GPU spends waiting on the host.  values[0..8] = for (a) the forwards' waits for their
 * instance count (the one host synchronisation of a forward, CR/rasterizer_impl.cu:313; here an
 * event behind the binning count), (b) whole forward calls, (c) whole backward calls: the number of
 * calls, their total host time in ms and the longest one in ms.  Up to n values are written. */
int gsr_host_stats(double* values, int n, int reset);

/* Runtime options (no reference counterpart): the library's alternative kernel paths, readable
 * and settable in-process so that every path it ships is parity-tested (tests/test_gpu_options.py).
 * Each default comes from the environment variable GSR_<NAME> (upper case) at first use.
 *   "fused_bin"  1|0    capacity-mode binning with the tile scan folded into the scatter (forward)
 *   "fwd_quads"  2|4    8x8 quadrants per forward wave: half tiles | whole tiles
 *   "bwd_seg_ck" 1..2^20 backward work unit length in 256-entry checkpoints; read by the forward, which
 *                        writes the units and records the value for its backward (a backward always
 *                        walks the segments its own forward made, whatever the option is by then)
 *   "host_total" 1|0    the binning kernels store num_rendered into mapped host memory | a copy is queued
 *   "zero_fill"  3|1|2|0 dense backward outputs zero-filled by extra blocks of render_bwd's launch
 *                        (default) | on a side stream | on the launch stream before gauss_bwd | not at
 *                        all (gauss_bwd writes every row)
 *   "live_list"  1|0    gauss_bwd over the list of Gaussians with a render gradient | a lane per Gaussian
 *                        (only with zero_fill != 0)
 *   "sort_prefix" L|0   (L in 1..1024) when the frame's mean list length is at least 2 L: of the lists longer than
 *                        1024 entries sort only the first L (+ the rest of a bucket), the part the blend
 *                        reaches, and redo the rare tile whose walk passes it | sort whole lists
 *                        (default L = 1024)
 *   "count_wait" 2|1|0  capacity-hinted forwards: no event behind the instance count, the host polls the
 *                        mapped count slot the binning kernel stores into (spins 100 us, then yields the
 *                        core between polls) | polls the event recorded behind the count (20 ms at most,
 *                        then blocks) | blocks in hipEventSynchronize (woken by the completion interrupt)
 *   "bwd_grid"   0|1|2  render_bwd's grid: 2 blocks per tile, each walking units i, i + G, ... when the
 *                        grid sized for the shortest segments would be over 4x that (5M@4K) | that worst-case
 *                        grid, one unit per block | always the strided grid
 *   "bwd_atomic" 0|1    the render backward writes one gradient record per (tile, Gaussian) instance, summed
 *                        per Gaussian by gauss_reduce in a fixed order: bitwise deterministic | adds
 *                        each instance's ten sums into per-Gaussian rows with float atomics (no records, no
 *                        gauss_reduce; the order of the adds follows the hardware: default, 1M@1080p -1.5 µs,
 *                        5M@4K -104 µs per step).  Read by the forward,
 *                        which zeroes the rows when it is 1 and marks its geometry buffer; a backward takes
 *                        the atomic path iff the option is 1 and its geometry buffer carries that mark (a
 *                        buffer from a forward without the option, or one copied in, gets the record path).
 *                        A forward with the option also skips the record path's inputs (record starts,
 *                        content bits); a record-path backward of its buffer writes them first.
 *                        The screen-space backward (view blocks) follows the same rule: its block's sums
 *                        come from the rows (gauss_live_views) instead of gauss_reduce
 *   "near_mass"  M|0    near-first binning (capacity-hinted forwards with the fused scan): only the Gaussians
 *                        in front of the depth at which the screen-averaged opacity mass (the integral of
 *                        alpha over the plane, summed front to back, over the image area) reaches M get keys
 *                        and are sorted; a tile whose forward walk passes its near entries is redone with its
 *                        whole list, so every output is the whole lists' (default M = 30; a pixel saturates
 *                        at 9.2) | every instance keyed and sorted
 *   "touched_run" 0|N   the atomic backward's per-Gaussian pass: one workgroup lists the touched Gaussians of
 *                        128 x N consecutive ones (N a power of two up to 32; others round down) and runs
 *                        their backward 128 at a time | 0: by the frame -- N = 16 where the mean tile list holds
 *                        2048 entries or more (few Gaussians touched: 5M@4K), else 1 (default)
 * Every option is read once per forward / backward call, so a concurrent gsr_option_set never splits
 * one call's launches between two values.
 * gsr_option_get returns -1 for an unknown name; gsr_option_set returns GSR_ERR_ARGUMENT for an
 * unknown name or an out-of-range value.  Not synchronised against calls running on other threads. */
int gsr_option_set(const char* name, int value);
int gsr_option_get(const char* name);
/* The same options for calls made on THIS thread only, over the process-wide values (e.g. a forward that no
 * backward will follow: "bwd_atomic" 0 skips zeroing the atomic backward's accumulator rows -- a backward of
 * it then takes the record path).  gsr_option_get reports the value in force on the calling thread.
 * gsr_option_clear_thread(name) drops one override, (NULL) all of them.  Errors as gsr_option_set. */
int gsr_option_set_thread(const char* name, int value);
int gsr_option_clear_thread(const char* name);

/* Forget what the library recorded about a geometry buffer's last forward (whether its accumulator rows were
 * zeroed and its record inputs written).  A buffer the library did not write at that address -- a copy, one
 * restored from a checkpoint -- must be forgotten before its backward, which then writes the record inputs
 * and takes the deterministic record path.  (The Python layer calls it for any geometry tensor that is not
 * the one its forward returned.)  Always GSR_OK. */
int gsr_geom_forget(const void* geom_buffer);

/* Message of the last error on this thread ("" if none). */
const char* gsr_last_error(void);

/* Library version string, e.g. "gsr 0.1.0 gfx950". */
const char* gsr_version(void);

/* The build's input hash: sha256 (hex) over every source, header and compiler flag the library was
 * compiled from (gaussian_splatting_amd/build.py input_hash), compiled into the library.  The loader
 * compares it with the hash of the tree it runs from, so a library built from other sources is
 * detected instead of used (no reference counterpart). */
const char* gsr_build_id(void);

/* Per-stage device timing with hipEvents recorded on the launch stream.
 * stage_mask selects the stages to time (bit s = stage s, -1 = all, 0 = off);
 * each timed stage adds one event pair to the stream (~10 us of idle GPU per
 * event on gfx950, so time only what you need inside a measured region).
 * collect() waits for the recorded events and adds their elapsed times to
 * running per-stage totals; it returns the number of stages and fills up to
 * max_stages totals (ms) and call counts.  Stage names come from
 * gsr_profile_stage_name(). */
int gsr_profile_enable(int stage_mask);
int gsr_profile_collect(double* total_ms, long long* calls, int max_stages);
void gsr_profile_reset(void);
const char* gsr_profile_stage_name(int stage);

/* Census (diagnostic; no reference counterpart): with a device buffer of 10 zeroed uint64
 * counters set, the render kernels of later forward / backward calls run their census
 * instantiations (slower: a few extra wave-uniform ops per evaluation) and add, per call:
 *   [0] forward list entries staged (per half-tile wave; each tile's two halves both stage)
 *   [1] forward (entry, 8x8 quadrant) evaluations  (64 pixel evaluations each)
 *   [2] forward (pixel, entry) pairs with alpha > 0 reaching a live pixel
 *   [3] forward (pixel, entry) pairs blended (alpha > 0 and the pixel does not end there)
 *   [4] backward list entries staged
 *   [5] backward (entry, quadrant) evaluations
 *   [6] backward (pixel, entry) pairs with a gradient term (alpha > 0, before n_contrib)
 *   [7] backward per-entry wave reductions (gradient records with content)
 *   [8] backward evaluations in which no pixel has a gradient term (idle)
 *   [9] forward evaluations in which no pixel blends (idle)
 * NULL turns the census off.  Not thread-safe against concurrent calls. */
int gsr_census_set(void* device_counters);

#ifdef __cplusplus
}
#endif

#endif /* GSR_H_INCLUDED */
