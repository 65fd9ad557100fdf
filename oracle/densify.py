"""CPU oracle of adaptive density control: TEST INFRASTRUCTURE ONLY -- imported by tests/
and tools/, never by the product path (gaussian_splatting_amd/densify.py, csrc/densify.hip).

A numpy float32 restatement of the reference's GaussianModel methods, step for step in the
reference's own order (scene/gaussian_model.py):

    densify_and_prune :574-640   grads = accum / denom, NaN -> 0; clone; split; prune
    densify_and_clone :552-571   |grad| >= max_grad and max(exp(s)) <= percent_dense * extent
    densify_and_split :508-550   grad >= max_grad and max(exp(s)) >  percent_dense * extent;
                                 children: bmm(build_rotation(q), sample) + xyz,
                                 log(exp(s) / (0.8 N)); parents dropped
    densification_postfix :483-506 / cat_tensors_to_optimizer :439-481
                                 new rows appended, zero Adam moments, stats zeroed
    prune_points :420-437 / _prune_optimizer :400-418
                                 rows (and moments) of pruned Gaussians dropped
    build_rotation  utils/general_utils.py:78-99

The split's normal samples are an input (the reference draws them with torch.normal; the
tests draw the same numbers for both sides).  numpy float32 arithmetic rounds every
operation; exp/log may differ from the GPU's by an ulp, so the tests compare copies
bitwise and computed values (children's xyz and scaling) within 1e-6.  The reference's
own tests cover none of this.  Pinned (tests/test_densify.py, CPU, in the container where
the reference is mounted) against the reference's OWN GaussianModel.densify_and_prune /
add_densification_stats, compiled from its source with the device literal "cuda" read as
"cpu", on the same inputs and the same torch.normal samples; and by known-answer cases.
"""
from __future__ import annotations

import numpy as np

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
f32 = np.float32


def build_rotation(r):
    """utils/general_utils.py:78-99 (float32, every operation rounded)."""
    r = np.asarray(r, f32)
    norm = np.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = np.zeros((q.shape[0], 3, 3), f32)
    r0, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    two, one = f32(2), f32(1)
    R[:, 0, 0] = one - two * (y * y + z * z)
    R[:, 0, 1] = two * (x * y - r0 * z)
    R[:, 0, 2] = two * (x * z + r0 * y)
    R[:, 1, 0] = two * (x * y + r0 * z)
    R[:, 1, 1] = one - two * (x * x + z * z)
    R[:, 1, 2] = two * (y * z - r0 * x)
    R[:, 2, 0] = two * (x * z - r0 * y)
    R[:, 2, 1] = two * (y * z + r0 * x)
    R[:, 2, 2] = one - two * (x * x + y * y)
    return R


class State:
    """The slice of GaussianModel the densification touches: params[name] [P, ...] float32,
    moments[name] = (exp_avg, exp_avg_sq) or None, accum/denom [P, 1], max_radii2D [P]."""

    def __init__(self, params, moments, accum, denom, max_radii2D=None):
        self.params = {k: np.asarray(v, f32).copy() for k, v in params.items()}
        self.moments = {k: (None if moments.get(k) is None else tuple(np.asarray(t, f32).copy() for t in moments[k]))
                        for k in NAMES}
        self.accum = np.asarray(accum, f32).reshape(-1, 1).copy()
        self.denom = np.asarray(denom, f32).reshape(-1, 1).copy()
        P = self.params["xyz"].shape[0]
        self.max_radii2D = np.zeros(P, f32) if max_radii2D is None else np.asarray(max_radii2D, f32).copy()

    @property
    def P(self):
        return self.params["xyz"].shape[0]

    def get_scaling(self):
        return np.exp(self.params["scaling"])

    def get_opacity(self):
        return f32(1) / (f32(1) + np.exp(-self.params["opacity"]))

    # cat_tensors_to_optimizer + densification_postfix
    def postfix(self, new):
        for k in NAMES:
            self.params[k] = np.concatenate([self.params[k], new[k]], axis=0)
            if self.moments[k] is not None:
                z = np.zeros_like(new[k])
                self.moments[k] = tuple(np.concatenate([m, z], axis=0) for m in self.moments[k])
        P = self.P
        self.accum = np.zeros((P, 1), f32)
        self.denom = np.zeros((P, 1), f32)
        self.max_radii2D = np.zeros(P, f32)

    # prune_points + _prune_optimizer
    def prune(self, mask):
        keep = ~mask
        for k in NAMES:
            self.params[k] = self.params[k][keep]
            if self.moments[k] is not None:
                self.moments[k] = tuple(m[keep] for m in self.moments[k])
        self.accum, self.denom, self.max_radii2D = self.accum[keep], self.denom[keep], self.max_radii2D[keep]


def densify_and_clone(st: State, grads, grad_threshold, extent, percent_dense):
    sel = np.sqrt(np.sum(grads * grads, axis=-1)) >= f32(grad_threshold)
    sel = sel & (st.get_scaling().max(axis=1) <= f32(percent_dense * extent))
    st.postfix({k: st.params[k][sel] for k in NAMES})


def split_mask(st: State, grads, grad_threshold, extent, percent_dense):
    n_init = st.P
    padded = np.zeros(n_init, f32)
    padded[:grads.shape[0]] = grads.reshape(-1)
    sel = padded >= f32(grad_threshold)
    return sel & (st.get_scaling().max(axis=1) > f32(percent_dense * extent))


def densify_and_split(st: State, grads, grad_threshold, extent, percent_dense, samples, N=2):
    sel = split_mask(st, grads, grad_threshold, extent, percent_dense)
    ns = int(sel.sum())
    samples = np.asarray(samples, f32).reshape(N * ns, 3)
    rots = np.tile(build_rotation(st.params["rotation"][sel]), (N, 1, 1))
    # bmm(rots, samples[..., None]): per row, three products summed in order
    d = rots[:, :, 0] * samples[:, 0:1] + rots[:, :, 1] * samples[:, 1:2] + rots[:, :, 2] * samples[:, 2:3]
    new = {"xyz": d + np.tile(st.params["xyz"][sel], (N, 1)),
           "scaling": np.log(np.tile(st.get_scaling()[sel], (N, 1)) / f32(0.8 * N))}
    for k in ("f_dc", "f_rest", "opacity", "rotation"):
        new[k] = np.tile(st.params[k][sel], (N,) + (1,) * (st.params[k].ndim - 1))
    st.postfix(new)
    st.prune(np.concatenate([sel, np.zeros(N * ns, bool)]))


def densify_and_prune(st: State, max_grad, min_opacity, extent, max_screen_size, percent_dense, samples, N=2):
    """gaussian_model.py:574-640 on `st` (in place); returns st."""
    with np.errstate(divide="ignore", invalid="ignore"):
        grads = st.accum / st.denom
    grads[np.isnan(grads)] = f32(0)
    densify_and_clone(st, grads, max_grad, extent, percent_dense)
    densify_and_split(st, grads, max_grad, extent, percent_dense, samples, N)
    prune = (st.get_opacity() < f32(min_opacity)).reshape(-1)
    if max_screen_size:
        big_vs = st.max_radii2D > max_screen_size
        big_ws = st.get_scaling().max(axis=1) > f32(0.1 * extent)
        prune = prune | big_vs | big_ws
    st.prune(prune)
    return st


def densification_stats(vgrad, accum, denom, max_radii2D, radii, visible=None):
    """add_densification_stats (gaussian_model.py:643-654) + train.py:212-213, in place."""
    vis = (np.asarray(radii) > 0) if visible is None else np.asarray(visible, bool)
    g = np.asarray(vgrad, f32)
    accum[vis] += np.sqrt(g[vis, 0] * g[vis, 0] + g[vis, 1] * g[vis, 1]).reshape(accum[vis].shape)
    denom[vis] += f32(1)
    if max_radii2D is not None:
        max_radii2D[vis] = np.maximum(max_radii2D[vis], np.asarray(radii, f32)[vis])
