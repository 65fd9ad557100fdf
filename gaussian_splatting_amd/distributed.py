"""View-sharded data parallelism over GPUs.

The reference trains on one GPU, one view per iteration (train.py:131-143).  Views
are independent, so N ranks each render their own view with a replicated copy of
the Gaussians, and exchange one step's gradient information over RCCL (backend
"nccl" on ROCm).  Two exchanges are provided:

* ``GradArena.all_reduce`` -- north_star's form: the six parameter groups of
  ``GaussianModel`` (``_xyz``, ``_features_dc``, ``_features_rest``, ``_opacity``,
  ``_scaling``, ``_rotation``; scene/gaussian_model.py:235-242) back to back in one flat
  fp32 arena (59 floats per Gaussian at SH degree 3) that the backward writes into
  directly, reduced by ONE all-reduce;
* ``ViewExchange`` -- the per-view render-gradient sums (10 floats of the Gaussians that
  have one, ~14% of a 1M@1080p view) all-gathered, and the per-Gaussian backward run over
  all gathered views on every rank.

``bench.py --exchange auto`` times both in its warm-up on the real fabric and keeps the
faster.  Either way every rank ends with the same summed gradients and applies the same
optimizer step, so the replicas stay identical without a broadcast.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist

# block order inside the arena; shapes are per-Gaussian
_BLOCKS = (("dL_dmeans3D", (3,)), ("dL_dsh", None), ("dL_dopacity", (1,)), ("dL_dscales", (3,)),
           ("dL_drotations", (4,)))
# separate-SH arena: exactly GaussianModel's parameter groups, in its order (gaussian_model.py:235-242)
_BLOCKS_SEPARATE = (("dL_dmeans3D", (3,)), ("dL_ddc", (1, 3)), ("dL_dsh", None), ("dL_dopacity", (1,)),
                    ("dL_dscales", (3,)), ("dL_drotations", (4,)))
_GROUP_OF = {"dL_dmeans3D": "xyz", "dL_ddc": "f_dc", "dL_dopacity": "opacity", "dL_dscales": "scaling",
             "dL_drotations": "rotation"}


class GradArena:
    """Flat gradient buffer with per-parameter views, reduced by a single collective.

    ``separate_sh=False``: the vendored rasterizer's outputs (one ``dL_dsh`` [P,M,3] block).
    ``separate_sh=True``: the 3DGS-accel outputs -- ``dL_ddc`` [P,1,3] and ``dL_dsh`` [P,M-1,3] as two
    contiguous blocks, so every block is exactly one GaussianModel parameter's gradient and can be
    handed to the optimizer without a copy (``param_grads()``)."""

    def __init__(self, P: int, M: int, device, dtype=torch.float32, separate_sh: bool = False):
        self.P, self.M, self.separate_sh = P, M, separate_sh
        rest = M - 1 if separate_sh else M
        per = {"dL_dmeans3D": 3, "dL_ddc": 3, "dL_dsh": 3 * rest, "dL_dopacity": 1, "dL_dscales": 3,
               "dL_drotations": 4}
        blocks = _BLOCKS_SEPARATE if separate_sh else _BLOCKS
        self.floats_per_gaussian = sum(per[name] for name, _ in blocks)
        self.flat = torch.empty(P * self.floats_per_gaussian, device=device, dtype=dtype)
        self._views: Dict[str, torch.Tensor] = {}
        off = 0
        for name, shape in blocks:
            n = P * per[name]
            shp = (P, rest, 3) if name == "dL_dsh" else (P,) + shape
            self._views[name] = self.flat[off:off + n].view(shp)
            off += n

    def views(self) -> Dict[str, torch.Tensor]:
        """Output tensors for ``_C.rasterize_gaussians_backward(..., out=...)``."""
        return self._views

    def param_grads(self) -> Dict[str, torch.Tensor]:
        """Gradient of each GaussianModel parameter group, by group name (separate-SH arena only)."""
        if not self.separate_sh:
            raise RuntimeError("param_grads() needs separate_sh=True (f_dc / f_rest as their own blocks)")
        out = {_GROUP_OF[k]: v for k, v in self._views.items() if k in _GROUP_OF}
        out["f_rest"] = self._views["dL_dsh"]
        return out

    def all_reduce(self, op=None, group: Optional[dist.ProcessGroup] = None, average: bool = False) -> None:
        """Sum (or average) the arena over all ranks in one collective."""
        if not dist.is_initialized():  # a group of one still runs the collective (RCCL exercised at N = 1)
            return
        dist.all_reduce(self.flat, op=op or dist.ReduceOp.SUM, group=group)
        if average:
            self.flat.div_(dist.get_world_size(group))

    def split_features(self):
        """(f_dc, f_rest) gradient views, matching GaussianModel._features_dc / _features_rest."""
        if self.separate_sh:
            return self._views["dL_ddc"], self._views["dL_dsh"]
        sh = self._views["dL_dsh"]
        return sh[:, :1, :], sh[:, 1:, :]


def reduce_densification_stats(grad_norm_sum: torch.Tensor, denom: torch.Tensor, max_radii2D: torch.Tensor,
                               group: Optional[dist.ProcessGroup] = None) -> None:
    """Make densification statistics global (train.py:212-215, gaussian_model.py:643-654):
    SUM of the screen-space gradient norms and their counts, MAX of the 2-D radii.

    Call it EXACTLY ONCE per densification interval, on the running accumulators
    (``xyz_gradient_accum``, ``denom``, ``max_radii2D``), right before ``densify_and_prune``:
    each rank accumulates its own views' statistics locally every iteration (the reference's
    ``add_densification_stats``), and this one reduction makes every rank's accumulators the sum
    over all ranks' views.  The SUM is in place, so a second call on the same accumulators would
    add the other ranks' totals again (N-fold growth per call)."""
    if not dist.is_initialized():
        return
    stats = torch.cat([grad_norm_sum.reshape(-1), denom.reshape(-1)])
    dist.all_reduce(stats, op=dist.ReduceOp.SUM, group=group)
    n = grad_norm_sum.numel()
    grad_norm_sum.copy_(stats[:n].view_as(grad_norm_sum))
    denom.copy_(stats[n:].view_as(denom))
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX, group=group)


def _lib_scratch_bytes(P: int) -> int:
    from . import _lib

    return int(_lib.load().gsr_view_pack_scratch_bytes(int(P)))


class ViewExchange:
    """The multi-GPU exchange of view blocks (include/gsr.h, "Multi-GPU view exchange").

    Instead of all-reducing the parameter gradients (``GradArena.all_reduce``: 2 (N-1)/N x 59
    floats per Gaussian through every rank's xGMI links), each rank writes its view's
    per-Gaussian render-gradient sums into a view block (~44 B per Gaussian), ONE
    ``all_gather_into_tensor`` gives every rank all N blocks, and ``_C.gauss_backward_views``
    turns them into the summed parameter gradients on every rank -- the same bytes in, the same
    kernel, so the replicas agree bit for bit.  At N = 2 a rank receives 11 floats per Gaussian
    instead of 59; at N = 8, 77 instead of 103.

    ``sparse=True`` (the default) sends the blocks packed (include/gsr.h, "Sparse view blocks"):
    only Gaussians with a non-zero render-gradient sum, 48 B each (~14% of a 1M@1080p frame's
    Gaussians).  The gather size is a capacity hint carried from earlier steps (a decaying maximum
    of the largest packed block over the ranks, plus a margin), as the forward sizes its binning
    buffer, so the host never waits for this step's count before queuing the collective: every
    rank queues pack, the MAX of the counts (on the device), the all-gather at the hint, the
    index and the multi-view backward, and only then (``finish``, called by ``views_backward``)
    reads the step's largest count -- while the GPU still works through the queue.  A count over
    the hint (rare: the view changed a lot) re-gathers at the exact size and reruns the index and
    the backward, on every rank alike (they all read the same MAX).  The first exchange has no
    hint and waits for the count first.  Left-out Gaussians had all-zero sums, so the result
    equals the dense exchange's bit for bit; when a packed block would not be smaller than a dense
    one, the dense blocks are sent (``last_entries`` is then None).

        ex = ViewExchange(P, device)
        _C.rasterize_gaussians_backward_screen(*backward_args, view_block=ex.local_block())
        ex.exchange()
        ex.views_backward(means3D, dc, sh, degree, opacities, scales, rotations, 1.0, out=arena.views())
    """

    CAP_MARGIN = 1.05
    CAP_DECAY = 0.98

    def __init__(self, P: int, device, group: Optional[dist.ProcessGroup] = None, sparse: bool = True,
                 chunks: int = 1):
        from . import _C

        self.P, self.group, self.sparse, self.device = P, group, sparse and P > 0, torch.device(device)
        # chunks > 1 (sparse only): the Gaussians in `chunks` index ranges, each packed and gathered on its
        # own (async all-gathers, all queued at once on the collective stream), so chunk k+1's all-gather
        # runs while the multi-view backward works on chunk k ("Chunked exchange")
        self.chunks = max(1, int(chunks)) if self.sparse else 1
        # every collective runs whenever a process group exists, a group of one included, so the N = 1
        # bench and the nccl-group-of-one GPU test drive RCCL exactly as the N-rank run does
        self.collective = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.collective else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.block_floats = _C.view_block_floats(P) if P > 0 else 0
        self._gathered = None  # dense [N, block] buffer: allocated on first use (dense mode or fallback)
        self.last_entries = None  # sparse: entries each rank sent in the last exchange
        self.resyncs = 0          # sparse exchanges redone because the capacity hint was too small
        self._cap_last = 0        # decaying maximum of the largest packed block (entries)
        self._pending = None      # sparse: (hint used, whether the zero fill runs) until finish()
        if self.sparse:
            # this rank's dense block, its packed form (room for every Gaussian), the packed blocks
            # of all ranks, and the pack's scratch / count
            self._local = torch.empty(self.block_floats, dtype=torch.float32, device=device)
            self._packed = torch.empty(_C.view_pack_floats(P), dtype=torch.float32, device=device)
            self._recv = torch.empty(self.world * _C.view_pack_floats(P), dtype=torch.float32, device=device)
            nbytes = int(_lib_scratch_bytes(P))
            self._scratch = torch.empty(nbytes, dtype=torch.uint8, device=device)
            self._count = torch.zeros(1, dtype=torch.int32, device=device)
            self._count64 = torch.zeros(1, dtype=torch.int64, device=device)
            self._count_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self._count_ev = torch.cuda.Event()
            self._flags = torch.empty(self.world, P, dtype=torch.int32, device=device)  # view_block_index
            self._live = torch.empty(_C.views_live_floats(P), dtype=torch.int32, device=device)
        if self.chunks > 1:
            K = self.chunks
            self.bounds = [P * k // K for k in range(K + 1)]
            sizes = [self.bounds[k + 1] - self.bounds[k] for k in range(K)]
            self._cpacked = [torch.empty(_C.view_pack_floats(n), dtype=torch.float32, device=device) for n in sizes]
            self._crecv = [torch.empty(self.world * _C.view_pack_floats(n), dtype=torch.float32, device=device)
                           for n in sizes]
            self._ccount = torch.zeros(K, dtype=torch.int32, device=device)
            self._ccount64 = torch.zeros(K, dtype=torch.int64, device=device)
            self._ccount_host = torch.zeros(K, dtype=torch.int64, pin_memory=True)
            self._ccap_last = [-1] * K  # -1: no history yet (0 is a real, empty chunk)
            self._cworks = None   # the chunks' async all-gathers, waited for one at a time
            self._chint = None    # entries gathered per chunk
            self._crecv_views = [None] * K
        self._view_blocks, self._view_flags, self._view_live = None, None, None  # views_backward reads
        self._side = None      # the stream zeroing the outputs during the exchange
        self._zeroed = None    # the flat output buffer it zeroes
        self._last_bwd = None  # the arguments of the last views_backward (rerun after a resync)

    @property
    def gathered(self) -> torch.Tensor:
        """All ranks' dense view blocks, [N, block_floats] (allocated on first use)."""
        if self._gathered is None:
            self._gathered = torch.empty(self.world, self.block_floats, dtype=torch.float32, device=self.device)
        return self._gathered

    def local_block(self) -> torch.Tensor:
        """Where this rank's backward writes its view block."""
        return self._local if self.sparse else self.gathered[self.rank]

    def capacity_hint(self) -> int:
        """Entries the next sparse exchange gathers per rank (0: none yet, the count is waited for)."""
        if self._cap_last <= 0:
            return 0
        return min(self.P, int(self._cap_last * self.CAP_MARGIN) + 1024)

    def _note_count(self, n: int) -> None:
        self._cap_last = max(int(n), int(self._cap_last * self.CAP_DECAY))

    def chunk_hint(self, k: int) -> int:
        """Entries the next chunked exchange gathers per rank for chunk k (0: none yet)."""
        if self._ccap_last[k] < 0:
            return 0
        n = self.bounds[k + 1] - self.bounds[k]
        return min(n, int(self._ccap_last[k] * self.CAP_MARGIN) + 256)

    def _exchange_chunked(self) -> None:
        """Chunked sparse exchange: pack every chunk, one MAX all-reduce of the K counts, then the K
        all-gathers queued at once (async); views_backward waits for chunk k's gather just before its
        part of the multi-view backward, so the later gathers overlap the earlier chunks' backward."""
        from . import _C

        K = self.chunks
        for k in range(K):
            _C.view_block_pack(self._local, self._cpacked[k], self._scratch, self._ccount[k:k + 1], self.P,
                               rng=(self.bounds[k], self.bounds[k + 1]))
        self._ccount64.copy_(self._ccount)
        if self.collective:
            if dist.get_backend(self.group) == "nccl":
                dist.all_reduce(self._ccount64, op=dist.ReduceOp.MAX, group=self.group)
                self._ccount_host.copy_(self._ccount64, non_blocking=True)
            else:  # gloo (CPU rehearsals): the collective needs a host tensor
                host = self._ccount64.cpu()
                dist.all_reduce(host, op=dist.ReduceOp.MAX, group=self.group)
                self._ccount_host.copy_(host)
        else:
            self._ccount_host.copy_(self._ccount64, non_blocking=True)
        self._count_ev.record()
        hints = [self.chunk_hint(k) for k in range(K)]
        if min(self._ccap_last) < 0:  # no history: wait for this step's counts
            self._count_ev.synchronize()
            hints = [min(int(self._ccount_host[k]), self.bounds[k + 1] - self.bounds[k]) for k in range(K)]
        self._chint = hints
        self._cworks = [self._gather_chunk(k, hints[k], async_op=True) for k in range(K)]
        self.last_entries = sum(hints)
        self._pending = (hints, True)

    def _gather_chunk(self, k: int, n: int, async_op: bool):
        from . import _C

        size = _C.view_pack_floats(n)
        recv = self._crecv[k][: self.world * size].view(self.world, size)
        self._crecv_views[k] = recv
        if self.collective:
            return dist.all_gather_into_tensor(recv.view(-1), self._cpacked[k][:size], group=self.group,
                                               async_op=async_op)
        recv[0].copy_(self._cpacked[k][:size])
        return None

    def _chunk_backward(self, k: int, bwd_args) -> None:
        """Index, list and run the multi-view backward over chunk k's gathered blocks (after its gather)."""
        from . import _C

        means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier, out = bwd_args
        rng = (self.bounds[k], self.bounds[k + 1])
        recv = self._crecv_views[k]
        _C.view_block_index(recv, self._flags, self.P, rng=rng)
        # always the live-list form: chunk k's pass must write only chunk k's rows (a pass over all P rows
        # would read other chunks' stale flags and overwrite their results); the outputs were zeroed, either
        # on the side stream (exchange(zero=...)) or by _run_views_backward
        _C.views_live_list(self._flags, self._live, self.P, rng=rng)
        _C.gauss_backward_views(means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier, recv, out,
                                flags=self._flags, live=self._live)

    def _finish_chunked(self) -> bool:
        hints, _ = self._pending
        self._pending = None
        self._count_ev.synchronize()
        redone = False
        for k in range(self.chunks):
            n = min(int(self._ccount_host[k]), self.bounds[k + 1] - self.bounds[k])
            self._ccap_last[k] = max(n, int(self._ccap_last[k] * self.CAP_DECAY))
            if n > hints[k]:  # this chunk's hint was too small: gather it again at its exact size, rerun its part
                redone = True
                self._gather_chunk(k, n, async_op=False)
                if self._last_bwd is not None:
                    self._chunk_backward(k, self._last_bwd)
        if redone:
            self.resyncs += 1
        return redone

    def exchange(self, zero: Optional[torch.Tensor] = None) -> None:
        """Give every rank all N view blocks.

        Dense: one in-place ``all_gather_into_tensor`` of the blocks (44 B per Gaussian).
        Sparse (default): the block is packed to the Gaussians with a non-zero render gradient
        (``_C.view_block_pack``, 48 B each, ~14% of a 1M@1080p view); the largest entry count over
        the ranks is formed on the device (MAX all-reduce) and copied to pinned host memory without
        waiting; ONE ``all_gather_into_tensor`` moves the packed blocks at the capacity hint; and
        ``_C.view_block_index`` indexes them on every rank.  The host reads the count only in
        ``finish`` -- after the multi-view backward is queued -- and redoes the exchange if the hint
        was too small.  Without a hint (the first exchange) it waits for the count here.

        ``zero`` (optional): the flat buffer behind the ``out`` views later given to
        ``views_backward`` (e.g. ``GradArena.flat``).  It is zeroed on a second stream while the
        exchange runs, and the multi-view backward then writes only the rows of Gaussians some
        view has a gradient for (a live list, ``_C.views_live_list``)."""
        from . import _C

        if self._pending is not None:
            self.finish()
        self._view_blocks, self._view_flags, self._view_live = None, None, None
        self._zeroed = None
        self._last_bwd = None
        if zero is not None and self.sparse:
            cur = torch.cuda.current_stream(zero.device)
            if self._side is None:
                self._side = torch.cuda.Stream(device=zero.device)
            self._side.wait_stream(cur)
            with torch.cuda.stream(self._side):
                zero.zero_()
            zero.record_stream(self._side)
            self._zeroed = zero
        if not self.sparse:
            if self.collective:
                dist.all_gather_into_tensor(self.gathered.view(-1), self.local_block(), group=self.group)
            self._view_blocks = self.gathered
            return
        if self.chunks > 1:
            self._exchange_chunked()
            return
        _C.view_block_pack(self._local, self._packed, self._scratch, self._count, self.P)
        self._count64.copy_(self._count)
        if self.collective:
            if dist.get_backend(self.group) == "nccl":
                dist.all_reduce(self._count64, op=dist.ReduceOp.MAX, group=self.group)
                self._count_host.copy_(self._count64, non_blocking=True)
            else:  # gloo (CPU rehearsals): the collective needs a host tensor, i.e. a synchronisation
                host = self._count64.cpu()
                dist.all_reduce(host, op=dist.ReduceOp.MAX, group=self.group)
                self._count_host.copy_(host)
        else:
            self._count_host.copy_(self._count64, non_blocking=True)
        self._count_ev.record()
        hint = self.capacity_hint()
        if hint == 0:  # no history: wait for this step's count (like the forward without a hint)
            self._count_ev.synchronize()
            hint = min(int(self._count_host.item()), self.P)
        self._pending = (hint, True)
        self._gather(hint)

    def _gather(self, n: int) -> None:
        """All-gather the packed blocks at ``n`` entries per rank (or the dense blocks if that is not
        smaller), then index them."""
        from . import _C

        size = _C.view_pack_floats(n)
        if size >= self.block_floats:  # hardly any occlusion: the dense blocks are the smaller message
            self.gathered[self.rank].copy_(self._local)
            if self.collective:
                dist.all_gather_into_tensor(self.gathered.view(-1), self.gathered[self.rank], group=self.group)
            self.last_entries = None
            self._view_blocks, self._view_flags, self._view_live = self.gathered, None, None
            return
        self.last_entries = n
        recv = self._recv[: self.world * size].view(self.world, size)
        if self.collective:
            dist.all_gather_into_tensor(recv.view(-1), self._packed[:size], group=self.group)
        else:
            recv[0].copy_(self._packed[:size])
        _C.view_block_index(recv, self._flags, self.P)
        self._view_blocks, self._view_flags, self._view_live = recv, self._flags, None
        if self._zeroed is not None:
            _C.views_live_list(self._flags, self._live, self.P)
            self._view_live = self._live

    def finish(self) -> bool:
        """Complete the last sparse exchange: read its largest count (queued as a non-blocking copy;
        by now the GPU is usually past it) and, if it exceeded the gather's capacity, gather again
        at the exact size -- rerunning the multi-view backward if it was already queued.  Returns
        True if the exchange was redone.  Called by ``views_backward``; idempotent."""
        if self._pending is None:
            return False
        if self.chunks > 1:
            return self._finish_chunked()
        hint, _ = self._pending
        self._pending = None
        self._count_ev.synchronize()
        n = min(int(self._count_host.item()), self.P)  # a pinned host tensor: no device sync
        self._note_count(n)
        if n <= hint:
            return False
        self.resyncs += 1
        self._gather(n)
        if self._last_bwd is not None:
            self._run_views_backward(*self._last_bwd)
        return True

    def views_backward(self, means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier, out) -> None:
        """The per-Gaussian backward summed over all ranks' views (``_C.gauss_backward_views`` over
        what the last ``exchange`` gathered: dense view blocks, or packed blocks and their index).
        Queues the kernel, then completes a sparse exchange (``finish``)."""
        self._last_bwd = (means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier, out)
        self._run_views_backward(*self._last_bwd)
        self.finish()

    def _run_views_backward(self, means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier, out):
        from . import _C

        if self._zeroed is not None:  # the outputs' zero fill (exchange(zero=...)) must be done
            torch.cuda.current_stream(self._zeroed.device).wait_stream(self._side)
        if self.chunks > 1:
            args = (means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier, out)
            if self._zeroed is None:  # no side-stream fill: the live-list passes need zeroed outputs
                for t in out.values():
                    t.zero_()
            for k in range(self.chunks):
                w = self._cworks[k] if self._cworks is not None else None
                if w is not None:
                    w.wait()  # (RCCL: the compute stream waits for the gather, not the host)
                self._chunk_backward(k, args)
            self._cworks = None
            return
        _C.gauss_backward_views(means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier,
                                self._view_blocks, out, flags=self._view_flags, live=self._view_live)

    def received_bytes(self) -> int:
        """Bytes this rank received from the others in the last exchange."""
        from . import _C

        if not self.sparse:
            return (self.world - 1) * self.block_floats * 4
        if self.chunks > 1:
            return (self.world - 1) * sum(_C.view_pack_floats(n) for n in (self._chint or [0])) * 4
        if self.last_entries is None:  # the last exchange fell back to the dense blocks
            return (self.world - 1) * self.block_floats * 4
        return (self.world - 1) * _C.view_pack_floats(self.last_entries) * 4

    def means2D_grad(self, rank: Optional[int] = None) -> torch.Tensor:
        """dL/dmeans2D (x, y) of a rank's view, [P, 2]: the densification statistics' input
        (train.py:215).  This rank's own view (and every view of a dense exchange) is a strided
        view of its block; another rank's view after a sparse exchange is built from its packed
        entries, zeros for the Gaussians the packed block left out."""
        r = self.rank if rank is None else rank
        if self.sparse and r == self.rank:
            return self._local[64 + 4 * self.P: 64 + 8 * self.P].view(self.P, 4)[:, :2]
        if self.chunks > 1:  # packed chunks: scatter each chunk's entries of view r
            g = torch.zeros(self.P, 2, dtype=torch.float32, device=self.device)
            for k in range(self.chunks):
                pk = self._crecv_views[k][r]
                n = int(pk[63].view(torch.int32).item())
                ent = pk[64: 64 + 12 * n].view(n, 12)
                g[ent[:, 0].view(torch.int32).long()] = ent[:, 5:7]
            return g
        if self._view_flags is None:  # dense blocks
            return self.gathered[r][64 + 4 * self.P: 64 + 8 * self.P].view(self.P, 4)[:, :2]
        pk = self._view_blocks[r]  # packed: scatter its entries' (b.x, b.y) -- entry layout, include/gsr.h
        n = int(pk[63].view(torch.int32).item())
        ent = pk[64: 64 + 12 * n].view(n, 12)
        g = torch.zeros(self.P, 2, dtype=pk.dtype, device=pk.device)
        g[ent[:, 0].view(torch.int32).long()] = ent[:, 5:7]
        return g
