"""Multi-GPU host logic of the GNOT hot path.  One process per GPU.

Two modes; in both the parameter gradients are summed over the ranks, either by one all-reduce of the
flat gradient buffer after the backward or -- `GNOT.set_grad_allreduce` -- group by group inside the
backward, overlapped with it (gnot_plan_set_grad_comm):

* sample data parallel (small meshes, BASELINE configs[1]/[4]): every rank owns whole meshes
  (`lpt_partition` balances them by point count); gradients are averaged / summed.
* point sharding (one large mesh, configs[3]): every sample's points are split over the ranks
  (`shard_range`); the engine calls back into `PointShardComm` for the two exchanges the reference's
  attention needs (include/gnot_hip.h: state all-reduce, scramble all-to-all) and the caller sums
  gradients over ranks.  `rel_l2_loss_sharded` is the reference loss (loss.py:14-23) on a sharded
  mesh: its per-sample sums are all-reduced.

The reference itself is single-device (main.py:27); nothing here has a reference counterpart beyond
the arithmetic it must reproduce.
"""
import contextlib
import ctypes
import heapq
import traceback

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def shard_range(n, rank, world):
    """[lo, hi) of the points of an n-point sample owned by `rank` (gnot_shard_range)."""
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.load().gnot_shard_range(int(n), int(rank), int(world), ctypes.byref(lo), ctypes.byref(hi)))
    return lo.value, hi.value


def shard_offsets(n_global, rank, world):
    """Local packed offsets [B+1] of this rank's slices, and the (lo, hi) range of every sample."""
    ranges = [shard_range(n, rank, world) for n in n_global]
    off = [0]
    for lo, hi in ranges:
        off.append(off[-1] + hi - lo)
    return off, ranges


def exchange_plan(n_global, n_head, head_dim, rank, world):
    """This rank's side of the scramble all-to-all (gnot_shard_exchange): send/recv counts per peer
    (floats) and the copy segments [k, 4] = (dir, local_off, buf_off, len)."""
    lib = _lib.load()
    B = len(n_global)
    ng = (ctypes.c_int64 * B)(*[int(n) for n in n_global])
    sc, rc = (ctypes.c_int64 * world)(), (ctypes.c_int64 * world)()
    nseg = ctypes.c_int64()
    _lib.check(lib.gnot_shard_exchange(B, ng, n_head, head_dim, rank, world, sc, rc, None, 0, ctypes.byref(nseg)))
    segs = (ctypes.c_int64 * (4 * max(nseg.value, 1)))()
    _lib.check(lib.gnot_shard_exchange(B, ng, n_head, head_dim, rank, world, sc, rc, segs, nseg.value,
                                       ctypes.byref(nseg)))
    arr = np.frombuffer(segs, dtype=np.int64)[: 4 * nseg.value].reshape(-1, 4).copy()
    return list(sc), list(rc), arr


def lpt_partition(sizes, world):
    """Longest-processing-time assignment of samples (point counts) to ranks: biggest first onto the
    least-loaded rank (ties -> lowest rank).  Returns per-rank lists of sample indices (ascending)."""
    heap = [(0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + sizes[i], r))
    return [sorted(v) for v in out]


class PointShardComm:
    """gnot_comm backed by a torch.distributed process group: the point-shard exchanges
    (GNOT.set_point_shard) and the overlapped gradient all-reduce (GNOT.set_grad_allreduce).

    The engine hands over raw pointers into its workspace; they are wrapped as float32 views of the
    workspace tensor (no copies).  With RCCL (`nccl` backend) every collective is issued on the
    stream the engine passes (the one its kernels run on, wrapped as a torch ExternalStream), so it is
    ordered after the producing kernels and before the consumers whatever torch's current stream is.
    `stage_via_host` routes them through host tensors instead (for the gloo backend, e.g. several
    ranks sharing one GPU in tests); the host copies then synchronise on that same stream."""

    def __init__(self, group=None, stage_via_host=False):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.stage = stage_via_host
        self.ws = None                        # the engine's uint8 workspace tensor (set by Engine)
        self.fail_next_captured = 0           # test knob: the n-th collective issued under capture fails (0: off)
        self._ar = _lib.ALLREDUCE_FN(self._allreduce)
        self._a2a = _lib.ALLTOALLV_FN(self._alltoallv)
        self.struct = _lib.GnotComm(None, self._ar, self._a2a)

    def _view(self, ptr, n):
        off = int(ptr) - self.ws.data_ptr()
        if off < 0 or off % 4 or off + 4 * n > self.ws.numel():
            raise RuntimeError("gnot_comm buffer outside the engine workspace")
        return self.ws[off: off + 4 * n].view(torch.float32)

    def _on(self, stream):
        """torch stream context for the engine's HIP stream handle (no-op for host buffers).  The null
        stream (handle 0: a caller whose current stream is torch's default stream) is torch's own default
        stream object, not ExternalStream(0) (tests/test_gpu_shard.py::test_comm_stream_orders_after_kernels)."""
        if self.ws is None or not self.ws.is_cuda:
            return contextlib.nullcontext()
        if not stream:
            return torch.cuda.stream(torch.cuda.default_stream(self.ws.device))
        return torch.cuda.stream(torch.cuda.ExternalStream(int(stream), device=self.ws.device))

    def _injected_failure(self):
        if self.fail_next_captured > 0 and torch.cuda.is_current_stream_capturing():
            self.fail_next_captured -= 1
            if self.fail_next_captured == 0:
                raise RuntimeError("injected collective failure under capture (PointShardComm.fail_next_captured)")

    def _allreduce(self, user, buf, count, stream):
        try:
            if count > 0:
                t = self._view(buf, count)
                with self._on(stream):
                    self._injected_failure()
                    if self.stage:
                        _no_capture()
                        # host staging (gloo, tests): the whole device first, then blocking copies.  Under
                        # ExternalStream(0) (a rank whose current stream is the null stream) .cpu() did NOT
                        # wait for the engine's kernels: the 2-rank sharded 70k test read state buffers before
                        # the state kernels ended (NaN forward at the first step, wrong gradients later;
                        # r04sf, r05c-f)
                        torch.cuda.synchronize(t.device)
                        h = t.cpu()
                        dist.all_reduce(h, group=self.group)
                        t.copy_(h)
                        torch.cuda.synchronize(t.device)
                    else:
                        dist.all_reduce(t, group=self.group)
            return 0
        except Exception:
            traceback.print_exc()
            return -1

    def _alltoallv(self, user, send, send_counts, recv, recv_counts, stream):
        try:
            sc = [int(send_counts[i]) for i in range(self.world)]
            rc = [int(recv_counts[i]) for i in range(self.world)]
            dev = self.ws.device
            with self._on(stream):
                self._injected_failure()
                s = self._view(send, sum(sc)) if sum(sc) else torch.empty(0, device=dev)
                r = self._view(recv, sum(rc)) if sum(rc) else torch.empty(0, device=dev)
                if self.stage:
                    _no_capture()
                    torch.cuda.synchronize(dev)
                    hr = torch.empty(sum(rc), dtype=torch.float32)
                    dist.all_to_all_single(hr, s.cpu(), rc, sc, group=self.group)
                    r.copy_(hr)
                    torch.cuda.synchronize(dev)
                else:
                    dist.all_to_all_single(r, s, rc, sc, group=self.group)
            return 0
        except Exception:
            traceback.print_exc()
            return -1


def _no_capture():
    """The host-staged collectives block on the device and copy through host memory, which a stream
    capture cannot record (and a device synchronize inside one invalidates the capture for the caller's
    later eager launches): refuse cleanly, so the engine call fails and bench.py runs eager steps."""
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("host-staged (gloo) collectives cannot be captured into a HIP graph")


class _SumOverRanks(torch.autograd.Function):
    """all-reduce(sum) whose backward is the identity: every rank evaluates the SAME loss from the
    reduced sums, so d loss / d (local partial) is the gradient of the reduced value itself."""

    @staticmethod
    def forward(ctx, t, group, stage):
        out = t.clone()
        if stage:
            _no_capture()
            h = out.cpu()
            dist.all_reduce(h, group=group)
            out.copy_(h)
        else:
            dist.all_reduce(out, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        return g, None, None


def rel_l2_loss_sharded(out, tgt, seg, B, group=None, stage_via_host=False):
    """RelL2Loss (loss.py:14-23) of meshes whose points are sharded over ranks: per-sample sums of
    (p - t)^2 and t^2 over ALL ranks' points, then mean over samples x channels of sqrt(num/den)."""
    C = out.shape[1]
    num = torch.zeros(B, C, device=out.device, dtype=out.dtype).index_add(0, seg, (out - tgt) ** 2)
    den = torch.zeros(B, C, device=out.device, dtype=out.dtype).index_add(0, seg, tgt ** 2)
    num = _SumOverRanks.apply(num, group, stage_via_host)
    den = _SumOverRanks.apply(den, group, stage_via_host)
    return (num / den).sqrt().mean()
