"""Collective / point-to-point helpers: ONE call path for RCCL and Gloo.

Every backend goes through the same torch.distributed calls —
``batch_isend_irecv`` for pipeline p2p, ``reduce_scatter_tensor`` /
``all_gather_into_tensor`` for ZeRO-1 — so the multi-process Gloo tests on
the CPU exercise exactly the op grouping, ordering and shapes that RCCL runs
over xGMI.  The only backend difference is host staging: Gloo moves host
tensors, so device tensors are copied through host memory around the call
(the GPU-box rehearsal of multi-rank schedules on one device); RCCL moves
device tensors directly and orders its work against the current HIP stream
(``Work.wait()`` makes the stream wait; the host does not block).

Reference parity: DeepSpeed's pipeline p2p (``deepspeed.runtime.pipe.p2p``,
[lib]) and ZeRO-1 reduce-scatter / all-gather (X13).
"""
import torch
import torch.distributed as dist

from ..obs.profiler import rng


def backend_of(group=None):
    return dist.get_backend(group) if dist.is_initialized() else "none"


def _host_staged(group, *tensors):
    return backend_of(group) == "gloo" and any(t.is_cuda for t in tensors)


class Pending:
    """Outstanding p2p exchange: ``wait()`` completes it and returns the received tensors."""

    def __init__(self, works, recvs, copies, keep):
        self._works, self._recvs, self._copies, self._keep = works, recvs, copies, keep
        self.done = False

    def wait(self):
        if not self.done:
            for w in self._works:
                w.wait()
            for dst, src in self._copies:  # host-staged receives land in their device tensors
                dst.copy_(src, non_blocking=False)
            self._works, self._keep, self.done = [], None, True
        return self._recvs


class P2P:
    """Grouped send/recv between pipeline stages (global ranks).

    ``group`` selects the communicator; the pipeline engine uses one group per
    DIRECTION (activations s→s+1, gradients s+1→s) so that a receive posted
    early on one direction never queues behind a send on the other (RCCL runs
    the p2p of one communicator and peer pair in issue order on one stream)."""

    def __init__(self, group=None):
        self.group = group

    def post(self, sends=(), recvs=()):
        """Issue ``sends`` [(tensor, dst)] and ``recvs`` [(tensor, src)] as ONE batch_isend_irecv."""
        sends, recvs = list(sends), list(recvs)
        if not sends and not recvs:
            return Pending([], [], [], None)
        staged = _host_staged(self.group, *[t for t, _ in sends + recvs])
        ops, copies, keep = [], [], []
        for t, peer in sends:
            src = t.detach()
            if staged and src.is_cuda:
                src = src.to("cpu")
            keep.append(src)
            ops.append(dist.P2POp(dist.isend, src.contiguous(), peer, group=self.group))
        for t, peer in recvs:
            dst = t
            if staged and t.is_cuda:
                dst = torch.empty(t.shape, dtype=t.dtype)
                copies.append((t, dst))
            keep.append(dst)
            ops.append(dist.P2POp(dist.irecv, dst, peer, group=self.group))
        with rng(f"mift.pp.p2p.s{len(sends)}r{len(recvs)}"):
            works = dist.batch_isend_irecv(ops)
        return Pending(works, [t for t, _ in recvs], copies, keep)

    def exchange(self, sends=(), recvs=()):
        """Blocking form of :meth:`post` (returns the received tensors)."""
        return self.post(sends, recvs).wait()


def reduce_scatter_flat(out, inp, group):
    """out[i] = sum over ranks of inp[rank_idx*n + i]   (n = out.numel())."""
    if _host_staged(group, out, inp):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(h, inp.detach().cpu(), group=group)
        out.copy_(h)
    else:
        dist.reduce_scatter_tensor(out, inp, group=group)


def all_gather_flat(out, shard, group):
    """out = concat over ranks of shard."""
    if _host_staged(group, out, shard):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, shard.detach().cpu().contiguous(), group=group)
        out.copy_(h)
    else:
        dist.all_gather_into_tensor(out, shard.contiguous(), group=group)
