"""Collective / point-to-point helpers that pick the right primitive per backend.

RCCL (backend "nccl" on ROCm) moves device tensors directly over xGMI and
orders work on the current HIP stream (``Work.wait()`` makes the stream wait;
the host does not block).  Gloo — the CPU plumbing backend, also used to
rehearse multi-rank pipelines on a single GPU box — only moves host tensors,
so device tensors are staged through pinned host memory there.

Reference parity: DeepSpeed's pipeline p2p (``deepspeed.runtime.pipe.p2p``,
[lib]) and ZeRO-1 reduce-scatter / all-gather (X13).
"""
import torch
import torch.distributed as dist


def backend_of(group=None):
    return dist.get_backend(group) if dist.is_initialized() else "none"


def _host_staged(group):
    return backend_of(group) == "gloo"


class P2P:
    """Paired send/recv between adjacent pipeline stages (global ranks)."""

    def __init__(self, group=None):
        self.group = group
        self.gloo = _host_staged(group)

    def exchange(self, sends=(), recvs=()):
        """sends: [(tensor, dst)], recvs: [(tensor, src)] -> completes all, returns recv tensors.

        NCCL/RCCL: one ``batch_isend_irecv`` (grouped, deadlock-free for the
        1F1B send-fwd/recv-bwd pairs); gloo: host copies + isend/irecv."""
        if not sends and not recvs:
            return []
        if not self.gloo:
            ops = [dist.P2POp(dist.isend, t, peer, group=self.group) for t, peer in sends]
            ops += [dist.P2POp(dist.irecv, t, peer, group=self.group) for t, peer in recvs]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            return [t for t, _ in recvs]
        works, stage = [], []
        for t, peer in sends:
            h = t.detach().to("cpu") if t.is_cuda else t.detach().contiguous()
            stage.append(h)
            works.append(dist.isend(h, peer, group=self.group))
        outs = []
        for t, peer in recvs:
            h = torch.empty(t.shape, dtype=t.dtype) if t.is_cuda else t
            outs.append((t, h))
            works.append(dist.irecv(h, peer, group=self.group))
        for w in works:
            w.wait()
        for t, h in outs:
            if h is not t:
                t.copy_(h)
        return [t for t, _ in recvs]


def reduce_scatter_flat(out, inp, group):
    """out[i] = sum over ranks of inp[rank_idx*n + i]   (n = out.numel())."""
    if backend_of(group) == "gloo":
        buf = inp.clone()
        dist.all_reduce(buf, group=group)
        r = dist.get_rank(group)
        out.copy_(buf[r * out.numel():(r + 1) * out.numel()])
    else:
        dist.reduce_scatter_tensor(out, inp, group=group)


def all_gather_flat(out, shard, group):
    """out = concat over ranks of shard."""
    if backend_of(group) == "gloo":
        n = shard.numel()
        views = [out[i * n:(i + 1) * n] for i in range(dist.get_world_size(group))]
        tmp = [torch.empty_like(shard) for _ in views]
        dist.all_gather(tmp, shard.contiguous(), group=group)
        for v, t in zip(views, tmp):
            v.copy_(t)
    else:
        dist.all_gather_into_tensor(out, shard.contiguous(), group=group)
