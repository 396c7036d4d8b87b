"""Per-optimizer-step packing of every adapter's 16-bit GEMM operands.

LoRA parameters only change at the optimizer step, so the padded bf16/fp16
operands the fused kernels consume (A32s = s·A [32,K], B32 [N,32],
B32t [32,N], At32 [K,32]) are produced for ALL adapted Linears by one
kernel launch per step (``pack_lora_all``) into one persistent buffer, and
each Linear keeps views into it.  With the reference's batch 1 × accum 32
schedule this is 32× fewer pack launches than packing per micro-batch.
"""
import torch

from ..ops.dispatch import C


class LoraPack:
    def __init__(self, arena, dtype):
        self.arena, self.dtype = arena, dtype
        rows, scales, off, self.max_elems = [], [], 0, 0
        dev = arena.param.device
        layouts = []
        for m in arena.modules:
            K, N, r = m.in_features, m.out_features, m.lora_r
            n = 64 * (K + N)
            rows.append([r, K, N, m._offA, m._offB, off])
            scales.append(m.lora_scaling)
            layouts.append((m, off, K, N))
            off += (n + 63) // 64 * 64
            self.max_elems = max(self.max_elems, n)
        self.buf = torch.zeros(max(off, 1), dtype=dtype, device=dev)
        self.table = torch.tensor(rows, dtype=torch.int64, device=dev).view(-1, 6)
        self.scales = torch.tensor(scales, dtype=torch.float32, device=dev)
        for m, o, K, N in layouts:
            b = self.buf
            A32s = b[o:o + 32 * K].view(32, K)
            o2 = o + 32 * K
            B32 = b[o2:o2 + 32 * N].view(N, 32)
            o3 = o2 + 32 * N
            B32t = b[o3:o3 + 32 * N].view(32, N)
            o4 = o3 + 32 * N
            At32 = b[o4:o4 + 32 * K].view(K, 32)
            m._pack = (A32s, B32, B32t, At32)
            m._pack_owner = self
        self.version = -1
        # shared-input adapter groups (ops.fused.MultiAdapterOps, e.g. OPT q/k/v): registered on first
        # use (an eager pass: the Trainer's warm-up precedes any capture), packed by one launch per step
        self.groups = {}
        self.mtable = self.mscales = None
        self.mmax = 0

    def refresh(self, force=False):
        if force or self.version != self.arena.version:
            C().pack_lora_all(self.arena.param, self.table, self.scales, self.buf, self.max_elems)
            if self.groups:
                C().pack_lora_multi(self.arena.param, self.mtable, self.mscales, self.mmax,
                                    self.dtype == torch.bfloat16)
            self.version = self.arena.version

    def multi(self, key, K, N, slots):
        """Views (A32s [32,K], B32 [N,32], B32t [32,N], At32 [K,32]) of the group ``key`` whose adapters
        are ``slots`` = [(lin, n0, n1, q)] (rank columns [q, q + r), output rows [n0, n1)); its operands
        are rebuilt with every other adapter's by ``refresh``."""
        g = self.groups.get(key)
        if g is None:
            assert len(slots) <= 4, "pack_lora_multi: at most 4 adapters per group"
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("LoraPack.multi: first use of an adapter group inside a graph capture")
            dev = self.arena.param.device
            buf = torch.zeros(64 * (K + N), dtype=self.dtype, device=dev)
            row = [K, N, len(slots), buf.data_ptr()]
            sc = []
            for lin, n0, n1, q in slots:
                row += [lin.lora_r, q, n0, n1, lin._offA, lin._offB]
                sc.append(lin.lora_scaling)
            row += [0] * (28 - len(row))
            sc += [0.0] * (4 - len(sc))
            views = (buf[:32 * K].view(32, K), buf[32 * K:32 * (K + N)].view(N, 32),
                     buf[32 * (K + N):32 * (K + 2 * N)].view(32, N), buf[32 * (K + 2 * N):].view(K, 32))
            g = self.groups[key] = (buf, views, row, sc)
            rows = [v[2] for v in self.groups.values()]
            self.mtable = torch.tensor(rows, dtype=torch.int64, device=dev)
            self.mscales = torch.tensor([v[3] for v in self.groups.values()], dtype=torch.float32, device=dev)
            self.mmax = max(self.mmax, 64 * (K + N))
            self.refresh(force=True)
        else:
            self.refresh()
        return g[1]


def attach(model, arena, dtype):
    """Create (or return) the model's LoraPack; kernels then use it automatically."""
    pk = getattr(model, "_lora_pack", None)
    if pk is None or pk.arena is not arena or pk.dtype != dtype:
        pk = LoraPack(arena, dtype)
        model._lora_pack = pk
    return pk
