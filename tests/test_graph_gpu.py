"""hipGraph-replayed training steps (mift.train.graph) vs the eager fused path.

Same seeds, same data: graph replay must draw the same dropout masks (device
micro-step counter, csrc/common.h mift_seed) and produce the same losses and
LoRA parameters as eager execution, step after step (tolerance only for the
fp32 atomic accumulation order of the LoRA weight-gradient kernels, which Adam
amplifies to +-lr on gradients that are zero up to rounding)."""
import pytest
import torch

import mift
from mift import lora as L
from mift.data import MicroBatcher, synthetic_openwebtext
from mift.models import build_causal_lm
from mift.train.trainer import TrainConfig, Trainer

pytestmark = pytest.mark.gpu


def _run(graph, model_name, steps=5, mb=4, accum=2, S=128, precision="bf16"):
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16 if precision == "bf16" else torch.float16
    model = build_causal_lm(model_name, dtype=dtype, device=dev, seed=0)
    targets = ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"] if "opt" in model_name else ["c_attn", "c_proj"]
    L.inject(model, L.LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=targets))
    with torch.no_grad():  # non-zero B so every LoRA path carries signal from step 1
        for n, p in model.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.02, generator=torch.Generator(device=dev).manual_seed(len(n)))
    ds = synthetic_openwebtext(mb * accum * steps, S, model.config.vocab_size, model.config.pad_token_id, seed=3,
                               full_length=False)
    batcher = MicroBatcher(ds, mb, accum)
    from mift.parallel import dist as D
    ctx = D.init(verbose=False, sanity=False)
    tr = Trainer(model, batcher, TrainConfig(epochs=1, batch=mb, accum=accum, lr=1e-3, precision=precision,
                                             logging_steps=0, save_steps=0, step_log="none",
                                             graph="on" if graph else "off"), ctx)
    model.train()
    losses, gnorms = [], []
    for mbs in batcher.epoch(0):
        loss, ntok = tr.train_step(mbs)
        losses.append(float(loss) / ntok)
        gnorms.append(float(tr.opt.stats()["grad_norm"]))
    torch.cuda.synchronize()
    return losses, tr.arena.param.clone(), tr, gnorms


@pytest.mark.parametrize("name,precision,steps", [("distilgpt2", "bf16", 20), ("facebook/opt-125m", "fp16", 5)])
def test_graph_replay_matches_eager(name, precision, steps):
    """20 optimizer steps (distilgpt2): graphed and eager loss AND grad-norm trajectories agree."""
    assert mift.kernels_available()
    le, pe, _, ge = _run(False, name, steps=steps, precision=precision)
    lg, pg, tr, gg = _run(True, name, steps=steps, precision=precision)
    assert tr.graphed is not None and len(tr.graphed.graphs) == 1, "graph was not captured"
    assert le[0] == pytest.approx(lg[0], rel=1e-6, abs=1e-6)  # step 1 is the eager warm-up in both
    for a, b in zip(le, lg):
        assert a == pytest.approx(b, rel=1e-4, abs=1e-4), (le, lg)
    for a, b in zip(ge, gg):
        assert a == pytest.approx(b, rel=1e-2, abs=1e-5), (ge, gg)  # Adam-amplified atomics noise
    # Neither path is bit-reproducible: the LoRA weight-gradient kernels accumulate with fp32
    # atomics, and Adam's first steps move every element by ~lr * sign(g), so a gradient that is
    # ~0 up to rounding can flip sign between runs and shift that element by up to 2*lr per step
    # (measured on MI355X: eager-vs-eager and graph-vs-graph both reach ~0.93*lr).  A real replay
    # bug (stale inputs, repeated masks, stale LoRA operands) moves the bulk of the parameters and
    # the losses instead, so bound the fraction of disagreeing elements and the losses.
    lr = 1e-3
    d = (pe - pg).abs()
    frac = (d > 0.2 * lr).float().mean().item()
    assert d.max().item() <= 2 * lr * steps + 1e-6, d.max().item()
    assert frac < 0.01, frac
    assert len(set(round(x, 6) for x in lg)) == len(lg), "replays must not repeat masks/losses"
