"""The P2 entry point (``finetune_lora_opt_pp.py`` CLI, mift.apps.pp_finetune) end to end on CPU:
2 pipeline ranks over gloo, tiny OPT, interleaved chunks, the reference's loss lines / timing log /
meta.json contract."""
import json
import os

from mift.utils import harness


def _run(rank, world, out, extra):
    from mift.apps.pp_finetune import main
    return main(["--model_name", "opt-tiny", "--data_file", os.path.join(out, "missing.txt"), "--synthetic", "64",
                 "--seq_len", "16", "--batch", "1", "--accum", "8", "--lr", "1e-3", "--log_every", "1",
                 "--max_steps", "2", "--out_root", out, "--logdir", os.path.join(out, "logs"),
                 "--ds_cfg", "none.json"] + extra)


def test_pp_app_interleaved_two_ranks(tmp_path):
    out = str(tmp_path)
    r = harness.run(_run, 2, out=out, extra=["--virtual_stages", "2", "--micro_batch", "2"])
    assert r[0]["steps"] == 2 and r[0]["virtual_stages"] == 2 and r[0]["micro_batch"] == 2
    assert len(r[0]["split"]) == 4 and min(r[0]["split"]) >= 1
    meta_dirs = [d for d in os.listdir(out) if d.startswith("opt27b_lora_pp_")]
    assert len(meta_dirs) == 1
    meta = json.load(open(os.path.join(out, meta_dirs[0], "meta.json")))
    assert meta["stages"] == 2 and meta["virtual_stages"] == 2 and meta["micro_batch"] == 2
    assert meta["micro_batches_per_step"] == 4
    assert os.path.exists(os.path.join(out, meta_dirs[0], "adapter_model.safetensors"))
    for rk in range(2):
        assert "[Training]" in open(os.path.join(out, "logs", f"timing_rank{rk}.log")).read()
    # the reference summariser (P2/summarize_opt_times.py CLI) reads the app's [Training] lines
    from mift.obs.logparse import summarize_times
    rep = summarize_times([os.path.join(out, "logs")], "OPT")
    assert "train=" in rep and "train=n/a" not in rep, rep
