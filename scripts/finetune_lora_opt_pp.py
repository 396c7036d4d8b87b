#!/usr/bin/env python
"""OPT LoRA pipeline-parallel fine-tune — drop-in for the reference
`Cluster/Project 2 - Course Project/finetune_lora_opt_pp.py` (same CLI, same env contract).
Launch (one 8x MI355X node, 4 stages x 2 replicas):
  PIPELINE_PARALLEL_SIZE=4 torchrun --nproc-per-node 8 --master-addr 127.0.0.1 \
      scripts/finetune_lora_opt_pp.py --data_file data.txt --seq_len 512 --accum 96 --ds_cfg configs/ds_pp_zero1_mi355x.json
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.apps.pp_finetune import main  # noqa: E402

if __name__ == "__main__":
    main()
