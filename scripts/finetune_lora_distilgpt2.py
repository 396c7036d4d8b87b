#!/usr/bin/env python
"""distilgpt2 LoRA DDP fine-tune — drop-in for the reference
`Cluster/Project 1 - Fine Tuning Distilgpt2/finetune_lora_distilgpt2.py` (same CLI).
Launch: torchrun --nproc-per-node 8 scripts/finetune_lora_distilgpt2.py --dataset medium
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.apps.ddp_finetune import main  # noqa: E402

if __name__ == "__main__":
    main()
