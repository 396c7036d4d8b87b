"""Zero1AdamW stands in for FusedAdamW inside the Trainer: every ``self.opt.<attr>`` the Trainer
uses must exist on it (a missing ``g`` / ``stats_buf`` broke the ZeRO-1 path at the setup-time
warm-up on GPU only, where the CPU tests could not see it)."""
import os
import re

import torch

from mift.parallel.zero import Zero1AdamW
from mift.train import trainer as T


class _Arena:
    def __init__(self, n):
        self.numel = n
        self.param = torch.zeros(n)
        self.grad = torch.zeros(n)


def test_zero1_has_trainer_optimizer_surface():
    src = open(T.__file__).read()
    used = sorted(set(re.findall(r"self\.opt\.(\w+)", src)))
    assert "g" in used and "stats_buf" in used, used
    z = Zero1AdamW(_Arena(64), None, 1, 0, lr=1e-3)
    missing = [a for a in used if not hasattr(z, a)]
    assert not missing, missing
    assert z.g.numel() == 64 and z.stats_buf.numel() == 2
