#!/usr/bin/env python
"""S(n)/E(n) table from bench.py JSON lines or log dirs: scaling_report.py SCALE.json|logdir ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift.obs.logparse import read_meta, scaling, training_seconds  # noqa: E402


def main(args):
    times = {}
    for a in args:
        if os.path.isdir(a):
            n = int(read_meta(a).get("world_size", read_meta(a).get("nnodes", 1)))
            times[n] = training_seconds(a)
            continue
        with open(a) as f:
            for line in f:
                line = line.strip()
                if line.startswith("{"):
                    d = json.loads(line)
                    # weak scaling: time per unit of work = ms_per_step / n
                    times[int(d["n_gpus"])] = d["ms_per_step"] / (d["n_gpus"] if d.get("scaling") == "weak" else 1)
    print(f"{'N':>3} {'T(N)':>12} {'S(N)':>8} {'E(N)':>8}")
    for n, (s, e) in scaling(times).items():
        print(f"{n:>3} {times[n]:>12.4f} {s:>8.3f} {e:>8.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
