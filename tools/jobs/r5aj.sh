#!/bin/bash
# round 5 final tree: full GPU suite, smoke, bench, 2-rank gloo rehearsal of the DDP bench path on one GPU
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5aj
mkdir -p $O
bash tools/gpu_job.sh \
  "r5aj/gpu_tests:1000:python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread" \
  "r5aj/smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r5aj/bench:300:python bench.py" \
  "r5aj/ddp2_gloo:400:MIFT_BACKEND=gloo python bench.py --gpus 2 --steps 10 --warmup 3 --epoch_lines 0" \
  "r5aj/probe:200:python -m mift.apps.gen_probe --repeat 10"
