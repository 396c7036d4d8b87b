#!/bin/bash
# Round-3 sixth GPU pass: 4-wave MFMA row projection (tests, bench, step A/B), eager-DDP replica
# divergence diagnosis, 2dp x 4pp rehearsal against a dp2 reference, wgrad block-count A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "f_rp_tests:200:python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k 'rowproj or lora_proj'" \
  "f_rp_bench:200:python tools/bench_rowproj.py" \
  "f_ddp:300:python tools/diag_ddp_eager.py --graph 0 --steps 3" \
  "f_ab:400:python tools/step_ab.py 'MIFT_ROWPROJ_V=0' 'MIFT_ROWPROJ_V=1' 'MIFT_WGRAD_BLOCKS=1024' 'MIFT_WGRAD_BLOCKS=512'" \
  "f_bench:300:python bench.py --epoch_lines 0" \
  "f_dp2pp4:300:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --dp 2 --seq 512 --mb 4 --accum 24 --steps 3"
