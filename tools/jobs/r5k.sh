#!/bin/bash
# round 5: rowproj MFMA row passes at the OPT widths (tests, kernel A/B, OPT step A/B) + decode breakdown
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r5k
mkdir -p $O
bash tools/gpu_job.sh \
  "r5k/tests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread -k 'rowproj or ln_bwd_mask or lora_proj_and or handoff or opt'" \
  "r5k/bench_rowproj:200:python tools/bench_rowproj_opt.py --json $O/bench_rowproj_opt.json" \
  "r5k/step_ab_opt:400:python tools/step_ab.py --model facebook/opt-2.7b 'MIFT_ROWPROJ_WIDE=0' 'MIFT_ROWPROJ_WIDE=1' --blocks 4 --steps 5 --json $O/step_ab_opt.json" \
  "r5k/probe:200:python -m mift.apps.gen_probe --repeat 5 && python -m mift.apps.gen_probe --repeat 5 --prompts distinct" \
  "r5k/kt:300:rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -m mift.apps.gen_probe --repeat 2 && python tools/gen_timeline.py $O/kt/run_kernel_trace.csv > $O/gen_timeline.txt"
