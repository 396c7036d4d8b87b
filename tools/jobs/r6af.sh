#!/bin/bash
# round 6: whole-sequence attention kernels with compile-time diagonal masks / keep-bit variants;
# LoRA wgrad reduce batches; attention + LoRA tests, step timeline, bench
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6af
mkdir -p $O
bash tools/gpu_job.sh \
  "r6af/tests:600:python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attn or attention or wgrad or lora or seq'" \
  "r6af/kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0 && python tools/step_timeline.py $O/kt/run_kernel_trace.csv > $O/step_timeline.txt" \
  "r6af/bench:300:python -u bench.py --steps 20 --warmup 5 --epoch_lines 0 > $O/bench.jsonl && python -u bench.py --steps 20 --warmup 5 --epoch_lines 0 >> $O/bench.jsonl"
