#!/bin/bash
# Round-3 third GPU pass: PP graph fix (per-slot pools) + eager-vs-graph diagnostics + PP4 rehearsal,
# attention after the dkdv padding rotation, step kernel trace, generation probe (padded) trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
bash tools/gpu_job.sh \
  "c_diag:300:python tools/diag_graph_eager.py --model facebook/opt-125m --precision fp16 --steps 3" \
  "c_tests:600:python -u -m pytest tests/test_pipeline_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py -q --timeout 300 --timeout-method thread -k 'pipeline or graph or attention or flash'" \
  "c_attn:120:python tools/bench_attn.py" \
  "c_pmcattn:120:rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmcattn -o run -- python3 tools/bench_attn.py && python tools/pmc_summary.py $O/pmcattn --top 12" \
  "c_kt:240:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --epoch_lines 0" \
  "c_gen:200:python scripts/gen_probe.py --prompts distinct --repeat 3 && python scripts/gen_probe.py --repeat 3" \
  "c_genkt:200:rocprofv3 --kernel-trace --stats --output-format csv -d $O/genkt -o run -- python3 scripts/gen_probe.py --prompts distinct" \
  "c_pp4:900:python tools/rehearse_pp.py --model facebook/opt-2.7b --pp 4 --seq 512 --mb 4 --accum 24 --steps 3"
