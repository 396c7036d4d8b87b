#!/bin/bash
# round 4, second GPU call: new GPU tests (graphed decode, loss scaler), generation probe eager vs graphed,
# RAG over the queries file (1 rank and 2 gloo ranks).
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r4b
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_job.sh \
  "r4b/pytest_new:400:python -u -m pytest tests/test_infer_gpu.py tests/test_loss_scale_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "r4b/gen_eager:200:MIFT_GEN_GRAPH=0 python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4b/gen_graph:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5" \
  "r4b/gen_graph_distinct:200:python scripts/gen_probe.py --n_prompts 64 --max_new_tokens 16 --repeat 5 --prompts distinct" \
  "r4b/rag1:300:python labs/ragging/rag_example.py --subset 2000 --queries_file labs/ragging/queries.txt --max_new_tokens 32" \
  "r4b/rag2:300:MIFT_BACKEND=gloo $TR --nproc-per-node 2 --master-port 29651 labs/ragging/rag_example.py --subset 2000 --queries_file labs/ragging/queries.txt --max_new_tokens 32"
