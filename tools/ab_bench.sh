#!/bin/bash
# Same-box A/B of env-switchable kernel choices: interleaved bench.py runs (guide rule 24).
# usage: bash tools/ab_bench.sh "<envA>" "<envB>" [rounds] [bench args...]
A="$1"; B="$2"; R=${3:-2}; shift 3
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for arm in A B; do
    E=$([ $arm = A ] && echo "$A" || echo "$B")
    timeout -k 10 200 env $E python bench.py --epoch_lines 0 "$@" > gpurun_out/ab/${arm}_$r.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab/${arm}_$r.json').read().strip().splitlines()[-1]); print('$arm', '$E', d['ms_per_step'])"
  done
done
