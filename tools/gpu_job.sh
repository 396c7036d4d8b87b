#!/bin/bash
# Run GPU steps in order; stop at the first fatal exit (fault/abort/timeout).
# usage: tools/gpu_job.sh "<name>:<timeout_s>:<cmd>" ...
# rc 0/1 (test failures) continue; 124/134/137/139 or any rc>=2 except 1 stop the chain.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] timeout=${to}s :: $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -5 "gpurun_out/${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
done
exit 0
