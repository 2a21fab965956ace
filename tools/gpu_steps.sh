#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that did not
# end with 0 (success) or 1 (test failures): a fault, abort, time limit or hang ends the call.
#   tools/gpu_steps.sh "<limit_s> <name> <command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  lim=${spec%% *}; rest=${spec#* }; name=${rest%% *}; cmd=${rest#* }
  echo "[gpu_steps] $name (limit ${lim}s): $cmd"
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_steps] stopping after $name"; exit $rc; fi
done
