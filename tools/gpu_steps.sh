#!/bin/bash
# Run GPU steps in order; each line of the step file is "<timeout_s> <command...>".
# Stops after a step that faulted, aborted, segfaulted or timed out (rc 124/134/137/139 or >128),
# continues after ordinary failures (rc 1/2). Logs go to gpurun_out/steps.log.
# usage: bash tools/gpu_steps.sh .steps/<stepfile> (step lists are untracked scratch under .steps/)
mkdir -p gpurun_out
while IFS= read -r line; do
  [ -z "$line" ] && continue
  case "$line" in \#*) continue;; esac
  t=${line%% *}; cmd=${line#* }
  echo "=== [$t s] $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" bash -c "$cmd" >> gpurun_out/steps.log 2>&1
  rc=$?
  echo "=== rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc" | tee -a gpurun_out/steps.log; exit $rc; fi
done < "$1"
