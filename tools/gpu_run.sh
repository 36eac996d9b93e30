#!/bin/bash
# Run GPU steps in order on the gpurun box; continue past ordinary test failures
# (exit 1) but stop at the first crash / abort / timeout (any other non-zero).
# usage: tools/gpu_run.sh "<timeout-seconds> <command...>" ["<timeout> <command...>" ...]
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
worst=0
for step in "$@"; do
  i=$((i+1))
  t=${step%% *}
  cmd=${step#* }
  echo "=== step $i (timeout ${t}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/step$i.log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 30 "gpurun_out/step$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $i exited $rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
