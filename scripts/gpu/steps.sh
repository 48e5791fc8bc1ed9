#!/bin/bash
# GPU-box driver: runs steps in order; continues past plain test failures
# (pytest rc=1) but stops at anything that looks like a fault/abort/timeout.
# usage: scripts/gpu/steps.sh "<step1 cmd>" "<step2 cmd>" ...
mkdir -p gpurun_out
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" | tee -a gpurun_out/steps.log
  bash -c "$cmd"
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
