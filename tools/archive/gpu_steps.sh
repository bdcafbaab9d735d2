#!/bin/bash
# Run GPU test steps one process each; continue past ordinary test failures
# (exit 1) but stop at the first crash-like exit (abort, segfault, timeout).
# usage: tools/gpu_steps.sh LOGDIR "step command" ["step command" ...]
out=$1; shift
mkdir -p "$out"
i=0
for cmd in "$@"; do
  i=$((i + 1))
  echo "=== step $i: $cmd" | tee -a "$out/steps.log"
  timeout -k 10 600 bash -c "$cmd" > "$out/step$i.log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc" | tee -a "$out/steps.log"
  tail -5 "$out/step$i.log" >> "$out/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc" | tee -a "$out/steps.log"; exit $rc; fi
done
exit 0
