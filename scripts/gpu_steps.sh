#!/bin/bash
# Run GPU steps in order; stop at the first step that ends in a GPU-fault-like way
# (abort 134, segfault 139, timeout 124/137, or any signal) -- never start another GPU step
# after one of those.  Plain test failures (rc 1) continue to the next step.
# usage: scripts/gpu_steps.sh "cmd1" "cmd2" ...
for cmd in "$@"; do
  echo "=== step: $cmd"
  bash -c "$cmd"
  rc=$?
  echo "=== rc=$rc"
  case $rc in
    0|1|2|4|5) ;;
    *) echo "=== stopping after rc=$rc"; exit $rc ;;
  esac
done
