#!/bin/bash
# Run GPU steps in order; each step under its own time limit.  A normal test
# failure (rc 1) continues; a fault / abort / segfault / time limit stops.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "== stopping after $name (rc=$rc)"; exit $rc ;;
  esac
done
