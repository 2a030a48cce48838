#!/bin/bash
# texture-path counters of the cfg3 pass (GPU box, repo root): TA / TD busy and
# TCP requests per kernel (separate passes, no trace domains)
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/prof_ta}
mkdir -p "$out"
args="--steps 5 --warmup 1 --no-cpu-baseline"
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv \
    -- python3 bench.py $args > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; return $rc
}
run ta --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE &&
run td --pmc TD_BUSY_avr GRBM_COUNT &&
run tcp --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
