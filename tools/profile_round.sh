#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box, from the repo root):
#   trace: --kernel-trace --stats of the default bench command
#   pmc*:  separate counter passes (never combined with any trace domain):
#          HBM bytes (FETCH_SIZE and WRITE_SIZE cost 3 + 2 TCC slots: two passes)
#          and SQ occupancy / stall / LDS counters.
# usage: tools/profile_round.sh OUTDIR [bench args...]
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/prof}; shift
args=${*:---steps 10 --warmup 2 --no-cpu-baseline}
mkdir -p "$out"
run() {   # name seconds rocprof-args...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv \
    -- python3 bench.py $args > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$out/$name.log"
  return $rc
}
run trace 300 --kernel-trace --stats &&
run pmc_fetch 300 --pmc FETCH_SIZE &&
run pmc_write 300 --pmc WRITE_SIZE &&
run pmc_sq 300 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS &&
run pmc_lds 300 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
  SQ_INSTS_VMEM_WR SQ_INSTS_SALU
