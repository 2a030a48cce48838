#!/bin/bash
# Ladybug pass evidence (GPU box, repo root): kernel trace + stats, and one PMC
# pass with the MFMA-busy counters, under gpurun_out/<TAG>_ladybug_*.
# usage: tools/prof_ladybug.sh TAG
set -o pipefail
export TMPDIR=/tmp
tag=${1:?usage: tools/prof_ladybug.sh TAG}
out=gpurun_out/${tag}_ladybug
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv \
  -- python3 bench.py --config ladybug --steps 5 --warmup 1 --no-cpu-baseline \
  > $out/trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d $out/pmc -o pmc --output-format csv \
  -- python3 bench.py --config ladybug --steps 2 --warmup 1 --no-cpu-baseline \
  > $out/pmc.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/pmc > $out/pmc_summary.csv
