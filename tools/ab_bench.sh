#!/bin/bash
# cfg3 bench of every A/B build under tools/build/ab (tools/ab_build.sh), alternated
# REPS times (default 2), each under its own time limit; prints ms/pass and the
# fused / Schur / CR kernel averages.  usage: tools/ab_bench.sh [REPS]
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 ${1:-2}); do
  for v in $(ls tools/build/ab); do
    VLGBA_LIB=tools/build/ab/$v/libvlgba.so timeout -k 10 300 python -u bench.py --steps 100 \
      --warmup 50 --no-cpu-baseline --no-other-configs > gpurun_out/ab_${v}_$r.json \
      2> gpurun_out/ab_${v}_$r.log || { tail -5 gpurun_out/ab_${v}_$r.log; exit 1; }
    echo "$v run $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_$r.json) $(grep -o 'k_update_linearize=[0-9.]*us' gpurun_out/ab_${v}_$r.log | head -1) $(grep -o 'k_schur_mfma=[0-9.]*us' gpurun_out/ab_${v}_$r.log | head -1) $(grep -o 'k_cr32_fused=[0-9.]*us' gpurun_out/ab_${v}_$r.log | head -1)"
  done
done
