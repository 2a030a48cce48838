#!/bin/bash
# PMC passes of the cfg3 pass for each A/B build (tools/ab_build.sh), one counter
# set per run, no trace domains: gpurun_out/ab_pmc/<variant>_<set>/
set -o pipefail
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-$(ls tools/build/ab)}
args="--steps 3 --warmup 1 --no-cpu-baseline"
# PMC_SETS: counter sets separated by ';' (each at most 8 SQ counters)
if [ -n "$PMC_SETS" ]; then
  IFS=';' read -r -a sets <<< "$PMC_SETS"
else
  sets=("SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
        "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
        "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY")
fi
for v in $VARIANTS; do
  for i in "${!sets[@]}"; do
    out=gpurun_out/ab_pmc/${v}_$i
    mkdir -p $out
    VLGBA_LIB=tools/build/ab/$v/libvlgba.so timeout -k 10 120 rocprofv3 --pmc ${sets[$i]} -d $out -o pmc --output-format csv -- python3 bench.py $args > $out.log 2>&1
    rc=$?; echo "== $v set $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out.log; exit $rc; }
  done
done
exit 0
