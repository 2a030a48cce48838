#!/bin/bash
# A/B timing on the GPU box of the builds under tools/build/ab/ (tools/ab_build.sh),
# alternated R times; cfg3 pass unless BENCH_ARGS says otherwise.
R=${R:-2}
VARIANTS=${VARIANTS:-$(ls tools/build/ab)}
ARGS=${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu-baseline}
mkdir -p gpurun_out
: > gpurun_out/ab.log
for r in $(seq $R); do
  for v in $VARIANTS; do
    echo "== $v" >> gpurun_out/ab.log
    VLGBA_LIB=tools/build/ab/$v/libvlgba.so timeout -k 10 120 python -u bench.py $ARGS > gpurun_out/ab_$v.out 2>&1 || { echo "FAIL $v rc=$?"; tail -5 gpurun_out/ab_$v.out; exit 1; }
    grep -E "ms/iteration|kernels" gpurun_out/ab_$v.out >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
