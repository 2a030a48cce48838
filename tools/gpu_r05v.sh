#!/bin/bash
# round 5v: envelope trailing-workgroup cap (VLGBA_TRAIL_WGS) and
# k_schur_reduce's XCD-range block order (VLGBA_REDUCE_XCD): bit-identity
# tests, per-pass kernel times and stamps at cfg5x-900, PMC of the reduction
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reduce_xcd.py tests/test_gpu_nd.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for c in 0 200 128 256 0 200 128 256; do
  VLGBA_TRAIL_WGS=$c timeout -k 10 200 python -u tools/prof_cfg5x_solve.py 900 >> $O/solve_t$c.txt 2>&1 || exit 2
done
for c in 0 200; do
  VLGBA_TRAIL_WGS=$c VLGBA_LIB=tools/build/ab/stamps/libvlgba.so timeout -k 10 200 python -u tools/step_stamps.py cfg5x:900 > $O/stamps_t$c.txt 2>&1 || exit 3
done
for x in 1 0 1 0; do
  VLGBA_REDUCE_XCD=$x timeout -k 10 200 python -u tools/prof_cfg5x_solve.py 900 >> $O/solve_x$x.txt 2>&1 || exit 4
done
for x in 0 1 0 1; do
  VLGBA_LONG_ACC=$x timeout -k 10 200 python -u tools/prof_cfg5x_solve.py 900 >> $O/solve_la$x.txt 2>&1 || exit 4
done
sets=("SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"
      "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum")
for x in 0 1; do
  for i in 0 1; do
    VLGBA_LONG_ACC=$x timeout -s KILL 150 rocprofv3 --pmc ${sets[$i]} --kernel-include-regex 'k_schur_reduce|k_schur_long_acc' -d $O/pmc_x${x}_$i -o pmc --output-format csv -- python3 tools/prof_cfg5x_solve.py 900 > $O/pmc_x${x}_$i.log 2>&1 || exit 5
  done
done
