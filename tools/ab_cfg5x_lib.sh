#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_batch.sh ab || exit 1
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export VLGBA_LIB=tools/build/ab/base/libvlgba.so; else unset VLGBA_LIB; fi
    timeout -k 10 300 python3 -u bench.py --config cfg5x --no-cpu-baseline > gpurun_out/c5x_$v.json 2> gpurun_out/c5x_$v.log || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/c5x_$v.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print('$v', $r, round(d['value'],1), round(d['roofline']['device_busy_s'],3), {n:(round(v['ms']),v['launches']) for n,v in k.items() if n in ('k_factor_step','k_schur_reduce','k_assemble','k_schur_group','k_backward')})"
  done
done
