#!/bin/bash
# A/B of the device-decided LM loop against the host-decided one (GPU box):
# alternating whole-solve bench lines, cfg3 and cfg2, then cfg3 passes via
# vlgba_run_passes (--batch) against vlgba_step per pass
set -o pipefail
mkdir -p gpurun_out
val() { grep '^{' "$1" | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['value'],1), round(d['ms_per_step'],4))"; }
for i in 1 2 3; do
  for m in 1 0; do
    VLGBA_DEVICE_LM=$m timeout -k 10 200 python3 bench.py --mode solve --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/ab_s$m.log 2>&1 || exit 1
    echo "cfg3 solve dev=$m $(val gpurun_out/ab_s$m.log)"
    VLGBA_DEVICE_LM=$m timeout -k 10 200 python3 bench.py --config cfg2 --mode solve --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/ab_c$m.log 2>&1 || exit 1
    echo "cfg2 solve dev=$m $(val gpurun_out/ab_c$m.log)"
  done
done
