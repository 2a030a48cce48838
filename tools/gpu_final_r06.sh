#!/bin/bash
# Round-6 final measurements (GPU box, repo root), each step under its own time
# limit, stopping at the first failure:
#   pmc     FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes of the cfg3 bench (one
#           counter per run, no trace domains) -> gpurun_out/pmc_traffic_cfg3.json
#   kstats  rocprofv3 --kernel-trace --stats of the cfg3 bench -> gpurun_out/kstats/
#   bench   the driver's default line (--gpus 1 --steps 20 --warmup 5) and the 100 / 50 one
#   cfg5x   the 1000-camera growing replay with its CPU baseline
#   smoke   __graft_entry__.smoke()
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
args="--steps 5 --warmup 2 --no-cpu-baseline --no-other-configs"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    pmc)
      for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
        timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o pmc --output-format csv \
          -- python3 bench.py $args > gpurun_out/pmc_$c.log 2>&1 || { tail -5 gpurun_out/pmc_$c.log; exit 1; }
      done
      python3 tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE \
        --valu gpurun_out/pmc_SQ_INSTS_VALU --config cfg3 > gpurun_out/pmc_traffic_cfg3.json || exit 1
      cat gpurun_out/pmc_traffic_cfg3.json | head -40 ;;
    kstats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats -o ks \
        --output-format csv -- python3 bench.py --steps 50 --warmup 20 --no-cpu-baseline \
        --no-other-configs > gpurun_out/kstats.log 2>&1 || exit 1
      find gpurun_out/kstats -name "*kernel_stats.csv" | head -1 | xargs head -12 ;;
    bench)
      timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
        > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.log || exit 1
      timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default.json \
        2> gpurun_out/bench_default.log || exit 1
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_driver.json gpurun_out/bench_default.json ;;
    cfg5x)
      timeout -k 10 600 python3 -u bench.py --config cfg5x > gpurun_out/bench_cfg5x.json \
        2> gpurun_out/bench_cfg5x.log || exit 1
      grep -o '"value": [0-9.]*' gpurun_out/bench_cfg5x.json | head -3 ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
        > gpurun_out/smoke.log 2>&1 || exit 1
      tail -1 gpurun_out/smoke.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
