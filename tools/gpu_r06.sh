#!/bin/bash
# Round-6 GPU-box steps (run from the repo root on the box), each under its own
# time limit, stopping at the first failure:
#   counters  rocprofv3 -L -> gpurun_out/counters.txt
#   pmc       PMC passes of the cfg3 bench (one counter set per run, no trace
#             domains) -> gpurun_out/pmc/<set>/ ; PMC_SETS overrides the sets
#   kstats    rocprofv3 --kernel-trace --stats of the cfg3 bench -> gpurun_out/kstats/
#   stream    tools/build/ubench_stream (HBM read / write / copy rates)
#   bias      tools/converged_bias.py --sets cfg2,cfg3 --big-seeds 12
# usage: tools/gpu_r06.sh step [step ...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
args="--steps 5 --warmup 2 --no-cpu-baseline --no-other-configs"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    counters)
      timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || exit 1 ;;
    pmc)
      if [ -n "$PMC_SETS" ]; then
        IFS=';' read -r -a sets <<< "$PMC_SETS"
      else
        sets=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
              "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
              "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum")
      fi
      for i in "${!sets[@]}"; do
        out=gpurun_out/pmc/set$i
        mkdir -p $out
        timeout -s KILL 120 rocprofv3 --pmc ${sets[$i]} -d $out -o pmc --output-format csv \
          -- python3 bench.py $args > $out.log 2>&1
        rc=$?; echo "== set $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out.log; exit $rc; }
      done ;;
    kstats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats -o ks \
        --output-format csv -- python3 bench.py --steps 50 --warmup 20 --no-cpu-baseline \
        --no-other-configs > gpurun_out/kstats.log 2>&1 || exit 1 ;;
    fused)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 \
        --timeout-method thread > gpurun_out/test_fused.log 2>&1; rc=$?
      tail -15 gpurun_out/test_fused.log; [ $rc -eq 0 ] || exit $rc ;;
    ablin)
      # bit identity of the A/B builds (tools/ab_build.sh) against AB_REF (default v0) on
      # tools/lin_dump.py's scenes, then the cfg3 bench of each, alternated twice
      ref=${AB_REF:-v0}
      for v in $(ls tools/build/ab); do
        VLGBA_LIB=tools/build/ab/$v/libvlgba.so timeout -k 10 300 python -u tools/lin_dump.py \
          gpurun_out/lin_$v.npz > gpurun_out/lin_$v.log 2>&1 || { tail -5 gpurun_out/lin_$v.log; exit 1; }
      done
      for v in $(ls tools/build/ab); do
        echo "$v vs $ref: $(python tools/lin_dump.py --compare gpurun_out/lin_$v.npz gpurun_out/lin_$ref.npz | tail -1)"
      done
      rm -f gpurun_out/lin_*.npz   # (the merge back is capped at 64 MiB)
      for r in 1 2; do
        for v in $(ls tools/build/ab); do
          VLGBA_LIB=tools/build/ab/$v/libvlgba.so timeout -k 10 300 python -u bench.py --steps 100 \
            --warmup 50 --no-cpu-baseline --no-other-configs > gpurun_out/ab_${v}_$r.json \
            2> gpurun_out/ab_${v}_$r.log || { tail -5 gpurun_out/ab_${v}_$r.log; exit 1; }
          echo "$v run $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_$r.json) $(grep -o 'k_update_linearize=[0-9.]*us' gpurun_out/ab_${v}_$r.log | head -1) $(grep -o 'k_schur_mfma=[0-9.]*us' gpurun_out/ab_${v}_$r.log | head -1) $(grep -o 'k_cr32_fused=[0-9.]*us' gpurun_out/ab_${v}_$r.log | head -1) $(grep -o 'k_schur_reduce=[0-9.]*us' gpurun_out/ab_${v}_$r.log | head -1)"
        done
      done ;;
    stream)
      timeout -k 10 120 tools/build/ubench_stream > gpurun_out/ubench_stream.txt 2>&1 || exit 1
      cat gpurun_out/ubench_stream.txt ;;
    bias)
      timeout -k 10 900 python -u tools/converged_bias.py --sets cfg2,cfg3 --big-seeds 12 \
        --out gpurun_out/bias_big.json > gpurun_out/bias_big.log 2>&1 || exit 1
      tail -4 gpurun_out/bias_big.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
