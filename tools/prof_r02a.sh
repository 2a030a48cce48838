set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh gpurun_out/r02a_cfg3 --steps 10 --warmup 2 --no-cpu-baseline || exit $?
out=gpurun_out/r02a_lady
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python3 bench.py --config ladybug --steps 5 --warmup 2 --no-cpu-baseline > $out/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE -d $out/pmc_mfma -o pmc_mfma --output-format csv -- python3 bench.py --config ladybug --steps 5 --warmup 2 --no-cpu-baseline > $out/pmc_mfma.log 2>&1
echo rc_mfma=$?
