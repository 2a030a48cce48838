#!/bin/bash
# kernel trace of a few cfg3 passes (GPU box): gpurun_out/trace_pass/ (analyse
# with tools/timeline.py)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/trace_pass
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace -d $out -o tr --output-format csv -- python3 bench.py ${*:---steps 6 --warmup 2 --no-cpu-baseline} > $out/log 2>&1
