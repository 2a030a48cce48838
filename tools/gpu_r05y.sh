#!/bin/bash
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 60 tools/build/ubench_f16v > $O/ubench_f16v.txt 2>&1 || exit 1
