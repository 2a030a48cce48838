#!/bin/bash
# Round 4d checks on the GPU box (from the repo root): the envelope factor on
# wave_factor16x chains (BA_ENV_FACTOR_X=1, tools/build/ab/envx*) against the
# default build -- ubench, the solver tests, per-column stamps, cfg5x
# sub-problem passes, the ladybug bench -- then context-setup phases and the
# cfg5x replay with two prefetch workers.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
X=tools/build/ab/envx/libvlgba.so
XS=tools/build/ab/envxst/libvlgba.so
echo "== ubench $(date +%T)"
{ timeout -k 5 60 tools/build/ubench_chol && timeout -k 5 60 tools/build/ubench_chol_x; } \
  > gpurun_out/ubench_chol.txt 2>&1 || exit 1
echo "== tests (envx) $(date +%T)"
VLGBA_LIB=$X timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_nd.py tests/test_gpu_solve_status.py \
  > gpurun_out/envtests.log 2>&1 || { tail -30 gpurun_out/envtests.log; exit 1; }
tail -2 gpurun_out/envtests.log
echo "== stamps $(date +%T)"
for lib in bundleadjustmentmatlab_amd/libvlgba_stamps.so $XS; do
  tag=$([ $lib = $XS ] && echo x || echo base)
  VLGBA_LIB=$lib timeout -k 10 200 python -u tools/step_stamps.py cfg5x:900 auto \
    > gpurun_out/stamps_cfg5x900_$tag.txt 2>&1 &&
  VLGBA_LIB=$lib timeout -k 10 200 python -u tools/step_stamps.py ladybug auto \
    > gpurun_out/stamps_ladybug_$tag.txt 2>&1 || exit 1
done
echo "== solve $(date +%T)"
timeout -k 10 300 python -u tools/prof_cfg5x_solve.py 600 900 > gpurun_out/prof_cfg5x_solve.log 2>&1 &&
VLGBA_LIB=$X timeout -k 10 300 python -u tools/prof_cfg5x_solve.py 600 900 \
  > gpurun_out/prof_cfg5x_solve_x.log 2>&1 || exit 1
echo "== ladybug $(date +%T)"
timeout -k 10 300 python -u bench.py --config ladybug > gpurun_out/bench_ladybug.json \
  2> gpurun_out/bench_ladybug.log &&
VLGBA_LIB=$X timeout -k 10 300 python -u bench.py --config ladybug > gpurun_out/bench_ladybug_x.json \
  2> gpurun_out/bench_ladybug_x.log || exit 1
echo "== cr granules $(date +%T)"
G=tools/build/ab/gran/libvlgba.so
VLGBA_LIB=$G timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "cr or cyclic" tests/test_gpu_solve_status.py \
  > gpurun_out/grantests.log 2>&1 || { tail -30 gpurun_out/grantests.log; exit 1; }
tail -2 gpurun_out/grantests.log
VLGBA_LIB=tools/build/ab/granst/libvlgba.so timeout -k 10 200 python -u tools/cr_timeline.py cfg3 \
  > gpurun_out/cr_timeline_gran.txt 2>&1 &&
timeout -k 10 200 python -u tools/cr_timeline.py cfg3 > gpurun_out/cr_timeline_base.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.log &&
VLGBA_LIB=$G timeout -k 10 300 python -u bench.py > gpurun_out/bench_cfg3_gran.json \
  2> gpurun_out/bench_cfg3_gran.log || exit 1
echo "== setup $(date +%T)"
timeout -k 10 300 python -u tools/prof_cfg5x_setup.py 300 600 900 1000 > gpurun_out/setup_trace.log 2>&1 || exit 1
echo "== cfg5x $(date +%T)"
timeout -k 10 600 python -u bench.py --config cfg5x > gpurun_out/bench_cfg5x.json \
  2> gpurun_out/bench_cfg5x.log || exit 1
echo "== done $(date +%T)"
