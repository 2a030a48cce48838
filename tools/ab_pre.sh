#!/bin/bash
# A/B on the GPU box against tools/build/ab/pre (tools/ab_build.sh pre): bit
# identity of da / db / the pass scalars on several scenes (da_dump /
# da_compare), untimed pass times of both builds, then the solver tests.
set -o pipefail
export TMPDIR=/tmp
for sc in ${AB_SCENES:-ladybug long "cfg5x 600" "cfg5x 900"}; do
  tag=${sc// /_}
  VLGBA_LIB=tools/build/ab/pre/libvlgba.so timeout -k 10 300 python -u tools/da_dump.py gpurun_out/abp_base_$tag.npz $sc > gpurun_out/abp_$tag.log 2>&1 &&
  timeout -k 10 300 python -u tools/da_dump.py gpurun_out/abp_new_$tag.npz $sc >> gpurun_out/abp_$tag.log 2>&1 &&
  python tools/da_compare.py gpurun_out/abp_base_$tag.npz gpurun_out/abp_new_$tag.npz > gpurun_out/abp_cmp_$tag.txt || { cat gpurun_out/abp_cmp_$tag.txt; exit 1; }
  echo "$tag: $(grep -c identical gpurun_out/abp_cmp_$tag.txt) identical"
done
echo pre; VLGBA_LIB=tools/build/ab/pre/libvlgba.so timeout -k 10 200 python -u tools/pass_time.py 600 900 ladybug || exit 1
echo new; timeout -k 10 200 python -u tools/pass_time.py 600 900 ladybug || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_nd.py tests/test_gpu_parity.py tests/test_gpu_solve_status.py tests/test_gpu_lm_parity.py > gpurun_out/abp_tests.log 2>&1; tail -3 gpurun_out/abp_tests.log
