#!/bin/bash
# Build libvlgba.so variants for an A/B timing on the GPU box (tools/ab_run.sh):
#   tools/ab_build.sh base[SUFFIX] [REV]    -> tools/build/ab/base[SUFFIX]  (git REV, default HEAD)
#   tools/ab_build.sh NAME [-DFLAG=V ...]   -> tools/build/ab/NAME  (working tree + flags)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
src=/tmp/ab_src_$name
rm -rf $src && mkdir -p $src/bundleadjustmentmatlab_amd tools/build/ab/$name
if [[ "$name" == base* ]]; then
  git archive "${1:-HEAD}" bundleadjustmentmatlab_amd/csrc include | tar -x -C $src
  flags=""
else
  cp -r bundleadjustmentmatlab_amd/csrc $src/bundleadjustmentmatlab_amd/ && cp -r include $src/
  rm -rf $src/bundleadjustmentmatlab_amd/csrc/build
  flags="$*"
fi
make -s -C $src/bundleadjustmentmatlab_amd/csrc -j8 OUT=$PWD/tools/build/ab/$name \
  HIPCC="/opt/rocm/bin/hipcc $flags"
