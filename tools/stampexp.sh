#!/bin/bash
# Stamps of the split block kernels for the base diagnostic build and SW_EXP variants.
# usage: tools/stampexp.sh base 8 9 10    (libastyle_stamps[_expN].so built beforehand)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = base ]; then L=audio_style_transfer_amd/libastyle_stamps.so; else L=audio_style_transfer_amd/libastyle_stamps_exp$v.so; fi
  echo "== $v"
  ASTYLE_LIB=$L timeout -k 10 200 python tools/stamps.py ${STAMP_CLIPS:-64} bwd > gpurun_out/stamps_$v.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/stamps_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps_$v.log
done
