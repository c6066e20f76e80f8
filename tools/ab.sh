#!/bin/bash
# A/B of library variants over quick benches: tools/ab.sh base <variant> ...
# (base = libastyle.so, else libastyle_<variant>.so built by ASTYLE_VARIANT=... _build.py)
set -o pipefail
mkdir -p gpurun_out
for V in "$@"; do
  if [ $V = base ]; then L=audio_style_transfer_amd/libastyle.so; else L=audio_style_transfer_amd/libastyle_$V.so; fi
  ASTYLE_LIB=$L timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/ab_$V.log 2>&1 || { echo "$V failed"; tail gpurun_out/ab_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_$V.log').read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels_ms_per_step']; print('$V', round(d['value'],3), 'fwd', round(r['fwd']['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'gram', round(k['gram_fwd'],2), round(k['gram_bwd'],2), 'grad', d['grad_rel_l2'])"
done
