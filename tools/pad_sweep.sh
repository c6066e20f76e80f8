#!/bin/bash
# Gram kernel times vs the activation-tensor spacing (ASTYLE_TPAD, elements): tools/pad_sweep.sh pad1 pad2 ...
set -o pipefail
mkdir -p gpurun_out
for p in "$@"; do
  ASTYLE_TPAD=$p timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/pad_$p.log 2>&1 || { echo "bench pad $p failed"; tail -5 gpurun_out/pad_$p.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('pad %8s value %.3f gram fwd %.2f bwd %.2f blocks %.1f/%.1f' % (sys.argv[2], d['value'], k['gram_fwd'], k['gram_bwd'], k['block_fwd'], k['block_bwd']))" gpurun_out/pad_$p.log $p
done
