#!/bin/bash
# Gram time-chunk length sweep (ASTYLE_GRAM_ROWS): tools/rows_sweep.sh rows1 rows2 ...
set -o pipefail
mkdir -p gpurun_out
for p in "$@"; do
  ASTYLE_GRAM_ROWS=$p timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/rows_$p.log 2>&1 || { echo "bench rows $p failed"; tail -5 gpurun_out/rows_$p.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('rows %6s value %.3f gram fwd %.2f bwd %.2f other %.2f grad %.4g' % (sys.argv[2], d['value'], k['gram_fwd'], k['gram_bwd'], k['other'], d['grad_rel_l2']))" gpurun_out/rows_$p.log $p
done
