#!/bin/bash
# A/B of one environment setting over quick benches: tools/ab_env.sh VAR v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
VAR=$1; shift
for V in "$@"; do
  env $VAR=$V timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/ab_${VAR}_$V.log 2>&1 || { echo "$VAR=$V failed"; tail gpurun_out/ab_${VAR}_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_${VAR}_$V.log').read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels_ms_per_step']; print('$VAR=$V', round(d['value'],3), 'fwd', round(r['fwd']['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'gram', round(k['gram_fwd'],2), round(k['gram_bwd'],2), 'grad', d['grad_rel_l2'])"
done
