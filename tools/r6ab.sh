#!/bin/bash
# Round-6 A/B on the GPU box: quick benches of this tree under different settings / libraries
# (ASTYLE_LIB=... selects an A/B or diagnostic library).
# usage: tools/r6ab.sh "tag|ENV=v ENV2=w|bench args" ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  IFS='|' read -r tag envs args <<< "$v"
  (env $envs timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 --steps 10 $args) > gpurun_out/r6_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r6_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r6_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels_ms_per_step']; print('$tag', round(d['value'],3), round(d['ms_per_step'],2), 'fwd', round(r['fwd']['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'gram', round(k['gram_fwd'],2), round(k['gram_bwd'],2), 'other', round(k['other'],2), 'grad', d['grad_rel_l2'], 'loss', d['loss_first_last'])"
done
