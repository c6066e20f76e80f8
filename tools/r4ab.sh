#!/bin/bash
# Quick-bench A/B variants on the GPU box: tools/r4ab.sh "tag:bench args[:ENV=v ...]" ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  tag=${v%%:*}; rest=${v#*:}; args=${rest%%:*}; envs=""; [ "$rest" != "$args" ] && envs=${rest#*:}
  env $envs timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 --steps 10 $args > gpurun_out/r4_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels_ms_per_step']; print('$tag', round(d['value'],3), round(d['ms_per_step'],2), 'fwd', round(r['fwd']['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'gram', round(k['gram_fwd'],2), round(k['gram_bwd'],2), 'other', round(k['other'],2), 'grad', d['grad_rel_l2'], 'flagged', d.get('range_flagged_clips'), 'loss', d['loss_first_last'])"
done
