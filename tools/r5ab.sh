#!/bin/bash
# Round-5 A/B on the GPU box: quick benches of this tree under different settings / libraries
# (ASTYLE_LIB=...), and of a round-4 build checked out at tools/_r4 (git worktree of round 4's
# last commit; not kept in the tree).  usage: tools/r5ab.sh "tag|ENV=v ENV2=w|bench args" ...
# (a tag starting with r4 runs the round-4 tree)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  IFS='|' read -r tag envs args <<< "$v"
  if [ "${tag:0:2}" = r4 ]; then dir=tools/_r4; else dir=.; fi
  (cd $dir && env $envs timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 --steps 10 $args) > gpurun_out/r5_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r5_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r5_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels_ms_per_step']; print('$tag', round(d['value'],3), round(d['ms_per_step'],2), 'fwd', round(r['fwd']['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'gram', round(k['gram_fwd'],2), round(k['gram_bwd'],2), 'other', round(k['other'],2), 'grad', d['grad_rel_l2'], 'loss', d['loss_first_last'])"
done
