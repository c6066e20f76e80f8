#!/bin/bash
# Few-clip A/B on the GPU box: quick benches at --clips B under different settings / libraries.
# usage: tools/fewab.sh B "tag|ENV=v ENV2=w" ...
set -o pipefail
mkdir -p gpurun_out
B=$1; shift
for v in "$@"; do
  IFS='|' read -r tag envs <<< "$v"
  (env $envs timeout -k 10 200 python bench.py --clips $B --steps 30 --warmup 3 --side-steps 0 --cpu-baseline-seconds 0) > gpurun_out/fb_${B}_$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/fb_${B}_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/fb_${B}_$tag.log').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('B=$B $tag', round(d['value']*256,1), 'clip-iters/s', round(d['ms_per_step'],4), 'ms', {a: round(b,4) for a,b in k.items()}, 'loss', d['loss_first_last'])"
done
