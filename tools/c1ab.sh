#!/bin/bash
# One-clip (configs[1]) A/B on the GPU box: quick benches at --clips 1 under different settings /
# libraries.  usage: tools/c1ab.sh "tag|ENV=v ENV2=w" ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  IFS='|' read -r tag envs <<< "$v"
  (env $envs timeout -k 10 200 python bench.py --clips 1 --steps 200 --warmup 5 --side-steps 0 --cpu-baseline-seconds 0) > gpurun_out/c1_$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/c1_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/c1_$tag.log').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$tag', round(d['value']*256,1), 'clip-iters/s', round(d['ms_per_step'],4), 'ms', {a: round(b,4) for a,b in k.items()}, 'loss', d['loss_first_last'])"
done
