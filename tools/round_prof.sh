#!/bin/bash
# Round evidence on the GPU box: the full default bench (side keys + CPU baseline), the
# --gatys bench, then rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of both workloads.
# usage: tools/round_prof.sh <tag>   (then on the build box: python tools/summarize_prof.py ...)
set -o pipefail
TAG=${1:?tag}; shift
mkdir -p gpurun_out
timeout -k 10 400 python bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
timeout -k 10 400 python bench.py --gatys --cpu-baseline-seconds 0 --side-steps 0 "$@" > gpurun_out/${TAG}_gatys.log 2>&1 || { echo "gatys bench failed"; tail -30 gpurun_out/${TAG}_gatys.log; exit 1; }
tail -1 gpurun_out/${TAG}_gatys.log | cut -c1-200
bash tools/profile.sh ${TAG}s "$@" || { echo "profile failed"; exit 1; }
bash tools/profile.sh ${TAG}g --gatys "$@" || { echo "gatys profile failed"; exit 1; }
