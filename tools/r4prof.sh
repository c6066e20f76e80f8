#!/bin/bash
# Round-4 evidence on the GPU box: full default bench (side keys + CPU baseline), --gatys bench,
# then rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the default workload.
# usage: tools/r4prof.sh <tag> [extra bench args, e.g. --groups 2]
set -o pipefail
TAG=${1:?tag}; shift
mkdir -p gpurun_out
timeout -k 10 400 python bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
timeout -k 10 400 python bench.py --gatys --cpu-baseline-seconds 0 --side-steps 0 "$@" > gpurun_out/${TAG}_gatys.log 2>&1 || { echo "gatys bench failed"; tail -30 gpurun_out/${TAG}_gatys.log; exit 1; }
tail -1 gpurun_out/${TAG}_gatys.log | cut -c1-200
bash tools/profile.sh $TAG "$@" || { echo "profile failed"; exit 1; }
