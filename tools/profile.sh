#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root):
#   1. --kernel-trace --stats  (per-kernel durations; must agree with bench.py's HIP events)
#   2. --pmc FETCH_SIZE        (separate pass, MI355X_MICROARCH.md rocprofv3 PMC slots)
#   3. --pmc WRITE_SIZE
# Usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="--cpu-baseline-seconds 0 --side-steps 0 $*"
sha256sum audio_style_transfer_amd/libastyle.so > "$OUT/lib.sha256"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/bench_write.log" 2>&1
echo "profile $TAG done"
