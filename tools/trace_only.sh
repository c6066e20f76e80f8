#!/bin/bash
# rocprofv3 kernel trace (no counters) of a quick bench run: tools/trace_only.sh <tag> [env assignments...]
set -euo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT" -o run -- python3 bench.py --cpu-baseline-seconds 0 --side-steps 0 > "$OUT/bench.log" 2>&1
echo "trace $TAG done"
