#!/bin/bash
# One rocprofv3 --pmc pass (counters in their own run, kernel-trace only) over a small bench.
# Usage: tools/pmc.sh <tag> "<counters>" [bench args...]
set -euo pipefail
TAG=${1:?tag}; CNT=${2:?counters}; shift 2
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $CNT -T --output-format csv -d "$OUT" -o run -- python3 bench.py --cpu-baseline-seconds 0 --fp32-steps 0 "$@" > "$OUT/bench.log" 2>&1
echo "pmc $TAG done"
