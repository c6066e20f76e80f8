#!/bin/bash
# GPU test suite + default bench (+ optional stamps of the split block kernels) on the GPU box.
# usage: tools/gpucheck.sh [tests] [bench] [quick] [gatys] [stamps]   (run from the repo root)
set -o pipefail
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest.log; exit 1; }
           tail -2 gpurun_out/gputest.log ;;
    bench) timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
           tail -1 gpurun_out/bench.log | cut -c1-400 ;;
    quick) timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/quick.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/quick.log; exit 1; }
           tail -1 gpurun_out/quick.log | cut -c1-600 ;;
    gatys) timeout -k 10 400 python bench.py --gatys --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/bench_gatys.log 2>&1 || { echo "gatys bench failed"; tail -30 gpurun_out/bench_gatys.log; exit 1; }
           tail -1 gpurun_out/bench_gatys.log | cut -c1-300 ;;
    stamps) timeout -k 10 200 python tools/stamps.py 64 fwd > gpurun_out/stamps_fwd.log 2>&1 && \
            timeout -k 10 200 python tools/stamps.py 64 bwd > gpurun_out/stamps_bwd.log 2>&1 || { echo "stamps failed"; exit 1; }
            cat gpurun_out/stamps_fwd.log gpurun_out/stamps_bwd.log ;;
  esac
done
