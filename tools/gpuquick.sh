#!/bin/bash
# Split-path parity tests + stamps + A/B quick benches (iteration loop on the GPU box).
# usage: tools/gpuquick.sh [variants for ab.sh...]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpuq_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpuq_tests.log; exit 1; }
tail -1 gpurun_out/gpuq_tests.log
bash tools/gpucheck.sh stamps && bash tools/ab.sh base "$@"
