#!/bin/bash
# GPU suite, then the small-batch and headline quick benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
bash tools/r4ab.sh "c1:--clips 1 --steps 50" "c8:--clips 8 --steps 30" "g1:--groups 1"
