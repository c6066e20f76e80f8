#!/bin/bash
# Round-4 GPU check: the GPU suite, then the first A/B set (default, clip groups 2 / 4, Gram
# stage counts), each step under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
bash tools/r4ab.sh "g1:--groups 1" "g2:--groups 2" "g4:--groups 4" "nt2:--groups 1:ASTYLE_GRAM_NT=2" "nt3:--groups 1:ASTYLE_GRAM_NT=3" "nf4:--groups 1:ASTYLE_GRAM_NT=4"
