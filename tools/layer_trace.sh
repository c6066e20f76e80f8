#!/bin/bash
# Per-layer block-kernel durations (rocprofv3 kernel trace of tools/fwd_layers.py).
set -o pipefail
mkdir -p gpurun_out/layers
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/layers -o run -- python3 tools/fwd_layers.py 256 bwd > gpurun_out/layers/log 2>&1 || { echo "trace failed"; tail gpurun_out/layers/log; exit 1; }
python3 tools/trace_blocks.py $(find gpurun_out/layers -name '*kernel_trace.csv' | head -1)
