#!/bin/bash
# One --pmc pass (PMC="..." or the instruction-fetch set) over tools/fwd_layers.py 256 bwd (one --pmc pass).
set -o pipefail
mkdir -p gpurun_out/pmc_if
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_SALU} --output-format csv -d gpurun_out/pmc_if -o run -- python3 tools/fwd_layers.py 256 bwd > gpurun_out/pmc_if/log 2>&1 || { echo "pass failed"; tail -5 gpurun_out/pmc_if/log; exit 1; }
python3 tools/pmc_sum.py $(find gpurun_out/pmc_if -name '*counter_collection.csv' | head -1)
