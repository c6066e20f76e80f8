#!/bin/bash
# SQ counter pass over the encoder forward (tools/fwdonly.py); usage: tools/sqpmc.sh tag [env...]
set -euo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/sq_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM -T --output-format csv -d "$OUT" -o run -- python3 tools/fwdonly.py 64 2 > "$OUT/log" 2>&1
echo "sq $TAG done"
