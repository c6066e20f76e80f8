#!/bin/bash
# PMC passes (each its own run) over tools/fwd_layers.py 256 <mode>: memory-path stall counters.
set -o pipefail
MODE=${1:-fwd}
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
while read -r CNT; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/fwd_layers.py 256 $MODE > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  python3 tools/pmc_sum.py $(find gpurun_out/pmc/p$i -name '*counter_collection.csv' | head -1)
done <<'LIST'
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum
TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES
SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM
LIST
