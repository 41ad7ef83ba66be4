#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, each its own run).
# usage: [PASSES="grp1;grp2"] tools/pmc.sh TAG [bench args...]
TAG=${1:-pmc}; shift
mkdir -p gpurun_out
DEFAULT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INSTS;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TA_BUSY_avr TA_BUSY_max"
IFS=';' read -ra GROUPS_ <<< "${PASSES:-$DEFAULT}"
i=0
for P in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_pmc$i -o run -- python3 bench.py --child "$@" > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "pass $i failed" >> gpurun_out/${TAG}_pmc$i.log; exit 1; }
done
