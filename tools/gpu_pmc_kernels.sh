#!/bin/bash
# Issue / memory-pipe counters of single entry points at BASELINE size (N=1e8, j=128 by default):
# the tuning tool's ops (e.g. rotate_25 = the solver's 25-kept restart rotation, dot2 = the DCGS2
# multi-dot, dcgs2_update = the dual update) under separate --pmc passes, each its own run (limits
# per pass: 8 SQ, 4 TCP, 2 TA, 4 TCC with FETCH_SIZE taking 3 and WRITE_SIZE 2, 2 GRBM).
# usage (on the box): OPS=rotate_25,dot2,dcgs2_update VARIANTS=base bash tools/gpu_pmc_kernels.sh TAG
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export NKV_TUNE_VRAND=${NKV_TUNE_VRAND:-1}
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P3="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL GRBM_GUI_ACTIVE"
P4="FETCH_SIZE GRBM_GUI_ACTIVE"
P5="WRITE_SIZE GRBM_GUI_ACTIVE"
PASSES=${NKV_PMC_PASSES:-1 2 3 4 5}
T="$R/tools/tune_kernels.py run --variants ${VARIANTS:-base} --js ${JS:-128} --ops ${OPS:-rotate_25,dot2,dcgs2_update} --rounds 1"
for p in $PASSES; do
  eval C=\$P$p
  D=$O/p$p
  mkdir -p $D
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $D -o run -- python3 $T --out $D/tune.json > $D/out.txt 2>&1 || { echo "pass $p failed"; tail -5 $D/out.txt; exit 1; }
done
cd $R && python3 tools/pmc_kernel_table.py $O $O/kernel_counters.json
