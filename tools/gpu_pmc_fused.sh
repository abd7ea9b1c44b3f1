#!/bin/bash
# Stall / LDS / VALU / TCP counters of the CGS2 fused middle pass (k_update_dot) beside the DCGS2
# dual update (k_dcgs2_update), per Arnoldi step j, over one N=1e8 factorisation of each mode.
# Each --pmc pass is its own run (limits: 8 SQ, 4 TCP, 2 GRBM per pass).
# usage (on the box): bash tools/gpu_pmc_fused.sh TAG
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
P3="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_LFIFO_STALL_CYCLES_sum TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
PASSES=${NKV_PMC_PASSES:-1 2 3}
for mode in cgs2 dcgs2; do
  for p in $PASSES; do
    eval C=\$P$p
    D=$O/${mode}_p$p
    mkdir -p $D
    timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $D -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-ks --no-restart --mode $mode > $D/bench.json 2> $D/err.txt || { echo "$mode p$p failed"; tail -5 $D/err.txt; exit 1; }
  done
done
D=""
for mode in cgs2 dcgs2; do for p in $PASSES; do D="$D $O/${mode}_p$p"; done; done
cd $R && python3 tools/pmc_by_j.py $O/fused_by_j.json $D > /dev/null && echo ok
