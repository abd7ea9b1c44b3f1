#!/bin/bash
# Write-path counters of the DCGS2 kernels (two --pmc passes, each its own run).
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O/p1 $O/p2
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-ks --no-restart"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 $B > $O/p1/bench.json 2> $O/p1/err.txt || { echo "p1 failed"; tail $O/p1/err.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $B > $O/p2/bench.json 2> $O/p2/err.txt || { echo "p2 failed"; tail $O/p2/err.txt; exit 1; }
cd $R && python3 tools/pmc_write_path.py $O/write_path.json $O/p1 $O/p2
