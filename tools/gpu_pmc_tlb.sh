#!/bin/bash
# Address-translation (UTCL1/UTCL2) counters of the DCGS2 kernels per Arnoldi step j: two --pmc
# passes over one factorisation at N=1e8, each its own run (counter limits: 4 TCP, 2 GRBM per pass).
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O/t1 $O/t2
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-ks --no-restart"
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY --output-format csv -d $O/t1 -o run -- python3 $B > $O/t1/bench.json 2> $O/t1/err.txt || { echo "t1 failed"; tail $O/t1/err.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/t2 -o run -- python3 $B > $O/t2/bench.json 2> $O/t2/err.txt || { echo "t2 failed"; tail $O/t2/err.txt; exit 1; }
cd $R && python3 tools/pmc_by_j.py $O/tlb_by_j.json $O/t1 $O/t2 > /dev/null && echo ok
