#!/bin/bash
# Column-split two-vector multi-dot (tools/experiments/d2_colsplit.patch): correctness against the
# product build, then an interleaved A/B at N=1e8 and at the 8-GPU shard.
# usage (on the box): bash tools/gpu_ab_colsplit.sh TAG "variant,variant,..."
set -o pipefail
TAG=${1:-colsplit}
VARS=${2:-base,d2cs2,d2cs2_b512,d2cs4_b512,d2cs4_b1024,d2cs2_j32,d2cs2_b512_j32}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for v in ${VARS//,/ }; do
  [ "$v" == base ] && continue
  timeout -k 10 240 python -u tools/check_variant_dot2.py base $v > $O/check_$v.log 2>&1 || { echo "check $v failed"; tail -20 $O/check_$v.log; exit 1; }
  tail -1 $O/check_$v.log
done
timeout -k 10 400 python -u tools/tune_kernels.py run --variants $VARS --js 16,32,48,64,80,96,112,128 --ops dot2 --rounds 5 --out $O/tune_E44176.json > $O/tune_E44176.log 2>&1 || { echo "tune failed"; tail -20 $O/tune_E44176.log; exit 1; }
cat $O/tune_E44176.log
timeout -k 10 300 python -u tools/tune_kernels.py run --E 5522 --variants $VARS --js 32,64,96,128 --ops dot2 --rounds 5 --out $O/tune_E5522.json > $O/tune_E5522.log 2>&1 || { echo "tune shard failed"; tail -20 $O/tune_E5522.log; exit 1; }
cat $O/tune_E5522.log
echo done
