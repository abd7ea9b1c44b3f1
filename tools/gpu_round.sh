#!/bin/bash
# One GPU-box profiling pass: the driver's exact bench command under a kernel-trace profile (wall
# time recorded), then the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs,
# MI355X_MICROARCH.md §HBM) and the traffic file.
# usage (on the box): NKV_HEAD=<git head> bash tools/gpu_round.sh TAG [--pytest]
#   NKV_BENCH_ARGS (default "--gpus 1 --steps 20 --warmup 5", the driver's command)
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
BARGS=${NKV_BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
mkdir -p $O $O/pmcF $O/pmcW
cd $R
if [ "$2" == "--pytest" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu ${NKV_PYTEST_ARGS:--x} -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
cd /tmp && export TMPDIR=/tmp
T0=$(date +%s.%N)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py $BARGS > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
T1=$(date +%s.%N)
python3 -c "import json,sys; print(json.dumps({'command': 'rocprofv3 --kernel-trace --stats -- python3 bench.py $BARGS', 'wall_s': round($T1-$T0, 1), 'head': '${NKV_HEAD:-unknown}', 'box': '$(hostname)'}))" > $O/bench_wall.json
cat $O/bench.json $O/bench_wall.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcF -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-ks > $O/pmcF/bench.json 2> $O/pmcF/err.txt || { echo "pmcF failed"; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcW -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-ks > $O/pmcW/bench.json 2> $O/pmcW/err.txt || { echo "pmcW failed"; exit 1; }
cd $R
F=$(find $O/pmcF -name '*counter_collection.csv' | head -1); W=$(find $O/pmcW -name '*counter_collection.csv' | head -1)
python3 tools/pmc_traffic.py $(dirname $F) $(dirname $W) $O/pmcF/bench.json $O/pmc_traffic.json --tag $TAG --head "${NKV_HEAD:-unknown}" --box "$(hostname)" > /dev/null && echo traffic ok
S=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 tools/check_profile.py $S $O/bench.json > $O/profile_vs_events.txt && cat $O/profile_vs_events.txt
echo done
