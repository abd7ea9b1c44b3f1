#!/bin/bash
# One GPU-box pass: parity tests, a kernel-trace profile of bench.py, then the two PMC passes.
# usage (on the box): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O $O/pmcF $O/pmcW
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcF -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $O/pmcF/bench.json 2> $O/pmcF/err.txt || { echo "pmcF failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcW -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $O/pmcW/bench.json 2> $O/pmcW/err.txt || { echo "pmcW failed"; exit 1; }
echo done
