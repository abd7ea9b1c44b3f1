#!/bin/bash
# PMC HBM traffic of one rank's shard: bench.py at world 1 on the element count
# rank 0 holds at world 2 / 4 / 8 (E = 22088 / 11044 / 5522 of BASELINE's 44176), FETCH_SIZE and
# WRITE_SIZE in separate passes, then tools/pmc_traffic.py -> gpurun_out/TAG/traffic_E<E>.json
# (copy to profiles/: bench.py's find_traffic attaches it to the world > 1 line of that shard size).
# usage (on the box): NKV_HEAD=<git head> bash tools/gpu_shard_traffic.sh TAG [E ...]
set -o pipefail
TAG=${1:-run}
shift
ES=${@:-22088 11044 5522}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
for E in $ES; do
  mkdir -p $O/E$E/pmcF $O/E$E/pmcW
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/E$E/pmcF -o run -- python3 $R/bench.py --E $E --steps 1 --warmup 0 --no-cpu --no-ks --no-restart > $O/E$E/pmcF/bench.json 2> $O/E$E/pmcF/err.txt || { echo "pmcF E=$E failed"; tail -5 $O/E$E/pmcF/err.txt; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/E$E/pmcW -o run -- python3 $R/bench.py --E $E --steps 1 --warmup 0 --no-cpu --no-ks --no-restart > $O/E$E/pmcW/bench.json 2> $O/E$E/pmcW/err.txt || { echo "pmcW E=$E failed"; tail -5 $O/E$E/pmcW/err.txt; exit 1; }
  cd $R
  F=$(find $O/E$E/pmcF -name '*counter_collection.csv' | head -1); W=$(find $O/E$E/pmcW -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_traffic.py $(dirname $F) $(dirname $W) $O/E$E/pmcF/bench.json $O/traffic_E$E.json --tag $TAG --head "${NKV_HEAD:-unknown}" --box "$(hostname)" > /dev/null && echo "traffic E=$E ok"
done
