#!/bin/bash
# Per-rank shards of the 2/4/8-GPU N=1e8 runs, each on this one GPU (what one rank computes), with
# every partial routed through a world-1 RCCL group (--force-collectives: the collective code path
# minus the peers).  usage (on the box): bash tools/gpu_shards.sh TAG
set -o pipefail
TAG=${1:-shards}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
for E in 22088 11044 5522; do
  timeout -k 10 200 python3 bench.py --E $E --steps 5 --warmup 2 --no-cpu --no-restart --no-ks --force-collectives > $O/shard_E$E.json 2> $O/shard_E$E.err || { echo "E=$E failed"; tail $O/shard_E$E.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/shard_E$E.json')); print($E, d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['achieved'], d['gram_schmidt']['allreduce_ms_per_factorisation'])"
done
