#!/bin/bash
# Copy one gpu_round.sh pass (gpurun_out/TAG) into profiles/ under the round's naming.
# usage: bash tools/collect_profiles.sh TAG [--latest]   (--latest also refreshes traffic_latest.json)
set -e
TAG=$1
O=gpurun_out/$TAG
P=profiles
[ -f $O/bench.json ] && cp $O/bench.json $P/${TAG}_bench_n1.json
[ -f $O/bench_wall.json ] && cp $O/bench_wall.json $P/${TAG}_bench_wall.json
S=$(find $O/prof -name '*kernel_stats.csv' 2>/dev/null | head -1 || true)
[ -n "$S" ] && cp $S $P/${TAG}_bench_n1_kernel_stats.csv
[ -f $O/profile_vs_events.txt ] && cp $O/profile_vs_events.txt $P/${TAG}_profile_vs_events.txt
[ -f $O/pmc_traffic.json ] && cp $O/pmc_traffic.json $P/${TAG}_pmc_traffic.json
[ -f $O/pytest_gpu.log ] && cp $O/pytest_gpu.log $P/${TAG}_pytest_gpu.log
if [ "$2" == "--latest" ] && [ -f $O/pmc_traffic.json ]; then cp $O/pmc_traffic.json $P/traffic_latest.json; fi
ls $P | grep "^${TAG}_"
