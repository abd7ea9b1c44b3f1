# r06r: the driver's multi-rank bench line rehearsed on ONE GPU with gloo ranks sharing it (VERDICT r5
# item 1 "done when"): 8 and 2 ranks at BASELINE size, complete lines (CPU lines on rank 0, shard
# traffic from profiles/traffic_E<E>.json).  Timings are NOT a scaling measurement (ranks share one GPU).
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
NKV_BACKEND=gloo timeout -k 10 700 python3 -u bench.py --gpus 8 --steps 2 --warmup 1 > $O/bench_8rank_gloo.json 2> $O/bench_8rank_gloo.err && \
NKV_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err
RC=$?
kill $HB
exit $RC
