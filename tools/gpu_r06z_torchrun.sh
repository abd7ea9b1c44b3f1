# r06z: the driver's exact multi-rank command line (torch.distributed.run) on one GPU with two gloo
# ranks sharing it, BASELINE size (the driver's SCALE runs use RCCL, one GPU per rank)
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
NKV_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_torchrun_2rank.json 2> $O/bench_torchrun_2rank.err
RC=$?
kill $HB
exit $RC
