set -o pipefail
O=gpurun_out/t4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 240 --timeout-method thread > $O/multirank.log 2>&1 || { echo multirank failed; tail -30 $O/multirank.log; exit 1; }
tail -3 $O/multirank.log
timeout -k 10 200 python bench.py --E 8000 --steps 2 --warmup 1 --no-cpu --no-restart > $O/b1.json 2> $O/b1.err || { echo b1 failed; tail $O/b1.err; exit 1; }
NKV_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --E 8000 --steps 2 --warmup 1 > $O/b2.json 2> $O/b2.err || { echo b2 failed; tail $O/b2.err; exit 1; }
NKV_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 8 --E 8000 --steps 2 --warmup 1 > $O/b8.json 2> $O/b8.err || { echo b8 failed; tail $O/b8.err; exit 1; }
echo ok
