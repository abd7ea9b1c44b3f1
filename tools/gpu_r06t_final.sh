# r06t: smoke() and the driver's exact bench command (no profiler) at the round-6 head
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err && \
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
