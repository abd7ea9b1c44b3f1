# r06v: the non-orthonormal-basis modes (the reference's default noise seed) at BASELINE size
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 400 python3 bench.py --mode mgs2-lagged --steps 5 --warmup 2 --no-cpu --no-ks > $O/bench_lagged.json 2> $O/bench_lagged.err && \
timeout -k 10 400 python3 bench.py --mode dcgs2 --steps 5 --warmup 2 --no-cpu --no-ks > $O/bench_dcgs2.json 2> $O/bench_dcgs2.err
