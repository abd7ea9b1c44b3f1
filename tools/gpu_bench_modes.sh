# One bench.py line per orthogonalisation mode at the headline size (N=1e8, m=128), one process each:
# the Python-driven sequences beside the one-call C drivers, and the reference's MGS2 order on the GPU.
# usage: bash tools/gpu_bench_modes.sh TAG [modes...]
set -o pipefail
tag=${1:-modes}; shift
modes=${*:-"dcgs2 dcgs2-native cgs2 cgs2-native mgs2 mgs2-native"}
mkdir -p gpurun_out
for m in $modes; do
  case $m in mgs2|mgs2-native) st=1; wu=0;; *) st=2; wu=1;; esac
  timeout -k 10 400 python -u bench.py --no-cpu --no-restart --no-ks --steps $st --warmup $wu --mode $m \
    > gpurun_out/${tag}_mode_$m.json 2> gpurun_out/${tag}_mode_$m.err || exit 1
done
