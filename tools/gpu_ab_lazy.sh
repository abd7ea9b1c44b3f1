# A/B on one box: eager vs lazy DCGS2 basis (bench, interleaved) and the update kernels per j (tuner)
set -o pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-restart --lazy-basis > $O/lazy_$r.json 2> $O/lazy_$r.err || { echo lazy failed; tail $O/lazy_$r.err; exit 1; }
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-restart > $O/eager_$r.json 2> $O/eager_$r.err || { echo eager failed; tail $O/eager_$r.err; exit 1; }
done
timeout -k 10 400 python tools/tune_kernels.py run --variants base,dl_u4,dl_u1,dl_g1024,dl_g512 --ops dcgs2_upd0,dcgs2_lazy --js 8,32,64,128 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1 || { echo tune failed; tail $O/tune.log; exit 1; }
echo ok
