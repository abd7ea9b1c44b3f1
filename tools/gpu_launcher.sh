#!/bin/bash
# bench.py's own N-rank launcher on a one-GPU box (the plain `python3 bench.py --gpus N` command):
# 1 rank, then 2 gloo ranks sharing the GPU at the full N=1e8 (same Ritz values expected), then the
# RCCL backend asked for 2 ranks on 1 GPU (must refuse with exit 2, not hang).
# usage (on the box): bash tools/gpu_launcher.sh TAG
set -o pipefail
TAG=${1:-launch}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-restart --no-ks > $O/b1.json 2> $O/b1.err || { echo b1 failed; tail $O/b1.err; exit 1; }
NKV_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > $O/b2.json 2> $O/b2.err || { echo b2 failed; tail $O/b2.err; exit 1; }
timeout -k 10 120 python3 bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu > $O/b2nccl.json 2> $O/b2nccl.err; rc=$?
echo "rccl 2 ranks on 1 GPU: rc=$rc"; tail -2 $O/b2nccl.err
[ $rc -eq 2 ] || exit 1
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
a, b = (json.load(open(f"{o}/{n}.json")) for n in ("b1", "b2"))
d = max(abs(complex(*x) - complex(*y)) / abs(complex(*x)) for x, y in zip(a["ritz_top8"], b["ritz_top8"]))
print(f"1 rank {a['value']} GB/s, {a['ms_per_step']} ms; 2 gloo ranks n_gpus={b['n_gpus']} {b['value']} GB/s "
      f"{b['ms_per_step']} ms; allreduces/fact {b['gram_schmidt']['allreduces_per_factorisation']}; "
      f"top-8 Ritz max rel diff 1 vs 2 ranks {d:.2e}")
json.dump({"b1": a, "b2": b, "top8_rel_diff": d}, open(f"{o}/summary.json", "w"))
assert b["n_gpus"] == 2 and d < 1e-12
PY
