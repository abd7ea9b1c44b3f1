#!/bin/bash
# Basis column-stride experiment: the 8-GPU shard size (E=5522, 100 MB columns) with the column
# stride left at 100 MB or padded to 800 MB (the N=1e8 stride); same bytes moved.
set -o pipefail
mkdir -p gpurun_out
for pad in 0 87523328 0 87523328; do
  echo "== E=5522 NKV_TUNE_LDPAD=$pad"
  NKV_TUNE_LDPAD=$pad timeout -k 10 200 python -u tools/tune_kernels.py run --E 5522 --variants base --js 32,128 \
      --rounds 3 --ops dot2,dcgs2_upd0 --out gpurun_out/stride_$pad.json 2>&1 | grep -v amdgpu.ids || exit 1
done
