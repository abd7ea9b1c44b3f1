#!/bin/bash
# Basis stride experiment: pads that are NOT multiples of 32 KiB (the "ldany" build relaxes the
# stride check to even), one process per pad, all on one box.
set -o pipefail
mkdir -p gpurun_out
for pad in 0 256 1024 2048 0 8 512 3072; do
  echo "== NKV_TUNE_LDPAD=$pad"
  NKV_TUNE_LDPAD=$pad timeout -k 10 200 python -u tools/tune_kernels.py run --variants ldany --js 32,128 \
      --rounds 3 --ops dot2,dcgs2_upd0 --out gpurun_out/ldodd_$pad.json 2>&1 | grep -v amdgpu.ids || exit 1
done
