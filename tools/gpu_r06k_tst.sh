set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 300 python3 tools/check_variant_rotate.py rot_old base --report-only > $O/check_base.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 600 python3 tools/tune_kernels.py run --variants rot_old,rotg_off,base,rotg_d5,rotg_d6 --js 128 --ops rotate_16,rotate_20,rotate_25,rotate_32,rotate_48,rotate_64 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 300 python3 tools/tune_kernels.py run --variants rot_old,rotg_off,base --js 64,100,200 --ops rotate_25,rotate_48 --rounds 2 --out $O/tune_k.json > $O/tune_k.log 2>&1
