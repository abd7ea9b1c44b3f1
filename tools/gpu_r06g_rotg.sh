set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 300 python3 tools/check_variant_rotate.py rot_old base --report-only > $O/check_rotg.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 500 python3 tools/tune_kernels.py run --variants rot_old,base,rotg_diag3,rotg_diag5 --js 128 --ops rotate_16,rotate_25,rotate_32,rotate_48 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1
