set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 300 python3 tools/check_variant_rotate.py rotw_off base --report-only > $O/check_rotw.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 500 python3 tools/tune_kernels.py run --variants rotw_off,base,rotw_diag1,rotw_diag2,rotw_apre,rotw_w4 --js 128 --ops rotate_16,rotate_20,rotate_25,rotate_32,rotate_48,rotate_64 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1
