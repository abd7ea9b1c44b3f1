set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python3 tools/check_variant_rotate.py rotw_off base --report-only > $O/check_rotw.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 400 python3 tools/tune_kernels.py run --variants rotw_off,base,rotw_w4,rotw_u2 --js 128 --ops rotate_20,rotate_25,rotate_32,rotate_40,rotate_48,rotate_64,rotate_half --rounds 3 --out $O/tune.json > $O/tune.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 300 python3 tools/tune_kernels.py run --variants rotw_off,base,rotw_w4 --js 64,100,200 --ops rotate_20,rotate_25,rotate_32,rotate_48 --rounds 2 --out $O/tune_k.json > $O/tune_k.log 2>&1
