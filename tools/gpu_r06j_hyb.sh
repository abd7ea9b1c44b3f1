set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python3 tools/check_variant_rotate.py rot_old base --report-only > $O/check_base.log 2>&1 && \
timeout -k 10 300 python3 tools/check_variant_rotate.py rot_old rotg_w8d3 --report-only > $O/check_w8d3.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 700 python3 tools/tune_kernels.py run --variants rot_old,rotg_off,base,rotg_nohyb,rotg_w8d3,rotg_w8d3_nohyb,rotg_w8d3_pf,rotg_d5_pf --js 128 --ops rotate_16,rotate_20,rotate_25,rotate_32,rotate_48 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1
