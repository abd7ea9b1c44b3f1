# r06o: wide-load rotation with workgroup visits of NKV_ROTW_SPAN consecutive tiles in row bands
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
V=base,rotw_s16,rotw_s16_r1,rotw_s16_r2,rotw_s4_r4,rotw_s8_r2,rotw_s32_r1
timeout -k 10 200 python3 tools/check_variant_rotate.py base rotw_s16_r2 > $O/check_s16_r2.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 500 python3 tools/tune_kernels.py run --variants $V --js 128 --ops rotate_20,rotate_25,rotate_32,rotate_48,rotate_64 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 300 python3 tools/tune_kernels.py run --variants base,rotw_s16_r1,rotw_s16_r2,rotw_s8_r2 --js 64,200 --ops rotate_25,rotate_48 --rounds 2 --out $O/tune_k.json > $O/tune_k.log 2>&1
