# r06u: the VALU few-column rotation past 16 kept columns against the MFMA wide-load kernel
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 200 python3 tools/check_variant_rotate.py base rotf32 --report-only > $O/check_rotf32.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 400 python3 tools/tune_kernels.py run --variants base,rotf32,rotf32_p2 --js 64,128,200 --ops rotate_20,rotate_25,rotate_32 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1
