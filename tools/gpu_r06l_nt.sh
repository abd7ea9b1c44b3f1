set -o pipefail
# wide rotation: non-temporal load/store policy and column-stride padding at 25 / 48 kept, k = 128
O=gpurun_out/r06l
mkdir -p $O
NKV_TUNE_VRAND=1 timeout -k 10 400 python3 tools/tune_kernels.py run --variants rotg_off,rw_ntst0,rw_nt0,rw_nt00 --js 128 --ops rotate_25,rotate_48 --rounds 3 --out $O/tune_nt.json > $O/tune_nt.log 2>&1 && \
NKV_TUNE_LDPAD=4096 NKV_TUNE_VRAND=1 timeout -k 10 300 python3 tools/tune_kernels.py run --variants rotg_off,rw_ntst0 --js 128 --ops rotate_25,rotate_48 --rounds 2 --out $O/tune_ld1.json > $O/tune_ld1.log 2>&1 && \
NKV_TUNE_LDPAD=12288 NKV_TUNE_VRAND=1 timeout -k 10 300 python3 tools/tune_kernels.py run --variants rotg_off --js 128 --ops rotate_25,rotate_48 --rounds 2 --out $O/tune_ld3.json > $O/tune_ld3.log 2>&1
