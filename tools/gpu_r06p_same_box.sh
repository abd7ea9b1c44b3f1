# r06p: the plain access shape (tools/write_streams) and the product's rotations on ONE box
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 200 tools/write_streams 100014464 128 25 > $O/write_streams_25.log 2>&1 && \
timeout -k 10 200 tools/write_streams 100014464 128 16 > $O/write_streams_16.log 2>&1 && \
NKV_TUNE_VRAND=1 timeout -k 10 300 python3 tools/tune_kernels.py run --variants base,rotf_off --js 128 --ops rotate_16,rotate_25 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1
