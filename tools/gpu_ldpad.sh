# Column-stride experiment: the basis stride ld (800,129,024 B = 2^19 x 12209 at N=1e8) padded by
# NKV_TUNE_LDPAD doubles, base kernels, one process per padding on one box.
set -o pipefail
O=gpurun_out/${1:-ldpad}; mkdir -p $O
for pad in 0 4096 12288 61440 0; do
  NKV_TUNE_LDPAD=$pad timeout -k 10 300 python tools/tune_kernels.py run --variants base --ops dcgs2_upd0,dot2,op_diag --js 8,32,128 --rounds 3 --out $O/tune_$pad.json > $O/tune_$pad.log 2>&1 || { echo "pad $pad failed"; tail $O/tune_$pad.log; exit 1; }
  echo "pad=$pad"; grep -v amdgpu.ids $O/tune_$pad.log
done
