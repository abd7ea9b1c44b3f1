# r06w: multi-dot with the same bytes in flight per CU spread over more waves (fewer loads each)
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 600 python3 tools/tune_kernels.py run --variants base,d2p4_b512,d2p4_b256,d2p2_b1024,d2p8_u1_b512,d2p4_u4_b256 --js 8,32,64,96,128 --ops dot2 --rounds 3 --out $O/tune.json > $O/tune.log 2>&1
