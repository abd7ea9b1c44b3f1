# r06e: per-shard PMC traffic for the world > 1 bench lines, the multi-dot vs dual-update counter
# comparison at the same shape, counters of the 25- and 48-kept restart rotation
# (item 2), and the optimised CPU line at full size (item 4).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06e
mkdir -p $O
cd $R
NKV_HEAD=${NKV_HEAD:-unknown} timeout -k 10 900 bash tools/gpu_shard_traffic.sh r06e_shards 22088 11044 5522 > $O/shards.log 2>&1 && \
OPS=dot2,dcgs2_upd0 NKV_PMC_PASSES="1 2 3" timeout -k 10 400 bash tools/gpu_pmc_kernels.sh r06e_pmc > $O/pmc.log 2>&1 && \
OPS=rotate_25,rotate_48 timeout -k 10 400 bash tools/gpu_pmc_kernels.sh r06e_pmc_rot > $O/pmc_rot.log 2>&1 && \
cd $R && timeout -k 10 600 python3 -u tools/cpu_factorisation.py $O/cpu_full_cgs2.json 44176 --variant cgs2 > $O/cpu_full_cgs2.log 2>&1
