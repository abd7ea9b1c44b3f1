set -o pipefail
O=gpurun_out/t8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py -x -q --timeout 240 --timeout-method thread -k "dcgs2 or golden or arnoldi" > $O/p.log 2>&1 || { echo pytest failed; tail -30 $O/p.log; exit 1; }
tail -2 $O/p.log
timeout -k 10 300 python tools/bench_configs.py > $O/configs.log 2> $O/configs.err || { echo configs failed; tail $O/configs.err; exit 1; }
cat $O/configs.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/host_overhead.py dcgs2 > $GRAFT_REPO_ROOT/$O/ho.txt 2>&1 || { echo ho failed; exit 1; }
grep wall $GRAFT_REPO_ROOT/$O/ho.txt
