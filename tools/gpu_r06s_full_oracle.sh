# r06s: the gated complete full-size oracle runs at the round-6 head (config 3 factorisation at
# N=1e8, config 5 direct/adjoint at N=5e7), a heartbeat file so the long host-side oracle phases
# are not taken for a hang
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
NKV_FULL_ORACLE=1 NKV_FULL_ORACLE_OUT=$O/full_oracle_config3.json NKV_FULL_ORACLE_OUT5=$O/full_oracle_config5.json \
  timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_full_oracle.py -m gpu -x -v -s --timeout 1000 --timeout-method thread \
  -k "config3_full_size_factorisation or config5_full_size" > $O/pytest_full_oracle.log 2>&1
RC=$?
kill $HB
exit $RC
