# r06y: the gated full-size oracle comparisons with a restart, at the round-6 head: TEST selects
# the config-3 restart run or the noise-seed run (one per call: ~14 minutes of host time each)
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
(while sleep 50; do date >> $O/heartbeat_$TEST.txt; done) &
HB=$!
NKV_FULL_ORACLE=1 NKV_FULL_ORACLE_OUT_RS=$O/full_oracle_restart.json NKV_FULL_ORACLE_OUT_NS=$O/full_oracle_noise.json \
  timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_full_oracle.py -m gpu -x -v -s --timeout 1050 --timeout-method thread \
  -k "$TEST" > $O/pytest_$TEST.log 2>&1
RC=$?
kill $HB
exit $RC
