# Round 6: the config-4 rank-count tests (B = 256 vs 2 / 4 / 8 shards, B = 64 vs two B = 32 halves) and the default
# bench line on this build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py -m gpu -q -rfE -k "config4" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_c4_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r06_c4_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench1.log 2>&1 || exit $?
tail -1 gpurun_out/r06_bench1.log | cut -c1-600
