# Round 6: the new GPU tests (config-4 rank shard invariance, fixed-point statistics range, capturable AdamW
# checkpoint round trip) and a default bench line on this build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_edge.py tests/test_gpu_train_step.py -m gpu -q -rfE \
  -k "config4 or fixed_point or roundtrip or graph_matches" --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06_new_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06_new_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-parity-mode --no-e2e > gpurun_out/r06_bench0.log 2>&1 || exit $?
tail -1 gpurun_out/r06_bench0.log | cut -c1-400
