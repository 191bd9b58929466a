# Generic round-4 GPU cycle: optional pytest selection, optional bench, optional extra command.
#   PYTEST="tests/test_x.py -k y"  BENCH="--steps 10"  EXTRA="python tools/..."  bash tools/gpu/gpu_run.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$PYTEST" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest $PYTEST -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${EXTRA_TIMEOUT:-600} $EXTRA > gpurun_out/extra.log 2>&1 || { tail -20 gpurun_out/extra.log; exit 3; }
  tail -${EXTRA_TAIL:-5} gpurun_out/extra.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py $BENCH > gpurun_out/bench.log 2>&1 || exit $?
  tail -1 gpurun_out/bench.log | cut -c1-400
fi
exit 0
