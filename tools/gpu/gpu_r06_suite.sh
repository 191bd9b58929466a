# Round 6: the whole -m gpu suite on the current build (then smoke)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r06_pytest_gpu.log
tail -15 gpurun_out/r06_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r06_smoke.log
