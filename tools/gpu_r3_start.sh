# Round-3 re-entry check: the -m gpu suite on the current tree, the default bench line, and the
# STTS_OPT_EXP A/B (tools/ab_engine.py) of the last session's engine experiments.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 python -u tools/ab_engine.py 13 0 1 2 4 > gpurun_out/ab_exp.log 2>&1 || exit $?
head -5 gpurun_out/ab_exp.log
