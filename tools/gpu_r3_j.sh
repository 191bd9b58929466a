# Round-3 batch: the two-group ping-pong resconv (STTS_OPT_EXP 32) - parity vs lock-step, then the A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -k pingpong -q -x -rfE --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_j.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_j.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_engine.py 13 0 32 --rounds 3 > gpurun_out/ab_pp.log 2>&1 || exit $?
head -3 gpurun_out/ab_pp.log
