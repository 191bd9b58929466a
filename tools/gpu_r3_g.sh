# Round-3 batch: ups[3] on the resconv engine (STTS_OPT_UPS) - conv + decoder parity, step A/B, bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_decoder.py -q -x -rfE --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ups3.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ups3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_engine.py 14 0 1 > gpurun_out/ab_ups3.log 2>&1 || exit $?
head -3 gpurun_out/ab_ups3.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_ups3.json 2> gpurun_out/bench_ups3.err || exit $?
cat gpurun_out/bench_ups3.json
