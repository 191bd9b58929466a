# Round-3 batch: resconv with unconditional tile-loop memory ops - conv + decoder parity, phase probe, bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_decoder.py tests/test_gpu_train_conv.py -q -x -rfE --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_h.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_h.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_engine.py 4 0 2 4 6 --rounds 2 > gpurun_out/ab_dbg_h.log 2>&1 || exit $?
head -5 gpurun_out/ab_dbg_h.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || exit $?
cat gpurun_out/bench_h.json
