# Round-3 batch: STTS_OPT_RCPP (ping-pong resconv for residual / running-sum K >= 7 launches by default):
# conv + decoder + training-conv parity, the in-process A/B 0 / 1 / 2, the bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_decoder.py tests/test_gpu_train_conv.py -q -x -rfE --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_k.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_engine.py 18 0 1 2 --rounds 3 > gpurun_out/ab_rcpp.log 2>&1 || exit $?
head -4 gpurun_out/ab_rcpp.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err || exit $?
cut -c1-250 gpurun_out/bench_k.json
