# Round-3 batch: UPS engine + decoder parity tests, A/B of the new engine options, then the data batch.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_decoder.py -q -x -rfE --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ups.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ups.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_engine.py 14 0 1 > gpurun_out/ab_ups.log 2>&1 || exit $?
head -3 gpurun_out/ab_ups.log
bash tools/gpu_r3_data.sh
