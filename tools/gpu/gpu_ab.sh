# Engine-option A/B on the headline workload (tools/ab_engine.py), then the conv tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_engine.py ${AB_ARGS:-7 1 2 3} > gpurun_out/ab.log 2>&1 || exit $?
cat gpurun_out/ab.log | head -5
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_decoder.py -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
