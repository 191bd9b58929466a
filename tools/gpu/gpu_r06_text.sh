# Round 6: the text / duration chain against the reference in eval and train mode (injected dropout masks)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_text.py -m gpu -q -rfE -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06_text_tests.log 2>&1
rc=$?
grep -E "output|loss_|style input|passed|failed|Error" gpurun_out/r06_text_tests.log | tail -30
exit $rc
