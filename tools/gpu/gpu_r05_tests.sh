# Round 5: run a pytest selection on the GPU (args: pytest selection)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest "$@" -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sel.log 2>&1
rc=$?
grep -E "passed|failed|error|Error|assert|FAILED|^E " gpurun_out/pytest_sel.log | tail -40
exit $rc
