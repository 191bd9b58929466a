# Round 5: the split-operand bigconv2 variant: parity A/Bs + accuracy-mode A/B + noise-branch A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_split.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_split.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_engine.py 25 0 1 --dtype bf16x3 --rounds 2 > gpurun_out/ab_bigsplit.log 2>&1 || { tail -20 gpurun_out/ab_bigsplit.log; exit 3; }
tail -40 gpurun_out/ab_bigsplit.log
