# Round 6: the v3 engine (bigconv3.hip) — A/B tests against bigconv2, then in-process timing A/B on the headline
# workload (STTS_OPT_BIG3 0 = bigconv2 / v1, 7 = v3 with C = 128 on 4-wave blocks, 15 = C = 128 on 8-wave blocks)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py -m gpu -q -rfE -k "bigconv3" --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06_big3_tests.log 2>&1
rc=$?
tail -12 gpurun_out/r06_big3_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/ab_engine.py 28 0 7 15 --rounds 3 > gpurun_out/r06_ab_big3.txt 2>&1 || exit $?
grep -v "^{" gpurun_out/r06_ab_big3.txt | head -60
