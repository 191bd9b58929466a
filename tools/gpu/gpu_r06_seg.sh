# Round 6: utterance-relative persistent tile ranges (STTS_OPT_SEGPART) — the config-4 rank-shard test, repeat /
# A/B decoder tests, and the in-process timing A/B on the headline workload
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py -m gpu -q -rfE -k "config4 or deterministic or config3 or shard_invariant" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_seg_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r06_seg_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/ab_engine.py 29 0 1 --rounds 3 > gpurun_out/r06_ab_segpart.txt 2>&1 || exit $?
grep "^opt" gpurun_out/r06_ab_segpart.txt
