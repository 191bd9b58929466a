# Round 6: where the v3 engine's time goes (STTS_OPT_DEBUG skip bits, v3 on: STTS_OPT_BIG3 7), and the burst-issue
# experiment (STTS_OPT_EXP bit 65536) against the spread issue, v3 and bigconv2 side by side
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_engine.py 4 0 1 4 8 16 32 61 --rounds 2 --set 28=7 > gpurun_out/r06_phases_big3.txt 2>&1 || exit $?
grep "k_bigconv', \(128\|256\), \(3\|7\|11\), 1, 0\|^opt" gpurun_out/r06_phases_big3.txt
timeout -k 10 600 python -u tools/ab_engine.py 13 0 65536 --rounds 3 --set 28=7 > gpurun_out/r06_ab_burst.txt 2>&1 || exit $?
grep "k_bigconv\|^opt" gpurun_out/r06_ab_burst.txt | head -40
