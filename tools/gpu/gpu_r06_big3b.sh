# Round 6: bigconv3 with C = 256 on two 4-wave blocks per CU (STTS_OPT_BIG3 17: resblocks on v3, C = 256 4-wave) vs
# v3 8-wave (1) vs bigconv2 (0), in-process
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_engine.py 28 0 1 17 --rounds 3 > gpurun_out/r06_ab_big3_4w.txt 2>&1 || exit $?
grep "^opt\|k_bigconv', 256" gpurun_out/r06_ab_big3_4w.txt | grep -v "^{"
