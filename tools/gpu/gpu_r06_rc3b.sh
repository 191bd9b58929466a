# Round 6: resconv C = 32 held to three blocks per CU (STTS_OPT_EXP 8192, 168 VGPRs) vs the default two, in-process
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_engine.py 13 0 8192 --rounds 4 > gpurun_out/r06_ab_rc3b.txt 2>&1 || exit $?
grep "^opt\|k_resconv', 32" gpurun_out/r06_ab_rc3b.txt
