# Round 6: STTS_OPT_RCOCC (C = 32 K >= 7 launches without a residual on three blocks per CU) off / on, in-process,
# after the conv / decoder / edge suites
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/gpu_r06_iltest.sh || exit $?
timeout -k 10 600 python -u tools/ab_engine.py 30 0 1 --rounds 4 > gpurun_out/r06_ab_rcocc.txt 2>&1 || exit $?
grep "^opt\|k_resconv', 32" gpurun_out/r06_ab_rcocc.txt
