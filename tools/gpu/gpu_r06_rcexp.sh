# Round 6: resconv prefetch options re-measured on the final build (STTS_OPT_EXP bit 4: residual rows one tile ahead
# on the dilation-1 residual launches; 8 / 16: window prefetch three tiles deep at C = 64 / 32), in-process
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u tools/ab_engine.py 13 0 4 8 16 --rounds 3 > gpurun_out/r06_ab_rcexp.txt 2>&1 || exit $?
grep "^opt" gpurun_out/r06_ab_rcexp.txt
