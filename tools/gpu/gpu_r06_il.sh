# Round 6: resconv with the epilogue of tile t - 1 interleaved into tile t's MFMA loop (STTS_OPT_EXP bit 32768) vs the
# default, in-process, with the ping-pong kernel on (default) and off (STTS_OPT_RCPP 0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_engine.py 13 0 32768 --rounds 3 > gpurun_out/r06_ab_il.txt 2>&1 || exit $?
timeout -k 10 600 python -u tools/ab_engine.py 13 0 32768 --set 18=0 --rounds 3 > gpurun_out/r06_ab_il_nopp.txt 2>&1 || exit $?
grep "^opt" gpurun_out/r06_ab_il.txt gpurun_out/r06_ab_il_nopp.txt
