# Round 6: resconv C = 64 on 4-wave blocks (STTS_OPT_EXP bits 262144: 4 x 2 waves, 524288: 4 x 1 waves, + 1048576: K = 3
# only) vs the 8-wave default, in-process; then the same with the ping-pong kernel off (STTS_OPT_RCPP 0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_engine.py 13 0 262144 524288 1310720 --rounds 3 > gpurun_out/r06_ab_rc4w.txt 2>&1 || exit $?
timeout -k 10 600 python -u tools/ab_engine.py 13 0 262144 524288 --set 18=0 --rounds 3 > gpurun_out/r06_ab_rc4w_nopp.txt 2>&1 || exit $?
grep "^opt" gpurun_out/r06_ab_rc4w.txt gpurun_out/r06_ab_rc4w_nopp.txt
