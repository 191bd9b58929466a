# Round 6: the upsamplers' column-part-fastest tile order (default) vs frame-tile fastest (STTS_OPT_EXP 262144), in-process
# A/B in bf16 and bf16x3, then the family's FETCH / WRITE passes again on the new default
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_engine.py 13 262144 0 --rounds 3 > gpurun_out/r06_ab_upsorder.txt 2>&1 || exit $?
grep "^opt\|2560\|640\|192" gpurun_out/r06_ab_upsorder.txt | grep -v "^{" | head
timeout -k 10 500 python -u tools/ab_engine.py 13 262144 0 --rounds 2 --dtype bf16x3 > gpurun_out/r06_ab_upsorder_split.txt 2>&1 || exit $?
grep "^opt\|2560\|640\|192" gpurun_out/r06_ab_upsorder_split.txt | grep -v "^{" | head
rm -rf gpurun_out/traffic
export BENCH_ARGS="--no-parity-mode --no-accuracy-mode --no-e2e"
export STTS_OPTS=24=0
KERNEL=k_bigconv OUT=gpurun_out/r06_traffic_raw2.json bash tools/gpu/gpu_traffic.sh > gpurun_out/r06_traffic2.log 2>&1 || exit $?
echo traffic ok
