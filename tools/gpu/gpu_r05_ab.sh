# Round 5: generic in-process A/B of an engine option on bf16 and bf16x3 (args: OPT V1 V2 ...)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_engine.py "$@" --rounds 3 > gpurun_out/ab_bf16.log 2>&1 || { tail -20 gpurun_out/ab_bf16.log; exit 3; }
grep -E "k_bigconv|^opt" gpurun_out/ab_bf16.log | head -60
timeout -k 10 300 python -u tools/ab_engine.py "$@" --rounds 2 --dtype bf16x3 > gpurun_out/ab_split.log 2>&1 || { tail -20 gpurun_out/ab_split.log; exit 3; }
grep -E "k_bigconv|^opt" gpurun_out/ab_split.log | head -40
