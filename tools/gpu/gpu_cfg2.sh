# config 2 (B = 1, 10-s utterance, iSTFTNet decoder fp32): the concurrent small-batch branches off / on
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--decoder istftnet --dtype fp32 --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e"
STTS_OPTS=23=0,24=0 timeout -k 10 300 python -u bench.py $A > gpurun_out/bench_cfg2_off.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py $A > gpurun_out/bench_cfg2_on.log 2>&1 || exit 3
tail -1 gpurun_out/bench_cfg2_off.log | cut -c1-220; tail -1 gpurun_out/bench_cfg2_on.log | cut -c1-220
