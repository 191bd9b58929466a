cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-parity-mode --no-accuracy-mode > gpurun_out/bench_b1.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b1 -o b1 -- python -u bench.py --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-parity-mode --no-accuracy-mode --no-profile > gpurun_out/prof_b1.log 2>&1
tail -c 600 gpurun_out/bench_b1.log
