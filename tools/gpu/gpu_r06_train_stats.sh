# Round 6: kernel stats of the replayed config-5 bf16 step (same command as gpu_r05_train_graph.sh's profile), to
# compare per-kernel durations with profiles/r05_train_step_graph_kernel_stats_bf16.csv
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/prof_train_graph6
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_graph6 -o train --output-format csv -- python3 tools/bench_train_step.py --steps 4 --warmup 3 --dtypes bf16 --no-grad-check --graph > gpurun_out/prof_train_graph6.log 2>&1 || exit $?
tail -1 gpurun_out/prof_train_graph6.log | cut -c1-300
find gpurun_out/prof_train_graph6 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r06_train_step_graph_kernel_stats_bf16.csv \;
find gpurun_out/prof_train_graph6 -name "*kernel_trace.csv" -delete
