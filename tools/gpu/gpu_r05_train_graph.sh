# Round 5: config-5 train step, eager vs hipGraph replay (bf16, fp32, bf16x3), then a kernel trace of the bf16 graph run
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_train_step.py --steps 10 --warmup 3 --dtypes bf16,fp32,bf16x3 --no-grad-check > gpurun_out/train_eager.jsonl 2> gpurun_out/train_eager.err || exit $?
cut -c1-260 gpurun_out/train_eager.jsonl
timeout -k 10 600 python -u tools/bench_train_step.py --steps 10 --warmup 3 --dtypes bf16,fp32,bf16x3 --graph > gpurun_out/train_graph.jsonl 2> gpurun_out/train_graph.err || exit $?
cut -c1-260 gpurun_out/train_graph.jsonl
rm -rf gpurun_out/prof_train_graph
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_graph -o train --output-format csv -- python3 tools/bench_train_step.py --steps 4 --warmup 3 --dtypes bf16 --no-grad-check --graph > gpurun_out/prof_train_graph.log 2>&1 || exit $?
tail -1 gpurun_out/prof_train_graph.log | cut -c1-300
