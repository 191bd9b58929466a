# Round 6 closing: config-5 step on the final build, eager vs hipGraph replay in bf16 / fp32 / bf16x3, then config 2
# (iSTFTNet fp32 B = 1) via tools/gpu/gpu_cfg2.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_train_step.py --steps 10 --warmup 3 --dtypes bf16,fp32,bf16x3 --no-grad-check > gpurun_out/r06_final_train_eager.jsonl 2> gpurun_out/r06_final_train_eager.err || exit $?
timeout -k 10 600 python -u tools/bench_train_step.py --steps 10 --warmup 3 --dtypes bf16,fp32,bf16x3 --graph > gpurun_out/r06_final_train_graph.jsonl 2> gpurun_out/r06_final_train_graph.err || exit $?
cut -c1-300 gpurun_out/r06_final_train_eager.jsonl gpurun_out/r06_final_train_graph.jsonl
