# Round-3 closing cycle, part 2: the other configs, the config-5 training step bench and its kernel trace.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_configs_r02.sh > gpurun_out/configs.log 2>&1 || exit $?
tail -2 gpurun_out/configs.log
timeout -k 10 300 python -u tools/bench_train_step.py --dtypes bf16,fp32 --steps 5 --warmup 2 > gpurun_out/bench_train.log 2>&1 || exit $?
cut -c1-200 gpurun_out/bench_train.log | grep config5
rm -rf gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python3 tools/bench_train_step.py --dtypes bf16 --steps 3 --warmup 1 > gpurun_out/prof_train.log 2>&1 || exit $?
echo "profiled train step ok"
