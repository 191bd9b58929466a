# per-kernel time of the config-5 training step (bf16): rocprofv3 --kernel-trace --stats over tools/bench_train_step.py
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/prof_train
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python3 tools/bench_train_step.py --steps 4 --warmup 1 --dtypes ${PROF_DT:-bf16} --no-grad-check > gpurun_out/prof_train.log 2>&1 || exit $?
tail -1 gpurun_out/prof_train.log | cut -c1-300
