# Round 6: config-5 train step (bf16), eager vs hipGraph replay, unprofiled, alternated twice in separate processes
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/r06_train_eg.jsonl
for rep in 1 2; do
  for G in "" "--graph"; do
    timeout -k 10 300 python -u tools/bench_train_step.py --steps 10 --warmup 3 --dtypes bf16 --no-grad-check $G >> gpurun_out/r06_train_eg.jsonl 2> gpurun_out/r06_train_eg.err || exit $?
  done
done
cut -c1-330 gpurun_out/r06_train_eg.jsonl
