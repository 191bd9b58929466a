# Round 6: HIP runtime graph settings vs the replayed config-5 bf16 step (same process command per setting)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/r06_graph_env.txt
run() {
  echo "== $1" >> gpurun_out/r06_graph_env.txt
  env $1 timeout -k 10 300 python -u tools/bench_train_step.py --steps 10 --warmup 3 --dtypes bf16 --no-grad-check $2 2>/dev/null | cut -c1-260 >> gpurun_out/r06_graph_env.txt || return 1
}
run "X=0" "" && run "X=0" "--graph" && run "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "--graph" && run "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "--graph" \
  && run "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "--graph" && run "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "--graph" \
  && run "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "--graph" && run "DEBUG_HIP_GRAPH_BATCH_SIZE=1024" "--graph" || exit 3
cat gpurun_out/r06_graph_env.txt
