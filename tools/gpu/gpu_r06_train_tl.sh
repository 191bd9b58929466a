# Round 6: why the replayed config-5 step is slower than eager — kernel traces of both (bf16,
# B = 2 x 155 frames), reduced to GPU busy / idle / overlap by tools/analyze_timeline.py
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for mode in eager graph; do
  G=""; [ $mode = graph ] && G="--graph"
  rm -rf gpurun_out/tl_$mode
  timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/tl_$mode -o tl --output-format csv -- python3 tools/bench_train_step.py --steps 6 --warmup 3 --dtypes bf16 --no-grad-check $G > gpurun_out/tl_$mode.log 2>&1 || exit $?
  tail -1 gpurun_out/tl_$mode.log | cut -c1-200
  python3 tools/analyze_timeline.py gpurun_out/tl_$mode --tail 0.4 > gpurun_out/tl_$mode.txt || exit $?
  cat gpurun_out/tl_$mode.txt
  rm -rf gpurun_out/tl_$mode
done
