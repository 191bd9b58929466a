# BASELINE configs other than the headline, on the current tree: config 2 (iSTFTNet fp32, B = 1,
# 10 s), B = 1 HiFi-GAN bf16 eager and hipGraph, the duration / tokens -> waveform path (config 1's
# chain at 10 s), the training-step forward pieces (config 5 shape) and Vocos.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --decoder istftnet --dtype fp32 --batch 1 --no-parity-mode > gpurun_out/cfg/cfg2.log 2>&1 || exit $?
tail -1 gpurun_out/cfg/cfg2.log | cut -c1-200
timeout -k 10 300 python -u bench.py --batch 1 --no-parity-mode --no-cpu-baseline > gpurun_out/cfg/b1_bf16.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_graph.py > gpurun_out/cfg/graph_b1.json 2>/dev/null || exit $?
timeout -k 10 300 python -u tools/bench_duration.py > gpurun_out/cfg/duration.json 2>/dev/null || exit $?
timeout -k 10 200 python -u tools/bench_train_fwd.py > gpurun_out/cfg/train_fwd.json 2>/dev/null || exit $?
echo configs ok
