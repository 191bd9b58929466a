# host-side cost of the config-5 training step: cProfile over tools/bench_train_step.py (bf16, 3 steps)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16 --no-grad-check > gpurun_out/host_bench.log 2>&1 || exit 3
grep -h ms_per_step gpurun_out/host_bench.log | cut -c1-260
timeout -k 10 400 python -u -m cProfile -o gpurun_out/host.prof tools/bench_train_step.py --steps 3 --warmup 1 --dtypes bf16 --no-grad-check > gpurun_out/host_prof.log 2>&1 || exit 3
python -c "
import pstats
p = pstats.Stats('gpurun_out/host.prof'); p.sort_stats('tottime').print_stats(45)
" > gpurun_out/host_prof.txt 2>&1
head -80 gpurun_out/host_prof.txt | tail -60
