# Round 5: hardware rehearsal of bench.py's N-rank path on a one-GPU box (config 4 cannot run here: one MI355X).
# N = 2 and 4 ranks share cuda:0 (STTS_BENCH_SHARE_GPU=1, gloo collectives staged through host memory), each decoding
# its utterance shard of the same global batch of 8 x 10 s; the audio gathered to rank 0 must match the N = 1 decode
# utterance by utterance (noise keyed by the global utterance id). The check runs in fp32: the per-rank batch (8 / 4 / 2)
# picks different engines (split-K, concurrent branches, block shapes by tile count), so bf16 decodes of one utterance
# differ at the bf16 mode's own error level (~1.5e-2, measured) while fp32 ones agree to summation order. Throughput
# lines are printed but are NOT scaling figures.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rehearsal
export TMPDIR=/tmp
F="--dtype fp32 --steps 2 --warmup 1 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e --no-profile"
timeout -k 10 300 python -u bench.py --gpus 1 --batch 8 $F --dump-checksum gpurun_out/rehearsal/n1.npy > gpurun_out/rehearsal/n1.log 2>&1 || { tail -20 gpurun_out/rehearsal/n1.log; exit 3; }
STTS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --batch 4 $F --dump-checksum gpurun_out/rehearsal/n2.npy > gpurun_out/rehearsal/n2.log 2>&1 || { tail -20 gpurun_out/rehearsal/n2.log; exit 3; }
STTS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 4 --batch 2 $F --dump-checksum gpurun_out/rehearsal/n4.npy > gpurun_out/rehearsal/n4.log 2>&1 || { tail -20 gpurun_out/rehearsal/n4.log; exit 3; }
python - <<'PY'
import json, numpy as np
a = np.load("gpurun_out/rehearsal/n1.npy")
for n in (2, 4):
    b = np.load(f"gpurun_out/rehearsal/n{n}.npy")
    err = np.abs(a - b).reshape(a.shape[0], -1).max(1)
    print(f"N = {n} vs N = 1 (fp32): shape {b.shape} vs {a.shape}, per-utterance max-abs {np.array2string(err, precision=2)}, "
          f"max {err.max():.2e}, {'PASS' if a.shape == b.shape and err.max() < 1e-4 else 'FAIL'} (bound 1e-4)")
for n in (1, 2, 4):
    d = json.loads([l for l in open(f"gpurun_out/rehearsal/n{n}.log") if l.startswith("{")][-1])
    print(n, d["n_gpus"], d["config"]["parallelism"], "with_gather" in d and d.get("with_gather") is not None,
          {k: (d[k] or {}).get("ms_per_step") if isinstance(d.get(k), dict) else d.get(k) for k in ("ms_per_step", "with_gather", "with_scatter_gather")})
PY
