# Round 6: the N-rank path of bench.py on a one-GPU box (ranks sharing cuda:0 over gloo, STTS_BENCH_SHARE_GPU=1), in the
# headline mode (bf16) at config 4's per-rank batch of 32 x 10 s: the audio gathered to rank 0 from N = 2 ranks (global
# 64) and N = 4 ranks (global 128) must equal the N = 1 decodes of the same global batches BIT FOR BIT (utterance-relative
# tile ranges).  Not a scaling figure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rehearsal6
export TMPDIR=/tmp
D=/tmp/rehearsal6
mkdir -p $D
F="--dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e --no-profile"
timeout -k 10 300 python -u bench.py --gpus 1 --batch 64 $F --dump-checksum $D/n1_64.npy > gpurun_out/rehearsal6/n1_64.log 2>&1 || { tail -20 gpurun_out/rehearsal6/n1_64.log; exit 3; }
STTS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --batch 32 $F --dump-checksum $D/n2.npy > gpurun_out/rehearsal6/n2.log 2>&1 || { tail -20 gpurun_out/rehearsal6/n2.log; exit 3; }
timeout -k 10 300 python -u bench.py --gpus 1 --batch 128 $F --dump-checksum $D/n1_128.npy > gpurun_out/rehearsal6/n1_128.log 2>&1 || { tail -20 gpurun_out/rehearsal6/n1_128.log; exit 3; }
STTS_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 4 --batch 32 $F --dump-checksum $D/n4.npy > gpurun_out/rehearsal6/n4.log 2>&1 || { tail -20 gpurun_out/rehearsal6/n4.log; exit 3; }
python - <<'PY'
import numpy as np
D = "/tmp/rehearsal6"
for n, ref in ((2, "n1_64"), (4, "n1_128")):
    a, b = np.load(f"{D}/{ref}.npy"), np.load(f"{D}/n{n}.npy")
    same = a.shape == b.shape and np.array_equal(a, b)
    err = float(np.abs(a - b).max()) if a.shape == b.shape else float("nan")
    print(f"N = {n} ranks x 32 vs N = 1 x {a.shape[0]} (bf16): shapes {b.shape} / {a.shape}, bitwise equal: {same}, "
          f"max-abs {err:.2e}, {'PASS' if same else 'FAIL'}")
PY
