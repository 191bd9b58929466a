"""The bench's N-rank launch path on the CPU (gloo, --selftest-cpu): `bench.py --gpus 2` spawns two
ranks through torch.distributed.run, shards the global batch by rank, takes the max over ranks,
reports n_gpus = 2, and the audio gathered to rank 0 equals the single-rank run's bit for bit."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, tmp_path, batch=3, extra=()):
    dump = str(tmp_path / f"audio_{n}.npy")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--selftest-cpu",
                        "--steps", "2", "--warmup", "1", "--batch", str(batch), "--frames", "4",
                        "--dump-checksum", dump, *extra], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # ONE JSON line, from rank 0
    return json.loads(lines[0]), np.load(dump)


def test_two_rank_launch_matches_one_rank(tmp_path):
    one, a1 = _run(1, tmp_path)
    two, a2 = _run(2, tmp_path)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["global_batch"] == 6 and one["config"]["global_batch"] == 3
    assert two["scaling"] == "weak" and "with_gather" in two and "with_scatter_gather" in two
    assert a2.shape == (6, 1, 2400)
    # weak scaling: rank r holds global utterances [3r, 3r + 3); the single-rank run is utterances 0-2
    assert np.array_equal(a2[:3], a1)
    assert not np.array_equal(a2[3:], a1)


def test_world_size_mismatch_fails_loudly(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--selftest-cpu"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
