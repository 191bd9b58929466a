"""Multi-process (gloo, world size 2) test of the utterance sharding used by bench.py and
stts2_mi355x.shard: each rank synthesises its shard's inputs from the global utterance ids,
decodes them with the CPU oracle (tiny T), and rank 0 gathers; the result must equal the
single-process full batch bit for bit."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from stts2_mi355x.shard import shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, T, q):
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from helpers import decoder_case, make_decoder
    from oracle import stts_oracle as orc
    from stts2_mi355x.shard import gather_to_rank0, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = shard_range(B, world, rank)
    dec, cfg = make_decoder("hifigan")
    sd = {k: v.detach() for k, v in dec.state_dict().items()}
    asr, f0, n, s, noise = decoder_case(count, T, utt0=start)
    with torch.no_grad():
        out = orc.decoder_hifigan(asr, f0, n, s, sd, cfg, noise)
    full = gather_to_rank0(out.contiguous(), world, rank)
    if rank == 0:
        q.put(full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for B in (1, 7, 32, 256):
        for W in (1, 2, 3, 8):
            spans = [shard_range(B, W, r) for r in range(W)]
            assert sum(c for _, c in spans) == B
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c


@pytest.mark.slow
def test_two_rank_gloo_decode_equals_single_process():
    from helpers import decoder_case, make_decoder
    from oracle import stts_oracle as orc
    B, T, world = 3, 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    dec, cfg = make_decoder("hifigan")
    sd = {k: v.detach() for k, v in dec.state_dict().items()}
    asr, f0, n, s, noise = decoder_case(B, T)
    with torch.no_grad():
        ref = orc.decoder_hifigan(asr, f0, n, s, sd, cfg, noise).numpy()
    assert got.shape == ref.shape
    assert abs(got - ref).max() < 1e-5


def _scatter_worker(rank, world, port, q):
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
    import torch.distributed as dist
    from stts2_mi355x.shard import gather_to_rank0, scatter_from_rank0, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    for N, shape, dtype in ((5, (3, 4), torch.float32), (2, (7,), torch.int64), (1, (2, 2, 2), torch.float64)):
        full = (torch.arange(N * int(torch.tensor(shape).prod())).reshape((N,) + shape) * 3 - 7).to(dtype)
        mine = scatter_from_rank0(full if rank == 0 else None, world, rank)
        start, count = shard_range(N, world, rank)
        ok = mine.dtype == dtype and tuple(mine.shape) == (count,) + shape and torch.equal(mine, full[start:start + count])
        back = gather_to_rank0(mine.contiguous(), world, rank)  # the round trip restores rank 0's tensor
        res[N] = (ok, rank != 0 or torch.equal(back, full))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_scatter_from_rank0():
    """shard.scatter_from_rank0 (the input side of the data-parallel path): every rank receives exactly its
    shard_range slice of rank 0's global batch (ragged and single-utterance batches, three dtypes), and the
    gather restores the global tensor on rank 0."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        for N, (ok, round_trip) in got[r].items():
            assert ok, (r, N)
            assert round_trip, (r, N)
