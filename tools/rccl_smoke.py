"""RCCL plumbing on one MI355X: the config-4 launcher's collectives at world size 1 (a one-GPU box cannot host
two RCCL ranks).  Initialises the "nccl" (= RCCL) process group with device_id as bench.py does, runs the
barrier + all_reduce(MAX) timing pattern and shard.gather_to_rank0 over a real decode, and checks the gathered
audio equals the local decode.  Run: python tools/rccl_smoke.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("LOCAL_RANK", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from helpers import decoder_case, make_decoder
    from stts2_mi355x import shard
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    print(f"init_process_group(nccl) world={dist.get_world_size()} backend={dist.get_backend()} "
          f"in {time.perf_counter() - t0:.2f} s")
    dec, _ = make_decoder("hifigan")
    dec = dec.cuda()
    asr, f0, n, s, nz = decoder_case(2, 16)
    dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.no_grad():
        out = dec(asr.cuda(), f0.cuda(), n.cuda(), s.cuda(), noise=nz.cuda(), dtype="bf16")
    torch.cuda.synchronize()
    ms = torch.tensor([(time.perf_counter() - t) * 1e3], device="cuda")
    dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    full = shard.gather_to_rank0(out, dist.get_world_size(), dist.get_rank())
    ok = full is not None and torch.equal(full, out)
    print(f"decode {float(ms):.2f} ms (all_reduce MAX), gather_to_rank0 {tuple(full.shape)} equal to local: {ok}")
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)
    print("rccl smoke ok")


if __name__ == "__main__":
    main()
