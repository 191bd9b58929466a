"""Utterance-level data parallelism.

Utterances are independent through the whole synthesis path (InstanceNorm statistics are
per utterance, reference hifigan.py:17), so a batch shards by contiguous utterance ranges
with no collective on the audio path.  Noise drawn on the device is keyed by the GLOBAL
utterance id (stts_decoder_fwd's utt_offset), so every rank count produces the same audio.
"""
from __future__ import annotations


def shard_range(global_batch: int, world: int, rank: int):
    """Contiguous, balanced [start, start+count) of utterances for `rank` of `world`."""
    if world <= 0 or not (0 <= rank < world) or global_batch < 0:
        raise ValueError("bad shard spec")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


_DTYPES = ("float32", "float64", "float16", "bfloat16", "int64", "int32", "uint8")


def _staged(group, dev):
    """gloo runs scatter / gather / all_gather on host tensors only: device tensors are staged through host memory
    there (the CPU tests and bench.py's shared-GPU rehearsal); RCCL takes them in place."""
    import torch.distributed as dist
    return dev.type != "cpu" and dist.get_backend(group) == "gloo"


def scatter_from_rank0(t, world, rank, device=None, group=None):
    """Rank 0's [N, ...] tensor `t` (N = the global batch) split into the contiguous utterance shards of
    `shard_range(N, world, r)`: every rank gets its own [count_r, ...] slice (rank r's shard of the global
    batch, the input side of bench.py's data-parallel path; torch.distributed scatter, RCCL on the GPU box,
    gloo on the CPU).  Other ranks pass t = None: rank 0 broadcasts the shape and dtype first.  Input
    scatter only; nothing on the audio path needs a collective."""
    import torch
    import torch.distributed as dist
    dev = torch.device(device) if device is not None else (t.device if t is not None else torch.device("cpu"))
    out_dev = dev
    if _staged(group, dev):
        dev = torch.device("cpu")
    if rank == 0:
        if t is None:
            raise ValueError("scatter_from_rank0: rank 0 must hold the global tensor")
        name = str(t.dtype).replace("torch.", "")
        if name not in _DTYPES or t.dim() > 6:
            raise ValueError(f"scatter_from_rank0: unsupported tensor {t.dtype} / {t.dim()}-D")
        head = [t.dim(), _DTYPES.index(name)] + list(t.shape) + [0] * (6 - t.dim())
        hdr = torch.tensor(head, dtype=torch.long, device=dev)
    else:
        hdr = torch.zeros(8, dtype=torch.long, device=dev)
    dist.broadcast(hdr, src=0, group=group)
    nd, code = int(hdr[0]), int(hdr[1])
    shape = [int(v) for v in hdr[2:2 + nd].tolist()]
    dtype = getattr(torch, _DTYPES[code])
    spans = [shard_range(shape[0], world, r) for r in range(world)]
    mx = max(c for _, c in spans)
    recv = torch.empty([mx] + shape[1:], dtype=dtype, device=dev)
    if rank == 0:
        src = t.to(dev).contiguous()
        parts = []
        for s, c in spans:
            p = torch.zeros([mx] + shape[1:], dtype=dtype, device=dev)
            p[:c] = src[s:s + c]
            parts.append(p)
        dist.scatter(recv, parts, src=0, group=group)
    else:
        dist.scatter(recv, None, src=0, group=group)
    return recv[: spans[rank][1]].to(out_dev)


def gather_to_rank0(t, world, rank, group=None):
    """Collect per-rank [b_r, ...] tensors on rank 0 (utterance order); other ranks get None.
    Uses torch.distributed (RCCL on the GPU box, gloo on CPU) — output gather only."""
    import torch
    import torch.distributed as dist
    out_dev = t.device
    if _staged(group, t.device):
        t = t.cpu()
    sizes = [torch.zeros(1, dtype=torch.long, device=t.device) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([t.shape[0]], device=t.device), group=group)
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    if rank == 0:
        dist.gather(pad, bufs, dst=0, group=group)
        return torch.cat([b[: int(s.item())] for b, s in zip(bufs, sizes)]).to(out_dev)
    dist.gather(pad, None, dst=0, group=group)
    return None
