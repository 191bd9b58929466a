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


def gather_to_rank0(t, world, rank, group=None):
    """Collect per-rank [b_r, ...] tensors on rank 0 (utterance order); other ranks get None.
    Uses torch.distributed (RCCL on the GPU box, gloo on CPU) — output gather only."""
    import torch
    import torch.distributed as dist
    sizes = [torch.zeros(1, dtype=torch.long, device=t.device) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([t.shape[0]], device=t.device), group=group)
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    if rank == 0:
        dist.gather(pad, bufs, dst=0, group=group)
        return torch.cat([b[: int(s.item())] for b, s in zip(bufs, sizes)])
    dist.gather(pad, None, dst=0, group=group)
    return None
