"""Multi-GPU path: shard a gradient bucket across ranks, encode each shard on its own MI355X, all-gather the
compressed streams over RCCL (torch.distributed backend "nccl" is RCCL on ROCm) into the single-stream layout.

The reference never puts compressed bytes on a wire (its DDP all-reduce runs on fp32 before zfpy,
hw/models/train_imagenet.py:446-475); this is the exchange step north_star asks for.

Fixed rate: every block is maxbits long, so shard r's stream occupies bits [r*S*maxbits, ...) of the full stream;
with S*maxbits a multiple of 64 one all_gather_into_tensor of equal-size shard streams IS the single-GPU stream.
Variable rate: all-gather the per-rank bit lengths, all-gather streams padded to the longest, then bit-stitch each
shard at its exclusive-prefix bit offset on the device (gcow_stitch_device).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import codec
from ._ffi import GcowError


def shard_bounds(nvals: int, world: int, rank: int, block: int = 4, align_blocks: int = 1):
    """Contiguous block-aligned shard [lo, hi) of a 1-D bucket of nvals values for `rank`."""
    nblocks = (nvals + block - 1) // block
    per = (nblocks + world - 1) // world
    per = (per + align_blocks - 1) // align_blocks * align_blocks
    lo_b = min(per * rank, nblocks)
    hi_b = min(lo_b + per, nblocks)
    return min(lo_b * block, nvals), min(hi_b * block, nvals)


def allgather_fixed(enc: codec.Encoded, group=None) -> torch.Tensor:
    """All-gather equal-size fixed-rate shard streams: the result is the single-stream sw/ layout."""
    p = enc.params
    nblocks = 1
    for s in enc.shape:
        nblocks *= (s + 3) // 4
    if (nblocks * p.maxbits) % 64:
        raise GcowError("fixed-rate shard must end on a 64-bit boundary (shard blocks * maxbits % 64 == 0)")
    words = nblocks * p.maxbits // 64
    local = enc.words[:words]
    world = dist.get_world_size(group)
    out = torch.empty(world * words, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out


def allgather_variable(enc: codec.Encoded, group=None):
    """All-gather variable-rate shard streams and stitch them into one stream. Returns (words, total_bits)."""
    world = dist.get_world_size(group)
    bits_local = enc.bits_dev.reshape(1)
    lens = torch.empty(world, dtype=torch.int64, device=bits_local.device)
    dist.all_gather_into_tensor(lens, bits_local, group=group)
    lens_h = lens.cpu().tolist()
    maxw = max((b + 63) // 64 for b in lens_h) if lens_h else 0
    maxw = max(maxw, 1)
    local = torch.zeros(maxw, dtype=torch.int64, device=bits_local.device)
    nw = (lens_h[dist.get_rank(group)] + 63) // 64
    local[:nw] = enc.words[:nw]
    gathered = torch.empty(world * maxw, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(gathered, local, group=group)
    total = sum(lens_h)
    out = torch.zeros((total + 63) // 64 + 1, dtype=torch.int64, device=local.device)
    off = 0
    for r in range(world):
        codec.stitch(out, off, gathered[r * maxw:(r + 1) * maxw], lens_h[r])
        off += lens_h[r]
    return out[: (total + 63) // 64], total


def encode_allgather(bucket_shard: torch.Tensor, params, group=None):
    """Encode this rank's 1-D shard and rebuild the full stream on every rank. Returns (words, total_bits)."""
    enc = codec.encode(bucket_shard, params)
    if codec.is_fixed(params):
        words = allgather_fixed(enc, group)
        return words, words.numel() * 64
    return allgather_variable(enc, group)
