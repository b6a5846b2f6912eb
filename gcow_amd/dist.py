"""Multi-GPU path: shard a gradient bucket across ranks, encode each shard on its own MI355X, all-gather the
compressed streams over RCCL (torch.distributed backend "nccl" is RCCL on ROCm) into the single-stream layout.

The reference never puts compressed bytes on a wire (its DDP all-reduce runs on fp32 before zfpy,
hw/models/train_imagenet.py:446-475); this is the exchange step north_star asks for.

Fixed rate: every block is maxbits long, so shard r's stream occupies bits [r*S*maxbits, ...) of the full stream;
with S*maxbits a multiple of 64 one all-gather of equal-size shard streams IS the single-GPU stream (byte-identical
to encoding the whole bucket on one GPU).
Variable rate: all-gather the per-rank bit lengths, all-gather the streams padded to the longest, then bit-stitch
shard r at its exclusive-prefix bit offset (gcow_stitch_device on the GPU). Per-shard flush padding is dropped:
offsets use the unflushed bit counts.

The protocol functions take plain int64 word tensors, so the same code runs over RCCL on device tensors and over
gloo on CPU tensors (tests/test_dist_cpu.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ._ffi import GcowError


def shard_bounds(nvals: int, world: int, rank: int, block: int = 4, align_blocks: int = 16):
    """Contiguous block-aligned shard [lo, hi) of a 1-D bucket of nvals values for `rank`. align_blocks = 16 makes
    every full shard end on a 64-bit stream boundary at any rate with 4 * rate integral."""
    nblocks = (nvals + block - 1) // block
    per = (nblocks + world - 1) // world
    per = (per + align_blocks - 1) // align_blocks * align_blocks
    lo_b = min(per * rank, nblocks)
    hi_b = min(lo_b + per, nblocks)
    return min(lo_b * block, nvals), min(hi_b * block, nvals)


def _allgather_into(out: torch.Tensor, local: torch.Tensor, group=None):
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)
    else:
        world = dist.get_world_size(group)
        dist.all_gather(list(out.chunk(world)), local, group=group)


def allgather_fixed(words: torch.Tensor, nblocks: int, maxbits: int, group=None) -> torch.Tensor:
    """All-gather equal-size fixed-rate shard streams (each shard nblocks blocks of maxbits bits)."""
    if (nblocks * maxbits) % 64:
        raise GcowError("fixed-rate shard must end on a 64-bit boundary (shard blocks * maxbits % 64 == 0)")
    nw = nblocks * maxbits // 64
    local = words[:nw].contiguous()
    world = dist.get_world_size(group)
    out = torch.empty(world * nw, dtype=torch.int64, device=local.device)
    _allgather_into(out, local, group)
    return out


def allgather_variable(words: torch.Tensor, bits: int, group=None, stitch=None):
    """All-gather variable-rate shard streams and stitch them into one stream. Returns (words, total_bits).
    `stitch(dst, dst_bit_offset, src, src_bits)` defaults to the device kernel (gcow_stitch_device)."""
    if stitch is None:
        from .codec import stitch as _dev_stitch
        stitch = _dev_stitch
    world = dist.get_world_size(group)
    dev = words.device
    lens = torch.zeros(world, dtype=torch.int64, device=dev)
    mine = torch.tensor([int(bits)], dtype=torch.int64, device=dev)
    _allgather_into(lens, mine, group)
    lens_h = [int(v) for v in lens.cpu().tolist()]
    maxw = max(1, max((b + 63) // 64 for b in lens_h))
    local = torch.zeros(maxw, dtype=torch.int64, device=dev)
    nw = (int(bits) + 63) // 64
    local[:nw] = words[:nw]
    gathered = torch.empty(world * maxw, dtype=torch.int64, device=dev)
    _allgather_into(gathered, local, group)
    total = sum(lens_h)
    out = torch.zeros((total + 63) // 64 + 1, dtype=torch.int64, device=dev)
    off = 0
    for r in range(world):
        if lens_h[r]:
            stitch(out, off, gathered[r * maxw:(r + 1) * maxw], lens_h[r])
        off += lens_h[r]
    return out[: (total + 63) // 64], total


def encode_allgather(bucket: torch.Tensor, params, group=None):
    """Encode this rank's contiguous shard of a 1-D bucket (replicated on every rank: the C4 layout) and rebuild the
    full stream on every rank. Returns (words, total_bits)."""
    from . import codec
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    bounds = [shard_bounds(bucket.numel(), world, r) for r in range(world)]
    lo, hi = bounds[rank]
    enc = codec.encode(bucket[lo:hi], params)
    sizes = {b - a for a, b in bounds}
    nb = (hi - lo + 3) // 4
    if codec.is_fixed(params) and len(sizes) == 1 and (hi - lo) % 4 == 0 and (nb * params.maxbits) % 64 == 0:
        words = allgather_fixed(enc.words, nb, params.maxbits, group)
        return words, world * nb * params.maxbits
    return allgather_variable(enc.words, enc.bits, group)
