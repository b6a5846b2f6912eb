"""Multi-GPU path: shard a gradient bucket across ranks, encode each shard on its own MI355X, all-gather the
compressed streams over RCCL (torch.distributed backend "nccl" is RCCL on ROCm) into the single-stream layout.

The reference never puts compressed bytes on a wire (its DDP all-reduce runs on fp32 before zfpy,
hw/models/train_imagenet.py:446-475); this is the exchange step north_star asks for.

Fixed rate: every block is maxbits long, so shard r's stream occupies bits [r*S*maxbits, ...) of the full stream;
with S*maxbits a multiple of 64 one all-gather of equal-size shard streams IS the single-GPU stream (byte-identical
to encoding the whole bucket on one GPU).
Variable rate: all-gather the per-rank bit lengths (device tensors), all-gather the streams padded to the longest,
then one launch stitches every shard at its exclusive-prefix bit offset (gcow_stitch_shards_device: the prefix is
taken on the device from the gathered lengths). Per-shard flush padding is dropped: offsets use the unflushed bit
counts. The host reads the gathered lengths once, to size the padded buffers.

The codec work is injectable: every function takes `codec=` (default `DeviceCodec`, the gfx950 kernels), so the
protocol code itself runs unchanged over gloo on CPU tensors with an oracle-backed codec in tests/test_dist_cpu.py.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.distributed as dist

from ._ffi import GcowError


class DeviceCodec:
    """The codec calls the exchange needs, on device tensors through libgcow.so. Encoders are cached per
    (slot, shape, dtype, params, index stride) so a repeated bucket allocates nothing. Eviction is by idleness, not by
    a fixed count: an entry not used during the last `idle_factor` x (number of cached entries) + `idle_slack` encode
    calls is dropped. A model with B buckets reuses each key every B calls, so its steady-state encoders are never
    evicted however large B is, while the first iteration's encoders (DDP rebuilds its buckets after it: new indices
    and sizes) are released after a few iterations instead of holding their output / index / workspace buffers for
    the life of the process. An evicted encoder's buffers live on while a caller still references them; callers that
    read them on another stream record that stream on them (gcow_amd.ddp does)."""

    def __init__(self, idle_factor: int = 2, idle_slack: int = 8):
        self._enc = OrderedDict()  # key -> [encoder, last tick], least recently used first
        self.idle_factor = max(1, int(idle_factor))
        self.idle_slack = max(0, int(idle_slack))
        self._tick = 0

    def encode(self, x: torch.Tensor, params, index_stride: int = 0, slot=None):
        """-> (words int64 tensor, bits int64[1] tensor on x.device, block index or None). Calls with the same shape,
        params and `slot` reuse (overwrite) one set of output buffers; callers whose streams are still in flight on
        another stream pass distinct slots (the DDP hook: one per bucket)."""
        from . import codec
        x = x.reshape(-1)
        self._tick += 1
        key = (slot, x.numel(), x.dtype, x.device, params.tuple(), index_stride)
        ent = self._enc.get(key)
        if ent is None:
            ent = self._enc[key] = [codec.Encoder((x.numel(),), x.dtype, params, x.device, index_stride), self._tick]
        else:
            ent[1] = self._tick
            self._enc.move_to_end(key)
        self._evict_idle()
        e = ent[0](x if x.is_contiguous() else x.contiguous())
        return e.words, e.bits_dev, e.index

    def _evict_idle(self):
        limit = self.idle_factor * len(self._enc) + self.idle_slack
        while self._enc:
            key, ent = next(iter(self._enc.items()))
            if self._tick - ent[1] <= limit:
                break
            del self._enc[key]

    def stitch_shards(self, dst, src, shard_words: int, lens, nshards: int):
        from . import codec
        return codec.stitch_shards(dst, src, shard_words, lens[:nshards])

    def decode(self, words, n: int, params, index=None, index_stride: int = 0, out=None):
        from . import codec
        return codec.decode(words, (n,), params, index=index, index_stride=index_stride, out=out)

    def decode_mean(self, streams, stream_words: int, nstreams: int, n: int, params, index=None,
                    index_words: int = 0, index_stride: int = 0, out=None):
        from . import codec
        return codec.decode_mean(streams, stream_words, nstreams, n, params, index, index_words, index_stride, out)


_DEVICE = None


def device_codec() -> DeviceCodec:
    global _DEVICE
    if _DEVICE is None:
        _DEVICE = DeviceCodec()
    return _DEVICE


def shard_bounds(nvals: int, world: int, rank: int, block: int = 4, align_blocks: int = 16):
    """Contiguous block-aligned shard [lo, hi) of a 1-D bucket of nvals values for `rank`. align_blocks = 16 makes
    every full shard end on a 64-bit stream boundary at any rate with 4 * rate integral. Small buckets leave the last
    ranks an empty shard (lo == hi == nvals); they still take part in every collective."""
    nblocks = (nvals + block - 1) // block
    per = (nblocks + world - 1) // world
    per = (per + align_blocks - 1) // align_blocks * align_blocks
    lo_b = min(per * rank, nblocks)
    hi_b = min(lo_b + per, nblocks)
    return min(lo_b * block, nvals), min(hi_b * block, nvals)


def is_nccl(group=None) -> bool:
    return dist.get_backend(group) == "nccl"


def allgather_into(out: torch.Tensor, local: torch.Tensor, group=None):
    """out = concat over ranks of `local` (equal sizes): one all_gather_into_tensor on RCCL, a list all_gather on
    gloo."""
    if is_nccl(group):
        dist.all_gather_into_tensor(out, local, group=group)
    else:
        world = dist.get_world_size(group)
        dist.all_gather(list(out.chunk(world)), local, group=group)
    return out


def allgather_into_async(out: torch.Tensor, local: torch.Tensor, group=None) -> torch.futures.Future:
    """allgather_into with async_op=True: -> the collective's Future (RCCL: completed once enqueued, its waiters
    synchronise on the collective's stream; gloo: completed when the data has arrived)."""
    if is_nccl(group):
        work = dist.all_gather_into_tensor(out, local, group=group, async_op=True)
    else:
        world = dist.get_world_size(group)
        work = dist.all_gather(list(out.chunk(world)), local, group=group, async_op=True)
    return work.get_future()


def allgather_fixed(words: torch.Tensor, nblocks: int, maxbits: int, group=None) -> torch.Tensor:
    """All-gather equal-size fixed-rate shard streams (each shard nblocks blocks of maxbits bits)."""
    if (nblocks * maxbits) % 64:
        raise GcowError("fixed-rate shard must end on a 64-bit boundary (shard blocks * maxbits % 64 == 0)")
    nw = nblocks * maxbits // 64
    local = words[:nw].contiguous()
    world = dist.get_world_size(group)
    out = torch.empty(world * nw, dtype=torch.int64, device=local.device)
    allgather_into(out, local, group)
    return out


def gather_lengths(bits, device, group=None):
    """All-gather one unflushed bit count per rank (an int or an int64[1] tensor): -> (device tensor, host list)."""
    world = dist.get_world_size(group)
    mine = bits.reshape(1).to(device=device, dtype=torch.int64) if isinstance(bits, torch.Tensor) else \
        torch.tensor([int(bits)], dtype=torch.int64, device=device)
    lens = torch.empty(world, dtype=torch.int64, device=device)
    allgather_into(lens, mine, group)
    return lens, [int(v) for v in lens.tolist()]  # the one host read: it sizes the padded buffers


def allgather_padded(words: torch.Tensor, nw: int, maxw: int, group=None, pad: int = 0) -> torch.Tensor:
    """All-gather each rank's first nw words padded with zeros to maxw: -> world * maxw (+ pad zero) words."""
    world = dist.get_world_size(group)
    local = torch.zeros(maxw, dtype=torch.int64, device=words.device)
    if nw:
        local[:nw] = words[:nw]
    out = torch.zeros(world * maxw + pad, dtype=torch.int64, device=words.device)
    allgather_into(out[: world * maxw], local, group)
    return out


def allgather_variable(words: torch.Tensor, bits, group=None, codec=None):
    """All-gather variable-rate shard streams and stitch them into one stream. `bits`: this rank's unflushed bit
    count (int or int64[1] tensor on words' device). Returns (words, total_bits)."""
    codec = codec or device_codec()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lens, lens_h = gather_lengths(bits, words.device, group)
    maxw = max(1, max((b + 63) // 64 for b in lens_h))
    gathered = allgather_padded(words, (lens_h[rank] + 63) // 64, maxw, group)
    total = sum(lens_h)
    out = torch.empty(max((total + 63) // 64, 1), dtype=torch.int64, device=words.device)
    codec.stitch_shards(out, gathered, maxw, lens, world)
    return out[: (total + 63) // 64], total


def encode_allgather(bucket: torch.Tensor, params, group=None, codec=None):
    """Encode this rank's contiguous shard of a 1-D bucket (replicated on every rank: the C4 layout) and rebuild the
    full stream on every rank. Returns (words, total_bits). A rank whose shard is empty (small buckets) joins the
    exchange with zero bits instead of encoding."""
    codec = codec or device_codec()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    bounds = [shard_bounds(bucket.numel(), world, r) for r in range(world)]
    lo, hi = bounds[rank]
    fixed = params.minbits == params.maxbits
    if hi > lo:
        words, bits, _ = codec.encode(bucket[lo:hi], params)
    else:
        words, bits = torch.zeros(1, dtype=torch.int64, device=bucket.device), 0
    sizes = {b - a for a, b in bounds}
    nb = (hi - lo + 3) // 4
    if fixed and len(sizes) == 1 and (hi - lo) % 4 == 0 and (nb * params.maxbits) % 64 == 0:
        out = allgather_fixed(words, nb, params.maxbits, group)
        return out, world * nb * params.maxbits
    if fixed:  # ragged shards: the bit counts are known on the host
        bits = nb * params.maxbits
    return allgather_variable(words, bits, group, codec)
