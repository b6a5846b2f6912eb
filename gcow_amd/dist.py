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

    def pack_index16(self, index8, n: int, params):
        from . import codec
        return codec.pack_index16(index8, n, params)

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


# ---------------------------------------------------------------------------------------------- sharded receive
# The receive side of the compressed DDP exchange without decoding every rank's whole stream on every rank: rank r
# owns one block-aligned shard of the bucket. Every rank cuts its own stream at the shard boundaries (fixed rate: at
# b * maxbits; variable rate: at the block index), sends piece r to rank r (one all-to-all), rank r decodes and
# averages the W pieces of its shard (gcow_decode_mean_device on W "streams" of one shard -- the same per-value
# arithmetic, in the same rank order, as decoding the whole streams), and one all-gather of the mean shards rebuilds
# the bucket on every rank. Per rank, against all-gathering the streams and decoding them all: (W - 1) / W of ONE
# stream received instead of W - 1 streams, 1 / W of the decode work, plus the all-gather of the mean (fp32 / bf16).
SHARD_ALIGN_BLOCKS = 64  # shard starts on 64-block multiples: a whole 16-block index chunk, and 64 maxbits % 64 == 0


def shard_plan(nvals: int, world: int):
    """Block-aligned shards [lo, hi) (values) of a 1-D bucket for every rank, and the values in a full shard."""
    bounds = [shard_bounds(nvals, world, r, align_blocks=SHARD_ALIGN_BLOCKS) for r in range(world)]
    per = max(hi - lo for lo, hi in bounds)
    return bounds, per


def alltoall_into(out: torch.Tensor, inp: torch.Tensor, group=None):
    """Equal-split all-to-all: chunk r of `inp` to rank r, chunk s of `out` from rank s."""
    dist.all_to_all_single(out, inp, group=group)
    return out


def shard_pieces_fixed(words: torch.Tensor, nvals: int, maxbits: int, group=None):
    """Fixed rate: this rank's stream cut at the shard boundaries and exchanged. Returns (pieces, piece_words, lo,
    hi): pieces holds rank s's piece of this rank's shard at s * piece_words (+ 2 zero words), [lo, hi) the shard."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    bounds, _ = shard_plan(nvals, world)
    nb = (nvals + 3) // 4
    # piece r = the words holding shard r's blocks: from the word its first block starts in (a 64-block multiple of
    # maxbits bits is whole words) to the word its last bit falls in -- a partial last block and a shard whose bits
    # are not a multiple of 64 (the last shard, or a one-shard bucket) end inside a word that must travel too
    spans = [((lo // 4) * maxbits // 64, (min((hi + 3) // 4, nb) * maxbits + 63) // 64) if hi > lo else (0, 0)
             for lo, hi in bounds]
    pw = max(1, max(w1 - w0 for w0, w1 in spans))
    send = torch.zeros(world * pw, dtype=torch.int64, device=words.device)
    for r, (w0, w1) in enumerate(spans):
        if w1 > w0:
            send[r * pw:r * pw + (w1 - w0)] = words[w0:w1]
    pieces = torch.zeros(world * pw + 2, dtype=torch.int64, device=words.device)
    alltoall_into(pieces[: world * pw], send, group)
    lo, hi = bounds[rank]
    return pieces, pw, lo, hi


def shard_pieces_variable(words: torch.Tensor, bits, index: torch.Tensor, nvals: int, index_stride: int = 16,
                          group=None):
    """Variable rate (block index every `index_stride` blocks): this rank's stream cut at the shard boundaries (the
    bit where each shard's first block starts, from the index), every piece starting at the stream word that holds
    its first bit, and its index entries rebased to that word. One all-gather of every rank's W + 1 cut positions
    (the host read that sizes the padded pieces), then two all-to-alls (words, index). Returns (pieces, piece_words,
    pidx, pidx_words, lo, hi): rank s's piece of this rank's shard at s * piece_words (+ 2 zero words) with its index
    at s * pidx_words."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    bounds, per = shard_plan(nvals, world)
    dev = words.device
    nb = (nvals + 3) // 4
    if index_stride not in (8, 16):  # the block-index spacings gcow_decode_mean_device takes
        raise GcowError("shard_pieces_variable: index_stride must be 8 or 16, got %r" % (index_stride,))
    starts = [lo // 4 // index_stride for lo, _ in bounds]  # index chunk of each shard's first block
    bits_t = bits.reshape(1).to(device=dev, dtype=torch.int64) if isinstance(bits, torch.Tensor) else \
        torch.tensor([int(bits)], dtype=torch.int64, device=dev)
    cut = torch.empty(world + 1, dtype=torch.int64, device=dev)
    for r, (lo, hi) in enumerate(bounds):  # an empty shard (lo = nvals) starts at the stream's end
        if lo // 4 < nb:
            cut[r:r + 1] = index[starts[r]:starts[r] + 1]
        else:
            cut[r:r + 1] = bits_t
    cut[world:] = bits_t
    allcuts = torch.empty(world * (world + 1), dtype=torch.int64, device=dev)
    allgather_into(allcuts, cut, group)
    C_h = [int(v) for v in allcuts.tolist()]  # the one host read: sizes the padded pieces
    def span(c0, c1):
        return (c0 >> 6, (c1 + 63) >> 6 if c1 > c0 else c0 >> 6)
    pw = 1
    for s in range(world):
        cs = C_h[s * (world + 1):(s + 1) * (world + 1)]
        for r in range(world):
            a, b = span(cs[r], cs[r + 1])
            pw = max(pw, b - a)
    mine = C_h[rank * (world + 1):(rank + 1) * (world + 1)]
    nchunk = [(min((hi + 3) // 4, nb) - lo // 4 + index_stride - 1) // index_stride if hi > lo else 0
              for lo, hi in bounds]
    iw = max(1, max(nchunk))
    send = torch.zeros(world * pw, dtype=torch.int64, device=dev)
    isend = torch.zeros(world * iw, dtype=torch.int64, device=dev)
    for r in range(world):
        a, b = span(mine[r], mine[r + 1])
        if b > a:
            send[r * pw:r * pw + (b - a)] = words[a:b]
        if nchunk[r]:
            isend[r * iw:r * iw + nchunk[r]] = index[starts[r]:starts[r] + nchunk[r]] - 64 * a
    pieces = torch.zeros(world * pw + 2, dtype=torch.int64, device=dev)
    alltoall_into(pieces[: world * pw], send, group)
    pidx = torch.empty(world * iw, dtype=torch.int64, device=dev)
    alltoall_into(pidx, isend, group)
    lo, hi = bounds[rank]
    return pieces, pw, pidx, iw, lo, hi


def allgather_shards(flat: torch.Tensor, shard: torch.Tensor, nvals: int, group=None):
    """Every rank's decoded shard (shard_plan bounds; `shard` = this rank's values) gathered into `flat` (n values,
    the bucket, any dtype)."""
    world = dist.get_world_size(group)
    _, per = shard_plan(nvals, world)
    mine = torch.zeros(per, dtype=flat.dtype, device=flat.device)
    mine[: shard.numel()] = shard
    if flat.is_contiguous() and flat.numel() == world * per:
        allgather_into(flat, mine, group)  # straight into the bucket
    else:
        full = torch.empty(world * per, dtype=flat.dtype, device=flat.device)
        allgather_into(full, mine, group)
        flat.copy_(full[: flat.numel()])
    return flat
