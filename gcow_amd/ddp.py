"""torch DDP communication hooks over the gcow codec.

The reference caller (hw/models/train_imagenet.py:446-475, train_resnet_cifar10.py:74-125) all-reduces fp32
gradients with DDP, then copies the flattened gradient vector to the host, runs zfpy compress -> decompress on it
and copies it back (:453, :459-465, :471): the wire carries fp32 and the codec only simulates the loss, with two
PCIe copies per step. Two device-resident replacements:

* `roundtrip_hook` -- the reference's exact semantics (mean all-reduce, then encode -> decode of the reduced
  bucket), on the GPU: no `.cpu()`, no `torch.from_numpy(...).to(device)`.
* `compressed_allgather_hook` -- gradients compressed *before* the wire: each rank encodes its bucket, the
  compressed streams are all-gathered over RCCL, and one launch decodes every rank's stream and averages them
  (gcow_decode_mean_device: acc = 0 + x_0 + x_1 + ... in rank order, then / world). At rate r the wire carries r/32
  of the fp32 bytes per rank.

All register with `ddp_model.register_comm_hook(make_hook_state(hook=hook, ...), hook)` (variable rate and the sharded
hook: the state's exchange group is created by `GcowHookState.setup()`, a collective every rank calls at the same
point). `GcowHookState.codec` defaults to the
device codec (gcow_amd.dist.DeviceCodec); tests inject an oracle-backed codec to run the hook bodies over gloo.
"""
import contextlib
import queue
import threading
from dataclasses import dataclass, field
from datetime import timedelta

import torch
import torch.distributed as dist

from . import codec as _codec
from . import dist as gdist
from ._ffi import GcowParams

INDEX_STRIDE = 16  # block index spacing of the round-trip hook's decode (one entry per 16 blocks)
# The sharded hook's index spacing: 8 blocks. decode_mean then runs one lane per 8 blocks (32 fp32 sums per lane, no
# register spills, 5 waves per SIMD): a rank's shard decodes in 0.50 instead of 0.66 ms at W = 8 (accuracy 1e-6,
# 256 Mi values; profiles/r05_dmean_stride8_ab.log) for an index of 1 byte per block instead of 0.5 -- ~6 % more bytes
# in the all-to-all. The all-gather hook gathers every rank's whole index, so it encodes with the same 8-block index
# and sends it packed (codec.pack_index16: the 16-block index's size, the 8-block midpoint as a 16-bit offset), and
# decode_mean reads the packed entries as 8-block chunks.
SHARDED_INDEX_STRIDE = 8


@dataclass
class GcowHookState:
    """Hook state, one per DDP model. `timeout_s` bounds every collective of the variable-rate exchange, which runs
    over a process group of its own. That group is created by `setup()` -- a collective: call it on every rank of
    `process_group`, at the same point of each rank's setup, after init_process_group and before the first backward
    (or build the state with `make_hook_state`, which does). Constructing, copying or `dataclasses.replace`-ing a
    state issues no collective.

    Failure: a rank whose exchange raises stops its comm thread (that bucket's future and every later one fail at
    once) and aborts the exchange group. Over gloo that closes the connections and peers blocked in an exchange
    collective error out at once; over RCCL/NCCL a peer already blocked in a collective only fails when `timeout_s`
    expires (the communicator's watchdog then tears the process group -- and by default the process -- down)."""
    params: GcowParams = field(default_factory=lambda: _codec.rate(16, 1))
    process_group: object = None
    codec: object = None  # None: gcow_amd.dist.device_codec()
    timeout_s: float = 300.0
    # the state is registered with compressed_sharded_hook (its exchange runs on the comm thread at any rate); set by
    # make_hook_state(hook=compressed_sharded_hook)
    sharded: bool = False
    _worker: object = field(default=None, repr=False)
    _side: dict = field(default_factory=dict, repr=False)
    _comm_group: object = field(default=None, repr=False)

    def get_codec(self):
        return self.codec or gdist.device_codec()

    def worker(self) -> "_CommWorker":
        if self._worker is None:
            self._worker = _CommWorker(self._abort_comm_group)
        return self._worker

    def needs_comm_group(self) -> bool:
        """A multi-rank state whose hook runs collectives on the comm thread: variable rate (the all-gather hook's
        length exchange) or the sharded hook at any rate. The fixed-rate all-gather and round-trip hooks issue theirs
        from the autograd thread on `process_group` and get no extra communicator."""
        return (dist.is_available() and dist.is_initialized() and dist.get_world_size(self.process_group) > 1
                and (self.sharded or not _codec.is_fixed(self.params)))

    def setup(self) -> "GcowHookState":
        """Create the exchange's process group (a collective over `process_group`'s ranks; a no-op for a one-rank
        group): the hook's ranks, in a group of their own so that its collectives (issued
        from the comm thread) never interleave with collectives DDP issues on `process_group` from the autograd
        thread (e.g. the find_unused_parameters all-reduce). Idempotent. Returns self."""
        if self._comm_group is None and self.needs_comm_group():
            ranks = dist.get_process_group_ranks(self.process_group or dist.group.WORLD)
            self._comm_group = dist.new_group(ranks=ranks, timeout=timedelta(seconds=self.timeout_s),
                                              use_local_synchronization=True)
        return self

    def comm_group(self):
        """The exchange group created by setup(). Never created lazily: creating it from the comm thread would race
        with process-group creation on the main thread, and creating it in the hook would block the autograd thread
        until every rank reached that bucket."""
        if self._comm_group is None:
            raise RuntimeError("GcowHookState has no exchange group: the variable-rate and sharded exchanges need "
                               "one, created by setup() on every rank before training -- use "
                               "make_hook_state(hook=<the hook>, ...), or GcowHookState(..., sharded=True).setup() "
                               "for compressed_sharded_hook")
        return self._comm_group

    def _abort_comm_group(self, ex):
        g = self._comm_group
        if g is None:
            return
        try:
            g.abort()  # NCCL/RCCL: tears down this rank's communicator (peers fail only at their timeout)
        except Exception:  # noqa: BLE001 -- gloo has no abort; destroying closes its connections
            try:
                dist.destroy_process_group(g)
            except Exception:  # noqa: BLE001
                pass

    def side_stream(self, dev):
        if dev not in self._side:
            self._side[dev] = torch.cuda.Stream(dev)
        return self._side[dev]


def make_hook_state(hook=None, **kw) -> GcowHookState:
    """GcowHookState(**kw).setup() for `hook` (the function the state is registered with; compressed_sharded_hook
    sets `sharded`): call on every rank of the hook's process group at the same point of setup."""
    if hook is not None and getattr(hook, "__name__", "") == "compressed_sharded_hook":
        kw.setdefault("sharded", True)
    return GcowHookState(**kw).setup()


def _done(t: torch.Tensor) -> torch.futures.Future[torch.Tensor]:
    fut = torch.futures.Future()
    fut.set_result(t)
    return fut


def _flat(buf: torch.Tensor):
    flat = buf.reshape(-1)
    return flat, (flat if flat.dtype in (torch.float32, torch.bfloat16) else flat.float())


def _mean_into(cdc, flat: torch.Tensor, *args):
    """decode_mean written straight into the bucket when it is fp32 or bf16 (bf16: the fp32 mean rounded to nearest
    even in the kernel -- no fp32 temporary, no cast pass); other dtypes through an fp32 temporary."""
    if flat.dtype in (torch.float32, torch.bfloat16) and flat.is_contiguous():
        cdc.decode_mean(*args, out=flat)
    else:
        flat.copy_(cdc.decode_mean(*args).to(flat.dtype))


def roundtrip_hook(state: GcowHookState, bucket) -> torch.futures.Future[torch.Tensor]:
    """Mean all-reduce, then the lossy encode -> decode the reference applies (zfpy), device-resident."""
    group = state.process_group
    buf = bucket.buffer()
    world = dist.get_world_size(group)
    fut = dist.all_reduce(buf.div_(world), group=group, async_op=True).get_future()
    cdc = state.get_codec()

    def lossy(f):
        t = f.value()[0]
        flat, x = _flat(t)
        stride = 0 if _codec.is_fixed(state.params) else INDEX_STRIDE
        # per-bucket buffers: DDP may run several buckets' callbacks before the first one's decode has read its words
        words, _, index = cdc.encode(x, state.params, stride,
                                     slot=("roundtrip", bucket.index() if hasattr(bucket, "index") else None))
        if flat.dtype in (torch.float32, torch.bfloat16) and flat.is_contiguous():
            cdc.decode(words, x.numel(), state.params, index=index, index_stride=stride, out=flat)  # in place
        else:
            out = cdc.decode(words, x.numel(), state.params, index=index, index_stride=stride)
            flat.copy_(out.to(flat.dtype))
        return t

    return fut.then(lossy)


class _CommWorker:
    """One FIFO thread per hook state for the variable-rate exchange: its host read of the gathered lengths (which
    size the padded all-gather) blocks this thread only, never the autograd thread, and the collectives it issues
    keep DDP's bucket order on every rank (one queue).

    Fail fast: the first exception stops the worker. That bucket's future and every future queued or submitted after
    it fail at once (DDP raises in its wait instead of hanging on a bucket that never runs), and `on_error` aborts the
    exchange's process group: gloo peers blocked in a collective with this rank error out at once, RCCL peers when
    the group's timeout expires."""

    def __init__(self, on_error=None):
        self.q = queue.Queue()
        self.failed = None
        self.on_error = on_error
        self.t = threading.Thread(target=self._loop, name="gcow-comm", daemon=True)
        self.t.start()

    def _stopped(self):
        return RuntimeError("gcow comm thread stopped after an earlier failure: %r" % (self.failed,))

    def _loop(self):
        while True:
            fn, fut = self.q.get()
            if self.failed is not None:
                if not fut.done():
                    fut.set_exception(self._stopped())
                continue
            try:
                fn(fut)  # completes fut itself, inside its stream context
            except Exception as ex:  # surfaces in DDP's wait on the hook future
                self.failed = ex
                if not fut.done():
                    fut.set_exception(ex)
                if self.on_error is not None:
                    self.on_error(ex)

    def submit(self, fn, fut):
        if self.failed is not None:
            fut.set_exception(self._stopped())
            return fut
        self.q.put((fn, fut))
        return fut


def compressed_allgather_hook(state: GcowHookState, bucket) -> torch.futures.Future[torch.Tensor]:
    """Encode locally, all-gather the compressed streams, decode every rank's stream and average (one launch).

    Asynchronous: the hook enqueues and returns, so bucket i's exchange overlaps the backward of the next buckets
    (DDP's point; hw/models/train_imagenet.py:194-195, 219, 224 relies on it). Fixed rate chains encode -> all-gather
    (async_op) -> decode-mean through Future.then. Variable rate needs the gathered lengths on the host to size the
    padded all-gather; that read and the collectives after it run on the state's comm thread (on a side stream that
    waits for the encode), and the returned future completes when the mean is written. Each bucket encodes into its
    own buffers (slot = bucket index), so a later bucket's encode never overwrites a stream still in flight."""
    group = state.process_group
    buf = bucket.buffer()
    world = dist.get_world_size(group)
    flat, x = _flat(buf)
    n = x.numel()
    p = state.params
    cdc = state.get_codec()
    slot = bucket.index() if hasattr(bucket, "index") else None
    if _codec.is_fixed(p):
        words, _, _ = cdc.encode(x, p, 0, slot=slot)
        nw = ((n + 3) // 4 * p.maxbits + 63) // 64
        gathered = torch.zeros(world * nw + 2, dtype=torch.int64, device=x.device)
        fut = gdist.allgather_into_async(gathered[: world * nw], words[:nw].contiguous(), group)

        def finish(f):
            f.wait()
            if gathered.is_cuda:
                # the callback runs on a pool stream; without this the allocator could hand `gathered` to the next
                # bucket's torch.zeros on the autograd stream before the decode below has read it
                gathered.record_stream(torch.cuda.current_stream(gathered.device))
            _mean_into(cdc, flat, gathered, nw, world, n, p)
            return buf

        return fut.then(finish)
    cgroup = state.comm_group() if world > 1 else group  # raises here, on the autograd thread, without setup()
    words, bits, index8 = cdc.encode(x, p, SHARDED_INDEX_STRIDE, slot=slot)
    index = cdc.pack_index16(index8, n, p)  # what travels: one entry per 16 blocks
    dev = x.device
    if dev.type == "cuda":
        ev = torch.cuda.Event()
        ev.record()
        side = state.side_stream(dev)
        fut = torch.futures.Future(devices=[dev])
    else:
        ev = side = None
        fut = torch.futures.Future()

    def exchange(fut):
        if side is not None:
            torch.cuda.set_device(dev)  # this thread's current device: the bucket's, on every LOCAL_RANK
        ctx = torch.cuda.stream(side) if side is not None else contextlib.nullcontext()
        with ctx:
            if side is not None:
                side.wait_event(ev)
                for t in (words, bits, index):  # read on the side stream: keep them out of the allocator until then
                    t.record_stream(side)
            lens, lens_h = gdist.gather_lengths(bits, dev, cgroup)  # host read: this thread waits, autograd does not
            maxw = max(1, max((b + 63) // 64 for b in lens_h))
            rank = dist.get_rank(cgroup)
            gathered = gdist.allgather_padded(words, (lens_h[rank] + 63) // 64, maxw, cgroup, pad=2)
            ni = index.numel()
            idx = torch.empty(world * ni, dtype=torch.int64, device=dev)
            gdist.allgather_into(idx, index[:ni].contiguous(), cgroup)
            _mean_into(cdc, flat, gathered, maxw, world, n, p, idx, ni, _codec.INDEX_PACKED16)
            # completed inside the side-stream context: the future records its event on this stream, so DDP's wait
            # orders its use of the bucket after the mean is written
            fut.set_result(buf)

    return state.worker().submit(exchange, fut)


def compressed_sharded_hook(state: GcowHookState, bucket) -> torch.futures.Future[torch.Tensor]:
    """The compressed exchange with a sharded receive side (gcow_amd.dist "sharded receive"): each rank encodes its
    bucket, cuts its stream at the shard boundaries (fixed rate: at b * maxbits; variable rate: at the block index)
    and sends piece r to rank r in one all-to-all; rank r decodes and averages the W pieces of its shard in one launch
    (gcow_decode_mean_device), and an all-gather of the mean shards (in the bucket's dtype: fp32, or bf16 rounded to
    nearest even in the kernel) rebuilds the bucket on every rank. The result is bit-identical to
    compressed_allgather_hook's (the same fp32 sums in rank order); per rank it receives (W - 1) / W of one stream
    instead of W - 1 streams and decodes 1 / W of the values, for an extra all-gather of the mean. Collectives run on
    the state's comm thread over its exchange group (GcowHookState.setup, every rank), on a side stream that waits
    for the encode; the returned future completes when the bucket holds the mean."""
    group = state.process_group
    buf = bucket.buffer()
    world = dist.get_world_size(group)
    flat, x = _flat(buf)
    n = x.numel()
    p = state.params
    cdc = state.get_codec()
    fixed = _codec.is_fixed(p)
    stride = 0 if fixed else SHARDED_INDEX_STRIDE
    cgroup = state.comm_group() if world > 1 else group  # raises here, on the autograd thread, without setup()
    slot = ("sharded", bucket.index() if hasattr(bucket, "index") else None)
    words, bits, index = cdc.encode(x, p, stride, slot=slot)
    dev = x.device
    if dev.type == "cuda":
        ev = torch.cuda.Event()
        ev.record()
        side = state.side_stream(dev)
        fut = torch.futures.Future(devices=[dev])
    else:
        ev = side = None
        fut = torch.futures.Future()

    def exchange(fut):
        if side is not None:
            torch.cuda.set_device(dev)
        ctx = torch.cuda.stream(side) if side is not None else contextlib.nullcontext()
        with ctx:
            if side is not None:
                side.wait_event(ev)
                for t in (words, bits, index):
                    if t is not None:
                        t.record_stream(side)
            if fixed:
                pieces, pw, lo, hi = gdist.shard_pieces_fixed(words, n, p.maxbits, cgroup)
                pidx, iw = None, 0
            else:
                pieces, pw, pidx, iw, lo, hi = gdist.shard_pieces_variable(words, bits, index, n, stride, cgroup)
            direct = flat.dtype in (torch.float32, torch.bfloat16) and flat.is_contiguous()
            shard = flat[lo:hi] if direct else torch.empty(hi - lo, dtype=torch.float32, device=dev)
            if hi > lo:
                cdc.decode_mean(pieces, pw, world, hi - lo, p, pidx, iw, stride, out=shard)
            gdist.allgather_shards(flat, shard if direct else shard.to(flat.dtype), n, cgroup)
            fut.set_result(buf)

    return state.worker().submit(exchange, fut)
