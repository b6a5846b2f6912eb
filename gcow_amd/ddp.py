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

Both register with `ddp_model.register_comm_hook(GcowHookState(...), hook)`. `GcowHookState.codec` defaults to the
device codec (gcow_amd.dist.DeviceCodec); tests inject an oracle-backed codec to run the hook bodies over gloo.
"""
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from . import codec as _codec
from . import dist as gdist
from ._ffi import GcowParams

INDEX_STRIDE = 16  # block index spacing the multi-stream decoder reads (one entry per 16 blocks)


@dataclass
class GcowHookState:
    params: GcowParams = field(default_factory=lambda: _codec.rate(16, 1))
    process_group: object = None
    codec: object = None  # None: gcow_amd.dist.device_codec()

    def get_codec(self):
        return self.codec or gdist.device_codec()


def _done(t: torch.Tensor) -> torch.futures.Future[torch.Tensor]:
    fut = torch.futures.Future()
    fut.set_result(t)
    return fut


def _flat(buf: torch.Tensor):
    flat = buf.reshape(-1)
    return flat, (flat if flat.dtype in (torch.float32, torch.bfloat16) else flat.float())


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
        words, _, index = cdc.encode(x, state.params, stride)
        out = cdc.decode(words, x.numel(), state.params, index=index, index_stride=stride)
        flat.copy_(out.to(flat.dtype))
        return t

    return fut.then(lossy)


def compressed_allgather_hook(state: GcowHookState, bucket) -> torch.futures.Future[torch.Tensor]:
    """Encode locally, all-gather the compressed streams, decode every rank's stream and average (one launch)."""
    group = state.process_group
    buf = bucket.buffer()
    world = dist.get_world_size(group)
    flat, x = _flat(buf)
    n = x.numel()
    p = state.params
    cdc = state.get_codec()
    if _codec.is_fixed(p):
        words, _, _ = cdc.encode(x, p)
        nw = ((n + 3) // 4 * p.maxbits + 63) // 64
        gathered = gdist.allgather_padded(words, nw, nw, group, pad=2)
        mean = cdc.decode_mean(gathered, nw, world, n, p)
    else:
        words, bits, index = cdc.encode(x, p, INDEX_STRIDE)
        lens, lens_h = gdist.gather_lengths(bits, x.device, group)
        maxw = max(1, max((b + 63) // 64 for b in lens_h))
        rank = dist.get_rank(group)
        gathered = gdist.allgather_padded(words, (lens_h[rank] + 63) // 64, maxw, group, pad=2)
        ni = index.numel()
        idx = torch.empty(world * ni, dtype=torch.int64, device=x.device)
        gdist.allgather_into(idx, index[:ni].contiguous(), group)
        mean = cdc.decode_mean(gathered, maxw, world, n, p, idx, ni, INDEX_STRIDE)
    flat.copy_(mean.to(flat.dtype))
    return _done(buf)
