"""torch DDP communication hooks over the gcow codec.

The reference caller (hw/models/train_imagenet.py:446-475, train_resnet_cifar10.py:74-125) all-reduces fp32
gradients with DDP, then copies the flattened gradient vector to the host, runs zfpy compress -> decompress on it
and copies it back (:453, :459-465, :471): the wire carries fp32 and the codec only simulates the loss, with two
PCIe copies per step. Two device-resident replacements:

* `roundtrip_hook` -- the reference's exact semantics (mean all-reduce, then encode -> decode of the reduced
  bucket), on the GPU: no `.cpu()`, no `torch.from_numpy(...).to(device)`.
* `compressed_allgather_hook` -- gradients compressed *before* the wire: each rank encodes its bucket, the
  compressed streams are all-gathered over RCCL, every rank decodes all of them and averages. At rate r the wire
  carries r/32 of the fp32 bytes per rank.

Both register with `ddp_model.register_comm_hook(GcowHookState(...), hook)`.
"""
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from . import codec
from ._ffi import GcowParams


@dataclass
class GcowHookState:
    params: GcowParams = field(default_factory=lambda: codec.rate(16, 1))
    process_group: object = None
    index_stride: int = 16  # variable-rate streams carry a block index for parallel decode
    encoders: dict = field(default_factory=dict)

    def encoder(self, n: int, dtype, device, index_stride=0):
        key = (n, dtype, device, index_stride)
        if key not in self.encoders:
            self.encoders[key] = codec.Encoder((n,), dtype, self.params, device, index_stride)
        return self.encoders[key]


def _done(t: torch.Tensor) -> torch.futures.Future[torch.Tensor]:
    fut = torch.futures.Future()
    fut.set_result(t)
    return fut


def roundtrip_hook(state: GcowHookState, bucket) -> torch.futures.Future[torch.Tensor]:
    """Mean all-reduce, then the lossy encode -> decode the reference applies (zfpy), device-resident."""
    group = state.process_group
    buf = bucket.buffer()
    world = dist.get_world_size(group)
    fut = dist.all_reduce(buf.div_(world), group=group, async_op=True).get_future()

    def lossy(f):
        t = f.value()[0]
        flat = t.reshape(-1)
        x = flat if flat.dtype in (torch.float32, torch.bfloat16) else flat.float()
        stride = 0 if codec.is_fixed(state.params) else state.index_stride
        e = state.encoder(x.numel(), x.dtype, x.device, stride)(x)
        out = codec.decode(e)
        flat.copy_(out.to(flat.dtype))
        return t

    return fut.then(lossy)


def compressed_allgather_hook(state: GcowHookState, bucket) -> torch.futures.Future[torch.Tensor]:
    """Encode locally, all-gather compressed streams, decode every rank's stream and average."""
    group = state.process_group
    buf = bucket.buffer()
    world = dist.get_world_size(group)
    flat = buf.reshape(-1)
    x = flat if flat.dtype in (torch.float32, torch.bfloat16) else flat.float()
    n = x.numel()
    p = state.params
    if codec.is_fixed(p):
        e = state.encoder(n, x.dtype, x.device)(x)
        nb = (n + 3) // 4
        nw = (nb * p.maxbits + 63) // 64
        local = e.words[:nw].contiguous()
        gathered = torch.empty(world * nw, dtype=torch.int64, device=x.device)
        dist.all_gather_into_tensor(gathered, local, group=group)
        acc = torch.zeros(n, dtype=torch.float32, device=x.device)
        tmp = torch.empty(n, dtype=torch.float32, device=x.device)
        for r in range(world):
            words = torch.cat([gathered[r * nw:(r + 1) * nw], torch.zeros(2, dtype=torch.int64, device=x.device)])
            codec.decode(words, (n,), p, out=tmp)
            acc += tmp
    else:
        stride = state.index_stride
        e = state.encoder(n, x.dtype, x.device, stride)(x)
        lens = torch.empty(world, dtype=torch.int64, device=x.device)
        dist.all_gather_into_tensor(lens, e.bits_dev.reshape(1), group=group)
        lens_h = lens.cpu().tolist()
        maxw = max(1, max((b + 63) // 64 for b in lens_h)) + 2
        local = torch.zeros(maxw, dtype=torch.int64, device=x.device)
        nw = (lens_h[dist.get_rank(group)] + 63) // 64
        local[:nw] = e.words[:nw]
        gathered = torch.empty(world * maxw, dtype=torch.int64, device=x.device)
        dist.all_gather_into_tensor(gathered, local, group=group)
        ni = e.index.numel()
        idx = torch.empty(world * ni, dtype=torch.int64, device=x.device)
        dist.all_gather_into_tensor(idx, e.index, group=group)
        acc = torch.zeros(n, dtype=torch.float32, device=x.device)
        tmp = torch.empty(n, dtype=torch.float32, device=x.device)
        for r in range(world):
            codec.decode(gathered[r * maxw:(r + 1) * maxw], (n,), p, index=idx[r * ni:(r + 1) * ni],
                         index_stride=stride, out=tmp)
            acc += tmp
    flat.copy_((acc / world).to(flat.dtype))
    return _done(buf)
