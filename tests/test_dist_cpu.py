"""The N>1 exchange protocol (gcow_amd/dist.py) on world_size 2 / 3 gloo process groups on the CPU.

Each rank encodes its block-aligned shard with the oracle (CPU stand-in for the device encoder), then runs the same
all-gather / stitch protocol the GPU path runs over RCCL; the rebuilt stream must equal the single-stream encode
of the whole bucket, byte for byte (fixed and variable rate, ragged shards)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def np_stitch(dst, off, src, bits):
    """CPU model of k_stitch: OR `bits` bits of src into dst at bit offset off."""
    d = dst.numpy().view(np.uint64)
    s = src.numpy().view(np.uint64)
    nsw = (bits + 63) // 64
    w0, w1 = off // 64, (off + bits + 63) // 64
    for w in range(w0, w1):
        sbit = 64 * w - off
        if sbit < 0:
            v = int(s[0]) << (-sbit)
        else:
            i, sh = sbit // 64, sbit % 64
            v = int(s[i]) >> sh
            if sh and i + 1 < nsw:
                v |= int(s[i + 1]) << (64 - sh)
        lo = 64 * w
        if off + bits < lo + 64:
            v &= (1 << (off + bits - lo)) - 1
        d[w] = np.uint64(int(d[w]) | (v & (2 ** 64 - 1)))


def _worker(rank, world, port, mode, nvals, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from gcow_amd import dist as gdist
        from oracle import oracle as O
        a = O.gen_normal(nvals, 1e-3, 77, True)
        p = O.rate(16, 1) if mode == "fixed" else O.accuracy(1e-6)
        lo, hi = gdist.shard_bounds(nvals, world, rank)
        w, bits = O.compress(a[lo:hi], p)
        words = torch.from_numpy(np.concatenate([w, np.zeros(2, np.uint64)]).view(np.int64))
        if mode == "fixed":
            out = gdist.allgather_fixed(words, (hi - lo) // 4, p.maxbits)
            total = out.numel() * 64
        else:
            out, total = gdist.allgather_variable(words, bits, stitch=np_stitch)
        ref, ref_bits = O.compress(a, p)
        ok = out.numpy().view(np.uint64)[: len(ref)].tobytes() == ref.tobytes()
        ok = ok and (total == ref_bits if mode != "fixed" else total >= ref_bits)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,nvals", [(2, "fixed", 4 * 4096), (2, "variable", 4 * 5003 + 2),
                                               (3, "variable", 4 * 3001), (2, "variable", 6)])
def test_allgather_protocol_gloo(world, mode, nvals):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, nvals, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def test_shard_bounds_cover_and_align():
    from gcow_amd.dist import shard_bounds
    for nvals in (1, 4, 7, 4096, 268435456, 10 ** 6 + 3):
        for world in (1, 2, 3, 4, 8):
            b = [shard_bounds(nvals, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == nvals
            for (lo, hi), (lo2, _) in zip(b, b[1:]):
                assert hi == lo2 and (lo % 4 == 0 or lo == hi == nvals)
            for lo, hi in b[:-1]:
                assert (hi - lo) % 64 == 0 or hi == nvals  # 16 blocks: 64-bit aligned at rate >= 1/4



def _ddp_register(rank, world, port, q):
    import sys
    import torch.nn as nn
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        from gcow_amd import ddp
        for h in (ddp.roundtrip_hook, ddp.compressed_allgather_hook):
            m = nn.parallel.DistributedDataParallel(nn.Linear(4, 4))
            m.register_comm_hook(ddp.GcowHookState(), h)  # DDP validates the hook signature here
        q.put((rank, True))
    except Exception as ex:
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_ddp_hooks_register():
    """gcow_amd.ddp hooks pass DDP's comm-hook signature check (compute runs in the -m gpu DDP tests)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_register, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok is True for _, ok in res), res
