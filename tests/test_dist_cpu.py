"""The N>1 exchange code on world_size 2 / 3 (and 8 for empty shards) gloo process groups on the CPU.

The product functions run exactly as written -- gcow_amd.dist.encode_allgather / allgather_variable and both
gcow_amd.ddp hooks -- with only their codec calls injected: tests/oracle_codec.OracleCodec does the encoding,
stitching and decoding with the oracle on CPU tensors. The rebuilt stream must equal the oracle's single-stream
encode of the whole bucket, byte for byte (fixed and variable rate, fp32 and bf16, ragged and empty shards); the
hooks' gradients must equal the mean over ranks of the oracle's decode(encode(local gradient)), bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    bad = [r for r in res if r[1] is not True]
    assert not bad, bad
    return res


def _params(mode):
    from gcow_amd import codec
    return {"rate16": codec.rate(16, 1), "rate8": codec.rate(8, 1), "rate2.5": codec.rate(2.5, 1),
            "acc1e-6": codec.accuracy(1e-6), "acc1e-3": codec.accuracy(1e-3), "prec20": codec.precision(20)}[mode]


def _allgather_worker(rank, world, port, q, mode, nvals, bf16):
    _init(rank, world, port)
    try:
        from gcow_amd import dist as gdist
        from oracle import oracle as O
        from oracle_codec import OracleCodec
        a = O.gen_normal(nvals, 1e-3, 77, True)
        if bf16:
            a = (a.view(np.uint32) >> 16).astype(np.uint16)
            bucket = torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
        else:
            bucket = torch.from_numpy(a.copy())
        p = _params(mode)
        cdc = OracleCodec()
        out, total = gdist.encode_allgather(bucket, p, codec=cdc)
        ref, ref_bits = O.compress(a, O.expert(*p.tuple()))
        got = out.numpy().view(np.uint64)
        ok = total == ref_bits and got.size == ref.size and got.tobytes() == ref.tobytes()
        lo, hi = gdist.shard_bounds(nvals, world, rank)
        encoded = [r for r in cdc.records if r[0] == "encode"]
        ok = ok and (len(encoded) == (1 if hi > lo else 0))  # an empty shard joins the exchange without encoding
        q.put((rank, True if ok else ("mismatch", total, ref_bits, got.size, ref.size)))
    except Exception as ex:  # pragma: no cover - reported through the queue
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,nvals,bf16", [
    (2, "rate16", 4 * 4096, False),       # equal aligned shards: one all-gather is the stream
    (3, "rate16", 4 * 3001 + 2, False),   # ragged shards: stitched at nb * maxbits offsets
    (2, "rate2.5", 4 * 999, False),       # maxbits 10: shard ends inside a word
    (2, "acc1e-6", 4 * 5003 + 2, False),
    (3, "acc1e-6", 4 * 3001, False),
    (3, "acc1e-3", 4 * 2000 + 1, True),   # bf16 variable rate (C5 shape, small)
    (2, "prec20", 6, False),              # one rank holds the whole tiny bucket
    (8, "acc1e-6", 400, False),           # world > nblocks / 16: ranks 7.. have empty shards (no hang)
    (8, "rate16", 400, False),
])
def test_encode_allgather_gloo(world, mode, nvals, bf16):
    _run(_allgather_worker, world, mode, nvals, bf16)


def _hook_worker(rank, world, port, q, hook_name, mode):
    _init(rank, world, port)
    try:
        import torch.nn as nn
        from gcow_amd import ddp
        from oracle import oracle as O
        from oracle_codec import OracleCodec
        torch.manual_seed(0)
        model = nn.Linear(53, 37, bias=False)  # one parameter: the bucket is its flattened gradient (1961 values)
        ref = nn.Linear(53, 37, bias=False)
        ref.load_state_dict(model.state_dict())
        dm = nn.parallel.DistributedDataParallel(model)
        p = _params(mode)
        hook = getattr(ddp, hook_name)
        dm.register_comm_hook(ddp.make_hook_state(hook=hook, params=p, codec=OracleCodec()), hook)
        torch.manual_seed(100 + rank)  # a different batch per rank
        x = torch.randn(16, 53)
        dm(x).square().mean().backward()
        ref(x).square().mean().backward()
        local = ref.weight.grad.reshape(-1).contiguous()
        allg = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(allg, local)
        op = O.expert(*p.tuple())
        if hook_name in ("compressed_allgather_hook", "compressed_sharded_hook"):
            acc = np.zeros(local.numel(), np.float32)
            for g in allg:
                w, _ = O.compress(g.numpy(), op)
                acc = acc + O.decompress(w, (local.numel(),), op)
            want = acc / np.float32(world)
        else:  # the reference's order: mean all-reduce (x / world summed), then encode -> decode
            mean = allg[0] / world
            for g in allg[1:]:
                mean = mean + g / world  # world 2: exact in any order (halving is exact)
            w, _ = O.compress(mean.numpy(), op)
            want = O.decompress(w, (local.numel(),), op)
        got = dm.module.weight.grad.reshape(-1).numpy()
        ok = np.array_equal(got.view(np.uint32), want.view(np.uint32))
        q.put((rank, True if ok else "gradient != mean of oracle decode(encode(local grads))"))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["rate16", "acc1e-6", "rate2.5"])
def test_compressed_sharded_hook_gloo(world, mode):
    """The sharded-receive hook end to end over gloo (cut positions all-gather, word and index all-to-alls, one
    decode-mean of the rank's shard, all-gather of the mean shards): bit-identical to the all-gather hook's result,
    the oracle's mean of decode(encode(each rank's gradient))."""
    _run(_hook_worker, world, "compressed_sharded_hook", mode)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["rate16", "acc1e-6", "rate2.5"])
def test_compressed_allgather_hook_gloo(world, mode):
    """The hook body end to end over gloo: encode, length exchange, padded stream + index all-gather, one
    decode-mean; bit-exact against the oracle's mean of decode(encode(each rank's gradient))."""
    _run(_hook_worker, world, "compressed_allgather_hook", mode)


class _Bucket:
    """The two GradBucket methods the hook uses."""

    def __init__(self, t, i):
        self.t, self.i = t, i

    def buffer(self):
        return self.t

    def index(self):
        return self.i


def _async_hook_worker(rank, world, port, q, mode):
    _init(rank, world, port)
    try:
        import time

        from gcow_amd import ddp
        from oracle import oracle as O
        from oracle_codec import OracleCodec
        p = _params(mode)
        op = O.expert(*p.tuple())
        state = ddp.make_hook_state(params=p, codec=OracleCodec())
        grads = [O.gen_normal(4 * 1000 + 3, 1e-3, 300 + r, False) for r in range(world)]
        g = torch.from_numpy(grads[rank].copy())
        if rank != 0:
            time.sleep(1.5)  # rank 0's collective cannot complete before this rank joins
        t0 = time.perf_counter()
        fut = ddp.compressed_allgather_hook(state, _Bucket(g, 0))
        ret = time.perf_counter() - t0
        pending = not fut.done()
        out = fut.wait()
        acc = np.zeros(g.numel(), np.float32)
        for a in grads:
            acc = acc + O.decompress(O.compress(a, op)[0], a.shape, op)
        want = acc / np.float32(world)
        ok = np.array_equal(out.numpy().view(np.uint32), want.view(np.uint32))
        if rank == 0:
            ok = ok and pending and ret < 1.0
        q.put((rank, True if ok else ("rank %d: returned after %.3f s, pending %s, bits ok %s" % (
            rank, ret, pending, np.array_equal(out.numpy().view(np.uint32), want.view(np.uint32))))))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def _fail_fast_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        import time

        from gcow_amd import ddp
        from oracle import oracle as O
        from oracle_codec import OracleCodec

        class Failing(OracleCodec):
            def decode_mean(self, *a, **k):
                if rank == 1:
                    raise RuntimeError("injected codec failure")
                return super().decode_mean(*a, **k)

        p = _params("acc1e-6")
        state = ddp.make_hook_state(params=p, codec=Failing(), timeout_s=20.0)
        g = [torch.from_numpy(O.gen_normal(4 * 500 + 1, 1e-3, 40 + 10 * rank + i, False)) for i in range(2)]
        t0 = time.perf_counter()
        futs = [ddp.compressed_allgather_hook(state, _Bucket(g[i], i)) for i in range(2)]
        errs = []
        for f in futs:
            try:
                f.wait()
                errs.append(None)
            except Exception as ex:  # noqa: BLE001
                errs.append(repr(ex))
        dt = time.perf_counter() - t0
        if rank == 1:  # the failing bucket, then the queued one fails at once (its exchange never runs)
            ok = errs[0] and "injected" in errs[0] and errs[1] and "earlier failure" in errs[1] and dt < 10
        else:  # bucket 0 completed; bucket 1's collectives fail (the peer aborted the group), well before the timeout
            ok = errs[0] is None and errs[1] is not None and dt < 15
        q.put((rank, True if ok else ("rank %d: %s after %.1f s" % (rank, errs, dt))))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_compressed_allgather_hook_fails_fast():
    """an exception inside one rank's variable-rate exchange (here its decode) must not leave DDP hanging.
    That rank's bucket future fails with the error, every later bucket's future fails at once, and its exchange
    group is torn down, so the peer -- blocked in the next bucket's length all-gather -- errors out too."""
    _run(_fail_fast_worker, 2)


@pytest.mark.parametrize("mode", ["rate16", "acc1e-6"])
def test_compressed_allgather_hook_is_async(mode):
    """The hook returns a pending future before the collective can complete (the other rank joins 1.5 s later) --
    bucket i's exchange overlaps the next buckets' backward -- and the future's value is still bit-exact."""
    _run(_async_hook_worker, 2, mode)


@pytest.mark.parametrize("mode", ["rate16", "acc1e-6"])
def test_roundtrip_hook_gloo(mode):
    _run(_hook_worker, 2, "roundtrip_hook", mode)


def test_shard_bounds_cover_and_align():
    from gcow_amd.dist import shard_bounds
    for nvals in (1, 4, 7, 400, 4096, 268435456, 10 ** 6 + 3):
        for world in (1, 2, 3, 4, 8):
            b = [shard_bounds(nvals, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == nvals
            for (lo, hi), (lo2, _) in zip(b, b[1:]):
                assert hi == lo2 and (lo % 4 == 0 or lo == hi == nvals)
            for lo, hi in b[:-1]:
                assert (hi - lo) % 64 == 0 or hi == nvals  # 16 blocks: 64-bit aligned at rate >= 1/4


def test_oracle_codec_stitch_model():
    """The CPU stand-in's stitch equals the oracle's single stream (sanity of the test double itself)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O
    from oracle_codec import OracleCodec
    a = O.gen_normal(4 * 777 + 1, 1e-3, 5, True)
    op = O.accuracy(1e-5)
    cuts = [0, 4 * 100, 4 * 100, 4 * 500, a.size]
    shards = [O.compress(a[x:y], op) for x, y in zip(cuts, cuts[1:])]
    maxw = max(len(w) for w, _ in shards) + 1
    src = np.zeros(maxw * len(shards), np.uint64)
    for r, (w, _) in enumerate(shards):
        src[r * maxw:r * maxw + len(w)] = w
    lens = torch.tensor([b for _, b in shards], dtype=torch.int64)
    total = int(lens.sum())
    dst = torch.full(((total + 63) // 64,), -1, dtype=torch.int64)
    OracleCodec().stitch_shards(dst, torch.from_numpy(src.view(np.int64)), maxw, lens, len(shards))
    ref, bits = O.compress(a, op)
    assert bits == total and dst.numpy().view(np.uint64).tobytes() == ref.tobytes()


def _ddp_register(rank, world, port, q):
    _init(rank, world, port)
    try:
        import torch.nn as nn
        from gcow_amd import ddp
        for h in (ddp.roundtrip_hook, ddp.compressed_allgather_hook):
            m = nn.parallel.DistributedDataParallel(nn.Linear(4, 4))
            m.register_comm_hook(ddp.make_hook_state(), h)  # DDP validates the hook signature here
        q.put((rank, True))
    except Exception as ex:
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_ddp_hooks_register():
    """gcow_amd.ddp hooks pass DDP's comm-hook signature check."""
    _run(_ddp_register, 2)


def _state_setup_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        import dataclasses

        from gcow_amd import ddp
        from oracle_codec import OracleCodec
        p = _params("acc1e-6")
        # construction, copies and dataclasses.replace issue no collective: rank 1 builds extra states that rank 0
        # never builds, then both call setup() -- a mismatched new_group would hang here
        if rank == 1:
            for _ in range(3):
                s = ddp.GcowHookState(params=p, codec=OracleCodec())
                dataclasses.replace(s, timeout_s=5.0)
        st = ddp.GcowHookState(params=p, codec=OracleCodec(), timeout_s=30.0)
        try:
            st.comm_group()
            ok = False  # must refuse before setup()
        except RuntimeError as ex:
            ok = "setup()" in str(ex)
        st.setup()
        ok = ok and st.comm_group() is not None and st.setup().comm_group() is st.comm_group()  # idempotent
        # the sharded hook's state has a group at any rate; a fixed-rate all-gather / round-trip state needs none
        ok = ok and ddp.make_hook_state(hook=ddp.compressed_sharded_hook, params=_params("rate16"))._comm_group \
            is not None
        ok = ok and ddp.make_hook_state(hook=ddp.compressed_allgather_hook, params=_params("rate16"))._comm_group \
            is None
        q.put((rank, True if ok else "rank %d: setup semantics" % rank))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_hook_state_setup_is_explicit():
    """GcowHookState's constructor issues no collective (ranks may build, copy or replace states
    independently); the variable-rate exchange group is created by setup() on every rank, and the hook refuses to
    run without it instead of creating the group lazily on the comm thread."""
    _run(_state_setup_worker, 2)


def test_device_codec_cache_evicts_idle_only(monkeypatch):
    """the DeviceCodec encoder cache keeps every key a model reuses each iteration, however many buckets
    it has (no fixed cap that misses every step past 64 buckets), and drops the keys of buckets that stopped being
    used (DDP's first-iteration buckets) after a few iterations. Encoder construction is stubbed (no GPU here)."""
    from gcow_amd import codec, dist as gdist
    built = []

    class FakeEnc:
        def __init__(self, shape, dtype, params, device, stride):
            built.append(shape)

        def __call__(self, x):
            class E:
                words = bits_dev = index = None
            return E()

    monkeypatch.setattr(codec, "Encoder", FakeEnc)
    c = gdist.DeviceCodec()
    p = codec.rate(16, 1)
    x = torch.zeros(64)
    first = 100  # first-iteration buckets
    for slot in range(first):
        c.encode(x, p, slot=("first", slot))
    B = 300  # rebuilt buckets, more than the old fixed cap of 64
    for it in range(6):
        for slot in range(B):
            c.encode(x, p, slot=slot)
    assert len(built) == first + B  # no steady-state bucket was ever rebuilt
    assert not any(isinstance(k[0], tuple) for k in c._enc)  # the first iteration's entries are gone
    assert len(c._enc) == B


def _sharded_exchange_worker(rank, world, port, q, mode, nvals, bf16, stride=16):
    _init(rank, world, port)
    try:
        from gcow_amd import codec
        from gcow_amd import dist as gdist
        from oracle import oracle as O
        from oracle_codec import OracleCodec
        p = _params(mode)
        op = O.expert(*p.tuple())
        cdc = OracleCodec()
        grads = []
        for r in range(world):
            a = O.gen_normal(nvals, 1e-3, 500 + r, True)
            if bf16:
                a = (a.view(np.uint32) >> 16).astype(np.uint16)
            grads.append(a)
        mine = torch.from_numpy(grads[rank].copy())
        x = mine.view(torch.bfloat16) if bf16 else mine
        fixed = codec.is_fixed(p)
        words, bits, index = cdc.encode(x, p, 0 if fixed else stride)
        if fixed:
            pieces, pw, lo, hi = gdist.shard_pieces_fixed(words, nvals, p.maxbits)
            pidx, iw = None, 0
        else:
            pieces, pw, pidx, iw, lo, hi = gdist.shard_pieces_variable(words, bits, index, nvals, stride)
        flat = torch.full((nvals,), -7.0, dtype=torch.float32)
        shard = flat[lo:hi]
        if hi > lo:
            cdc.decode_mean(pieces, pw, world, hi - lo, p, pidx, iw, 0 if fixed else stride, out=shard)
        gdist.allgather_shards(flat, shard, nvals)
        acc = np.zeros(nvals, np.float32)
        for a in grads:
            acc = acc + O.decompress(O.compress(a, op)[0], (nvals,), op)
        want = acc / np.float32(world)
        ok = np.array_equal(flat.numpy().view(np.uint32), want.view(np.uint32))
        q.put((rank, True if ok else "rank %d: mean over shards != oracle mean (shard %d..%d)" % (rank, lo, hi)))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("mode,nvals,bf16", [("rate16", 4 * 3000 + 2, False), ("rate2.5", 4 * 3001 + 1, False),
                                             ("acc1e-6", 4 * 3000 + 3, False), ("acc1e-3", 4 * 2999, True),
                                             ("acc1e-6", 300, False), ("rate16", 300, False)])
def test_sharded_pieces_gloo(world, mode, nvals, bf16):
    """gcow_amd.dist's sharded receive on its own (the exchange under compressed_sharded_hook): streams cut at 64-block
    shard boundaries, pieces and rebased index slices all-to-all'd, the shard's mean decoded from W pieces, the mean
    shards all-gathered -- equal, bit for bit, to the mean of the oracle decodes of the whole streams. Ragged last
    shards, partial last blocks, bf16 buckets, and buckets too small for every rank to own a shard (empty shards)."""
    _run(_sharded_exchange_worker, world, mode, nvals, bf16)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode,nvals,bf16", [("acc1e-6", 4 * 3000 + 3, False), ("acc1e-3", 4 * 2999, True)])
def test_sharded_pieces_index8_gloo(world, mode, nvals, bf16):
    """The same exchange with the block index every 8 blocks (the sharded hook's spacing, ddp.SHARDED_INDEX_STRIDE):
    pieces cut and index slices rebased at 8-block granularity, bit for bit against the oracle mean."""
    _run(_sharded_exchange_worker, world, mode, nvals, bf16, 8)


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("mode", ["rate16", "rate8", "rate2.5"])
@pytest.mark.parametrize("nvals", [10, 29, 4 * 63 + 3])
def test_sharded_pieces_fixed_small_buckets(world, mode, nvals):
    """Fixed-rate buckets of 64 blocks or fewer: one rank owns the whole bucket, and its bits (a partial last block,
    or blocks * maxbits not a multiple of 64) end inside a word. The piece must carry that word (the piece
    size was floor((values // 4) * maxbits / 64) words, one short at rate 8 / 2.5)."""
    _run(_sharded_exchange_worker, world, mode, nvals, False)
