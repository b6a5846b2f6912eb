"""GPU parity of the multi-GPU exchange path against the oracle, bit-exact.

* gcow_stitch_shards_device (one launch for every shard) vs the oracle's single-stream encode of the whole bucket;
* gcow_decode_mean_device (one launch decodes every rank's stream and averages) vs the oracle's decodes summed in
  rank order;
* the product exchange code (gcow_amd.dist.encode_allgather, gcow_amd.ddp.compressed_allgather_hook) in 2 and 3
  processes sharing the one GPU: the collectives run over gloo on host copies, every codec call runs the gfx950
  kernels (a host-staging wrapper around gcow_amd.dist.DeviceCodec);
* both DDP hooks at world 1 over RCCL, each gradient compared bit-exactly with the oracle.
"""
import os
import tempfile
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gc():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a device")
    from gcow_amd import codec
    return codec


def _P(gc, op):
    return gc.expert(*op.tuple())


def _bucket(orc, n, seed, bf16=False):
    a = orc.gen_normal(n, 1e-3, seed, True)
    if bf16:
        a = (a.view(np.uint32) >> 16).astype(np.uint16)
    return a


def _dev(a):
    x = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return x.view(torch.bfloat16) if a.dtype == np.uint16 else x


# ---------------------------------------------------------------------------------------------- stitch_shards
@pytest.mark.parametrize("mode", ["acc1e-6", "acc1e-3_bf16", "rate2.5", "prec20"])
@pytest.mark.parametrize("k", [2, 3, 8])
def test_stitch_shards_equals_single_stream(gc, orc, mode, k):
    """Shards cut at 16-block multiples (and one empty shard) encoded on the device separately, laid out shard_words
    apart as after a padded all-gather, stitched in one launch == the oracle's stream of the whole bucket."""
    bf16 = mode.endswith("bf16")
    a = _bucket(orc, 4 * 10001 + 3, 11 + k, bf16)
    op = {"acc1e-6": orc.accuracy(1e-6), "acc1e-3_bf16": orc.accuracy(1e-3), "rate2.5": orc.rate(2.5, 1),
          "prec20": orc.precision(20)}[mode]
    nb = (a.size + 3) // 4
    per = (nb // k + 15) // 16 * 16
    cuts = [min(4 * per * r, a.size) for r in range(k)] + [a.size]
    if k >= 3:
        cuts[1] = cuts[0]  # an empty shard
    x = _dev(a)
    enc = [gc.encode(x[lo:hi], _P(gc, op)) if hi > lo else None for lo, hi in zip(cuts, cuts[1:])]
    lens = [e.bits if e is not None else 0 for e in enc]
    maxw = max(1, max((b + 63) // 64 for b in lens))
    src = torch.zeros(k * maxw, dtype=torch.int64, device="cuda")
    for r, e in enumerate(enc):
        if e is not None and lens[r]:
            src[r * maxw:r * maxw + e.nwords] = e.stream()
    total = sum(lens)
    dst = torch.full(((total + 63) // 64,), -1, dtype=torch.int64, device="cuda")  # written whole, no zeroing
    gc.stitch_shards(dst, src, maxw, torch.tensor(lens, dtype=torch.int64, device="cuda"))
    ref, bits = orc.compress(a, op)
    torch.cuda.synchronize()
    assert total == bits
    assert dst.cpu().numpy().view(np.uint64).tobytes() == ref.tobytes()


# ---------------------------------------------------------------------------------------------- decode_mean
def _oracle_mean(orc, streams, op, n):
    acc = np.zeros(n, np.float32)
    for w in streams:
        acc = acc + orc.decompress(w, (n,), op)
    return acc / np.float32(len(streams))


MEAN_MODES = {"rate16": (16,), "rate8": (8,), "rate2.5": (2.5,), "expert_generic": (64, 64, 20, -1074),
              "acc1e-6": 1e-6, "acc1e-3": 1e-3, "bf16_acc1e-6": 1e-6,
              # variable rate outside the closed-form domain: minbits > 1 pads, maxbits < 160 truncates
              "expert_var_minbits": (8, 512, 32, -1074), "expert_var_trunc": (1, 100, 64, -30)}


def _enc_stride(stride):
    """The encoder's index spacing for a decode_mean index form: 8, 16, or "packed" (encoded every 8 blocks, sent as
    the packed 16-block index, ddp.compressed_allgather_hook's form)."""
    return 8 if stride == "packed" else stride


def _mean_index(gc, encs, stride, n, p):
    """(index tensor, entries per stream, decode_mean index_stride) of the encodes `encs` in the form `stride`."""
    if stride == "packed":
        pk = [gc.pack_index16(e.index, n, p) for e in encs]
        return torch.cat(pk), pk[0].numel(), gc.INDEX_PACKED16
    ni = encs[0].index.numel()
    return torch.cat([e.index[:ni] for e in encs]), ni, stride


def _mean_op(orc, mode):
    v = MEAN_MODES[mode]
    if isinstance(v, float):
        return orc.accuracy(v)
    return orc.rate(v[0], 1) if len(v) == 1 else orc.expert(*v)


@pytest.mark.parametrize("mode", list(MEAN_MODES))
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("stride", [16, 8, "packed"])
def test_decode_mean_vs_oracle(gc, orc, mode, world, stride):
    n = 4 * 20001 + 2  # a partial last block; > 128 index chunks; 5001 blocks: the last 16-block entry has no midpoint
    op = _mean_op(orc, mode)
    fixed = op.minbits == op.maxbits
    if fixed and stride != 16:
        pytest.skip("fixed rate takes no index")
    buckets = [_bucket(orc, n, 900 + r, mode.startswith("bf16")) for r in range(world)]
    encs = [gc.encode(_dev(b), _P(gc, op), index_stride=0 if fixed else _enc_stride(stride)) for b in buckets]
    lens = [e.bits for e in encs]
    sw = max((b + 63) // 64 for b in lens) + (0 if fixed else 1)
    streams = torch.zeros(world * sw + 2, dtype=torch.int64, device="cuda")
    for r, e in enumerate(encs):
        streams[r * sw:r * sw + e.nwords] = e.stream()
    idx, ni, st = None, 0, 0
    if not fixed:
        idx, ni, st = _mean_index(gc, encs, stride, n, _P(gc, op))
    got = gc.decode_mean(streams, sw, world, n, _P(gc, op), idx, ni, st)
    want = _oracle_mean(orc, [orc.compress(b, op)[0] for b in buckets], op, n)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32))


def _bf16_rne(a: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 bits, round to nearest even (torch's conversion; the means here are finite)."""
    u = a.view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


@pytest.mark.parametrize("mode", list(MEAN_MODES))
@pytest.mark.parametrize("world", [1, 3])
@pytest.mark.parametrize("layout", ["contiguous", "strided"])
@pytest.mark.parametrize("stride", [16, 8, "packed"])
def test_decode_mean_bf16_output(gc, orc, mode, world, layout, stride):
    """decode_mean into a bf16 bucket (the hook's receive side for bf16 gradients): the fp32 mean of the oracle
    decodes, rounded to nearest even, written in place -- contiguous (8-byte block stores, the lean kernels' transposed
    stores) and strided (value stores)."""
    n = 4 * 20001 + 2
    op = _mean_op(orc, mode)
    fixed = op.minbits == op.maxbits
    if fixed and stride != 16:
        pytest.skip("fixed rate takes no index")
    buckets = [_bucket(orc, n, 700 + r, mode.startswith("bf16")) for r in range(world)]
    encs = [gc.encode(_dev(b), _P(gc, op), index_stride=0 if fixed else _enc_stride(stride)) for b in buckets]
    sw = max((e.bits + 63) // 64 for e in encs) + (0 if fixed else 1)
    streams = torch.zeros(world * sw + 2, dtype=torch.int64, device="cuda")
    for r, e in enumerate(encs):
        streams[r * sw:r * sw + e.nwords] = e.stream()
    idx, ni, st = None, 0, 0
    if not fixed:
        idx, ni, st = _mean_index(gc, encs, stride, n, _P(gc, op))
    base = torch.full((2 * n,), -1.0, dtype=torch.bfloat16, device="cuda")
    out = base[:n] if layout == "contiguous" else base[::2]
    got = gc.decode_mean(streams, sw, world, n, _P(gc, op), idx, ni, st, out=out)
    want = _bf16_rne(_oracle_mean(orc, [orc.compress(b, op)[0] for b in buckets], op, n))
    torch.cuda.synchronize()
    assert got.data_ptr() == out.data_ptr()
    assert np.array_equal(got.cpu().view(torch.int16).numpy().view(np.uint16), want)
    untouched = base[n:] if layout == "contiguous" else base[1::2]
    assert bool((untouched == -1.0).all())


@pytest.mark.parametrize("out_dtype", ["f32", "bf16"])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("stride", [16, 8, "packed"])
def test_decode_mean_stage_parts(gc, orc, world, out_dtype, stride):
    """k_decode_mean1d_var_lean stages each stream's span of a workgroup (128 chunks of 16 blocks) in 1, 2 or 4 parts
    (a stage of 64 bits per block). Ranks hold data of very different magnitudes at accuracy 1e-6: N(0, 1e4) codes
    ~137 bits per block (every group in 4 parts), N(0, 1) ~100 (2 parts), N(0, 1e-3) ~64 (1 part, or 2); inside rank 0 the
    groups alternate between the first two. nchunks is a whole number of workgroups, so the last group's span runs to
    stream_words, far past the shorter ranks' streams. Bit-exact vs the oracle mean, fp32 and bf16 out."""
    wg = 128 * _enc_stride(stride) * 4  # values per workgroup (128 chunks of `stride` blocks)
    n = wg * 7
    rng = np.random.default_rng(31337 + world)
    scales = [1e4, 1.0, 1e-3]
    buckets = []
    for r in range(world):
        a = rng.standard_normal(n).astype(np.float32) * np.float32(scales[r])
        if r == 0:
            for g in range(1, 7, 2):
                a[g * wg:(g + 1) * wg] *= np.float32(1e-4)  # groups at ~N(0, 1): 2 parts
        buckets.append(a)
    op = orc.accuracy(1e-6)
    p = _P(gc, op)
    encs = [gc.encode(_dev(b), p, index_stride=_enc_stride(stride)) for b in buckets]
    lens = [e.bits for e in encs]
    bpb = [b / (n // 4) for b in lens]
    assert bpb[0] > 100 and (world < 2 or 80 < bpb[1] < 128) and (world < 3 or bpb[2] < 72), bpb
    sw = max((b + 63) // 64 for b in lens) + 1
    streams = torch.zeros(world * sw + 2, dtype=torch.int64, device="cuda")
    for r, e in enumerate(encs):
        streams[r * sw:r * sw + e.nwords] = e.stream()
    idx, ni, st = _mean_index(gc, encs, stride, n, p)
    want = _oracle_mean(orc, [orc.compress(b, op)[0] for b in buckets], op, n)
    if out_dtype == "f32":
        got = gc.decode_mean(streams, sw, world, n, p, idx, ni, st)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32))
    else:
        out = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        gc.decode_mean(streams, sw, world, n, p, idx, ni, st, out=out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().view(torch.int16).numpy().view(np.uint16), _bf16_rne(want))


@pytest.mark.parametrize("mode", ["rate16", "acc1e-6"])
def test_decode_mean_full_size_w8(gc, orc, mode):
    """The hook's receive side at the bench's size: 8 streams of 256 Mi fp32 values (8 different buckets, the bench's
    fill_normal with seeds 0x67636F77 + r) decoded and averaged in one launch == the threaded oracle decodes summed
    in rank order in fp32, divided by 8, over the whole bucket. Variable rate with the all-gather hook's packed
    16-block index (8-block chunks)."""
    W, n = 8, 256 * 1024 * 1024
    T = min(16, os.cpu_count() or 1)
    op = orc.rate(16, 1) if mode == "rate16" else orc.accuracy(1e-6)
    fixed = op.minbits == op.maxbits
    p = _P(gc, op)
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    enc = gc.Encoder((n,), torch.float32, p, index_stride=0 if fixed else 8)
    acc = np.zeros(n, np.float32)
    parts, idx = [], []
    for r in range(W):
        gc.fill_normal(x, 1e-3, seed=0x67636F77 + r, inject=True)
        e = enc(x)
        parts.append(e.stream().clone())
        if not fixed:  # the all-gather hook's index: every 8 blocks, sent packed into the 16-block entries
            idx.append(gc.pack_index16(e.index, n, p).clone())
        w_ref, bits, offs = orc.compress(x.cpu().numpy(), op, threads=T, offsets=True)
        assert e.bits == bits
        acc = acc + orc.decompress(w_ref, (n,), op, threads=T, offsets=None if fixed else offs)
        del w_ref
    want = acc / np.float32(W)
    del acc
    sw = max(s.numel() for s in parts)
    streams = torch.zeros(W * sw + 2, dtype=torch.int64, device="cuda")
    for r, s in enumerate(parts):
        streams[r * sw:r * sw + s.numel()] = s
    ni = idx[0].numel() if idx else 0
    got = gc.decode_mean(streams, sw, W, n, p, torch.cat(idx) if idx else None, ni, 0 if fixed else gc.INDEX_PACKED16,
                         out=x)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("nblocks", [1, 7, 8, 9, 16, 17, 24, 4096 + 9])
def test_pack_index16(gc, orc, nblocks):
    """gcow_index_pack16_device: entry c = idx8[2c] | (idx8[2c+1] - idx8[2c]) << 48, the offset 0 where block 16c + 8
    does not exist; parameters that let 8 blocks pass 65535 bits, and 2-D fields, are refused."""
    n = 4 * nblocks - 1
    p = gc.accuracy(1e-6)
    e = gc.encode(_dev(_bucket(orc, n, 11)), p, index_stride=8)
    pk = gc.pack_index16(e.index, n, p).cpu().numpy().view(np.uint64)
    i8 = e.index.cpu().numpy().view(np.uint64)[: (nblocks + 7) // 8]
    a = i8[0::2]
    d = np.zeros_like(a)
    d[: i8[1::2].size] = i8[1::2] - a[: i8[1::2].size]
    torch.cuda.synchronize()
    assert pk.size == (nblocks + 15) // 16 and np.array_equal(pk, a | (d << np.uint64(48)))
    with pytest.raises(gc.GcowError):
        gc.pack_index16(e.index, n, gc.expert(8192, 16658, 64, -1074))
    f2 = gc.field_of_shape((4, nblocks), torch.float32)
    with pytest.raises(gc.GcowError):
        gc.check(gc.load().gcow_index_pack16_device(gc.C.byref(f2), gc.C.byref(p), e.index.data_ptr(),
                                                    e.index.data_ptr(), None), "pack")


def test_decode_mean_argument_checks(gc, orc):
    """The C entry validates what its kernels assume: 2 readable words past the last stream, and no block index on
    the fixed-rate path."""
    n = 4 * 1000
    p = gc.rate(16, 1)
    e = gc.encode(_dev(_bucket(orc, n, 3)), p)
    sw = e.nwords
    with pytest.raises(gc.GcowError):
        gc.decode_mean(e.words[:sw].contiguous(), sw, 1, n, p)  # no padding words
    buf = torch.zeros(sw + 2, dtype=torch.int64, device="cuda")
    buf[:sw] = e.stream()
    with pytest.raises(gc.GcowError):
        gc.decode_mean(buf, sw, 1, n, p, buf, 1, 16)  # an index on a fixed-rate stream
    got = gc.decode_mean(buf, sw, 1, n, p)
    torch.cuda.synchronize()
    ref = orc.decompress(orc.compress(_bucket(orc, n, 3), orc.rate(16, 1))[0], (n,), orc.rate(16, 1))
    assert np.array_equal(got.cpu().numpy().view(np.uint32), ref.view(np.uint32))


# ---------------------------------------------------------------------------------------------- multi-process
class HostStagedDeviceCodec:
    """gcow_amd.dist.DeviceCodec behind host copies: the exchange code moves CPU tensors over gloo (two processes
    cannot share one GPU over RCCL), every codec call runs the device kernels."""

    def __init__(self):
        from gcow_amd.dist import DeviceCodec
        self.d = DeviceCodec()
        self.calls = []

    def encode(self, x, params, index_stride=0, slot=None):
        w, b, i = self.d.encode(x.cuda(), params, index_stride, slot=slot)
        self.calls.append("encode")
        return w.cpu(), b.cpu(), (i.cpu() if i is not None else None)

    def stitch_shards(self, dst, src, shard_words, lens, nshards):
        dd = dst.cuda()
        self.d.stitch_shards(dd, src.cuda(), shard_words, lens.cuda(), nshards)
        dst.copy_(dd.cpu())
        self.calls.append("stitch")
        return dst

    def decode(self, words, n, params, index=None, index_stride=0, out=None):
        o = self.d.decode(words.cuda(), n, params, index.cuda() if index is not None else None, index_stride).cpu()
        return out.copy_(o) if out is not None else o

    def pack_index16(self, index8, n, params):
        return self.d.pack_index16(index8.cuda(), n, params).cpu()

    def decode_mean(self, streams, stream_words, nstreams, n, params, index=None, index_words=0, index_stride=0,
                    out=None):
        o = self.d.decode_mean(streams.cuda(), stream_words, nstreams, n, params,
                               index.cuda() if index is not None else None, index_words, index_stride).cpu()
        self.calls.append("decode_mean")
        return out.copy_(o) if out is not None else o


def _mp_worker(rank, world, port, q, what, mode):
    import torch.distributed as dist
    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)  # a file:// rendezvous
    try:
        from gcow_amd import codec, ddp
        from gcow_amd import dist as gdist
        from oracle import oracle as O
        p = {"rate16": codec.rate(16, 1), "acc1e-6": codec.accuracy(1e-6), "bf16_acc1e-3": codec.accuracy(1e-3)}[mode]
        op = O.expert(*p.tuple())
        cdc = HostStagedDeviceCodec()
        if what.startswith("encode_allgather"):
            # "_equal": 8 x 6400 values, equal 16-block-aligned shards at world 8 (the C4 layout: one all-gather of the
            # shard streams is the stream); otherwise ragged shards and a partial last block (stitched)
            a = O.gen_normal(8 * 6400 if what.endswith("_equal") else 4 * 30011 + 1, 1e-3, 5, True)
            if mode.startswith("bf16"):
                a = (a.view(np.uint32) >> 16).astype(np.uint16)
                bucket = torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
            else:
                bucket = torch.from_numpy(a.copy())
            out, total = gdist.encode_allgather(bucket, p, codec=cdc)
            ref, bits = O.compress(a, op)
            ok = total == bits and out.numpy().view(np.uint64).tobytes() == ref.tobytes()
        else:
            import torch.nn as nn
            torch.manual_seed(0)
            # 4087 values = 1022 blocks (world 8: seven 128-block shards and a ragged one ending in a partial block);
            # "_small": 600 values = 150 blocks, so at world 8 ranks 3..7 own empty shards
            fi, fo = (20, 30) if what.endswith("_small") else (67, 61)
            model = nn.Linear(fi, fo, bias=False)
            refm = nn.Linear(fi, fo, bias=False)
            refm.load_state_dict(model.state_dict())
            dm = nn.parallel.DistributedDataParallel(model)
            hook = ddp.compressed_sharded_hook if what.startswith("sharded_hook") else ddp.compressed_allgather_hook
            dm.register_comm_hook(ddp.make_hook_state(hook=hook, params=p, codec=cdc), hook)
            torch.manual_seed(10 + rank)
            x = torch.randn(8, fi)
            dm(x).square().mean().backward()
            refm(x).square().mean().backward()
            g = refm.weight.grad.reshape(-1).contiguous()
            allg = [torch.empty_like(g) for _ in range(world)]
            dist.all_gather(allg, g)
            acc = np.zeros(g.numel(), np.float32)
            for t in allg:
                acc = acc + O.decompress(O.compress(t.numpy(), op)[0], (g.numel(),), op)
            want = acc / np.float32(world)
            got = dm.module.weight.grad.reshape(-1).numpy()
            # every rank decodes on the device -- except, in the sharded hook, a rank whose shard is empty
            lo, hi = gdist.shard_plan(g.numel(), world)[0][rank]
            decodes = not (what.startswith("sharded_hook") and hi == lo)
            ok = np.array_equal(got.view(np.uint32), want.view(np.uint32)) and ("decode_mean" in cdc.calls) == decodes
        q.put((rank, True if ok else "mismatch"))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("what,mode", [("encode_allgather", "rate16"), ("encode_allgather", "acc1e-6"),
                                       ("encode_allgather", "bf16_acc1e-3"), ("hook", "rate16"), ("hook", "acc1e-6"),
                                       ("sharded_hook", "rate16"), ("sharded_hook", "acc1e-6")])
@pytest.mark.parametrize("world", [2, 3])
def test_exchange_multiprocess_device_codec(gc, what, mode, world):
    _run_mp(what, mode, world)


@pytest.mark.parametrize("what,mode", [("encode_allgather_equal", "rate16"), ("encode_allgather", "rate16"),
                                       ("encode_allgather", "bf16_acc1e-3"), ("sharded_hook", "acc1e-6"), ("sharded_hook_small", "acc1e-6"),
                                       ("sharded_hook_small", "rate16"), ("hook", "acc1e-6")])
def test_exchange_multiprocess_device_codec_world8(gc, what, mode):
    """The C4 / C5-8-GPU exchange shape: 8 processes sharing the one GPU, every codec call on the gfx950
    kernels, the collectives over gloo. encode_allgather at rate 16 (equal 16-block-aligned shards: one all-gather;
    ragged shards: stitched) and bf16 accuracy 1e-3 (length exchange, padded all-gather, one-launch stitch) must equal the
    oracle's single-stream encode; the sharded hook at accuracy 1e-6 with a ragged last shard, and with ranks 3..7
    owning empty shards, must give every rank the oracle's mean of decode(encode(g_r)) bit for bit."""
    _run_mp(what, mode, 8, timeout=300)


def _run_mp(what, mode, world, timeout=100):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:  # a file rendezvous: no port to race other jobs on the box for
        init = "file://" + os.path.join(d, "rdv")
        procs = [ctx.Process(target=_mp_worker, args=(r, world, init, q, what, mode)) for r in range(world)]
        for pr in procs:
            pr.start()
        try:
            res = [q.get(timeout=timeout) for _ in procs]
        finally:
            for pr in procs:
                pr.join(timeout=60)
                if pr.is_alive():
                    pr.kill()
    assert all(ok is True for _, ok in res), res


# ---------------------------------------------------------------------------------------------- DDP hooks, RCCL
@pytest.fixture
def nccl_world1():
    import torch.distributed as dist
    # an in-process store: no port to race another job on the box for (a free port picked, closed and bound again
    # was once taken in between: EADDRINUSE)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("hook", ["roundtrip_hook", "compressed_allgather_hook", "compressed_sharded_hook"])
@pytest.mark.parametrize("mode", ["rate16", "acc1e-6", "rate8", "expert_var_minbits", "expert_var_trunc"])
def test_ddp_hooks_world1_bit_exact(gc, orc, nccl_world1, hook, mode):
    """One rank over RCCL: every weight gradient equals the oracle's decode(encode(local grad)) -- (0 + x) / 1 for the
    all-gather hook -- bit for bit. Three equal-size layers give three buckets of one shape in
    flight at once (the asynchronous hook must not let a later bucket's encode overwrite an earlier stream), and two
    training steps reuse every buffer."""
    from gcow_amd import ddp
    params = {"rate16": gc.rate(16, 1), "acc1e-6": gc.accuracy(1e-6), "rate8": gc.rate(8, 1),
              "expert_var_minbits": gc.expert(8, 512, 32, -1074), "expert_var_trunc": gc.expert(1, 100, 64, -30)}[mode]
    torch.manual_seed(0)
    # 640 x 640 fp32 weights (1.6 MB) each fill a bucket of their own past DDP's 1 MiB first-bucket cap
    layers = lambda: torch.nn.Sequential(*[torch.nn.Linear(640, 640, bias=False) for _ in range(3)]).cuda()  # noqa
    model, ref = layers(), layers()
    ref.load_state_dict(model.state_dict())
    dm = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], bucket_cap_mb=1)
    seen = []

    def counted(state, bucket):
        seen.append(bucket.index())
        return getattr(ddp, hook)(state, bucket)

    dm.register_comm_hook(ddp.make_hook_state(params=params), counted)
    op = orc.expert(*params.tuple())
    for step in range(2):
        model.zero_grad()
        ref.zero_grad()
        x = torch.randn(32, 640, device="cuda")
        dm(x).square().mean().backward()
        ref(x).square().mean().backward()
        for lm, lr in zip(model, ref):
            g = lr.weight.grad.reshape(-1).cpu().numpy()
            dec = orc.decompress(orc.compress(g, op)[0], g.shape, op)
            want = (np.zeros_like(dec) + dec) / np.float32(1) if hook != "roundtrip_hook" else dec
            got = lm.weight.grad.reshape(-1).cpu().numpy()
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), step
    assert len(set(seen)) >= 2, seen  # several buckets per step


@pytest.mark.parametrize("hook", ["roundtrip_hook", "compressed_allgather_hook", "compressed_sharded_hook"])
@pytest.mark.parametrize("mode", ["rate16", "acc1e-6"])
def test_ddp_allgather_hook_bf16_world1(gc, orc, nccl_world1, mode, hook):
    """bf16 model over RCCL: both hooks decode straight into the bf16 bucket; every weight gradient equals the
    oracle's decode of its (exactly widened) bf16 gradient (divided by 1 for the all-gather hook), rounded to nearest
    even, bit for bit, over two steps and several buckets."""
    from gcow_amd import ddp
    params = gc.rate(16, 1) if mode == "rate16" else gc.accuracy(1e-6)
    torch.manual_seed(0)
    layers = lambda: torch.nn.Sequential(  # noqa: E731
        *[torch.nn.Linear(768, 768, bias=False) for _ in range(3)]).cuda().to(torch.bfloat16)
    model, ref = layers(), layers()
    ref.load_state_dict(model.state_dict())
    dm = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], bucket_cap_mb=1)
    dm.register_comm_hook(ddp.make_hook_state(hook=getattr(ddp, hook), params=params), getattr(ddp, hook))
    op = orc.expert(*params.tuple())
    for step in range(2):
        model.zero_grad()
        ref.zero_grad()
        x = torch.randn(32, 768, device="cuda", dtype=torch.bfloat16)
        dm(x).float().square().mean().backward()
        ref(x).float().square().mean().backward()
        for lm, lr in zip(model, ref):
            gb = lr.weight.grad.reshape(-1).view(torch.int16).cpu().numpy().view(np.uint16)
            dec = orc.decompress(orc.compress(gb, op)[0], gb.shape, op)
            want = _bf16_rne((np.zeros_like(dec) + dec) / np.float32(1) if hook != "roundtrip_hook" else dec)
            got = lm.weight.grad.reshape(-1).view(torch.int16).cpu().numpy().view(np.uint16)
            assert np.array_equal(got, want), step


def test_allgather_hook_delayed_decode_stream(gc, orc, nccl_world1):
    """the fixed-rate hook's decode runs in a Future.then callback on a pool stream; the gathered
    buffer must stay out of the allocator until that decode has read it. Six equal-size buckets (each a same-size
    `gathered` request right after the previous bucket's callback returned), and every decode delayed behind a long
    spin on its stream: every gradient still equals the oracle's decode(encode(local grad)) bit for bit."""
    from gcow_amd import ddp
    from gcow_amd.dist import DeviceCodec

    class Delayed(DeviceCodec):
        def decode_mean(self, *a, **k):
            torch.cuda._sleep(20_000_000)  # ~10 ms of spinning on the decode's stream before the decode
            return super().decode_mean(*a, **k)

    params = gc.rate(16, 1)
    torch.manual_seed(1)
    layers = lambda: torch.nn.Sequential(*[torch.nn.Linear(640, 640, bias=False) for _ in range(6)]).cuda()  # noqa
    model, ref = layers(), layers()
    ref.load_state_dict(model.state_dict())
    dm = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], bucket_cap_mb=1)
    dm.register_comm_hook(ddp.make_hook_state(params=params, codec=Delayed()), ddp.compressed_allgather_hook)
    op = orc.expert(*params.tuple())
    for step in range(2):
        model.zero_grad()
        ref.zero_grad()
        x = torch.randn(32, 640, device="cuda")
        dm(x).square().mean().backward()
        ref(x).square().mean().backward()
        for lm, lr in zip(model, ref):
            g = lr.weight.grad.reshape(-1).cpu().numpy()
            want = np.zeros(g.size, np.float32) + orc.decompress(orc.compress(g, op)[0], g.shape, op)
            got = lm.weight.grad.reshape(-1).cpu().numpy()
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), step


# ---------------------------------------------------------------------------------------------- bench N > 1 legs
def test_bench_multi_legs_world1(gc):
    """bench.py's multi-GPU legs (C4 exchange with the oracle check of the gathered stream, the sub-communicator
    curve, strong scaling, C5 sharded with the stitch checked against the oracle, the hook exchange in both forms)
    run on the GPU over a one-rank RCCL
    group (--multi-legs), small sizes: the code the driver's 8-GPU run executes, exercised on a one-GPU box."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--multi-legs", "--steps", "3", "--warmup", "1",
           "--values", str(1 << 22), "--strong-gib", "0.0625", "--c5-values", str(1 << 22), "--no-cpu-baseline"]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1
    assert d["encode_allgather"]["gathered_stream_matches_oracle"] is True
    assert d["c5_sharded"]["stitched_stream_matches_oracle"] is True
    assert [c["k"] for c in d["subgroups"]] == [1] and [c["k"] for c in d["strong"]["curve"]] == [1]
    for mode in ("rate16", "acc1e-6"):  # the DDP hook's exchange: all-gather form vs sharded receive
        h = d["hook_exchange"][mode]
        assert h["sharded_equals_allgather"] is True and h["sharded_mean_matches_oracle"] is True, h
