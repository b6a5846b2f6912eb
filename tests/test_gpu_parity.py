"""GPU parity: the HIP codec (through the C ABI) against the pinned oracle and fixtures. Bit-exact everywhere.

Sizes: fixtures/goldens as the reference holds them; random cases the oracle finishes in well under a second; the
BASELINE configs at full size (256 Mi fp32 1-D fixed rate, 512^3 3-D round trip) against the threaded oracle.
"""
import ctypes as C
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def gc():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a device")
    from gcow_amd import codec
    return codec


def P(gc, orc_params):
    return gc.expert(*orc_params.tuple())


def dev_encode_bytes(gc, arr, params, index_stride=0):
    x = torch.from_numpy(np.ascontiguousarray(arr)).cuda()
    if arr.dtype == np.uint16:
        x = x.view(torch.bfloat16)
    e = gc.encode(x, params, index_stride=index_stride)
    torch.cuda.synchronize()
    return e, e.to_bytes()


# ---------------------------------------------------------------------------------------------- reference goldens
GOLDENS = json.load(open(os.path.join(GOLD, "reference_goldens.json")))["goldens"]


@pytest.mark.parametrize("g", GOLDENS, ids=lambda g: g["file"])
def test_reference_goldens_device(gc, orc, g):
    a = orc.gen_bump2d(g["n"], g["recipe"] == "bump_f32sum")
    _, b = dev_encode_bytes(gc, a, gc.accuracy(g["tolerance"]))
    assert len(b) == g["bytes"]
    assert _sha(b) == g["sha256"]


# ---------------------------------------------------------------------------------------------- libzfp fixtures
FX = json.load(open(os.path.join(GOLD, "libzfp_fixtures.json")))["cases"]


@pytest.fixture(scope="module")
def fxa():
    return np.load(os.path.join(GOLD, "libzfp_fixtures.npz"))


@pytest.mark.parametrize("c", FX, ids=lambda c: c["name"])
def test_libzfp_fixture_device(gc, fxa, c):
    a = fxa["input__" + c["input"]]
    p = gc.expert(*c["params"])
    stride = 4 if len(a.shape) < 3 else 1
    e, b = dev_encode_bytes(gc, a, p, index_stride=0 if gc.is_fixed(p) else stride)
    assert len(b) == c["bytes"]
    assert _sha(b) == c["stream_sha256"]
    d = gc.decode(e)
    torch.cuda.synchronize()
    assert _sha(d.cpu().numpy().tobytes()) == c["decoded_sha256"]


@pytest.mark.parametrize("c", [c for c in FX if c["mode"] in ("acc", "prec", "expert")][::7], ids=lambda c: c["name"])
def test_sequential_decode_without_index(gc, fxa, c):
    """A foreign variable-rate stream (no block index) decodes on one sequential GPU lane."""
    a = fxa["input__" + c["input"]]
    p = gc.expert(*c["params"])
    words = torch.from_numpy(fxa[c["name"] + "__stream"].view(np.int64).copy()).cuda()
    words = torch.cat([words, torch.zeros(2, dtype=torch.int64, device="cuda")])
    d = gc.decode(words, a.shape, p)
    torch.cuda.synchronize()
    assert _sha(d.cpu().numpy().tobytes()) == c["decoded_sha256"]


# ---------------------------------------------------------------------------------------------- random vs oracle
def _check_vs_oracle(gc, orc, a, op, index_stride=0, decode=True):
    w_ref, bits_ref = orc.compress(a, op)
    e, b = dev_encode_bytes(gc, a, P(gc, op), index_stride)
    assert e.bits == bits_ref
    assert b == w_ref.tobytes()
    if decode:
        ref = orc.decompress(w_ref, a.shape, op)
        d = gc.decode(e)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 255, 1023, 4097, (1 << 18) + 3])
@pytest.mark.parametrize("r", [16, 8])
def test_fast1d_fixed_rate(gc, orc, n, r):
    a = orc.gen_normal(n, 1e-3, 0x1234 + n, True)
    _check_vs_oracle(gc, orc, a, orc.rate(r, 1))


def _bf16_rne(a):
    u = a.view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


BF16_OUT_MODES = {"rate16": ("rate", 16), "rate8": ("rate", 8), "rate12": ("rate", 12), "acc1e-6": ("acc", 1e-6),
                  "acc1e-3": ("acc", 1e-3), "expert_trunc": ("expert", (1, 100, 64, -30))}


@pytest.mark.parametrize("mode", list(BF16_OUT_MODES))
@pytest.mark.parametrize("layout", ["contiguous", "strided"])
@pytest.mark.parametrize("n", [4 * 128 * 16 * 3 + 4 * 37 + 3, 4 * 20001])
def test_decode_1d_bf16_output(gc, orc, mode, layout, n):
    """1-D decode into a bf16 tensor: the oracle's fp32 decode rounded to nearest even, bit for bit -- the fixed-rate
    one-shot decoders (64- and 32-bit blocks), the lean variable-rate decoder (whole workgroups) with its general path
    (the partial chunk), the generic decoder, the partial last block, and a strided output (value stores)."""
    kind, v = BF16_OUT_MODES[mode]
    op = orc.rate(v, 1) if kind == "rate" else orc.accuracy(v) if kind == "acc" else orc.expert(*v)
    a = orc.gen_normal(n, 1e-3, 0xB16 + n, True)
    fixed = op.minbits == op.maxbits
    e, _ = dev_encode_bytes(gc, a, P(gc, op), 0 if fixed else 16)
    base = torch.full((2 * n,), -1.0, dtype=torch.bfloat16, device="cuda")
    out = base[:n] if layout == "contiguous" else base[::2]
    got = gc.decode(e, out=out)
    want = _bf16_rne(orc.decompress(orc.compress(a, op)[0], a.shape, op))
    torch.cuda.synchronize()
    assert got.data_ptr() == out.data_ptr()
    assert np.array_equal(got.cpu().view(torch.int16).numpy().view(np.uint16), want)
    untouched = base[n:] if layout == "contiguous" else base[1::2]
    assert bool((untouched == -1.0).all())


@pytest.mark.parametrize("tol", [2e-7, 1e-8, 1e-12])
@pytest.mark.parametrize("out_dtype", ["f32", "bf16"])
def test_var1d_decode_past_the_stage(gc, orc, tol, out_dtype):
    """1-D variable-rate streams coding more than the lean decoder's 64-bit-per-block stage (75-140 bits per block):
    the main kernel leaves those groups to the second pass (a stage that holds any span); whole groups, a partial last
    group and a partial last block, bit for bit against the oracle."""
    n = 4 * 16 * 128 * 5 + 4 * 16 * 37 + 4 * 5 + 2
    op = orc.accuracy(tol)
    a = orc.gen_normal(n, 1e-3, 0x51A6E, True)
    e, _ = dev_encode_bytes(gc, a, P(gc, op), 16)
    assert e.bits / ((n + 3) // 4) > 64
    ref = orc.decompress(orc.compress(a, op)[0], a.shape, op)
    if out_dtype == "f32":
        got = gc.decode(e)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    else:
        got = gc.decode(e, out=torch.empty(n, dtype=torch.bfloat16, device="cuda"))
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().view(torch.int16).numpy().view(np.uint16), _bf16_rne(ref))


@pytest.mark.parametrize("tol,mix", [(1e-2, False), (1e-3, False), (1e-3, True), (3e-4, False), (1e-4, False),
                                     (1e-4, True), (1e-6, True)])
def test_var1d_decode_exact_stream_buffer(gc, orc, tol, mix):
    """The lean variable-rate decoder given the stream in a buffer of its own size (e.stream(), not the encoder's
    capacity-sized one): launch_decode1d_var then sizes the main kernel's stage by the average bits per block (32, 48
    or 64), and groups past it take the second pass (mix: a quiet half and a loud half, so the average picks a small
    stage that the loud groups overflow). Bit for bit against the oracle, whole and partial groups."""
    n = 4 * 16 * 128 * 9 + 4 * 16 * 37 + 4 * 5 + 2
    a = orc.gen_normal(n, 1e-3, 0xE5AC7 + int(-np.log10(tol)), True)
    if mix:
        a[: n // 2] *= np.float32(1e-3)
        a[n // 2 + n // 8: n // 2 + n // 4] *= np.float32(30.0)
    op = orc.accuracy(tol)
    e, _ = dev_encode_bytes(gc, a, P(gc, op), 16)
    ref = orc.decompress(orc.compress(a, op)[0], a.shape, op)
    words = e.stream()
    got = gc.decode(words, e.shape, e.params, e.index, e.index_stride)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint32), ref.view(np.uint32)), e.bits / ((n + 3) // 4)


@pytest.mark.parametrize("tol,mix", [(1e-1, False), (1e-2, False), (1e-3, False), (1e-3, True), (1e-4, True),
                                     (1e-6, False), (1e-6, True), (1e-9, False)])
def test_var1d_decode_capacity_buffer_tiers(gc, orc, tol, mix):
    """The same streams decoded from the encoder's capacity-sized buffer (what a hook holds): the buffer's size says
    nothing about the stream, so launch_decode1d_var launches the 32 / 48 / 64-bit stage tiers gated on the stream's
    average from its own index (vdec_tier) and the second pass takes the chosen tier's overflow. Bit for bit against
    the oracle, sparse (1e-1: ~10 bits per block) to dense (1e-9: past every stage)."""
    n = 4 * 16 * 128 * 9 + 4 * 16 * 37 + 4 * 5 + 2
    a = orc.gen_normal(n, 1e-3, 0xCA9AC + int(-np.log10(tol)), True)
    if mix:
        a[: n // 2] *= np.float32(1e-3)
        a[n // 2 + n // 8: n // 2 + n // 4] *= np.float32(30.0)
    op = orc.accuracy(tol)
    e, _ = dev_encode_bytes(gc, a, P(gc, op), 16)
    assert e.words.numel() * 64 >= 128 * ((n + 3) // 4)  # the capacity buffer: the tiered launch
    ref = orc.decompress(orc.compress(a, op)[0], a.shape, op)
    got = gc.decode(e)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint32), ref.view(np.uint32)), e.bits / ((n + 3) // 4)


def test_decode_bf16_output_needs_1d(gc, orc):
    a = orc.gen_normal(16 * 16, 1e-3, 5, False).reshape(16, 16)
    e, _ = dev_encode_bytes(gc, a, gc.rate(16, 2))
    with pytest.raises(gc.GcowError):
        gc.decode(e, out=torch.empty((16, 16), dtype=torch.bfloat16, device="cuda"))


@pytest.mark.parametrize("r", [4, 2.5, 32, 12])
def test_1d_other_rates(gc, orc, r):
    a = orc.gen_normal(10007, 1e-3, 99, True)
    _check_vs_oracle(gc, orc, a, orc.rate(r, 1))


@pytest.mark.parametrize("shape", [(1000,), (4096 * 3 + 1,), (37, 53), (64, 64), (9, 10, 7), (16, 20, 24)])
@pytest.mark.parametrize("mode", ["acc3", "acc6", "prec12", "prec32", "rate8", "expert"])
def test_random_all_dims(gc, orc, shape, mode):
    rng = np.random.default_rng(zlib.crc32(repr((shape, mode)).encode()))
    a = (rng.standard_normal(shape) * 1e-2).astype(np.float32)
    flat = a.reshape(-1)
    flat[:: 97] = 0
    flat[5:9] = [1e-36, -2e-38, 7e-39, 0]  # tiny and subnormal members
    op = {"acc3": orc.accuracy(1e-3), "acc6": orc.accuracy(1e-6), "prec12": orc.precision(12),
          "prec32": orc.precision(32), "rate8": orc.rate(8, len(shape)), "expert": orc.expert(20, 160, 20, -30)}[mode]
    _check_vs_oracle(gc, orc, a, op, index_stride=0 if op.minbits == op.maxbits else 2)


@pytest.mark.parametrize("mode", ["prec32", "acc1e-30"])
def test_3d_var_oversized_tiles(gc, orc, mode):
    """3-D variable rate where some 64-block tiles exceed the LDS window (k_encode3d_var codes those straight into
    global memory) next to tiles that fit: zero slabs between near-lossless noise, so fitting and oversized tiles
    share edge words both ways."""
    rng = np.random.default_rng(31 if mode == "prec32" else 32)
    a = (rng.standard_normal((24, 40, 64)) * 1e-2).astype(np.float32)
    a[4:12] = 0
    a[16:20, :, :32] = 0
    op = orc.precision(32) if mode == "prec32" else orc.accuracy(1e-30)
    _check_vs_oracle(gc, orc, a, op, index_stride=1)


@pytest.mark.parametrize("shape", [(260, 256, 256), (4, 1024, 4100)])
def test_3d_var_many_tiles(gc, orc, shape):
    """More than 4096 tiles: the range scan runs as many workgroups (k_scan_ranges_mw), each summing the totals of
    the ranges before it; the tile count is not a multiple of the workgroup's 1024 ranges."""
    rng = np.random.default_rng(33)
    a = (rng.standard_normal(shape) * 1e-2).astype(np.float32)
    a[:, :, : shape[2] // 3] *= 1e-3
    _check_vs_oracle(gc, orc, a, orc.accuracy(1e-3), index_stride=1)


def test_subnormal_cast_members(gc, orc):
    """Blocks with emax in [-97, -90] whose members are subnormal: the cast must not flush them."""
    rng = np.random.default_rng(5)
    blocks = []
    for e in range(-97, -89):
        for _ in range(64):
            v = rng.standard_normal(4) * (2.0 ** e)
            v[rng.integers(0, 4)] = rng.standard_normal() * 2.0 ** -127
            v[rng.integers(0, 4)] = 2.0 ** -149 * rng.integers(1, 100)
            blocks.append(v)
    a = np.array(blocks, np.float32).reshape(-1)
    for op in (orc.rate(16, 1), orc.accuracy(1e-40), orc.precision(32)):
        _check_vs_oracle(gc, orc, a, op, index_stride=0 if op.minbits == op.maxbits else 1)


@pytest.mark.parametrize("tol", [1e-40, 1e-42, 1e-38, 1e-45, 3e-37])
def test_var1d_subnormal_maxima(gc, orc, tol):
    """1-D variable-rate blocks whose largest member is subnormal (biased exponent 0: emax clamps to -126, not -125)
    at tolerances that put minexp in [-154, -122], where the block's precision -- and so where every later block
    starts -- depends on that clamp; interleaved with normal and zero blocks. Stream, index and decode vs the oracle."""
    rng = np.random.default_rng(int(-np.log10(tol) * 10))
    nb = 3000
    sub = rng.integers(-(2 ** 23) + 1, 2 ** 23, (nb, 4)).astype(np.float64) * 2.0 ** -149  # all members subnormal
    small = rng.integers(-(2 ** 8), 2 ** 8, (nb, 4)).astype(np.float64) * 2.0 ** -149
    norm = rng.standard_normal((nb, 4)) * 2.0 ** rng.integers(-126, -100, (nb, 1))
    kind = rng.integers(0, 4, nb)
    a = np.where(kind[:, None] == 0, sub, np.where(kind[:, None] == 1, small,
                                                   np.where(kind[:, None] == 2, norm, 0.0)))
    a = a.astype(np.float32).reshape(-1)[:-1]  # partial last block
    op = orc.accuracy(tol)
    assert -154 <= op.minexp <= -122
    _check_vs_oracle(gc, orc, a, op, index_stride=16)


@pytest.mark.parametrize("mode", ["rate16", "rate8", "acc6", "acc3"])
def test_bf16(gc, orc, mode):
    f = orc.gen_normal(50001, 1e-3, 7, True)
    bf = (f.view(np.uint32) >> 16).astype(np.uint16)  # truncation is as good as any bf16 input
    op = {"rate16": orc.rate(16, 1), "rate8": orc.rate(8, 1), "acc6": orc.accuracy(1e-6),
          "acc3": orc.accuracy(1e-3)}[mode]
    _check_vs_oracle(gc, orc, bf, op, index_stride=0 if op.minbits == op.maxbits else 8, decode=False)


def test_strided_views(gc, orc):
    rng = np.random.default_rng(3)
    base = (rng.standard_normal((40, 66)) * 1e-3).astype(np.float32)
    x = torch.from_numpy(base).cuda()
    for view, ref in [(x.t(), base.T), (x[:, ::2], base[:, ::2]), (x[3:35, 5:60], base[3:35, 5:60]),
                      (x.reshape(-1)[1::3], base.reshape(-1)[1::3])]:
        for op in (orc.accuracy(1e-4), orc.rate(8, len(ref.shape))):
            w_ref, bits = orc.compress(np.ascontiguousarray(ref), op)
            e = gc.encode(view, P(gc, op))
            torch.cuda.synchronize()
            assert e.bits == bits and e.to_bytes() == w_ref.tobytes()


def test_empty_and_tiny(gc, orc):
    for n in (1, 2, 3):
        a = np.array([1.5, -2.0, 3.25][:n], np.float32)
        _check_vs_oracle(gc, orc, a, orc.accuracy(1e-3))
        _check_vs_oracle(gc, orc, a, orc.rate(16, 1))


# ---------------------------------------------------------------------------------------------- stitch (multi-GPU)
@pytest.mark.parametrize("k", [2, 3, 8])
def test_stitch_equals_single_stream(gc, orc, k):
    a = orc.gen_normal(4 * 10001, 1e-3, 11, True)
    op = orc.accuracy(1e-6)
    w_ref, bits_ref = orc.compress(a, op)
    nb = len(a) // 4
    cuts = [4 * (nb * i // k) for i in range(k + 1)]
    out = torch.zeros((bits_ref + 63) // 64 + 1, dtype=torch.int64, device="cuda")
    off = 0
    for i in range(k):
        e, _ = dev_encode_bytes(gc, a[cuts[i]:cuts[i + 1]], P(gc, op))
        gc.stitch(out, off, e.words, e.bits)
        off += e.bits
    torch.cuda.synchronize()
    assert off == bits_ref
    assert out[: (bits_ref + 63) // 64].cpu().numpy().tobytes() == w_ref.tobytes()


# ---------------------------------------------------------------------------------------------- stage kernels
def test_stage_kernels(gc, orc):
    from gcow_amd import _ffi
    L = _ffi.load()
    rng = np.random.default_rng(2)
    for dims in (1, 2, 3):
        B = 4 ** dims
        nb = 300
        f = (rng.standard_normal((nb, B)) * 10.0 ** rng.integers(-40, 30, (nb, 1))).astype(np.float32)
        f[0, :3] = [np.nan, np.inf, 1e-40]
        df = torch.from_numpy(f).cuda()
        de = torch.zeros(nb, dtype=torch.int32, device="cuda")
        _ffi.check(L.gcow_stage_emax_device(df.data_ptr(), nb, dims, de.data_ptr(), None))
        dq = torch.zeros((nb, B), dtype=torch.int32, device="cuda")
        _ffi.check(L.gcow_stage_cast_device(df.data_ptr(), de.data_ptr(), nb, dims, dq.data_ptr(), None))
        torch.cuda.synchronize()
        em = de.cpu().numpy()
        q = dq.cpu().numpy()
        for i in range(nb):
            assert em[i] == orc.block_exponent(f[i])
            assert np.array_equal(q[i], orc.fwd_cast(f[i], int(em[i])))
        _ffi.check(L.gcow_stage_xform_device(dq.data_ptr(), nb, dims, 0, None))
        du = torch.zeros((nb, B), dtype=torch.int32, device="cuda")
        _ffi.check(L.gcow_stage_reorder_device(dq.data_ptr(), nb, dims, du.data_ptr(), None))
        torch.cuda.synchronize()
        qx = dq.cpu().numpy()
        u = du.cpu().numpy().view(np.uint32)
        for i in range(nb):
            ref = orc.fwd_xform(q[i], dims)
            assert np.array_equal(qx[i], ref)
            assert np.array_equal(u[i], orc.fwd_reorder(ref, dims))
        _ffi.check(L.gcow_stage_xform_device(dq.data_ptr(), nb, dims, 1, None))
        torch.cuda.synchronize()
        back = dq.cpu().numpy()
        for i in range(nb):
            assert np.array_equal(back[i], orc.inv_xform(qx[i], dims))


# ---------------------------------------------------------------------------------------------- drop-in surface
def _host_input(L, arr, dim):
    """init_zfp_input over a malloc'd host copy (free_zfp_input frees it, as sw/ does)."""
    libc = C.CDLL("libc.so.6")
    libc.malloc.restype = C.c_void_p
    libc.malloc.argtypes = [C.c_size_t]
    buf = libc.malloc(arr.nbytes)
    C.memmove(buf, arr.ctypes.data, arr.nbytes)
    dims = [C.c_uint(s) for s in reversed(arr.shape)]
    return L.init_zfp_input(C.c_void_p(buf), 3, C.c_uint(dim), *dims)


def test_dropin_golden_flow(gc, orc):
    """sw/tests/test_zfp.cpp:61-107 flow through the drop-in C ABI, host pointers."""
    from gcow_amd import _ffi
    L = _ffi.load()
    for g in GOLDENS[:6]:
        a = orc.gen_bump2d(g["n"], g["recipe"] == "bump_f32sum")
        inp = _host_input(L, a, 2)
        out = L.init_zfp_output(inp)
        L.set_zfp_output_accuracy(out, 1e-3)
        nbytes = L.zfp_compress(out, inp)
        assert nbytes == g["bytes"]
        b = C.string_at(out.contents.data.contents.begin, nbytes)
        assert _sha(b) == g["sha256"]
        # round trip through zfp_decompress (libzfp semantics)
        L.stream_rewind(out.contents.data)
        back = np.zeros_like(a)
        inp2 = L.alloc_zfp_input()
        inp2.contents.dtype = 3
        inp2.contents.data = back.ctypes.data
        inp2.contents.nx, inp2.contents.ny = g["n"], g["n"]
        L.zfp_decompress(out, inp2)
        ref = orc.decompress(np.frombuffer(b, np.uint64), a.shape, orc.accuracy(1e-3))
        assert np.array_equal(back.view(np.uint32), ref.view(np.uint32))
        inp2.contents.data = None
        L.free_zfp_input(inp2)
        L.cleanup(inp, out)


def test_dropin_1d_3d_and_modes(gc, orc, fxa):
    from gcow_amd import _ffi
    L = _ffi.load()
    for c in [c for c in FX if c["input"] in ("1d_n1000", "3d_9x10x7", "2d_special")]:
        a = fxa["input__" + c["input"]]
        inp = _host_input(L, a, a.ndim)
        out = L.init_zfp_output(inp)
        assert L.set_zfp_output_expert(out, *c["params"]) == 1
        nbytes = L.zfp_compress(out, inp)
        b = C.string_at(out.contents.data.contents.begin, nbytes)
        assert _sha(b) == c["stream_sha256"], c["name"]
        L.stream_rewind(out.contents.data)
        back = np.zeros_like(a)
        inp2 = L.alloc_zfp_input()
        inp2.contents.dtype = 3
        inp2.contents.data = back.ctypes.data
        for i, s in enumerate(reversed(a.shape)):
            setattr(inp2.contents, ["nx", "ny", "nz"][i], s)
        L.zfp_decompress(out, inp2)
        assert _sha(back.tobytes()) == c["decoded_sha256"], c["name"]
        inp2.contents.data = None
        L.free_zfp_input(inp2)
        L.cleanup(inp, out)


@pytest.mark.parametrize("layout", ["sx2_sy_pad", "transposed", "negative_sy", "1d_sx3"])
def test_dropin_strided_host_arrays(gc, orc, layout):
    """sw/ honours sx / sy on host memory (sw/src/zfp.c:37-39, 45, 86-92): zfp_compress of a strided host view and
    zfp_decompress into a strided host view match the oracle on the dense copy; the gaps between the strided elements
    are left untouched."""
    from gcow_amd import _ffi
    L = _ffi.load()
    rng = np.random.default_rng(zlib.crc32(layout.encode()))
    ny, nx = 37, 29
    if layout == "1d_sx3":
        ny = 0
        base = (rng.standard_normal(3 * 1001) * 1e-2).astype(np.float32)
        view = base[::3]
        sx, sy, off = 3, 0, 0
    elif layout == "sx2_sy_pad":
        sy = 2 * nx + 3
        base = (rng.standard_normal(sy * ny) * 1e-2).astype(np.float32)
        view = np.lib.stride_tricks.as_strided(base, (ny, nx), (4 * sy, 8))
        sx, off = 2, 0
    elif layout == "transposed":
        base = (rng.standard_normal(nx * ny) * 1e-2).astype(np.float32)
        view = base.reshape(nx, ny).T  # (ny, nx) with x stride ny, y stride 1
        sx, sy, off = ny, 1, 0
    else:  # rows stored bottom-up: data points at the last row, sy < 0
        base = (rng.standard_normal(nx * ny) * 1e-2).astype(np.float32)
        view = base.reshape(ny, nx)[::-1]
        sx, sy, off = 1, -nx, (ny - 1) * nx
    dense = np.ascontiguousarray(view)
    for op in (orc.accuracy(1e-4), orc.rate(8, dense.ndim)):
        w_ref, bits = orc.compress(dense, op)
        inp = L.alloc_zfp_input()
        inp.contents.dtype = 3
        inp.contents.data = base.ctypes.data + 4 * off
        inp.contents.nx, inp.contents.ny = nx if dense.ndim == 2 else dense.size, ny
        inp.contents.sx, inp.contents.sy = sx, sy
        out = L.init_zfp_output(inp)
        assert L.set_zfp_output_expert(out, *op.tuple()) == 1
        nbytes = L.zfp_compress(out, inp)
        assert nbytes == 8 * ((bits + 63) // 64), L.gcow_last_error()
        assert C.string_at(out.contents.data.contents.begin, nbytes) == w_ref.tobytes()
        # decode into a strided host view of a buffer whose gaps hold a sentinel
        L.stream_rewind(out.contents.data)
        back = np.full_like(base, 7.5)
        inp.contents.data = back.ctypes.data + 4 * off
        assert L.zfp_decompress(out, inp) == nbytes
        ref = orc.decompress(w_ref, dense.shape, op)
        if layout == "1d_sx3":
            got = back[::3]
        elif layout == "sx2_sy_pad":
            got = np.lib.stride_tricks.as_strided(back, (ny, nx), (4 * sy, 8))
        elif layout == "transposed":
            got = back.reshape(nx, ny).T
        else:
            got = back.reshape(ny, nx)[::-1]
        assert np.array_equal(np.ascontiguousarray(got).view(np.uint32), ref.view(np.uint32))
        mask = np.ones(base.size, bool)
        idx = np.arange(base.size).reshape(-1)
        touched = {"1d_sx3": idx[::3], "sx2_sy_pad": np.lib.stride_tricks.as_strided(
            idx, (ny, nx), (idx.itemsize * sy, 2 * idx.itemsize)).reshape(-1)}.get(layout, idx)
        mask[touched] = False
        assert np.all(back[mask] == 7.5)
        inp.contents.data = None
        L.free_zfp_input(inp)
        L.free_zfp_output(out)


def test_dropin_decompress_sees_rewritten_stream(gc, orc):
    """zfp_decompress reuses the device copy of the stream zfp_compress left behind only while the caller's buffer
    still holds that stream: after the caller overwrites the buffer with another stream (same params and shape) and
    rewinds, the new stream is decoded."""
    from gcow_amd import _ffi
    L = _ffi.load()
    a = orc.gen_normal(4 * 5000, 1e-3, 3, True)
    b = orc.gen_normal(4 * 5000, 1e-3, 4, True)
    op = orc.accuracy(1e-5)
    wb, _ = orc.compress(b, op)
    inp = _host_input(L, a, 1)
    out = L.init_zfp_output(inp)
    assert L.set_zfp_output_expert(out, *op.tuple()) == 1
    L.zfp_compress(out, inp)
    C.memmove(out.contents.data.contents.begin, wb.ctypes.data, wb.nbytes)  # another stream into the same buffer
    L.stream_rewind(out.contents.data)
    back = np.zeros_like(b)
    inp2 = L.alloc_zfp_input()
    inp2.contents.dtype = 3
    inp2.contents.data = back.ctypes.data
    inp2.contents.nx = b.size
    L.zfp_decompress(out, inp2)
    assert np.array_equal(back.view(np.uint32), orc.decompress(wb, b.shape, op).view(np.uint32))
    inp2.contents.data = None
    L.free_zfp_input(inp2)
    L.cleanup(inp, out)


@pytest.mark.parametrize("where", ["host", "device"])
def test_dropin_decompress_sees_one_word_edit(gc, orc, where):
    """A local edit of ONE word of the stream (any word, not a sampled one) between zfp_compress and zfp_decompress is
    decoded: the cache check covers every word (host: a hash of all words; device: a device-side compare)."""
    from gcow_amd import _ffi
    L = _ffi.load()
    n = 4 * 5000
    a = orc.gen_normal(n, 1e-3, 5, True)
    op = orc.rate(16, 1)
    w, _ = orc.compress(a, op)
    inp = _host_input(L, a, 1)
    out = L.init_zfp_output(inp)
    assert L.set_zfp_output_expert(out, *op.tuple()) == 1
    dbuf = None
    if where == "device":
        dbuf = torch.zeros(w.size + 8, dtype=torch.int64, device="cuda")
        out.contents.data = L.stream_init(C.c_void_p(dbuf.data_ptr()), dbuf.numel() * 8)
    assert L.zfp_compress(out, inp) == w.nbytes
    k = 3001  # word 3001 = block 3001 at rate 16
    edited = w.copy()
    edited[k] ^= np.uint64(0x5A5A5A5A00000000)
    if where == "device":
        torch.cuda.synchronize()
        dbuf[k] = int(edited.view(np.int64)[k])
        torch.cuda.synchronize()
    else:
        C.memmove(out.contents.data.contents.begin, edited.ctypes.data, edited.nbytes)
    L.stream_rewind(out.contents.data)
    back = np.zeros_like(a)
    inp2 = L.alloc_zfp_input()
    inp2.contents.dtype = 3
    inp2.contents.data = back.ctypes.data
    inp2.contents.nx = n
    L.zfp_decompress(out, inp2)
    want = orc.decompress(edited, a.shape, op)
    assert not np.array_equal(want.view(np.uint32), orc.decompress(w, a.shape, op).view(np.uint32))
    assert np.array_equal(back.view(np.uint32), want.view(np.uint32))
    # unedited: the cached device copy is used and decodes the same
    if where == "device":
        dbuf[k] = int(w.view(np.int64)[k])
        torch.cuda.synchronize()
    else:
        C.memmove(out.contents.data.contents.begin, w.ctypes.data, w.nbytes)
    L.stream_rewind(out.contents.data)
    L.zfp_decompress(out, inp2)
    assert np.array_equal(back.view(np.uint32), orc.decompress(w, a.shape, op).view(np.uint32))
    inp2.contents.data = None
    L.free_zfp_input(inp2)
    L.cleanup(inp, out)  # a device stream's buffer is the caller's (not freed)


def test_block_api_known_answers(gc, orc):
    """sw/tests/test_stages.cpp ENCODE_IBLOCK / ENCODE_ALL_BITPLANES / CAST through the drop-in block API."""
    from gcow_amd import _ffi
    L = _ffi.load()
    KA = json.load(open(os.path.join(GOLD, "reference_known_answers.json")))
    buf = (C.c_uint64 * 64)()
    s = L.stream_init(C.cast(buf, C.c_void_p), C.sizeof(buf))
    k = KA["encode_iblock"]
    L.stream_write_bits(s, 2 * k["e"] + 1, 9)
    ib = (C.c_int32 * 16)(*k["iblock"])
    bits = L.encode_iblock(s, 1, 16658, k["expected_maxprec"], ib, 2)
    assert bits == k["expected_iblock_bits"]
    L.stream_flush(s)
    assert [buf[0], buf[1]] == [int(x) for x in k["expected_words"]]
    k = KA["encode_all_bitplanes"]
    L.stream_rewind(s)
    ub = (C.c_uint32 * 16)(*k["ublock"])
    for _ in range(k["repeat"]):
        L.stream_write_bits(s, 2 * (k["emax"] + 127) + 1, 9)
        L.encode_all_bitplanes(s, ub, k["expected_maxprec"], 16)
    L.stream_flush(s)
    assert [buf[i] for i in range(9)] == [int(x) for x in k["expected_words"]]
    k = KA["cast"]
    bump = orc.gen_bump2d(3)
    fb = (C.c_float * 16)()
    L.gather_partial_2d_block(fb, bump.ctypes.data_as(C.POINTER(C.c_float)), 3, 3, 1, 3)
    assert L.get_block_exponent(fb, 16) == 1
    q = (C.c_int32 * 16)()
    L.fwd_cast_block(q, fb, 16, 1)
    assert list(q) == k["expected"]
    L.fwd_decorrelate_2d_block(q)
    assert list(q) == KA["decorrelate"]["expected"]
    u = (C.c_uint32 * 16)()
    perm = (C.c_ubyte * 16).in_dll(L, "PERM_2D")
    L.fwd_reorder_int2uint(u, q, perm, 16)
    assert list(u) == KA["reorder"]["expected"]


def test_encode_fblock_decode_fblock(gc, orc):
    from gcow_amd import _ffi
    L = _ffi.load()
    a = orc.gen_bump2d(8)
    op = orc.accuracy(1e-3)
    out = L.alloc_zfp_output()
    L.set_zfp_output_accuracy(out, 1e-3)
    buf = (C.c_uint64 * 256)()
    out.contents.data = L.stream_init(C.cast(buf, C.c_void_p), C.sizeof(buf))
    fb = (C.c_float * 16)()
    for by in range(2):
        for bx in range(2):
            src = C.cast(C.c_void_p(a.ctypes.data + (4 * by * 8 + 4 * bx) * 4), C.POINTER(C.c_float))
            L.gather_2d_block(fb, src, 1, 8)
            L.encode_fblock(out, fb, 2)
    L.stream_flush(out.contents.data)
    nbytes = L.stream_size_bytes(out.contents.data)
    w_ref, _ = orc.compress(a, op)
    assert bytes(buf)[:nbytes] == w_ref.tobytes()
    L.stream_rewind(out.contents.data)
    ref = orc.decompress(w_ref, a.shape, op)
    for by in range(2):
        for bx in range(2):
            L.decode_fblock(out, fb, 2)
            blk = np.frombuffer(bytes(fb), np.float32).reshape(4, 4)
            assert np.array_equal(blk.view(np.uint32), ref[4 * by:4 * by + 4, 4 * bx:4 * bx + 4].view(np.uint32))


# ---------------------------------------------------------------------------------------------- full-size configs
def test_c2_full_size_fixed_rate(gc, orc):
    """BASELINE config 2: 256 Mi contiguous fp32, 1-D fixed rate 16 and 8, bit-exact vs the threaded oracle -- on the
    very bucket bench.py times (codec.fill_normal, seed 0x67636F77, zero / tiny / subnormal blocks injected). The
    whole decode of each stream (the bench times the rate-16 one) is compared with the threaded oracle decode."""
    n = 256 * 1024 * 1024
    T = min(16, os.cpu_count() or 1)
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    gc.fill_normal(x, 1e-3, seed=0x67636F77, inject=True)
    a = x.cpu().numpy()
    # the injected special blocks are there (bench.data claims them)
    blk = np.abs(a.reshape(-1, 4)).max(axis=1)
    assert (blk == 0).sum() > n // 4 // 128 and ((blk > 0) & (blk < 2.0 ** -98)).sum() > n // 4 // 4096
    del blk
    for r in (16, 8):
        op = orc.rate(r, 1)
        w_ref, bits_ref = orc.compress(a, op, threads=T)
        e = gc.encode(x, P(gc, op))
        torch.cuda.synchronize()
        assert e.bits == bits_ref
        got = e.stream().cpu().numpy().view(np.uint64)
        assert np.array_equal(got, w_ref)
        del got
        d = gc.decode(e).cpu().numpy()
        ref = orc.decompress(w_ref, a.shape, op, threads=T)
        assert np.array_equal(d.view(np.uint32), ref.view(np.uint32)), r
        del w_ref, d, ref, e


def test_c3_full_size_roundtrip(gc, orc):
    """BASELINE config 3: 512^3 fp32 volume, 3-D fixed rate 8 and accuracy 1e-3, encode + decode vs the oracle -- on
    the field bench.py times (codec.c3_field). The whole decoded field is compared bit for bit with the threaded
    oracle decode (libzfp semantics, sw/src/decode.c:113-183 with the block-size fix)."""
    xt = gc.c3_field(torch.device("cuda", 0))
    a = xt.cpu().numpy()
    T = min(16, os.cpu_count() or 1)
    for op, stride in ((orc.rate(8, 3), 0), (orc.accuracy(1e-3), 1)):
        w_ref, bits_ref, offs = orc.compress(a, op, threads=T, offsets=True)
        e = gc.encode(xt, P(gc, op), index_stride=stride)
        torch.cuda.synchronize()
        assert e.bits == bits_ref
        assert np.array_equal(e.stream().cpu().numpy().view(np.uint64), w_ref)
        d = gc.decode(e).cpu().numpy()
        ref = orc.decompress(w_ref, a.shape, op, threads=T, offsets=offs)
        assert np.array_equal(d.view(np.uint32), ref.view(np.uint32)), op
        if op.minbits != op.maxbits:
            assert float(np.max(np.abs(d - a))) <= 1e-3
        del w_ref, d, ref, e


def test_multichunk_fixed_rate_1d(gc, orc):
    """More than 2^27 blocks: the fixed-rate 1-D encoder and decoder launch the grid in chunks of 2^27 blocks (buffer
    offsets stay below 2^32; gcow_kernels.hip launch_fixed1d_t / launch_decode_fixed1d), as C4's strong-scaling legs
    do with 1-2 Gi values per rank. n = 2^29 + 4 * 1001 + 3 values (2 GiB): two chunks and a padded last block. Whole
    stream and whole decode vs the threaded oracle at rates 16 and 8."""
    n = (1 << 29) + 4 * 1001 + 3
    T = min(16, os.cpu_count() or 1)
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    gc.fill_normal(x, 1e-3, seed=0x67636F77 + 99, inject=True)
    a = x.cpu().numpy()
    nb = (n + 3) // 4
    for r in (16, 8):
        op = orc.rate(r, 1)
        w_ref, bits_ref = orc.compress(a, op, threads=T)
        e = gc.encode(x, P(gc, op))
        torch.cuda.synchronize()
        assert e.bits == bits_ref == nb * 4 * r
        got = e.stream().cpu().numpy().view(np.uint64)
        assert np.array_equal(got, w_ref)
        del got
        d = gc.decode(e).cpu().numpy()
        ref = orc.decompress(w_ref, (n,), op, threads=T)
        assert np.array_equal(d.view(np.uint32), ref.view(np.uint32)), r
        del d, ref, e, w_ref


@pytest.mark.parametrize("r", [16, 8])
def test_fast1d_adversarial_blocks(gc, orc, r):
    """Blocks whose coefficients differ by many binades (long group-test phases beyond one 16-plane window),
    constant / alternating blocks (zero high-frequency coefficients), powers of two, mixed signs."""
    rng = np.random.default_rng(17)
    nb = 1 << 16
    sign = np.where(rng.random((nb, 4)) < 0.5, -1.0, 1.0)
    wide = sign * 2.0 ** rng.uniform(-40, 0, (nb, 4))
    const = np.repeat(rng.standard_normal((nb // 4, 1)), 4, axis=1)
    alt = np.repeat(rng.standard_normal((nb // 4, 1)), 4, axis=1) * np.array([1, -1, 1, -1])
    pow2 = 2.0 ** rng.integers(-30, 30, (nb // 4, 4)) * np.where(rng.random((nb // 4, 4)) < 0.5, -1.0, 1.0)
    ramp = np.cumsum(rng.standard_normal((nb // 4, 4)) * 1e-6, axis=1) + 1.0
    a = np.concatenate([wide, const, alt, pow2, ramp]).astype(np.float32).reshape(-1)
    _check_vs_oracle(gc, orc, a, orc.rate(r, 1))


@pytest.mark.parametrize("r", [16, 8])
def test_fast1d_decode_arbitrary_streams(gc, orc, r):
    """The 1-D fixed-rate decoder on arbitrary bit patterns (not only encoder output): every header exponent, long
    runs of empty planes, group phases that never reach n = 3, all-verbatim words; bit-exact vs libzfp semantics."""
    rng = np.random.default_rng(5 + r)
    nw = (1 << 16) * r // 64
    w = rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64) * np.uint64(2) + rng.integers(0, 2, nw).astype(np.uint64)
    # sparse words: long zero runs after the header
    sparse = w & (rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64) & rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64))
    # very sparse words (one bit in eight after the header): group phases past the 16-plane window, plane codes that
    # cross the budget, steps from the window's last nibble -- the pair decoder's special blocks
    dense8 = np.zeros(nw, np.uint64)
    for _ in range(3):
        dense8 |= rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64)
    very = (~dense8 & rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64)) | np.uint64(1)
    words = np.concatenate([w, sparse | np.uint64(0x0101010101010101), very])
    n = words.size * 64 // r
    op = orc.rate(r, 1)
    ref = orc.decompress(words, (n,), op)
    d = gc.decode(torch.from_numpy(np.concatenate([words, np.zeros(2, np.uint64)]).view(np.int64)).cuda(), (n,),
                  P(gc, op))
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("world", [3, 4])
def test_decode_mean_arbitrary_streams(gc, orc, world):
    """decode_mean (the fixed-rate pair decoder with gather tables, and its special blocks) on arbitrary and very
    sparse 64-bit words: the fp32 mean, in rank order, of the oracle's decode of each stream (a power-of-two world
    scales by the reciprocal, the other divides)."""
    rng = np.random.default_rng(40 + world)
    nw = 1 << 15
    streams = []
    for r in range(world):
        w = rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64) * np.uint64(2) + rng.integers(0, 2, nw).astype(np.uint64)
        d8 = np.zeros(nw, np.uint64)
        for _ in range(3):
            d8 |= rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64)
        very = (~d8 & rng.integers(0, 2 ** 63, nw, dtype=np.int64).view(np.uint64)) | np.uint64(1)
        streams.append(np.where(rng.random(nw) < 0.5, w, very))
    n = nw * 4
    op = orc.rate(16, 1)
    acc = np.zeros(n, np.float32)
    with np.errstate(over="ignore", invalid="ignore"):  # arbitrary headers decode to +-inf; inf - inf is NaN
        for st in streams:
            acc = acc + orc.decompress(np.concatenate([st, np.zeros(2, np.uint64)]), (n,), op)
        want = acc / np.float32(world)
    buf = torch.from_numpy(np.concatenate(streams + [np.zeros(2, np.uint64)]).view(np.int64)).cuda()
    got = gc.decode_mean(buf, nw, world, n, P(gc, op)).cpu().numpy()
    # inf + -inf: a NaN whose bit pattern is the device's (x86 and the GPU differ in the default NaN's sign)
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), want[~nan].view(np.uint32))


@pytest.mark.parametrize("params", [(64, 64, 20, -1074), (64, 64, 64, -100), (32, 32, 12, -1074), (32, 32, 64, -60)])
def test_fixed1d_generic_coder(gc, orc, params):
    """Whole-word fixed-rate 1-D blocks outside the lean coder's domain (kmin > 0 possible): generic coder and
    generic decoder, vs the oracle."""
    a = np.concatenate([orc.gen_normal(4 * 5000 + 3, 1e-3, 31, True), orc.gen_normal(4000, 1.0, 32, False)])
    _check_vs_oracle(gc, orc, a, orc.expert(*params))


def _adversarial_1d(seed):
    rng = np.random.default_rng(seed)
    nb = 1 << 14
    sign = np.where(rng.random((nb, 4)) < 0.5, -1.0, 1.0)
    wide = sign * 2.0 ** rng.uniform(-60, 10, (nb, 4))
    const = np.repeat(rng.standard_normal((nb // 4, 1)), 4, axis=1)
    alt = np.repeat(rng.standard_normal((nb // 4, 1)), 4, axis=1) * np.array([1, -1, 1, -1])
    pow2 = 2.0 ** rng.integers(-60, 30, (nb // 4, 4)) * np.where(rng.random((nb // 4, 4)) < 0.5, -1.0, 1.0)
    ramp = np.cumsum(rng.standard_normal((nb // 4, 4)) * 1e-6, axis=1) + 1.0
    tiny = rng.standard_normal((nb // 8, 4)) * 1e-38
    return np.concatenate([wide, const, alt, pow2, ramp, tiny]).astype(np.float32).reshape(-1)


@pytest.mark.parametrize("mode", ["acc1e-6", "acc1e-3", "acc1e-20", "acc1e-30", "prec32", "prec20", "prec5",
                                  "expert_max", "expert_maxprec12"])
def test_var1d_closed_form_coder(gc, orc, mode):
    """1-D variable-rate blocks through the closed-form coder (long group phases, many planes, tiny / subnormal /
    const / alternating blocks, partial last block), stream and decode vs the oracle, with a block index."""
    a = np.concatenate([_adversarial_1d(3), orc.gen_normal((1 << 18) + 3, 1e-3, 77, True)])
    op = {"acc1e-6": orc.accuracy(1e-6), "acc1e-3": orc.accuracy(1e-3), "acc1e-20": orc.accuracy(1e-20),
          "acc1e-30": orc.accuracy(1e-30), "prec32": orc.precision(32), "prec20": orc.precision(20),
          "prec5": orc.precision(5), "expert_max": orc.expert(1, 16658, 64, -1074),
          "expert_maxprec12": orc.expert(1, 16658, 12, -30)}[mode]
    _check_vs_oracle(gc, orc, a, op, index_stride=16)


@pytest.mark.parametrize("env", ["spin0", "single_pass", "range"])
@pytest.mark.parametrize("mode", ["acc1e-6", "acc1e-3", "prec32", "expert_max", "bf16_acc1e-6"])
def test_var1d_encoder_forms(gc, orc, env, mode):
    """The 1-D variable-rate encoder's other forms (the default is a count per 1024-block tile + scan + the tile coder
    placed by the scan), bit-exact vs the oracle: `single_pass` places the tiles by a decoupled look-back, `spin0`
    also makes every tile compute a not-yet-published predecessor's total itself (its no-dispatch-order fallback),
    `range` is count + scan + k_encode1d_var over larger ranges (selected through the test-only
    gcow_debug_set_var1d_variant)."""
    form = "range" if env == "range" else "single_pass"
    with gc.var1d_variant(form, spin=0 if env == "spin0" else -1):
        _var1d_form_case(gc, orc, mode)


def _var1d_form_case(gc, orc, mode):
    a = np.concatenate([_adversarial_1d(11), orc.gen_normal((1 << 20) + 3, 1e-3, 78, True)])
    if mode.startswith("bf16"):
        a = (a.view(np.uint32) >> 16).astype(np.uint16)
    op = {"acc1e-6": orc.accuracy(1e-6), "acc1e-3": orc.accuracy(1e-3), "prec32": orc.precision(32),
          "expert_max": orc.expert(1, 16658, 64, -1074), "bf16_acc1e-6": orc.accuracy(1e-6)}[mode]
    w_ref, bits_ref = orc.compress(a, op)
    e, b = dev_encode_bytes(gc, a, P(gc, op), 16)
    assert e.bits == bits_ref
    assert b == w_ref.tobytes()
    d = gc.decode(e)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().view(np.uint32), orc.decompress(w_ref, a.shape, op).view(np.uint32))


@pytest.mark.parametrize("bits", ["low", "mid", "high", "max"])
def test_var1d_decode_stage_parts(gc, orc, bits):
    """The lean 1-D variable-rate decoder stages a workgroup's stream (128 chunks of 16 blocks) in an LDS stage sized
    for 64 bits per block; a workgroup above that takes the general path. Workgroups at ~24, ~63, ~110 and ~140 bits
    per block, interleaved with low-rate ones, decode bit-exactly."""
    rng = np.random.default_rng(4242)
    wg = 128 * 16 * 4  # values per workgroup
    n = wg * 6
    a = rng.standard_normal(n).astype(np.float32)
    scale = {"low": 1e-3, "mid": 1e-3, "high": 1.0, "max": 1.0}[bits]
    a[wg:3 * wg] *= np.float32(scale)
    a[:wg] *= np.float32(1e-6)
    a[3 * wg:] *= np.float32(1e-5)
    op = {"low": orc.accuracy(1e-3), "mid": orc.accuracy(1e-6), "high": orc.accuracy(1e-6),
          "max": orc.precision(32)}[bits]
    _check_vs_oracle(gc, orc, a, op, index_stride=16)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("appended", [False, True])
def test_var1d_mixed_tile_sizes(gc, orc, dtype, appended):
    """The default 1-D variable-rate form codes tiles of up to 95 bits per block in a small LDS window
    (k_encode1d_var_tile) and larger ones in a second pass (k_encode1d_var_tile_big). Tiles (4096 values) alternate
    between N(0, 1) (about 110 bits per block at accuracy 1e-6) and N(0, 1e-3) (about 60), with Inf / NaN blocks in
    both kinds and a ragged tail, so both kernels write words their neighbours share. `appended`: the stream starts
    at a device bit offset (gcow_encode_device_append through a chunked encode)."""
    rng = np.random.default_rng(97)
    n = 4096 * 21 + 4 * 333 + 3
    a = rng.standard_normal(n).astype(np.float32)
    for t in range(0, n, 4096):
        if (t // 4096) % 3 != 1:
            a[t:t + 4096] *= np.float32(1e-3)
    a[4096 * 4 + 17] = np.inf
    a[4096 * 7 + 401] = np.nan
    if dtype == "bf16":
        a = (a.view(np.uint32) >> 16).astype(np.uint16)
    op = orc.accuracy(1e-6)
    if not appended:
        _check_vs_oracle(gc, orc, a, op, index_stride=16)
        return
    w_ref, bits_ref = orc.compress(a, op)
    x = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    if dtype == "bf16":
        x = x.view(torch.bfloat16)
    params = P(gc, op)
    words = torch.zeros(gc.max_output_bytes(x.shape, params, x.dtype) // 8 + 4, dtype=torch.int64, device="cuda")
    cuts = [0, 4096 * 9 + 4 * 77, n]  # block-aligned: the second chunk starts mid-word
    bits = torch.zeros(len(cuts), dtype=torch.int64, device="cuda")
    for i in range(len(cuts) - 1):
        gc.encode_append(x[cuts[i]:cuts[i + 1]], params, words, bits[i:i + 1], bits[i + 1:i + 2])
    torch.cuda.synchronize()
    assert int(bits[-1]) == bits_ref
    nw = (bits_ref + 63) // 64
    assert np.array_equal(words[:nw].cpu().numpy().view(np.uint64), w_ref.view(np.uint64)[:nw])


@pytest.mark.parametrize("tol", [1e-6, 1e-3])
@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_c5_full_size_accuracy(gc, orc, dtype, tol):
    """BASELINE config 5 shape (bf16) and its fp32 twin: 256 Mi values of the bench's bucket (bf16 by exact
    widening), accuracy 1e-6 and 1e-3 (both timed by bench.py), stream vs the threaded oracle, and the whole
    variable-rate decode (k_decode1d_var_lean, the receive side of the DDP hook) vs the threaded oracle decode."""
    n = 256 * 1024 * 1024
    T = min(16, os.cpu_count() or 1)
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    gc.fill_normal(x, 1e-3, seed=0x67636F77, inject=True)
    if dtype == "bf16":
        x = x.to(torch.bfloat16)
        h = x.cpu().view(torch.int16).numpy().view(np.uint16)
    else:
        h = x.cpu().numpy()
    op = orc.accuracy(tol)
    w_ref, bits_ref, offs = orc.compress(h, op, threads=T, offsets=True)
    e = gc.encode(x, P(gc, op), index_stride=16)
    torch.cuda.synchronize()
    assert e.bits == bits_ref
    assert np.array_equal(e.stream().cpu().numpy().view(np.uint64), w_ref)
    d = gc.decode(e).cpu().numpy()
    ref = orc.decompress(w_ref, (n,), op, threads=T, offsets=offs)
    assert np.array_equal(d.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("case", ["c5_bf16_acc1e-6", "c5_bf16_acc1e-3", "c2_f32_rate16"])
def test_host_encoder_full_size(gc, orc, case):
    """The host-resident paths bench.py times, at the benched size and chunking: HostEncoder(chunks=16) on the full
    256 Mi-value bucket (C5: bf16 by exact widening, accuracy 1e-6 / 1e-3 -- BASELINE configs[4]'s timed region is
    pinned H2D + encode + D2H; C2: fp32 rate 16, the host_e2e leg). The whole host-resident stream, every one of the
    16 chunk seams included, vs the threaded oracle (caller contract: hw/models/train_imagenet.py:453,471)."""
    n = 256 * 1024 * 1024
    T = min(16, os.cpu_count() or 1)
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    gc.fill_normal(x, 1e-3, seed=0x67636F77, inject=True)
    if case.startswith("c5"):
        dtype, op = torch.bfloat16, orc.accuracy(1e-6 if case.endswith("1e-6") else 1e-3)
        h = x.to(torch.bfloat16).cpu()
        a = h.view(torch.int16).numpy().view(np.uint16)
    else:
        dtype, op = torch.float32, orc.rate(16, 1)
        h = x.cpu()
        a = h.numpy()
    del x
    h = h.pin_memory()
    params = P(gc, op)
    enc = gc.HostEncoder(n, dtype, params, chunks=16)
    assert len(enc.bounds) == 16
    out = torch.zeros(gc.max_output_bytes((n,), params, dtype) // 8 + 2, dtype=torch.int64).pin_memory()
    bits = enc(h, out)
    w_ref, bits_ref = orc.compress(a, op, threads=T)
    assert bits == bits_ref
    nw = (bits + 63) // 64
    got = out[:nw].numpy().view(np.uint64)
    if not np.array_equal(got, w_ref):
        bad = int(np.flatnonzero(got != w_ref)[0])
        seams = [lo for lo, _ in enc.bounds]
        pytest.fail("first differing word %d (bit %d); chunk starts (values) %s" % (bad, 64 * bad, seams))
    # the words past the stream stay untouched (no stray D2H past the flushed end)
    assert not out[nw:].any()


def test_var1d_more_than_64ki_tiles(gc, orc):
    """Past 64 Ki tiles of 1024 blocks (256 Mi values) the range scan of the 1-D variable-rate encoder relies on the
    count's 8-tile group totals (k_scan_ranges_mw with gsums); a ragged bucket just past that size, accuracy 1e-6 on
    bf16, vs the threaded oracle."""
    n = 256 * 1024 * 1024 + 3 * 4096 + 7
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    gc.fill_normal(x, 1e-3, seed=0x5EED, inject=True)
    xb = x.to(torch.bfloat16)
    del x
    hb = xb.cpu().view(torch.int16).numpy().view(np.uint16)
    op = orc.accuracy(1e-6)
    w_ref, bits_ref = orc.compress(hb, op, threads=min(16, os.cpu_count() or 1))
    e = gc.encode(xb, P(gc, op), index_stride=16)
    torch.cuda.synchronize()
    assert e.bits == bits_ref
    assert np.array_equal(e.stream().cpu().numpy().view(np.uint64), w_ref)


@pytest.mark.parametrize("nblocks", [1, 1023, 1024, 1025, 2048 + 5, 70001])
@pytest.mark.parametrize("layout", ["contig", "offset1", "offset8", "stride2"])
def test_var1d_bf16_load_paths(gc, orc, nblocks, layout):
    """Variable-rate 1-D bf16: the coalesced 16-B load paths of the count and encode passes (contiguous, 16-B aligned,
    whole tiles of 1024 full blocks) and the per-lane gather they fall back to (a 2-B or 16-B offset view, a strided
    view, partial tiles, a padded last block) give the oracle's stream and block index."""
    n = 4 * nblocks - (1 if nblocks > 1 else 0)
    a = orc.gen_normal(n, 1e-3, 500 + nblocks, True)
    hb = (a.view(np.uint32) >> 16).astype(np.uint16)
    op = orc.accuracy(1e-6)
    w_ref, bits_ref = orc.compress(hb, op)
    pad = {"contig": 0, "offset1": 1, "offset8": 8, "stride2": 0}[layout]
    step = 2 if layout == "stride2" else 1
    big = np.zeros(pad + step * n, np.uint16)
    big[pad::step] = hb
    x = torch.from_numpy(big).cuda().view(torch.bfloat16)[pad::step]
    assert x.numel() == n
    e = gc.encode(x, P(gc, op), index_stride=16)
    torch.cuda.synchronize()
    assert e.bits == bits_ref
    assert e.to_bytes() == w_ref.tobytes()
    d = gc.decode(e)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().view(np.uint32), orc.decompress(w_ref, hb.shape, op).view(np.uint32))


@pytest.mark.parametrize("nblocks", [1, 511, 512, 513, 1024, 5000, 100003])
@pytest.mark.parametrize("mode", ["acc1e-3", "sparse"])
def test_var1d_tiles(gc, orc, nblocks, mode):
    """Variable-rate 1-D encoder (count pass, range scan, tiles of 1024 blocks) across tile boundaries: partial last
    tile and block, exact multiples, mostly-zero tiles (1-bit blocks: tile boundaries on 32-bit words), stream + block
    index + decode vs the oracle."""
    n = 4 * nblocks - (1 if nblocks > 1 else 0)
    if mode == "acc1e-3":
        a = orc.gen_normal(n, 1e-3, 1000 + nblocks, True)
        op = orc.accuracy(1e-3)
    else:
        a = np.zeros(n, np.float32)
        rng = np.random.default_rng(nblocks)
        hit = rng.integers(0, n, max(1, n // 300))
        a[hit] = rng.standard_normal(hit.size).astype(np.float32)
        op = orc.accuracy(1e-6)
    _check_vs_oracle(gc, orc, a, op, index_stride=16)


@pytest.mark.parametrize("mode", ["acc1e-6", "acc1e-3", "bf16_acc1e-6", "prec20"])
def test_encode_append_chunks(gc, orc, mode):
    """gcow_encode_device_append: a bucket encoded in uneven chunks, each appended at the device-side end of the
    previous one, equals the oracle's single stream (and its block index is absolute)."""
    a = np.concatenate([orc.gen_normal(4 * 3001 + 2, 1e-3, 41, True), _adversarial_1d(5)[:4 * 997]])
    op = {"acc1e-6": orc.accuracy(1e-6), "acc1e-3": orc.accuracy(1e-3), "bf16_acc1e-6": orc.accuracy(1e-6),
          "prec20": orc.precision(20)}[mode]
    if mode.startswith("bf16"):
        a = (a.view(np.uint32) >> 16).astype(np.uint16)
    w_ref, bits_ref = orc.compress(a, op)
    x = torch.from_numpy(a).cuda()
    if a.dtype == np.uint16:
        x = x.view(torch.bfloat16)
    params = P(gc, op)
    words = torch.zeros(gc.max_output_bytes(x.shape, params, x.dtype) // 8 + 4, dtype=torch.int64, device="cuda")
    cuts = [0, 4 * 700, 4 * 701 + 0, 4 * 2500, 4 * 2516, a.size]  # an empty chunk, a 1-block chunk, a partial tail
    bits = torch.zeros(len(cuts), dtype=torch.int64, device="cuda")
    for i in range(len(cuts) - 1):
        gc.encode_append(x[cuts[i]:cuts[i + 1]], params, words, bits[i:i + 1], bits[i + 1:i + 2])
    torch.cuda.synchronize()
    assert int(bits[-1]) == bits_ref
    nw = (bits_ref + 63) // 64
    assert np.array_equal(words[:nw].cpu().numpy().view(np.uint64), w_ref.view(np.uint64)[:nw])


@pytest.mark.parametrize("mode", ["rate16", "rate8", "rate2.5", "rate2.25", "rate9.5", "acc1e-6", "bf16_acc1e-3"])
def test_host_encoder_pipelined(gc, orc, mode):
    """HostEncoder (pinned host in -> overlapped H2D / encode / D2H in chunks -> pinned host out) equals the oracle;
    fixed rates whose block is not a divisor of 64 bits (maxbits 10, 9, 38) cut chunks on 64-bit stream words."""
    a = orc.gen_normal(4 * 40000 + 3, 1e-3, 43, True)
    op = {"rate16": orc.rate(16, 1), "rate8": orc.rate(8, 1), "rate2.5": orc.rate(2.5, 1),
          "rate2.25": orc.rate(2.25, 1), "rate9.5": orc.rate(9.5, 1), "acc1e-6": orc.accuracy(1e-6),
          "bf16_acc1e-3": orc.accuracy(1e-3)}[mode]
    if mode.startswith("bf16"):
        a = (a.view(np.uint32) >> 16).astype(np.uint16)
    w_ref, bits_ref = orc.compress(a, op)
    h = torch.from_numpy(a)
    dtype = torch.float32
    if a.dtype == np.uint16:
        h, dtype = h.view(torch.bfloat16), torch.bfloat16
    h = h.pin_memory()
    params = P(gc, op)
    enc = gc.HostEncoder(a.size, dtype, params, chunks=5)
    out = torch.zeros(gc.max_output_bytes((a.size,), params, dtype) // 8 + 2, dtype=torch.int64).pin_memory()
    for _ in range(2):  # reusable
        out.zero_()
        bits = enc(h, out)
        assert bits == bits_ref
        nw = (bits + 63) // 64
        assert np.array_equal(out[:nw].numpy().view(np.uint64), w_ref.view(np.uint64)[:nw])


@pytest.mark.parametrize("r", [1, 2, 4, 8, 16, 32, 2.5])
def test_fixed3d_word_rates(gc, orc, r):
    """Fixed-rate 3-D blocks through the per-lane word-writer encoder and the LDS-staged decoder (block budgets of
    2..64 words; rate 2.5 = 160 bits takes the generic path), partial blocks on every axis, zero / tiny / Inf / NaN
    blocks, fp32 and bf16, stream and decode vs the oracle."""
    rng = np.random.default_rng(int(r * 10))
    a = (rng.standard_normal((13, 17, 21)) * 1e-2).astype(np.float32)
    a[:4, :4, :4] = 0
    a[4:8, :4, :4] = 1e-36
    a[8, 5, 5] = np.inf
    a[12, 16, 20] = np.nan
    _check_vs_oracle(gc, orc, a, orc.rate(r, 3))
    bf = (a.view(np.uint32) >> 16).astype(np.uint16)
    _check_vs_oracle(gc, orc, bf, orc.rate(r, 3), decode=False)


@pytest.mark.parametrize("mode", ["acc", "prec", "rate"])
def test_3d_emax_cast_edge_blocks(gc, orc, mode):
    """The 64-value finite-block prologue (codec_device.h emax_cast_finite: max |x| from unsigned and signed maxima of
    the bit patterns, fma + truncating conversion, INT_MIN for an infinite scale) against the oracle on the blocks it
    must get right: all-negative and all-positive blocks, -0.0, subnormal-only, tiny (scale overflow), maxima at
    2^k and just below, largest finite values, and Inf / NaN blocks (the generic path); fixed rate, accuracy and
    precision, fp32 and bf16."""
    rng = np.random.default_rng(3)
    a = (rng.standard_normal((16, 16, 12)) * 1e-2).astype(np.float32)
    a[:4, :4, :4] = -np.abs(a[:4, :4, :4])           # all negative
    a[:4, 4:8, :4] = np.abs(a[:4, 4:8, :4])          # all positive
    a[:4, 8:12, :4] = -0.0                           # negative zeros
    a[:4, 12:16, :4] = 1e-40                         # subnormal only
    a[4:8, :4, :4] = -3e-37                          # tiny, negative
    a[4:8, 4:8, :4] *= 1e-30                         # small normal
    a[4:8, 8:12, :4] = 1.0
    a[4:8, 8:12, 0] = -2.0                           # negative power-of-two maximum
    a[4:8, 12:16, :4] = np.float32(np.nextafter(np.float32(4.0), np.float32(0.0)))
    a[8:12, :4, :4] = np.finfo(np.float32).max * np.sign(a[8:12, :4, :4])
    a[8:12, 4:8, :4] = np.float32(-np.finfo(np.float32).tiny)
    a[8, 9, 1] = np.inf
    a[9, 13, 2] = -np.inf
    a[13, 2, 5] = np.nan
    a[14, 6, 9] = -np.nan
    p = {"acc": orc.accuracy(1e-3), "prec": orc.precision(20), "rate": orc.rate(8, 3)}[mode]
    _check_vs_oracle(gc, orc, a, p)
    bf = (a.view(np.uint32) >> 16).astype(np.uint16)
    _check_vs_oracle(gc, orc, bf, p, decode=False)


@pytest.mark.parametrize("shape", [(12, 12, 12), (40, 44), (4 * 4099 + 1,)])
def test_staged_decode_wide_blocks(gc, orc, shape):
    """LDS-staged decoders with spans over their capacity (precision 32 on values spread over 2^-60..2^10: blocks of
    up to ~2100 bits in 3-D): the over-capacity workgroups decode from global memory; vs the oracle."""
    rng = np.random.default_rng(len(shape))
    a = (np.where(rng.random(shape) < 0.5, -1.0, 1.0) * 2.0 ** rng.uniform(-60, 10, shape)).astype(np.float32)
    stride = 16 if len(shape) == 1 else 1
    _check_vs_oracle(gc, orc, a, orc.precision(32), index_stride=stride)
    _check_vs_oracle(gc, orc, a, orc.accuracy(1e-30), index_stride=stride)


FX4 = json.load(open(os.path.join(GOLD, "libzfp_fixtures_4d.json")))["cases"]


@pytest.fixture(scope="module")
def fxa4():
    return np.load(os.path.join(GOLD, "libzfp_fixtures_4d.npz"))


@pytest.mark.parametrize("c", FX4, ids=lambda c: c["name"])
def test_libzfp_fixture_4d_device(gc, fxa4, c):
    """4-D blocks on the GPU (one wave per block) against libzfp 0.5.5: stream bytes and decoded values."""
    a = fxa4["input__" + c["input"]]
    p = gc.expert(*c["params"])
    e, b = dev_encode_bytes(gc, a, p, index_stride=0 if gc.is_fixed(p) else 1)
    assert len(b) == c["bytes"]
    assert _sha(b) == c["stream_sha256"]
    d = gc.decode(e)
    torch.cuda.synchronize()
    assert _sha(d.cpu().numpy().tobytes()) == c["decoded_sha256"]


def test_4d_random_and_bf16(gc, orc):
    """4-D random fields (partial blocks on every axis) and a bf16 input vs the oracle."""
    rng = np.random.default_rng(44)
    a = (rng.standard_normal((6, 5, 7, 10)) * 1e-2).astype(np.float32)
    for op in (orc.rate(8, 4), orc.accuracy(1e-4), orc.precision(20)):
        _check_vs_oracle(gc, orc, a, op, index_stride=0 if op.minbits == op.maxbits else 1)
    bf = (a.view(np.uint32) >> 16).astype(np.uint16)
    _check_vs_oracle(gc, orc, bf, orc.accuracy(1e-3), index_stride=1, decode=False)


@pytest.mark.parametrize("stride", [0, 4])
def test_4d_variable_rate_sequential_decode(gc, orc, stride):
    """4-D variable-rate streams without a stride-1 block index decode by one wave walking the blocks in order."""
    rng = np.random.default_rng(45 + stride)
    a = (rng.standard_normal((5, 9, 4, 6)) * 1e-1).astype(np.float32)
    a[1:3] = 0.0  # zero blocks: one bit each
    for op in (orc.accuracy(1e-5), orc.precision(14), orc.expert(30, 600, 24, -20)):
        _check_vs_oracle(gc, orc, a, op, index_stride=stride)
