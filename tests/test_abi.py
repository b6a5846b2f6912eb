"""C-ABI boundary checks that need no GPU: libgcow.so loads, exports every symbol include/gcow.h declares, and the
host-side parts of the drop-in surface (parameters, descriptors, bit stream) behave as sw/ does."""
import ctypes as C
import subprocess

import numpy as np
import pytest

from gcow_amd import _ffi


@pytest.fixture(scope="module")
def L():
    return _ffi.load()


def test_exports_every_header_symbol(L):
    names = _ffi.header_functions()
    assert len(names) > 60
    out = subprocess.run(["nm", "-D", "--defined-only", _ffi.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert "PERM_2D" in exported
    for n in names:
        getattr(L, n)  # resolvable through ctypes


def test_no_torch_types_in_header():
    import re
    src = re.sub(r"/\*.*?\*/", "", open(_ffi.HEADER).read(), flags=re.S)
    for bad in ("torch", "at::", "hipStream_t", "#include <hip"):
        assert bad not in src


def test_accuracy_params(L):
    o = L.alloc_zfp_output()
    r = L.set_zfp_output_accuracy(o, 1e-3)  # sw/src/common.c:6-21
    assert (o.contents.minbits, o.contents.maxbits, o.contents.maxprec, o.contents.minexp) == (1, 16658, 64, -10)
    assert r == 2.0 ** -10
    L.set_zfp_output_accuracy(o, 1e-6)
    assert o.contents.minexp == -20
    assert L.set_zfp_output_rate(o, 16.0, 1) == 16.0
    assert (o.contents.minbits, o.contents.maxbits) == (64, 64)
    L.set_zfp_output_rate(o, 8.0, 3)
    assert (o.contents.minbits, o.contents.maxbits, o.contents.minexp) == (512, 512, -1074)
    assert L.set_zfp_output_precision(o, 20) == 20
    assert L.set_zfp_output_expert(o, 10, 5, 64, -10) == 0  # minbits > maxbits rejected, params kept
    assert o.contents.maxprec == 20
    L.free_zfp_output(o)


def test_descriptors(L):
    data = C.c_void_p(0)
    i2 = L.init_zfp_input(data, 3, C.c_uint(2), C.c_uint(5), C.c_uint(7))
    assert L.get_input_dimension(i2) == 2 and L.get_input_num_blocks(i2) == 4
    i1 = L.init_zfp_input(data, 3, C.c_uint(1), C.c_uint(10))  # 1-D extension
    assert L.get_input_dimension(i1) == 1 and L.get_input_num_blocks(i1) == 3
    i3 = L.init_zfp_input(data, 3, C.c_uint(3), C.c_uint(9), C.c_uint(10), C.c_uint(7))
    assert L.get_input_dimension(i3) == 3 and L.get_input_num_blocks(i3) == 3 * 3 * 2
    o = L.alloc_zfp_output()
    # sw/src/common.c:187-224 for a 2-D float array with default params: (148 + nb * (9 + 15 + 16*32)) -> bytes
    nb = 4
    assert L.get_max_output_bytes(o, i2) == ((148 + nb * (9 + 15 + 16 * 32) + 63) // 64 * 64) // 8
    assert L.get_precision(1, 64, -10, 2) == 17 and L.get_precision(-30, 64, -10, 2) == 0
    assert L.exceeded_maxbits(55, 64, 4) == 1 and L.exceeded_maxbits(16658, 17, 16) == 0
    for p in (i1, i2, i3):
        p.contents.data = None
        L.free_zfp_input(p)
    L.free_zfp_output(o)


def _py_stream_bits(chunks):
    """Reference model of LSB-first packing into 64-bit words (sw/src/stream.c:61-138)."""
    acc, pos = 0, 0
    for v, n in chunks:
        acc |= (v & ((1 << n) - 1)) << pos
        pos += n
    nw = (pos + 63) // 64
    return [(acc >> (64 * i)) & ((1 << 64) - 1) for i in range(nw)], pos


def test_bit_stream_roundtrip(L):
    rng = np.random.default_rng(0)
    buf = (C.c_uint64 * 512)()
    s = L.stream_init(C.cast(buf, C.c_void_p), C.sizeof(buf))
    chunks = []
    for _ in range(600):
        n = int(rng.integers(0, 65))
        v = int(rng.integers(0, 2 ** 63)) * 2 + int(rng.integers(0, 2))
        chunks.append((v, n))
        if n == 1 and rng.random() < 0.5:
            L.stream_write_bit(s, v & 1)
        else:
            L.stream_write_bits(s, v, n)
    words, pos = _py_stream_bits(chunks)
    assert L.stream_woffset(s) == pos
    L.stream_flush(s)
    assert L.stream_size_bytes(s) == 8 * len(words)
    assert [buf[i] for i in range(len(words))] == words
    L.stream_rewind(s)
    for v, n in chunks:
        got = L.stream_read_bits(s, n)
        assert got == (v & ((1 << n) - 1) if n < 64 else v & (2 ** 64 - 1))
    # seek / skip / align
    L.stream_rseek(s, 100)
    assert L.stream_roffset(s) == 100
    L.stream_skip(s, 28)
    assert L.stream_roffset(s) == 128
    L.stream_rseek(s, 130)
    L.stream_algin_next_word(s)
    assert L.stream_roffset(s) == 192


def test_field_of_rejects_expanded_views():
    """A broadcast / expanded view has stride 0 on a dimension of size > 1; the ABI reads a 0 stride as "dense"
    (sw/src/zfp.c:37-38), so passing it through would read past the tensor's storage: field_of refuses it,
    and accepts the same data once contiguous, and size-1 dimensions with any stride."""
    torch = pytest.importorskip("torch")
    from gcow_amd import codec
    base = torch.arange(16, dtype=torch.float32)
    with pytest.raises(codec.GcowError):
        codec.field_of(base.view(1, 16).expand(8, 16))
    with pytest.raises(codec.GcowError):
        codec.field_of(base[:1].expand(64))
    f = codec.field_of(base.view(1, 16).expand(8, 16).contiguous())
    assert (f.nx, f.ny, f.sx, f.sy) == (16, 8, 1, 16)
    g = codec.field_of(base.view(16, 1))  # size-1 dimension: its stride never matters
    assert (g.nx, g.ny) == (1, 16)
