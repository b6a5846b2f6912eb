"""Host-side API over libgcow.so for device-resident torch tensors.

Mirrors the reference's codec interface (fpgasystems/gcow sw/include/types.h + zfp.h): the four expert parameters
(minbits, maxbits, maxprec, minexp) and the accuracy / rate / precision setters, `encode` = zfp_compress
(sw/src/zfp.c:10-28) and `decode` = zfp_decompress with libzfp 0.5.5 semantics. torch is used only for device
memory and streams; every byte of codec work runs in the gfx950 kernels of gcow_amd/csrc.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import math
from dataclasses import dataclass

import torch

from ._ffi import DTYPE_BF16, DTYPE_FLOAT, GcowError, GcowParams, ZfpInput, check, load

ZFP_MIN_BITS, ZFP_MAX_BITS, ZFP_MAX_PREC, ZFP_MIN_EXP = 1, 16658, 64, -1074
# index_stride of decode_mean for the packed 16-block index (include/gcow.h GCOW_INDEX_PACKED16)
INDEX_PACKED16 = 0x1010


# ------------------------------------------------------------------------------------------- parameters
def accuracy(tolerance: float) -> GcowParams:
    """set_zfp_output_accuracy (sw/src/common.c:6-21)."""
    emin = ZFP_MIN_EXP
    if tolerance > 0:
        _, e = math.frexp(tolerance)
        emin = e - 1
    return GcowParams(ZFP_MIN_BITS, ZFP_MAX_BITS, ZFP_MAX_PREC, emin)


def rate(bits_per_value: float, dims: int) -> GcowParams:
    """libzfp 0.5.5 zfp_stream_set_rate (float, no write-random-access): minbits = maxbits = floor(4^d r + 0.5)."""
    n = 1 << (2 * dims)
    bits = max(int(math.floor(n * bits_per_value + 0.5)), 9)
    return GcowParams(bits, bits, ZFP_MAX_PREC, ZFP_MIN_EXP)


def precision(prec: int) -> GcowParams:
    """libzfp 0.5.5 zfp_stream_set_precision."""
    p = min(prec, ZFP_MAX_PREC) if prec else ZFP_MAX_PREC
    return GcowParams(ZFP_MIN_BITS, ZFP_MAX_BITS, p, ZFP_MIN_EXP)


def expert(minbits: int, maxbits: int, maxprec: int, minexp: int) -> GcowParams:
    return GcowParams(minbits, maxbits, maxprec, minexp)


def is_fixed(p: GcowParams) -> bool:
    return p.minbits == p.maxbits


# ------------------------------------------------------------------------------------------- fields
def field_of(t: torch.Tensor, dims: int | None = None) -> ZfpInput:
    """zfp_input for a 1-4 dim tensor (numpy order: the last axis is x, the fastest)."""
    if t.dim() < 1 or t.dim() > 4:
        raise GcowError("tensors of 1-4 dims are supported, got %d" % t.dim())
    if t.dtype == torch.float32:
        dt = DTYPE_FLOAT
    elif t.dtype == torch.bfloat16:
        dt = DTYPE_BF16
    else:
        raise GcowError("dtype %s not supported (float32, bfloat16)" % t.dtype)
    f = ZfpInput()
    f.dtype = dt
    f.data = t.data_ptr()
    shp = list(reversed(t.shape))
    st = list(reversed(t.stride()))
    names_n = ["nx", "ny", "nz", "nw"]
    names_s = ["sx", "sy", "sz", "sw"]
    for i in range(t.dim()):
        if st[i] == 0 and shp[i] > 1:
            # an expanded / broadcast view: the ABI reads stride 0 as "dense" (sw/src/zfp.c:37-38), which would walk
            # past the tensor's storage
            raise GcowError("stride 0 on a dimension of size %d (expanded view): pass t.contiguous()" % shp[i])
        setattr(f, names_n[i], int(shp[i]))
        setattr(f, names_s[i], int(st[i]))
    return f


def _stream_ptr(stream) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def max_output_bytes(shape, p: GcowParams, dtype=torch.float32) -> int:
    t = torch.empty(0)
    f = ZfpInput()
    f.dtype = DTYPE_FLOAT if dtype == torch.float32 else DTYPE_BF16
    shp = list(reversed(shape))
    for i, n in enumerate(shp):
        setattr(f, ["nx", "ny", "nz", "nw"][i], int(n))
    del t
    return load().gcow_max_output_bytes(C.byref(f), C.byref(p))


@dataclass
class Encoded:
    """A compressed stream on the device: `words` (int64 tensor holding little-endian uint64 stream words),
    `bits_dev` (int64[1] device tensor with the unflushed bit count), optional block `index` for parallel decode."""
    words: torch.Tensor
    bits_dev: torch.Tensor
    shape: tuple
    params: GcowParams
    index: torch.Tensor | None = None
    index_stride: int = 0

    @property
    def bits(self) -> int:
        return int(self.bits_dev.item())

    @property
    def nwords(self) -> int:
        return (self.bits + 63) // 64

    def stream(self) -> torch.Tensor:
        """The flushed stream: ceil(bits/64) words (sw/src/stream.c:132-138 + :176-179)."""
        return self.words[: self.nwords]

    def to_bytes(self) -> bytes:
        return self.stream().cpu().numpy().tobytes()


class Encoder:
    """Preallocated encoder for a fixed shape / dtype / params (bench and repeated-bucket use)."""

    def __init__(self, shape, dtype, params: GcowParams, device=None, index_stride: int = 0):
        self.L = load()
        self.shape = tuple(shape)
        self.dtype = dtype
        self.params = params
        self.device = torch.device(device or "cuda")
        f = field_of_shape(self.shape, dtype)
        self.cap = self.L.gcow_max_output_bytes(C.byref(f), C.byref(params))
        if self.cap == 0:
            raise GcowError("unsupported shape %s" % (self.shape,))
        self.words = torch.zeros((self.cap + 7) // 8, dtype=torch.int64, device=self.device)
        self.bits_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.fixed = is_fixed(params)
        if self.fixed:  # fixed rate: the bit count is known on the host; no device write per call
            nb = 1
            for n in self.shape:
                nb *= (n + 3) // 4
            self.bits_dev.fill_(nb * params.maxbits)
        ws = self.L.gcow_encode_workspace_bytes(C.byref(f), C.byref(params))
        self.ws = torch.zeros(max(ws // 8, 1), dtype=torch.int64, device=self.device)
        self.ws_bytes = ws
        self.index_stride = index_stride
        ne = self.L.gcow_index_entries(C.byref(f), index_stride) if index_stride else 0
        self.index = torch.zeros(max(ne, 1), dtype=torch.int64, device=self.device) if index_stride else None

    def __call__(self, x: torch.Tensor, stream=None) -> Encoded:
        if tuple(x.shape) != self.shape or x.dtype != self.dtype:
            raise GcowError("Encoder built for %s %s, got %s %s" % (self.shape, self.dtype, tuple(x.shape), x.dtype))
        if not x.is_cuda:
            raise GcowError("Encoder expects a device tensor")
        f = field_of(x)
        st = self.L.gcow_encode_device(C.byref(f), C.byref(self.params), self.words.data_ptr(), self.cap,
                                       None if self.fixed else self.bits_dev.data_ptr(), self.ws.data_ptr(),
                                       self.ws_bytes,
                                       self.index.data_ptr() if self.index is not None else None,
                                       self.index_stride, _stream_ptr(stream))
        check(st, "gcow_encode_device")
        return Encoded(self.words, self.bits_dev, self.shape, self.params, self.index, self.index_stride)


def field_of_shape(shape, dtype) -> ZfpInput:
    f = ZfpInput()
    f.dtype = DTYPE_BF16 if dtype == torch.bfloat16 else DTYPE_FLOAT
    for i, n in enumerate(reversed(tuple(shape))):
        setattr(f, ["nx", "ny", "nz", "nw"][i], int(n))
    return f


def encode(x: torch.Tensor, params: GcowParams, index_stride: int = 0, stream=None) -> Encoded:
    """zfp_compress of a device tensor (1-4 dims, fp32 or bf16, any strides)."""
    if not x.is_cuda:
        raise GcowError("encode expects a device tensor (host arrays: the sw/ drop-in zfp_compress in libgcow.so, see INTEGRATION.md; or codec.HostEncoder for a pinned 1-D bucket)")
    enc = Encoder(x.shape, x.dtype, params, x.device, index_stride)
    L = enc.L
    f = field_of(x)
    st = L.gcow_encode_device(C.byref(f), C.byref(params), enc.words.data_ptr(), enc.cap, enc.bits_dev.data_ptr(),
                              enc.ws.data_ptr(), enc.ws_bytes,
                              enc.index.data_ptr() if enc.index is not None else None, index_stride,
                              _stream_ptr(stream))
    check(st, "gcow_encode_device")
    return Encoded(enc.words, enc.bits_dev, tuple(x.shape), params, enc.index, index_stride)


def decode(enc_or_words, shape=None, params: GcowParams | None = None, index: torch.Tensor | None = None,
           index_stride: int = 0, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """zfp_decompress (libzfp 0.5.5 semantics) into an fp32 device tensor, or into `out` (fp32; a 1-D out may be bf16:
    the fp32 decode rounded to nearest even, as `.to(torch.bfloat16)`)."""
    if isinstance(enc_or_words, Encoded):
        e = enc_or_words
        words, shape, params = e.words, e.shape, e.params
        if index is None and e.index is not None:
            index, index_stride = e.index, e.index_stride
    else:
        words = enc_or_words
    if out is None:
        out = torch.empty(tuple(shape), dtype=torch.float32, device=words.device)
    f = field_of(out)
    L = load()
    st = L.gcow_decode_device(C.byref(f), C.byref(params), words.data_ptr(), words.numel() * 8,
                              index.data_ptr() if index is not None else None, index_stride, _stream_ptr(stream))
    check(st, "gcow_decode_device")
    return out


def stitch(dst: torch.Tensor, dst_bit_offset: int, src: torch.Tensor, src_bits: int, stream=None):
    """OR src_bits bits of src into dst at dst_bit_offset (device words; dst zeroed beyond earlier content)."""
    L = load()
    check(L.gcow_stitch_device(dst.data_ptr(), dst_bit_offset, src.data_ptr(), src_bits, _stream_ptr(stream)),
          "gcow_stitch_device")


def stitch_shards(dst: torch.Tensor, src: torch.Tensor, shard_words: int, lens: torch.Tensor, stream=None):
    """Concatenate len(lens) shard streams (lens: int64 device tensor of bit counts; shard r at src[r * shard_words:])
    bit-exactly into dst (every word of dst is written; one launch, no host sync)."""
    n = lens.numel()
    if src.numel() < n * shard_words:
        raise GcowError("stitch_shards: src holds %d words, %d shards of %d expected" % (src.numel(), n, shard_words))
    check(load().gcow_stitch_shards_device(dst.data_ptr(), dst.numel(), src.data_ptr(), shard_words, lens.data_ptr(),
                                           n, _stream_ptr(stream)), "gcow_stitch_shards_device")
    return dst


def decode_mean(streams: torch.Tensor, stream_words: int, nstreams: int, n: int, params: GcowParams,
                index: torch.Tensor | None = None, index_words: int = 0, index_stride: int = 0,
                out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Mean of the decodes of nstreams 1-D streams of n values (stream r at streams[r * stream_words:], 2 readable
    words after the last one), accumulated in rank order in fp32 (gcow_decode_mean_device): one launch."""
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=streams.device)
    f = field_of(out)
    check(load().gcow_decode_mean_device(C.byref(f), C.byref(params), streams.data_ptr(), streams.numel() * 8,
                                         stream_words, nstreams,
                                         index.data_ptr() if index is not None else None, index_words, index_stride,
                                         _stream_ptr(stream)), "gcow_decode_mean_device")
    return out


def pack_index16(index8: torch.Tensor, n: int, params: GcowParams, out: torch.Tensor | None = None,
                 stream=None) -> torch.Tensor:
    """The packed 16-block index (gcow_index_pack16_device) of one stream of n values from its index every 8 blocks:
    ceil(n / 64) int64 entries, low 48 bits block 16 c's bit position, high 16 bits block 16 c + 8's offset from it.
    decode_mean(..., index_stride=INDEX_PACKED16) reads it as 8-block chunks."""
    n16 = (n + 63) // 64
    if out is None:
        out = torch.empty(max(n16, 1), dtype=torch.int64, device=index8.device)
    if out.numel() < n16 or index8.numel() < (n + 31) // 32 or not (index8.is_cuda and out.is_cuda):
        raise GcowError("pack_index16: device index of ceil(n / 32) entries and an output of ceil(n / 64)")
    f = field_of_shape((n,), torch.float32)
    check(load().gcow_index_pack16_device(C.byref(f), C.byref(params), index8.data_ptr(), out.data_ptr(),
                                          _stream_ptr(stream)), "gcow_index_pack16_device")
    return out[:n16] if n16 else out[:0]


def fill_normal(out: torch.Tensor, sigma: float = 1e-3, seed: int = 0x67636F77, inject: bool = True, stream=None):
    """Deterministic synthetic gradient bucket on the device (SURVEY 8(d) distribution)."""
    assert out.dtype == torch.float32 and out.is_cuda and out.is_contiguous()
    check(load().gcow_fill_normal_device(out.data_ptr(), out.numel(), sigma, seed, int(inject),
                                         _stream_ptr(stream)), "gcow_fill_normal_device")
    return out


def copy_pattern(x: torch.Tensor, out: torch.Tensor, bits_per_block: int = 64, stream=None):
    """The fixed-rate 1-D encoder's memory access pattern without coding (gcow_copy_pattern_device): the HBM floor
    of that kernel, for bench.py's roofline.copy_ceiling."""
    dt = DTYPE_BF16 if x.dtype == torch.bfloat16 else DTYPE_FLOAT
    if not (x.is_cuda and x.is_contiguous()) or out.numel() * out.element_size() * 8 < x.numel() // 4 * bits_per_block:
        raise GcowError("copy_pattern: contiguous device input and an output of nblocks * bits_per_block bits")
    check(load().gcow_copy_pattern_device(x.data_ptr(), dt, x.numel(), bits_per_block, out.data_ptr(),
                                          _stream_ptr(stream)), "gcow_copy_pattern_device")
    return out


def c3_field(device=None, side: int = 512, seed: int = 21) -> torch.Tensor:
    """SURVEY 8(d) C3 volume on the device: f = sin(6 pi x) cos(4 pi y) sin(2 pi z) + 1e-3 N(0, 1) on the [0, 1)^3
    grid (z slowest), the noise from fill_normal. The bench times this field and the full-size parity test checks the
    same one (copied to the host) against the oracle."""
    import math as _m
    dev = torch.device(device or "cuda")
    g = torch.arange(side, device=dev, dtype=torch.float64) / side
    sx = torch.sin(6 * _m.pi * g).float()
    cy = torch.cos(4 * _m.pi * g).float()
    sz = torch.sin(2 * _m.pi * g).float()
    f = torch.empty(side ** 3, dtype=torch.float32, device=dev)
    fill_normal(f, 1.0, seed=seed, inject=False)
    f = f.view(side, side, side).mul_(1e-3)
    f += sx[None, None, :] * cy[None, :, None] * sz[:, None, None]
    return f.contiguous()


VAR1D_FORMS = {"tile": 0, "range": 1, "single_pass": 2}


@contextlib.contextmanager
def var1d_variant(form: str = "tile", spin: int = -1, stats: bool = False):
    """TEST / MEASUREMENT ONLY: run the 1-D variable-rate encoder in one of its measured-and-not-kept forms inside the
    `with` block (gcow_debug_set_var1d_variant; process-wide, restored to the default tile form on exit)."""
    L = load()
    check(L.gcow_debug_set_var1d_variant(VAR1D_FORMS[form], int(spin), int(bool(stats))),
          "gcow_debug_set_var1d_variant")
    try:
        yield
    finally:
        check(L.gcow_debug_set_var1d_variant(0, -1, 0), "gcow_debug_set_var1d_variant")


# ------------------------------------------------------------------------------------------- zfpy byte streams
def write_header(shape, params: GcowParams, dtype=torch.float32):
    """(header words [3 x uint64 as python ints], header bits) of zfp_write_header(ZFP_HEADER_FULL)."""
    f = field_of_shape(shape, dtype)
    w = (C.c_uint64 * 3)()
    bits = load().gcow_write_header(C.byref(f), C.byref(params), w)
    if not bits:
        raise GcowError("shape %s has no zfp header form" % (tuple(shape),))
    return [int(x) for x in w], int(bits)


def read_header(words):
    """Parse a zfp 0.5.5 header from the first words (host ints, numpy or a tensor) -> (shape, params, bits)."""
    if isinstance(words, torch.Tensor):
        words = words[:3].cpu().tolist()
    w = [int(x) & 0xFFFFFFFFFFFFFFFF for x in list(words)[:3]]
    w += [0] * (3 - len(w))
    arr = (C.c_uint64 * 3)(*w)
    f, p = ZfpInput(), GcowParams()
    bits = load().gcow_read_header(arr, 3, C.byref(f), C.byref(p))
    if not bits:
        raise GcowError("not a zfp 0.5.5 float stream (bad magic, version or type)")
    shape = tuple(n for n in (f.nw, f.nz, f.ny, f.nx) if n)
    return shape, p, int(bits)


def compress_numpy(x: torch.Tensor, tolerance: float = -1, rate: float = -1, precision: int = -1,
                   stream=None) -> torch.Tensor:
    """zfpy.compress_numpy for a device tensor: header + stream, byte-identical to zfpy/libzfp 0.5.5 (returned as an
    int64 device tensor of ceil(bits/64) words). Same keyword semantics as zfpy: exactly one of tolerance / rate /
    precision >= 0 selects the mode."""
    if tolerance >= 0:
        p = accuracy(tolerance)
    elif rate >= 0:
        p = globals()["rate"](rate, x.dim())
    elif precision >= 0:
        p = globals()["precision"](precision)
    else:
        p = expert(ZFP_MIN_BITS, ZFP_MAX_BITS - 1, ZFP_MAX_PREC, ZFP_MIN_EXP)  # zfpy default: lossless-ish expert
    return compress_zfp(x, p, stream)


def compress_zfp(x: torch.Tensor, params: GcowParams, stream=None) -> torch.Tensor:
    if not x.is_cuda:
        raise GcowError("compress_zfp expects a device tensor")
    L = load()
    f = field_of(x)
    cap = L.gcow_max_output_bytes(C.byref(f), C.byref(params)) + 24
    ws_bytes = L.gcow_encode_zfp_workspace_bytes(C.byref(f), C.byref(params))
    out = torch.zeros((cap + 7) // 8, dtype=torch.int64, device=x.device)
    ws = torch.zeros((ws_bytes + 7) // 8, dtype=torch.int64, device=x.device)
    bits = torch.zeros(1, dtype=torch.int64, device=x.device)
    check(L.gcow_encode_device_zfp(C.byref(f), C.byref(params), out.data_ptr(), cap, bits.data_ptr(), ws.data_ptr(),
                                   ws_bytes, _stream_ptr(stream)), "gcow_encode_device_zfp")
    return out[: (int(bits.item()) + 63) // 64]


def decompress_numpy(words: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """zfpy.decompress_numpy for a device stream with a zfp header: shape and mode come from the header."""
    shape, p, hb = read_header(words)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=words.device)
    elif tuple(out.shape) != shape:
        raise GcowError("output shape %s does not match the header's %s" % (tuple(out.shape), shape))
    w = torch.cat([words.reshape(-1), torch.zeros(2, dtype=torch.int64, device=words.device)])
    f = field_of(out)
    check(load().gcow_decode_device_at(C.byref(f), C.byref(p), w.data_ptr(), w.numel() * 8, hb, None, 0,
                                       _stream_ptr(stream)), "gcow_decode_device_at")
    return out


# ------------------------------------------------------------------------------------------- chunked / host paths
def encode_append(x: torch.Tensor, params: GcowParams, words: torch.Tensor, d_base: torch.Tensor,
                  d_total: torch.Tensor, ws: torch.Tensor | None = None, index: torch.Tensor | None = None,
                  index_stride: int = 0, stream=None):
    """Append a variable-rate encode of device tensor x to the stream in `words` whose first d_base[0] bits are
    already written (gcow_encode_device_append); d_total[0] receives the new end. d_base / d_total are int64 device
    tensors (one element each); chunks appended this way equal one encode of their concatenation."""
    L = load()
    f = field_of(x)
    need = L.gcow_encode_workspace_bytes(C.byref(f), C.byref(params))
    if ws is None or ws.numel() * 8 < need:
        ws = torch.empty(max(need // 8, 1), dtype=torch.int64, device=x.device)
    st = L.gcow_encode_device_append(C.byref(f), C.byref(params), words.data_ptr(), words.numel() * 8,
                                     d_base.data_ptr(), d_total.data_ptr(), ws.data_ptr(), ws.numel() * 8,
                                     index.data_ptr() if index is not None else None, index_stride,
                                     _stream_ptr(stream))
    check(st, "gcow_encode_device_append")
    return ws


class HostEncoder:
    """Encode a 1-D bucket that starts and ends in pinned host memory (the gradient bucket headed for the NIC,
    BASELINE config 5), with the PCIe copies overlapped: the bucket is cut into `chunks` block-aligned chunks and
    chunk i+1's H2D copy, chunk i's encode and chunk i-1's D2H copy run on three streams at once. Variable rate
    appends each chunk at the device-side end of the previous one (gcow_encode_device_append); fixed rate writes
    chunk i at its known word offset. Only whole 64-bit words that no later chunk touches are copied back early.
    The result is byte-identical to one device encode of the whole bucket."""

    def __init__(self, n: int, dtype, params: GcowParams, chunks: int = 8, device=None):
        self.n, self.dtype, self.params = int(n), dtype, params
        self.device = torch.device(device or "cuda")
        self.fixed = is_fixed(params)
        nb = (self.n + 3) // 4
        # chunks of a multiple of 16 blocks; fixed rate also needs every chunk to start on a 64-bit stream word
        # (written at a byte offset as its own stream): blocks * maxbits % 64 == 0
        align = 16
        if self.fixed:
            g = 64 // math.gcd(int(params.maxbits), 64)
            align = align * g // math.gcd(align, g)
        per = max(align, ((nb + chunks - 1) // chunks + align - 1) // align * align)
        self.bounds = []
        b = 0
        while b < nb:
            e = min(b + per, nb)
            self.bounds.append((4 * b, min(4 * e, self.n)))
            b = e
        self.L = load()
        self.cap = max_output_bytes((self.n,), params, dtype)
        self.words = torch.zeros((self.cap + 7) // 8 + 2, dtype=torch.int64, device=self.device)
        self.bufs = [torch.empty(4 * per, dtype=dtype, device=self.device) for _ in range(2)]
        f = field_of_shape((4 * per,), dtype)
        need = self.L.gcow_encode_workspace_bytes(C.byref(f), C.byref(params))
        self.ws = torch.empty(max(need // 8, 1), dtype=torch.int64, device=self.device)
        k = len(self.bounds)
        self.d_bits = torch.zeros(k + 1, dtype=torch.int64, device=self.device)
        self.h_bits = torch.zeros(k + 1, dtype=torch.int64).pin_memory()
        self.s_h2d, self.s_enc, self.s_d2h = (torch.cuda.Stream(self.device) for _ in range(3))

    def __call__(self, h_in: torch.Tensor, h_out: torch.Tensor) -> int:
        """h_in: pinned host 1-D tensor (n values); h_out: pinned host int64 tensor with room for the stream.
        Returns the stream's bit count; h_out[:ceil(bits / 64)] holds the flushed stream."""
        if h_in.numel() != self.n or h_in.dtype != self.dtype or h_in.is_cuda:
            raise GcowError("HostEncoder built for %d %s host values" % (self.n, self.dtype))
        p = self.params
        k = len(self.bounds)
        ev_h2d = [torch.cuda.Event() for _ in range(k)]
        ev_enc = [torch.cuda.Event() for _ in range(k)]
        done = 0  # words already copied back

        def copy_back(end_word, after):
            nonlocal done
            if end_word > done:
                self.s_d2h.wait_event(after)
                with torch.cuda.stream(self.s_d2h):
                    h_out[done:end_word].copy_(self.words[done:end_word], non_blocking=True)
                done = end_word

        for i, (lo, hi) in enumerate(self.bounds):
            buf = self.bufs[i % 2]
            if i >= 2:
                self.s_h2d.wait_event(ev_enc[i - 2])  # the buffer's previous chunk is encoded
            with torch.cuda.stream(self.s_h2d):
                buf[: hi - lo].copy_(h_in[lo:hi], non_blocking=True)
                ev_h2d[i].record(self.s_h2d)
            self.s_enc.wait_event(ev_h2d[i])
            x = buf[: hi - lo]
            if self.fixed:
                f = field_of(x)
                off = (lo // 4) * p.maxbits // 8
                check(self.L.gcow_encode_device(C.byref(f), C.byref(p), self.words.data_ptr() + off,
                                                self.cap - off, None, None, 0, None, 0,
                                                _stream_ptr(self.s_enc)), "gcow_encode_device")
            else:
                encode_append(x, p, self.words, self.d_bits[i:i + 1], self.d_bits[i + 1:i + 2], self.ws,
                              stream=self.s_enc)
                with torch.cuda.stream(self.s_enc):
                    self.h_bits[i + 1:i + 2].copy_(self.d_bits[i + 1:i + 2], non_blocking=True)
            ev_enc[i].record(self.s_enc)
            if i >= 1:  # chunk i-1's complete words (chunk i only ORs into the word its first bit falls in)
                if self.fixed:
                    end = (self.bounds[i - 1][1] + 3) // 4 * p.maxbits
                else:
                    ev_enc[i - 1].synchronize()
                    end = int(self.h_bits[i])
                copy_back(end // 64, ev_enc[i - 1])
        if self.fixed:
            bits = ((self.n + 3) // 4) * p.maxbits
        else:
            ev_enc[k - 1].synchronize()
            bits = int(self.h_bits[k])
        copy_back((bits + 63) // 64, ev_enc[k - 1])
        self.s_d2h.synchronize()
        return bits
