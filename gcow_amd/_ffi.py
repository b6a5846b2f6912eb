"""ctypes binding of libgcow.so (include/gcow.h).

This is the binding a Python caller of the reference would add: the reference's Python path (hw/models/*.py)
talks to zfpy; here the same flattened-gradient contract goes through the C ABI with device pointers.
The library is built in-tree (gcow_amd/lib/libgcow.so); importing fails loudly if it is missing -- there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "lib", "libgcow.so")
HEADER = os.path.join(ROOT, "include", "gcow.h")

# data_type (sw/include/types.h:39-45 + bf16)
DTYPE_NONE, DTYPE_INT32, DTYPE_INT64, DTYPE_FLOAT, DTYPE_DOUBLE, DTYPE_BF16 = 0, 1, 2, 3, 4, 5

GCOW_OK = 0
STATUS = {0: "ok", 1: "invalid argument", 2: "output capacity too small", 3: "HIP runtime error",
          4: "no usable gfx950 device", 5: "unsupported"}


class GcowError(RuntimeError):
    pass


class Stream(C.Structure):
    """struct stream (sw/include/stream.h:6-16)."""
    _fields_ = [("buffered_bits", C.c_size_t), ("buffer", C.c_uint64), ("begin", C.POINTER(C.c_uint64)),
                ("idx", C.c_ssize_t), ("end", C.c_ssize_t)]


class ZfpInput(C.Structure):
    """zfp_input (sw/include/types.h:51-56)."""
    _fields_ = [("dtype", C.c_int), ("data", C.c_void_p), ("nx", C.c_size_t), ("ny", C.c_size_t),
                ("nz", C.c_size_t), ("nw", C.c_size_t), ("sx", C.c_ssize_t), ("sy", C.c_ssize_t),
                ("sz", C.c_ssize_t), ("sw", C.c_ssize_t)]


class ZfpOutput(C.Structure):
    """zfp_output (sw/include/types.h:58-65)."""
    _fields_ = [("minbits", C.c_uint), ("maxbits", C.c_uint), ("maxprec", C.c_uint), ("minexp", C.c_int),
                ("data", C.POINTER(Stream))]


class GcowParams(C.Structure):
    _fields_ = [("minbits", C.c_uint), ("maxbits", C.c_uint), ("maxprec", C.c_uint), ("minexp", C.c_int)]

    def tuple(self):
        return (self.minbits, self.maxbits, self.maxprec, self.minexp)

    def __repr__(self):
        return "GcowParams(%d, %d, %d, %d)" % self.tuple()

    def __eq__(self, other):
        return self.tuple() == tuple(other.tuple() if hasattr(other, "tuple") else other)


_lib = None


def header_functions() -> list[str]:
    """Every function name declared in include/gcow.h."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src)
    skip = {"if", "defined", "sizeof", "extern", "while", "for", "switch", "return"}
    out = []
    for n in names:
        if n in skip or n.isupper():
            continue
        if n not in out:
            out.append(n)
    return out


def load():
    """Load libgcow.so (raises GcowError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GcowError("libgcow.so not built (%s); run __graft_entry__.build() or make -C gcow_amd/csrc" % LIB_PATH)
    # Share torch's HIP runtime when torch is importable (one runtime per process).
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
        pass
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    vp, sz, u32, u64, i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int
    pi, po, pp = P(ZfpInput), P(ZfpOutput), P(GcowParams)
    sig = {
        "gcow_status_string": (C.c_char_p, [i32]),
        "gcow_last_error": (C.c_char_p, []),
        "gcow_version": (C.c_char_p, []),
        "gcow_max_output_bytes": (sz, [pi, pp]),
        "gcow_encode_workspace_bytes": (sz, [pi, pp]),
        "gcow_index_entries": (sz, [pi, u32]),
        "gcow_encode_device": (i32, [pi, pp, vp, sz, vp, vp, sz, vp, u32, vp]),
        "gcow_encode_device_append": (i32, [pi, pp, vp, sz, vp, vp, vp, sz, vp, u32, vp]),
        "gcow_decode_device": (i32, [pi, pp, vp, sz, vp, u32, vp]),
        "gcow_stitch_device": (i32, [vp, u64, vp, u64, vp]),
        "gcow_stitch_shards_device": (i32, [vp, u64, vp, u64, vp, u32, vp]),
        "gcow_decode_mean_device": (i32, [pi, pp, vp, sz, u64, u32, vp, u64, u32, vp]),
        "gcow_index_pack16_device": (i32, [pi, pp, vp, vp, vp]),
        "gcow_header_bits": (C.c_uint, [pp]),
        "gcow_write_header": (C.c_uint, [pi, pp, P(u64)]),
        "gcow_read_header": (C.c_uint, [P(u64), sz, pi, pp]),
        "gcow_encode_zfp_workspace_bytes": (sz, [pi, pp]),
        "gcow_encode_device_zfp": (i32, [pi, pp, vp, sz, vp, vp, sz, vp]),
        "gcow_decode_device_at": (i32, [pi, pp, vp, sz, u64, vp, u32, vp]),
        "gcow_fill_normal_device": (i32, [vp, sz, C.c_double, u64, i32, vp]),
        "gcow_copy_pattern_device": (i32, [vp, i32, sz, u32, vp, vp]),
        "gcow_debug_set_var1d_variant": (i32, [i32, i32, i32]),
        "gcow_stage_emax_device": (i32, [vp, u32, u32, vp, vp]),
        "gcow_stage_cast_device": (i32, [vp, vp, u32, u32, vp, vp]),
        "gcow_stage_xform_device": (i32, [vp, u32, u32, i32, vp]),
        "gcow_stage_reorder_device": (i32, [vp, u32, u32, vp, vp]),
        "gcow_stage_encode_ints_device": (i32, [vp, u32, u32, u32, u32, vp, u32, vp, vp]),
        # drop-in sw/ surface
        "set_zfp_output_accuracy": (C.c_double, [po, C.c_double]),
        "set_zfp_output_rate": (C.c_double, [po, C.c_double, C.c_uint]),
        "set_zfp_output_precision": (C.c_uint, [po, C.c_uint]),
        "set_zfp_output_expert": (i32, [po, C.c_uint, C.c_uint, C.c_uint, i32]),
        "alloc_zfp_input": (pi, []),
        "alloc_zfp_output": (po, []),
        "free_zfp_input": (None, [pi]),
        "free_zfp_output": (None, [po]),
        "cleanup": (None, [pi, po]),
        "init_zfp_output": (po, [pi]),
        "is_reversible": (C.c_uint, [po]),
        "get_input_dimension": (C.c_uint, [pi]),
        "get_input_num_blocks": (sz, [pi]),
        "get_input_size": (sz, [pi, P(sz)]),
        "get_dtype_size": (sz, [i32]),
        "get_input_precision": (C.c_uint, [pi]),
        "get_max_output_bytes": (sz, [po, pi]),
        "get_precision": (C.c_uint, [i32, C.c_uint, i32, i32]),
        "exceeded_maxbits": (i32, [C.c_uint, C.c_uint, C.c_uint]),
        "zfp_compress": (sz, [po, pi]),
        "zfp_decompress": (sz, [po, pi]),
        "stream_init": (P(Stream), [vp, sz]),
        "stream_rewind": (None, [P(Stream)]),
        "stream_size_bytes": (sz, [P(Stream)]),
        "stream_flush": (sz, [P(Stream)]),
        "stream_woffset": (u64, [P(Stream)]),
        "stream_roffset": (u64, [P(Stream)]),
        "stream_pad": (None, [P(Stream), u64]),
        "stream_read_word": (u64, [P(Stream)]),
        "stream_write_word": (None, [P(Stream), u64]),
        "stream_read_bits": (u64, [P(Stream), sz]),
        "stream_write_bits": (u64, [P(Stream), u64, sz]),
        "stream_read_bit": (C.c_uint, [P(Stream)]),
        "stream_write_bit": (C.c_uint, [P(Stream), C.c_uint]),
        "stream_rseek": (None, [P(Stream), u64]),
        "stream_skip": (None, [P(Stream), u64]),
        "stream_algin_next_word": (sz, [P(Stream)]),
        "get_scaler_exponent": (i32, [C.c_float]),
        "get_block_exponent": (i32, [P(C.c_float), C.c_uint]),
        "fwd_cast_block": (None, [P(C.c_int32), P(C.c_float), C.c_uint, i32]),
        "fwd_decorrelate_2d_block": (None, [P(C.c_int32)]),
        "fwd_reorder_int2uint": (None, [P(C.c_uint32), P(C.c_int32), P(C.c_ubyte), C.c_uint]),
        "encode_all_bitplanes": (C.c_uint, [P(Stream), P(C.c_uint32), C.c_uint, C.c_uint]),
        "encode_partial_bitplanes": (C.c_uint, [P(Stream), P(C.c_uint32), C.c_uint, C.c_uint, C.c_uint]),
        "encode_iblock": (C.c_uint, [P(Stream), C.c_uint, C.c_uint, C.c_uint, P(C.c_int32), sz]),
        "encode_fblock": (C.c_uint, [po, P(C.c_float), sz]),
        "decode_fblock": (C.c_uint, [po, P(C.c_float), sz]),
        "gather_2d_block": (None, [P(C.c_float), P(C.c_float), C.c_ssize_t, C.c_ssize_t]),
        "gather_partial_2d_block": (None, [P(C.c_float), P(C.c_float), sz, sz, C.c_ssize_t, C.c_ssize_t]),
        "scatter_2d_block": (None, [P(C.c_float), P(C.c_float), C.c_ssize_t, C.c_ssize_t]),
        "scatter_partial_2d_block": (None, [P(C.c_float), P(C.c_float), sz, sz, C.c_ssize_t, C.c_ssize_t]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    # variadic: declare fixed part only
    L.init_zfp_input.restype = pi
    _lib = L
    return L


def check(status: int, what: str = "gcow"):
    if status != GCOW_OK:
        L = load()
        raise GcowError("%s failed: %s (%s)" % (what, STATUS.get(status, status), L.gcow_last_error().decode()))
