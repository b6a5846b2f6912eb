// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// extern "C" entry points over the reference sw/ sources compiled in place from /root/reference/sw/src
// (oracle/Makefile builds them into oracle/_ref/libgcow_ref.so; nothing from the reference is copied).
// sw/ is compiled as C++ (sw/Makefile:4,47-49), so its symbols are mangled; these wrappers give ctypes a C ABI.
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "encode.h"
#include "stream.h"
#include "types.h"
#include "zfp.h"

extern "C" {

// zfp_compress on a 2-D float array with explicit expert params (sw/src/zfp.c:10-56). Returns flushed bytes.
size_t gcow_ref_compress_2d(const float* data, size_t nx, size_t ny, unsigned minbits, unsigned maxbits,
                            unsigned maxprec, int minexp, uint64_t* out, size_t out_bytes)
{
  zfp_input* in = alloc_zfp_input();
  in->dtype = dtype_float;
  in->data = (void*)data;
  in->nx = nx;
  in->ny = ny;
  zfp_output* o = alloc_zfp_output();
  o->minbits = minbits;
  o->maxbits = maxbits;
  o->maxprec = maxprec;
  o->minexp = minexp;
  std::memset(out, 0, out_bytes);
  o->data = stream_init(out, out_bytes);
  size_t bytes = zfp_compress(o, in);
  std::free(o->data);
  std::free(o);
  std::free(in);  // not free_zfp_input: it would free the caller's data (sw/src/common.c:54-62)
  return bytes;
}

// set_zfp_output_accuracy (sw/src/common.c:6-21): writes the 4 expert params.
double gcow_ref_set_accuracy(double tol, unsigned* minbits, unsigned* maxbits, unsigned* maxprec, int* minexp)
{
  zfp_output* o = alloc_zfp_output();
  double r = set_zfp_output_accuracy(o, tol);
  *minbits = o->minbits;
  *maxbits = o->maxbits;
  *maxprec = o->maxprec;
  *minexp = o->minexp;
  std::free(o);
  return r;
}

int gcow_ref_block_exponent(const float* block, unsigned n) { return get_block_exponent(block, n); }

void gcow_ref_fwd_cast(int32_t* iblock, const float* fblock, unsigned n, int emax)
{
  fwd_cast_block(iblock, fblock, n, emax);
}

void gcow_ref_fwd_decorrelate_2d(int32_t* iblock) { fwd_decorrelate_2d_block(iblock); }

void gcow_ref_fwd_reorder_2d(uint32_t* ublock, const int32_t* iblock)
{
  uint32_t tmp[17];  // fwd_reorder_int2uint writes one element past n (sw/src/encode.c:272-274)
  fwd_reorder_int2uint(tmp, iblock, PERM_2D, 16);
  std::memcpy(ublock, tmp, 16 * sizeof(uint32_t));
}

// encode_iblock on a fresh stream (sw/src/encode.c:412-455); returns bits, stream words in out.
unsigned gcow_ref_encode_iblock(uint64_t* out, size_t out_bytes, unsigned header, unsigned minbits,
                                unsigned maxbits, unsigned maxprec, int32_t* iblock, uint64_t* total_bits)
{
  std::memset(out, 0, out_bytes);
  stream* s = stream_init(out, out_bytes);
  stream_write_bits(s, header, 9);
  unsigned bits = encode_iblock(s, minbits, maxbits, maxprec, iblock, 2);
  *total_bits = stream_woffset(s);
  stream_flush(s);
  std::free(s);
  return bits;
}

}  // extern "C"
