/*
 * zfp_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * CPU restatement of the gcow sw/ encoder/decoder (fpgasystems/gcow, sw/src/{encode,decode,stream,common,zfp}.c),
 * generalised to d = 1, 2, 3, 4 exactly as LLNL zfp 0.5.5 does (the library sw/ is byte-identical to).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product path (gcow_amd/, libgcow.so) never links or calls it.
 *
 * Parity pins: the reference's own golden streams (the compressed_2d_<n>.zfp files under sw/tests/data and hw/tests/data; via SHA-256
 * manifest in tests/golden/), sw/tests/test_stages.cpp known answers, hw/tests/test_encblock.cpp known answer, the
 * reference sw/ sources compiled into oracle/_ref (2-D), and libzfp 0.5.5 generated fixtures (1-D/3-D/4-D/decode).
 */
#ifndef GCOW_ZFP_ORACLE_H
#define GCOW_ZFP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dtype codes shared with include/gcow.h (gcow_dtype) */
#define ORC_F32 3
#define ORC_BF16 5

typedef struct {
  unsigned minbits, maxbits, maxprec;
  int minexp;
} orc_params;

/* ---- per-stage functions (sw/src/encode.c) ---- */
int orc_block_exponent(const float* block, unsigned n);                   /* encode.c:128-152 */
void orc_fwd_cast(int32_t* iblock, const float* fblock, unsigned n, int emax); /* encode.c:162-187 */
void orc_fwd_xform(int32_t* iblock, unsigned dims);                       /* encode.c:189-260 (+1-D/3-D per zfp) */
void orc_inv_xform(int32_t* iblock, unsigned dims);                       /* decode.c:58-111 (+1-D/3-D) */
void orc_fwd_reorder(uint32_t* ublock, const int32_t* iblock, unsigned dims); /* encode.c:263-275 */
const unsigned char* orc_perm(unsigned dims);                             /* types.h:71-97 PERM_2D, identity, PERM_3, PERM_4 */
/* Embedded bit-plane coder (encode.c:279-408). Appends to a word buffer at bit offset *pos; returns bits written. */
unsigned orc_encode_ints(uint64_t* words, uint64_t* pos, const uint32_t* ublock, unsigned maxbits,
                         unsigned maxprec, unsigned size);
/* encode_iblock (encode.c:412-455): xform + reorder + coder + pad to minbits. */
unsigned orc_encode_iblock(uint64_t* words, uint64_t* pos, unsigned minbits, unsigned maxbits,
                           unsigned maxprec, int32_t* iblock, unsigned dims);
/* encode_fblock (encode.c:457-495) */
unsigned orc_encode_fblock(uint64_t* words, uint64_t* pos, const orc_params* p, const float* fblock, unsigned dims);
/* gather with partial-block padding (encode.c:41-126) */
void orc_gather_block(float* block, const void* data, int dtype, unsigned dims,
                      const size_t* n, const ptrdiff_t* s, const size_t* b);
unsigned orc_precision(int emax, unsigned maxprec, int minexp, unsigned dims); /* common.c:226-229 */

/* ---- array driver (zfp.c:10-56, generalised) ---- */
size_t orc_num_blocks(unsigned dims, const size_t* n);
/* Returns total bits written (unflushed); stream = ceil(bits/64) words. out must be zero-initialised by callee. */
uint64_t orc_compress(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                      const orc_params* p, uint64_t* out, size_t out_words);
/* Threaded CPU baseline: block-aligned shards encoded into private streams, then serial bit-stitch. */
uint64_t orc_compress_mt(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                         const orc_params* p, uint64_t* out, size_t out_words, int nthreads);
/* The same, with each shard's first bit in shard_off[0 .. T] (T = min(nthreads, nblocks); shard_off[T] = end). */
uint64_t orc_compress_mt_off(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                             const orc_params* p, uint64_t* out, size_t out_words, int nthreads, uint64_t* shard_off);
/* Per-block bit lengths (for offset checks). */
void orc_block_bits(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                    const orc_params* p, uint32_t* bits_out);
/* Decoder with libzfp 0.5.5 semantics (block size 4^d; sw/src/decode.c:113-253 with the block-size fix). Returns bits read. */
uint64_t orc_decompress(float* data, unsigned dims, const size_t* n, const ptrdiff_t* s, const orc_params* p,
                        const uint64_t* in, size_t in_words);

uint64_t orc_decompress_at(float* data, unsigned dims, const size_t* n, const ptrdiff_t* s, const orc_params* p,
                           const uint64_t* in, size_t in_words, uint64_t start_bit);
/* Threaded decode over the shards of orc_compress_mt_off (shard_off NULL: fixed rate). */
uint64_t orc_decompress_mt(float* data, unsigned dims, const size_t* n, const ptrdiff_t* s, const orc_params* p,
                           const uint64_t* in, size_t in_words, int nthreads, const uint64_t* shard_off);
/* OR `bits` bits of src into zeroed out[] at bit offset off (the multi-shard stream stitch). */
void orc_stitch(uint64_t* out, uint64_t off, const uint64_t* src, uint64_t bits);

/* ---- zfp 0.5.5 stream header (zfp_write_header / zfp_read_header, ZFP_HEADER_FULL) ---- */
unsigned orc_header_bits(const orc_params* p);  /* 96 (short mode) or 148 */
unsigned orc_write_header(uint64_t* words, unsigned dims, const size_t* n, unsigned zfp_type, const orc_params* p);
unsigned orc_read_header(const uint64_t* words, unsigned* dims, size_t* n, unsigned* zfp_type, orc_params* p);

/* ---- parameter helpers (common.c:6-21 accuracy; libzfp set_rate / set_precision) ---- */
void orc_set_accuracy(orc_params* p, double tol);
void orc_set_rate(orc_params* p, double rate, unsigned dims);
void orc_set_precision(orc_params* p, unsigned prec);

/* ---- deterministic inputs ---- */
void orc_gen_bump2d(float* out, size_t n, int f32sum);             /* sw/tests/test_zfp.cpp:13-25 */
void orc_gen_normal(float* out, size_t count, double sigma, uint64_t seed, int inject); /* splitmix64 + Box-Muller */

#ifdef __cplusplus
}
#endif
#endif
