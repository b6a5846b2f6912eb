/*
 * gcow.h -- MI355X-native ZFP-style gradient codec: the C ABI (libgcow.so).
 *
 * Part 1 is the drop-in boundary: the reference's sw/ encoder/decoder call surface with the same type layouts,
 * names, argument meaning and return values (fpgasystems/gcow sw/include/{types,zfp,stream,common}.h), each
 * declaration citing the reference interface it replaces. The codec behind it runs as hand-written CDNA4 (gfx950)
 * HIP kernels; there is no CPU codec in libgcow.so.
 *
 * Part 2 is the device API the drop-in layer is built on: device pointers, an explicit hipStream_t (passed as
 * void*), explicit status codes. No torch/HIP types appear in any signature.
 *
 * Deviations from sw/ (all documented in INTEGRATION.md):
 *   - 1-D (dim = 1) and 3-D inputs are supported (sw/ only encodes 2-D: sw/src/zfp.c:12-24, common.c:122-125).
 *   - data may be a device pointer; it is then encoded in place on the GPU. free_zfp_input() frees host data
 *     exactly as sw/ does (sw/src/common.c:54-62) but never frees device memory it does not own.
 *   - zfp_decompress() decodes with libzfp 0.5.5 semantics (block size 4^d); sw/'s decoder passes dim where the
 *     block size is needed (sw/src/decode.c:193-202) and is not reproduced.
 *   - dtype_bf16 (extension): bf16 values are widened exactly to fp32 and coded by the fp32 codec.
 *   - the library never prints (sw/src/common.c:109,190,193 do).
 */
#ifndef GCOW_H
#define GCOW_H

#include <stdarg.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ================================================================================================
 * Part 1 -- drop-in sw/ surface
 * ============================================================================================== */

/* sw/include/types.h:8-21 */
typedef unsigned char uchar;
typedef unsigned short ushort;
typedef unsigned int uint;
typedef unsigned long ulong;
typedef int8_t int8;
typedef uint8_t uint8;
typedef int16_t int16;
typedef uint16_t uint16;
typedef int32_t int32;
typedef uint32_t uint32;
typedef int64_t int64;
typedef uint64_t uint64;

/* sw/include/types.h:24 -- 64-bit stream words, bits appended LSB-first, words little-endian */
typedef uint64 stream_word;

/* sw/include/types.h:29-36 */
typedef enum {
  zfp_null = 0,
  zfp_expert = 1,
  zfp_fixed_rate = 2,
  zfp_fixed_precision = 3,
  zfp_fixed_accuracy = 4,
  zfp_reversible = 5
} zfp_mode;

/* sw/include/types.h:39-45 (+ dtype_bf16 extension) */
typedef enum {
  dtype_none = 0,
  dtype_int32 = 1,
  dtype_int64 = 2,
  dtype_float = 3,
  dtype_double = 4,
  dtype_bf16 = 5
} data_type;

/* sw/include/types.h:51-56 -- zero extents for unused dimensions, zero stride = contiguous a[nw][nz][ny][nx] */
typedef struct {
  data_type dtype;
  void* data;
  size_t nx, ny, nz, nw;
  ptrdiff_t sx, sy, sz, sw;
} zfp_input;

/* sw/include/stream.h:6-16 */
typedef struct stream stream;
struct stream {
  size_t buffered_bits;
  stream_word buffer;
  stream_word* begin;
  ptrdiff_t idx;
  ptrdiff_t end;
};

/* sw/include/types.h:58-65 */
typedef struct {
  uint minbits;
  uint maxbits;
  uint maxprec;
  int minexp;
  stream* data;
} zfp_output;

/* sw/include/common.h:10-13 */
#define ZFP_MIN_BITS 1
#define ZFP_MAX_BITS 16658
#define ZFP_MAX_PREC 64
#define ZFP_MIN_EXP -1074
#define ZFP_HEADER_MAX_BITS 148

/* ---- parameters / descriptors (sw/include/types.h:107-121, sw/src/common.c) ---- */
double set_zfp_output_accuracy(zfp_output* output, double tolerance);      /* common.c:6-21 */
zfp_input* alloc_zfp_input(void);                                           /* common.c:26-36 */
zfp_output* alloc_zfp_output(void);                                         /* common.c:41-52 */
void free_zfp_input(zfp_input* input);                                      /* common.c:54-62 */
void free_zfp_output(zfp_output* output);                                   /* common.c:64-75 */
void cleanup(zfp_input* input, zfp_output* output);                         /* common.c:77-81 */
zfp_input* init_zfp_input(void* data, data_type dtype, uint dim, ...);     /* common.c:83-103 (dim 1 added) */
zfp_output* init_zfp_output(const zfp_input* input);                        /* common.c:105-115 */
uint is_reversible(const zfp_output* output);                               /* common.c:117-120 */
uint get_input_dimension(const zfp_input* input);                           /* common.c:122-125 (1-D added) */
size_t get_input_num_blocks(const zfp_input* input);                        /* common.c:127-143 */
size_t get_input_size(const zfp_input* input, size_t* shape);               /* common.c:145-164 */
size_t get_dtype_size(data_type dtype);                                     /* common.c:166-180 */
uint get_input_precision(const zfp_input* input);                           /* common.c:182-185 */
size_t get_max_output_bytes(const zfp_output* output, const zfp_input* input); /* common.c:187-224 */
uint get_precision(int maxexp, uint maxprec, int minexp, int dim);          /* common.c:226-229 */
int exceeded_maxbits(uint maxbits, uint maxprec, uint size);                /* common.c:232-236 */

/* Extensions: the other libzfp 0.5.5 parameter setters (the Python caller uses rate / precision / accuracy,
 * hw/models/train_imagenet.py:459-464). */
double set_zfp_output_rate(zfp_output* output, double rate, uint dim);
uint set_zfp_output_precision(zfp_output* output, uint precision);
int set_zfp_output_expert(zfp_output* output, uint minbits, uint maxbits, uint maxprec, int minexp);

/* ---- array codec (sw/include/zfp.h:4-7, sw/src/zfp.c) ---- */
size_t zfp_compress(zfp_output* output, const zfp_input* input);            /* zfp.c:10-28 */
size_t zfp_decompress(zfp_output* output, const zfp_input* input);          /* zfp.c:58-76 */

/* ---- bit stream (sw/include/stream.h:18-33, sw/src/stream.c) ---- */
stream* stream_init(void* buffer, size_t bytes);                            /* stream.c:160-169 */
void stream_rewind(stream* s);                                              /* stream.c:153-158 */
size_t stream_size_bytes(const stream* s);                                  /* stream.c:176-179 */
size_t stream_flush(stream* s);                                             /* stream.c:132-138 */
uint64 stream_woffset(stream* s);                                           /* stream.c:141-144 */
uint64 stream_roffset(stream* s);                                           /* stream.c:147-150 */
void stream_pad(stream* s, uint64 n);                                       /* stream.c:121-129 */
stream_word stream_read_word(stream* s);                                    /* stream.c:6-15 */
void stream_write_word(stream* s, stream_word value);                       /* stream.c:18-26 */
uint64 stream_read_bits(stream* s, size_t n);                               /* stream.c:29-58 */
uint64 stream_write_bits(stream* s, uint64 value, size_t n);                /* stream.c:61-92 */
uint stream_read_bit(stream* s);                                            /* stream.c:95-106 */
uint stream_write_bit(stream* s, uint bit);                                 /* stream.c:109-118 */
void stream_rseek(stream* s, uint64 offset);                                /* stream.c:182-197 */
void stream_skip(stream* s, uint64 n);                                      /* stream.c:200-203 */
size_t stream_algin_next_word(stream* s);                                   /* stream.c:206-211 */

/* ---- block API (sw/include/encode.h:17-81, decode.h:8-12), batched onto the GPU stage kernels ---- */
void gather_2d_block(float* block, const float* raw, ptrdiff_t sx, ptrdiff_t sy);            /* encode.c:62-70 */
void gather_partial_2d_block(float* block, const float* raw, size_t nx, size_t ny, ptrdiff_t sx,
                             ptrdiff_t sy);                                                   /* encode.c:72-88 */
void gather_4d_block(float* block, const float* raw, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz,
                     ptrdiff_t sw);                                                           /* encode.c:90-99 */
void gather_partial_4d_block(float* block, const float* raw, size_t nx, size_t ny, size_t nz, size_t nw,
                             ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);        /* encode.c:101-126 */
int get_scaler_exponent(float x);                                           /* encode.c:128-140 */
int get_block_exponent(const float* block, uint n);                         /* encode.c:142-152 */
void fwd_cast_block(int32* iblock, const float* fblock, uint n, int emax); /* encode.c:178-187 */
void fwd_decorrelate_2d_block(int32* iblock);                               /* encode.c:251-260 */
void fwd_reorder_int2uint(uint32* ublock, const int32* iblock, const uchar* perm, uint n); /* encode.c:269-275 */
uint encode_all_bitplanes(stream* const s, const uint32* const ublock, uint maxprec, uint block_size);
                                                                            /* encode.c:343-408 */
uint encode_partial_bitplanes(stream* const s, const uint32* const ublock, uint maxbits, uint maxprec,
                              uint block_size);                             /* encode.c:279-339 */
uint encode_iblock(stream* const out_data, uint minbits, uint maxbits, uint maxprec, int32* iblock,
                   size_t dim);                                             /* encode.c:412-455 */
uint encode_fblock(zfp_output* output, const float* fblock, size_t dim);   /* encode.c:457-495 */
uint decode_fblock(zfp_output* output, float* fblock, size_t dim);         /* decode.c:220-253 */
void scatter_2d_block(const float* block, float* raw, ptrdiff_t sx, ptrdiff_t sy);           /* decode.c:27-34 */
void scatter_partial_2d_block(const float* block, float* raw, size_t nx, size_t ny, ptrdiff_t sx,
                              ptrdiff_t sy);                                                  /* decode.c:36-42 */

/* PERM_2D (sw/include/types.h:71-97) is exported as data for fwd_reorder_int2uint callers. */
extern const uchar PERM_2D[16];

/* ================================================================================================
 * Part 2 -- device API (what the drop-in layer and the Python/torch host binding call)
 * ============================================================================================== */

typedef enum {
  GCOW_OK = 0,
  GCOW_ERR_INVALID = 1,     /* bad arguments / parameters */
  GCOW_ERR_CAPACITY = 2,    /* output buffer smaller than the bound gcow_max_output_bytes() */
  GCOW_ERR_HIP = 3,         /* a HIP runtime call failed (gcow_last_error() has the text) */
  GCOW_ERR_NODEVICE = 4,    /* no gfx950 device / kernels not loadable */
  GCOW_ERR_UNSUPPORTED = 5  /* valid but not supported (e.g. int32/int64/double dtypes) */
} gcow_status;

/* The four ZFP expert parameters (sw/include/types.h:58-62). */
typedef struct {
  uint minbits, maxbits, maxprec;
  int minexp;
} gcow_params;

const char* gcow_status_string(gcow_status s);
const char* gcow_last_error(void);
const char* gcow_version(void);

/* Upper bound on the flushed stream for `field` under `p` (the sw/ bound without the 148-bit header term). */
size_t gcow_max_output_bytes(const zfp_input* field, const gcow_params* p);
/* Device scratch needed by gcow_encode_device (variable-rate passes); 0 for fixed rate. */
size_t gcow_encode_workspace_bytes(const zfp_input* field, const gcow_params* p);
/* Number of uint64 entries of the block-offset index written with `index_stride` (0 = no index). */
size_t gcow_index_entries(const zfp_input* field, uint32_t index_stride);

/*
 * Encode field->data (DEVICE pointer, fp32 or bf16, 1-4 dims, any element strides) into d_out (device).
 * The stream is byte-identical to sw/'s zfp_compress on the same values (headerless, LSB-first 64-bit words,
 * flushed with zero bits to a 64-bit boundary). *d_total_bits (device uint64, may be NULL) receives the unflushed
 * bit count. d_index (device, may be NULL) receives the bit offset of every index_stride-th block (1..256, power of
 * two), which gcow_decode_device uses to decode variable-rate streams in parallel.
 * Asynchronous with respect to the host on hip_stream (NULL = default stream); no host synchronisation.
 */
gcow_status gcow_encode_device(const zfp_input* field, const gcow_params* p, void* d_out, size_t out_capacity,
                               uint64_t* d_total_bits, void* d_workspace, size_t workspace_bytes,
                               uint64_t* d_index, uint32_t index_stride, void* hip_stream);

/*
 * Chunked encode of one variable-rate stream: append field's blocks to a stream whose first *d_base_bits bits (a
 * DEVICE uint64) are already in d_out, as sw/'s stream_write_bits appends at the stream's current position
 * (sw/src/stream.c:61-92), without the stream_flush padding a separate zfp_compress call would insert
 * (sw/src/zfp.c:10-28). Encoding an array in chunks this way is byte-identical to one gcow_encode_device call on
 * the whole array; *d_total_bits = *d_base_bits + the chunk's bits, so it is the next chunk's base. d_out must hold
 * the previous bits plus gcow_max_output_bytes(field, p) (only the latter is checked against out_capacity). Block
 * index entries (d_index) are absolute stream offsets. Fixed-rate streams are chunked by offsetting d_out on the
 * host instead (GCOW_ERR_UNSUPPORTED here).
 */
gcow_status gcow_encode_device_append(const zfp_input* field, const gcow_params* p, void* d_out, size_t out_capacity,
                                      const uint64_t* d_base_bits, uint64_t* d_total_bits, void* d_workspace,
                                      size_t workspace_bytes, uint64_t* d_index, uint32_t index_stride,
                                      void* hip_stream);

/*
 * Decode d_in into field->data (DEVICE fp32 pointer; for a 1-D field also dtype_bf16: the fp32 decode rounded to
 * nearest even, torch's conversion) with libzfp 0.5.5 semantics. Fixed-rate streams
 * (minbits == maxbits) decode one block per thread; variable-rate streams need the index written by
 * gcow_encode_device (d_index/index_stride), or, with d_index == NULL, are decoded by a single sequential GPU lane.
 * in_bytes may be the buffer's capacity; given the stream's own length (ceil(bits / 64) words), the 1-D
 * variable-rate decoder sizes its LDS stage from the stream's average bits per block (more waves for compressible
 * streams; the result is the same either way).
 */
gcow_status gcow_decode_device(const zfp_input* field, const gcow_params* p, const void* d_in, size_t in_bytes,
                               const uint64_t* d_index, uint32_t index_stride, void* hip_stream);

/*
 * Bit-stitch for sharded variable-rate streams: OR `src_bits` bits of d_src into d_dst starting at bit
 * `dst_bit_offset` (d_dst words covering the target range must be zero beyond what earlier shards wrote).
 * Used after an all-gather of per-rank shard streams to rebuild the single-stream sw/ layout.
 */
gcow_status gcow_stitch_device(uint64_t* d_dst, uint64_t dst_bit_offset, const uint64_t* d_src, uint64_t src_bits,
                               void* hip_stream);

/*
 * The whole receive side of a sharded variable-rate all-gather in one launch: nshards shard
 * streams of d_lens[r] bits (DEVICE uint64 array; the per-rank unflushed bit counts), stored shard_words apart from
 * d_src (the padded all-gather buffer), are concatenated bit-exactly -- shard r at bit d_lens[0] + ... + d_lens[r-1],
 * its flush padding dropped -- into d_dst, all of whose dst_words words are written (zero past the stream's end: the
 * single stream's flush). Equal to one gcow_encode_device of the unsharded bucket. d_dst needs no zeroing.
 */
gcow_status gcow_stitch_shards_device(uint64_t* d_dst, uint64_t dst_words, const uint64_t* d_src, uint64_t shard_words,
                                      const uint64_t* d_lens, uint32_t nshards, void* hip_stream);

/*
 * Decode-and-average of nstreams 1-D streams of one bucket shape (the compressed all-gather DDP hook's receive side;
 * hw/models/train_imagenet.py:446-475 is the caller contract): field->data (DEVICE, 1-D, fp32 or bf16) receives,
 * elementwise in fp32, ((0 + x_0) + x_1 + ... + x_{n-1}) / nstreams with x_r the libzfp decode of stream r (a bf16
 * field -- a bf16 gradient bucket -- receives that fp32 mean rounded to nearest even, torch's conversion). Streams start
 * stream_words words apart at d_streams; streams_bytes is the buffer's size, which must cover nstreams * stream_words
 * + 2 words (the decoders read 64-bit windows past a stream's last bit; GCOW_ERR_INVALID otherwise). Fixed rate: any
 * parameters, d_index NULL and index_words = index_stride = 0. Variable rate: any parameters (minbits <= 1,
 * maxbits >= 160 take the closed-form decoder, others the generic one) and every stream's block index (index_stride
 * 8 or 16, entries index_words apart at d_index, as gcow_encode_device writes them; or GCOW_INDEX_PACKED16, entries
 * as gcow_index_pack16_device writes them -- the size of the 16-block index, decoded in 8-block chunks).
 */
gcow_status gcow_decode_mean_device(const zfp_input* field, const gcow_params* p, const uint64_t* d_streams,
                                    size_t streams_bytes, uint64_t stream_words, uint32_t nstreams,
                                    const uint64_t* d_index, uint64_t index_words, uint32_t index_stride,
                                    void* hip_stream);

/*
 * Packed 16-block index (index_stride GCOW_INDEX_PACKED16 in gcow_decode_mean_device): one uint64 per 16 blocks, the
 * low 48 bits the stream bit position of block 16 c (as the index every 16 blocks holds it), the high 16 bits the
 * offset of block 16 c + 8 from it (0 where that block does not exist). It carries the 8-block chunk starts at the
 * 16-block index's size, so a receiver of every rank's index (the compressed all-gather hook) decodes in 8-block
 * chunks without the doubled index on the wire. gcow_index_pack16_device builds it on the device from the index every
 * 8 blocks of one stream of `field`'s shape (gcow_index_entries(field, 8) entries at d_index8) into
 * gcow_index_entries(field, 16) entries at d_out. GCOW_ERR_UNSUPPORTED when p lets 8 blocks exceed 65535 bits
 * (minbits > 8191) or the stream 2^48 bits; 1-D fields only.
 */
#define GCOW_INDEX_PACKED16 0x1010u
gcow_status gcow_index_pack16_device(const zfp_input* field, const gcow_params* p, const uint64_t* d_index8,
                                     uint64_t* d_out, void* hip_stream);

/*
 * zfp 0.5.5 stream header: the byte format zfpy.compress_numpy writes (hw/models/train_imagenet.py:459-465 calls
 * it), i.e. libzfp zfp_write_header(ZFP_HEADER_FULL): magic 'z','f','p' + codec version 5 (32 bits), field metadata
 * (52 bits: sizes, dims - 1, type - 1) and the compression mode (12-bit short form for rate / precision /
 * accuracy, else 64 bits). sw/ declares ZFP_HEADER_* (sw/include/common.h:16-21) but never writes a header.
 * Header metadata records zfp_type_float for fp32 and bf16 inputs (bf16 is coded by exact widening).
 */
uint gcow_header_bits(const gcow_params* p); /* 96 or 148 */
/* Host: write the header of (field shape, p) into words[0..3) (zeroed by the call); returns its bit count. */
uint gcow_write_header(const zfp_input* field, const gcow_params* p, uint64_t* words);
/* Host: parse a header (at least 3 words). Fills field->nx..nz and dtype (data/strides untouched) and p; returns
 * the header bit count, 0 when the magic or version does not match or the type is not float. */
uint gcow_read_header(const uint64_t* words, size_t nwords, zfp_input* field, gcow_params* p);
/* Workspace for gcow_encode_device_zfp: the headerless stream plus gcow_encode_workspace_bytes(). */
size_t gcow_encode_zfp_workspace_bytes(const zfp_input* field, const gcow_params* p);
/* Device encode to a header-prefixed stream (byte-identical to zfpy.compress_numpy). Capacity:
 * gcow_max_output_bytes() + 24. *d_total_bits (device, optional) = header bits + stream bits. */
gcow_status gcow_encode_device_zfp(const zfp_input* field, const gcow_params* p, void* d_out, size_t out_capacity,
                                   uint64_t* d_total_bits, void* d_workspace, size_t workspace_bytes,
                                   void* hip_stream);
/* Decode a stream whose first block starts at bit_offset (e.g. gcow_read_header()'s return value). */
gcow_status gcow_decode_device_at(const zfp_input* field, const gcow_params* p, const void* d_in, size_t in_bytes,
                                  uint64_t bit_offset, const uint64_t* d_index, uint32_t index_stride,
                                  void* hip_stream);

/* Per-stage batched device kernels (the hw/stages split, for parity bisection; sw/tests/test_stages.cpp). */
gcow_status gcow_stage_emax_device(const float* d_blocks, uint32_t nblocks, uint32_t dims, int32_t* d_emax,
                                   void* hip_stream);
gcow_status gcow_stage_cast_device(const float* d_blocks, const int32_t* d_emax, uint32_t nblocks, uint32_t dims,
                                   int32_t* d_iblocks, void* hip_stream);
gcow_status gcow_stage_xform_device(int32_t* d_iblocks, uint32_t nblocks, uint32_t dims, int inverse,
                                    void* hip_stream);
gcow_status gcow_stage_reorder_device(const int32_t* d_iblocks, uint32_t nblocks, uint32_t dims,
                                      uint32_t* d_ublocks, void* hip_stream);
/* Embedded coder on one ublock per lane, each into its own zeroed slot of slot_words words after `header_bits`
 * bits of header (value header); bits written per block to d_bits. */
gcow_status gcow_stage_encode_ints_device(const uint32_t* d_ublocks, uint32_t nblocks, uint32_t dims,
                                          uint32_t budget, uint32_t maxprec, uint64_t* d_slots, uint32_t slot_words,
                                          uint32_t* d_bits, void* hip_stream);

/* Measurement kernel (bench.py roofline.copy_ceiling): the fixed-rate 1-D encoder's memory access pattern without the
 * coding -- the same grid, loads of every full 4-value block (16 B fp32 / 8 B bf16) and one out_bits_per_block (32 or
 * 64) store per block -- i.e. the HBM floor that kernel can reach. Output bytes are not a stream. */
gcow_status gcow_copy_pattern_device(const void* d_in, int dtype, size_t nvals, uint32_t out_bits_per_block,
                                     void* d_out, void* hip_stream);

/* Deterministic synthetic gradient bucket on the device (bench / smoke inputs; SURVEY 8(d) distribution):
 * N(0, sigma) via counter-based splitmix64 + Box-Muller, with zero / tiny / subnormal 4-value blocks injected at
 * 1/64, 1/4096, 1/4096. */
gcow_status gcow_fill_normal_device(float* d_out, size_t count, double sigma, uint64_t seed, int inject,
                                    void* hip_stream);

/* TEST / MEASUREMENT ONLY -- not part of the drop-in surface. Selects a measured-and-not-kept form of the 1-D
 * variable-rate encoder for the whole process (bit-identical output; tests cover each form): form 0 = the tile form
 * (the default), 1 = count + scan + range coder, 2 = the decoupled look-back single pass; spin (form 2) = polls before
 * a missing predecessor's total is computed locally (< 0: default); stats != 0 (form 2) records look-back statistics.
 * No reference counterpart. */
gcow_status gcow_debug_set_var1d_variant(int form, int spin, int stats);

#ifdef __cplusplus
}
#endif
#endif /* GCOW_H */
