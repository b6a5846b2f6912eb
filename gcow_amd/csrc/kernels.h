// kernels.h -- host-visible kernel launch interface (internal to libgcow.so).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec_device.h"

namespace gcow {

// Field geometry as the kernels see it: extents/strides fastest-first, unused dims have extent 1.
struct FieldDesc {
  const void* data;  // input (encode) or output (decode) device pointer
  uint64_t n[4];
  int64_t s[4];
  uint32_t bx, by, bz, bw;
  uint32_t nblocks;
  uint32_t dims;
  uint32_t dtype;
  uint32_t vec;  // rows of 4 values are contiguous and vector-aligned
};

// Workgroup range decomposition for the tile kernels.
struct TilePlan {
  uint32_t threads;    // blocks per tile (= workgroup size)
  uint32_t range;      // blocks per workgroup range (multiple of threads)
  uint32_t nranges;    // grid size
  uint32_t lds_words;  // LDS window (32-bit words)
  bool fixed;          // minbits == maxbits: offsets are b * maxbits
};

hipError_t launch_encode_fixed1d(const void* in, int dtype, uint64_t nvals, uint32_t nblocks, const Params& p,
                                 void* out, void* stream);
hipError_t launch_encode_tiles(const FieldDesc& F, const Params& p, const TilePlan& plan, uint32_t* out32,
                               uint64_t* ws_sums, uint64_t* ws_base, uint64_t* d_total, uint64_t* index,
                               uint32_t index_shift, const uint64_t* d_base, void* stream);
// in_words: stream buffer size in uint64 (0 = unknown: no LDS staging)
hipError_t launch_decode(const FieldDesc& F, const Params& p, const uint64_t* in, const uint64_t* index,
                         uint32_t chunk, uint64_t nchunks, bool fixed, uint64_t base_bits, uint64_t* end_out,
                         void* stream, uint64_t in_words = 0);
// fixed-rate 1-D whole-word blocks (maxbits 64 / 32, maxprec >= 32, minexp <= -154), contiguous fp32 output,
// base_bits % 32 == 0
hipError_t launch_decode_fixed1d(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t base_bits,
                                 void* stream);
// fixed-rate 3-D blocks of a whole number of 32-bit words (fixed3d_ok); decode needs base_bits % 32 == 0
bool fixed3d_ok(uint32_t maxbits);
hipError_t launch_encode3d_fixed(const FieldDesc& F, const Params& p, uint32_t* out32, void* stream);
hipError_t launch_decode3d_fixed(const FieldDesc& F, const Params& p, const uint32_t* in32, void* stream);
// variable-rate 1-D, contiguous fp32 output, blocks never truncated (minbits <= 1, maxbits >= 160)
// in_words: stream buffer size (0 = unknown: no LDS staging)
hipError_t launch_decode1d_var(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t in_words,
                               const uint64_t* index, uint32_t chunk, uint64_t nchunks, uint64_t base_bits,
                               uint64_t* end_out, void* stream);
// 4-D blocks (one wave per block): lens (count pass), or write at rbase (variable) / b * maxbits (fixed, rbase null)
hipError_t launch_encode4d(const FieldDesc& F, const Params& p, uint32_t* lens, const uint64_t* rbase, uint32_t* out32,
                           uint64_t* index, uint32_t index_shift, void* stream);
hipError_t launch_decode4d(const FieldDesc& F, const Params& p, const uint64_t* in, const uint64_t* index,
                           uint64_t base_bits, void* stream);
hipError_t launch_decode4d_seq(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t base_bits,
                               uint64_t* end, void* stream);
hipError_t launch_scan_blocks(const uint32_t* lens, uint32_t nblocks, uint64_t* sums, uint64_t* base, uint64_t* total,
                              uint32_t* out32, void* stream);
// 2-D / 3-D tiles (gcow_blocks.hip); launch_encode_tiles forwards d >= 2 here
hipError_t launch_encode_tiles23(const FieldDesc& F, const Params& p, const TilePlan& plan, uint32_t* out32,
                                 uint64_t* ws_sums, uint64_t* ws_base, uint64_t* d_total, uint64_t* index,
                                 uint32_t index_shift, const uint64_t* d_base, void* stream);
// gsums (optional): totals of consecutive groups of 8 ranges, which the many-workgroup scan sums instead of the ranges
hipError_t launch_scan_ranges(const uint64_t* sums, uint32_t nranges, uint64_t* base, uint64_t* total, uint32_t* out32,
                              const uint64_t* d_base, void* stream, const uint64_t* gsums = nullptr);
hipError_t launch_set_u64(uint64_t* p, uint64_t v, void* stream);
// Single-pass 1-D variable-rate encoder (var1d.hip): minbits <= 1, maxbits >= 160; ws = var1d_sp_workspace_bytes().
size_t var1d_sp_workspace_bytes(uint64_t nblocks);
// A/B variants of the 1-D variable-rate encoder, for tests and measurement tools only (set through the C ABI's
// gcow_debug_set_var1d_variant; the product default is the tile form): form 0 = tile, 1 = range (count + scan +
// k_encode1d_var), 2 = the look-back single pass; spin = polls before a missing predecessor's total is computed
// locally (< 0: V1SPIN); stats != 0: the look-back records its statistics in the workspace.
struct Var1dVariant {
  int form, spin, stats;
};
extern Var1dVariant g_var1d_variant;

hipError_t launch_encode1d_var_sp(const FieldDesc& F, const Params& p, uint32_t* out32, uint64_t* ws,
                                  uint64_t* d_total, uint64_t* index, uint32_t index_shift, const uint64_t* d_base,
                                  void* stream);
// The default 1-D variable-rate form (var1d.hip): count per tile + scan + the tile coder placed by the scan;
// ws = var1d_tile_workspace_bytes().
size_t var1d_tile_workspace_bytes(uint64_t nblocks);
hipError_t launch_encode1d_var_tile(const FieldDesc& F, const Params& p, uint32_t* out32, uint64_t* ws,
                                    uint64_t* d_total, uint64_t* index, uint32_t index_shift, const uint64_t* d_base,
                                    void* stream);
hipError_t launch_copy_pattern1d(const void* in, int dtype, uint64_t nvals, uint32_t wb, void* out, void* stream);
// *flag = 0, then 1 if a[i] != b[i] for any i < n
hipError_t launch_words_differ(const uint64_t* a, const uint64_t* b, uint64_t n, uint64_t* flag, void* stream);
hipError_t launch_prepend_header(uint64_t* dst, uint32_t off, const uint64_t* src, const uint64_t* d_bits,
                                 const uint64_t* header, uint64_t max_words, uint64_t* d_total, void* stream);
hipError_t launch_stitch(uint64_t* dst, uint64_t off, const uint64_t* src, uint64_t bits, void* stream);
// all shards of a sharded variable-rate stream in one launch (dst written whole: no zeroing needed)
hipError_t launch_stitch_shards(uint64_t* dst, uint64_t dst_words, const uint64_t* src, uint64_t shard_words,
                                const uint64_t* lens, uint32_t nshards, void* stream);
// GCOW_INDEX_PACKED16 (include/gcow.h): one uint64 per 16 blocks, the 8-block midpoint as a 16-bit offset on top
constexpr uint32_t kIndexPacked16 = 0x1010u;
// packed16 index (ceil(n8 / 2) entries) from an index every 8 blocks (n8 entries)
hipError_t launch_index_pack16(const uint64_t* idx8, uint64_t n8, uint64_t* out, void* stream);
// mean of nstreams 1-D streams (fixed rate: any params; variable: any params, index every 8 or 16 blocks or packed16)
hipError_t launch_decode_mean1d(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t stream_words,
                                uint32_t nstreams, const uint64_t* index, uint64_t index_words, void* stream,
                                uint32_t chunk = 16);  // chunk: variable rate's index stride, 8 or 16, or kIndexPacked16
hipError_t launch_stage(int which, int dims, const void* a, const void* b, uint32_t n, void* out, uint32_t x0,
                        uint32_t x1, void* out2, uint32_t slot_words, void* stream);
hipError_t launch_fill_normal(float* out, uint64_t count, double sigma, uint64_t seed, int inject, void* stream);

}  // namespace gcow
