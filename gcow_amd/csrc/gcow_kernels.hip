// gcow_kernels.hip -- hand-written gfx950 kernels for the gcow codec path (no hipify, no CUDA shims).
//
// Kernel map (reference counterparts in fpgasystems/gcow):
//   k_encode_fixed1d   fused 1-D fixed-rate encoder, one 4-value block per lane, block b at bits [b*maxbits, ...)
//                      (sw/src/zfp.c:31-56 loop + sw/src/encode.c:41-495; hw/src/zfp.cpp:31-75 dataflow stages)
//   k_count            pass 1 of variable rate: per-block bit lengths reduced per workgroup range
//   k_scan_ranges      exclusive scan of the range totals, zeroes the words two ranges share
//   k_encode_tiles     pass 2 (and generic fixed rate): encode a tile of blocks per workgroup, assemble the
//                      variable-length codes in an LDS window (ds_or), store whole 32-bit words coalesced; only
//                      the first/last word of a range is shared and uses a global atomicOr
//                      (replaces hw/src/io.cpp:185-320 ordered burst writer)
//   k_decode           libzfp-semantics decoder, one block per lane (fixed rate) or one index chunk per lane
//   k_stitch           bit-stitch of a shard stream at an arbitrary bit offset (multi-GPU variable rate)
//   k_stage_*          per-stage kernels for parity bisection (hw/stages/*.cpp counterparts)
//   k_fill_normal      deterministic synthetic gradients
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "codec_device.h"
#include "kernels.h"
#include "lean1d.h"
#include "tiles.h"

namespace gcow {

// ------------------------------------------------------------------------------------------------ 1-D fast path
template <int DT>
__device__ __forceinline__ void load_block1d(const void* in, uint64_t nvals, uint32_t b, float* f)
{
  const uint64_t i0 = 4ull * b;
  if (i0 + 4 <= nvals) {
    load_row4<DT>(in, (int64_t)i0, f);
  } else {
    const uint32_t nv = (uint32_t)(nvals - i0);
#pragma unroll
    for (int x = 0; x < 4; x++) f[x] = load_elem<DT>(in, (int64_t)(i0 + pad_index(x, nv)));
  }
}

// Spread the low 16 bits of x to the even bit positions of a 32-bit word.
__device__ __forceinline__ uint32_t spread2_16(uint32_t x)
{
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}

// 4-way bit interleave of four 16-bit values: bit 4j + i of the result = bit j of value i.
__device__ __forceinline__ uint64_t interleave4_16(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
  const uint32_t P = spread2_16(a) | (spread2_16(c) << 1);  // a_j at 2j, c_j at 2j+1
  const uint32_t Q = spread2_16(b) | (spread2_16(d) << 1);  // b_j at 2j, d_j at 2j+1
  const uint32_t lo = spread2_16(P & 0xffffu) | (spread2_16(Q & 0xffffu) << 1);
  const uint32_t hi = spread2_16(P >> 16) | (spread2_16(Q >> 16) << 1);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// One 4-value block -> WB bits (WB = 32 or 64), header included (sw/src/encode.c:457-495 for d = 1).
// The embedded coder (encode.c:279-339) is evaluated in three closed-form phases from the coefficients' leading
// one-bit planes L_i (M0 = max L_i): planes above M0 are empty and cost one '0' bit each (n = 0); planes M0..L3
// run the group tests through the LDS plane table while n < 4; from plane L3 - 1 down every coefficient is
// significant (n = 4) and each plane is its 4 bits verbatim, i.e. a contiguous run of the 4-way interleave of the
// bit-reversed coefficients, built with shift/mask spreads instead of a per-plane loop.
template <uint32_t WB>
__device__ __forceinline__ uint64_t encode_block1d_fixed(const float* f, const Params& p, const uint16_t* tab)
{
  float fa[4] = {f[0], f[1], f[2], f[3]};
  const int emax = block_emax<4>(fa);
  const uint32_t prec = precision(emax, p.maxprec, p.minexp, 1);
  if (!prec || emax == -127) return 0ull;  // zero block: one 0 bit padded with zeros
  const float s = cast_scale(emax);
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = cast1(fa[i], s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  const int kmin = prec < 32 ? 32 - (int)prec : 0;
  uint64_t acc = 2ull * (uint32_t)(emax + 127) + 1ull;
  uint32_t pos = 9;
  {
    // leading one-bit plane of each coefficient (-1 for zero)
    const int L0 = 31 - (int)__builtin_clz(u[0] | 1u) - (u[0] ? 0 : 1);
    const int L1 = 31 - (int)__builtin_clz(u[1] | 1u) - (u[1] ? 0 : 1);
    const int L2 = 31 - (int)__builtin_clz(u[2] | 1u) - (u[2] ? 0 : 1);
    const int L3 = 31 - (int)__builtin_clz(u[3] | 1u) - (u[3] ? 0 : 1);
    const int M0 = max(max(L0, L1), max(L2, L3));
    // phase 1: empty planes 31 .. max(M0, kmin - 1) + 1, one '0' bit each
    const int top = max(M0, kmin - 1);
    pos += (uint32_t)(31 - top);
    // phase 2: group tests while n < 4 (planes top .. max(L3, kmin))
    uint32_t n = 0;
    const int glo = max(L3, kmin);
    for (int k = top; k >= glo && pos < WB; --k) {
      const uint32_t x = ((u[0] >> k) & 1u) | (((u[1] >> k) & 1u) << 1) | (((u[2] >> k) & 1u) << 2) |
                         (((u[3] >> k) & 1u) << 3);
      const uint32_t e = tab[(n << 4) | x];
      acc |= (uint64_t)(e & 127u) << pos;
      pos += (e >> 7) & 7u;
      n = e >> 10;
    }
    // phase 3: all significant: planes L3-1 .. kmin verbatim (at most 16 planes are ever needed here)
    const int kt = L3 - 1;
    if (pos < WB && kt >= kmin) {
      const uint32_t sh = (uint32_t)(31 - kt);
      const uint32_t g0 = __builtin_bitreverse32(u[0]) >> sh, g1 = __builtin_bitreverse32(u[1]) >> sh;
      const uint32_t g2 = __builtin_bitreverse32(u[2]) >> sh, g3 = __builtin_bitreverse32(u[3]) >> sh;
      uint64_t J = interleave4_16(g0 & 0xffffu, g1 & 0xffffu, g2 & 0xffffu, g3 & 0xffffu);
      const uint32_t cnt = (uint32_t)(kt - kmin + 1);  // planes available
      if (cnt < 16) J &= (1ull << (4 * cnt)) - 1ull;
      acc |= J << pos;
    }
  }
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}

// 4 x 16 bit-matrix transpose in a 64-bit word: input row r = bits [16r, 16r + 16), output bit 4c + r = input
// bit 16r + c. The index map is a rotation of the 6 index bits, done as 4 index-bit swaps (delta swaps, each one
// 64-bit shift pair and two 3-input bit ops).
__device__ __forceinline__ uint64_t dswap64(uint64_t x, uint64_t m, uint32_t d)
{
  const uint64_t t = ((x >> d) ^ x) & m;
  return x ^ t ^ (t << d);
}

__device__ __forceinline__ uint64_t transpose4x16(uint64_t x)
{
  x = dswap64(x, 0x0000AAAA0000AAAAull, 15);  // index bits 0 <-> 4
  x = dswap64(x, 0x00000000CCCCCCCCull, 30);  // 1 <-> 5
  x = dswap64(x, 0x0000F0F00000F0F0ull, 12);  // 2 <-> 4
  x = dswap64(x, 0x00000000FF00FF00ull, 24);  // 3 <-> 5
  return x;
}

// 16 bit planes starting at plane `top` going down, as nibbles: nibble j of the result = bits (top - j) of u0..u3.
__device__ __forceinline__ uint64_t plane_window(const uint32_t* u, uint32_t sh)
{
  const uint32_t g0 = (__builtin_bitreverse32(u[0]) >> sh) & 0xffffu;
  const uint32_t g1 = (__builtin_bitreverse32(u[1]) >> sh) & 0xffffu;
  const uint32_t g2 = (__builtin_bitreverse32(u[2]) >> sh) & 0xffffu;
  const uint32_t g3 = (__builtin_bitreverse32(u[3]) >> sh) & 0xffffu;
  const uint64_t x = (uint64_t)(g0 | (g1 << 16)) | ((uint64_t)(g2 | (g3 << 16)) << 32);
  return transpose4x16(x);
}

// Lean-5 block: same stream as lean-4 (and encode.c:457-495 for d = 1, fixed rate, kmin = 0).
//  * tiny (all values cast to INT_MIN) and zero blocks are selected from constants at the end, so the cast needs
//    no per-value range select;
//  * pair 0 always starts at n = 0 and pair 1 is taken by ~92 % of waves: both accumulate in 32 bits (<= 28 code
//    bits), one 64-bit shift places them; only pairs 2.. (about half the waves) use the budget-guarded 64-bit path.
template <uint32_t WB>
__device__ __forceinline__ uint64_t encode_block1d_lean5(const float* f, const uint32_t* tab, bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = m >= 0x7f800000u;  // Inf or NaN present
  const uint32_t E = m >> 23;
  const float s = __uint_as_float((283u - E) << 23);  // 2^(30 - e); meaningless for tiny / special lanes
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = cvt_i32_hw(f[i] * s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  const uint32_t o23 = u[2] | u[3];
  const uint32_t sh = __builtin_clz(u[0] | u[1] | o23 | 1u);  // 31 - M0
  const int M0 = 31 - (int)sh;
  const int jg = o23 ? (int)__builtin_clz(o23) - (int)sh : M0;  // group phase: window nibbles 0 .. jg
  const uint64_t Y = plane_window(u, sh);
  uint32_t pos = 9 + sh;
  uint32_t e = tab[(uint32_t)Y & 255u];
  uint32_t G = e >> 17, gl = (e >> 13) & 15u;
  int j = 2;
  if (__any(jg >= 2)) {
    e = tab5_next(tab, e, ((uint32_t)Y >> 8) & 255u);
    G |= (e >> 17) << gl;
    gl += (e >> 13) & 15u;
    j = 4;
  }
  uint64_t acc = (2ull * E + 3ull) | ((uint64_t)G << pos);
  pos += gl;
#pragma unroll
  for (int jj = 4; jj < 16; jj += 2) {
    if (j < jj || !__any(jj <= jg)) break;
    e = tab5_next(tab, e, (uint32_t)(Y >> (4 * jj)) & 255u);
    const uint32_t code = pos < WB ? (e >> 17) : 0u;  // 64-bit shifts wrap: nothing past the budget
    acc |= (uint64_t)code << pos;
    pos += (e >> 13) & 15u;
    j = jj + 2;
  }
  special = special || (jg >= 16 && pos < WB);  // group phase runs past the 16-plane window (generic coder)
  if (j < 16 && pos < WB) acc |= (Y >> (4 * j)) << pos;  // rest of the window, verbatim
  const uint32_t p2 = pos + 4u * (uint32_t)(16 - j);      // where plane M0 - 16 lands
  if (__any(p2 < WB && M0 >= 16)) {
    const uint64_t Y2 = plane_window(u, (uint32_t)max(47 - M0, 0));  // planes M0 - 16 .. M0 - 31
    if (p2 < WB && M0 >= 16) acc |= Y2 << p2;
  }
  constexpr uint64_t TINY = tiny_payload_cx((int)WB - 9) << 9;
  const uint64_t tv = m ? (TINY | (2ull * E + 3ull)) : 0ull;
  acc = E < 29u ? tv : acc;  // zero, subnormal and tiny-normal maxima: every value casts to INT_MIN (or is 0)
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}

#ifndef GCOW_C2_PAIR1_ALWAYS
#define GCOW_C2_PAIR1_ALWAYS 1  // lean-6: the second pair step without a wave vote
#endif

// Lean-6 block: the lean-5 stream (encode.c:457-495 for d = 1, fixed rate, kmin = 0) with
//  * the block maximum as a float max3 of |f| (NaN caught by two unordered compares: it never wins the maximum,
//    encode.c:146-150, but it casts to INT_MIN, so such blocks take the generic coder);
//  * the lift and the negabinary map fused, the map's add folded into the last lifting add where there is one;
//  * the window from window_lds;
//  * the group-phase end jg = clz(u2 | u3) - sh, with 31 for o23 = 0 (jg = M0);
//  * zero blocks coded by the main path (u = 0 codes to all-zero bits after a zero header), so only tiny-normal and
//    subnormal maxima (0 < E < 29) take the constant payload.
template <uint32_t WB, bool W2LOW = false>
__device__ __forceinline__ uint64_t encode_block1d_lean6(const float* f, const uint32_t* tab, const uint32_t* rs,
                                                         bool& special)
{
  uint32_t m;  // max |f| as bits: v_max3_f32 / v_max_f32 with |.| modifiers (no canonicalising fmaxf)
  asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(m) : "v"(f[0]), "v"(f[1]), "v"(f[2]));
  asm("v_max_f32_e64 %0, %0, |%1|" : "+v"(m) : "v"(f[3]));
  special = m >= 0x7f800000u || __builtin_isunordered(f[0], f[1]) || __builtin_isunordered(f[2], f[3]);
  const uint32_t E = m >> 23;
  const float s = __uint_as_float((283u - E) << 23);  // 2^(30 - e); meaningless for tiny / special lanes
  uint32_t x = (uint32_t)cvt_i32_hw(f[0] * s), y = (uint32_t)cvt_i32_hw(f[1] * s);
  uint32_t z = (uint32_t)cvt_i32_hw(f[2] * s), w = (uint32_t)cvt_i32_hw(f[3] * s);
  // fwd_lift (encode.c:212-225), int32 wraparound; arithmetic shifts on the signed view
  auto asr = [](uint32_t v) { return (uint32_t)((int32_t)v >> 1); };
  constexpr uint32_t NB = 0xaaaaaaaau;
  x = asr(x + w); w -= x;
  z = asr(z + y); y -= z;
  x = asr(x + z); z -= x;
  w = asr(w + y); y -= w;
  const uint32_t u3 = (w + asr(y) + NB) ^ NB;  // w += y >> 1, then the negabinary map
  const uint32_t u1 = (y - asr(w + asr(y)) + NB) ^ NB;
  const uint32_t u0 = (x + NB) ^ NB, u2 = (z + NB) ^ NB;
  const uint32_t o23 = u2 | u3;
  const uint32_t sh = __builtin_clz(u0 | u1 | o23 | 1u);  // 31 - M0
  const int M0 = 31 - (int)sh;
  const int jg = (int)min(ffbh_hw(o23), 31u) - (int)sh;  // group phase: window nibbles 0 .. jg (o23 = 0: M0)
  const uint32_t w0 = u0 << sh, w1 = u1 << sh, w2 = u2 << sh, w3 = u3 << sh;
  const uint64_t Y = window_lds(rs, w0, w1, w2, w3);
  uint32_t pos = 9 + sh;
  uint32_t e = tab[(uint32_t)Y & 255u];
  uint32_t G = e >> 17, gl = (e >> 13) & 15u;
#if GCOW_C2_PAIR1_ALWAYS
  // pair 1 for every lane, no wave vote (~92 % of waves take it anyway): past a lane's group phase the table's rows
  // n >= 3 code planes 2 and 3 as their verbatim nibbles, the bits the verbatim run would give them
  int j = 4;
  e = tab5_next(tab, e, ((uint32_t)Y >> 8) & 255u);
  G |= (e >> 17) << gl;
  gl += (e >> 13) & 15u;
#else
  int j = 2;
  if (__any(jg >= 2)) {
    e = tab5_next(tab, e, ((uint32_t)Y >> 8) & 255u);
    G |= (e >> 17) << gl;
    gl += (e >> 13) & 15u;
    j = 4;
  }
#endif
  const uint32_t hdr = m ? 2u * E + 3u : 0u;  // zero block: a single 0 bit, every later bit 0 as well
  uint64_t acc = (uint64_t)hdr | ((uint64_t)G << pos);
  pos += gl;
#pragma unroll
  for (int jj = 4; jj < 16; jj += 2) {
    if (j < jj || !__any(jj <= jg)) break;
    e = tab5_next(tab, e, (uint32_t)(Y >> (4 * jj)) & 255u);
    const uint32_t code = pos < WB ? (e >> 17) : 0u;  // 64-bit shifts wrap: nothing past the budget
    acc |= (uint64_t)code << pos;
    pos += (e >> 13) & 15u;
    j = jj + 2;
  }
  const bool tiny = m - 1u < (29u << 23) - 1u;  // 0 < E < 29: tiny-normal and subnormal maxima (coded below)
  special = special || (!tiny && jg >= 16 && pos < WB);  // group phase runs past the 16-plane window
  if (j < 16 && pos < WB) acc |= (Y >> (4 * j)) << pos;  // rest of the window, verbatim
  const uint32_t p2 = pos + 4u * (uint32_t)(16 - j);      // where plane M0 - 16 lands
  if (__any(p2 < WB && M0 >= 16)) {
    uint64_t Y2;  // planes M0-16 .. M0-31
    if constexpr (W2LOW) {
      Y2 = window_lds_low(rs, w0, w1, w2, w3);
    } else {
      const uint32_t s2 = sh + 16u;  // <= 31 where used (M0 >= 16)
      Y2 = window_lds(rs, u0 << s2, u1 << s2, u2 << s2, u3 << s2);
    }
    if (p2 < WB && M0 >= 16) acc |= Y2 << p2;
  }
  constexpr uint64_t TINY = tiny_payload_cx((int)WB - 9) << 9;
  acc = tiny ? (TINY | hdr) : acc;  // every value casts to INT_MIN
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}

// ---- hand-counted memory pipeline for the persistent fixed-rate 1-D encoder
// Loads and stores are raw buffer instructions issued from inline asm, so the compiler's waitcnt pass does not see
// them; the waits are counted here instead. (With compiler-tracked loads the conditional / loop-carried prefetch
// collapsed to s_waitcnt vmcnt(0) at the loop head, i.e. every block waited for the previous block's store ack:
// vmcnt counts stores and loads together, in issue order.) Out-of-range lanes read zeros and their stores are dropped
// by the buffer range check (num_records), which keeps the loop exit wave-uniform and every step's op count fixed.
typedef int pipe_v4i __attribute__((ext_vector_type(4)));
typedef float pipe_v4f __attribute__((ext_vector_type(4)));
typedef unsigned int pipe_v2u __attribute__((ext_vector_type(2)));
typedef unsigned int pipe_v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ pipe_v4i buf_rsrc(const void* p, uint32_t bytes)
{
  const uint64_t a = (uint64_t)p;
  pipe_v4i r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((uint32_t)(a >> 32) & 0xffffu);  // stride 0
  r.z = (int)bytes;                             // num_records: range check in bytes
  r.w = 0x00020000;                             // gfx9 dword-3 config (raw buffer, no swizzle)
  return r;
}

template <int DT> struct PipeRow;
template <> struct PipeRow<DT_F32> {
  typedef pipe_v4f T;
  static __device__ __forceinline__ T load(uint32_t off, pipe_v4i rs)
  {
    T v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(rs) : "memory");
    return v;
  }
  static __device__ __forceinline__ void unpack(const T& v, float* f) { f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w; }
};
template <> struct PipeRow<DT_BF16> {
  typedef pipe_v2u T;
  static __device__ __forceinline__ T load(uint32_t off, pipe_v4i rs)
  {
    T v;
    asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(rs) : "memory");
    return v;
  }
  static __device__ __forceinline__ void unpack(const T& v, float* f)
  {
    f[0] = __uint_as_float(v.x << 16);
    f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16);
    f[3] = __uint_as_float(v.y & 0xffff0000u);
  }
};

template <int N, typename T>
__device__ __forceinline__ void pipe_wait(T& v)
{
  asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v) : "n"(N) : "memory");  // ties v's uses to after the wait
}

template <uint32_t WB>
__device__ __forceinline__ void pipe_store(uint32_t off, pipe_v4i rs, uint64_t w)
{
  if constexpr (WB == 64)
    asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen nt" : : "v"(w), "v"(off), "s"(rs) : "memory");
  else
    asm volatile("buffer_store_dword %0, %1, %2, 0 offen nt" : : "v"((uint32_t)w), "v"(off), "s"(rs) : "memory");
}

// One-shot (non-persistent) fixed-rate 1-D encoder: each lane codes U blocks 256 apart inside its workgroup's chunk
// of 256 U blocks. All U loads are issued first (before the LDS table fill), then each block waits for its own load
// only: with U loads followed by k stores outstanding, load k has landed once at most U - 1 operations remain
// (vmcnt counts loads and stores together, in issue order). Out-of-range lanes read zeros and their stores are
// dropped by the buffer range check, so control flow stays wave-uniform. Measured against the persistent grid-stride
// pipeline above, the one-shot shape streams HBM like a plain copy kernel.
__device__ __forceinline__ uint32_t buf_load_u32(uint32_t off, pipe_v4i rs)
{
  uint32_t v;
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(rs) : "memory");
  return v;
}

__device__ __forceinline__ pipe_v4u buf_load_b128(uint32_t off, pipe_v4i rs)
{
  pipe_v4u v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(rs) : "memory");
  return v;
}

template <int DT, uint32_t WB, int U, uint32_t T = 256, int V = 0>
__global__ __launch_bounds__(T) void k_encode_fixed1d_np(const void* __restrict__ in, uint32_t nfull, Params p,
                                                         void* __restrict__ out)
{
  __shared__ __attribute__((aligned(16))) uint32_t tab[1280 + 1024];  // pair table, then the four window spread tables
  constexpr uint32_t IB = DT == DT_BF16 ? 8u : 16u;  // input bytes per block
  const pipe_v4i rin = buf_rsrc(in, nfull * IB), rout = buf_rsrc(out, nfull * (WB / 8));
  const uint32_t b0 = blockIdx.x * (T * U) + threadIdx.x;
  typename PipeRow<DT>::T r[U];
  if constexpr ((V & 1) != 0) {
    // pair-table loads issued first (hand-counted like the data loads), so waiting for them is vmcnt(U) and block 0
    // can start as soon as its own load lands (a compiler-issued table load after the data loads waits vmcnt(0))
    static_assert(T == 256, "table fill assumes 256 threads");
    constexpr int NT = 1280 / 256;
    const pipe_v4i rt = buf_rsrc(&g_plane_tab5, sizeof(PlaneTab2));
    uint32_t tv[NT];
#pragma unroll
    for (int i = 0; i < NT; i++) tv[i] = buf_load_u32((threadIdx.x + 256u * i) * 4u, rt);
#pragma unroll
    for (int k = 0; k < U; k++) r[k] = PipeRow<DT>::load((b0 + T * k) * IB, rin);
#pragma unroll
    for (uint32_t t = threadIdx.x; t < 1024; t += T) tab[1280 + t] = rspread_entry(t);
    asm volatile("s_waitcnt vmcnt(%5)" : "+v"(tv[0]), "+v"(tv[1]), "+v"(tv[2]), "+v"(tv[3]), "+v"(tv[4]) : "n"(U)
                 : "memory");
#pragma unroll
    for (int i = 0; i < NT; i++) tab[threadIdx.x + 256u * i] = tv[i];
  } else {
#pragma unroll
    for (int k = 0; k < U; k++) r[k] = PipeRow<DT>::load((b0 + T * k) * IB, rin);
#pragma unroll
    for (uint32_t t = threadIdx.x; t < 1280; t += T) tab[t] = g_plane_tab5.v[t];
    // the spread tables are computed, not loaded: entry 256 i + b = byte b reversed onto nibble bit i
#pragma unroll
    for (uint32_t t = threadIdx.x; t < 1024; t += T) tab[1280 + t] = rspread_entry(t);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < U; k++) {
    pipe_wait<U - 1>(r[k]);
    float f[4];
    PipeRow<DT>::unpack(r[k], f);
    bool special;
    uint64_t w = encode_block1d_lean6<WB, (V & 2) != 0>(f, tab, tab + 1280, special);
    if (special) {
      RegWriter64 rw{0ull, 0u};
      encode_block<1>(rw, f, p);
      w = WB == 64 ? rw.acc : (rw.acc & ((1ull << WB) - 1ull));
    }
    pipe_store<WB>((b0 + T * k) * (WB / 8), rout, w);
  }
}

// The memory floor of the fixed-rate 1-D encoder's access pattern (bench.py `roofline.copy_ceiling`): the same
// one-shot grid, U = 8 blocks per lane, the same raw buffer loads (16 B fp32 / 8 B bf16 per block) and WB-bit
// non-temporal stores with the same hand-counted waits, and no coding (each block's store is an xor-fold of its load).
template <int DT, uint32_t WB, int U>
__global__ __launch_bounds__(256) void k_copy_pattern1d(const void* __restrict__ in, uint32_t nfull,
                                                        void* __restrict__ out)
{
  constexpr uint32_t T = 256;
  constexpr uint32_t IB = DT == DT_BF16 ? 8u : 16u;
  const pipe_v4i rin = buf_rsrc(in, nfull * IB), rout = buf_rsrc(out, nfull * (WB / 8));
  const uint32_t b0 = blockIdx.x * (T * U) + threadIdx.x;
  typename PipeRow<DT>::T r[U];
#pragma unroll
  for (int k = 0; k < U; k++) r[k] = PipeRow<DT>::load((b0 + T * k) * IB, rin);
#pragma unroll
  for (int k = 0; k < U; k++) {
    pipe_wait<U - 1>(r[k]);
    float f[4];
    PipeRow<DT>::unpack(r[k], f);
    const uint64_t w = ((uint64_t)(__float_as_uint(f[0]) ^ __float_as_uint(f[1])) << 32) |
                       (__float_as_uint(f[2]) ^ __float_as_uint(f[3]));
    pipe_store<WB>((b0 + T * k) * (WB / 8), rout, w);
  }
}

// Generic fixed-rate 1-D encoder over the full 4-value blocks [0, nfull) for parameters outside the lean coder's
// domain (maxprec < 32 or minexp > -154: kmin > 0 possible); two blocks per lane, loads issued first.
template <int DT, uint32_t WB>
__global__ __launch_bounds__(256) void k_encode_fixed1d_generic(const void* __restrict__ in, uint32_t nfull, Params p,
                                                                void* __restrict__ out)
{
  __shared__ uint16_t tab[80];
  if (threadIdx.x < 80) tab[threadIdx.x] = plane_entry4(threadIdx.x);
  __syncthreads();
  constexpr int U = 2;
  const uint32_t b0 = blockIdx.x * (256u * U) + threadIdx.x;
  float f[U][4];
#pragma unroll
  for (int j = 0; j < U; j++) {
    const uint32_t b = b0 + 256u * j;
    if (b < nfull) load_row4<DT>(in, 4ll * b, f[j]);
  }
#pragma unroll
  for (int j = 0; j < U; j++) {
    const uint32_t b = b0 + 256u * j;
    if (b < nfull) {
      const uint64_t w = encode_block1d_fixed<WB>(f[j], p, tab);
      if constexpr (WB == 64) ((uint64_t*)out)[b] = w;
      else ((uint32_t*)out)[b] = (uint32_t)w;
    }
  }
}

// The partial last block of a 1-D bucket (nvals % 4 != 0): padded gather (encode.c:41-60), one lane.
template <int DT, uint32_t WB>
__global__ void k_encode_fixed1d_tail(const void* __restrict__ in, uint64_t nvals, uint32_t b, Params p,
                                      void* __restrict__ out)
{
  __shared__ uint16_t tab[80];
  if (threadIdx.x < 80) tab[threadIdx.x] = plane_entry4(threadIdx.x);
  __syncthreads();
  if (threadIdx.x) return;
  float f[4];
  load_block1d<DT>(in, nvals, b, f);
  const uint64_t w = encode_block1d_fixed<WB>(f, p, tab);
  if constexpr (WB == 64) ((uint64_t*)out)[b] = w;
  else ((uint32_t*)out)[b] = (uint32_t)w;
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x)
{
  const uint32_t lane = __lane_id();
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t lo = __shfl_up((uint32_t)x, o), hi = __shfl_up((uint32_t)(x >> 32), o);
    if (lane >= o) x += (uint64_t)lo | ((uint64_t)hi << 32);
  }
  return x;
}

// Exclusive scan of the range totals (one workgroup). base[] gets nranges + 1 entries (last = total bits); the
// 32-bit words two ranges share are zeroed so both sides can atomicOr into them; the stream's flush word too.
// d_base (optional): the stream already holds *d_base bits (chunked / appended encode); every offset starts there and
// the first range ORs its first word into the bits before it.
// One workgroup: the range totals are read in coalesced chunks of 8192 through LDS (each thread then scans 8
// consecutive totals; wave prefix by shuffles, 16 wave totals through LDS), so every global access is coalesced --
// a per-thread walk over its own contiguous slice touched 64 cache lines per wave load (82 us at 32 Ki ranges).
__global__ __launch_bounds__(1024) void k_scan_ranges(const uint64_t* __restrict__ sums, uint32_t nranges,
                                                      uint64_t* __restrict__ base, uint64_t* __restrict__ total,
                                                      uint32_t* __restrict__ out32, const uint64_t* __restrict__ d_base)
{
  constexpr uint32_t T = 1024, K = 8, C = T * K;
  __shared__ uint64_t v[C];
  __shared__ uint64_t wsum[T / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  uint64_t carry = d_base ? *d_base : 0ull;
  for (uint32_t c0 = 0; c0 < nranges; c0 += C) {
    const uint32_t n = min(C, nranges - c0);
#pragma unroll
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t j = t + T * k;
      v[j] = j < n ? sums[c0 + j] : 0ull;
    }
    __syncthreads();
    uint64_t loc[K], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < K; k++) {
      loc[k] = v[t * K + k];
      s += loc[k];
    }
    const uint64_t incl = wave_incl_scan64(s);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint64_t before = 0, chunk = 0;
#pragma unroll
    for (uint32_t w = 0; w < T / 64; w++) {
      const uint64_t x = wsum[w];
      before += w < wv ? x : 0ull;
      chunk += x;
    }
    uint64_t run = carry + before + incl - s;
#pragma unroll
    for (uint32_t k = 0; k < K; k++) {
      v[t * K + k] = run;
      run += loc[k];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t j = t + T * k;
      if (j < n) {
        const uint64_t b = v[j];
        base[c0 + j] = b;
        if (c0 + j > 0 && (b & 31)) out32[b >> 5] = 0u;  // a word two ranges share: zeroed for their atomicOr
      }
    }
    carry += chunk;
    __syncthreads();
  }
  if (t == 0) {
    base[nranges] = carry;
    if (total) *total = carry;
  }
}

// ------------------------------------------------------------------------------------------------ 1-D variable rate
// Closed-form coder for variable-rate 1-D blocks (accuracy / precision / expert modes whose budget never truncates a
// block: minbits <= 1, maxbits >= 160). Same structure as lean-5, with the plane range ending at kmin = 32 - prec:
//   header (9) | empty planes 31 .. max(M0, kmin - 1) + 1 ('0' each) | group phase M0 .. max(T2, kmin), two planes
//   per wave-uniform step through the pair table (lanes past their own group phase emit verbatim nibbles, lanes
//   past kmin emit nothing) | verbatim nibbles down to kmin from the 32-plane window.
// Returns the block's bit length; with CODE the bits in c[0..2] (a block is at most 140 bits). special: Inf/NaN, or a
// group phase longer than 16 planes or 64 bits -> generic coder.
template <bool CODE>
__device__ __forceinline__ uint32_t encode_block1d_var(const float* f, const uint16_t* tab, const uint32_t* tab2,
                                                      const uint32_t* rs, int minexp, uint32_t maxprec, uint64_t* c,
                                                      bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = m >= 0x7f800000u;
  const uint32_t E = special ? 150u : (m >> 23);
  const int emax = E ? (int)E - 126 : -126;  // frexp exponent of max|x|; subnormal maxima clamp to -126
  const int prec = min((int)maxprec, max(0, emax - minexp + 4));
  if (CODE) c[0] = c[1] = c[2] = 0ull;
  if (m == 0 || prec == 0) return 1u;  // one 0 bit
  const int kmin = prec < 32 ? 32 - prec : 0;
  const bool tiny = E < 29u;
  const float s = __uint_as_float((283u - (tiny ? 150u : E)) << 23);
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = tiny ? (int32_t)0x80000000 : (int32_t)(f[i] * s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  const uint32_t o23 = u[2] | u[3];
  const int M0 = 31 - (int)__builtin_clz(u[0] | u[1] | o23 | 1u);
  const int T2 = o23 ? 31 - (int)__builtin_clz(o23) : 0;
  const uint32_t pos0 = 9u + (uint32_t)(31 - max(M0, kmin - 1));  // header + empty planes
  const int nplanes = max(M0 - kmin + 1, 0);                        // planes M0 .. kmin
  const int jg = M0 - max(T2, kmin);                                 // last group-phase plane (window index)
  const uint32_t sh = (uint32_t)(31 - M0);  // M0 >= 0: the |1 in the clz
  const uint64_t Y = window_lds(rs, u[0] << sh, u[1] << sh, u[2] << sh, u[3] << sh);
  uint64_t g = 0;  // group-phase bits, relative to pos0
  uint32_t glen = 0, n = 0;
  int j = 0;
  // two planes per step through the lean-5 pair table (tab2: n' << 10 | len << 13 | code << 17); a pair whose second
  // plane is below kmin takes its first plane's code from the single-plane table (tab)
#pragma unroll
  for (; j < 16; j += 2) {
    if (!__any(j <= jg)) break;
    const uint32_t byte = (uint32_t)(Y >> (4 * j)) & 255u;
    const uint32_t e = tab2[(n << 8) | byte];
    const bool act2 = j + 1 < nplanes, act1 = j < nplanes;
    uint32_t code = act2 ? e >> 17 : 0u, len = act2 ? (e >> 13) & 15u : 0u;
    if (__any(act1 && !act2)) {
      const uint32_t e1 = tab[(n << 4) | (byte & 15u)];
      if (act1 && !act2) {
        code = e1 & 127u;
        len = (e1 >> 7) & 7u;
      }
    }
    if (CODE) g |= (uint64_t)(glen < 64 ? code : 0u) << glen;
    glen += len;
    n = act2 ? (e >> 10) & 7u : n;
  }
  j = min(j, 16);
  special = special || jg >= 16 || glen > 64;
  const int tplanes = max(nplanes - j, 0);  // verbatim planes after the group phase
  const uint32_t len = pos0 + glen + 4u * (uint32_t)tplanes;
  if (CODE) {
    const uint64_t hdr = 2ull * E + 3ull;
    c[0] = hdr | (pos0 < 64 ? g << pos0 : 0ull);
    c[1] = pos0 ? g >> (64 - pos0) : 0ull;  // pos0 >= 9
    if (tplanes > 0) {
      // tail nibbles j .. nplanes-1 of the 32-plane window (Y, then planes M0-16 .. M0-31)
      const uint32_t s2 = sh + 16u;  // <= 31 where used (nplanes > 16 needs M0 >= 16)
      const uint64_t Y2 = nplanes > 16 ? window_lds(rs, u[0] << s2, u[1] << s2, u[2] << s2, u[3] << s2) : 0ull;
      // j is the wave-uniform group-loop count, 1..16 (16 when another lane's group phase filled the window)
      uint64_t t0 = j == 16 ? Y2 : (Y >> (4 * j)) | (Y2 << (64 - 4 * j));
      uint64_t t1 = j == 16 ? 0ull : Y2 >> (4 * j);
      const uint32_t tb = 4u * (uint32_t)tplanes;  // <= 128
      if (tb < 64) { t0 &= (1ull << tb) - 1ull; t1 = 0; }
      else if (tb < 128) t1 &= (1ull << (tb - 64)) - 1ull;
      const uint32_t pt = pos0 + glen;  // in [9, 137]
      if (pt < 64) {
        c[0] |= t0 << pt;
        c[1] |= (t0 >> (64 - pt)) | (t1 << pt);
        c[2] |= t1 >> (64 - pt);
      } else if (pt < 128) {
        const uint32_t q2 = pt - 64;
        c[1] |= t0 << q2;
        c[2] |= (q2 ? t0 >> (64 - q2) : 0ull) | (t1 << q2);
      } else {
        c[2] |= t0 << (pt - 128);
      }
    }
  }
  return len;
}

// Bit length of a variable-rate 1-D block (same domain as encode_block1d_var; Inf/NaN -> special) from the leading
// one-bit planes L_i of its four negabinary coefficients alone. With n_k = 1 + max{i : L_i >= k} the prefix after
// plane k (encode.c:279-339 carries n across planes), plane k costs n_{k+1} verbatim bits plus, when n_{k+1} < 4,
// either one '0' (nothing new) or m + (q == 3 ? 3 : q + 2) - n_{k+1} bits (m new one-bits, the last at q: one group
// flag each, the run up to q, a closing '0' unless q is the implied last position). With R_j = max_{i >= j} L_i summed
// over planes kmin .. 31:
//   sum_j max(0, R_j - kmin) + (32 - max(kmin, L_3)) + #{j : L_j = R_j >= kmin}
//   + sum_j [R_j >= kmin, last index at its level] (j < 3 ? j + 1 : 2) - sum_j [R_j >= kmin, first at its level] j,
// where the last two sums cancel except where R crosses kmin (see encode_ints_length).
__device__ __forceinline__ uint32_t count_block1d_var(const float* f, int minexp, uint32_t maxprec, bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = m >= 0x7f800000u;
  const uint32_t E = special ? 150u : (m >> 23);
  const int emax = E ? (int)E - 126 : -126;
  const int prec = min((int)maxprec, max(0, emax - minexp + 4));
  if (m == 0 || prec == 0) return 1u;
  const bool tiny = E < 29u;
  const float s = __uint_as_float((283u - (tiny ? 150u : E)) << 23);
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = tiny ? (int32_t)0x80000000 : (int32_t)(f[i] * s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  return 9u + encode_ints_length<4>(u, (uint32_t)prec);  // closed form (codec_device.h), prec >= 1 here
}

// Variable-rate 1-D pass 1: per-range sums of block bit lengths (closed form from the leading planes; generic for
// Inf/NaN blocks).
// Tiles of 256 U blocks; contiguous bf16 input takes coalesced 16-B loads with the next tile prefetched.
template <int DT, int U>
__global__ __launch_bounds__(256) void k_count1d_var(FieldDesc F, Params p, uint32_t range, uint64_t* __restrict__ sums)
{
  constexpr uint32_t TILE = 256u * U;
  constexpr int BPL = DT == DT_BF16 ? 2 : 1;  // blocks per 16-B load
  constexpr int NL = U / BPL;                 // 16-B loads per lane per tile
  static_assert(U % BPL == 0, "U must hold whole 16-B loads");
  __shared__ uint64_t red[4];
  const uint32_t tid = threadIdx.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * range;
  const uint64_t b1 = min<uint64_t>(b0 + range, F.nblocks);
  uint64_t acc = 0;
  uint64_t t0 = b0;
  // Contiguous, 16-B aligned bf16 input: whole tiles of full blocks read with coalesced 16-B loads (load j of lane t
  // covers blocks t0 + (256 j + t) BPL ..; the sum is order-free), the next tile's loads issued before this tile is
  // counted (C5 acc 1e-6 0.878 -> 0.843 ms). The same form measured slower for fp32 (0.876 -> 1.043 ms): fp32 keeps the
  // per-lane gather below.
  if (DT == DT_BF16 && F.vec && F.s[0] == 1 && (((uintptr_t)F.data) & 15u) == 0) {
    const uint64_t lim = min<uint64_t>(b1, F.n[0] / 4);
    const uint64_t tend = lim > b0 ? b0 + (lim - b0) / TILE * TILE : b0;
    const uint4* src = (const uint4*)F.data;  // 16-B units: one f32 block or two bf16 blocks
    uint4 cur[NL], nxt[NL];
    if (t0 < tend) {
#pragma unroll
      for (int j = 0; j < NL; j++) cur[j] = src[t0 / BPL + 256u * j + tid];
    }
    for (; t0 < tend; t0 += TILE) {
      if (t0 + TILE < tend) {
#pragma unroll
        for (int j = 0; j < NL; j++) nxt[j] = src[(t0 + TILE) / BPL + 256u * j + tid];
      }
#pragma unroll
      for (int j = 0; j < NL; j++) {
        float f[BPL][4];
        if constexpr (DT == DT_BF16) {
          const uint32_t w[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
#pragma unroll
          for (int h = 0; h < 2; h++) {
            f[h][0] = __uint_as_float(w[2 * h] << 16);
            f[h][1] = __uint_as_float(w[2 * h] & 0xffff0000u);
            f[h][2] = __uint_as_float(w[2 * h + 1] << 16);
            f[h][3] = __uint_as_float(w[2 * h + 1] & 0xffff0000u);
          }
        } else {
          f[0][0] = __uint_as_float(cur[j].x); f[0][1] = __uint_as_float(cur[j].y);
          f[0][2] = __uint_as_float(cur[j].z); f[0][3] = __uint_as_float(cur[j].w);
        }
#pragma unroll
        for (int h = 0; h < BPL; h++) {
          bool special;
          uint32_t len = count_block1d_var(f[h], p.minexp, p.maxprec, special);
          if (special) len = count_block<1>(f[h], p);
          acc += len;
        }
      }
#pragma unroll
      for (int j = 0; j < NL; j++) cur[j] = nxt[j];
    }
  }
  for (; t0 < b1; t0 += TILE) {  // the rest (partial tiles, the padded last block, strided input)
    float f[U][4];
#pragma unroll
    for (int k = 0; k < U; k++) {
      const uint64_t b = t0 + (uint64_t)tid * U + k;
      f[k][0] = f[k][1] = f[k][2] = f[k][3] = 0.0f;
      if (b < b1) gather_block<1, DT>(F, (uint32_t)b, f[k]);
    }
#pragma unroll
    for (int k = 0; k < U; k++) {
      const uint64_t b = t0 + (uint64_t)tid * U + k;
      bool special;
      uint32_t len = count_block1d_var(f[k], p.minexp, p.maxprec, special);
      if (special && b < b1) len = count_block<1>(f[k], p);
      acc += b < b1 ? len : 0u;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) sums[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Variable-rate 1-D pass 2: k_encode_tiles with the closed-form coder over tiles of 256 U blocks (U consecutive
// blocks per lane: U times the work per barrier round); each lane ORs its <= 140-bit codes into the tile's LDS window
// with 64-bit LDS atomics.
template <int DT, int U>
__global__ __launch_bounds__(256) void k_encode1d_var(FieldDesc F, Params p, uint32_t range,
                                                      const uint64_t* __restrict__ rbase, uint32_t* __restrict__ out32,
                                                      uint64_t* __restrict__ index, uint32_t index_shift)
{
  constexpr uint32_t T = 256;
  __shared__ uint64_t lds64[(31 + T * U * 160 + 63) / 64 + 4];
  __shared__ uint32_t scan_sh[T / 64];
  __shared__ uint16_t tab[80];
  __shared__ __attribute__((aligned(16))) uint32_t tab2[1280];
  __shared__ uint32_t rs[1024];  // window spread tables (window_lds)
  uint32_t* lds = (uint32_t*)lds64;
  const uint32_t tid = threadIdx.x;
  if (tid < 80) tab[tid] = plane_entry4(tid);
  stage_table<T, 1280>(tab2, g_plane_tab5.v);
#pragma unroll
  for (uint32_t t = 0; t < 1024 / T; t++) rs[tid + T * t] = rspread_entry(tid + T * t);
  const uint64_t b0 = (uint64_t)blockIdx.x * range;
  const uint64_t b1 = min<uint64_t>(b0 + range, F.nblocks);
  const bool final_range = b1 == F.nblocks;
  uint64_t base = rbase[blockIdx.x];
  const uint64_t first_word = base >> 5;
  const bool first_shared = (base & 31) != 0;
  uint32_t carry = 0;
  // Contiguous, 16-B aligned bf16: a lane's U consecutive blocks are U/2 16-B loads, issued one tile ahead (before
  // this tile's scan / LDS / store rounds) for every tile made of full blocks only. (The same for fp32, U 16-B loads
  // per lane, measured slower: 0.875 -> 0.968 ms at accuracy 1e-6.)
  constexpr bool WIDE = DT == DT_BF16 && U % 2 == 0;
  constexpr int NW = WIDE ? U / 2 : 1;
  const bool wide = WIDE && F.vec && F.s[0] == 1 && (((uintptr_t)F.data) & 15u) == 0;
  const uint64_t full_end = min<uint64_t>(b1, F.n[0] / 4);  // blocks below this are full
  const uint4* src = (const uint4*)F.data;
  uint4 nxt[NW];
  auto wide_tile = [&](uint64_t t) { return wide && t + T * U <= full_end; };
  if (wide_tile(b0)) {
#pragma unroll
    for (int h = 0; h < NW; h++) nxt[h] = src[(b0 + (uint64_t)tid * U) / 2 + h];
  }
  __syncthreads();
  for (uint64_t t0 = b0; t0 < b1; t0 += T * U) {
    float f[U][4];
    if (wide_tile(t0)) {
      uint4 cur[NW];
#pragma unroll
      for (int h = 0; h < NW; h++) cur[h] = nxt[h];
      if (wide_tile(t0 + T * U)) {
#pragma unroll
        for (int h = 0; h < NW; h++) nxt[h] = src[(t0 + T * U + (uint64_t)tid * U) / 2 + h];
      }
#pragma unroll
      for (int h = 0; h < NW; h++) {
        const uint32_t w[4] = {cur[h].x, cur[h].y, cur[h].z, cur[h].w};
#pragma unroll
        for (int g = 0; g < 2 && 2 * h + g < U; g++) {
          f[2 * h + g][0] = __uint_as_float(w[2 * g] << 16);
          f[2 * h + g][1] = __uint_as_float(w[2 * g] & 0xffff0000u);
          f[2 * h + g][2] = __uint_as_float(w[2 * g + 1] << 16);
          f[2 * h + g][3] = __uint_as_float(w[2 * g + 1] & 0xffff0000u);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < U; k++) {
        const uint64_t b = t0 + (uint64_t)tid * U + k;
        f[k][0] = f[k][1] = f[k][2] = f[k][3] = 0.0f;
        if (b < b1) gather_block<1, DT>(F, (uint32_t)b, f[k]);
      }
    }
    uint64_t c[U][3];
    uint32_t len[U];
    bool sp[U];
    uint32_t lsum = 0;
#pragma unroll
    for (int k = 0; k < U; k++) {
      const bool valid = t0 + (uint64_t)tid * U + k < b1;
      len[k] = encode_block1d_var<true>(f[k], tab, tab2, rs, p.minexp, p.maxprec, c[k], sp[k]);
      sp[k] = sp[k] && valid;
      if (sp[k]) {
        len[k] = count_block<1>(f[k], p);
      }
      len[k] = valid ? len[k] : 0u;
      lsum += len[k];
    }
    uint32_t tile_total;
    const uint32_t excl = block_exclusive_scan<T>(lsum, &tile_total, scan_sh);
    const uint32_t lbase = (uint32_t)(base & 31);
    const uint32_t end_local = lbase + tile_total;
    const uint32_t W = (end_local + 31) >> 5;
    for (uint32_t j = tid; j < (W + 3) / 2; j += T) lds64[j] = 0ull;
    __syncthreads();
    if (tid == 0) lds[0] |= carry;
    __syncthreads();
    uint32_t o = lbase + excl;
#pragma unroll
    for (int k = 0; k < U; k++) {
      if (len[k]) {
        if (sp[k]) {
          LdsWriter w{lds, o, o + len[k]};
          encode_block<1>(w, f[k], p);
        } else {
          const uint32_t qw = o >> 6, sh = o & 63u;
          const uint32_t nq = (sh + len[k] + 63) >> 6;  // 1..4 qwords touched
          atomicOr((unsigned long long*)&lds64[qw], (unsigned long long)(c[k][0] << sh));
          if (nq > 1) atomicOr((unsigned long long*)&lds64[qw + 1],
                               (unsigned long long)((sh ? c[k][0] >> (64 - sh) : 0ull) | (c[k][1] << sh)));
          if (nq > 2) atomicOr((unsigned long long*)&lds64[qw + 2],
                               (unsigned long long)((sh ? c[k][1] >> (64 - sh) : 0ull) | (c[k][2] << sh)));
          if (nq > 3) atomicOr((unsigned long long*)&lds64[qw + 3], (unsigned long long)(c[k][2] >> (64 - sh)));
        }
        const uint64_t b = t0 + (uint64_t)tid * U + k;
        if (index && ((b & ((1ull << index_shift) - 1)) == 0)) index[b >> index_shift] = base + (o - lbase);
      }
      o += len[k];
    }
    __syncthreads();
    const bool last_tile = t0 + T * U >= b1;
    const bool partial = (end_local & 31) != 0;
    const uint32_t Wstore = (last_tile || !partial) ? W : (end_local >> 5);
    const uint64_t gw0 = base >> 5;
    for (uint32_t j = tid; j < Wstore; j += T) {
      const uint64_t gw = gw0 + j;
      const uint32_t v = lds[j];
      const bool shared = (gw == first_word && first_shared) || (last_tile && partial && !final_range && j == W - 1);
      if (shared) atomicOr(out32 + gw, v);
      else out32[gw] = v;
    }
    if (last_tile && final_range && tid == 0) {
      const uint64_t endw = (base + tile_total + 31) >> 5;
      if (endw & 1) out32[endw] = 0u;
    }
    carry = (!last_tile && partial) ? lds[end_local >> 5] : 0u;
    base += tile_total;
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------ 4-D blocks
// sw/ declares the 4-D gather (gather_partial_4d_block, sw/src/encode.c:90-126) and zfp_input's
// nw / sw (sw/include/types.h:51-56) but never codes 4-D; libzfp 0.5.5 does, with perm_4 and x, y, z, w lifts.
// One wave per 256-value block: lane l holds the x-row (y, z, w) = (l & 3, (l >> 2) & 3, l >> 4); the lifts run over
// LDS lines (one line per lane per direction); the bit planes are wave ballots (word j = coefficients 64j .. 64j+63,
// lane l owning coefficients l + 64j); the embedded coder runs wave-uniformly on the 256-bit planes with a
// count-trailing-zeros group-test scan, and lane 0 writes the bits into the block's LDS bit buffer.
__device__ const uint8_t g_perm4[256] = {
    0,   1,   4,   16,  64,  5,   80,  17,  68,  65,  20,  2,   8,   32,  128, 84,  81,  69,  21,  6,   18,  66,
    24,  72,  9,   96,  33,  36,  129, 132, 144, 3,   12,  48,  192, 85,  82,  70,  22,  73,  25,  88,  37,  100,
    97,  148, 145, 133, 10,  160, 34,  136, 130, 40,  7,   19,  67,  28,  76,  13,  112, 49,  52,  193, 196, 208,
    86,  89,  101, 149, 161, 137, 41,  134, 38,  164, 26,  152, 146, 104, 98,  74,  83,  71,  23,  77,  29,  92,
    53,  116, 113, 212, 209, 197, 11,  35,  131, 44,  140, 14,  176, 50,  56,  194, 200, 224, 90,  165, 102, 153,
    150, 105, 168, 162, 138, 42,  87,  93,  117, 213, 27,  75,  99,  39,  135, 147, 108, 45,  141, 156, 30,  78,
    177, 180, 54,  114, 120, 57,  198, 210, 216, 201, 225, 228, 15,  240, 51,  204, 195, 60,  169, 166, 154, 106,
    91,  103, 151, 109, 157, 94,  181, 118, 121, 214, 217, 229, 163, 139, 43,  142, 46,  172, 58,  184, 178, 232,
    226, 202, 241, 205, 61,  199, 55,  244, 31,  220, 211, 124, 115, 79,  170, 167, 155, 107, 158, 110, 173, 122,
    185, 182, 233, 230, 218, 95,  245, 119, 221, 215, 125, 242, 206, 62,  203, 59,  248, 47,  236, 227, 188, 179,
    143, 171, 174, 186, 234, 246, 222, 126, 219, 123, 249, 111, 237, 231, 189, 183, 159, 252, 243, 207, 63,  175,
    250, 187, 238, 235, 190, 253, 247, 223, 127, 254, 251, 239, 191, 255};

struct Plane256 {
  uint64_t w[4];
  __device__ __forceinline__ uint64_t bits(uint32_t o) const  // 64 bits from bit o (zeros past 256)
  {
    const uint32_t i = o >> 6, sh = o & 63;
    uint64_t v = i < 4 ? w[i] >> sh : 0ull;
    if (sh && i + 1 < 4) v |= w[i + 1] << (64 - sh);
    return v;
  }
  __device__ __forceinline__ void shr(uint32_t m)
  {
    uint64_t y[4];
#pragma unroll
    for (int i = 0; i < 4; i++) y[i] = m + 64u * i < 256u ? bits(m + 64u * i) : 0ull;
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = y[i];
  }
  __device__ __forceinline__ uint32_t ctz() const  // 256 when zero
  {
    return w[0] ? __builtin_ctzll(w[0]) : w[1] ? 64 + __builtin_ctzll(w[1]) : w[2] ? 128 + __builtin_ctzll(w[2])
           : w[3] ? 192 + __builtin_ctzll(w[3]) : 256u;
  }
};

// Wave-uniform writer into a zeroed LDS bit buffer; lane 0 stores. Bits past `limit` are dropped.
struct UniWriter {
  uint32_t* buf;
  uint32_t pos, limit, lane;
  __device__ __forceinline__ void put(uint64_t v, uint32_t n)
  {
    if (pos < limit && n) {
      const uint32_t k = min(n, limit - pos);
      v &= lowmask64(k);
      if (lane == 0) {
        const uint32_t i = pos >> 5, sh = pos & 31;
        buf[i] |= (uint32_t)(v << sh);
        const uint64_t r = sh ? v >> (32 - sh) : v >> 32;
        if (k + sh > 32) buf[i + 1] |= (uint32_t)r;
        if (k + sh > 64) buf[i + 2] |= (uint32_t)(r >> 32);
      }
    }
    pos += n;
  }
  __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
};

__device__ __forceinline__ void block4d_coords(const FieldDesc& F, uint32_t b, uint32_t* ib)
{
  uint32_t r = b / F.bx;
  ib[0] = b - r * F.bx;
  uint32_t r2 = r / F.by;
  ib[1] = r - r2 * F.by;
  ib[3] = r2 / F.bz;
  ib[2] = r2 - ib[3] * F.bz;
}

// LDS line lifts of a 4 x 4 x 4 x 4 int block, one line per lane, in libzfp's direction order
__device__ __forceinline__ void lift4d_lines(int32_t* q, uint32_t lane, bool inverse)
{
#pragma unroll
  for (int step = 0; step < 4; step++) {
    const int dir = inverse ? 3 - step : step;
    uint32_t base, st;
    if (dir == 0) { base = 4 * lane; st = 1; }
    else if (dir == 1) { base = (lane & 3) + 16 * (lane >> 2); st = 4; }
    else if (dir == 2) { base = (lane & 15) + 64 * (lane >> 4); st = 16; }
    else { base = lane; st = 64; }
    int32_t x = q[base], y = q[base + st], z = q[base + 2 * st], w = q[base + 3 * st];
    if (inverse) inv_lift(x, y, z, w);
    else fwd_lift(x, y, z, w);
    q[base] = x; q[base + st] = y; q[base + 2 * st] = z; q[base + 3 * st] = w;
    __syncthreads();
  }
}

// encode: lens != null -> bit count per block; else write at rbase[b] (variable) or b * maxbits (fixed)
template <int DT>
__global__ __launch_bounds__(64) void k_encode4d(FieldDesc F, Params p, uint32_t* __restrict__ lens,
                                                 const uint64_t* __restrict__ rbase, uint32_t* __restrict__ out32,
                                                 uint64_t* __restrict__ index, uint32_t index_shift)
{
  constexpr uint32_t OBW = (31 + 9 + 255 + 256 * 32 + 16658 + 31) / 32 + 3;  // header + bound (+ pad to minbits)
  __shared__ int32_t q[256];
  __shared__ uint32_t obuf[OBW];
  const uint32_t lane = threadIdx.x, b = blockIdx.x;
  uint32_t ib[4];
  block4d_coords(F, b, ib);
  uint32_t nv[4];
#pragma unroll
  for (int a = 0; a < 4; a++) nv[a] = (uint32_t)min<uint64_t>(4, F.n[a] - 4ull * ib[a]);
  const uint32_t y = lane & 3, z = (lane >> 2) & 3, t = lane >> 4;
  const int64_t row = (int64_t)(4ull * ib[1] + pad_index(y, nv[1])) * F.s[1] +
                      (int64_t)(4ull * ib[2] + pad_index(z, nv[2])) * F.s[2] +
                      (int64_t)(4ull * ib[3] + pad_index(t, nv[3])) * F.s[3] + (int64_t)(4ull * ib[0]) * F.s[0];
  float f[4];
#pragma unroll
  for (int x = 0; x < 4; x++) f[x] = load_elem<DT>(F.data, row + (int64_t)pad_index(x, nv[0]) * F.s[0]);
  uint32_t m = 0;
#pragma unroll
  for (int x = 0; x < 4; x++) {
    const uint32_t a = __float_as_uint(f[x]) & 0x7fffffffu;
    m = (a <= 0x7f800000u && a > m) ? a : m;  // NaN never wins (encode.c:146-150)
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  const int emax = m == 0 ? -127 : (m >= 0x7f800000u ? 0 : max((int)(m >> 23) - 126, -126));
  const uint32_t prec = precision(emax, p.maxprec, p.minexp, 4);
  const uint32_t be = prec ? (uint32_t)(emax + 127) : 0u;
  const uint32_t o0 = lens ? 0u : (uint32_t)((rbase ? rbase[b] : (uint64_t)b * p.maxbits) & 31u);
  for (uint32_t i = lane; i < OBW; i += 64) obuf[i] = 0u;
  __syncthreads();
  UniWriter w{obuf, o0, o0 + p.maxbits, lane};
  uint32_t total;
  if (!be) {
    total = max(1u, p.minbits);
  } else {
    w.put(2ull * be + 1ull, 9);
    const float sc = cast_scale(emax);
    int32_t qq[4];
#pragma unroll
    for (int x = 0; x < 4; x++) qq[x] = cast1(f[x], sc);
#pragma unroll
    for (int x = 0; x < 4; x++) q[4 * lane + x] = qq[x];
    __syncthreads();
    lift4d_lines(q, lane, false);
    uint32_t u[4];
#pragma unroll
    for (int j = 0; j < 4; j++) u[j] = ((uint32_t)q[g_perm4[lane + 64 * j]] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
    const uint32_t maxb = p.maxbits - 9u, minb = p.minbits - min(p.minbits, 9u);
    const uint32_t budget = exceeded_maxbits(maxb, prec, 256) ? maxb : 0xffffffffu;
    const int kmin = prec < 32 ? 32 - (int)prec : 0;
    uint32_t bits = 0, n = 0;  // encode_partial_bitplanes (encode.c:279-339), planes of 256 bits
    for (int k = 31; k >= kmin && bits < budget; --k) {
      Plane256 x;
#pragma unroll
      for (int j = 0; j < 4; j++) x.w[j] = __ballot((u[j] >> k) & 1u);
      for (uint32_t o = 0; o < n; o += 64) w.put(x.bits(o) & lowmask64(min(64u, n - o)), min(64u, n - o));
      bits += n;
      x.shr(n);
      while (n < 256 && bits < budget) {
        const uint32_t tz = x.ctz();
        if (tz == 256) {  // negative group test
          w.skip(1);
          bits += 1;
          break;
        }
        if (n + tz < 255) {  // group '1', tz zeros, the one-bit
          w.put(1ull, 1);
          w.skip(tz);
          w.put(1ull, 1);
          bits += tz + 2;
          n += tz + 1;
          x.shr(tz + 1);
        } else {  // the one-bit sits in the last position and is implied
          w.put(1ull, 1);
          w.skip(255 - n);
          bits += 256 - n;
          n = 256;
        }
      }
    }
    bits = bits < budget ? bits : budget;
    total = 9 + max(bits, minb);
  }
  if (lens) {
    if (lane == 0) lens[b] = total;
    return;
  }
  __syncthreads();
  const uint64_t base = rbase ? rbase[b] : (uint64_t)b * p.maxbits;
  const uint32_t W = (o0 + total + 31) >> 5;
  const uint64_t gw0 = base >> 5;
  for (uint32_t j = lane; j < W; j += 64) {
    const uint32_t v = obuf[j];
    if ((j == 0 && o0) || (j == W - 1 && ((o0 + total) & 31))) atomicOr(out32 + gw0 + j, v);  // shared words
    else out32[gw0 + j] = v;
  }
  if (index && lane == 0 && (b & ((1u << index_shift) - 1)) == 0) index[b >> index_shift] = base;
  if (lane == 0 && b == F.nblocks - 1) {
    const uint64_t endw = (base + total + 31) >> 5;
    if (endw & 1) out32[endw] = 0u;  // stream_flush: zero-pad to a 64-bit boundary
  }
}

// decode one 4-D block at r.pos (wave-uniform reads; every lane ends with the same r.pos), then scatter it;
// libzfp decode_ints semantics. Returns the bits the block occupies in a variable-rate stream (padded to minbits).
__device__ __forceinline__ uint64_t decode4d_block(const FieldDesc& F, const Params& p, BitReader& r, uint32_t b,
                                                   int32_t* q, uint32_t lane)
{
  const uint64_t start = r.pos;
  uint32_t u[4] = {0u, 0u, 0u, 0u};
  int emax = 0;
  const bool nonzero = r.bit();
  if (nonzero) {
    emax = (int)r.get(8) - 127;
    const uint32_t prec = precision(emax, p.maxprec, p.minexp, 4);
    const uint32_t maxb = p.maxbits - 9u;
    uint32_t bits = exceeded_maxbits(maxb, prec, 256) ? maxb : 0xffffffffu;
    const int kmin = prec < 32 ? 32 - (int)prec : 0;
    uint32_t n = 0;
    for (int k = 31; bits && k >= kmin; --k) {  // decode.c:141-183 with 256-bit planes
      Plane256 x{{0ull, 0ull, 0ull, 0ull}};
      const uint32_t m = min(n, bits);
      bits -= m;
      for (uint32_t o = 0; o < m; o += 64) x.w[o >> 6] = r.get(min(64u, m - o));
      while (n < 256 && bits) {
        bits--;
        if (!r.bit()) break;  // negative group test
        uint32_t lim = min(255u - n, bits), adv = 0;  // zeros the scan may read
        for (;;) {
          const uint64_t v = r.peek64();
          const uint32_t zz = v ? (uint32_t)__builtin_ctzll(v) : 64u;
          if (adv + zz < lim && zz < 64) {  // zeros, then the one-bit
            r.pos += zz + 1;
            bits -= zz + 1;
            n += zz;
            break;
          }
          if (zz == 64 && adv + 64 < lim) {
            r.pos += 64;
            bits -= 64;
            n += 64;
            adv += 64;
            continue;
          }
          r.pos += lim - adv;  // the scan ran into the last coefficient or the budget: the one is implied
          bits -= lim - adv;
          n += lim - adv;
          break;
        }
        x.w[n >> 6] |= 1ull << (n & 63);
        n++;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) u[j] |= (uint32_t)((x.w[j] >> lane) & 1u) << k;
    }
  }
  const uint64_t used = max<uint64_t>(r.pos - start, p.minbits);
#pragma unroll
  for (int j = 0; j < 4; j++) q[g_perm4[lane + 64 * j]] = (int32_t)((u[j] ^ 0xaaaaaaaau) - 0xaaaaaaaau);
  __syncthreads();
  lift4d_lines(q, lane, true);
  const float sc = dequant_scale(emax);
  uint32_t ib[4];
  block4d_coords(F, b, ib);
  uint32_t nv[4];
#pragma unroll
  for (int a = 0; a < 4; a++) nv[a] = (uint32_t)min<uint64_t>(4, F.n[a] - 4ull * ib[a]);
  const uint32_t y = lane & 3, z = (lane >> 2) & 3, t = lane >> 4;
  if (y < nv[1] && z < nv[2] && t < nv[3]) {
    float* out = (float*)F.data;
    const int64_t row = (int64_t)(4ull * ib[0]) * F.s[0] + (int64_t)(4ull * ib[1] + y) * F.s[1] +
                        (int64_t)(4ull * ib[2] + z) * F.s[2] + (int64_t)(4ull * ib[3] + t) * F.s[3];
    for (uint32_t x = 0; x < nv[0]; x++) out[row + (int64_t)x * F.s[0]] = nonzero ? sc * (float)q[4 * lane + x] : 0.0f;
  }
  __syncthreads();  // q is reused by the next block of a sequential walk
  return used;
}

// decode: blocks at index[b] (variable, index stride 1) or b * maxbits (fixed), one wave per block
__global__ __launch_bounds__(64) void k_decode4d(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                 const uint64_t* __restrict__ index, uint64_t base_bits)
{
  __shared__ int32_t q[256];
  const uint32_t b = blockIdx.x;
  BitReader r{in, base_bits + (index ? index[b] : (uint64_t)b * p.maxbits)};
  decode4d_block(F, p, r, b, q, threadIdx.x);
}

// variable-rate stream without a block index (e.g. a zfpy stream): one wave walks the blocks in order, each block
// starting where the previous one ended; the end bit goes to *end when asked
__global__ __launch_bounds__(64) void k_decode4d_seq(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                     uint64_t base_bits, uint64_t* __restrict__ end)
{
  __shared__ int32_t q[256];
  uint64_t pos = base_bits;
  for (uint32_t b = 0; b < F.nblocks; b++) {
    BitReader r{in, pos};
    pos += decode4d_block(F, p, r, b, q, threadIdx.x);
  }
  if (end && threadIdx.x == 0) *end = pos;
}

// exclusive scan of per-block lengths: one "range" per block through k_scan_ranges (which also zeroes the words
// two blocks share)
__global__ void k_widen_u32(const uint32_t* __restrict__ a, uint32_t n, uint64_t* __restrict__ o)
{
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) o[i] = a[i];
}

// ------------------------------------------------------------------------------------------------ fast 1-D decode
// Fixed-rate 1-D decoder for whole-word blocks (maxbits 64 / 32, kmin = 0), the inverse of the lean-4 encoder:
//  * header: bit 0 = 0 -> zero block; else biased emax in bits 1..8;
//  * the empty planes above M0 are single '0' bits, so M0 = 31 - ctz(word >> 9);
//  * group phase: one stream-window lookup per plane in a (n, next 7 bits) -> (nibble, length, n') table that
//    restates libzfp decode_ints' unary run-length decode (decode.c:156-189 with the block-size fix); rows n >= 3
//    are verbatim nibbles, so a wave-uniform loop runs until every lane has n >= 3 and the rest is a contiguous
//    nibble run taken straight from the word;
//  * the nibble window is turned back into four coefficients by the inverse 4 x 16 bit transpose.
// A lane whose group phase runs past the 16-plane window falls back to the generic decoder.
// Entry (n, r, b): decode one plane from state n with the next 7 stream bits b of which only r + 1 are inside the
// block's bit budget (r = 7: at least 8). The budget matters exactly like libzfp's: when it runs out inside the
// unary scan, decode_ints still deposits the coefficient at the current n (x += 1 << n++ after the inner loop).
struct alignas(16) DecTab1 {
  uint16_t v[5 * 8 * 128];
};

__host__ __device__ constexpr uint32_t dec_plane_cx(uint32_t t)
{
  const uint32_t n0 = t >> 10, r = (t >> 7) & 7u, b = t & 127u;
  uint32_t n = n0, bits = r + 1, pos = 0, x = 0;
  if (n >= 4) {  // verbatim nibble (zero past the budget)
    const uint32_t m = bits < 4 ? bits : 4;
    return (b & ((1u << m) - 1u)) | (m << 4) | (4u << 8);
  }
  const uint32_t m = n < bits ? n : bits;  // first n bits verbatim
  x = b & ((1u << m) - 1u);
  pos = m;
  bits -= m;
  while (n < 4 && bits) {
    bits--;
    if (!((b >> pos++) & 1u)) break;  // group test
    while (n < 3 && bits) {
      bits--;
      if ((b >> pos++) & 1u) break;
      n++;
    }
    x += 1u << n;
    n++;
  }
  return x | (pos << 4) | (n << 8);
}

__host__ __device__ constexpr DecTab1 make_dec_tab1()
{
  DecTab1 T{};
  for (uint32_t t = 0; t < 5 * 8 * 128; t++) T.v[t] = (uint16_t)dec_plane_cx(t);
  return T;
}

__device__ const DecTab1 g_dec_tab1 = make_dec_tab1();

// The no-budget rows (r = 7) of the plane table, indexed (n, 7 bits): what the variable-rate decoders use (640 entries,
// 1280 bytes: one 16-byte load for 80 lanes).
struct alignas(16) DecTab7 {
  uint16_t v[5 * 128];
};

__host__ __device__ constexpr DecTab7 make_dec_tab7()
{
  DecTab7 T{};
  for (uint32_t t = 0; t < 5 * 128; t++) T.v[t] = (uint16_t)dec_plane_cx(((((t >> 7) << 3) | 7u) << 7) | (t & 127u));
  return T;
}

__device__ const DecTab7 g_dec_tab7 = make_dec_tab7();

__device__ __forceinline__ uint64_t inv_transpose4x16(uint64_t x)
{
  x = dswap64(x, 0x00000000FF00FF00ull, 24);
  x = dswap64(x, 0x0000F0F00000F0F0ull, 12);
  x = dswap64(x, 0x00000000CCCCCCCCull, 30);
  x = dswap64(x, 0x0000AAAA0000AAAAull, 15);
  return x;
}

// coefficient i's bits for 16 planes starting at plane `top` going down, from a nibble window
__device__ __forceinline__ void window_to_coeffs(uint64_t Y, int top, uint32_t* u)
{
  const uint64_t x = inv_transpose4x16(Y);
  const uint32_t sh = (uint32_t)(31 - top);
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] |= __builtin_bitreverse32((uint32_t)(x >> (16 * i)) & 0xffffu) >> sh;
}

template <uint32_t WB>
__device__ __forceinline__ void decode_block1d_fast(uint64_t w, const uint16_t* dtab, float* f, bool& special)
{
  const bool nonzero = w & 1u;
  const int emax = (int)((w >> 1) & 255u) - 127;
  const uint64_t r = w >> 9;
  const int z = r ? (int)__builtin_ctzll(r) : 64;
  const int M0 = 31 - z;  // < 0: every coded plane empty
  uint32_t pos = 9u + (uint32_t)z;
  uint64_t Y = 0;
  uint32_t n = 0;
  int j = 0;
#pragma unroll
  for (; j < 16; j++) {
    if (!__any(n < 3 && pos < WB && j <= M0)) break;
    const uint32_t b7 = pos < WB ? (uint32_t)(w >> pos) & 127u : 0u;
    const uint32_t rb = min(WB - pos, 8u) - 1u;  // budget bits left in this plane (pos >= WB: b7 = 0, any row)
    const uint32_t e = dtab[(((n << 3) | rb) << 7) | b7];
    Y |= (uint64_t)(e & 15u) << (4 * j);
    pos += (e >> 4) & 15u;
    n = e >> 8;
  }
  special = n < 3 && pos < WB && j <= M0;  // still in the group phase after 16 planes
  if (j < 16 && pos < WB) Y |= (w >> pos) << (4 * j);  // verbatim nibbles (bits past the word are zero)
  uint32_t u[4] = {0, 0, 0, 0};
  if (M0 >= 0) {
    window_to_coeffs(Y, M0, u);
    const uint32_t p2 = pos + 4u * (uint32_t)(16 - j);  // stream position of plane M0 - 16
    if (__any(p2 < WB && M0 >= 16)) {
      const uint64_t Y2 = p2 < WB && M0 >= 16 ? w >> p2 : 0ull;
      if (M0 >= 16) window_to_coeffs(Y2, M0 - 16, u);
    }
  }
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = (int32_t)((u[i] ^ 0xaaaaaaaau) - 0xaaaaaaaau);
  inv_lift(q[0], q[1], q[2], q[3]);
  const float sc = dequant_scale(emax);
#pragma unroll
  for (int i = 0; i < 4; i++) f[i] = nonzero ? sc * (float)q[i] : 0.0f;  // header bit 0: +0 whatever follows
}

#ifndef GCOW_DEC_PAIR
#define GCOW_DEC_PAIR 1
#endif
#ifndef GCOW_DEC_GATHER
#define GCOW_DEC_GATHER 1  // decode_mean's pair decoder: the inverse window transpose through LDS gather tables
#endif
#ifndef GCOW_DEC_PAIR2
#define GCOW_DEC_PAIR2 1  // decode_block1d_pair: select-free steps (budget / window overruns only flag the block special)
#endif
// ---- two planes per lookup (64-bit blocks). The group phase lasts 1.5 planes on average on gradient-like data but
// the wave-uniform loop above runs the wave's maximum (4.6 planes: profiles/r04_dec_pair_table.log), so each step
// here decodes as many of the next two planes as the next 10 stream bits determine, and lanes step on their own.
// Entry (n < 3, 10 bits): nibbles of plane 1 [0, 4) and plane 2 [4, 8), plane 1's length [8, 12), both planes'
// length [12, 16), min(n, 3) after plane 1 [16, 18) and after plane 2 [18, 20), plane 2 decoded [20] (only when its
// code ends inside the 10 bits: decoded with the bits past them zero, a code that stops before them read none).
struct alignas(16) DecTabP {
  uint32_t v[3 * 1024];
};

__host__ __device__ constexpr uint32_t dec_pair_cx(uint32_t t)
{
  const uint32_t n = t >> 10, b = t & 1023u;
  const uint32_t e1 = dec_plane_cx((((n << 3) | 7u) << 7) | (b & 127u));
  const uint32_t x1 = e1 & 15u, l1 = (e1 >> 4) & 15u, n1 = e1 >> 8;
  const uint32_t e2 = dec_plane_cx((((n1 << 3) | 7u) << 7) | ((b >> l1) & 127u));
  const uint32_t x2 = e2 & 15u, l2 = (e2 >> 4) & 15u, n2 = e2 >> 8;
  const uint32_t r1 = n1 < 3 ? n1 : 3u, r2 = n2 < 3 ? n2 : 3u;
  if (l1 + l2 <= 10u) return x1 | (x2 << 4) | (l1 << 8) | ((l1 + l2) << 12) | (r1 << 16) | (r2 << 18) | (1u << 20);
  return x1 | (l1 << 8) | (l1 << 12) | (r1 << 16) | (r1 << 18);
}

__host__ __device__ constexpr DecTabP make_dec_pair()
{
  DecTabP T{};
  for (uint32_t t = 0; t < 3 * 1024; t++) T.v[t] = dec_pair_cx(t);
  return T;
}

__device__ const DecTabP g_dec_pair = make_dec_pair();

// The inverse of the encoder's spread tables (lean1d.h SpreadTab): the nibble window back to coefficient bytes by
// lookups. Window byte k (nibbles 2k, 2k + 1: planes top - 2k, top - 2k - 1) through table s = k mod 4 puts
// coefficient i's two bits at bits 7 - 2s and 6 - 2s of byte i; OR-ing bytes 0..3 gives A (byte i = coefficient i's
// planes top .. top - 7, MSB first), bytes 4..7 give B (planes top - 8 .. top - 15), and one v_perm_b32 per
// coefficient lays A_i, B_i into bits 31..16 ahead of the shift to `top`. 8 LDS reads and ~20 VALU per window where
// window_to_coeffs' four 64-bit delta swaps, bit reversals and shifts take ~52.
struct alignas(16) GatherTab {
  uint32_t v[4 * 256];
};

__host__ __device__ constexpr GatherTab make_gather_tab()
{
  GatherTab T{};
  for (uint32_t s = 0; s < 4; s++)
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t r = 0;
      for (uint32_t i = 0; i < 4; i++) {
        r |= ((b >> i) & 1u) << (8 * i + 7 - 2 * s);
        r |= ((b >> (4 + i)) & 1u) << (8 * i + 6 - 2 * s);
      }
      T.v[256 * s + b] = r;
    }
  return T;
}

// the pair table and the gather tables as one LDS image (the fixed-rate pair decoders stage both in one pass)
struct alignas(16) DecTabPG {
  uint32_t v[3 * 1024 + 4 * 256];
};

__host__ __device__ constexpr DecTabPG make_dec_pair_gather()
{
  DecTabPG T{};
  const DecTabP P = make_dec_pair();
  const GatherTab G = make_gather_tab();
  for (uint32_t t = 0; t < 3 * 1024; t++) T.v[t] = P.v[t];
  for (uint32_t t = 0; t < 4 * 256; t++) T.v[3 * 1024 + t] = G.v[t];
  return T;
}

__device__ const DecTabPG g_dec_pair_gather = make_dec_pair_gather();

// The variable-rate lean decoder's LDS image: the pair table as 16-bit entries (n < 3, next 10 bits) -> nibbles
// [0, 8), bits taken [8, 12), min(n, 3) after [12, 14), two planes taken [14] (dec_pair_cx's fields), then the plane
// table's 640 entries (DecTab7) for a step that may take one plane only (the block's last coded plane, or the last
// of the 8-plane group window) and for the general decoder. 7424 bytes.
struct alignas(16) DecTabLP {
  uint16_t v[3 * 1024 + 5 * 128];
};

__host__ __device__ constexpr DecTabLP make_dec_lean_pair()
{
  DecTabLP T{};
  for (uint32_t t = 0; t < 3 * 1024; t++) {
    const uint32_t e = dec_pair_cx(t);
    T.v[t] = (uint16_t)((e & 255u) | (((e >> 12) & 15u) << 8) | (((e >> 18) & 3u) << 12) | (((e >> 20) & 1u) << 14));
  }
  const DecTab7 S = make_dec_tab7();
  for (uint32_t t = 0; t < 5 * 128; t++) T.v[3 * 1024 + t] = S.v[t];
  return T;
}

__device__ const DecTabLP g_dec_lean_pair = make_dec_lean_pair();


__device__ __forceinline__ void window_to_coeffs_lds(const uint32_t* gt, uint64_t Y, int top, uint32_t* u)
{
  const uint32_t lo = (uint32_t)Y, hi = (uint32_t)(Y >> 32);
  const uint32_t A = gt[lo & 255u] | gt[256 + ((lo >> 8) & 255u)] | gt[512 + ((lo >> 16) & 255u)] | gt[768 + (lo >> 24)];
  const uint32_t B = gt[hi & 255u] | gt[256 + ((hi >> 8) & 255u)] | gt[512 + ((hi >> 16) & 255u)] | gt[768 + (hi >> 24)];
  const uint32_t sh = (uint32_t)(31 - top);
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) u[i] |= __builtin_amdgcn_perm(A, B, ((4u + i) << 24) | (i << 16) | 0x0c0cu) >> sh;
}

// decode_block1d_fast<64> with the pair table: a lane leaves the loop when its group phase ends (n >= 3), its planes
// run out (j > M0) or the 16-plane window is full; a plane that would cross the 64-bit budget goes to the generic
// decoder (special), as does a group phase longer than the window.
template <bool GATHER>
__device__ __forceinline__ void decode_block1d_pair(uint64_t w, const uint32_t* dtp, float* f, bool& special)
{
  const bool nonzero = w & 1u;
  const int emax = (int)((w >> 1) & 255u) - 127;
#if GCOW_DEC_PAIR2
  // header bit 0: +0 whatever follows -- taken as a block whose planes are all empty (u = 0, so every value is
  // sc * 0 = +0 with sc >= 0), not selected per value at the end
  const uint64_t r = nonzero ? w >> 9 : 0ull;
#else
  const uint64_t r = w >> 9;
#endif
  const int z = r ? (int)__builtin_ctzll(r) : 64;
  const int M0 = 31 - z;  // < 0: every coded plane empty
  uint32_t pos = 9u + (uint32_t)z;
  uint64_t Y = 0;
  uint32_t n = 0;
  int j = 0;
#if GCOW_DEC_PAIR2
  // Every step takes the entry's two-plane fields (which fall back to the first plane's when the second is not
  // decoded within the 10 bits), with no per-step budget or window selects; what they would have guarded only makes
  // the block special: a plane code crossing the 64-bit budget leaves pos > 64, and a step from nibble 15 (j ends at
  // 17) consumed plane M0 - 16, which belongs to the second window. A second plane below plane 0 (a step from j = M0)
  // lands past the coefficients' low bit and is shifted out by window_to_coeffs; its length only matters for pos > 64.
  const int jm = min(M0, 15);
#pragma unroll
  for (int it = 0; it < 16; it++) {
    // the first step is every lane with a coded plane (n = 0, j = 0, pos <= 40): no wave vote
    const bool act = it == 0 ? M0 >= 0 : n < 3 && pos < 64u && j <= jm;
    if (it > 0 && !__any(act)) break;
    if (act) {
      const uint32_t e = dtp[(n << 10) | ((uint32_t)(w >> pos) & 1023u)];
      Y |= (uint64_t)(e & 255u) << (4 * j);
      pos += (e >> 12) & 15u;
      n = (e >> 18) & 3u;
      j += 1 + (int)((e >> 20) & 1u);
    }
  }
  // special: a plane code crossed the budget, or the steps reached nibble 16 (a group phase as long as the window, or
  // a step from nibble 15 that consumed plane M0 - 16; a group phase that ended exactly at nibble 16 is decoded
  // generically too, which only costs time). Otherwise every coded plane is in Y: the loop stopped with n >= 3, with
  // the budget used up (pos = 64), or past plane 0.
  special = M0 >= 0 && (pos > 64u || j >= 16);
#else
  bool cross = false;
#pragma unroll
  for (int it = 0; it < 16; it++) {
    const uint32_t rem = 64u - min(pos, 64u);
    const bool act = n < 3 && rem && j <= M0 && j < 16 && !cross;
    if (!__any(act)) break;
    if (act) {
      const uint32_t e = dtp[(n << 10) | ((uint32_t)(w >> pos) & 1023u)];
      const uint32_t l1 = (e >> 8) & 15u, l2 = (e >> 12) & 15u;
      cross = l1 > rem;
      const bool two = ((e >> 20) & 1u) && l2 <= rem && j < M0 && j < 15;
      if (!cross) {
        Y |= (uint64_t)(two ? (e & 255u) : (e & 15u)) << (4 * j);
        pos += two ? l2 : l1;
        n = (e >> (two ? 18 : 16)) & 3u;
        j += two ? 2 : 1;
      }
    }
  }
  special = cross || (n < 3 && pos < 64u && j <= M0);  // budget inside a group plane, or a group phase past 16 planes
#endif
#if GCOW_DEC_PAIR2
  // verbatim nibbles (bits past the word are zero): pos >= 9, so the two-step shift gives 0 at pos = 64; lanes with
  // pos > 64 or j >= 16 are special and their Y is not used
  Y |= ((w >> (pos - 1u)) >> 1) << (4 * j);
#else
  if (j < 16 && pos < 64u) Y |= (w >> pos) << (4 * j);  // verbatim nibbles (bits past the word are zero)
#endif
  uint32_t u[4] = {0, 0, 0, 0};
  if (M0 >= 0) {
    if constexpr (GATHER) window_to_coeffs_lds(dtp + 3 * 1024, Y, M0, u);
    else window_to_coeffs(Y, M0, u);
    const uint32_t p2 = pos + 4u * (uint32_t)(16 - min(j, 16));  // stream position of plane M0 - 16
    if (__any(p2 < 64u && M0 >= 16)) {
      const uint64_t Y2 = p2 < 64u && M0 >= 16 ? w >> p2 : 0ull;
      if (M0 >= 16) {
        if constexpr (GATHER) window_to_coeffs_lds(dtp + 3 * 1024, Y2, M0 - 16, u);
        else window_to_coeffs(Y2, M0 - 16, u);
      }
    }
  }
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = (int32_t)((u[i] ^ 0xaaaaaaaau) - 0xaaaaaaaau);
  inv_lift(q[0], q[1], q[2], q[3]);
#if GCOW_DEC_PAIR2
  // (float)q * 2^(emax - 30) as one v_ldexp_f32 per value: the product by the exact power of two that dequant_scale
  // gives, rounded once alike (denormal results included); below 2^-149 dequant_scale's 0 gives a signed zero, which
  // the ldexp gives at any exponent under -181 (|q| < 2^31)
  const int e = emax - 30 < -149 ? -256 : emax - 30;
#pragma unroll
  for (int i = 0; i < 4; i++) f[i] = __builtin_amdgcn_ldexpf((float)q[i], e);  // header bit 0: q = 0 above
#else
  const float sc = dequant_scale(emax);
#pragma unroll
  for (int i = 0; i < 4; i++) f[i] = nonzero ? sc * (float)q[i] : 0.0f;  // header bit 0: +0 whatever follows
#endif
}

template <uint32_t WB> struct PipeWord;
template <> struct PipeWord<64> {
  typedef pipe_v2u T;
  static __device__ __forceinline__ T load(uint32_t off, pipe_v4i rs)
  {
    T v;
    asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(rs) : "memory");
    return v;
  }
  static __device__ __forceinline__ uint64_t get(const T& v) { return (uint64_t)v.x | ((uint64_t)v.y << 32); }
};
template <> struct PipeWord<32> {
  typedef uint32_t T;
  static __device__ __forceinline__ T load(uint32_t off, pipe_v4i rs)
  {
    T v;
    asm volatile("buffer_load_dword %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(rs) : "memory");
    return v;
  }
  static __device__ __forceinline__ uint64_t get(const T& v) { return (uint64_t)v; }
};

// Wait until at most N vector memory operations are outstanding, tying the TR table registers to after the wait.
template <int N, uint32_t TR>
__device__ __forceinline__ void table_wait(pipe_v4u (&tv)[TR])
{
  if constexpr (TR == 3) {
    asm volatile("s_waitcnt vmcnt(%3)" : "+v"(tv[0]), "+v"(tv[1]), "+v"(tv[2]) : "n"(N) : "memory");
  } else {
    static_assert(TR == 4, "three or four table registers per lane");
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(tv[0]), "+v"(tv[1]), "+v"(tv[2]), "+v"(tv[3]) : "n"(N) : "memory");
  }
}

// decode_mean's pair-decoder LDS image: the pair table, then (GCOW_DEC_GATHER) the gather tables
__device__ __forceinline__ const void* dec_pair_image()
{
  return GCOW_DEC_GATHER ? (const void*)&g_dec_pair_gather : (const void*)&g_dec_pair;
}

// One-shot fixed-rate 1-D decoder (the shape of k_encode_fixed1d_np): each lane decodes U blocks 256 apart inside
// its workgroup's chunk; the U word loads are issued before the table fill, and block k waits for its own word only
// (U loads then k stores outstanding: vmcnt(U - 1)).
template <uint32_t WB, int U, bool BF = false>
__global__ __launch_bounds__(256) void k_decode_fixed1d_np(const void* __restrict__ in, uint32_t nfull, Params p,
                                                           void* __restrict__ out, uint64_t base_bits)
{
  // 64-bit blocks: the two-plane table, at U = 8 (at U = 16 the unrolled pair loop keeps the block loop rolled, which
  // its counted waits cannot take; profiles/r04_dec_pair_table.log)
#ifndef GCOW_C2DEC_PAIR
#define GCOW_C2DEC_PAIR 1
#endif
  constexpr bool PAIR = WB == 64 && GCOW_C2DEC_PAIR;
  using PTab = DecTabP;  // the delta-swap inverse transpose: gather tables measured +4.5 % steady here (-6 % cold)
  using Tab = typename std::conditional<PAIR, PTab, DecTab1>::type;
  __shared__ __attribute__((aligned(16))) uint32_t dtab32[sizeof(Tab) / 4];
  const uint16_t* dtab = (const uint16_t*)dtab32;
  constexpr uint32_t WBYTES = WB / 8;
  const pipe_v4i rin = buf_rsrc((const char*)in + base_bits / 8, nfull * WBYTES);
  // output: 16 B per block (fp32), or 8 B (BF: bf16, rounded to nearest even)
  const __amdgpu_buffer_rsrc_t rout_b = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(nfull * (BF ? 8u : 16u)), 0x00020000);
  const uint32_t b0 = blockIdx.x * (256u * U) + threadIdx.x;
  // the plane table (10 KiB, 640 16-byte chunks; 64-bit blocks: the 12 KiB pair table and the 4 KiB gather tables,
  // 1024 chunks; 3-4 per lane, the range check zeroes the rest) is requested first and
  // waited for with vmcnt(U): the U word loads behind it stay in flight, and no wait counts a memory round trip per
  // table chunk (as a compiler-issued copy loop does)
  constexpr uint32_t TCH = sizeof(Tab) / 16, TR = (TCH + 255) / 256;
  const pipe_v4i rt = PAIR ? buf_rsrc(&g_dec_pair, sizeof(PTab)) : buf_rsrc(&g_dec_tab1, sizeof(DecTab1));
  pipe_v4u tv[TR];
#pragma unroll
  for (uint32_t i = 0; i < TR; i++) tv[i] = buf_load_b128((threadIdx.x + 256u * i) * 16u, rt);
  typename PipeWord<WB>::T r[U];
#pragma unroll
  for (int k = 0; k < U; k++) r[k] = PipeWord<WB>::load((b0 + 256u * k) * WBYTES, rin);
  table_wait<U>(tv);
#pragma unroll
  for (uint32_t i = 0; i < TR; i++)
    if (threadIdx.x + 256u * i < TCH) ((pipe_v4u*)dtab32)[threadIdx.x + 256u * i] = tv[i];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < U; k++) {
    pipe_wait<U - 1>(r[k]);
    const uint32_t b = b0 + 256u * k;
    float f[4];
    bool special;
    if constexpr (PAIR) decode_block1d_pair<false>(PipeWord<WB>::get(r[k]), dtab32, f, special);
    else decode_block1d_fast<WB>(PipeWord<WB>::get(r[k]), dtab, f, special);
    if (special && b < nfull) {
      BitReader rd{(const uint64_t*)in, base_bits + (uint64_t)b * WB};
      decode_block<1>(rd, p, f);
    }
    // 16-B (8-B) store through the compiler (it inserts the VALU-write -> wide-store wait states that an inline-asm
    // store would need by hand; with an asm store lanes 12-15 of each row stored stale data). It still counts in vmcnt
    // exactly once per block, as the hand-counted waits assume; aux 2 = non-temporal.
    if constexpr (BF) {
      pipe_v2u v;
      v.x = bf16x2_rne(f[0], f[1]);
      v.y = bf16x2_rne(f[2], f[3]);
      __builtin_amdgcn_raw_buffer_store_b64(v, rout_b, (int)(b * 8u), 0, 2);
    } else {
      pipe_v4u v;
      v.x = __float_as_uint(f[0]); v.y = __float_as_uint(f[1]); v.z = __float_as_uint(f[2]); v.w = __float_as_uint(f[3]);
      __builtin_amdgcn_raw_buffer_store_b128(v, rout_b, (int)(b * 16u), 0, 2);
    }
  }
}

// ------------------------------------------------------------------------------------------------ 1-D variable-rate
// decode. Variable-rate 1-D streams whose budget never truncates a block (minbits <= 1, maxbits >= 160: accuracy,
// precision, expert) decode block by block with the fixed-rate decoder's plane table instead of bit by bit: header,
// then the empty planes (one '0' each: a count-trailing-zeros), the group phase (one (n, 7 stream bits) lookup per
// plane while n < 3, down to kmin), then the remaining planes as a verbatim nibble run (a plane with n >= 3 is its
// nibble) and the inverse bit transpose; libzfp decode_ints semantics (decode.c:141-183 with the block-size fix).
// One lane per block-index chunk, blocks in sequence (each block's start is the previous block's end).
__device__ __forceinline__ uint64_t stream_window(const uint64_t* in, uint64_t pos)
{
  const uint64_t i = pos >> 6;
  const uint32_t sh = (uint32_t)(pos & 63);
  const uint64_t lo = in[i] >> sh;
  return sh ? lo | (in[i + 1] << (64 - sh)) : lo;
}

// 64 stream bits at a bit position, from global memory or from words staged in LDS (positions relative to them)
struct GlobalWindow {
  const uint64_t* in;
  __device__ __forceinline__ uint64_t operator()(uint64_t pos) const { return stream_window(in, pos); }
};
struct LdsWindow {
  const uint64_t* w;
  __device__ __forceinline__ uint64_t operator()(uint64_t pos) const
  {
    const uint32_t i = (uint32_t)(pos >> 6), sh = (uint32_t)(pos & 63);
    const uint64_t lo = w[i] >> sh;
    return sh ? lo | (w[i + 1] << (64 - sh)) : lo;
  }
};

// The same over a span staged with stage_lds16<.., SWZ = true> (qword q at lds_qword_swz(q)).
struct LdsWindowSwz {
  const uint64_t* w;
  __device__ __forceinline__ uint64_t operator()(uint64_t pos) const
  {
    const uint32_t i = (uint32_t)(pos >> 6), sh = (uint32_t)(pos & 63);
    const uint64_t lo = w[lds_qword_swz(i)] >> sh;
    return sh ? lo | (w[lds_qword_swz(i + 1)] << (64 - sh)) : lo;
  }
};

// dtab: the full (n, r, 7 bits) plane table, or (COMPACT) its r = 7 rows only, indexed (n, 7 bits)
template <class Win, bool COMPACT = true>
__device__ __forceinline__ void decode_block1d_var(const Win& win, uint64_t& pos, const uint16_t* dtab, int minexp,
                                                   uint32_t maxprec, float* f)
{
  uint64_t w = win(pos);
  if (!(w & 1u)) {  // zero block (or prec = 0): one 0 bit
    f[0] = f[1] = f[2] = f[3] = 0.0f;
    pos += 1;
    return;
  }
  const int emax = (int)((w >> 1) & 255u) - 127;
  const int prec = min((int)maxprec, max(0, emax - minexp + 4));
  const int kmin = prec < 32 ? 32 - prec : 0;
  const int np = 32 - kmin;  // coded planes 31 .. kmin
  pos += 9;
  w = win(pos);
  const int z = w ? (int)__builtin_ctzll(w) : 64;
  uint32_t u[4] = {0u, 0u, 0u, 0u};
  if (z >= np) {
    pos += (uint32_t)np;  // every coded plane empty
  } else {
    pos += (uint32_t)z;
    const int M0 = 31 - z;
    const int nbelow = M0 - kmin + 1;  // planes M0 .. kmin
    uint64_t Ylo = 0, Yhi = 0;         // plane nibbles M0 - j, j = 0..31
    uint32_t n = 0, used = 0;
    int j = 0;
    w = win(pos);
    while (n < 3 && j < nbelow) {
      if (used > 56) {
        pos += used;
        used = 0;
        w = win(pos);
      }
      const uint32_t e = dtab[(COMPACT ? (n << 7) : ((((n << 3) | 7u)) << 7)) | ((uint32_t)(w >> used) & 127u)];
      const uint64_t nib = e & 15u;
      if (j < 16) Ylo |= nib << (4 * j);
      else Yhi |= nib << (4 * (j - 16));
      used += (e >> 4) & 15u;
      n = e >> 8;
      j++;
    }
    pos += used;
    const int t = nbelow - j;  // planes left: 4 bits each, verbatim
    if (t > 0) {
      const uint32_t nb = 4u * (uint32_t)t;  // <= 128
      uint64_t v0 = win(pos), v1 = nb > 64 ? win(pos + 64) : 0ull;
      if (nb < 64) v0 &= (1ull << nb) - 1ull;
      else if (nb < 128) v1 &= (1ull << (nb - 64)) - 1ull;
      const uint32_t sft = 4u * (uint32_t)j;  // nibble position of the run; sft + nb <= 128
      if (sft == 0) {
        Ylo |= v0;
        Yhi |= v1;
      } else if (sft < 64) {
        Ylo |= v0 << sft;
        Yhi |= (v0 >> (64 - sft)) | (v1 << sft);
      } else {
        Yhi |= v0 << (sft - 64);
      }
      pos += nb;
    }
    window_to_coeffs(Ylo, M0, u);
    if (M0 >= 16) window_to_coeffs(Yhi, M0 - 16, u);
  }
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = (int32_t)((u[i] ^ 0xaaaaaaaau) - 0xaaaaaaaau);
  inv_lift(q[0], q[1], q[2], q[3]);
  const float sc = dequant_scale(emax);
#pragma unroll
  for (int i = 0; i < 4; i++) f[i] = sc * (float)q[i];
}

__global__ __launch_bounds__(256) void k_decode1d_var(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                      const uint64_t* __restrict__ index, uint32_t chunk,
                                                      uint64_t nchunks, uint64_t base_bits,
                                                      uint64_t* __restrict__ end_out)
{
  __shared__ __attribute__((aligned(16))) uint16_t dtab[5 * 128];  // r = 7 rows of the plane table
  stage_lds16<256, sizeof(DecTab7) / 16>(dtab, &g_dec_tab7, sizeof(DecTab7));
  __syncthreads();
  const uint64_t c = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (c >= nchunks) return;
  uint64_t pos = base_bits + (index ? index[c] : 0ull);
  const uint64_t b0 = c * chunk, b1 = min<uint64_t>(b0 + chunk, F.nblocks);
  float* out = (float*)F.data;
  if (chunk == 16 && 4 * b1 <= F.n[0] && b1 - b0 == 16) {
    // the chunk's 256 output bytes are decoded into registers and stored in one burst: stored as they are decoded,
    // every 128-B line stays half-written in L2 for most of the chunk's decode time
    float g[16][4];
#pragma unroll
    for (int k = 0; k < 16; k++) decode_block1d_var(GlobalWindow{in}, pos, dtab, p.minexp, p.maxprec, g[k]);
    if (F.dtype == DT_BF16) {
#pragma unroll
      for (int k = 0; k < 16; k++) store_block1d(F, b0 + k, g[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) *(float4*)(out + 4 * (b0 + k)) = make_float4(g[k][0], g[k][1], g[k][2], g[k][3]);
    }
    if (end_out && c == nchunks - 1) *end_out = pos;
    return;
  }
  for (uint64_t b = b0; b < b1; b++) {
    float f[4];
    decode_block1d_var(GlobalWindow{in}, pos, dtab, p.minexp, p.maxprec, f);
    if (F.dtype != DT_BF16 && 4 * b + 4 <= F.n[0]) *(float4*)(out + 4 * b) = make_float4(f[0], f[1], f[2], f[3]);
    else store_block1d(F, b, f);
  }
  if (end_out && c == nchunks - 1) *end_out = pos;
}

// ------------------------------------------------------------------------------------------------ lean 1-D var decode
// The variable-rate block decoder of the staged kernels, cut to what a block needs (libzfp decode_ints semantics,
// decode.c:141-183 with the block-size fix; minbits <= 1, maxbits >= 160, so no budget truncates):
//  * one 64-bit window at the block start gives the header, the precision and the run of empty planes (ctz over the
//    55 bits after the header covers any np <= 32) and, in the common case, the group phase's bits too (the window
//    is re-read only when a group plane's 7 lookup bits would run past it);
//  * the group phase (planes while fewer than 3 coefficients are significant) is at most 8 planes here, its nibbles
//    packed into one 32-bit word; a block whose group phase is longer takes the general decoder (rare: three
//    coefficients spread over more than 8 planes);
//  * the verbatim nibble run (4 bits per remaining plane) is one window, two past 64 bits;
//  * the inverse 4 x 16 bit transposes run for the planes present: the second half only when more than 16 planes
//    are coded (accuracy 1e-6 on gradient-scale data codes ~14).
// Positions are 32-bit, relative to the staged words (LDS), and windows are built from three 32-bit words with two
// v_alignbit_b32.
template <bool SWZ = false>
__device__ __forceinline__ uint64_t lds_win64(const uint32_t* w, uint32_t pos)
{
  if constexpr (SWZ) {  // two aligned qword reads of the swizzled span (ds_read_b64: 64 banks), three words selected
    const uint32_t q = pos >> 6;
    const uint2 lo = ((const uint2*)w)[lds_qword_swz(q)], hi = ((const uint2*)w)[lds_qword_swz(q + 1)];
    const bool up = (pos & 32u) != 0;
    const uint32_t a = up ? lo.y : lo.x, b = up ? hi.x : lo.y, c = up ? hi.y : hi.x;
    return ((uint64_t)__builtin_amdgcn_alignbit(c, b, pos) << 32) | __builtin_amdgcn_alignbit(b, a, pos);
  }
  const uint32_t i = pos >> 5;
  const uint32_t a = w[i], b = w[i + 1], c = w[i + 2];
  return ((uint64_t)__builtin_amdgcn_alignbit(c, b, pos) << 32) | __builtin_amdgcn_alignbit(b, a, pos);
}

// returns false when the block needs the general decoder (pos unchanged then). PAIR: tab is the DecTabLP image and
// the group phase decodes up to two planes per lookup; else tab is DecTab7.
template <bool PAIR = false, bool SWZ = false>
__device__ __forceinline__ bool dec_block1d_lean(const uint32_t* sw, uint32_t& pos, const uint16_t* tab, int cexp,
                                                 int maxprec, float* f)
{
  const uint64_t w = lds_win64<SWZ>(sw, pos);
  const int emax = (int)((w >> 1) & 255u) - 127;
  const int np = min(32, min(maxprec, max(0, emax + cexp)));  // coded planes 31 .. 32 - np
  // empty planes: ctz of the 55 bits after the header, a sentinel one at bit 55 for none (any np <= 32 < 55)
  const int z = (int)__builtin_ctzll((w >> 9) | (1ull << 55));
  f[0] = f[1] = f[2] = f[3] = 0.0f;
  if (!(w & 1u)) {  // zero block (or no precision): one 0 bit
    pos += 1;
    return true;
  }
  if (z >= np) {  // every coded plane empty: the values are +0
    pos += 9u + (uint32_t)np;
    return true;
  }
  const int M0 = 31 - z, nbelow = np - z;  // planes M0 .. M0 - nbelow + 1
  // group phase: one (n, 7 bits) lookup per plane while n < 3
  uint64_t gw = w;
  uint32_t off = 9u + (uint32_t)z, wbase = pos;
  uint32_t n = 0, G = 0;
  int j = 0;
  if constexpr (PAIR) {
    // (n, 10 bits) -> one or two planes; a second plane past the block's coded planes or past the 8-plane window is
    // not taken: that step re-reads the plane table for the first plane alone
    const uint16_t* dt7 = tab + 3 * 1024;
    const int lim = min(nbelow, 8);
    while (n < 3 && j < lim) {
      if (off > 54u) {
        wbase += off;
        gw = lds_win64<SWZ>(sw, wbase);
        off = 0;
      }
      const uint32_t b = (uint32_t)(gw >> off) & 1023u;
      const uint32_t e = tab[(n << 10) | b];
      uint32_t nib = e & 255u, len = (e >> 8) & 15u, nn = (e >> 12) & 3u, two = e >> 14;
      if (two && j + 1 >= lim) {
        const uint32_t e7 = dt7[(n << 7) | (b & 127u)];
        nib = e7 & 15u;
        len = (e7 >> 4) & 15u;
        nn = e7 >> 8;
        two = 0;
      }
      G |= nib << (4 * j);
      off += len;
      n = nn;
      j += 1 + (int)two;
    }
  } else {
    const uint16_t* dt7 = tab;
    while (n < 3 && j < nbelow && j < 8) {
      if (off > 57u) {
        wbase += off;
        gw = lds_win64<SWZ>(sw, wbase);
        off = 0;
      }
      const uint32_t e = dt7[(n << 7) | ((uint32_t)(gw >> off) & 127u)];
      G |= (e & 15u) << (4 * j);
      off += (e >> 4) & 15u;
      n = e >> 8;
      j++;
    }
  }
  if (n < 3 && j < nbelow) return false;  // group phase longer than 8 planes
  const uint32_t vpos = wbase + off;
  const uint32_t t = (uint32_t)(nbelow - j);  // verbatim planes, 4 bits each
  const uint32_t nb = 4u * t;                 // <= 128
  // the run's window is not masked at nb: the next block's bits beyond it land on planes below kmin = 32 - np, which
  // one mask of the coefficients clears
  uint64_t v0 = lds_win64<SWZ>(sw, vpos), v1 = 0;
  if (nb > 64) v1 = lds_win64<SWZ>(sw, vpos + 64);
  const uint32_t sft = 4u * (uint32_t)j;  // <= 32
  const uint64_t Ylo = (uint64_t)G | (v0 << sft);
  uint32_t u[4] = {0u, 0u, 0u, 0u};
  window_to_coeffs(Ylo, M0, u);
  if (nbelow > 16) {
    const uint64_t Yhi = ((v0 >> 1) >> (63u - sft)) | (v1 << sft);
    window_to_coeffs(Yhi, M0 - 16, u);
  }
  const uint32_t keep = ~0u << (uint32_t)(32 - np);  // planes 31 .. kmin (np >= 1 here)
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] &= keep;
  pos = vpos + nb;
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = (int32_t)((u[i] ^ 0xaaaaaaaau) - 0xaaaaaaaau);
  inv_lift(q[0], q[1], q[2], q[3]);
  const int e = emax - 30 < -149 ? -256 : emax - 30;  // as decode_block1d_pair: ldexp = dequant_scale(emax) * q
#pragma unroll
  for (int i = 0; i < 4; i++) f[i] = __builtin_amdgcn_ldexpf((float)q[i], e);
  return true;
}

// One stage of the 8 x 8 transpose of float4 elements across the 8-lane groups of a wave (butterfly over lane bit D:
// lanes exchange with lane ^ D the elements whose index differs from theirs in bit D). DPP moves, no LDS.
template <int D>
__device__ __forceinline__ void xpose8_stage(float (&g)[8][4], uint32_t lane)
{
  const bool hi = (lane & D) != 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (!(k & D)) continue;
    const int a = k ^ D, b = k;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int send = __float_as_int(hi ? g[a][c] : g[b][c]);
      int recv;
      if constexpr (D == 1) {
        recv = __builtin_amdgcn_mov_dpp(send, 0xB1, 0xf, 0xf, false);  // quad_perm [1, 0, 3, 2]
      } else if constexpr (D == 2) {
        recv = __builtin_amdgcn_mov_dpp(send, 0x4E, 0xf, 0xf, false);  // quad_perm [2, 3, 0, 1]
      } else {
        const int up = __builtin_amdgcn_mov_dpp(send, 0x104, 0xf, 0xf, false);  // row_shl:4 (lane + 4)
        const int dn = __builtin_amdgcn_mov_dpp(send, 0x114, 0xf, 0xf, false);  // row_shr:4 (lane - 4)
        recv = hi ? dn : up;
      }
      if (hi) g[a][c] = __int_as_float(recv);
      else g[b][c] = __int_as_float(recv);
    }
  }
}

// One lane per 16-block index chunk, LANES chunks per workgroup, the workgroup's stream span staged in LDS (one round
// trip, stage_lds16). A lane decodes its chunk in two rounds of eight blocks; an 8 x 8 transpose across each group of
// 8 lanes (DPP) then gives lane 8q + m block m of the group's chunk 8q + i for i = 0..7, so every store instruction
// writes whole 128-byte lines (8 lanes x 16 bytes of one chunk). Stored as decoded -- each lane's 16 bytes 256 bytes
// apart, 64 lines per instruction -- the stores alone cost as much as the decode: 1 GiB in 0.37 ms against 0.19 ms
// for full-line instructions (tools/ubench/store_pattern.hip, modes 1 / 4).
// The stage is sized for 64 bits per block on average (accuracy 1e-6 on gradient-scale data codes ~63), which sets the
// occupancy (LDS-bound: 4.5 waves per SIMD at 64 bits, 3.5 at 80 -- C5 bucket 0.469 against 0.535 ms,
// profiles/r04_var_decode_occupancy_ab.log). A workgroup whose span does not fit (a higher rate), partial chunks and
// strided outputs take the general path (global-memory windows; staging such a workgroup in 2 or 4 parts instead
// measured slower on the common path, profiles/r04_var_decode_parts_negative.log).
#ifndef GCOW_VDEC_CAPB
#define GCOW_VDEC_CAPB 64
#endif
#ifndef GCOW_VDEC_ADAPT
#define GCOW_VDEC_ADAPT 1  // launch_decode1d_var sizes the main kernel's stage by the stream buffer's average bits
#endif
#ifndef GCOW_VDEC_LPAIR
#define GCOW_VDEC_LPAIR 0  // k_decode1d_var_lean's group phase through the pair table (7.4 KB more LDS per workgroup)
#endif
#ifndef GCOW_VDEC_BIGB
#define GCOW_VDEC_BIGB 144
#endif
#ifndef GCOW_VDEC_SWZ
#define GCOW_VDEC_SWZ 0  // the staged spans XOR-swizzled by bank row (lds_qword_swz), windows by qword reads
#endif
// Stage capacity in stream words: the main kernel's (GCOW_VDEC_CAPB bits per block on average) and the second pass's
// (any span: a 1-D block codes at most 140 bits, plus the 16-byte alignment of the span's start)
template <uint32_t LANES, uint32_t CAPB = GCOW_VDEC_CAPB> constexpr uint32_t vdec_cap() { return LANES * 16 * CAPB / 64; }
template <uint32_t LANES> constexpr uint32_t vdec_cap_big() { return LANES * 16 * GCOW_VDEC_BIGB / 64; }

// A group of LANES index chunks (one workgroup's work) whose span does not fit the main kernel's stage, and which is
// whole (no partial chunk or block) with a contiguous output: left by the main kernel to k_decode1d_var_lean_big.
// Not the last group: its span ends at the stream's end, which the index does not give (the buffer's end bounds it),
// so it takes the main kernel's general path.
template <uint32_t LANES>
__device__ __forceinline__ bool vdec_left_to_big_w(const FieldDesc& F, const uint64_t* index, uint64_t in_words,
                                                   uint64_t nchunks, uint64_t base_bits, uint64_t c0, uint64_t capw)
{
  const bool whole = c0 + LANES < nchunks && 16 * (c0 + LANES) <= (uint64_t)F.n[0] / 4;
  if (!whole || !F.vec) return false;
  const uint64_t w0 = ((base_bits + index[c0]) >> 6) & ~1ull;
  const uint64_t wend = (base_bits + index[c0 + LANES] + 63) >> 6;
  return min<uint64_t>(wend, in_words) - w0 > capw;
}

template <uint32_t LANES, uint32_t CAPB>
__device__ __forceinline__ bool vdec_left_to_big(const FieldDesc& F, const uint64_t* index, uint64_t in_words,
                                                 uint64_t nchunks, uint64_t base_bits, uint64_t c0)
{
  return vdec_left_to_big_w<LANES>(F, index, in_words, nchunks, base_bits, c0, vdec_cap<LANES, CAPB>());
}

// The stage tier of a stream from its block index (1: the 32-bit-per-block stage, 3: the 64-bit one): 1 when the
// 32-bit stage holds 1.25 x the stream's average bits per block over chunks 0 .. nchunks - 2 -- the rule the launcher
// applies to an exact-length buffer, taken here on the device for a buffer whose size says nothing (a capacity-sized
// Encoder.words). The two tiers are launched gated; the workgroups of the one that does not match return after two
// index loads (~13 us for the whole empty launch; a 48-bit tier measured as a second empty launch and was dropped).
__device__ __forceinline__ uint32_t vdec_tier(const uint64_t* index, uint64_t nchunks)
{
  if (nchunks < 2) return 1;
  const uint64_t span = index[nchunks - 1] - index[0], nbk = (nchunks - 1) * 16;
  return span * 5 <= nbk * 32 * 4 ? 1u : 3u;
}

// One group: its span staged in sw (CAP words), each lane's 16 blocks decoded by the lean block decoder, stored
// through the 8 x 8 lane transposes. BIG: the second pass (stage the caller's sw only after a barrier: the previous
// group's readers are done); else the main kernel, which stages dt7 with the span in one round trip.
template <uint32_t LANES, uint32_t CAP, bool BIG, bool LP = false>
__device__ __forceinline__ void vdec_group(const FieldDesc& F, const Params& p, const uint64_t* __restrict__ in,
                                           uint64_t in_words, const uint64_t* __restrict__ index, uint64_t nchunks,
                                           uint64_t base_bits, uint64_t* __restrict__ end_out, uint64_t c0,
                                           uint16_t* dtab, uint64_t* sw)
{
  uint16_t* dt7 = LP ? dtab + 3 * 1024 : dtab;  // LP: dtab holds the DecTabLP image
  const uint32_t tid = threadIdx.x;
  const uint64_t w0 = ((base_bits + index[c0]) >> 6) & ~1ull;  // 16-byte aligned start
  const uint64_t wend = c0 + LANES < nchunks ? ((base_bits + index[c0 + LANES] + 63) >> 6) : in_words;
  const uint64_t span = min<uint64_t>(wend, in_words) - w0;
  const bool staged = span <= CAP;
  const uint64_t c = c0 + tid;
  const uint64_t mine = c < nchunks ? index[c] : 0ull;
  if constexpr (BIG) __syncthreads();
  else if constexpr (LP) stage_lds16<LANES, sizeof(DecTabLP) / 16>(dtab, &g_dec_lean_pair, sizeof(DecTabLP));
  else stage_lds16<LANES, sizeof(DecTab7) / 16>(dt7, &g_dec_tab7, sizeof(DecTab7));
  constexpr bool SWZ = GCOW_VDEC_SWZ;
  if (staged) stage_lds16<LANES, (CAP + 4) / 2, SWZ>(sw, in + w0, (uint32_t)(8 * span));
  __syncthreads();
  float* out = (float*)F.data;
  const bool whole = c0 + LANES <= nchunks && 16 * (c0 + LANES) <= (uint64_t)F.n[0] / 4;  // no partial chunk or block
  if (!staged || !whole || !F.vec) {  // the general path (wave-uniform: the whole workgroup)
    if (c >= nchunks) return;
    const uint64_t b0 = c * 16, b1 = min<uint64_t>(b0 + 16, F.nblocks);
    uint64_t pos = base_bits + mine;
    if (staged) {
      pos -= 64 * w0;
      for (uint64_t b = b0; b < b1; b++) {
        float f[4];
        if constexpr (SWZ) decode_block1d_var(LdsWindowSwz{sw}, pos, dt7, p.minexp, p.maxprec, f);
        else decode_block1d_var(LdsWindow{sw}, pos, dt7, p.minexp, p.maxprec, f);
        store_block1d(F, b, f);
      }
      pos += 64 * w0;
    } else {
      for (uint64_t b = b0; b < b1; b++) {
        float f[4];
        decode_block1d_var(GlobalWindow{in}, pos, dt7, p.minexp, p.maxprec, f);
        store_block1d(F, b, f);
      }
    }
    if (end_out && c == nchunks - 1) *end_out = pos;
    return;
  }
  const uint32_t* sw32 = (const uint32_t*)sw;
  const int cexp = 4 - p.minexp, maxprec = (int)min(p.maxprec, 64u);
  uint32_t pos = (uint32_t)(base_bits + mine - 64 * w0);
  const uint32_t lane = tid & 63u, m = lane & 7u;
  float4* o4 = (float4*)out + (c - m) * 16 + m;  // block m of the group's first chunk
  uint2* o2 = (uint2*)F.data + (c - m) * 16 + m;  // bf16 output: 8 bytes per block
  const bool bf = F.dtype == DT_BF16;
#pragma unroll 1  // two copies of the 8-block body are past the unroller's size limit (nothing here needs them)
  for (int rnd = 0; rnd < 2; rnd++) {
    float g[8][4];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t start = pos;
      if (!dec_block1d_lean<LP, SWZ>(sw32, pos, dtab, cexp, maxprec, g[k])) {
        uint64_t p64 = start;
        if constexpr (SWZ) decode_block1d_var(LdsWindowSwz{sw}, p64, dt7, p.minexp, p.maxprec, g[k]);
        else decode_block1d_var(LdsWindow{sw}, p64, dt7, p.minexp, p.maxprec, g[k]);
        pos = (uint32_t)p64;
      }
    }
    xpose8_stage<1>(g, lane);
    xpose8_stage<2>(g, lane);
    xpose8_stage<4>(g, lane);
    if (bf) {
#pragma unroll
      for (int i = 0; i < 8; i++)
        o2[16 * i + 8 * rnd] = make_uint2(bf16x2_rne(g[i][0], g[i][1]), bf16x2_rne(g[i][2], g[i][3]));
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) o4[16 * i + 8 * rnd] = make_float4(g[i][0], g[i][1], g[i][2], g[i][3]);
    }
  }
  if (end_out && c == nchunks - 1) *end_out = pos + 64 * w0;
}

template <uint32_t LANES, uint32_t CAPB>
__global__ __launch_bounds__(LANES) void k_decode1d_var_lean(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                             uint64_t in_words, const uint64_t* __restrict__ index,
                                                             uint64_t nchunks, uint64_t base_bits,
                                                             uint64_t* __restrict__ end_out, uint64_t* __restrict__ left,
                                                             uint64_t seq, uint32_t tier)
{
  constexpr bool LP = GCOW_VDEC_LPAIR;
  __shared__ __attribute__((aligned(16))) uint16_t dtab[LP ? 3 * 1024 + 5 * 128 : 5 * 128];
  __shared__ __attribute__((aligned(16))) uint64_t sw[vdec_cap<LANES, CAPB>() + 4];
  if (tier && vdec_tier(index, nchunks) != tier) return;  // gated: another tier's launch decodes this stream
  const uint64_t c0 = (uint64_t)blockIdx.x * LANES;
  if (vdec_left_to_big<LANES, CAPB>(F, index, in_words, nchunks, base_bits, c0)) {  // workgroup-uniform
    if (left && threadIdx.x == 0) atomicMax((unsigned long long*)left, (unsigned long long)seq);  // second pass has work
    return;
  }
  vdec_group<LANES, vdec_cap<LANES, CAPB>(), false, LP>(F, p, in, in_words, index, nchunks, base_bits, end_out, c0, dtab, sw);
}

template <uint32_t LANES>
__device__ __forceinline__ void vdec_group_big(const FieldDesc& F, const Params& p, const uint64_t* __restrict__ in,
                                            uint64_t in_words, const uint64_t* __restrict__ index, uint64_t nchunks,
                                            uint64_t base_bits, uint64_t* __restrict__ end_out, uint64_t c0,
                                            uint16_t* dt7, uint64_t* sw)
{
  vdec_group<LANES, vdec_cap_big<LANES>(), true>(F, p, in, in_words, index, nchunks, base_bits, end_out, c0, dt7, sw);
}

template <uint32_t LANES, uint32_t CAPB>
__global__ __launch_bounds__(LANES) void k_decode1d_var_lean_big(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                                 uint64_t in_words, const uint64_t* __restrict__ index,
                                                                 uint64_t nchunks, uint64_t base_bits,
                                                                 uint64_t* __restrict__ end_out,
                                                                 const uint64_t* __restrict__ left, uint64_t seq,
                                                                 bool tiered)
{
  __shared__ __attribute__((aligned(16))) uint16_t dt7[5 * 128];
  __shared__ __attribute__((aligned(16))) uint64_t sw[vdec_cap_big<LANES>() + 4];
  __shared__ uint32_t todo[LANES];
  __shared__ uint32_t ntodo;
  if (left && *left < seq) return;  // the main kernel left nothing (no flag word: check every group)
  // the stage of the main launch that decoded this stream: CAPB, or (tiered) the tier vdec_tier picks
  uint64_t capw = vdec_cap<LANES, CAPB>();
  if (tiered) {
    const uint32_t t = vdec_tier(index, nchunks);
    capw = t == 1 ? vdec_cap<LANES, 32>() : vdec_cap<LANES, 64>();
  }
  const uint64_t ng = (nchunks + LANES - 1) / LANES;
  bool staged_tab = false;
  // sweep k: workgroup w checks groups k G LANES + t G + w (t < LANES, G = gridDim.x): the groups spread over every
  // workgroup of the grid
  const uint64_t G = gridDim.x;
  for (uint64_t gb = 0; gb < ng; gb += G * LANES) {
    if (threadIdx.x == 0) ntodo = 0;
    __syncthreads();
    const uint64_t g = gb + (uint64_t)threadIdx.x * G + blockIdx.x;
    if (g < ng && vdec_left_to_big_w<LANES>(F, index, in_words, nchunks, base_bits, g * LANES, capw))
      todo[atomicAdd(&ntodo, 1u)] = threadIdx.x;
    __syncthreads();
    const uint32_t nt = ntodo;
    if (nt && !staged_tab) {  // the decode table only once there is work
      stage_lds16<LANES, sizeof(DecTab7) / 16>(dt7, &g_dec_tab7, sizeof(DecTab7));
      staged_tab = true;
    }
    for (uint32_t i = 0; i < nt; i++)
      vdec_group_big<LANES>(F, p, in, in_words, index, nchunks, base_bits, end_out,
                            (gb + (uint64_t)todo[i] * G + blockIdx.x) * LANES, dt7, sw);
    __syncthreads();  // todo / ntodo are rewritten next sweep
  }
}

// the partial last block of a 1-D field (generic decoder, one lane)
__global__ void k_decode_tail1d(FieldDesc F, Params p, const uint64_t* __restrict__ in, uint64_t base_bits,
                                uint32_t b)
{
  BitReader r{in, base_bits + (uint64_t)b * p.maxbits};
  float f[4];
  decode_block<1>(r, p, f);
  store_block1d(F, b, f);
}

// Many-workgroup form of k_scan_ranges for up to kScanMwMax ranges: workgroup g scans ranges [1024 g, 1024 g + 1024)
// and finds its starting offset by summing every earlier range total itself (O(n^2 / 2048) loads in all, from L2:
// 0.5 M loads at 32 Ki ranges), so no second launch, no partials buffer and no inter-workgroup protocol.
constexpr uint32_t kScanMwMax = 1u << 16;

// gsums (optional): totals of consecutive groups of 8 ranges (the 1-D tile count writes them), so the earlier totals
// each workgroup sums are 1/8 as many.
__global__ __launch_bounds__(256) void k_scan_ranges_mw(const uint64_t* __restrict__ sums, uint32_t nranges,
                                                        uint64_t* __restrict__ base, uint64_t* __restrict__ total,
                                                        uint32_t* __restrict__ out32,
                                                        const uint64_t* __restrict__ d_base,
                                                        const uint64_t* __restrict__ gsums)
{
  constexpr uint32_t T = 256, K = 4, C = T * K;
  __shared__ uint64_t v[C];
  __shared__ uint64_t wsum[T / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t c0 = blockIdx.x * C;
  const uint32_t n = min(C, nranges - c0);
#pragma unroll
  for (uint32_t k = 0; k < K; k++) {
    const uint32_t j = t + T * k;
    v[j] = j < n ? sums[c0 + j] : 0ull;
  }
  uint64_t pre = 0;  // every earlier range total (or group total), 8 loads in flight per thread
  const uint64_t* ps = gsums ? gsums : sums;
  const uint32_t pn = gsums ? c0 / 8u : c0;
  uint32_t i = t;
  for (; i + 7 * T < pn; i += 8 * T) {
    uint64_t a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = ps[i + k * T];
#pragma unroll
    for (int k = 0; k < 8; k++) pre += a[k];
  }
  for (; i < pn; i += T) pre += ps[i];
  __syncthreads();
  uint64_t loc[K], s = 0;
#pragma unroll
  for (uint32_t k = 0; k < K; k++) {
    loc[k] = v[t * K + k];
    s += loc[k];
  }
  const uint64_t incl = wave_incl_scan64(s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)pre, o), hi = __shfl_xor((uint32_t)(pre >> 32), o);
    pre += (uint64_t)lo | ((uint64_t)hi << 32);
  }
  __shared__ uint64_t wpre[T / 64];
  if (lane == 63) wsum[wv] = incl;
  if (lane == 0) wpre[wv] = pre;
  __syncthreads();
  uint64_t before = 0, chunk = 0, carry = d_base ? *d_base : 0ull;
#pragma unroll
  for (uint32_t w = 0; w < T / 64; w++) {
    before += w < wv ? wsum[w] : 0ull;
    chunk += wsum[w];
    carry += wpre[w];
  }
  uint64_t run = carry + before + incl - s;
#pragma unroll
  for (uint32_t k = 0; k < K; k++) {
    v[t * K + k] = run;
    run += loc[k];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < K; k++) {
    const uint32_t j = t + T * k;
    if (j < n) {
      const uint64_t b = v[j];
      base[c0 + j] = b;
      if (c0 + j > 0 && (b & 31)) out32[b >> 5] = 0u;
    }
  }
  if (blockIdx.x == gridDim.x - 1 && t == 0) {
    base[nranges] = carry + chunk;
    if (total) *total = carry + chunk;
  }
}

static void scan_ranges(const uint64_t* sums, uint32_t nranges, uint64_t* base, uint64_t* total, uint32_t* out32,
                        const uint64_t* d_base, hipStream_t st, const uint64_t* gsums = nullptr)
{
  if (nranges > 4096 && (nranges <= kScanMwMax || gsums))
    k_scan_ranges_mw<<<(nranges + 1023) / 1024, 256, 0, st>>>(sums, nranges, base, total, out32, d_base, gsums);
  else
    k_scan_ranges<<<1, 1024, 0, st>>>(sums, nranges, base, total, out32, d_base);
}

__global__ void k_set_u64(uint64_t* p, uint64_t v) { *p = v; }

// zfp_decompress's cache check: flag = 1 where the caller's device stream differs from the cached copy (plain
// vector stores of the same value; the flag was zeroed by a preceding launch on the stream)
__global__ void k_words_differ(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint64_t n,
                               uint64_t* __restrict__ flag)
{
  bool d = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    d = d || a[i] != b[i];
  if (d) *flag = 1ull;
}

// ------------------------------------------------------------------------------------------------ header stream
// dst = header bits [0, off) followed by src bits [0, *d_bits), flushed to whole words (zfp_write_header then
// zfp_compress at the following bit). Plain stores, one lane per destination word; lanes past the end exit. Lane 0
// also publishes the total bit count.
__global__ void k_prepend_header(uint64_t* __restrict__ dst, uint32_t off, const uint64_t* __restrict__ src,
                                 const uint64_t* __restrict__ d_bits, uint64_t h0, uint64_t h1, uint64_t h2,
                                 uint64_t* __restrict__ d_total)
{
  const uint64_t bits = *d_bits, end = off + bits;
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w == 0 && d_total) *d_total = end;
  if ((w << 6) >= end) return;
  const uint64_t nsw = (bits + 63) >> 6;
  uint64_t v = 0;
  if (w < 3 && (w << 6) < off) {  // header part of this word
    const uint64_t h = w == 0 ? h0 : (w == 1 ? h1 : h2);
    const uint64_t hb = off - (w << 6);
    v = hb >= 64 ? h : (h & ((1ull << hb) - 1ull));
  }
  const int64_t s = (int64_t)(w << 6) - (int64_t)off;  // source bit landing on bit 0 of dst[w]
  if (s + 64 > 0 && nsw) {
    if (s < 0) {
      v |= src[0] << (uint32_t)(-s);
    } else {
      const uint64_t i = (uint64_t)s >> 6;
      const uint32_t sh = (uint32_t)(s & 63);
      uint64_t x = i < nsw ? src[i] >> sh : 0ull;
      if (sh && i + 1 < nsw) x |= src[i + 1] << (64 - sh);
      v |= x;
    }
  }
  const uint64_t lo = w << 6;
  if (end < lo + 64) v &= (1ull << (end - lo)) - 1ull;  // end > lo here
  dst[w] = v;
}

// ------------------------------------------------------------------------------------------------ stitch
__global__ void k_stitch(uint64_t* __restrict__ dst, uint64_t off, const uint64_t* __restrict__ src, uint64_t bits)
{
  // dst bit range [off, off + bits) |= src bits [0, bits); one lane per destination word.
  const uint64_t w0 = off >> 6, w1 = (off + bits + 63) >> 6;
  const uint64_t w = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= w1) return;
  const uint64_t nsw = (bits + 63) >> 6;
  const int64_t s = (int64_t)(w << 6) - (int64_t)off;  // source bit that lands on bit 0 of dst[w]
  uint64_t v;
  if (s < 0) {
    v = src[0] << (uint32_t)(-s);
  } else {
    const uint64_t i = (uint64_t)s >> 6;
    const uint32_t sh = (uint32_t)(s & 63);
    v = src[i] >> sh;
    if (sh && i + 1 < nsw) v |= src[i + 1] << (64 - sh);
  }
  const uint64_t lo = w << 6;
  if (off + bits < lo + 64) v &= (1ull << (off + bits - lo)) - 1ull;  // off + bits > lo here
  dst[w] |= v;
}

// All shard streams in one launch (the receive side of a variable-rate all-gather): shard r
// holds lens[r] bits at src + r * shard_words and lands at bit O_r = lens[0] + ... + lens[r - 1] (a per-lane running
// sum over the shards: nshards is the world size). One lane per destination word, which it writes whole -- the OR of
// every shard's bits that fall on it, zero past the stream's end -- so dst needs no zeroing and no atomics.
__global__ __launch_bounds__(256) void k_stitch_shards(uint64_t* __restrict__ dst, uint64_t dst_words,
                                                       const uint64_t* __restrict__ src, uint64_t shard_words,
                                                       const uint64_t* __restrict__ lens, uint32_t nshards)
{
  const uint64_t w = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (w >= dst_words) return;
  const uint64_t lo = w << 6;
  uint64_t v = 0, off = 0;
  for (uint32_t r = 0; r < nshards; r++) {
    const uint64_t bits = lens[r];
    const uint64_t end = off + bits;
    if (bits && off < lo + 64 && end > lo) {
      const uint64_t* sr = src + (uint64_t)r * shard_words;
      const uint64_t nsw = (bits + 63) >> 6;
      const int64_t sb = (int64_t)lo - (int64_t)off;  // shard bit landing on bit 0 of dst[w]
      uint64_t x;
      if (sb < 0) {
        x = sr[0] << (uint32_t)(-sb);  // -sb < 64: the shard starts inside this word
      } else {
        const uint64_t i = (uint64_t)sb >> 6;  // < nsw: sb < bits
        const uint32_t sh = (uint32_t)(sb & 63);
        x = sr[i] >> sh;
        if (sh && i + 1 < nsw) x |= sr[i + 1] << (64 - sh);
      }
      if (end < lo + 64) x &= (1ull << (end - lo)) - 1ull;  // drop the shard's own flush padding
      v |= x;
    }
    off = end;
  }
  dst[w] = v;
}

// ------------------------------------------------------------------------------------------------ decode + mean
// acc / nstreams for the N sums of a lane: an IEEE division, or -- nstreams a power of two (the usual world size) --
// the product by the exact reciprocal, which is the same correctly rounded value of the same quotient (a uniform
// branch: the division's expansion runs only for other world sizes).
template <int N>
__device__ __forceinline__ void mean_scale(float* a, uint32_t nstreams)
{
#pragma clang fp contract(off)
  if ((nstreams & (nstreams - 1u)) == 0u) {
    const float inv = 1.0f / (float)nstreams;
#pragma unroll
    for (int i = 0; i < N; i++) a[i] = a[i] * inv;
  } else {
    const float nf = (float)nstreams;
#pragma unroll
    for (int i = 0; i < N; i++) a[i] = a[i] / nf;
  }
}

// The receive side of the compressed all-gather hook: nstreams 1-D streams of the same shape
// (one per rank, stream_words apart) are decoded and averaged in one launch instead of one decode and one add per
// rank. Each lane accumulates in fp32 in rank order, acc = ((0 + x_0) + x_1) + ..., then stores acc / nstreams: the
// values a sequence of decode -> add kernels would give (no contraction of the dequantising multiply into the add).

// Fixed rate. WB = 64 / 32: the one-shot table decoder (whole-word blocks, kmin = 0); WB = 0: the generic decoder
// (any fixed rate). One block per lane.
template <uint32_t WB>
__global__ __launch_bounds__(256) void k_decode_mean_fixed1d(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                             uint64_t stream_words, uint32_t nstreams, uint64_t bfirst)
{
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) uint16_t dtab[WB ? 5 * 8 * 128 : 8];
  if (WB) {
    stage_lds16<256, sizeof(DecTab1) / 16>(dtab, &g_dec_tab1, sizeof(DecTab1));
    __syncthreads();
  }
  const uint64_t b = bfirst + (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (b >= F.nblocks) return;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (uint32_t r = 0; r < nstreams; r++) {
    const uint64_t* sr = in + (uint64_t)r * stream_words;
    float f[4];
    bool special = true;
    if constexpr (WB == 64) decode_block1d_fast<64>(sr[b], dtab, f, special);
    else if constexpr (WB == 32) decode_block1d_fast<32>(((const uint32_t*)sr)[b], dtab, f, special);
    if (special) {
      BitReader rd{sr, b * p.maxbits};
      decode_block<1>(rd, p, f);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] = acc[i] + f[i];
  }
  mean_scale<4>(acc, nstreams);
  store_block1d(F, b, acc);
}

// The fixed-rate mean in the shape of k_decode_fixed1d_np (whole-word blocks, kmin = 0): one-shot, U blocks per lane
// 256 apart, the plane table requested first (raw loads, hand-counted wait); stream s + 1's U words are requested
// before stream s's blocks are decoded. The stream words are compiler-visible buffer loads: they are carried across
// the stream loop, and a value loaded by inline asm must not be carried (the loop's register copies would read the
// destination before the load has written it). Full blocks only (the launcher sends a partial last block to
// k_decode_mean_fixed1d).
template <uint32_t WB> struct MeanWord;
template <> struct MeanWord<64> {
  typedef uint64_t T;
  static __device__ __forceinline__ T load(__amdgpu_buffer_rsrc_t rs, uint32_t b)
  {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(b * 8u), 0, 0);
    return (uint64_t)v[0] | ((uint64_t)v[1] << 32);
  }
};
template <> struct MeanWord<32> {
  typedef uint32_t T;
  static __device__ __forceinline__ T load(__amdgpu_buffer_rsrc_t rs, uint32_t b)
  {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(b * 4u), 0, 0);
  }
};

template <uint32_t WB, int U, int D>
__global__ __launch_bounds__(256) void k_decode_mean_fixed1d_np(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                                uint64_t stream_words, uint32_t nstreams,
                                                                uint32_t nfull)
{
#pragma clang fp contract(off)
  constexpr bool PAIR = WB == 64 && GCOW_DEC_PAIR;  // 64-bit blocks: the two-plane table
  using PTab = typename std::conditional<GCOW_DEC_GATHER, DecTabPG, DecTabP>::type;
  using Tab = typename std::conditional<PAIR, PTab, DecTab1>::type;
  __shared__ __attribute__((aligned(16))) uint32_t dtab32[sizeof(Tab) / 4];
  const uint16_t* dtab = (const uint16_t*)dtab32;
  constexpr uint32_t WBYTES = WB / 8;
  const uint32_t b0 = blockIdx.x * (256u * U) + threadIdx.x;
  constexpr uint32_t TCH = sizeof(Tab) / 16, TR = (TCH + 255) / 256;
  const pipe_v4i rt = PAIR ? buf_rsrc(dec_pair_image(), sizeof(PTab)) : buf_rsrc(&g_dec_tab1, sizeof(DecTab1));
  pipe_v4u tv[TR];
#pragma unroll
  for (uint32_t i = 0; i < TR; i++) tv[i] = buf_load_b128((threadIdx.x + 256u * i) * 16u, rt);
  auto rsrc = [&](uint32_t r) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(in + (uint64_t)r * stream_words), 0, (int)(nfull * WBYTES),
                                             0x00020000);
  };
  typename MeanWord<WB>::T cur[U], nx1[U];
  {
    const auto rs = rsrc(0);
#pragma unroll
    for (int k = 0; k < U; k++) cur[k] = MeanWord<WB>::load(rs, b0 + 256u * k);
    if (D == 2 && nstreams > 1) {
      const auto rs1 = rsrc(1);
#pragma unroll
      for (int k = 0; k < U; k++) nx1[k] = MeanWord<WB>::load(rs1, b0 + 256u * k);
    }
  }
  // the table loads are the oldest: once at most D U loads are outstanding they have landed
  table_wait<D * U>(tv);
#pragma unroll
  for (uint32_t i = 0; i < TR; i++)
    if (threadIdx.x + 256u * i < TCH) ((pipe_v4u*)dtab32)[threadIdx.x + 256u * i] = tv[i];
  __syncthreads();
  float acc[U][4];
#pragma unroll
  for (int k = 0; k < U; k++) acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0.0f;
  for (uint32_t r = 0; r < nstreams; r++) {
    typename MeanWord<WB>::T nxt[U];  // stream r + D's words
    if (r + D < nstreams) {
      const auto rs = rsrc(r + D);
#pragma unroll
      for (int k = 0; k < U; k++) nxt[k] = MeanWord<WB>::load(rs, b0 + 256u * k);
    }
    const uint64_t* sr = in + (uint64_t)r * stream_words;
#pragma unroll
    for (int k = 0; k < U; k++) {
      const uint32_t b = b0 + 256u * k;
      float f[4];
      bool special;
      if constexpr (PAIR) decode_block1d_pair<GCOW_DEC_GATHER>((uint64_t)cur[k], dtab32, f, special);
      else decode_block1d_fast<WB>((uint64_t)cur[k], dtab, f, special);
      if (special && b < nfull) {
        BitReader rd{sr, (uint64_t)b * WB};
        decode_block<1>(rd, p, f);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) acc[k][i] = acc[k][i] + f[i];
    }
#pragma unroll
    for (int k = 0; k < U; k++) {
      if (D == 2) {
        cur[k] = nx1[k];
        nx1[k] = nxt[k];
      } else {
        cur[k] = nxt[k];
      }
    }
  }
  mean_scale<U * 4>(&acc[0][0], nstreams);
  float* out = (float*)F.data;
#pragma unroll
  for (int k = 0; k < U; k++) {
    const uint32_t b = b0 + 256u * k;
    if (b < nfull) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = acc[k][i];
      if (F.vec && F.dtype != DT_BF16) *(float4*)(out + 4 * (uint64_t)b) = make_float4(v[0], v[1], v[2], v[3]);
      else store_block1d(F, b, v);
    }
  }
}

#ifndef GCOW_DMV_WAVES
#define GCOW_DMV_WAVES 3  // 16-block chunks: 64 sums per lane, no spills at 3 waves (4 waves: 33 spilled VGPRs)
#endif
#ifndef GCOW_DMV8_WAVES
#define GCOW_DMV8_WAVES 5  // 8-block chunks: 32 sums per lane, 96 VGPRs (2 spilled) at 5 waves: 3.43 -> 3.05 ms (W = 8)
#endif
#ifndef GCOW_DMV8_SCALE
#define GCOW_DMV8_SCALE 1  // 8-block chunks: the mean through mean_scale (a power-of-two world: the exact reciprocal)
#endif
#ifndef GCOW_DMV16_LPAIR
#define GCOW_DMV16_LPAIR 1  // 16-block chunks too, at 3 waves (LDS): 3.67 -> 3.59 ms (profiles/r05_dmean16_lp_w3_ab.log)
#endif
#ifndef GCOW_DMV_SWZ
#define GCOW_DMV_SWZ 0  // decode_mean's staged spans XOR-swizzled by bank row (lds_qword_swz), windows by qword reads
#endif
#ifndef GCOW_DMV_LPAIR
#define GCOW_DMV_LPAIR 1  // the lean block decoder's group phase through the 16-bit pair table (DecTabLP)
#endif
// Block-index readers of the variable-rate decode_mean kernels: plain (one uint64 bit position per index chunk), or
// packed16 (GCOW_INDEX_PACKED16: one uint64 per 16 blocks -- low 48 bits the position of block 16 c, high 16 bits the
// offset of block 16 c + 8 from it -- read as the positions of 8-block chunks).
template <bool PK> struct IndexRd {
  const uint64_t* ix;
  __device__ __forceinline__ uint64_t operator[](uint64_t c) const { return ix[c]; }
};
template <> struct IndexRd<true> {
  const uint64_t* ix;
  __device__ __forceinline__ uint64_t operator[](uint64_t c) const
  {
    const uint64_t v = ix[c >> 1];
    return (v & 0xffffffffffffull) + ((c & 1) ? (v >> 48) : 0ull);
  }
};

// Variable rate (1-D closed-form domain), the lean decoder's shape (k_decode1d_var_lean): LANES 16-block chunks per
// workgroup; for each stream in rank order its span is staged in LDS (in 1, 2 or 4 parts, as there) and each lane
// decodes its chunk into 64 registers of sums; the means leave through the 8 x 8 lane transposes as whole-line
// stores. Complete workgroups only (whole chunks, full blocks, contiguous output); the launcher sends the rest to
// k_decode_mean1d_var.
template <uint32_t LANES, uint32_t CAPB, uint32_t CH, bool PK = false>
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(CH == 8 ? GCOW_DMV8_WAVES : GCOW_DMV_WAVES, 8))) void k_decode_mean1d_var_lean(FieldDesc F, Params p,
                                                                  const uint64_t* __restrict__ in,
                                                                  uint64_t stream_words,
                                                                  const uint64_t* __restrict__ index,
                                                                  uint64_t index_words, uint64_t nchunks,
                                                                  uint32_t nstreams)
{
#pragma clang fp contract(off)
  constexpr uint32_t CAP = LANES * CH * CAPB / 64;
  static_assert(LANES % 32 == 0 && CAP >= 32 * CH * 140 / 64 + 4 && CH % 8 == 0, "a quarter workgroup's longest span must fit");
  constexpr bool LP = GCOW_DMV_LPAIR && (CH == 8 || GCOW_DMV16_LPAIR);
  __shared__ __attribute__((aligned(16))) uint16_t dtab[LP ? 3 * 1024 + 5 * 128 : 5 * 128];
  const uint16_t* dt7 = LP ? dtab + 3 * 1024 : dtab;
  __shared__ __attribute__((aligned(16))) uint64_t sw[CAP + 4];
  const uint32_t tid = threadIdx.x;
  const uint64_t c0 = (uint64_t)blockIdx.x * LANES;
  const uint64_t c = c0 + tid;
  const uint32_t* sw32 = (const uint32_t*)sw;
  const int cexp = 4 - p.minexp, maxprec = (int)min(p.maxprec, 64u);
  if constexpr (LP) stage_lds16<LANES, sizeof(DecTabLP) / 16>(dtab, &g_dec_lean_pair, sizeof(DecTabLP));
  else stage_lds16<LANES, sizeof(DecTab7) / 16>(dtab, &g_dec_tab7, sizeof(DecTab7));
  float acc[CH][4];
#pragma unroll
  for (int k = 0; k < (int)CH; k++) acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0.0f;
  for (uint32_t r = 0; r < nstreams; r++) {
    const uint64_t* sr = in + (uint64_t)r * stream_words;
    const IndexRd<PK> ix{index + (uint64_t)r * index_words};
    const uint64_t sbase = (uint64_t)r * stream_words;
    // a span starts on a 16-byte boundary of the whole buffer (streams are stream_words apart, which may be odd):
    // w0 may be one word before this stream's first word (the previous stream's last word, never decoded)
    auto w_first = [&](uint64_t a) { return (int64_t)((sbase + (ix[a] >> 6)) & ~1ull) - (int64_t)sbase; };
    auto w_end = [&](uint64_t b) { return (int64_t)min<uint64_t>(b < nchunks ? (ix[b] + 63) >> 6 : stream_words, stream_words); };
    const uint64_t mine = ix[c];
    uint32_t P = 4;
    if (w_end(c0 + LANES) - w_first(c0) <= (int64_t)CAP) P = 1;
    else if (w_end(c0 + LANES / 2) - w_first(c0) <= (int64_t)CAP && w_end(c0 + LANES) - w_first(c0 + LANES / 2) <= (int64_t)CAP)
      P = 2;
    const uint32_t per = LANES / P;
    for (uint32_t part = 0; part < P; part++) {
      const uint64_t a = c0 + part * per;
      const int64_t w0 = w_first(a);
      const uint64_t span = (uint64_t)(w_end(a + per) - w0);
      __syncthreads();  // the previous span is no longer read
      stage_lds16<LANES, (CAP + 4) / 2, GCOW_DMV_SWZ>(sw, sr + w0, (uint32_t)(8 * span));
      __syncthreads();
      if (tid / per != part) continue;
      uint32_t pos = (uint32_t)((int64_t)mine - 64 * w0);
#pragma unroll
      for (int k = 0; k < (int)CH; k++) {
        const uint32_t start = pos;
        float f[4];
        if (!dec_block1d_lean<LP, GCOW_DMV_SWZ>(sw32, pos, dtab, cexp, maxprec, f)) {
          uint64_t p64 = start;
          if constexpr (GCOW_DMV_SWZ) decode_block1d_var(LdsWindowSwz{sw}, p64, dt7, p.minexp, p.maxprec, f);
          else decode_block1d_var(LdsWindow{sw}, p64, dt7, p.minexp, p.maxprec, f);
          pos = (uint32_t)p64;
        }
#pragma unroll
        for (int i = 0; i < 4; i++) acc[k][i] = acc[k][i] + f[i];
      }
    }
  }
  // CH = 16: a plain division (the two-path mean_scale costs that kernel registers, +4 %)
  if constexpr (CH == 8 && GCOW_DMV8_SCALE) mean_scale<CH * 4>(&acc[0][0], nstreams);
  const float nf = CH == 8 && GCOW_DMV8_SCALE ? 1.0f : (float)nstreams;
  const uint32_t lane = tid & 63u, m = lane & 7u;
  float4* o4 = (float4*)F.data + (c - m) * CH + m;
  uint2* o2 = (uint2*)F.data + (c - m) * CH + m;  // bf16 output: 8 bytes per block, a chunk is one 128-byte line
  const bool bf = F.dtype == DT_BF16;
#pragma unroll
  for (int rnd = 0; rnd < (int)CH / 8; rnd++) {
    float g[8][4];
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
      for (int i = 0; i < 4; i++) g[k][i] = acc[8 * rnd + k][i] / nf;
    xpose8_stage<1>(g, lane);
    xpose8_stage<2>(g, lane);
    xpose8_stage<4>(g, lane);
    if (bf) {
#pragma unroll
      for (int i = 0; i < 8; i++)
        o2[CH * i + 8 * rnd] = make_uint2(bf16x2_rne(g[i][0], g[i][1]), bf16x2_rne(g[i][2], g[i][3]));
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) o4[CH * i + 8 * rnd] = make_float4(g[i][0], g[i][1], g[i][2], g[i][3]);
    }
  }
}

// Variable rate (1-D closed-form domain) with each stream's block index every 16 blocks (index_words entries apart):
// the shape of k_decode1d_var_lean -- LANES chunks of 16 blocks per workgroup, the workgroup's span of each stream
// staged in LDS in turn -- with the 16 blocks' 64 values accumulated in registers across the streams and stored once.
template <uint32_t LANES, uint32_t CH, bool PK = false>
__global__ __launch_bounds__(LANES) void k_decode_mean1d_var(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                             uint64_t stream_words, const uint64_t* __restrict__ index,
                                                             uint64_t index_words, uint64_t nchunks, uint32_t nstreams,
                                                             uint64_t cfirst)
{
#pragma clang fp contract(off)
  constexpr uint32_t CAP = LANES * CH * 80 / 64;
  __shared__ __attribute__((aligned(16))) uint16_t dt7[5 * 128];
  __shared__ __attribute__((aligned(16))) uint64_t sw[CAP + 4];
  const uint32_t tid = threadIdx.x;
  stage_lds16<LANES, sizeof(DecTab7) / 16>(dt7, &g_dec_tab7, sizeof(DecTab7));
  const uint64_t c0 = cfirst + (uint64_t)blockIdx.x * LANES;
  const uint64_t c = c0 + tid;
  const uint64_t b0 = c * CH, b1 = min<uint64_t>(b0 + CH, F.nblocks);
  float acc[CH][4];
#pragma unroll
  for (int k = 0; k < (int)CH; k++) acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0.0f;
  for (uint32_t r = 0; r < nstreams; r++) {
    const uint64_t* sr = in + (uint64_t)r * stream_words;
    const IndexRd<PK> ix{index + (uint64_t)r * index_words};
    // the staged span starts on a 16-byte boundary of the whole buffer (streams are stream_words apart, which may be
    // odd): w0 may be one word before this stream's first word (the previous stream's last word, never decoded)
    const uint64_t sbase = (uint64_t)r * stream_words;
    const int64_t w0 = (int64_t)((sbase + (ix[c0] >> 6)) & ~1ull) - (int64_t)sbase;
    const uint64_t wend = c0 + LANES < nchunks ? ((ix[c0 + LANES] + 63) >> 6) : stream_words;
    const uint64_t span = (uint64_t)((int64_t)min<uint64_t>(wend, stream_words) - w0);
    const bool staged = span <= CAP;
    __syncthreads();  // the previous stream's span is no longer read
    if (staged) stage_lds16<LANES, (CAP + 4) / 2>(sw, sr + w0, (uint32_t)(8 * span));
    __syncthreads();
    if (c >= nchunks) continue;
    uint64_t pos = ix[c];
    auto run = [&](const auto& win) {
#pragma unroll
      for (int k = 0; k < (int)CH; k++) {
        if (b0 + k < b1) {
          float f[4];
          decode_block1d_var(win, pos, dt7, p.minexp, p.maxprec, f);
#pragma unroll
          for (int i = 0; i < 4; i++) acc[k][i] = acc[k][i] + f[i];
        }
      }
    };
    if (staged) {
      pos = (uint64_t)((int64_t)pos - 64 * w0);
      run(LdsWindow{sw});
    } else {
      run(GlobalWindow{sr});
    }
  }
  if (c >= nchunks) return;
  mean_scale<CH * 4>(&acc[0][0], nstreams);
  float* out = (float*)F.data;
#pragma unroll
  for (int k = 0; k < (int)CH; k++) {
    const uint64_t b = b0 + k;
    if (b < b1) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = acc[k][i];
      if (F.vec && F.dtype != DT_BF16 && 4 * b + 4 <= F.n[0]) *(float4*)(out + 4 * b) = make_float4(v[0], v[1], v[2], v[3]);
      else store_block1d(F, b, v);
    }
  }
}

// Variable rate outside the closed-form domain (expert parameters with minbits > 1 or maxbits < 160: a budget can
// truncate blocks): one lane per 16-block index chunk, the generic libzfp decoder (decode_block) on each stream in
// rank order, the same fp32 accumulation as above.
template <bool PK = false>
__global__ __launch_bounds__(256) void k_decode_mean1d_generic(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                               uint64_t stream_words, const uint64_t* __restrict__ index,
                                                               uint64_t index_words, uint64_t nchunks,
                                                               uint32_t nstreams, uint32_t chunk)
{
#pragma clang fp contract(off)
  const uint64_t c = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (c >= nchunks) return;
  const uint64_t b0 = c * chunk, b1 = min<uint64_t>(b0 + chunk, F.nblocks);  // chunk <= 16
  float acc[16][4];
#pragma unroll
  for (int k = 0; k < 16; k++) acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0.0f;
  for (uint32_t r = 0; r < nstreams; r++) {
    BitReader rd{in + (uint64_t)r * stream_words, IndexRd<PK>{index + (uint64_t)r * index_words}[c]};
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (b0 + k < b1) {
        float f[4];
        decode_block<1>(rd, p, f);
#pragma unroll
        for (int i = 0; i < 4; i++) acc[k][i] = acc[k][i] + f[i];
      }
    }
  }
  mean_scale<64>(&acc[0][0], nstreams);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    if (b0 + k < b1) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = acc[k][i];
      store_block1d(F, b0 + k, v);
    }
  }
}

// ------------------------------------------------------------------------------------------------ stages
template <int D>
__global__ void k_stage_emax(const float* __restrict__ blocks, uint32_t n, int32_t* __restrict__ emax)
{
  constexpr int B = Dim<D>::B;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float f[B];
#pragma unroll
  for (int j = 0; j < B; j++) f[j] = blocks[(uint64_t)i * B + j];
  emax[i] = block_emax<B>(f);
}

template <int D>
__global__ void k_stage_cast(const float* __restrict__ blocks, const int32_t* __restrict__ emax, uint32_t n,
                             int32_t* __restrict__ q)
{
  constexpr int B = Dim<D>::B;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = cast_scale(emax[i]);
  for (int j = 0; j < B; j++) q[(uint64_t)i * B + j] = cast1(blocks[(uint64_t)i * B + j], s);
}

template <int D>
__global__ void k_stage_xform(int32_t* __restrict__ q, uint32_t n, int inverse)
{
  constexpr int B = Dim<D>::B;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t a[B];
#pragma unroll
  for (int j = 0; j < B; j++) a[j] = q[(uint64_t)i * B + j];
  if (inverse) inv_xform<D>(a);
  else fwd_xform<D>(a);
#pragma unroll
  for (int j = 0; j < B; j++) q[(uint64_t)i * B + j] = a[j];
}

template <int D>
__global__ void k_stage_reorder(const int32_t* __restrict__ q, uint32_t n, uint32_t* __restrict__ u)
{
  constexpr int B = Dim<D>::B;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t a[B];
  uint32_t o[B];
#pragma unroll
  for (int j = 0; j < B; j++) a[j] = q[(uint64_t)i * B + j];
  fwd_reorder<D>(o, a);
#pragma unroll
  for (int j = 0; j < B; j++) u[(uint64_t)i * B + j] = o[j];
}

// Coder on one ublock per lane into its own zeroed slot (32-bit LDS-free variant: a private global window).
struct GlobalSlotWriter {
  uint32_t* w;
  uint32_t pos, limit;
  __device__ __forceinline__ void put(uint64_t v, uint32_t n)
  {
    if (pos >= limit || n == 0) { pos += n; return; }
    uint32_t room = limit - pos;
    if (n > room) v &= lowmask64(room);
    uint32_t i = pos >> 5, sh = pos & 31;
    w[i] |= (uint32_t)(v << sh);
    w[i + 1] |= (uint32_t)((v << sh) >> 32);
    if (sh) w[i + 2] |= (uint32_t)(v >> (64 - sh));
    pos += n;
  }
  __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
};

template <int D>
__global__ void k_stage_encode_ints(const uint32_t* __restrict__ ublocks, uint32_t n, uint32_t budget,
                                    uint32_t maxprec, uint64_t* __restrict__ slots, uint32_t slot_words,
                                    uint32_t* __restrict__ bits)
{
  constexpr int B = Dim<D>::B;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t u[B];
#pragma unroll
  for (int j = 0; j < B; j++) u[j] = ublocks[(uint64_t)i * B + j];
  uint32_t lim = slot_words * 64 - 64;  // keep the spill word inside the slot
  GlobalSlotWriter w{(uint32_t*)(slots + (uint64_t)i * slot_words), 0, budget < lim ? budget : lim};
  bits[i] = encode_ints<B>(w, u, budget, maxprec);
}

// ------------------------------------------------------------------------------------------------ synthetic data
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill_normal(float* __restrict__ out, uint64_t count, double sigma, uint64_t seed, int inject)
{
  // one lane per 4-value block: two Box-Muller pairs from counter-based splitmix64
  const uint64_t blk = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk * 4 >= count) return;
  float v[4];
#pragma unroll
  for (int pr = 0; pr < 2; pr++) {
    const uint64_t c = blk * 4 + 2 * pr;
    const double u1 = ((double)(mix64(seed ^ (c * 0xD1B54A32D192ED03ull)) >> 11) + 1.0) * 0x1.0p-53;
    const double u2 = (double)(mix64(seed ^ ((c + 1) * 0xD1B54A32D192ED03ull)) >> 11) * 0x1.0p-53;
    const double r = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    v[2 * pr] = (float)(sigma * r * cs);
    v[2 * pr + 1] = (float)(sigma * r * sn);
  }
  if (inject) {
    const uint64_t h = mix64(blk ^ seed);
    double scale = 1.0;
    if (h % 64 == 0) scale = 0.0;
    else if (h % 4096 == 1) scale = 1e-35 / sigma;
    else if (h % 4096 == 2) scale = 1e-40 / sigma;
    if (scale != 1.0)
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = (float)((double)v[i] * scale);
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (blk * 4 + i < count) out[blk * 4 + i] = v[i];
}

// ------------------------------------------------------------------------------------------------ launchers
static inline hipStream_t S(void* s) { return (hipStream_t)s; }

template <int DT, uint32_t WB>
static void launch_fixed1d_t(const void* in, uint64_t nvals, const Params& p, void* out, hipStream_t st)
{
  const uint32_t nfull = (uint32_t)(nvals / 4);
  if (nfull) {
    // the lean coder needs prec >= 32 for every nonzero block: e >= -126 => e - minexp + 4 >= 32
    const bool kmin0 = p.maxprec >= 32 && p.minexp <= -154;
    if (!kmin0) {
      k_encode_fixed1d_generic<DT, WB><<<(nfull + 511) / 512, 256, 0, st>>>(in, nfull, p, out);
    } else {
      // one-shot grid, U = 8 blocks per lane; chunks keep every buffer offset below 2^32
      constexpr uint32_t CH = 1u << 27;
      constexpr uint32_t IB = DT == DT_BF16 ? 8u : 16u;
      for (uint32_t c0 = 0; c0 < nfull; c0 += CH) {
        const uint32_t nc = min(CH, nfull - c0);
        const void* ic = (const char*)in + (size_t)c0 * IB;
        void* oc = (char*)out + (size_t)c0 * (WB / 8);
#ifndef GCOW_C2_U
#define GCOW_C2_U 8  // A/B builds only (tools/build_variant.sh -DGCOW_C2_U=4)
#endif
        constexpr int U = GCOW_C2_U;
#ifndef GCOW_C2_LDS_PAD
#define GCOW_C2_LDS_PAD 0  // A/B builds only: unused dynamic LDS per workgroup, i.e. fewer workgroups per CU
#endif
        k_encode_fixed1d_np<DT, WB, U, 256, 3><<<(nc + 256 * U - 1) / (256 * U), 256, GCOW_C2_LDS_PAD, st>>>(ic, nc, p,
                                                                                                          oc);
      }
    }
  }
  if (nvals % 4) k_encode_fixed1d_tail<DT, WB><<<1, 128, 0, st>>>(in, nvals, nfull, p, out);
}

hipError_t launch_copy_pattern1d(const void* in, int dtype, uint64_t nvals, uint32_t wb, void* out, void* stream)
{
  const uint32_t nfull = (uint32_t)(nvals / 4);
  constexpr uint32_t CH = 1u << 27;
  const uint32_t IB = dtype == DT_BF16 ? 8u : 16u;
  for (uint32_t c0 = 0; c0 < nfull; c0 += CH) {
    const uint32_t nc = std::min(CH, nfull - c0);
    const void* ic = (const char*)in + (size_t)c0 * IB;
    void* oc = (char*)out + (size_t)c0 * (wb / 8);
    const uint32_t g = (nc + 2047) / 2048;
    if (dtype == DT_BF16) {
      if (wb == 64) k_copy_pattern1d<DT_BF16, 64, 8><<<g, 256, 0, S(stream)>>>(ic, nc, oc);
      else k_copy_pattern1d<DT_BF16, 32, 8><<<g, 256, 0, S(stream)>>>(ic, nc, oc);
    } else {
      if (wb == 64) k_copy_pattern1d<DT_F32, 64, 8><<<g, 256, 0, S(stream)>>>(ic, nc, oc);
      else k_copy_pattern1d<DT_F32, 32, 8><<<g, 256, 0, S(stream)>>>(ic, nc, oc);
    }
  }
  return hipGetLastError();
}

hipError_t launch_encode_fixed1d(const void* in, int dtype, uint64_t nvals, uint32_t nblocks, const Params& p,
                                 void* out, void* stream)
{
  (void)nblocks;
  hipStream_t st = S(stream);
  if (dtype == DT_F32) {
    if (p.maxbits == 64) launch_fixed1d_t<DT_F32, 64>(in, nvals, p, out, st);
    else launch_fixed1d_t<DT_F32, 32>(in, nvals, p, out, st);
  } else {
    if (p.maxbits == 64) launch_fixed1d_t<DT_BF16, 64>(in, nvals, p, out, st);
    else launch_fixed1d_t<DT_BF16, 32>(in, nvals, p, out, st);
  }
  return hipGetLastError();
}

template <int D, int DT, uint32_t T>
static hipError_t launch_tiles_t(const FieldDesc& F, const Params& p, const TilePlan& plan, uint32_t* out32,
                                 uint64_t* ws_sums, uint64_t* ws_base, uint64_t* d_total, uint64_t* index,
                                 uint32_t index_shift, const uint64_t* d_base, hipStream_t st)
{
  const size_t lds = (size_t)plan.lds_words * 4;
  if (plan.fixed) {
    auto kern = k_encode_tiles<D, DT, T, true>;
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<plan.nranges, T, lds, st>>>(F, p, plan.range, nullptr, out32, index, index_shift);
    return hipGetLastError();
  }
  const bool var1d = D == 1 && T == 256 && p.minbits <= 1 && p.maxbits >= 160;
  // variant 2 (A/B, tests): the single-pass look-back encoder (var1d.hip). Not the default: on C5 it ran 0.907 ms
  // against 0.757 ms for count + scan + encode (profiles/r03_c5_single_pass_ab.log)
  const int form = g_var1d_variant.form;
  if (var1d && form == 2) return launch_encode1d_var_sp(F, p, out32, ws_sums, d_total, index, index_shift, d_base, st);
  // variant 1 (A/B, tests): the count + scan + k_encode1d_var form over ranges of plan.range blocks.
  // Default: the tile form (var1d.hip: count per tile with byte lengths, scan, the tile coder placed by the scan)
  if (var1d && form != 1)
    return launch_encode1d_var_tile(F, p, out32, ws_sums, d_total, index, index_shift, d_base, st);
  if (var1d) k_count1d_var<DT, 4><<<plan.nranges, T, 0, st>>>(F, p, plan.range, ws_sums);
  else k_count<D, DT, T><<<plan.nranges, T, 0, st>>>(F, p, plan.range, ws_sums);
  scan_ranges(ws_sums, plan.nranges, ws_base, d_total, out32, d_base, st);
  if (var1d) {
    // U = 4 blocks per lane (U = 8 measured 0.835 -> 1.083 ms on C5 acc 1e-6: register pressure)
    k_encode1d_var<DT, 4><<<plan.nranges, T, 0, st>>>(F, p, plan.range, ws_base, out32, index, index_shift);
    return hipGetLastError();
  }
  auto kern = k_encode_tiles<D, DT, T, false>;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<plan.nranges, T, lds, st>>>(F, p, plan.range, ws_base, out32, index, index_shift);
  return hipGetLastError();
}

hipError_t launch_encode_tiles(const FieldDesc& F, const Params& p, const TilePlan& plan, uint32_t* out32,
                               uint64_t* ws_sums, uint64_t* ws_base, uint64_t* d_total, uint64_t* index,
                               uint32_t index_shift, const uint64_t* d_base, void* stream)
{
  hipStream_t st = S(stream);
  const bool bf = F.dtype == DT_BF16;
#define GCOW_TILES(D, T)                                                                                       \
  return bf ? launch_tiles_t<D, DT_BF16, T>(F, p, plan, out32, ws_sums, ws_base, d_total, index, index_shift, d_base, st) \
            : launch_tiles_t<D, DT_F32, T>(F, p, plan, out32, ws_sums, ws_base, d_total, index, index_shift, d_base, st)
  if (F.dims != 1) return launch_encode_tiles23(F, p, plan, out32, ws_sums, ws_base, d_total, index, index_shift, d_base, st);
  if (plan.threads == 256) { GCOW_TILES(1, 256); } else { GCOW_TILES(1, 64); }
#undef GCOW_TILES
}

hipError_t launch_encode4d(const FieldDesc& F, const Params& p, uint32_t* lens, const uint64_t* rbase, uint32_t* out32,
                           uint64_t* index, uint32_t index_shift, void* stream)
{
  if (F.dtype == DT_BF16)
    k_encode4d<DT_BF16><<<F.nblocks, 64, 0, S(stream)>>>(F, p, lens, rbase, out32, index, index_shift);
  else
    k_encode4d<DT_F32><<<F.nblocks, 64, 0, S(stream)>>>(F, p, lens, rbase, out32, index, index_shift);
  return hipGetLastError();
}

hipError_t launch_decode4d(const FieldDesc& F, const Params& p, const uint64_t* in, const uint64_t* index,
                           uint64_t base_bits, void* stream)
{
  k_decode4d<<<F.nblocks, 64, 0, S(stream)>>>(F, p, in, index, base_bits);
  return hipGetLastError();
}

hipError_t launch_decode4d_seq(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t base_bits,
                               uint64_t* end, void* stream)
{
  k_decode4d_seq<<<1, 64, 0, S(stream)>>>(F, p, in, base_bits, end);
  return hipGetLastError();
}

hipError_t launch_scan_blocks(const uint32_t* lens, uint32_t nblocks, uint64_t* sums, uint64_t* base, uint64_t* total,
                              uint32_t* out32, void* stream)
{
  k_widen_u32<<<(nblocks + 255) / 256, 256, 0, S(stream)>>>(lens, nblocks, sums);
  scan_ranges(sums, nblocks, base, total, out32, nullptr, S(stream));
  return hipGetLastError();
}

// The second-pass flag words of launch_decode1d_var: kVdecFlagRing zeroed uint64 words per device, allocated on first
// use and kept for the life of the process (nullptr if the allocation fails: the second pass then checks every group).
// The first use allocates and zeroes on the caller's stream and waits for it; a first use inside stream capture
// (where neither is allowed) returns nullptr instead -- that decode checks every group, and the ring is allocated by
// the next uncaptured call.
constexpr uint32_t kVdecFlagRing = 256;
static uint64_t* vdec_flag_ring(hipStream_t st)
{
  static std::mutex mu;
  static uint64_t* ring[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(mu);
  if (!ring[dev]) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
      (void)hipGetLastError();
      return nullptr;
    }
    uint64_t* r = nullptr;
    if (hipMalloc((void**)&r, kVdecFlagRing * sizeof(uint64_t)) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    if (hipMemsetAsync(r, 0, kVdecFlagRing * sizeof(uint64_t), st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipFree(r);
      return nullptr;
    }
    ring[dev] = r;
  }
  return ring[dev];
}

hipError_t launch_decode1d_var(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t in_words,
                               const uint64_t* index, uint32_t chunk, uint64_t nchunks, uint64_t base_bits,
                               uint64_t* end_out, void* stream)
{
  if (index && chunk == 16 && in_words) {  // the workgroup's stream span staged in LDS, 128 lanes
    constexpr uint32_t L = 128;
    const uint64_t ng = (nchunks + L - 1) / L;
    // a stream-ordered flag word: a main-kernel workgroup that leaves its group to the second pass raises the word to
    // this call's sequence number (atomicMax), and the second pass returns at once unless the word is >= its number,
    // so an empty second pass costs one load per workgroup instead of every group's span check (~40 us). The words
    // are a persistent per-device ring (no allocation per call, nothing captured into a graph but the pointer):
    // numbers only grow, so a word raised by a later call or by a concurrent decode on another stream can only make a
    // second pass check every group (slower, still exact), never skip one that has work.
    static std::atomic<uint64_t> g_seq{1};
    const uint64_t seq = g_seq.fetch_add(1);
    hipStream_t st = S(stream);
    uint64_t* left = vdec_flag_ring(st);
    if (left) left += seq % kVdecFlagRing;
    // the main kernel's stage: the smallest of 32 / 48 / 64 bits per block that holds 1.25 x the buffer's average
    // (LDS sets its occupancy: 8 / 6 / 4.5 waves per SIMD; accuracy 1e-3 bf16, 24 bits per block: 0.43 -> 0.35 ms).
    // The buffer is the caller's: a capacity-sized one (Encoder.words) reads as dense and keeps 64.
    const uint64_t nb = F.nblocks ? F.nblocks : 1, avail = in_words * 64 - std::min<uint64_t>(base_bits, in_words * 64);
    const uint32_t gbig = (uint32_t)std::min<uint64_t>(ng, 1024);
    if (GCOW_VDEC_ADAPT && avail >= nb * 128) {
      // a buffer of (near) the encoder's capacity (140 bits per block) says nothing about the stream: the 32- and
      // 64-bit stage tiers launched gated on the stream's own average from its index (vdec_tier), the one that does not
      // match returning after two index loads per workgroup (accuracy 1e-3 in a capacity buffer: 0.42 -> 0.37 ms;
      // 1e-6: +13 us for the empty tier, profiles/r06_vdec_capacity_tiers.log)
      k_decode1d_var_lean<L, 32><<<(uint32_t)ng, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits, end_out,
                                                             left, seq, 1u);
      k_decode1d_var_lean<L, 64><<<(uint32_t)ng, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits, end_out,
                                                             left, seq, 3u);
      k_decode1d_var_lean_big<L, 64><<<gbig, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits, end_out, left,
                                                         seq, true);
    } else if (GCOW_VDEC_ADAPT && avail * 5 <= nb * 32 * 4) {
      k_decode1d_var_lean<L, 32><<<(uint32_t)ng, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits, end_out,
                                                             left, seq, 0u);
      k_decode1d_var_lean_big<L, 32><<<gbig, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits, end_out, left,
                                                         seq, false);
    } else if (GCOW_VDEC_ADAPT && avail * 5 <= nb * 48 * 4) {
      k_decode1d_var_lean<L, 48><<<(uint32_t)ng, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits, end_out,
                                                             left, seq, 0u);
      k_decode1d_var_lean_big<L, 48><<<gbig, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits, end_out, left,
                                                         seq, false);
    } else {
      k_decode1d_var_lean<L, GCOW_VDEC_CAPB><<<(uint32_t)ng, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits,
                                                                         end_out, left, seq, 0u);
      k_decode1d_var_lean_big<L, GCOW_VDEC_CAPB><<<gbig, L, 0, st>>>(F, p, in, in_words, index, nchunks, base_bits,
                                                                     end_out, left, seq, false);
    }
    return hipGetLastError();
  }
  k_decode1d_var<<<(uint32_t)((nchunks + 255) / 256), 256, 0, S(stream)>>>(F, p, in, index, chunk, nchunks, base_bits,
                                                                           end_out);
  return hipGetLastError();
}

hipError_t launch_decode_fixed1d(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t base_bits,
                                 void* stream)
{
  const uint32_t nfull = (uint32_t)(F.n[0] / 4);
  constexpr uint32_t CH = 1u << 27;
  for (uint32_t c0 = 0; c0 < nfull; c0 += CH) {  // one-shot grid, U = 8 (64-bit blocks) / 16 (32-bit) words per lane
    const uint32_t nc = min(CH, nfull - c0);
    const bool bf = F.dtype == DT_BF16;
    void* out = (char*)F.data + (size_t)c0 * 4 * (bf ? 2 : 4);
    const uint64_t bb = base_bits + (uint64_t)c0 * p.maxbits;
#ifndef GCOW_C2DEC_U
#define GCOW_C2DEC_U 8
#endif
    constexpr uint32_t U64 = GCOW_C2DEC_U;
    const uint32_t g64 = (nc + 256 * U64 - 1) / (256 * U64), g32 = (nc + 4095) / 4096;
    if (p.maxbits == 64 && bf) k_decode_fixed1d_np<64, U64, true><<<g64, 256, 0, S(stream)>>>(in, nc, p, out, bb);
    else if (p.maxbits == 64) k_decode_fixed1d_np<64, U64><<<g64, 256, 0, S(stream)>>>(in, nc, p, out, bb);
    else if (bf) k_decode_fixed1d_np<32, 16, true><<<g32, 256, 0, S(stream)>>>(in, nc, p, out, bb);
    else k_decode_fixed1d_np<32, 16><<<g32, 256, 0, S(stream)>>>(in, nc, p, out, bb);
  }
  if (F.n[0] % 4) k_decode_tail1d<<<1, 1, 0, S(stream)>>>(F, p, in, base_bits, nfull);
  return hipGetLastError();
}

hipError_t launch_scan_ranges(const uint64_t* sums, uint32_t nranges, uint64_t* base, uint64_t* total, uint32_t* out32,
                              const uint64_t* d_base, void* stream, const uint64_t* gsums)
{
  scan_ranges(sums, nranges, base, total, out32, d_base, S(stream), gsums);
  return hipGetLastError();
}

hipError_t launch_set_u64(uint64_t* p, uint64_t v, void* stream)
{
  k_set_u64<<<1, 1, 0, S(stream)>>>(p, v);
  return hipGetLastError();
}

hipError_t launch_words_differ(const uint64_t* a, const uint64_t* b, uint64_t n, uint64_t* flag, void* stream)
{
  k_set_u64<<<1, 1, 0, S(stream)>>>(flag, 0ull);
  if (n) {
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 4096);
    k_words_differ<<<(uint32_t)g, 256, 0, S(stream)>>>(a, b, n, flag);
  }
  return hipGetLastError();
}

hipError_t launch_prepend_header(uint64_t* dst, uint32_t off, const uint64_t* src, const uint64_t* d_bits,
                                 const uint64_t* header, uint64_t max_words, uint64_t* d_total, void* stream)
{
  const uint64_t grid = (max_words + 255) / 256;
  k_prepend_header<<<(uint32_t)(grid ? grid : 1), 256, 0, S(stream)>>>(dst, off, src, d_bits, header[0], header[1],
                                                                      header[2], d_total);
  return hipGetLastError();
}

hipError_t launch_stitch(uint64_t* dst, uint64_t off, const uint64_t* src, uint64_t bits, void* stream)
{
  if (!bits) return hipSuccess;
  const uint64_t words = ((off + bits + 63) >> 6) - (off >> 6);
  const uint64_t grid = (words + 255) / 256;
  k_stitch<<<grid, 256, 0, S(stream)>>>(dst, off, src, bits);
  return hipGetLastError();
}

hipError_t launch_stitch_shards(uint64_t* dst, uint64_t dst_words, const uint64_t* src, uint64_t shard_words,
                                const uint64_t* lens, uint32_t nshards, void* stream)
{
  const uint64_t grid = (dst_words + 255) / 256;
  if (!grid) return hipSuccess;
  k_stitch_shards<<<(uint32_t)grid, 256, 0, S(stream)>>>(dst, dst_words, src, shard_words, lens, nshards);
  return hipGetLastError();
}

// GCOW_INDEX_PACKED16 from an index every 8 blocks: entry c = idx8[2c] | (idx8[2c + 1] - idx8[2c]) << 48 (offset 0
// where block 16 c + 8 does not exist).
__global__ __launch_bounds__(256) void k_index_pack16(const uint64_t* __restrict__ idx8, uint64_t n8,
                                                      uint64_t* __restrict__ out, uint64_t n16)
{
  const uint64_t c = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (c >= n16) return;
  const uint64_t a = idx8[2 * c];
  const uint64_t d = 2 * c + 1 < n8 ? idx8[2 * c + 1] - a : 0ull;
  out[c] = a | (d << 48);
}

hipError_t launch_index_pack16(const uint64_t* idx8, uint64_t n8, uint64_t* out, void* stream)
{
  const uint64_t n16 = (n8 + 1) / 2;
  if (!n16) return hipSuccess;
  k_index_pack16<<<(uint32_t)((n16 + 255) / 256), 256, 0, S(stream)>>>(idx8, n8, out, n16);
  return hipGetLastError();
}

hipError_t launch_decode_mean1d(const FieldDesc& F, const Params& p, const uint64_t* in, uint64_t stream_words,
                                uint32_t nstreams, const uint64_t* index, uint64_t index_words, void* stream,
                                uint32_t chunk)
{
  if (!F.nblocks) return hipSuccess;
  hipStream_t st = S(stream);
  if (p.minbits == p.maxbits) {
    const bool lean = p.maxprec >= 32 && p.minexp <= -154 && (p.maxbits == 64 || p.maxbits == 32);
    const uint32_t nfull = (uint32_t)(F.n[0] / 4);
    uint64_t done = 0;
#ifndef GCOW_DMEAN_LEAN
#define GCOW_DMEAN_LEAN 1
#endif
    if (GCOW_DMEAN_LEAN && lean && nfull && F.nblocks < (1u << 27)) {  // one-shot grid, U = 2 per lane (U = 1 / 4 / 8: 2.47 / 2.37 / 3.0 against 2.33 ms, W = 8 rate 16: profiles/r04_decode_mean_blocks_per_lane.log)
#ifndef GCOW_DMEAN_U
#define GCOW_DMEAN_U 2
#endif
#ifndef GCOW_DMEAN_D
#define GCOW_DMEAN_D 1
#endif
      constexpr int U = GCOW_DMEAN_U, D = GCOW_DMEAN_D;
      const uint32_t g = (nfull + 256 * U - 1) / (256 * U);
      if (p.maxbits == 64) k_decode_mean_fixed1d_np<64, U, D><<<g, 256, 0, st>>>(F, p, in, stream_words, nstreams, nfull);
      else k_decode_mean_fixed1d_np<32, U, D><<<g, 256, 0, st>>>(F, p, in, stream_words, nstreams, nfull);
      done = nfull;
    }
    const uint64_t rest = F.nblocks - done;
    if (rest) {
      const uint32_t g = (uint32_t)((rest + 255) / 256);
      if (p.maxprec >= 32 && p.minexp <= -154 && p.maxbits == 64)
        k_decode_mean_fixed1d<64><<<g, 256, 0, st>>>(F, p, in, stream_words, nstreams, done);
      else if (p.maxprec >= 32 && p.minexp <= -154 && p.maxbits == 32)
        k_decode_mean_fixed1d<32><<<g, 256, 0, st>>>(F, p, in, stream_words, nstreams, done);
      else k_decode_mean_fixed1d<0><<<g, 256, 0, st>>>(F, p, in, stream_words, nstreams, done);
    }
    return hipGetLastError();
  }
  // variable rate: one lane per index chunk of `chunk` blocks (the streams' index stride, 8 or 16; the packed16
  // index is read as 8-block chunks)
  const bool pk = chunk == kIndexPacked16;
  if (pk) chunk = 8;
  if (chunk != 8 && chunk != 16) return hipErrorInvalidValue;
  const uint64_t nchunks = (F.nblocks + chunk - 1) / chunk;
  if (!(p.minbits <= 1 && p.maxbits >= 160)) {  // a budget can truncate blocks: generic decoder
    const uint32_t g = (uint32_t)((nchunks + 255) / 256);
    if (pk) k_decode_mean1d_generic<true><<<g, 256, 0, st>>>(F, p, in, stream_words, index, index_words, nchunks,
                                                             nstreams, chunk);
    else k_decode_mean1d_generic<false><<<g, 256, 0, st>>>(F, p, in, stream_words, index, index_words, nchunks,
                                                           nstreams, chunk);
    return hipGetLastError();
  }
  // complete workgroups (128 whole chunks of full blocks, contiguous output) by the lean kernel, the rest by the
  // general one
  uint64_t nlean = 0;
  if (F.vec) {
    const uint64_t fullchunks = (F.n[0] / 4) / chunk;
    nlean = std::min<uint64_t>(fullchunks, nchunks) / 128;
    if (nlean) {
      if (pk)
        k_decode_mean1d_var_lean<128, 64, 8, true><<<(uint32_t)nlean, 128, 0, st>>>(F, p, in, stream_words, index,
                                                                                    index_words, nchunks, nstreams);
      else if (chunk == 8)
        k_decode_mean1d_var_lean<128, 64, 8><<<(uint32_t)nlean, 128, 0, st>>>(F, p, in, stream_words, index,
                                                                              index_words, nchunks, nstreams);
      else
        k_decode_mean1d_var_lean<128, 64, 16><<<(uint32_t)nlean, 128, 0, st>>>(F, p, in, stream_words, index,
                                                                               index_words, nchunks, nstreams);
    }
  }
  const uint64_t cfirst = nlean * 128;
  if (cfirst < nchunks) {
    const uint32_t g = (uint32_t)((nchunks - cfirst + 127) / 128);
    if (pk)
      k_decode_mean1d_var<128, 8, true><<<g, 128, 0, st>>>(F, p, in, stream_words, index, index_words, nchunks,
                                                           nstreams, cfirst);
    else if (chunk == 8)
      k_decode_mean1d_var<128, 8><<<g, 128, 0, st>>>(F, p, in, stream_words, index, index_words, nchunks, nstreams,
                                                     cfirst);
    else
      k_decode_mean1d_var<128, 16><<<g, 128, 0, st>>>(F, p, in, stream_words, index, index_words, nchunks, nstreams,
                                                      cfirst);
  }
  return hipGetLastError();
}

hipError_t launch_stage(int which, int dims, const void* a, const void* b, uint32_t n, void* out, uint32_t x0,
                        uint32_t x1, void* out2, uint32_t slot_words, void* stream)
{
  const uint32_t grid = (n + 63) / 64;
  if (!grid) return hipSuccess;
  hipStream_t st = S(stream);
#define GCOW_STAGE(D)                                                                                          \
  switch (which) {                                                                                             \
    case 0: k_stage_emax<D><<<grid, 64, 0, st>>>((const float*)a, n, (int32_t*)out); break;                    \
    case 1: k_stage_cast<D><<<grid, 64, 0, st>>>((const float*)a, (const int32_t*)b, n, (int32_t*)out); break; \
    case 2: k_stage_xform<D><<<grid, 64, 0, st>>>((int32_t*)out, n, (int)x0); break;                           \
    case 3: k_stage_reorder<D><<<grid, 64, 0, st>>>((const int32_t*)a, n, (uint32_t*)out); break;              \
    case 4:                                                                                                    \
      k_stage_encode_ints<D><<<grid, 64, 0, st>>>((const uint32_t*)a, n, x0, x1, (uint64_t*)out, slot_words,   \
                                                  (uint32_t*)out2);                                            \
      break;                                                                                                   \
    default: return hipErrorInvalidValue;                                                                      \
  }
  if (dims == 1) { GCOW_STAGE(1) }
  else if (dims == 2) { GCOW_STAGE(2) }
  else { GCOW_STAGE(3) }
#undef GCOW_STAGE
  return hipGetLastError();
}

hipError_t launch_fill_normal(float* out, uint64_t count, double sigma, uint64_t seed, int inject, void* stream)
{
  const uint64_t blocks = (count + 3) / 4;
  const uint64_t grid = (blocks + 255) / 256;
  if (!grid) return hipSuccess;
  k_fill_normal<<<grid, 256, 0, S(stream)>>>(out, count, sigma, seed, inject);
  return hipGetLastError();
}

}  // namespace gcow
