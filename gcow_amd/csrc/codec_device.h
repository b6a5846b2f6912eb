// codec_device.h -- per-block ZFP-style codec primitives for CDNA4 (gfx950), one block per lane.
//
// Every function restates one stage of gcow's sw/ encoder (fpgasystems/gcow sw/src/encode.c) or libzfp 0.5.5's
// decoder (the semantics sw/src/decode.c intends), cited per function. Bit-exactness notes:
//   * block exponent is computed on the IEEE bit patterns (max over non-NaN |x|; Inf -> 0 as glibc frexp);
//   * the float->int cast emulates x86 cvttss2si: NaN / +-Inf / out-of-range -> INT_MIN (AMD's v_cvt_i32_f32
//     saturates instead, so the range test is explicit);
//   * lifting uses uint32 add/sub (int32 wraparound) and arithmetic right shifts;
//   * the embedded coder emits the untruncated code and the writer drops bits beyond the block budget -- the
//     budgeted coder's output (encode.c:279-339) is exactly that prefix.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gcow {

enum : uint32_t { DT_F32 = 3, DT_BF16 = 5 };

struct Params {
  uint32_t minbits, maxbits, maxprec;
  int32_t minexp;
};

// ------------------------------------------------------------------------------------------------ constants
template <int D> struct Dim;
template <> struct Dim<1> { static constexpr int B = 4; };
template <> struct Dim<2> { static constexpr int B = 16; };
template <> struct Dim<3> { static constexpr int B = 64; };

// sw/include/types.h:71-97 PERM_2D; identity for 1-D; libzfp 0.5.5 perm_3 for 3-D.
__device__ __host__ constexpr int perm_index(int D, int i)
{
  constexpr uint8_t P2[16] = {0, 1, 4, 5, 2, 8, 6, 9, 3, 12, 10, 7, 13, 11, 14, 15};
  constexpr uint8_t P3[64] = {0,  1,  4,  16, 20, 17, 5,  2,  8,  32, 21, 6,  18, 24, 9,  33,
                              36, 3,  12, 48, 22, 25, 37, 40, 34, 10, 7,  19, 28, 13, 49, 52,
                              41, 38, 26, 23, 29, 53, 11, 35, 44, 14, 50, 56, 42, 27, 39, 45,
                              30, 54, 57, 60, 51, 15, 43, 46, 58, 61, 55, 31, 62, 59, 47, 63};
  return D == 1 ? i : (D == 2 ? P2[i] : P3[i]);
}

template <int B> struct PlaneType { using T = uint32_t; };
template <> struct PlaneType<64> { using T = uint64_t; };

// v_ffbh_u32: leading zeros, all ones for 0 (not undefined, unlike __builtin_clz)
__device__ __forceinline__ uint32_t ffbh_u32(uint32_t x)
{
  uint32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

__device__ __forceinline__ uint64_t lowmask64(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }

// ------------------------------------------------------------------------------------------------ LDS staging
// Workgroup prologues (lookup tables, a stream span) copied global -> LDS with every load issued before the first LDS
// write: one memory round trip per prologue. The plain `for (j = tid; j < n; j += T) lds[j] = g[j]` has a trip count
// the compiler cannot see, and compiles to load -> s_waitcnt vmcnt(0) -> ds_write per iteration: one full memory
// latency per iteration (10-20 of them per workgroup in the decoders before this was changed).
typedef unsigned int st_v4u __attribute__((ext_vector_type(4)));

// nbytes (<= MAXC * 16) bytes from src (16-byte aligned) to dst[0 .. MAXC) as 16-byte chunks; chunks past nbytes read
// zero (buffer range check), so every lane issues the same loads. T threads.
// SWZ: a stream span for lane-parallel bit reads -- chunk k goes to chunk slot k ^ ((k >> 4) & 15), i.e. qword q of
// the span lives at lds_qword_swz(q): each 256-byte bank row's qword pairs XOR-permuted by the row index, so lanes
// reading chunk starts spaced a multiple of ~32 qwords apart (8- or 16-block chunks at any bit rate) land on
// different banks.
#ifndef GCOW_SWZ_OPAQUE_ZERO
#define GCOW_SWZ_OPAQUE_ZERO 0  // measurement builds: the same instructions with an identity mapping (an opaque 0 mask)
#endif
__device__ __forceinline__ uint32_t swz_mask(uint32_t m)
{
  if constexpr (GCOW_SWZ_OPAQUE_ZERO) {
    uint32_t z = 0;
    asm volatile("" : "+v"(z));
    return m & z;
  }
  return m;
}
__device__ __forceinline__ uint32_t lds_qword_swz(uint32_t q) { return q ^ ((q >> 4) & swz_mask(30u)); }

template <uint32_t T, uint32_t MAXC, bool SWZ = false>
__device__ __forceinline__ void stage_lds16(void* dst, const void* src, uint32_t nbytes)
{
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src), 0, (int)nbytes, 0x00020000);
  constexpr uint32_t R = (MAXC + T - 1) / T;
  // the swizzle permutes chunks within groups of 16: a partial last group must be one the swizzle leaves in place
  static_assert(!SWZ || MAXC % 16 == 0 || ((MAXC >> 4) & 15u) == 0, "swizzled chunks stay inside the stage");
  st_v4u v[R];
#pragma unroll
  for (uint32_t i = 0; i < R; i++) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((threadIdx.x + T * i) * 16u), 0, 0);
#pragma unroll
  for (uint32_t i = 0; i < R; i++) {
    const uint32_t k = threadIdx.x + T * i;
    if (MAXC % T == 0 || k < MAXC) ((st_v4u*)dst)[SWZ ? k ^ ((k >> 4) & swz_mask(15u)) : k] = v[i];
  }
}

// A constant table of N 32-bit words (N * 4 a multiple of 16) into LDS.
template <uint32_t T, uint32_t N>
__device__ __forceinline__ void stage_table(uint32_t* dst, const void* tab)
{
  static_assert(N % 4 == 0, "whole 16-byte chunks");
  stage_lds16<T, N / 4>(dst, tab, N * 4u);
}

// ------------------------------------------------------------------------------------------------ stages
// get_block_exponent + get_scaler_exponent (encode.c:128-152) on bit patterns.
template <int B>
__device__ __forceinline__ int block_emax(const float (&f)[B])
{
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < B; i++) {
    uint32_t a = __float_as_uint(f[i]) & 0x7fffffffu;
    m = (a <= 0x7f800000u && a > m) ? a : m;  // `max < f` never lets a NaN win
  }
  int e = (int)(m >> 23) - 126;
  e = e < -126 ? -126 : e;                       // MAX(e, 1 - EBIAS): subnormals clamp to -126
  return m == 0 ? -127 : (m >= 0x7f800000u ? 0 : e);  // zero -> -EBIAS; Inf -> 0 (glibc frexp)
}

// get_precision (sw/src/common.c:226-229)
__device__ __forceinline__ uint32_t precision(int emax, uint32_t maxprec, int minexp, int dims)
{
  int p = emax - minexp + 2 * dims + 2;
  uint32_t up = p > 0 ? (uint32_t)p : 0u;
  return up < maxprec ? up : maxprec;
}

// quantize_scaler / fwd_cast_block (encode.c:162-187): (int32)(2^(30-emax) * x) with x86 semantics.
__device__ __forceinline__ float cast_scale(int emax)
{
  int se = 30 - emax;  // >= -98, so the scale is a normal float or +inf
  return se >= 128 ? __uint_as_float(0x7f800000u) : __uint_as_float((uint32_t)(se + 127) << 23);
}

__device__ __forceinline__ int32_t cast1(float x, float scale)
{
  float p = scale * x;
  return (__builtin_fabsf(p) < 2147483648.0f) ? (int32_t)p : (int32_t)0x80000000;
}

// block_emax + the cast (encode.c:128-187) for a block without Inf or NaN, in about two operations per value (the
// two-pass 3-D tile kernels; the fixed-rate kernel keeps block_emax + cast1, whose register allocation it is tuned
// to): max |x| as the larger of an unsigned and a signed max over the bit patterns (the largest negative magnitude,
// the largest positive value: v_max3, no per-value masking), then one fma + the hardware truncating conversion per
// value. A finite block's products 2^(30 - emax) x lie below 2^30 in magnitude, so the conversion matches
// cvttss2si; with an infinite scale (emax <= -98, zero blocks included) x86 gives INT_MIN for every value, here
// fma(x, 0, -inf) -> saturated INT_MIN. Returns false when the block holds Inf or NaN (the caller takes block_emax
// + cast1).
template <int B>
__device__ __forceinline__ bool emax_cast_finite(const float* fa, int& emax, int32_t* q)
{
  uint32_t mu = 0;
  int32_t mi = 0;
#pragma unroll
  for (int i = 0; i < B; i += 2) {
    const uint32_t a = __float_as_uint(fa[i]), b = __float_as_uint(fa[i + 1]);
    mu = max(mu, max(a, b));
    mi = max(mi, max((int32_t)a, (int32_t)b));
  }
  const uint32_t m = max(mu & 0x7fffffffu, (uint32_t)mi & 0x7fffffffu);
  if (m >= 0x7f800000u) return false;
  emax = m == 0 ? -127 : max((int)(m >> 23) - 126, -126);
  const int se = 30 - emax;
  const bool tiny = se >= 128;
  const float s = tiny ? 0.0f : __uint_as_float((uint32_t)(se + 127) << 23);
  const float c = tiny ? -__builtin_inff() : 0.0f;
#pragma unroll
  for (int i = 0; i < B; i++) {
    int32_t v;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(v) : "v"(__builtin_fmaf(fa[i], s, c)));
    q[i] = v;
  }
  return true;
}

// fwd_lift_vector (encode.c:189-249), int32 wraparound made explicit.
__device__ __forceinline__ void fwd_lift(int32_t& x, int32_t& y, int32_t& z, int32_t& w)
{
  auto add = [](int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); };
  auto sub = [](int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); };
  x = add(x, w); x >>= 1; w = sub(w, x);
  z = add(z, y); z >>= 1; y = sub(y, z);
  x = add(x, z); x >>= 1; z = sub(z, x);
  w = add(w, y); w >>= 1; y = sub(y, w);
  w = add(w, y >> 1); y = sub(y, w >> 1);
}

// bwd_lift_vector (decode.c:58-100)
__device__ __forceinline__ void inv_lift(int32_t& x, int32_t& y, int32_t& z, int32_t& w)
{
  auto add = [](int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); };
  auto sub = [](int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); };
  auto shl = [](int32_t a) { return (int32_t)((uint32_t)a << 1); };
  y = add(y, w >> 1); w = sub(w, y >> 1);
  y = add(y, w); w = shl(w); w = sub(w, y);
  z = add(z, x); x = shl(x); x = sub(x, z);
  y = add(y, z); z = shl(z); z = sub(z, y);
  w = add(w, x); x = shl(x); x = sub(x, w);
}

// fwd_decorrelate (encode.c:251-260: x then y; 3-D x, y, z as libzfp)
template <int D>
__device__ __forceinline__ void fwd_xform(int32_t* q)
{
  if constexpr (D == 1) {
    fwd_lift(q[0], q[1], q[2], q[3]);
  } else if constexpr (D == 2) {
#pragma unroll
    for (int y = 0; y < 4; y++) fwd_lift(q[4 * y + 0], q[4 * y + 1], q[4 * y + 2], q[4 * y + 3]);
#pragma unroll
    for (int x = 0; x < 4; x++) fwd_lift(q[x + 0], q[x + 4], q[x + 8], q[x + 12]);
  } else {
#pragma unroll
    for (int z = 0; z < 4; z++)
#pragma unroll
      for (int y = 0; y < 4; y++) {
        int b = 16 * z + 4 * y;
        fwd_lift(q[b + 0], q[b + 1], q[b + 2], q[b + 3]);
      }
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
      for (int z = 0; z < 4; z++) {
        int b = 16 * z + x;
        fwd_lift(q[b + 0], q[b + 4], q[b + 8], q[b + 12]);
      }
#pragma unroll
    for (int y = 0; y < 4; y++)
#pragma unroll
      for (int x = 0; x < 4; x++) {
        int b = 4 * y + x;
        fwd_lift(q[b + 0], q[b + 16], q[b + 32], q[b + 48]);
      }
  }
}

// bwd_decorrelate (decode.c:102-111: y then x; 3-D z, y, x)
template <int D>
__device__ __forceinline__ void inv_xform(int32_t* q)
{
  if constexpr (D == 1) {
    inv_lift(q[0], q[1], q[2], q[3]);
  } else if constexpr (D == 2) {
#pragma unroll
    for (int x = 0; x < 4; x++) inv_lift(q[x + 0], q[x + 4], q[x + 8], q[x + 12]);
#pragma unroll
    for (int y = 0; y < 4; y++) inv_lift(q[4 * y + 0], q[4 * y + 1], q[4 * y + 2], q[4 * y + 3]);
  } else {
#pragma unroll
    for (int y = 0; y < 4; y++)
#pragma unroll
      for (int x = 0; x < 4; x++) {
        int b = 4 * y + x;
        inv_lift(q[b + 0], q[b + 16], q[b + 32], q[b + 48]);
      }
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
      for (int z = 0; z < 4; z++) {
        int b = 16 * z + x;
        inv_lift(q[b + 0], q[b + 4], q[b + 8], q[b + 12]);
      }
#pragma unroll
    for (int z = 0; z < 4; z++)
#pragma unroll
      for (int y = 0; y < 4; y++) {
        int b = 16 * z + 4 * y;
        inv_lift(q[b + 0], q[b + 1], q[b + 2], q[b + 3]);
      }
  }
}

// twoscomplement_to_negabinary + fwd_reorder_int2uint (encode.c:263-275), static permutation.
template <int D>
__device__ __forceinline__ void fwd_reorder(uint32_t* u, const int32_t* q)
{
  constexpr int B = Dim<D>::B;
#pragma unroll
  for (int i = 0; i < B; i++) u[i] = ((uint32_t)q[perm_index(D, i)] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
}

// negabinary_to_twoscomplement + bwd_reorder_uint2int (decode.c:44-56)
template <int D>
__device__ __forceinline__ void inv_reorder(int32_t* q, const uint32_t* u)
{
  constexpr int B = Dim<D>::B;
#pragma unroll
  for (int i = 0; i < B; i++) q[perm_index(D, i)] = (int32_t)((u[i] ^ 0xaaaaaaaau) - 0xaaaaaaaau);
}

// Bit plane k of B coefficients: bit i of the result = bit k of u[i] (encode.c:295-299).
template <int B>
__device__ __forceinline__ typename PlaneType<B>::T get_plane(const uint32_t* u, int k)
{
  using PT = typename PlaneType<B>::T;
  PT x = 0;
#pragma unroll
  for (int i = 0; i < B; i++) x |= (PT)((u[i] >> k) & 1u) << i;
  return x;
}

// In-place 32 x 32 bit-matrix transpose, LSB-first: bit c of a[i] <-> bit i of a[c]. Five delta-swap stages
// (16 swaps each); an involution, so the same call turns coefficient words into bit planes and back.
template <int S, uint32_t M>
__device__ __forceinline__ void transpose32_stage(uint32_t* a)
{
#pragma unroll
  for (int i = 0; i < 32; i++) {
    if (i & S) continue;
    const uint32_t t = ((a[i] >> S) ^ a[i + S]) & M;
    a[i + S] ^= t;
    a[i] ^= t << S;
  }
}

// The same transpose with every stage's results pinned in registers before the next stage starts: keeps the
// scheduler from interleaving the stages of two 32-word transposes (which needs ~100 extra VGPRs).
__device__ __forceinline__ void pin32(uint32_t* a)
{
#pragma unroll
  for (int i = 0; i < 32; i++) asm volatile("" : "+v"(a[i]));
}

__device__ __forceinline__ void transpose32_pinned(uint32_t* a)
{
  transpose32_stage<16, 0x0000FFFFu>(a);
  pin32(a);
  transpose32_stage<8, 0x00FF00FFu>(a);
  pin32(a);
  transpose32_stage<4, 0x0F0F0F0Fu>(a);
  pin32(a);
  transpose32_stage<2, 0x33333333u>(a);
  pin32(a);
  transpose32_stage<1, 0x55555555u>(a);
  pin32(a);
}

// The four S < 16 stages on 16 words: after the S = 16 stage of transpose32, words 16..31 (planes 16..31) and words
// 0..15 (planes 0..15) only mix among themselves (the stages commute), so a coder that stops above plane 16 never
// needs the lower half's stages.
template <int S, uint32_t M>
__device__ __forceinline__ void transpose16_stage(uint32_t* a)
{
#pragma unroll
  for (int i = 0; i < 16; i++) {
    if (i & S) continue;
    const uint32_t t = ((a[i] >> S) ^ a[i + S]) & M;
    a[i + S] ^= t;
    a[i] ^= t << S;
  }
}

__device__ __forceinline__ void pin16(uint32_t* a)
{
#pragma unroll
  for (int i = 0; i < 16; i++) asm volatile("" : "+v"(a[i]));
}

__device__ __forceinline__ void transpose_half_pinned(uint32_t* a)
{
  transpose16_stage<8, 0x00FF00FFu>(a);
  pin16(a);
  transpose16_stage<4, 0x0F0F0F0Fu>(a);
  pin16(a);
  transpose16_stage<2, 0x33333333u>(a);
  pin16(a);
  transpose16_stage<1, 0x55555555u>(a);
  pin16(a);
}

__device__ __forceinline__ void transpose32(uint32_t* a)
{
  transpose32_stage<16, 0x0000FFFFu>(a);
  transpose32_stage<8, 0x00FF00FFu>(a);
  transpose32_stage<4, 0x0F0F0F0Fu>(a);
  transpose32_stage<2, 0x33333333u>(a);
  transpose32_stage<1, 0x55555555u>(a);
}

// ------------------------------------------------------------------------------------------------ writers
// A writer appends bits LSB-first; put(v, n) requires v < 2^n (n <= 64), skip(n) appends zeros.
// Every writer truncates at its limit, which makes the untruncated coder below equal the budgeted one.

// Count-only writer (bit lengths for variable-rate offsets).
struct CountWriter {
  __device__ __forceinline__ void put(uint64_t, uint32_t) {}
  __device__ __forceinline__ void skip(uint32_t) {}
};

// Up to 64 bits in one register (fixed-rate blocks of <= 64 bits).
struct RegWriter64 {
  uint64_t acc;
  uint32_t pos;
  __device__ __forceinline__ void put(uint64_t v, uint32_t n)
  {
    if (pos < 64) acc |= v << pos;
    pos += n;
  }
  __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
};

// One lane's private run of 32-bit words (LDS), written a whole word at a time: no atomics, no zeroing. For
// fixed-rate blocks whose budget is a multiple of 32 bits, so each block owns its words. Bits past `limit` are
// dropped (the budgeted coder's output is that prefix); finish() zero-fills the rest of the block's words.
struct LaneWordWriter {
  uint32_t* w;
  uint64_t acc;
  uint32_t fill, pos, limit;
  __device__ __forceinline__ void put(uint64_t v, uint32_t n)
  {
    if (pos >= limit || n == 0) {
      pos += n;
      return;
    }
    if (n > limit - pos) {
      n = limit - pos;
      v &= lowmask64(n);
    }
    pos += n;
    const uint64_t hi = fill ? (v >> (64 - fill)) : 0ull;  // bits of v past acc's 64
    acc |= v << fill;
    fill += n;  // <= 95
    if (fill >= 32) {
      *w++ = (uint32_t)acc;
      acc = (acc >> 32) | (hi << 32);
      fill -= 32;
      if (fill >= 32) {
        *w++ = (uint32_t)acc;
        acc >>= 32;
        fill -= 32;
      }
    }
  }
  __device__ __forceinline__ void skip(uint32_t n)
  {
    while (n) {
      const uint32_t k = n < 64 ? n : 64;
      put(0ull, k);
      n -= k;
    }
  }
  __device__ __forceinline__ void finish(uint32_t* end)
  {
    if (fill) *w++ = (uint32_t)acc;
    while (w < end) *w++ = 0u;
  }
};

// Bits OR-ed into a zero-initialised LDS window of 32-bit words at a local bit offset.
struct LdsWriter {
  uint32_t* lds;
  uint32_t pos, limit;
  __device__ __forceinline__ void put(uint64_t v, uint32_t n)
  {
    if (pos >= limit || n == 0) { pos += n; return; }
    uint32_t room = limit - pos;
    if (n > room) v &= lowmask64(room);
    uint32_t w = pos >> 5, sh = pos & 31;
    uint32_t p0 = (uint32_t)(v << sh);
    uint32_t p1 = (uint32_t)((v << sh) >> 32);
    uint32_t p2 = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
    if (p0) atomicOr(&lds[w], p0);
    if (p1) atomicOr(&lds[w + 1], p1);
    if (p2) atomicOr(&lds[w + 2], p2);
    pos += n;
  }
  __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
};

// ------------------------------------------------------------------------------------------------ coder
// encode_partial_bitplanes / encode_all_bitplanes (encode.c:279-408). Emits the untruncated plane codes until the
// budget is consumed; returns min(untruncated bits, budget) = what the budgeted coder writes.
// One bit plane of the embedded coder: n bits verbatim, then the group tests of the remainder.
template <int B, class W>
__device__ __forceinline__ void encode_plane(W& w, typename PlaneType<B>::T x, uint32_t budget, uint32_t& bits,
                                             uint32_t& n)
{
  using PT = typename PlaneType<B>::T;
  // step 2: first n bits verbatim
  w.put((uint64_t)x & lowmask64(n), n);
  bits += n;
  PT r = n < (uint32_t)B ? (PT)(x >> n) : (PT)0;
  // step 3: unary run-length (group test) code of the remainder
  while (n < (uint32_t)B && bits < budget) {
    if (r == 0) {  // negative group test: done with this plane
      w.skip(1);
      bits += 1;
      break;
    }
    const uint32_t t = (B == 64) ? (uint32_t)__builtin_ctzll((uint64_t)r) : (uint32_t)__builtin_ctz((uint32_t)r);
    if (n + t < (uint32_t)B - 1) {  // group '1', t zeros, the one-bit
      w.put(1ull | (2ull << t), t + 2);
      bits += t + 2;
      n += t + 1;
      r = (PT)(r >> (t + 1));
    } else {  // the one-bit sits in the last position and is implied
      w.put(1ull, 1);
      w.skip(B - 1 - n);
      bits += B - n;
      n = B;
    }
  }
}

// Planes K, K-1, ..., 0 of a transposed 64-coefficient block with compile-time plane indices (a runtime index
// into the plane registers would put them in scratch).
template <int K, class W>
__device__ __forceinline__ void encode_planes64(W& w, const uint32_t* t, int kmin, uint32_t budget, uint32_t& bits,
                                                uint32_t& n)
{
  if constexpr (K >= 0) {
    if (K < kmin || bits >= budget) return;
    encode_plane<64>(w, (uint64_t)t[K] | ((uint64_t)t[32 + K] << 32), budget, bits, n);
    encode_planes64<K - 1>(w, t, kmin, budget, bits, n);
  }
}

// encode_partial_bitplanes / encode_all_bitplanes (encode.c:279-408). Emits the untruncated plane codes until the
// budget is consumed; returns min(untruncated bits, budget) = what the budgeted coder writes. 64-coefficient blocks
// form all 32 planes with two 32 x 32 bit transposes instead of 64 bit gathers per plane.
template <int B, class W>
__device__ __forceinline__ uint32_t encode_ints(W& w, const uint32_t* u, uint32_t budget, uint32_t maxprec)
{
  const int kmin = maxprec < 32 ? 32 - (int)maxprec : 0;
  uint32_t bits = 0;
  uint32_t n = 0;
  if constexpr (B == 64) {
    uint32_t t[64];
#pragma unroll
    for (int i = 0; i < 64; i++) t[i] = u[i];
    transpose32(t);
    transpose32(t + 32);
    encode_planes64<31>(w, t, kmin, budget, bits, n);
  } else {
    for (int k = 31; k >= kmin && bits < budget; --k) encode_plane<B>(w, get_plane<B>(u, k), budget, bits, n);
  }
  return bits < budget ? bits : budget;
}

// ---- the 64-coefficient coder, plane at a time without a loop over one-bits (3-D blocks)
// Plane k of encode.c:279-339 with n coefficients already significant and r = x >> n is
//   x[0 .. n-1] verbatim, then the group flag (r != 0), then -- if r != 0 -- E(r) through the last one-bit hb of r
//   and a closing '0',
// where E(r) writes every zero bit of r as '0' and every one-bit as '11' (the one-bit, then the flag that opens the
// next group); the last one-bit's second '1' is that closing '0' instead. When the last one-bit is coefficient 63
// (n + hb + 1 = 64) its one is implied: the code stops before it and there is no closing '0'. So a plane is two
// appends: n + 1 verbatim/flag bits, and E(r) (hb + m + 1 bits with m = popcount(r), or hb + m - 1 at coefficient
// 63) built from a 256-entry table of E over 8-bit chunks. Lanes do a fixed amount of work per plane; only chunks
// past the wave's largest hb are skipped.
struct alignas(16) DupTab {
  uint32_t v[256];
};

__host__ __device__ constexpr DupTab make_dup_tab()
{
  DupTab T{};
  for (uint32_t v = 0; v < 256; v++) {
    uint32_t code = 0, len = 0;
    for (uint32_t j = 0; j < 8; j++) {
      if ((v >> j) & 1u) {
        code |= 3u << len;
        len += 2;
      } else {
        len += 1;
      }
    }
    T.v[v] = code;
  }
  return T;
}

__device__ const DupTab g_dup_tab = make_dup_tab();

// Lane-private run of zeroed LDS words with slack words after the block's budget: bits are OR-ed in at their
// position (ds_or, no return), nothing is masked -- code past the budget lands in the slack, which is never stored.
struct OrWriter {
  uint32_t* w;
  uint32_t pos;
  __device__ __forceinline__ void put(uint64_t v, uint32_t n)
  {
    const uint32_t i = pos >> 5, sh = pos & 31u;
    const uint64_t lo = v << sh;
    const uint32_t hi = (uint32_t)((v >> 1) >> (63u - sh));  // bits 64 - sh .. of v (none for sh = 0)
    __hip_atomic_fetch_or(w + i, (uint32_t)lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(w + i + 1, (uint32_t)(lo >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(w + i + 2, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    pos += n;
  }
  __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
};

// The same appends straight into a global stream (atomicOr), clipped at the block's end: the fallback for a tile
// whose bits do not fit its LDS window. Only nonzero words are touched (nothing past the clipped code).
struct GlobalOrWriter {
  uint32_t* w;
  uint64_t pos, limit;
  __device__ __forceinline__ void put(uint64_t v, uint32_t n)
  {
    if (pos >= limit || n == 0) {
      pos += n;
      return;
    }
    if (n > limit - pos) v &= lowmask64((uint32_t)(limit - pos));
    const uint64_t i = pos >> 5;
    const uint32_t sh = (uint32_t)(pos & 31u);
    const uint64_t lo = v << sh;
    const uint32_t hi = (uint32_t)((v >> 1) >> (63u - sh));
    if ((uint32_t)lo) atomicOr(w + i, (uint32_t)lo);
    if ((uint32_t)(lo >> 32)) atomicOr(w + i + 1, (uint32_t)(lo >> 32));
    if (hi) atomicOr(w + i + 2, hi);
    pos += n;
  }
  __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
};

__device__ __forceinline__ uint32_t bfe8(uint32_t x, uint32_t o) { return (x >> o) & 255u; }

template <class W>
__device__ __forceinline__ void encode_plane64_dup(W& w, uint64_t P, uint32_t& bits, uint32_t& n, const uint32_t* dup)
{
  const bool full = n >= 64;
  const uint64_t r = full ? 0ull : P >> (n & 63u);
  const uint64_t V = full ? P : ((P & lowmask64(n)) | ((uint64_t)(r != 0) << n));
  const uint32_t vn = full ? 64u : n + 1u;
  w.put(V, vn);
  bits += vn;
  if (r != 0) {
    const uint32_t rl = (uint32_t)r, rh = (uint32_t)(r >> 32);
    const uint32_t hb = rh ? 63u - (uint32_t)__builtin_clz(rh) : 31u - (uint32_t)__builtin_clz(rl);
    const uint32_t m = (uint32_t)__builtin_popcount(rl) + (uint32_t)__builtin_popcount(rh);
    // E(r_lo): chunk c of r starts at 8c + popcount(r[0 .. 8c-1]) <= 48, so four 16-bit codes fit in 64 bits
    uint64_t E0 = dup[rl & 255u];
    uint32_t off = 8u + (uint32_t)__builtin_popcount(rl & 255u);
#pragma unroll
    for (uint32_t c = 1; c < 4; c++) {
      if (!__any(hb >= 8 * c)) break;
      const uint32_t v = bfe8(rl, 8 * c);
      E0 |= (uint64_t)dup[v] << off;
      off += 8u + (uint32_t)__builtin_popcount(v);
    }
    const uint32_t nout = n + hb + 1u;
    const uint32_t keep = hb + m - (nout >= 64 ? 1u : 0u);  // bits of E(r) written
    const uint32_t glen = keep + (nout < 64 ? 1u : 0u);     // and the closing '0'
    uint64_t E1 = 0;
    if (__any(hb >= 32)) {  // E(r_hi) after E(r_lo) (off = 32 + popcount(r_lo) there)
      uint64_t Eh = dup[rh & 255u];
      uint32_t oh = 8u + (uint32_t)__builtin_popcount(rh & 255u);
#pragma unroll
      for (uint32_t c = 1; c < 4; c++) {
        if (!__any(hb >= 32 + 8 * c)) break;
        const uint32_t v = bfe8(rh, 8 * c);
        Eh |= (uint64_t)dup[v] << oh;
        oh += 8u + (uint32_t)__builtin_popcount(v);
      }
      if (hb >= 32) {
        E0 |= off < 64 ? Eh << off : 0ull;
        E1 = (Eh >> 1) >> (63u - (off & 63u));  // off in 32 .. 64: bits of Eh past E0's 64
        E1 = off >= 64 ? Eh : E1;
      }
    }
    w.put(E0 & lowmask64(keep), glen < 64 ? glen : 64u);
    if (glen > 64) w.put(E1 & lowmask64(keep - 64u), glen - 64u);
    bits += glen;
    n = nout;
  }
}

template <int K, int KLO, class W>
__device__ __forceinline__ void encode_planes64_dup(W& w, const uint32_t* t, int kstart, int kmin, uint32_t budget,
                                                    uint32_t& bits, uint32_t& n, const uint32_t* dup)
{
  if constexpr (K >= KLO) {
    if (K < kmin || bits >= budget) return;
    if (K <= kstart) encode_plane64_dup(w, (uint64_t)t[K] | ((uint64_t)t[32 + K] << 32), bits, n, dup);
    encode_planes64_dup<K - 1, KLO>(w, t, kstart, kmin, budget, bits, n, dup);
  }
}

// encode_ints (encode.c:279-408) for 64 coefficients with the plane coder above: the planes above the highest
// one-bit (n = 0, r = 0: one '0' each) are appended as one run of zeros. u is transposed in place.
template <class W>
__device__ __forceinline__ uint32_t encode_ints64_dup(W& w, uint32_t* u, uint32_t budget, uint32_t maxprec,
                                                      const uint32_t* dup)
{
  const int kmin = maxprec < 32 ? 32 - (int)maxprec : 0;
  uint32_t any = 0;
#pragma unroll
  for (int i = 0; i < 64; i++) any |= u[i];
  // the planes are materialised stage by stage: left to itself the scheduler interleaves the two transposes and
  // sinks their last stages into the plane code, keeping their inputs live across it (208 VGPRs instead of ~100)
  asm volatile("" : "+v"(any));
  pin32(u);
  pin32(u + 32);
  // planes 16..31 first (the S = 16 stage, then the upper halves); the lower halves' stages only when some lane of
  // the wave codes a plane below 16 (a fixed-rate budget usually runs out above it)
  transpose32_stage<16, 0x0000FFFFu>(u);
  pin32(u);
  transpose32_stage<16, 0x0000FFFFu>(u + 32);
  pin32(u + 32);
  transpose_half_pinned(u + 16);
  transpose_half_pinned(u + 48);
  const int top = any ? 31 - (int)__builtin_clz(any) : -1;  // highest plane with a one-bit
  const int kstart = max(top, kmin - 1);
  uint32_t bits = min((uint32_t)(31 - kstart), budget);
  w.skip(bits);
  uint32_t n = 0;
  encode_planes64_dup<31, 16>(w, u, kstart, kmin, budget, bits, n, dup);
  if (__any(kmin <= 15 && bits < budget)) {
    transpose_half_pinned(u);
    transpose_half_pinned(u + 32);
    encode_planes64_dup<15, 0>(w, u, kstart, kmin, budget, bits, n, dup);
  }
  return bits < budget ? bits : budget;
}

__device__ __forceinline__ bool exceeded_maxbits(uint32_t maxbits, uint32_t maxprec, uint32_t size)
{
  return (maxprec + 1) * size - 1 > maxbits;  // common.c:232-236
}

// encode_fblock (encode.c:457-495) + encode_iblock (encode.c:412-455). Returns the block's bit count. With the
// E-table `dup` (DupTab in LDS), 64-coefficient blocks take the plane coder encode_ints64_dup.
template <int D, class W>
__device__ __forceinline__ uint32_t encode_block(W& w, const float* f, const Params& p, const uint32_t* dup = nullptr)
{
  constexpr int B = Dim<D>::B;
  float fa[B];
#pragma unroll
  for (int i = 0; i < B; i++) fa[i] = f[i];
  const int emax = block_emax<B>(fa);
  const uint32_t prec = precision(emax, p.maxprec, p.minexp, D);
  const uint32_t be = prec ? (uint32_t)(emax + 127) : 0u;
  if (!be) {  // single zero bit, then pad to minbits
    w.skip(1);
    uint32_t bits = 1;
    if (p.minbits > bits) {
      w.skip(p.minbits - bits);
      bits = p.minbits;
    }
    return bits;
  }
  w.put(2ull * be + 1ull, 9);
  int32_t q[B];
  const float s = cast_scale(emax);
#pragma unroll
  for (int i = 0; i < B; i++) q[i] = cast1(fa[i], s);
  fwd_xform<D>(q);
  uint32_t u[B];
  fwd_reorder<D>(u, q);
  const uint32_t maxb = p.maxbits - 9u;
  const uint32_t minb = p.minbits - (p.minbits < 9u ? p.minbits : 9u);
  const uint32_t budget = exceeded_maxbits(maxb, prec, B) ? maxb : 0xffffffffu;
  uint32_t bits;
  if constexpr (B == 64) bits = dup ? encode_ints64_dup(w, u, budget, prec, dup) : encode_ints<B>(w, u, budget, prec);
  else bits = encode_ints<B>(w, u, budget, prec);
  if (bits < minb) {
    w.skip(minb - bits);
    bits = minb;
  }
  return 9 + bits;
}

// Bit length of encode_ints' untruncated output from the coefficients' leading one-bit planes alone (B = 4^d). With
// L_j the leading plane of u_j (-1 for 0) and R_j = max_{i >= j} L_i, the prefix after plane k is
// n_k = #{j : R_j >= k}; plane k costs n_{k+1} verbatim bits plus, while n_{k+1} < B, one '0' if no coefficient turns
// significant, else m + (q == B-1 ? B-1 : q+2) - n_{k+1} (m new one-bits, the last at q; encode.c:279-339). Summed over
// planes kmin .. 31:
//   sum_j max(0, R_j - kmin) + 32 - max(kmin, L_{B-1}) + #{j : L_j = R_j >= kmin}
//   + sum_{j last at its level, R_j >= kmin} (j < B-1 ? j+1 : B-2) - sum_{j first at its level, R_j >= kmin} j.
template <int B>
__device__ __forceinline__ uint32_t encode_ints_length(const uint32_t* u, uint32_t maxprec)
{
  const int kmin = maxprec < 32 ? 32 - (int)maxprec : 0;
  if (kmin >= 32) return 0u;  // no plane is coded
  // Evaluated through the suffix ORs S_j = u_j | ... | u_{B-1}: R_j = 31 - ffbh(S_j), so with K = 31 - kmin and
  // z_j = ffbh(S_j) (all ones for S_j = 0): max(R_j, kmin) = 31 - min(z_j, K) (unsigned), R_j >= kmin <=> z_j <= K,
  // and L_j = R_j <=> u_j holds S_j's leading bit <=> (u_j ^ S_j) < u_j. sum_j max(0, R_j - kmin) = B K - sum min(z_j, K).
  // The last-/first-at-level sums cancel wherever both neighbours are >= kmin (R is non-increasing), leaving j + 1 at
  // the one j with R_j >= kmin > R_{j+1}: with c = #{j : R_j >= kmin} they add c, or B - 2 when c = B.
  const uint32_t K = (uint32_t)(31 - kmin);
  uint32_t S = u[B - 1];
  const uint32_t zl = min(ffbh_u32(S), K);  // 31 - max(kmin, L_{B-1})
  const bool onl = ffbh_u32(S) <= K;
  // len = 32 - max(kmin, L_{B-1}) + sum_j (max(R_j, kmin) - kmin) + #{j : L_j = R_j >= kmin} + (c or B - 2)
  uint32_t len = 1u + zl + (uint32_t)B * K - zl + (onl ? 1u : 0u);
  uint32_t c = onl ? 1u : 0u;
#pragma unroll
  for (int j = B - 2; j >= 0; j--) {
    S |= u[j];
    uint32_t z = ffbh_u32(S);
    asm volatile("" : "+v"(z));  // in order: hoisting all 64 leading-plane counts costs 64 VGPRs
    const bool on = z <= K;
    len -= min(z, K);
    len += (on && (u[j] ^ S) < u[j]) ? 1u : 0u;
    c += on ? 1u : 0u;
  }
  return len + (c == (uint32_t)B ? (uint32_t)B - 2u : c);
}

// encode_block's return value without coding: same header / cast / transform / reorder, then the closed-form length
// clipped to the budget and padded to minbits.
template <int D>
__device__ __forceinline__ uint32_t count_block(const float* f, const Params& p)
{
  constexpr int B = Dim<D>::B;
  float fa[B];
#pragma unroll
  for (int i = 0; i < B; i++) fa[i] = f[i];
  int emax = 0;
  int32_t q[B];
  bool fast = false;
  if constexpr (B == 64) fast = emax_cast_finite<B>(fa, emax, q);
  if (!fast) emax = block_emax<B>(fa);
  const uint32_t prec = precision(emax, p.maxprec, p.minexp, D);
  const uint32_t be = prec ? (uint32_t)(emax + 127) : 0u;
  if (!be) return p.minbits > 1u ? p.minbits : 1u;
  if (!fast) {
    const float s = cast_scale(emax);
#pragma unroll
    for (int i = 0; i < B; i++) q[i] = cast1(fa[i], s);
  }
  fwd_xform<D>(q);
  uint32_t u[B];
  fwd_reorder<D>(u, q);
  const uint32_t maxb = p.maxbits - 9u;
  const uint32_t minb = p.minbits - (p.minbits < 9u ? p.minbits : 9u);
  const uint32_t budget = exceeded_maxbits(maxb, prec, B) ? maxb : 0xffffffffu;
  uint32_t bits = encode_ints_length<B>(u, prec);
  bits = bits < budget ? bits : budget;
  return 9 + (bits < minb ? minb : bits);
}

// encode_fblock split in three for the two-pass tile encoder, which needs a block's length before it can place the
// block: prepare (header fields; cast, transform and reorder into u), length (count_block's value), code (the
// bits, encode_block's value). The coefficients are derived once instead of once per pass.
struct BlockHead {
  uint32_t be;      // biased exponent, 0 = empty block (a single '0' bit)
  uint32_t prec;    // get_precision
  uint32_t budget;  // encode_ints' bit budget (maxbits - 9, or unlimited)
  uint32_t minb;    // pad target after the header
};

template <int D>
__device__ __forceinline__ BlockHead prepare_block(const float* f, const Params& p, uint32_t* u)
{
  constexpr int B = Dim<D>::B;
  float fa[B];
#pragma unroll
  for (int i = 0; i < B; i++) fa[i] = f[i];
  int emax = 0;
  int32_t q[B];
  bool fast = false;
  if constexpr (B == 64) fast = emax_cast_finite<B>(fa, emax, q);
  if (!fast) {
    emax = block_emax<B>(fa);
    const float s = cast_scale(emax);
#pragma unroll
    for (int i = 0; i < B; i++) q[i] = cast1(fa[i], s);
  }
  BlockHead h;
  h.prec = precision(emax, p.maxprec, p.minexp, D);
  h.be = h.prec ? (uint32_t)(emax + 127) : 0u;
  fwd_xform<D>(q);
  fwd_reorder<D>(u, q);
  const uint32_t maxb = p.maxbits - 9u;
  h.minb = p.minbits - (p.minbits < 9u ? p.minbits : 9u);
  h.budget = exceeded_maxbits(maxb, h.prec, B) ? maxb : 0xffffffffu;
  return h;
}

template <int B>
__device__ __forceinline__ uint32_t block_length(const BlockHead& h, const uint32_t* u, const Params& p)
{
  if (!h.be) return p.minbits > 1u ? p.minbits : 1u;
  uint32_t bits = encode_ints_length<B>(u, h.prec);
  bits = bits < h.budget ? bits : h.budget;
  return 9 + (bits < h.minb ? h.minb : bits);
}

template <int D, class W>
__device__ __forceinline__ uint32_t code_block(W& w, const BlockHead& h, uint32_t* u, const Params& p,
                                               const uint32_t* dup = nullptr)
{
  constexpr int B = Dim<D>::B;
  if (!h.be) {
    const uint32_t n = p.minbits > 1u ? p.minbits : 1u;  // a '0', padded with zeros to minbits
    w.skip(n);
    return n;
  }
  w.put(2ull * h.be + 1ull, 9);
  uint32_t bits;
  if constexpr (B == 64) bits = dup ? encode_ints64_dup(w, u, h.budget, h.prec, dup) : encode_ints<B>(w, u, h.budget, h.prec);
  else bits = encode_ints<B>(w, u, h.budget, h.prec);
  return 9 + (bits < h.minb ? h.minb : bits);
}

// ------------------------------------------------------------------------------------------------ reader / decoder
struct BitReader {
  const uint64_t* w;
  uint64_t pos;
  __device__ __forceinline__ uint64_t peek64() const
  {
    uint64_t i = pos >> 6;
    uint32_t sh = (uint32_t)(pos & 63);
    uint64_t v = w[i] >> sh;
    if (sh) v |= w[i + 1] << (64 - sh);
    return v;
  }
  __device__ __forceinline__ uint64_t get(uint32_t n)
  {
    if (!n) return 0;
    uint64_t v = peek64() & lowmask64(n);
    pos += n;
    return v;
  }
  __device__ __forceinline__ uint32_t bit()
  {
    uint32_t b = (uint32_t)(w[pos >> 6] >> (pos & 63)) & 1u;
    pos++;
    return b;
  }
  __device__ __forceinline__ void skip(uint64_t k) { pos += k; }
};

// Reader over 32-bit words staged in LDS (two zero pad words after the last one read): a 32-bit position (a staged
// span is at most 2^16 words), and the 64-bit peek as two funnel shifts of three words (v_alignbit_b32).
struct WordBitReader {
  const uint32_t* w;
  uint32_t pos;
  __device__ __forceinline__ uint64_t peek64() const
  {
    const uint32_t i = pos >> 5, sh = pos & 31u;
    const uint32_t a = w[i], b = w[i + 1], c = w[i + 2];
    return (uint64_t)__builtin_amdgcn_alignbit(c, b, sh) << 32 | __builtin_amdgcn_alignbit(b, a, sh);
  }
  __device__ __forceinline__ uint64_t get(uint32_t n)  // n <= 64
  {
    if (!n) return 0;
    const uint32_t k = 64u - n;
    const uint64_t v = (peek64() << k) >> k;
    pos += n;
    return v;
  }
  __device__ __forceinline__ uint32_t bit()
  {
    uint32_t b = (w[pos >> 5] >> (pos & 31)) & 1u;
    pos++;
    return b;
  }
  __device__ __forceinline__ void skip(uint64_t k) { pos += (uint32_t)k; }
};


// decode_ints (libzfp 0.5.5; sw/src/decode.c:141-183 with block size 4^d). The unary scan of each group test
// (`for (; n < size - 1 && bits && (bits--, !read_bit()); n++)`) is done with one count-trailing-zeros of the next
// 64 stream bits instead of bit by bit.
// Zeros before the first one-bit among bits 1..63 of w, 63 when there is none (>= any scan limit): bits 1..63 as two
// funnel shifts with a sentinel one above them, then v_ffbl on each half (all ones for 0).
__device__ __forceinline__ uint32_t scan_zeros63(uint64_t w)
{
  const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
  const uint32_t slo = __builtin_amdgcn_alignbit(hi, lo, 1u), shi = __builtin_amdgcn_alignbit(1u, hi, 1u);
  uint32_t zl, zh;
  asm("v_ffbl_b32 %0, %1" : "=v"(zl) : "v"(slo));
  asm("v_ffbl_b32 %0, %1" : "=v"(zh) : "v"(shi));
  return min(zl, zh + 32u);
}

template <int B, class Rd>
__device__ __forceinline__ uint32_t decode_ints(Rd& r, uint32_t maxbits, uint32_t maxprec, uint32_t* u)
{
  const int kmin = maxprec < 32 ? 32 - (int)maxprec : 0;
  uint32_t bits = maxbits;
  uint32_t n = 0;
#pragma unroll
  for (int i = 0; i < B; i++) u[i] = 0;
  for (int k = 31; bits && k >= kmin; --k) {
    const uint32_t m = n < bits ? n : bits;
    bits -= m;
    uint64_t x = r.get(m);
    while (n < (uint32_t)B && bits) {
      // one peek per group test: bit 0 the test, bits 1..63 the unary scan after it
      const uint64_t w = r.peek64();
      bits--;
      if (!(w & 1u)) {  // negative group test
        r.skip(1);
        break;
      }
      const uint32_t lim = min((uint32_t)B - 1 - n, bits);  // zeros the scan may read
      const uint64_t s = w >> 1;
      const uint32_t z = s ? (uint32_t)__builtin_ctzll(s) : 64u;
      // zeros, then the one-bit; or the scan ran into the last coefficient or the budget: the one is implied
      const uint32_t adv = z < lim ? z + 1 : lim;
      r.skip(1 + adv);
      bits -= adv;
      n += min(z, lim);
      x += 1ull << n;
      n++;
    }
#pragma unroll
    for (int i = 0; i < B; i++) u[i] |= (uint32_t)((x >> i) & 1u) << k;
  }
  return maxbits - bits;
}

// decode_ints for 64 coefficients: plane k goes to t[k] (coefficients 0..31) / t[32 + k] (32..63) with a
// compile-time index, and one pair of 32 x 32 bit transposes at the end turns the planes into coefficients -- instead
// of depositing every plane's 64 bits into 64 coefficient words (three operations per coefficient per plane).
template <int K, class Rd>
__device__ __forceinline__ void decode_planes64(Rd& r, int kmin, uint32_t& bits, uint32_t& n, uint32_t* t)
{
  if constexpr (K >= 0) {
    uint64_t x = 0;
    if (bits && K >= kmin) {
      const uint32_t m = n < bits ? n : bits;
      bits -= m;
      x = r.get(m);
      while (n < 64u && bits) {
        // one peek per group test: bit 0 the test, bits 1..63 the unary scan after it
        const uint64_t w = r.peek64();
        bits--;
        if (!(w & 1u)) {  // negative group test
          r.skip(1);
          break;
        }
        const uint32_t lim = min(63u - n, bits);
        const uint32_t z = scan_zeros63(w);
        const uint32_t adv = z < lim ? z + 1 : lim;  // zeros + the one-bit, or up to the implied one
        r.skip(1 + adv);
        bits -= adv;
        n += min(z, lim);
        x += 1ull << n;
        n++;
      }
    }
    t[K] = (uint32_t)x;
    t[32 + K] = (uint32_t)(x >> 32);
    decode_planes64<K - 1>(r, kmin, bits, n, t);
  }
}

template <class Rd>
__device__ __forceinline__ uint32_t decode_ints64(Rd& r, uint32_t maxbits, uint32_t maxprec, uint32_t* u)
{
  const int kmin = maxprec < 32 ? 32 - (int)maxprec : 0;
  uint32_t bits = maxbits, n = 0;
  decode_planes64<31>(r, kmin, bits, n, u);
  transpose32(u);
  transpose32(u + 32);
  return maxbits - bits;
}

// dequantize (decode.c:12-25): ldexpf(1, emax - 30) exactly, including subnormal and zero scales.
__device__ __forceinline__ float dequant_scale(int emax)
{
  int e = emax - 30;
  if (e >= -126) return __uint_as_float((uint32_t)(e + 127) << 23);
  if (e >= -149) return __uint_as_float(1u << (e + 149));
  return 0.0f;
}

// decode_fblock (decode.c:220-253 with libzfp semantics). Writes B floats to f.
template <int D, class Rd>
__device__ __forceinline__ void decode_block(Rd& r, const Params& p, float* f)
{
  constexpr int B = Dim<D>::B;
  uint32_t bits = 1;
  if (r.bit()) {
    bits += 8;
    const int emax = (int)r.get(8) - 127;
    const uint32_t prec = precision(emax, p.maxprec, p.minexp, D);
    const uint32_t minb = p.minbits - (p.minbits < bits ? p.minbits : bits);
    const uint32_t maxb = p.maxbits - bits;
    uint32_t u[B];
    const uint32_t budget = exceeded_maxbits(maxb, prec, B) ? maxb : 0xffffffffu;
    uint32_t got;
    if constexpr (B == 64) got = decode_ints64(r, budget, prec, u);
    else got = decode_ints<B>(r, budget, prec, u);
    if (got < minb) r.skip(minb - got);
    int32_t q[B];
    inv_reorder<D>(q, u);
    inv_xform<D>(q);
    const float s = dequant_scale(emax);
#pragma unroll
    for (int i = 0; i < B; i++) f[i] = s * (float)q[i];
  } else {
#pragma unroll
    for (int i = 0; i < B; i++) f[i] = 0.0f;
    if (p.minbits > bits) r.skip(p.minbits - bits);
  }
}

}  // namespace gcow
