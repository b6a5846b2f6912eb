// lean1d.h -- pieces of the 1-D closed-form coder shared by the fixed-rate kernels (gcow_kernels.hip) and the
// single-pass variable-rate encoder (var1d.hip): the plane / plane-pair code tables, the all-INT_MIN ("tiny")
// payload, the byte-indexed spread tables that build the 16-plane window, and opaque v_cvt / v_ffbh wrappers.
// Embedded coder semantics: sw/src/encode.c:279-339 (4-value blocks).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gcow {

// Plane-code table for 4-value blocks: entry (n, x) = verbatim n bits of plane x followed by the group-test code of
// its remainder (encode.c:301-333), packed as code[0:7) | len[7:10) | n'[10:13).
__device__ __forceinline__ uint16_t plane_entry4(uint32_t t)
{
  uint32_t n = t >> 4, x = t & 15u;
  if (n >= 4) return (uint16_t)(x | (4u << 7) | (4u << 10));
  uint32_t code = x & ((1u << n) - 1u), len = n;
  uint32_t r = x >> n;
  while (n < 4) {
    if (!r) { len += 1; break; }
    uint32_t tz = __builtin_ctz(r);
    if (n + tz < 3) {
      code |= (1u | (2u << tz)) << len;
      len += tz + 2;
      n += tz + 1;
      r >>= tz + 1;
    } else {
      code |= 1u << len;
      len += 1 + (3 - n);
      n = 4;
    }
  }
  return (uint16_t)(code | (len << 7) | (n << 10));
}

// Compile-time plane-pair table (two plane codes per entry), copied to LDS by each workgroup.
struct alignas(16) PlaneTab2 {
  uint32_t v[1280];
};

__host__ __device__ constexpr uint32_t plane_entry4_cx(uint32_t t)
{
  uint32_t n = t >> 4, x = t & 15u;
  if (n >= 4) return x | (4u << 7) | (4u << 10);
  uint32_t code = x & ((1u << n) - 1u), len = n;
  uint32_t r = x >> n;
  while (n < 4) {
    if (!r) {
      len += 1;
      break;
    }
    uint32_t tz = 0;
    while (!((r >> tz) & 1u)) tz++;
    if (n + tz < 3) {
      code |= (1u | (2u << tz)) << len;
      len += tz + 2;
      n += tz + 1;
      r >>= tz + 1;
    } else {
      code |= 1u << len;
      len += 1 + (3 - n);
      n = 4;
    }
  }
  return code | (len << 7) | (n << 10);
}


// ---- lean-5: the pair table re-packed so a lookup chains into the next with one and-or, a 32-bit group-code
// accumulator for the first two pairs, and the all-INT_MIN ("tiny") block as a compile-time constant.
// Entry: n' << 10 (= the next row's byte offset) | len << 13 | code << 17 (two 7-bit codes, len <= 14).
__host__ __device__ constexpr PlaneTab2 make_plane_tab5()
{
  PlaneTab2 T{};
  for (uint32_t t = 0; t < 1280; t++) {
    const uint32_t n = t >> 8, b = t & 255u;
    const uint32_t e1 = plane_entry4_cx((n << 4) | (b & 15u));
    const uint32_t c1 = e1 & 127u, l1 = (e1 >> 7) & 7u, n1 = e1 >> 10;
    const uint32_t e2 = plane_entry4_cx((n1 << 4) | (b >> 4));
    const uint32_t c2 = e2 & 127u, l2 = (e2 >> 7) & 7u, n2 = e2 >> 10;
    T.v[t] = (n2 << 10) | ((l1 + l2) << 13) | ((c1 | (c2 << l1)) << 17);
  }
  return T;
}

__device__ const PlaneTab2 g_plane_tab5 = make_plane_tab5();

// Embedded coder of one 4-coefficient block with kmin = 0 (encode.c:279-339 restated for compile-time use): the
// first `budget` payload bits, LSB-first.
__host__ __device__ constexpr uint64_t code4_cx(const uint32_t* u, int budget)
{
  uint64_t acc = 0;
  int pos = 0, bits = budget;
  uint32_t n = 0;
  for (int k = 31; k >= 0 && bits > 0; --k) {
    uint32_t x = 0;
    for (int i = 0; i < 4; i++) x |= ((u[i] >> k) & 1u) << i;
    const int m = (int)n < bits ? (int)n : bits;
    acc |= (uint64_t)(x & ((1u << m) - 1u)) << pos;
    pos += m;
    x >>= m;
    bits -= m;
    while (bits > 0 && n < 4) {
      bits--;
      const uint32_t t = x != 0;
      acc |= (uint64_t)t << pos++;
      if (!t) break;
      while (bits > 0 && n < 3) {
        bits--;
        const uint32_t b = x & 1u;
        acc |= (uint64_t)b << pos++;
        if (b) break;
        x >>= 1;
        n++;
      }
      x >>= 1;
      n++;
    }
  }
  return acc;
}

// Payload of a block whose every value casts to INT_MIN (scale 2^(30-e) = +inf, e <= -98; x86 cvttss2si,
// encode.c:162-187): the lift (encode.c:212-225) and negabinary map (encode.c:263-275) of four INT_MIN.
__host__ __device__ constexpr uint64_t tiny_payload_cx(int budget)
{
  auto asr = [](uint32_t v) { return (v >> 1) | (v & 0x80000000u); };
  uint32_t x = 0x80000000u, y = x, z = x, w = x;
  x += w; x = asr(x); w -= x;
  z += y; z = asr(z); y -= z;
  x += z; x = asr(x); z -= x;
  w += y; w = asr(w); y -= w;
  w += asr(y); y -= asr(w);
  uint32_t u[4] = {(x + 0xaaaaaaaau) ^ 0xaaaaaaaau, (y + 0xaaaaaaaau) ^ 0xaaaaaaaau, (z + 0xaaaaaaaau) ^ 0xaaaaaaaau,
                   (w + 0xaaaaaaaau) ^ 0xaaaaaaaau};
  return code4_cx(u, budget);
}

// v_cvt_i32_f32 as an opaque instruction: saturating, NaN -> 0, never poison (lanes whose cast is out of range are
// the tiny / special ones, whose result is replaced).
__device__ __forceinline__ int32_t cvt_i32_hw(float x)
{
  int32_t r;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// v_ffbh_u32 as an opaque instruction: count of leading zeros, all ones (not UB) for 0
__device__ __forceinline__ uint32_t ffbh_hw(uint32_t x)
{
  uint32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// Pair-table lookup chained on the previous entry's row (n' << 10 is already a byte offset).
__device__ __forceinline__ uint32_t tab5_next(const uint32_t* tab, uint32_t e, uint32_t byte)
{
  return *(const uint32_t*)((const char*)tab + ((e & 0x1c00u) | (byte << 2)));
}

// ---- lean-6: the 16-plane window from byte-indexed LDS tables instead of a shift/mask transpose.
// With w_i = u_i << (31 - M0) (plane M0 at bit 31, planes below bit 0 shifted in as zeros), window nibble j holds bit
// 31 - j of w_0..w_3: nibbles 0..7 come from the top bytes, 8..15 from the next bytes. Table i spreads byte b reversed
// onto nibble bit i (bit k of b -> bit 4 (7 - k) + i), so each half-window is four lookups OR-ed together: 8 LDS reads
// and 14 VALU per block where plane_window's bit reversals and four 64-bit delta swaps took ~45.
struct SpreadTab {
  uint32_t v[4 * 256];
};

__host__ __device__ constexpr SpreadTab make_rspread()
{
  SpreadTab T{};
  for (uint32_t i = 0; i < 4; i++)
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t r = 0;
      for (uint32_t k = 0; k < 8; k++)
        if ((b >> k) & 1u) r |= 1u << (4 * (7 - k) + i);
      T.v[256 * i + b] = r;
    }
  return T;
}

__device__ const SpreadTab g_rspread = make_rspread();

// entry t of the spread tables computed in a kernel prologue (no table load): byte t & 255 onto nibble bit t >> 8
__device__ __forceinline__ uint32_t rspread_entry(uint32_t t)
{
  uint32_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; k++) v |= ((t >> k) & 1u) << (4 * (7 - k));
  return v << (t >> 8);
}


// 16 planes from plane 31 of w (already shifted so the window's top plane is bit 31) down, as nibbles
__device__ __forceinline__ uint64_t window_lds(const uint32_t* rs, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3)
{
  const uint32_t lo = rs[w0 >> 24] | rs[256 + (w1 >> 24)] | rs[512 + (w2 >> 24)] | rs[768 + (w3 >> 24)];
  const uint32_t hi = rs[(w0 >> 16) & 255u] | rs[256 + ((w1 >> 16) & 255u)] | rs[512 + ((w2 >> 16) & 255u)] |
                      rs[768 + ((w3 >> 16) & 255u)];
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// planes 16..31 below the top of w (bytes 1 and 0 of the same shifted words): the second window
__device__ __forceinline__ uint64_t window_lds_low(const uint32_t* rs, uint32_t w0, uint32_t w1, uint32_t w2,
                                                   uint32_t w3)
{
  const uint32_t lo = rs[(w0 >> 8) & 255u] | rs[256 + ((w1 >> 8) & 255u)] | rs[512 + ((w2 >> 8) & 255u)] |
                      rs[768 + ((w3 >> 8) & 255u)];
  const uint32_t hi = rs[w0 & 255u] | rs[256 + (w1 & 255u)] | rs[512 + (w2 & 255u)] | rs[768 + (w3 & 255u)];
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

}  // namespace gcow
