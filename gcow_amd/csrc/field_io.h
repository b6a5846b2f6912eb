// field_io.h -- block gather / scatter over a FieldDesc (strided fp32 / bf16 fields, partial blocks padded as
// sw/src/encode.c:41-126).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec_device.h"
#include "kernels.h"

namespace gcow {

// ------------------------------------------------------------------------------------------------ gather
__device__ __forceinline__ uint32_t pad_index(uint32_t i, uint32_t nv)
{
  // pad_partial_block fall-through (sw/src/encode.c:41-60): 1 -> v0 v0 v0 v0, 2 -> v0 v1 v1 v0, 3 -> v0 v1 v2 v0
  return nv >= 4 ? i : (nv == 1 ? 0u : (i == 3 ? 0u : (nv == 2 && i == 2 ? 1u : i)));
}

template <int DT>
__device__ __forceinline__ float load_elem(const void* base, int64_t off)
{
  if constexpr (DT == DT_BF16) {
    uint32_t h = ((const uint16_t*)base)[off];
    return __uint_as_float(h << 16);  // exact bf16 -> fp32 widening
  } else {
    return ((const float*)base)[off];
  }
}

// Load 4 consecutive values starting at element offset off (16-B aligned for f32, 8-B for bf16 when vec).
template <int DT>
__device__ __forceinline__ void load_row4(const void* base, int64_t off, float* f)
{
  if constexpr (DT == DT_BF16) {
    uint2 v = *(const uint2*)((const uint16_t*)base + off);
    f[0] = __uint_as_float(v.x << 16);
    f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16);
    f[3] = __uint_as_float(v.y & 0xffff0000u);
  } else {
    float4 v = *(const float4*)((const float*)base + off);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
}

// gather_2d_block / gather_partial_2d_block / gather_partial_4d_block (sw/src/encode.c:62-126), generic d.
template <int D, int DT>
__device__ __forceinline__ void gather_block(const FieldDesc& F, uint32_t b, float* f)
{
  uint32_t ix, iy = 0, iz = 0;
  if constexpr (D == 1) {
    ix = b;
  } else if constexpr (D == 2) {
    iy = b / F.bx;
    ix = b - iy * F.bx;
  } else {
    uint32_t r = b / F.bx;
    ix = b - r * F.bx;
    iz = r / F.by;
    iy = r - iz * F.by;
  }
  const uint64_t x0 = 4ull * ix, y0 = 4ull * iy, z0 = 4ull * iz;
  const uint32_t nvx = (uint32_t)min<uint64_t>(4, F.n[0] - x0);
  const uint32_t nvy = D > 1 ? (uint32_t)min<uint64_t>(4, F.n[1] - y0) : 1u;
  const uint32_t nvz = D > 2 ? (uint32_t)min<uint64_t>(4, F.n[2] - z0) : 1u;
  const int64_t base = (int64_t)x0 * F.s[0] + (int64_t)y0 * F.s[1] + (int64_t)z0 * F.s[2];
  const bool full = nvx == 4 && (D < 2 || nvy == 4) && (D < 3 || nvz == 4);
  if (full && F.vec) {
#pragma unroll
    for (int z = 0; z < (D > 2 ? 4 : 1); z++)
#pragma unroll
      for (int y = 0; y < (D > 1 ? 4 : 1); y++)
        load_row4<DT>(F.data, base + (int64_t)y * F.s[1] + (int64_t)z * F.s[2], f + 16 * z + 4 * y);
  } else {
#pragma unroll
    for (int z = 0; z < (D > 2 ? 4 : 1); z++) {
#pragma unroll
      for (int y = 0; y < (D > 1 ? 4 : 1); y++)
#pragma unroll
        for (int x = 0; x < 4; x++) {
          int64_t off = (int64_t)pad_index(x, nvx) * F.s[0];
          if (D > 1) off += (int64_t)pad_index(y, nvy) * F.s[1];
          if (D > 2) off += (int64_t)pad_index(z, nvz) * F.s[2];
          f[16 * z + 4 * y + x] = load_elem<DT>(F.data, base + off);
        }
      // one z-slice of loads in flight at a time: hoisting all 64 addresses (64-bit each) would cost 128 VGPRs
      if constexpr (D > 2)
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("" : "+v"(f[16 * z + i]));
    }
  }
}

// scatter_2d_block / scatter_partial_2d_block (sw/src/decode.c:27-42), generic d, fp32 output.
template <int D>
__device__ __forceinline__ void scatter_block(const FieldDesc& F, uint32_t b, const float* f)
{
  uint32_t ix, iy = 0, iz = 0;
  if constexpr (D == 1) {
    ix = b;
  } else if constexpr (D == 2) {
    iy = b / F.bx;
    ix = b - iy * F.bx;
  } else {
    uint32_t r = b / F.bx;
    ix = b - r * F.bx;
    iz = r / F.by;
    iy = r - iz * F.by;
  }
  const uint64_t x0 = 4ull * ix, y0 = 4ull * iy, z0 = 4ull * iz;
  const uint32_t nvx = (uint32_t)min<uint64_t>(4, F.n[0] - x0);
  const uint32_t nvy = D > 1 ? (uint32_t)min<uint64_t>(4, F.n[1] - y0) : 1u;
  const uint32_t nvz = D > 2 ? (uint32_t)min<uint64_t>(4, F.n[2] - z0) : 1u;
  float* out = (float*)F.data;
  const int64_t base = (int64_t)x0 * F.s[0] + (int64_t)y0 * F.s[1] + (int64_t)z0 * F.s[2];
  const bool full = nvx == 4 && (D < 2 || nvy == 4) && (D < 3 || nvz == 4);
  if (full && F.vec) {
#pragma unroll
    for (int z = 0; z < (D > 2 ? 4 : 1); z++)
#pragma unroll
      for (int y = 0; y < (D > 1 ? 4 : 1); y++) {
        const float* g = f + 16 * z + 4 * y;
        *(float4*)(out + base + (int64_t)y * F.s[1] + (int64_t)z * F.s[2]) = make_float4(g[0], g[1], g[2], g[3]);
      }
  } else {
    // static trip counts with guards: a dynamically indexed f[] would live in scratch
#pragma unroll
    for (uint32_t z = 0; z < (D > 2 ? 4u : 1u); z++)
#pragma unroll
      for (uint32_t y = 0; y < (D > 1 ? 4u : 1u); y++)
#pragma unroll
        for (uint32_t x = 0; x < 4u; x++)
          if (x < nvx && y < nvy && z < nvz)
            out[base + (int64_t)x * F.s[0] + (int64_t)y * F.s[1] + (int64_t)z * F.s[2]] = f[16 * z + 4 * y + x];
  }
}

// fp32 -> bf16 bits, rounded to nearest even (torch's conversion; NaN -> 0x7fc0)
__device__ __forceinline__ uint32_t bf16_rne(float x)
{
  const uint32_t u = __float_as_uint(x);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// two values packed, lo in bits 0..15: gfx950's v_cvt_pk_bf16_f32 (round to nearest even, the default mode)
__device__ __forceinline__ uint32_t bf16x2_rne(float lo, float hi)
{
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// One 1-D block of decoded values into the output field: fp32 (scatter_block), or bf16 (F.dtype == DT_BF16: each
// value rounded to nearest even; one 8-byte store for a full block of a contiguous, 8-byte aligned field).
__device__ __forceinline__ void store_block1d(const FieldDesc& F, uint64_t b, const float* v)
{
  if (F.dtype != DT_BF16) {
    scatter_block<1>(F, (uint32_t)b, v);
    return;
  }
  const uint64_t x0 = 4ull * b;
  const uint32_t nv = (uint32_t)min<uint64_t>(4, F.n[0] - x0);
  uint16_t* out = (uint16_t*)F.data;
  if (nv == 4 && F.vec) {
    *(uint2*)(out + x0) = make_uint2(bf16x2_rne(v[0], v[1]), bf16x2_rne(v[2], v[3]));
  } else {
#pragma unroll
    for (uint32_t x = 0; x < 4u; x++)
      if (x < nv) out[(int64_t)(x0 + x) * F.s[0]] = (uint16_t)bf16_rne(v[x]);
  }
}

}  // namespace gcow
