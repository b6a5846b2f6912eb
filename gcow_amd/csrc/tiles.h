// tiles.h -- the range/tile kernels shared by the 1-D and the 2-D / 3-D translation units: pass 1 (k_count),
// pass 2 / generic fixed rate (k_encode_tiles) and the workgroup exclusive scan they use.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field_io.h"

namespace gcow {

// ------------------------------------------------------------------------------------------------ tiles
#ifndef GCOW_DPP_SCAN
#define GCOW_DPP_SCAN 1
#endif
// Inclusive wave prefix sum through DPP moves (no LDS round trip per step, as __shfl_up's ds_bpermute takes): sums
// within rows of 16 lanes by row_shr 1, 2, 4, 8 (lanes shifted in from outside the row read 0), then row 15's total
// into rows 1 and 3 (row_bcast:15) and lane 31's into rows 2 and 3 (row_bcast:31).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x)
{
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Sum over the wave (wave-uniform), through the DPP prefix sum
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t x)
{
#if GCOW_DPP_SCAN
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_dpp(x), 63);
#else
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
#endif
}

// Exclusive prefix sum over the workgroup. GUARD: a trailing barrier so that `sh` can be reused at once; a caller
// that passes a barrier of its own before the next use of `sh` drops it.
template <uint32_t T, bool GUARD = true>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* total, uint32_t* sh)
{
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  uint32_t x = v;
#if GCOW_DPP_SCAN
  x = wave_incl_scan_dpp(x);
#else
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
#endif
  if (T > 64) {
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < T / 64; w++) {
      uint32_t s = sh[w];
      off += w < wid ? s : 0u;
      tot += s;
    }
    if (GUARD || !GCOW_DPP_SCAN) __syncthreads();
    *total = tot;
    return off + x - v;
  } else {
    *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    return x - v;
  }
}

// Pass 1: sum of block bit lengths per contiguous range of `range` blocks.
template <int D, int DT, uint32_t T>
__global__ __launch_bounds__(T) void k_count(FieldDesc F, Params p, uint32_t range, uint64_t* __restrict__ sums)
{
  constexpr int B = Dim<D>::B;
  __shared__ uint64_t red[T / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * range;
  const uint64_t b1 = min<uint64_t>(b0 + range, F.nblocks);
  uint64_t acc = 0;
  for (uint64_t b = b0 + threadIdx.x; b < b1; b += T) {
    float f[B];
    gather_block<D, DT>(F, (uint32_t)b, f);
    acc += count_block<D>(f, p);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
    for (uint32_t i = 0; i < T / 64; i++) s += red[i];
    sums[blockIdx.x] = s;
  }
}

// Pass 2 / generic fixed rate: each workgroup encodes blocks [range*wg, range*(wg+1)) tile by tile.
template <int D, int DT, uint32_t T, bool FIXED>
__global__ __launch_bounds__(T) void k_encode_tiles(FieldDesc F, Params p, uint32_t range,
                                                    const uint64_t* __restrict__ rbase, uint32_t* __restrict__ out32,
                                                    uint64_t* __restrict__ index, uint32_t index_shift)
{
  constexpr int B = Dim<D>::B;
  extern __shared__ uint32_t lds[];
  __shared__ uint32_t scan_sh[T / 64 > 0 ? T / 64 : 1];
  __shared__ __attribute__((aligned(16))) uint32_t dup[B == 64 ? 256 : 4];  // E table of the 64-coefficient plane coder
  const uint32_t tid = threadIdx.x;
  if constexpr (B == 64) {
    stage_table<T, 256>(dup, g_dup_tab.v);
    __syncthreads();
  }
  const uint64_t b0 = (uint64_t)blockIdx.x * range;
  const uint64_t b1 = min<uint64_t>(b0 + range, F.nblocks);
  const bool final_range = b1 == F.nblocks;
  uint64_t base = FIXED ? b0 * p.maxbits : rbase[blockIdx.x];
  const uint64_t first_word = base >> 5;
  const bool first_shared = (base & 31) != 0;
  uint32_t carry = 0;
  for (uint64_t t0 = b0; t0 < b1; t0 += T) {
    const uint64_t b = t0 + tid;
    const bool valid = b < b1;
    uint32_t u[B];
    BlockHead h{};
    uint32_t len = 0;
    if (valid) {
      float f[B];
      gather_block<D, DT>(F, (uint32_t)b, f);
      h = prepare_block<D>(f, p, u);
      len = FIXED ? p.maxbits : block_length<B>(h, u, p);
    }
    uint32_t tile_total;
    const uint32_t excl = block_exclusive_scan<T>(len, &tile_total, scan_sh);
    const uint32_t lbase = (uint32_t)(base & 31);
    const uint32_t end_local = lbase + tile_total;
    const uint32_t W = (end_local + 31) >> 5;
    for (uint32_t j = tid; j < W; j += T) lds[j] = (j == 0) ? carry : 0u;
    __syncthreads();
    if (valid) {
      LdsWriter w{lds, lbase + excl, lbase + excl + len};
      code_block<D>(w, h, u, p, B == 64 ? dup : nullptr);
      if (index && ((b & ((1ull << index_shift) - 1)) == 0)) index[b >> index_shift] = base + excl;
    }
    __syncthreads();
    const bool last_tile = t0 + T >= b1;
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
      // stream_flush: zero-pad to a 64-bit boundary
      const uint64_t endw = (base + tile_total + 31) >> 5;
      if (endw & 1) out32[endw] = 0u;
    }
    carry = (!last_tile && partial) ? lds[end_local >> 5] : 0u;
    base += tile_total;
    __syncthreads();
  }
}


}  // namespace gcow
