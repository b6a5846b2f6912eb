// gcow_blocks.hip -- the 2-D / 3-D block kernels (one block per lane): tiles encoder instantiations, fixed-rate 3-D
// encoder / decoder, the generic and LDS-staged decoders, and their launchers. A translation unit of its own so the
// heavy 64-coefficient instantiations compile in parallel with gcow_kernels.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "codec_device.h"
#include "kernels.h"
#include "tiles.h"

namespace gcow {

// Slack words after a 3-D fixed-rate block's budget in k_encode3d_fixed: a plane that starts inside the budget
// appends at most 1 + 64 verbatim/flag bits and 129 group bits (encode_plane64_dup) -- 194 bits, 7 words from any
// bit offset -- before the budget check stops the lane.
constexpr uint32_t E3_SLACK = 8;

// occupancy bounds of the 3-D fixed-rate kernels (waves per SIMD; A/B knobs, the defaults are the measured best)
#ifndef GCOW_E3F_WAVES
#define GCOW_E3F_WAVES 4
#endif
#ifndef GCOW_D3F_WAVES
#define GCOW_D3F_WAVES 6
#endif


// ------------------------------------------------------------------------------------------------ 3-D fixed rate
// Fixed-rate 3-D blocks whose budget is a whole number of 32-bit words (maxbits = 32 WPB; rates 1, 2, 4, 8, 16, 32):
// one block per lane, 256 consecutive blocks per workgroup. The lane codes its block (generic 64-coefficient coder,
// encode.c:457-495 with libzfp's 3-D transform and perm_3) into its own LDS words through LaneWordWriter -- whole
// words, no atomics -- and the workgroup then stores its 256 WPB contiguous stream words coalesced.
// Held to 128 VGPRs (4 waves per SIMD; 22 VGPRs spill): C3 rate 8 0.225 -> 0.211 ms. The same bound on the tile
// kernels spills in their hot loop (C3 accuracy 1e-3: 0.591 -> 0.829 ms), so they are left alone
// (profiles/r02_c3_occupancy_ab.log).
template <int DT, uint32_t WPB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GCOW_E3F_WAVES, 8))) void k_encode3d_fixed(FieldDesc F, Params p, uint32_t* __restrict__ out32)
{
  constexpr uint32_t STRIDE = WPB + E3_SLACK + 1;  // odd: lanes' words spread over the banks
  extern __shared__ uint32_t lds_w[];               // 256 x STRIDE words, then the E table
  uint32_t* dup = lds_w + 256 * STRIDE;
  const uint32_t tid = threadIdx.x;
  const uint32_t b0 = blockIdx.x * 256u;
  const uint32_t nvalid = min(256u, F.nblocks - b0);
  // the block's values requested with the E table, before the barrier
  float f[64];
  if (tid < nvalid) gather_block<3, DT>(F, b0 + tid, f);
  dup[tid] = g_dup_tab.v[tid];
  for (uint32_t j = tid; j < 64 * STRIDE; j += 256) ((uint4*)lds_w)[j] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  if (tid < nvalid) {
    OrWriter w{lds_w + tid * STRIDE, 0u};
    encode_block<3>(w, f, p, dup);
  }
  __syncthreads();
  uint32_t* dst = out32 + (uint64_t)b0 * WPB;
  bool wide = false;
  if constexpr (WPB >= 4) {
    wide = (((uintptr_t)out32) & 15u) == 0;
    if (wide) {
      // four stream words per thread and step: one 16-byte store (the rows' odd stride leaves four 4-byte LDS reads)
      constexpr uint32_t Q = WPB / 4;
      for (uint32_t j4 = tid; j4 < nvalid * Q; j4 += 256) {
        const uint32_t* row = lds_w + (j4 / Q) * STRIDE + 4u * (j4 % Q);
        ((uint4*)dst)[j4] = make_uint4(row[0], row[1], row[2], row[3]);
      }
    }
  }
  if (!wide)
    for (uint32_t j = tid; j < nvalid * WPB; j += 256) dst[j] = lds_w[(j / WPB) * STRIDE + (j % WPB)];
  if (blockIdx.x == gridDim.x - 1 && tid == 0 && (((uint64_t)F.nblocks * WPB) & 1))
    out32[(uint64_t)F.nblocks * WPB] = 0u;  // stream_flush: zero-pad to a 64-bit boundary
}

// ------------------------------------------------------------------------------------------------ 3-D variable rate
// Two passes over tiles of 64 blocks, one tile (one wave) per workgroup and no loop inside: a loop over tiles keeps
// loop-carried state next to the 64 coefficients (152-179 VGPRs against 113 for one block), one tile per workgroup
// does not, and 32 Ki workgroups for a 512^3 field still fill the chip.
//   k_count3d   block lengths (closed form, codec_device.h block_length) summed per tile -> sums[tile]
//   k_scan_ranges (gcow_kernels.hip) turns the sums into tile bit offsets and zeroes the words two tiles share
//   k_encode3d_var  re-derives the coefficients (the lengths come from k_count3d through the workspace), a wave
//                   prefix sum places each block in an LDS window
//                   of the tile, the plane coder ORs the block's bits in, and the window is stored coalesced (the two
//                   edge words shared with the neighbouring tiles by atomicOr).
// MASK: some block may hit the bit budget (exceeded_maxbits for maxprec), so writes are clipped at the block's end
// (LdsWriter); otherwise every block writes exactly its length and the unclipped OrWriter is used.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane)
{
#if GCOW_DPP_SCAN
  (void)lane;
  return wave_incl_scan_dpp(x);
#else
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    x += lane >= (uint32_t)o ? y : 0u;
  }
  return x;
#endif
}

template <int DT>
__global__ __launch_bounds__(64) void k_count3d(FieldDesc F, Params p, uint64_t* __restrict__ sums,
                                                uint16_t* __restrict__ lens)
{
  const uint32_t b = blockIdx.x * 64u + threadIdx.x;
  uint32_t len = 0;
  if (b < F.nblocks) {
    float f[64];
    gather_block<3, DT>(F, b, f);
    uint32_t u[64];
    const BlockHead h = prepare_block<3>(f, p, u);
    len = block_length<64>(h, u, p);
    lens[b] = (uint16_t)len;  // <= 9 + 64 * 33 bits
  }
  len = wave_sum_dpp(len);
  if (threadIdx.x == 0) sums[blockIdx.x] = len;
}

// The LDS window holds a tile of up to E3V_WIN_WORDS - 2 words (64 blocks of 24 bits per value on average): sized
// for the worst case (64 x 2120 bits, 17 KB) it would cap the kernel at 9 workgroups per CU, i.e. 2.25 waves per
// SIMD. A tile that does not fit zeroes its interior stream words and codes straight into global memory.
constexpr uint32_t E3V_WIN_WORDS = 64 * 1536 / 32 + 2;

template <int DT, bool MASK>
__global__ __launch_bounds__(64) void k_encode3d_var(FieldDesc F, Params p, const uint64_t* __restrict__ rbase,
                                                     const uint16_t* __restrict__ lens, uint32_t* __restrict__ out32,
                                                     uint64_t* __restrict__ index, uint32_t index_shift, uint32_t win_words)
{
  extern __shared__ uint32_t win[];  // the tile's bits, plus 2 words for the writers' third word
  __shared__ uint32_t dup[256];
  const uint32_t lane = threadIdx.x;
#pragma unroll
  for (uint32_t t = 0; t < 4; t++) dup[lane + 64 * t] = g_dup_tab.v[lane + 64 * t];
  const uint32_t b = blockIdx.x * 64u + lane;
  const bool valid = b < F.nblocks;
  // placement first (lengths from the count pass), so the 64 coefficients are live only from gather to code
  const uint32_t len = valid ? lens[b] : 0u;
  const uint32_t incl = wave_incl_scan(len, lane);
  const uint32_t excl = incl - len, total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  const uint64_t base = rbase[blockIdx.x];
  const uint32_t lb = (uint32_t)(base & 31);
  const uint32_t W = (lb + total + 31) >> 5;
  const uint64_t gw0 = base >> 5;
  const bool last = blockIdx.x == gridDim.x - 1;
  const bool tail_shared = ((lb + total) & 31) != 0 && !last;
  if (W + 2 > win_words) {  // oversized tile (wave-uniform): code into the zeroed stream words directly
    for (uint32_t j = lane; j < W; j += 64)
      if (!((j == 0 && lb != 0) || (j == W - 1 && tail_shared))) out32[gw0 + j] = 0u;  // edges zeroed by the scan
    __threadfence();
    __syncthreads();
    if (valid) {
      uint32_t u[64];
      float f[64];
      gather_block<3, DT>(F, b, f);
      const BlockHead h = prepare_block<3>(f, p, u);
      GlobalOrWriter w{out32, base + excl, base + excl + len};
      code_block<3>(w, h, u, p, dup);
      if (index && (b & ((1u << index_shift) - 1)) == 0) index[b >> index_shift] = base + excl;
    }
    if (last && lane == 0) {
      const uint64_t endw = (base + total + 31) >> 5;
      if (endw & 1) out32[endw] = 0u;
    }
    return;
  }
  for (uint32_t j = lane; j < W + 2; j += 64) win[j] = 0u;
  __syncthreads();
  if (valid) {
    uint32_t u[64];
    BlockHead h;
    {
      float f[64];
      gather_block<3, DT>(F, b, f);
      h = prepare_block<3>(f, p, u);
    }
    if constexpr (MASK) {
      LdsWriter w{win, lb + excl, lb + excl + len};
      code_block<3>(w, h, u, p, dup);
    } else {
      OrWriter w{win, lb + excl};
      code_block<3>(w, h, u, p, dup);
    }
    if (index && (b & ((1u << index_shift) - 1)) == 0) index[b >> index_shift] = base + excl;
  }
  __syncthreads();
  for (uint32_t j = lane; j < W; j += 64) {
    const uint32_t v = win[j];
    if ((j == 0 && lb != 0) || (j == W - 1 && tail_shared)) atomicOr(out32 + gw0 + j, v);
    else out32[gw0 + j] = v;
  }
  if (last && lane == 0) {
    const uint64_t endw = (base + total + 31) >> 5;  // stream_flush: zero-pad to a 64-bit boundary
    if (endw & 1) out32[endw] = 0u;
  }
}

// The matching decoder: the workgroup stages its 256 blocks' stream words in LDS (coalesced), each lane decodes its
// block from LDS (libzfp decode semantics) and scatters it.
// Bounded to 6 waves per SIMD (101 -> 80 VGPRs, 30 spilled to scratch): the decoder is VALU-bound with divergent
// group-test loops, and the extra waves hide more of it than the spills cost (C3 rate 8 decode 0.337 -> 0.297 ms,
// tools/bench_configs.py c3).
template <uint32_t WPB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GCOW_D3F_WAVES, 8))) void k_decode3d_fixed(
    FieldDesc F, Params p, const uint32_t* __restrict__ in32)
{
  extern __shared__ uint32_t lds_w[];  // 256 x (WPB + 2) words: the block, then two zero pad words for peek64
  const uint32_t tid = threadIdx.x;
  const uint32_t b0 = blockIdx.x * 256u;
  const uint32_t nvalid = min(256u, F.nblocks - b0);
  const uint32_t* src = in32 + (uint64_t)b0 * WPB;
  // word-wise: four words per thread and step (16-byte loads) measured 4 % slower here (r05_c3_wide_store_ab.log)
  for (uint32_t j = tid; j < nvalid * WPB; j += 256) lds_w[(j / WPB) * (WPB + 2) + (j % WPB)] = src[j];
  lds_w[tid * (WPB + 2) + WPB] = 0u;
  lds_w[tid * (WPB + 2) + WPB + 1] = 0u;
  __syncthreads();
  if (tid < nvalid) {
    WordBitReader r{lds_w + tid * (WPB + 2), 0};
    float f[64];
    decode_block<3>(r, p, f);
    scatter_block<3>(F, b0 + tid, f);
  }
}

// ------------------------------------------------------------------------------------------------ decode
template <int D>
__global__ __launch_bounds__(64) void k_decode(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                               const uint64_t* __restrict__ index, uint32_t chunk, uint64_t nchunks,
                                               uint32_t fixed, uint64_t base_bits, uint64_t* __restrict__ end_out)
{
  constexpr int B = Dim<D>::B;
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  BitReader r{in, 0};
  uint64_t b = c * chunk;
  const uint64_t bend = min<uint64_t>(b + chunk, F.nblocks);
  r.pos = base_bits + (fixed ? b * p.maxbits : (index ? index[c] : 0ull));
  for (; b < bend; b++) {
    float f[B];
    decode_block<D>(r, p, f);
    if constexpr (D == 1) store_block1d(F, b, f);  // fp32 or bf16 output
    else scatter_block<D>(F, (uint32_t)b, f);
  }
  if (end_out && c == nchunks - 1) *end_out = r.pos;
}

// One block per lane with the workgroup's stream span staged in LDS (coalesced copy) and read through
// WordBitReader: blocks start at the block index (stride 1) or at b * maxbits (fixed rate). A span above the
// capacity (1024 bits per block on average) decodes from global memory.
template <int D>
__global__ __launch_bounds__(64) void k_decode_staged(FieldDesc F, Params p, const uint64_t* __restrict__ in,
                                                      uint64_t in_words, const uint64_t* __restrict__ index,
                                                      uint32_t fixed, uint64_t base_bits,
                                                      uint64_t* __restrict__ end_out)
{
  constexpr int B = Dim<D>::B;
  constexpr uint32_t CAPW = 64 * 1024 / 32;  // 32-bit words
  __shared__ __attribute__((aligned(16))) uint32_t sw[CAPW + 8];
  const uint32_t tid = threadIdx.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * 64, nb = F.nblocks;
  auto start_of = [&](uint64_t b) { return base_bits + (fixed ? b * p.maxbits : index[b]); };
  const uint64_t b = b0 + tid;
  const uint64_t mine = b < nb ? start_of(b) : 0ull;  // requested with the span, not after it
  const uint64_t s0 = start_of(b0);
  const uint64_t w0 = (s0 >> 5) & ~3ull;  // 32-bit word index, 16-byte aligned
  const uint64_t in_w32 = 2 * in_words;
  const uint64_t wend = b0 + 64 < nb ? (start_of(b0 + 64) + 31) >> 5 : in_w32;
  const uint64_t span = min<uint64_t>(wend, in_w32) - w0;
  const bool staged = span <= CAPW;
  const uint32_t* in32 = (const uint32_t*)in;
  // the span (zeros after it: the reader looks up to 3 words past a block's last bit) in one memory round trip
  if (staged) stage_lds16<64, (CAPW + 8) / 4>(sw, in32 + w0, (uint32_t)(4 * span));
  __syncthreads();
  if (b >= nb) return;
  float f[B];
  uint64_t end;
  if (staged) {
    WordBitReader r{sw, (uint32_t)(mine - 32 * w0)};
    decode_block<D>(r, p, f);
    end = r.pos + 32 * w0;
  } else {
    BitReader r{in, mine};
    decode_block<D>(r, p, f);
    end = r.pos;
  }
  scatter_block<D>(F, (uint32_t)b, f);
  if (end_out && b == nb - 1) *end_out = end;
}

// ------------------------------------------------------------------------------------------------ launchers
static inline hipStream_t hip_stream(void* s) { return (hipStream_t)s; }

template <int D, int DT, uint32_t T>
static hipError_t launch_tiles23_t(const FieldDesc& F, const Params& p, const TilePlan& plan, uint32_t* out32,
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
  if constexpr (D == 3) {
    if (plan.range == 64) {  // one tile per workgroup (make_plan): k_count3d / k_encode3d_var
      uint16_t* lens = (uint16_t*)(ws_base + plan.nranges + 1);  // workspace: sums, base, lens
      k_count3d<DT><<<plan.nranges, 64, 0, st>>>(F, p, ws_sums, lens);
      hipError_t e = launch_scan_ranges(ws_sums, plan.nranges, ws_base, d_total, out32, d_base, st);
      if (e != hipSuccess) return e;
      const bool mask = (p.maxprec + 1) * 64u - 1u > p.maxbits - 9u;  // exceeded_maxbits at maxprec: a budget can clip
      auto kern = mask ? k_encode3d_var<DT, true> : k_encode3d_var<DT, false>;
      const uint32_t win = std::min<uint32_t>(plan.lds_words, E3V_WIN_WORDS);
      kern<<<plan.nranges, 64, (size_t)win * 4, st>>>(F, p, ws_base, lens, out32, index, index_shift, win);
      return hipGetLastError();
    }
  }
  k_count<D, DT, T><<<plan.nranges, T, 0, st>>>(F, p, plan.range, ws_sums);
  hipError_t e = launch_scan_ranges(ws_sums, plan.nranges, ws_base, d_total, out32, d_base, st);
  if (e != hipSuccess) return e;
  auto kern = k_encode_tiles<D, DT, T, false>;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<plan.nranges, T, lds, st>>>(F, p, plan.range, ws_base, out32, index, index_shift);
  return hipGetLastError();
}

hipError_t launch_encode_tiles23(const FieldDesc& F, const Params& p, const TilePlan& plan, uint32_t* out32,
                                 uint64_t* ws_sums, uint64_t* ws_base, uint64_t* d_total, uint64_t* index,
                                 uint32_t index_shift, const uint64_t* d_base, void* stream)
{
  hipStream_t st = hip_stream(stream);
  const bool bf = F.dtype == DT_BF16;
#define GCOW_TILES(D, T)                                                                                          \
  return bf ? launch_tiles23_t<D, DT_BF16, T>(F, p, plan, out32, ws_sums, ws_base, d_total, index, index_shift, d_base, st) \
            : launch_tiles23_t<D, DT_F32, T>(F, p, plan, out32, ws_sums, ws_base, d_total, index, index_shift, d_base, st)
  if (F.dims == 2) {
    if (plan.threads == 256) { GCOW_TILES(2, 256); } else { GCOW_TILES(2, 64); }
  }
  GCOW_TILES(3, 64);
#undef GCOW_TILES
}

hipError_t launch_decode(const FieldDesc& F, const Params& p, const uint64_t* in, const uint64_t* index,
                         uint32_t chunk, uint64_t nchunks, bool fixed, uint64_t base_bits, uint64_t* end_out,
                         void* stream, uint64_t in_words)
{
  if (chunk == 1 && in_words && (fixed || index) && F.dims >= 2) {
    const uint32_t g = (uint32_t)((F.nblocks + 63) / 64);
    if (F.dims == 2) k_decode_staged<2><<<g, 64, 0, hip_stream(stream)>>>(F, p, in, in_words, index, fixed, base_bits, end_out);
    else k_decode_staged<3><<<g, 64, 0, hip_stream(stream)>>>(F, p, in, in_words, index, fixed, base_bits, end_out);
    return hipGetLastError();
  }
  const uint32_t T = 64;
  const uint64_t grid = (nchunks + T - 1) / T;
  if (!grid) return hipSuccess;
  if (F.dims == 1) k_decode<1><<<grid, T, 0, hip_stream(stream)>>>(F, p, in, index, chunk, nchunks, fixed, base_bits, end_out);
  else if (F.dims == 2) k_decode<2><<<grid, T, 0, hip_stream(stream)>>>(F, p, in, index, chunk, nchunks, fixed, base_bits, end_out);
  else k_decode<3><<<grid, T, 0, hip_stream(stream)>>>(F, p, in, index, chunk, nchunks, fixed, base_bits, end_out);
  return hipGetLastError();
}

template <int DT, uint32_t WPB>
static hipError_t launch_enc3d_t(const FieldDesc& F, const Params& p, uint32_t* out32, hipStream_t st)
{
  const size_t lds = (256 * (WPB + E3_SLACK + 1) + 256) * 4;
  auto kern = k_encode3d_fixed<DT, WPB>;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<(F.nblocks + 255) / 256, 256, lds, st>>>(F, p, out32);
  return hipGetLastError();
}

template <uint32_t WPB>
static hipError_t launch_dec3d_t(const FieldDesc& F, const Params& p, const uint32_t* in32, hipStream_t st)
{
  const size_t lds = 256 * (WPB + 2) * 4;
  auto kern = k_decode3d_fixed<WPB>;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<(F.nblocks + 255) / 256, 256, lds, st>>>(F, p, in32);
  return hipGetLastError();
}

bool fixed3d_ok(uint32_t maxbits)
{
  const uint32_t w = maxbits / 32;
  return maxbits % 32 == 0 && (w == 2 || w == 4 || w == 8 || w == 16 || w == 32 || w == 64);
}

hipError_t launch_encode3d_fixed(const FieldDesc& F, const Params& p, uint32_t* out32, void* stream)
{
  hipStream_t st = hip_stream(stream);
  const bool bf = F.dtype == DT_BF16;
#define GCOW_E3(W) return bf ? launch_enc3d_t<DT_BF16, W>(F, p, out32, st) : launch_enc3d_t<DT_F32, W>(F, p, out32, st)
  switch (p.maxbits / 32) {
    case 2: GCOW_E3(2);
    case 4: GCOW_E3(4);
    case 8: GCOW_E3(8);
    case 16: GCOW_E3(16);
    case 32: GCOW_E3(32);
    case 64: GCOW_E3(64);
  }
#undef GCOW_E3
  return hipErrorInvalidValue;
}

hipError_t launch_decode3d_fixed(const FieldDesc& F, const Params& p, const uint32_t* in32, void* stream)
{
  hipStream_t st = hip_stream(stream);
  switch (p.maxbits / 32) {
    case 2: return launch_dec3d_t<2>(F, p, in32, st);
    case 4: return launch_dec3d_t<4>(F, p, in32, st);
    case 8: return launch_dec3d_t<8>(F, p, in32, st);
    case 16: return launch_dec3d_t<16>(F, p, in32, st);
    case 32: return launch_dec3d_t<32>(F, p, in32, st);
    case 64: return launch_dec3d_t<64>(F, p, in32, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace gcow
