// var1d.hip -- single-pass 1-D variable-rate encoder (accuracy / precision / expert with minbits <= 1,
// maxbits >= 160: no budget ever truncates a block), the C5 path of BASELINE configs[4].
//
// Reference: sw/src/zfp.c:31-56 (block loop), sw/src/encode.c:457-495 (encode_fblock) and :279-339 (the embedded
// coder), sw/src/stream.c:61-138 (LSB-first packing). The reference codes blocks one after another into one stream;
// the position of block b is the sum of the lengths of blocks 0 .. b-1, which is what this kernel computes in one
// pass over the input:
//
//  * one workgroup per tile of 1024 consecutive blocks (256 lanes x 4): every lane derives its blocks' coefficients
//    once, their lengths by the closed form and its offset in the tile by a workgroup scan;
//  * the tile's length total is published at once (a decoupled look-back status word, MI355X_MICROARCH.md
//    "Valid forms" R2 granule: value and flag in ONE 8-byte agent-scope store, no fence), the blocks are coded into
//    the tile's LDS window at tile-relative positions, and only then does one wave look back over the predecessors'
//    status words for the tile's stream offset -- by then they have published. A predecessor that has not published
//    after a bounded wait has its total computed here from its input instead, so no workgroup ever depends on
//    another one being scheduled (no dispatch-order assumption, no deadlock);
//  * each lane packs its consecutive blocks in a 64-bit register accumulator: whole words are plain LDS stores,
//    only the two words it shares with its neighbours are ds_or;
//  * the window is stored shifted to the tile's bit offset as coalesced 32-bit words; the one word a tile shares with
//    each neighbour is combined through a per-boundary 64-bit atomicOr (the second contributor writes it).
// The status and boundary words are zeroed by a memset node before every launch (gcow_amd/csrc/var1d.hip launcher).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>

#include "codec_device.h"
#include "field_io.h"
#include "kernels.h"
#include "lean1d.h"
#include "tiles.h"

namespace gcow {

#ifndef GCOW_V1T
#define GCOW_V1T 256
#endif
constexpr uint32_t V1T = GCOW_V1T;                           // lanes per workgroup
constexpr uint32_t V1U = 4;                                  // consecutive blocks per lane
constexpr uint32_t V1TILE = V1T * V1U;                       // blocks per tile
constexpr uint32_t V1MAXB = 140;                             // 9 + 3 + 4 * 32: the longest 1-D block
constexpr uint32_t V1Q = (V1TILE * V1MAXB + 63) / 64 + 2;    // LDS window, 64-bit words
constexpr uint64_t V1VAL = (1ull << 62) - 1;                 // status word: flag << 62 | value
// V1_ABLATE (measurement builds only, tools/ubench/var1d_ablate.sh; 0 in the product): 1 = no look-back (tile t at
// t * 64 Ki bits), 2 = no coding (zero codes / prepared words, lengths kept), 4 = no window store, 8 = no pair loop,
// 16 = no prepare in the tile coder (raw words as coefficients), 32 = no length computation in the tile count,
// 64 = no input / length loads in the tile coder (synthetic words, 58-bit blocks), 128 = no LDS window writes in the
// tile coder (the accumulator words folded into one register), 256 = no spread-table window lookups in the coder
#ifndef V1_ABLATE
#define V1_ABLATE 0
#endif
constexpr uint32_t V1SPIN = 96;  // polls (~1.5 us each) of a missing predecessor before computing its total here

// v_lshlrev_b32 as an opaque instruction: the shift count's low 5 bits (a count of 32 shifts by 0, not UB)
__device__ __forceinline__ uint32_t shl_hw(uint32_t x, uint32_t n)
{
  uint32_t r;
  asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "v"(n), "v"(x));
  return r;
}

// The lean-5 pair table with its rows n = 3 and 4 emptied (no bits, the row kept): from n = 3 on every plane is its
// nibble verbatim (encode.c:301-333 with one coefficient left), which the variable-rate coder takes from the window
// instead, so a lane whose group phase is over adds nothing more -- no per-lane selects in the pair loop.
// Row n' = 4 is folded into row 3 (both are empty), so the tile kernels keep only rows 0..3 (4 KB) in LDS.
__host__ __device__ constexpr PlaneTab2 make_plane_tab_var()
{
  PlaneTab2 T = make_plane_tab5();
  for (uint32_t t = 0; t < 3 * 256; t++)
    if ((T.v[t] & 0x1c00u) == (4u << 10)) T.v[t] = (T.v[t] & ~0x1c00u) | (3u << 10);
  for (uint32_t t = 3 * 256; t < 1280; t++) T.v[t] = 3u << 10;
  return T;
}
__device__ const PlaneTab2 g_plane_tab_var = make_plane_tab_var();

// One block's header, coefficients and bit length (encode_fblock's return value, sw/src/encode.c:457-495, for
// minbits <= 1 and maxbits >= 160). cexp = -122 - minexp (precision = emax - minexp + 4, emax = E - 126 for the
// biased exponent E of max |f|: subnormal maxima, E = 0, clamp to -126). hdr = the 9-bit header 2 (emax + 127) + 1,
// or 0 for a one-bit block (zero block or no precision); K = 31 - kmin. inf: Inf / NaN present (the generic coder takes the block).
__device__ __forceinline__ uint32_t v1_prep(const float* f, int cexp, int maxprec, uint32_t* u, uint32_t& hdr,
                                            uint32_t& K, bool& inf)
{
  uint32_t m;  // max |f| as bits (v_max3 with |.| modifiers; NaN is caught below, it never wins encode.c:146-150)
  asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(m) : "v"(f[0]), "v"(f[1]), "v"(f[2]));
  asm("v_max_f32_e64 %0, %0, |%1|" : "+v"(m) : "v"(f[3]));
  inf = m > 0x7f7fffffu || __builtin_isunordered(f[0], f[1]) || __builtin_isunordered(f[2], f[3]);
  const uint32_t E = m >> 23;
  // get_precision, d = 1 (common.c:226-229); subnormal maxima clamp emax to -126 (encode.c:142-152)
  // K = min(prec, 32) - 1 clamped to 0 = clamp(E + cexp - 1, 0, min(maxprec, 32) - 1); the block is a single bit
  // when prec = 0, i.e. E + cexp <= 0 or maxprec = 0
  const int ep = (int)E + cexp, kmax = min(maxprec, 32) - 1;  // kmax < 0: maxprec = 0, every block one bit
  K = (uint32_t)max(min(ep - 1, kmax), 0);
  const float s = __uint_as_float(0x8d800000u - (m & 0x7f800000u));  // 2^(30 - emax)
  // every value of a block with E < 29 casts to INT_MIN (the scale overflows; x86 cvttss2si, encode.c:162-187):
  // an integer mask selects it per value (v_bfi), no compare-to-mask selects
  const uint32_t tm = (uint32_t)((int32_t)(E - 29u) >> 31);
  auto cast = [&](float v) { return ((uint32_t)cvt_i32_hw(v * s) & ~tm) | (tm & 0x80000000u); };
  uint32_t x = cast(f[0]), y = cast(f[1]), z = cast(f[2]), w = cast(f[3]);
  auto asr = [](uint32_t v) { return (uint32_t)((int32_t)v >> 1); };
  constexpr uint32_t NB = 0xaaaaaaaau;
  x = asr(x + w); w -= x;  // fwd_lift (encode.c:212-225), int32 wraparound
  z = asr(z + y); y -= z;
  x = asr(x + z); z -= x;
  w = asr(w + y); y -= w;
  w += asr(y); y -= asr(w);
  u[0] = (x + NB) ^ NB;  // twoscomplement_to_negabinary (encode.c:263-275)
  u[1] = (y + NB) ^ NB;
  u[2] = (z + NB) ^ NB;
  u[3] = (w + NB) ^ NB;
  const bool one = m == 0 || ep <= 0 || kmax < 0;  // a single 0 bit (encode.c:471-475; prec = 0)
  hdr = one ? 0u : 2u * E + 3u;
  // encode_ints' length from the leading planes (codec_device.h encode_ints_length, B = 4), integer-only:
  //   4 + 4 K - sum_{j<3} c_j + sum_{j<3} e_j,  c_j = min(z_j, K + 1), z_j = ffbh(S_j) of the suffix OR S_j,
  //   e_j = [c_j <= K and bit 31 - z_j of u_j is set] (L_j = R_j: u_j holds the leading plane of S_j)
  // (the c = 4 case of the general form folded in; tests/test_length_formula.py checks it against the oracle)
  const uint32_t S2 = u[2] | u[3], S1 = u[1] | S2, S0 = u[0] | S1;
  const uint32_t K1 = K + 1u;
  const uint32_t c2 = min(ffbh_hw(S2), K1), c1 = min(ffbh_hw(S1), K1), c0 = min(ffbh_hw(S0), K1);
  const uint32_t e2 = (shl_hw(u[2], c2) >> 31) & min(K1 - c2, 1u);  // c_j = 32 (K = 31, S_j = 0): e_j = 0
  const uint32_t e1 = (shl_hw(u[1], c1) >> 31) & min(K1 - c1, 1u);
  const uint32_t e0 = (shl_hw(u[0], c0) >> 31) & min(K1 - c0, 1u);
  const uint32_t len = 4u + 4u * K - (c0 + c1 + c2) + (e0 + e1 + e2);
  return one ? 1u : 9u + len;
}

// A block's code (sw/src/encode.c:457-495 + :279-339) OR-ed into the lane's bit accumulator at bit `fill`, its full
// 64-bit words stored to the window: c = the first 128 bits of the code of every plane -- the code of planes 31 ..
// kmin is a prefix of it, so the coder ignores kmin and the length cuts it. Same evaluation as the fixed-rate lean-6
// coder (gcow_kernels.hip): header | one '0' per empty plane above M0 | group phase through the pair table, two
// planes per wave-uniform step, until no lane of the wave has a coded group plane left | the rest of the 32-plane
// window verbatim from the lane's nibble jl. special: the block needs the generic coder (a group phase past the
// 16-plane window, a group code of 64 bits or more, a code past 128 bits); its bits are left zero here.
__device__ __forceinline__ void v1_code(const uint32_t* u, uint32_t hdr, uint32_t len, uint32_t K, const uint32_t* tab,
                                        const uint32_t* rs, uint64_t& c0, uint64_t& c1, bool& special)
{
  const uint32_t S2 = u[2] | u[3];
  const uint32_t sh = ffbh_hw(u[0] | u[1] | S2 | 1u);  // 31 - M0
  const int M0 = 31 - (int)sh;
  // group phase: window nibbles 0 .. jg, of which planes >= kmin are coded (nibbles <= K - sh)
  const int jg = (int)min(ffbh_hw(S2), K) - (int)sh;
  const uint32_t w0 = u[0] << sh, w1 = u[1] << sh, w2 = u[2] << sh, w3 = u[3] << sh;
  const uint64_t Y = (V1_ABLATE & 256) ? (((uint64_t)(w0 ^ w1) << 32) | (w2 ^ w3))
                                        : window_lds(rs, w0, w1, w2, w3);  // planes M0 .. M0 - 15 as nibbles
  const uint32_t pos0 = 9u + sh;                      // header + one '0' per empty plane
  uint32_t e = tab[(uint32_t)Y & 255u];
  uint64_t G = e >> 17;
  uint32_t gl = (e >> 13) & 15u;
#pragma unroll
  for (int jj = 2; jj < ((V1_ABLATE & 8) ? 2 : 16); jj += 2) {
    if (!__any(jj <= jg)) break;
    e = tab5_next(tab, e, (uint32_t)(Y >> (4 * jj)) & 255u);  // rows n >= 3 add nothing
    G |= (uint64_t)(e >> 17) << (gl & 63u);
    gl += (e >> 13) & 15u;
  }
  const uint32_t jl = (uint32_t)min(max((jg & ~1) + 2, 2), 16);  // first nibble after the lane's last group pair
  special = special || gl > 63u || len > 128u || (jg >= 16 && pos0 + gl < len);
  // V = the 32-plane window from nibble jl on (planes M0 - 16 .. M0 - 31 only where a lane's code reaches them);
  // R = group code | V after it; c = header | R after the empty planes
  const uint32_t vs = 4u * jl - 8u;  // 0 .. 56: V = W >> (vs + 8)
  uint64_t V0 = (Y >> 8) >> vs, V1 = 0;
  if (__any(M0 >= 16 && pos0 + gl + 56u - vs < len)) {  // plane M0 - 16 lands at pos0 + gl + 4 (16 - jl)
    const uint64_t Y2 = (V1_ABLATE & 256) ? (((uint64_t)(w0 + w1) << 32) | (w2 + w3))
                                          : window_lds_low(rs, w0, w1, w2, w3);
    V0 |= Y2 << (56u - vs);
    V1 = (Y2 >> 8) >> vs;
  }
  const uint32_t g = gl & 63u;  // >= 2
  const uint64_t R0 = G | (V0 << g), R1 = (V0 >> (64u - g)) | (V1 << g);
  c0 = (uint64_t)hdr | (R0 << pos0);  // pos0: 9 .. 40
  c1 = (R0 >> (64u - pos0)) | (R1 << pos0);
}

// The lane's V1U consecutive blocks of tile t as raw words: 16-B loads of a whole tile of full, contiguous, 16-B
// aligned blocks (fp32: one per block; bf16: one per two blocks), else the padded / strided gather (encode.c:41-126)
// repacked into the same words (bf16 values narrowed back exactly).
template <int DT>
struct V1Raw {
  static constexpr int N = DT == DT_BF16 ? V1U / 2 : V1U;
  uint4 w[N];
  __device__ __forceinline__ void load(const FieldDesc& F, uint32_t t, bool wide_ok)
  {
    const uint64_t bl = (uint64_t)t * V1TILE + (uint64_t)threadIdx.x * V1U;
    if (wide_ok && (uint64_t)(t + 1) * V1TILE <= F.n[0] / 4) {
      const uint4* src = (const uint4*)F.data + (DT == DT_BF16 ? bl / 2 : bl);
#pragma unroll
      for (int h = 0; h < N; h++) w[h] = src[h];
    } else {
#pragma unroll
      for (uint32_t k = 0; k < V1U; k++) {
        float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (bl + k < F.nblocks) gather_block<1, DT>(F, (uint32_t)(bl + k), f);
        uint32_t* d = (uint32_t*)w;
        if constexpr (DT == DT_BF16) {
          d[2 * k] = (__float_as_uint(f[0]) >> 16) | (__float_as_uint(f[1]) & 0xffff0000u);
          d[2 * k + 1] = (__float_as_uint(f[2]) >> 16) | (__float_as_uint(f[3]) & 0xffff0000u);
        } else {
#pragma unroll
          for (int i = 0; i < 4; i++) d[4 * k + i] = __float_as_uint(f[i]);
        }
      }
    }
  }
  __device__ __forceinline__ void block(uint32_t k, float* f) const
  {
    const uint32_t* d = (const uint32_t*)w;
    if constexpr (DT == DT_BF16) {
      f[0] = __uint_as_float(d[2 * k] << 16);
      f[1] = __uint_as_float(d[2 * k] & 0xffff0000u);
      f[2] = __uint_as_float(d[2 * k + 1] << 16);
      f[3] = __uint_as_float(d[2 * k + 1] & 0xffff0000u);
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++) f[i] = __uint_as_float(d[4 * k + i]);
    }
  }
};

// Per-lane state of one tile between its preparation and its store: the blocks' coefficients, headers, K and
// lengths, the lane's offset in the tile and the tile's total.
struct V1Tile {
  uint32_t u[V1U][4], hdr[V1U], K[V1U], len[V1U];
  bool inf[V1U];
  uint32_t excl, total;
};

// Prepare tile t (coefficients, closed-form lengths, the lane's offset by a workgroup scan) and publish its total as
// its status word -- one 8-byte agent-scope store, value and flag in one granule (MI355X_MICROARCH.md "Valid forms").
template <int DT>
__device__ __forceinline__ void v1_prepare(const FieldDesc& F, const Params& p, const V1Raw<DT>& raw, uint32_t t,
                                           V1Tile& T, uint32_t* scan_sh, uint64_t* status, uint64_t incl_base)
{
  const uint64_t bl = (uint64_t)t * V1TILE + (uint64_t)threadIdx.x * V1U;
  uint32_t lsum = 0;
#pragma unroll
  for (uint32_t k = 0; k < V1U; k++) {
    float f[4];
    raw.block(k, f);
    const bool valid = bl + k < F.nblocks;
    T.len[k] = v1_prep(f, -122 - p.minexp, (int)min(p.maxprec, 64u), T.u[k], T.hdr[k], T.K[k], T.inf[k]);
    T.inf[k] = T.inf[k] && valid;
    if (T.inf[k]) T.len[k] = count_block<1>(f, p);
    T.len[k] = valid ? T.len[k] : 0u;
    lsum += T.len[k];
  }
  T.excl = block_exclusive_scan<V1T>(lsum, &T.total, scan_sh);
  if (threadIdx.x == 0)  // incl_base given (tile 0): the inclusive prefix at once
    __hip_atomic_store(status + t, incl_base != ~0ull ? ((2ull << 62) | (incl_base + T.total)) : ((1ull << 62) | T.total),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One of the two contributors of a 32-bit word shared by tiles x and x + 1 (role 0: tile x's last word, role 1: tile
// x + 1's first word): OR its bits and its arrival flag into the boundary's word; the second to arrive stores it.
__device__ __forceinline__ void v1_boundary(uint64_t* bnd, uint32_t x, uint32_t role, uint32_t* out, uint32_t val)
{
  const uint64_t old = atomicOr((unsigned long long*)(bnd + x), (unsigned long long)((1ull << (32 + role)) | val));
  if ((old >> (33 - role)) & 1ull) *out = val | (uint32_t)old;
}

// Total bit length of tile `tile` by one wave, from the input: the look-back's fallback for a predecessor without a
// status after a bounded wait (the same lengths the tile's own workgroup sums).
template <int DT>
__device__ uint64_t v1_wave_total(const FieldDesc& F, const Params& p, uint32_t tile, uint32_t lane)
{
  uint64_t s = 0;
  const uint64_t b0 = (uint64_t)tile * V1TILE;
  const uint64_t b1 = min<uint64_t>(b0 + V1TILE, F.nblocks);
  for (uint64_t b = b0 + lane; b < b1; b += 64) {
    float f[4];
    gather_block<1, DT>(F, (uint32_t)b, f);
    uint32_t u[4], hdr, K;
    bool inf;
    uint32_t len = v1_prep(f, -122 - p.minexp, (int)min(p.maxprec, 64u), u, hdr, K, inf);
    if (inf) len = count_block<1>(f, p);
    s += len;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// Decoupled look-back (one wave): the stream offset of tile t = base0 + the totals of tiles 0 .. t-1, from the
// predecessors' status words, 4 per lane = 256 per round trip (flag 2 = inclusive prefix: stop at the nearest one;
// flag 1 = the tile's own total). A predecessor without a status after `spin` polls has its total computed here
// (v1_wave_total), so no tile depends on another being scheduled.
template <int DT>
__device__ uint64_t v1_lookback(uint64_t* status, uint32_t t, uint64_t base0, const FieldDesc& F, const Params& p,
                                uint32_t lane, uint32_t spin, uint64_t* stats)
{
  constexpr int L = 4;
  uint64_t excl = 0;
  int64_t j = (int64_t)t - 1;  // nearest predecessor of the window
  uint32_t polls = 0, fallbacks = 0, windows = 0;
  uint64_t fb[L] = {0, 0, 0, 0};  // totals computed here (this window, this lane), flag in bit 62
  while (true) {
    uint64_t v[L];
    int first = L;  // this lane's nearest inclusive entry
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int64_t idx = j - (int64_t)(L * lane) - i;
      v[i] = idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : ((2ull << 62) | (idx == -1 ? base0 : 0ull));  // "tile -1": the stream's start
      if ((v[i] >> 62) == 0 && fb[i]) v[i] = fb[i];
    }
#pragma unroll
    for (int i = L - 1; i >= 0; i--) first = (v[i] >> 62) == 2 ? i : first;
    const uint64_t incl = __ballot(first < L);
    const uint32_t L0 = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;  // lane holding the nearest inclusive
    const int nneed = lane < L0 ? L : (lane == L0 ? first + 1 : 0);     // entries this lane contributes
    int miss = L;
#pragma unroll
    for (int i = L - 1; i >= 0; i--) miss = (i < nneed && (v[i] >> 62) == 0) ? i : miss;
    const uint64_t missing = __ballot(miss < L);
    if (missing) {
      if (++polls <= spin) {
        __builtin_amdgcn_s_sleep(8);
        continue;
      }
      const uint32_t k = (uint32_t)__builtin_ctzll(missing);
      const int mi = __shfl(miss, (int)k, 64);
      const uint64_t tot = v1_wave_total<DT>(F, p, (uint32_t)(j - (int64_t)(L * k) - mi), lane);
#pragma unroll
      for (int i = 0; i < L; i++)
        if (lane == k && i == mi) fb[i] = (1ull << 62) | tot;
      fallbacks++;
      continue;
    }
    windows++;
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < L; i++) x += i < nneed ? (v[i] & V1VAL) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    excl += x;
    if (incl) {
      if (stats && lane == 0) {  // variant stats: look-back behaviour, summed over the launch
        atomicAdd((unsigned long long*)stats, (unsigned long long)polls);
        atomicAdd((unsigned long long*)stats + 1, (unsigned long long)fallbacks);
        atomicAdd((unsigned long long*)stats + 2, (unsigned long long)windows);
        if (polls) {  // tiles that polled at all, the most polls of one tile, polls of the first 2048 tiles
          atomicAdd((unsigned long long*)stats + 3, 1ull);
          atomicMax((unsigned long long*)stats + 4, (unsigned long long)polls);
          if (t < 2048) atomicAdd((unsigned long long*)stats + 5, (unsigned long long)polls);
        }
      }
      return excl;
    }
    j -= 64 * L;
#pragma unroll
    for (int i = 0; i < L; i++) fb[i] = 0;
  }
}

// The encoder: one workgroup per tile of V1TILE blocks. Tile t: prepare (coefficients, closed-form lengths, the
// lanes' offsets by a workgroup scan) and publish its total at once; code into the LDS window at tile-relative
// positions; look back (one wave) for the stream offset; store the window shifted to the offset, the two words shared
// with the neighbouring tiles through v1_boundary.
template <int DT>
__global__ __launch_bounds__(V1T) void k_encode1d_var_sp(FieldDesc F, Params p, uint64_t* __restrict__ status,
                                                         uint64_t* __restrict__ bnd, uint32_t* __restrict__ out32,
                                                         uint64_t* __restrict__ index, uint32_t index_shift,
                                                         const uint64_t* __restrict__ d_base,
                                                         uint64_t* __restrict__ d_total, uint32_t ntiles,
                                                         uint32_t spin, uint64_t* __restrict__ stats)
{
  __shared__ __attribute__((aligned(16))) uint32_t tab[1280];  // pair table (lean-5 entries, rows n >= 3 empty)
  __shared__ uint32_t rs[1024];   // window spread tables
  __shared__ uint64_t win[V1Q];   // the tile's code, tile-relative bit positions
  __shared__ uint32_t scan_sh[V1T / 64];
  __shared__ uint64_t s_base;
  __shared__ uint32_t s_special;
  uint32_t* win32 = (uint32_t*)win;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t t = blockIdx.x;
  stage_table<V1T, 1280>(tab, g_plane_tab_var.v);
#pragma unroll
  for (uint32_t i = 0; i < 1024 / V1T; i++) rs[tid + V1T * i] = rspread_entry(tid + V1T * i);
  if (tid == 0) s_special = 0;
  const bool wide_ok = F.vec && (((uintptr_t)F.data) & 15u) == 0;
  const uint64_t base0 = d_base ? *d_base : 0ull;
  V1Raw<DT> raw;
  raw.load(F, t, wide_ok);
  V1Tile T;
  v1_prepare<DT>(F, p, raw, t, T, scan_sh, status, t == 0 ? base0 : ~0ull);
  const uint32_t excl = T.excl, total = T.total;
  uint32_t lsum = 0;
#pragma unroll
  for (uint32_t k = 0; k < V1U; k++) lsum += T.len[k];
  if (lsum) {  // the two words this lane shares with its neighbours start at zero
    win[excl >> 6] = 0ull;
    win[(excl + lsum - 1) >> 6] = 0ull;
  }
  __syncthreads();

  // ---- code the lane's blocks: a 64-bit accumulator; whole words are plain LDS stores, the two shared ones ds_or
  uint64_t acc = 0;
  uint32_t q = excl >> 6, fill = excl & 63u;
  const uint32_t qhead = q;
  bool sp[V1U];
  bool any_sp = false;
#pragma unroll
  for (uint32_t k = 0; k < V1U; k++) {
    uint64_t c0, c1;
    sp[k] = T.inf[k];
    if constexpr (V1_ABLATE & 2) {
      c0 = T.u[k][0] ^ T.u[k][1];
      c1 = T.u[k][2] ^ T.u[k][3];
    } else {
      v1_code(T.u[k], T.hdr[k], T.len[k], T.K[k], tab, rs, c0, c1, sp[k]);
    }
    sp[k] = sp[k] && T.len[k];
    if (sp[k]) c0 = c1 = 0ull;  // coded below by the generic coder, OR-ed into these zero bits
    any_sp = any_sp || sp[k];
    // bits past the block's length are cleared from the accumulator after the full words leave it (a full word
    // holds only bits below the length)
    acc |= c0 << fill;
    const uint64_t mid = ((c0 >> 1) >> (63u - fill)) | (c1 << fill);
    const uint64_t hi = (c1 >> 1) >> (63u - fill);
    const uint32_t nf = fill + T.len[k];
    if (nf >= 64u) {
      if (q == qhead) atomicOr((unsigned long long*)&win[q], (unsigned long long)acc);
      else win[q] = acc;
      q++;
      acc = mid;
      if (nf >= 128u) {
        win[q] = acc;
        q++;
        acc = hi;
        if (nf >= 192u) {  // a special block of up to 140 bits (its code is zero here) completes a third word
          win[q] = acc;
          q++;
          acc = 0ull;
        }
      }
    }
    fill = nf & 63u;
    acc &= (1ull << fill) - 1ull;
  }
  if (fill) atomicOr((unsigned long long*)&win[q], (unsigned long long)acc);
  if (any_sp) s_special = 1u;
  __syncthreads();
  if (s_special) {  // Inf / NaN blocks, long group phases, codes past 128 bits: the generic coder
    uint32_t o = excl;
#pragma unroll
    for (uint32_t k = 0; k < V1U; k++) {
      if (sp[k]) {
        float f[4];
        raw.block(k, f);
        LdsWriter wr{win32, o, o + T.len[k]};
        encode_block<1>(wr, f, p);
      }
      o += T.len[k];
    }
    __syncthreads();
  }

  // ---- the tile's stream offset (wave 0)
  if (tid < 64) {
    const uint64_t B = t == 0 ? base0
                              : ((V1_ABLATE & 1) ? (uint64_t)t << 16
                                                 : v1_lookback<DT>(status, t, base0, F, p, lane, spin, stats));
    if (lane == 0) {
      if (t) __hip_atomic_store(status + t, (2ull << 62) | (B + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_base = B;
    }
  }
  __syncthreads();
  const uint64_t B = s_base;
  const uint64_t bl = (uint64_t)t * V1TILE + (uint64_t)tid * V1U;
  if (index) {
    uint32_t o = excl;
#pragma unroll
    for (uint32_t k = 0; k < V1U; k++) {
      const uint64_t b = bl + k;
      if (T.len[k] && (b & ((1ull << index_shift) - 1ull)) == 0) index[b >> index_shift] = B + o;
      o += T.len[k];
    }
  }

  // ---- store the window shifted to the tile's offset: 32-bit words, coalesced
  const uint32_t rb = (uint32_t)(B & 31u);
  const uint64_t g0 = B >> 5;
  const uint32_t nw = (rb + total + 31u) >> 5;  // global words the tile touches
  const uint32_t lw = (total + 31u) >> 5;       // window words holding the tile's bits
  const bool last_tile = t == ntiles - 1;
  for (uint32_t k = tid; k < ((V1_ABLATE & 4) ? 0u : nw); k += V1T) {
    const uint32_t hi = k < lw ? win32[k] : 0u;
    const uint32_t lo = (k > 0 && k - 1 < lw) ? win32[k - 1] : 0u;
    const uint32_t val = rb ? (hi << rb) | (lo >> (32u - rb)) : hi;
    uint32_t* dst = out32 + g0 + k;
    const bool first = k == 0 && rb != 0;
    const bool tail = k == nw - 1 && ((rb + total) & 31u) != 0 && !last_tile;
    if (first) {
      if (t == 0) atomicOr(dst, val);  // bits already in the stream before d_base (append)
      else v1_boundary(bnd, t - 1, 1u, dst, val);
    } else if (tail) {
      v1_boundary(bnd, t, 0u, dst, val);
    } else {
      *dst = val;
    }
  }
  if (last_tile && tid == 0) {
    const uint64_t end = B + total;
    const uint64_t endw = (end + 31) >> 5;
    if (endw & 1) out32[endw] = 0u;  // stream_flush: zero-pad to a 64-bit boundary (stream.c:132-138)
    if (d_total) *d_total = end;
  }
}

// The workspace: status[ntiles] then bnd[ntiles] (uint64 each) and 4 words of statistics, zeroed before the launch.
Var1dVariant g_var1d_variant = {0, -1, 0};

size_t var1d_sp_workspace_bytes(uint64_t nblocks)
{
  const uint64_t ntiles = (nblocks + V1TILE - 1) / V1TILE;
  return (size_t)(16 * ntiles + 64);
}

hipError_t launch_encode1d_var_sp(const FieldDesc& F, const Params& p, uint32_t* out32, uint64_t* ws,
                                  uint64_t* d_total, uint64_t* index, uint32_t index_shift, const uint64_t* d_base,
                                  void* stream)
{
  hipStream_t st = (hipStream_t)stream;
  const uint32_t ntiles = (uint32_t)((F.nblocks + V1TILE - 1) / V1TILE);
  hipError_t e = hipMemsetAsync(ws, 0, (size_t)16 * ntiles + 64, st);
  if (e != hipSuccess) return e;
  uint64_t* status = ws;
  uint64_t* bnd = ws + ntiles;
  // spin (tests): polls before a missing predecessor's total is computed locally; 0 exercises that path
  const uint32_t spin = g_var1d_variant.spin >= 0 ? (uint32_t)g_var1d_variant.spin : V1SPIN;
  // stats (measurement): polls, fallbacks, look-back windows, polling tiles, most polls, polls of the first 2048
  // tiles into ws[2 ntiles .. + 6)
  uint64_t* stats = g_var1d_variant.stats ? ws + 2 * (size_t)ntiles : nullptr;
  if (F.dtype == DT_BF16)
    k_encode1d_var_sp<DT_BF16><<<ntiles, V1T, 0, st>>>(F, p, status, bnd, out32, index, index_shift, d_base, d_total,
                                                       ntiles, spin, stats);
  else
    k_encode1d_var_sp<DT_F32><<<ntiles, V1T, 0, st>>>(F, p, status, bnd, out32, index, index_shift, d_base, d_total,
                                                      ntiles, spin, stats);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------ tile form (default)
// count + scan + placed tile coder. The look-back above waits on predecessors spread over the eight XCDs (C5: 0.91 ms
// against 0.71 ms for this form, profiles/r03_c5_forms_ab.log); here the offsets come from a scan instead:
//   k_count1d_var_tile   V1CT tiles of V1TILE blocks per workgroup, the next tile's loads issued before a tile is counted:
//                        each block's length (closed form, v1_prep) as a byte (lens8: one 32-bit word per lane and
//                        tile, its V1U blocks) and each tile's total (sums[t]);
//   k_scan_ranges(_mw)   the tiles' stream offsets (base), zeroing the words two tiles share;
//   k_encode1d_var_tile  one tile per workgroup: the lane's offset in the tile by a workgroup scan of the stored
//                        lengths (before any block is prepared, so prepare and code run per block and the
//                        coefficients live only for one block), the blocks coded at their bit position relative to the
//                        16-byte stream boundary below the tile (base & 127 + the lane offset) into an LDS window
//                        through the lane accumulator, and the window stored as 16-byte chunks of stream words (no
//                        shifting; the two words shared with the neighbours by atomicOr). The window holds V1QS qwords (95 bits per block on
//                        average) so that 8 workgroups fit a CU (the kernel waits on memory and LDS latency: occupancy,
//                        not VALU issue, bounds it); a tile that needs more is skipped and coded by
//   k_encode1d_var_tile_big  the same body with the worst-case window (140 bits per block), a grid-stride loop over
//                        the list of oversized tiles k_encode1d_var_tile appended to (the count kernel empties it).
constexpr uint32_t V1CT = 8;                                      // tiles per count workgroup
#ifndef V1_COUNT_PF
#define V1_COUNT_PF 1  // tiles of loads in flight ahead of the counted one (k_count1d_var_tile), 1 .. 3
#endif
constexpr uint32_t V1QS = 1500 * (V1T / 256);                     // small window, qwords (95 bits per block)
constexpr uint32_t V1TAB = 1024;                                  // pair-table rows 0..3 in LDS

// Raw buffer loads issued from inline asm, invisible to the compiler's waitcnt pass, with hand-counted waits (the
// scheme of k_encode_fixed1d_np): vmcnt counts loads and stores together, in issue order.
typedef int v1_v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v1_v4i v1_rsrc(const void* p, uint32_t bytes)
{
  const uint64_t a = (uint64_t)p;
  v1_v4i r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((uint32_t)(a >> 32) & 0xffffu);  // stride 0
  r.z = (int)bytes;                             // num_records: range check in bytes
  r.w = 0x00020000;                             // raw buffer, no swizzle
  return r;
}

typedef unsigned v1_u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v1_u4 v1_ld16(uint32_t off, v1_v4i rs)
{
  v1_u4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(rs) : "memory");
  return v;
}

// wait until at most N vector memory operations are outstanding; ties the tile's raw words to after the wait
template <int N, int NL>
__device__ __forceinline__ void v1_wait_n(v1_u4 (&w)[NL])
{
  if constexpr (NL == 2)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(w[0]), "+v"(w[1]) : "n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]) : "n"(N) : "memory");
}

// the same for k tiles of NL loads each still in flight (k folds to a constant in the unrolled tile loop)
template <int NL>
__device__ __forceinline__ void v1_wait_tiles(v1_u4 (&w)[NL], uint32_t k)
{
  switch (k) {
    case 0: v1_wait_n<0>(w); break;
    case 1: v1_wait_n<NL>(w); break;
    case 2: v1_wait_n<2 * NL>(w); break;
    default: v1_wait_n<3 * NL>(w); break;
  }
}

// One tile's block lengths (bytes packed per lane) and the lane's sum. FULL: every block of the tile is inside the
// field (no per-block range check).
template <int DT, bool FULL = false>
__device__ __forceinline__ uint32_t v1_count_tile(const FieldDesc& F, const Params& p, const V1Raw<DT>& raw,
                                                  uint32_t t, uint32_t& lsum)
{
  const uint64_t bl = (uint64_t)t * V1TILE + (uint64_t)threadIdx.x * V1U;
  const int cexp = -122 - p.minexp, maxprec = (int)min(p.maxprec, 64u);
  uint32_t pk = 0;
  lsum = 0;
#pragma unroll
  for (uint32_t k = 0; k < V1U; k++) {
    float f[4];
    raw.block(k, f);
    uint32_t u[4], hdr, K;
    bool inf;
    uint32_t len;
    if constexpr ((V1_ABLATE & 32) != 0) {  // measurement builds: no length computation in the count
      len = 9u + ((__float_as_uint(f[0]) ^ __float_as_uint(f[3])) & 63u);
      inf = false;
    } else {
      len = v1_prep(f, cexp, maxprec, u, hdr, K, inf);
    }
    const bool valid = FULL || bl + k < F.nblocks;
    if (inf && valid) len = count_block<1>(f, p);
    len = valid ? len : 0u;  // <= 140
    pk |= len << (8 * k);
    lsum += len;
  }
  return pk;
}

template <int DT>
__global__ __launch_bounds__(V1T) void k_count1d_var_tile(FieldDesc F, Params p, uint32_t ntiles,
                                                          uint64_t* __restrict__ sums, uint32_t* __restrict__ lens8,
                                                          uint32_t* __restrict__ nover, uint64_t* __restrict__ gsums)
{
  static_assert(V1CT == 8, "the scan's group totals (gsums) cover 8 tiles");
  // V1CT consecutive tiles per workgroup. Full contiguous tiles are software-pipelined: tile i + 1's raw buffer loads
  // are issued before tile i is counted (hand-counted waits), and nothing is stored until the loop is done -- the
  // workgroups of a one-shot grid otherwise run in lock step, all loading and then all computing.
  __shared__ uint32_t red[V1CT][V1T / 64];
  const uint32_t tid = threadIdx.x, t0 = blockIdx.x * V1CT;
  if (blockIdx.x == 0 && tid == 0) *nover = 0u;  // the oversized-tile list of k_encode1d_var_tile starts empty
  const bool wide_ok = F.vec && (((uintptr_t)F.data) & 15u) == 0;
  constexpr int NL = V1Raw<DT>::N;                                 // 16-byte loads per lane per tile
  constexpr uint32_t TB = V1TILE * (DT == DT_BF16 ? 8u : 16u);     // bytes per tile
  uint32_t packed[V1CT];
  if (wide_ok && (uint64_t)(t0 + V1CT) * V1TILE <= F.n[0] / 4) {
    const v1_v4i rs = v1_rsrc((const char*)F.data + (size_t)t0 * TB, V1CT * TB);
    // a ring of PF + 1 tiles: tile i + PF is requested before tile i is counted, so PF tiles of loads stay in flight
    constexpr uint32_t PF = V1_COUNT_PF, RING = PF + 1;
    v1_u4 buf[RING][NL];
#pragma unroll
    for (uint32_t i = 0; i < PF && i < V1CT; i++)
#pragma unroll
      for (int h = 0; h < NL; h++) buf[i][h] = v1_ld16(i * TB + (tid * NL + h) * 16u, rs);
#pragma unroll
    for (uint32_t i = 0; i < V1CT; i++) {
      if (i + PF < V1CT) {
#pragma unroll
        for (int h = 0; h < NL; h++) buf[(i + PF) % RING][h] = v1_ld16((i + PF) * TB + (tid * NL + h) * 16u, rs);
      }
      // loads issued after tile i's: those of tiles i + 1 .. min(i + PF, V1CT - 1)
      v1_wait_tiles<NL>(buf[i % RING], (i + PF < V1CT ? PF : V1CT - 1 - i));
      V1Raw<DT> cur;
#pragma unroll
      for (int h = 0; h < NL; h++) {
        const v1_u4 v = buf[i % RING][h];
        cur.w[h] = make_uint4(v.x, v.y, v.z, v.w);
      }
      uint32_t lsum;
      packed[i] = v1_count_tile<DT, true>(F, p, cur, t0 + i, lsum);
      lsum = wave_sum_dpp(lsum);
      if ((tid & 63u) == 0) red[i][tid >> 6] = lsum;
    }
  } else {  // partial tiles, the padded last block, strided or unaligned input
#pragma unroll
    for (uint32_t i = 0; i < V1CT; i++) {
      uint32_t lsum = 0;
      packed[i] = 0;
      if (t0 + i < ntiles) {
        V1Raw<DT> raw;
        raw.load(F, t0 + i, wide_ok);
        packed[i] = v1_count_tile<DT>(F, p, raw, t0 + i, lsum);
      }
      lsum = wave_sum_dpp(lsum);
      if ((tid & 63u) == 0) red[i][tid >> 6] = lsum;
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < V1CT; i++)
    if (t0 + i < ntiles) lens8[(size_t)(t0 + i) * V1T + tid] = packed[i];
  __syncthreads();
  if (tid < 64) {  // wave 0: the tile totals, and their sum for the scan's group totals
    uint64_t tot = 0;
    if (tid < V1CT && t0 + tid < ntiles) {
#pragma unroll
      for (uint32_t w = 0; w < V1T / 64; w++) tot += red[tid][w];
      sums[t0 + tid] = tot;
    }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)tot, o, 64), hi = __shfl_xor((uint32_t)(tot >> 32), o, 64);
      tot += (uint64_t)lo | ((uint64_t)hi << 32);
    }
    if (tid == 0) gsums[blockIdx.x] = tot;
  }
}

// One tile (raw words and the lane's byte lengths lw given) coded into the window `win`, from bit B & 127 (the
// 16-byte stream boundary below the tile's first bit); tab / rs already in LDS. Ends with the window complete
// (barrier) and the block index written.
template <int DT>
__device__ __forceinline__ void v1_tile_code(const FieldDesc& F, const Params& p, uint32_t t, uint64_t B,
                                             const V1Raw<DT>& raw, uint32_t lw, uint64_t* __restrict__ index,
                                             uint32_t index_shift, const uint32_t* tab, const uint32_t* rs,
                                             uint64_t* win, uint32_t* scan_sh, uint32_t* s_special)
{
  uint32_t* win32 = (uint32_t*)win;
  const uint32_t tid = threadIdx.x;
  const uint32_t lb = (uint32_t)(B & 127u);
  uint32_t len[V1U], lsum = 0;
#pragma unroll
  for (uint32_t k = 0; k < V1U; k++) {
    len[k] = (lw >> (8 * k)) & 255u;
    lsum += len[k];
  }
  uint32_t tot_unused;
  const uint32_t excl = lb + block_exclusive_scan<V1T, false>(lsum, &tot_unused, scan_sh);  // barrier below
  if (lsum) {  // the two words this lane shares with its neighbours start at zero
    win[excl >> 6] = 0ull;
    win[(excl + lsum - 1) >> 6] = 0ull;
  }
  if (tid == 0) *s_special = 0;
  __syncthreads();

  // ---- prepare and code the lane's blocks one at a time: a 64-bit accumulator; whole words are plain LDS stores,
  // the two shared ones ds_or
  const uint64_t bl = (uint64_t)t * V1TILE + (uint64_t)tid * V1U;
  const int cexp = -122 - p.minexp, maxprec = (int)min(p.maxprec, 64u);
  uint64_t acc = 0;
  uint32_t q = excl >> 6, fill = excl & 63u;
  const uint32_t qhead = q;
  uint32_t spmask = 0;
  [[maybe_unused]] uint64_t sink = 0;
#pragma unroll
  for (uint32_t k = 0; k < V1U; k++) {
    float f[4];
    raw.block(k, f);
    uint32_t u[4], hdr, K;
    bool inf;
    if constexpr ((V1_ABLATE & 16) != 0) {
      for (int i = 0; i < 4; i++) u[i] = __float_as_uint(f[i]);
      hdr = 3u + (u[0] >> 23);
      K = 16;
      inf = false;
    } else {
      (void)v1_prep(f, cexp, maxprec, u, hdr, K, inf);  // the length comes from the count pass
    }
    bool sp = inf && bl + k < F.nblocks;
    uint64_t c0, c1;
    if constexpr ((V1_ABLATE & 2) != 0) {  // measurement builds: no coder (the prepared words stand in for the code)
      c0 = ((uint64_t)u[1] << 32 | u[0]) ^ hdr;
      c1 = (uint64_t)u[3] << 32 | u[2];
      sp = false;
    } else {
      v1_code(u, hdr, len[k], K, tab, rs, c0, c1, sp);
    }
    sp = sp && len[k];
    if (sp) c0 = c1 = 0ull;  // coded below by the generic coder, OR-ed into these zero bits
    spmask |= (uint32_t)sp << k;
    acc |= c0 << fill;
    const uint64_t mid = ((c0 >> 1) >> (63u - fill)) | (c1 << fill);
    const uint64_t hi = (c1 >> 1) >> (63u - fill);
    const uint32_t nf = fill + len[k];
    if (nf >= 64u) {
      if constexpr ((V1_ABLATE & 128) != 0) sink ^= acc;
      else if (q == qhead) atomicOr((unsigned long long*)&win[q], (unsigned long long)acc);
      else win[q] = acc;
      q++;
      acc = mid;
      if (nf >= 128u) {
        if constexpr ((V1_ABLATE & 128) != 0) sink ^= acc;
        else win[q] = acc;
        q++;
        acc = hi;
        if (nf >= 192u) {  // a special block of up to 140 bits (its code is zero here) completes a third word
          if constexpr ((V1_ABLATE & 128) != 0) sink ^= acc;
          else win[q] = acc;
          q++;
          acc = 0ull;
        }
      }
    }
    fill = nf & 63u;
    acc &= (1ull << fill) - 1ull;
  }
  if constexpr ((V1_ABLATE & 128) != 0) win[qhead] = sink ^ acc;  // keeps the code alive
  else if (fill) atomicOr((unsigned long long*)&win[q], (unsigned long long)acc);
  if (spmask) *s_special = 1u;
  __syncthreads();
  if (*s_special) {  // Inf / NaN blocks, long group phases, codes past 128 bits: the generic coder
    uint32_t o = excl;
#pragma unroll
    for (uint32_t k = 0; k < V1U; k++) {
      if ((spmask >> k) & 1u) {
        float f[4];
        raw.block(k, f);
        LdsWriter wr{win32, o, o + len[k]};
        encode_block<1>(wr, f, p);
      }
      o += len[k];
    }
    __syncthreads();
  }
  if (index) {
    uint32_t o = excl;
#pragma unroll
    for (uint32_t k = 0; k < V1U; k++) {
      const uint64_t b = bl + k;
      if (len[k] && (b & ((1ull << index_shift) - 1ull)) == 0) index[b >> index_shift] = (B & ~127ull) + o;
      o += len[k];
    }
  }

}

// The window's 16-byte chunks c (stream words 4c .. 4c + 3 from word g0 = (B >> 7) * 4): the tile owns words kf .. kl;
// the first / last chunk holds words of the neighbouring tiles and the two words it shares with them (atomicOr), so
// those two chunks go word by word.
__device__ __forceinline__ void v1_edge_chunk(uint32_t c, const uint32_t* win32, uint32_t* __restrict__ out32,
                                              uint64_t g0, uint32_t kf, uint32_t kl, bool head_shared,
                                              bool tail_shared)
{
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t k = 4u * c + j;
    if (k < kf || k > kl) continue;
    const uint32_t val = win32[k];
    if ((k == kf && head_shared) || (k == kl && tail_shared)) atomicOr(out32 + g0 + k, val);
    else out32[g0 + k] = val;
  }
}

// Store the coded window of tile t (total bits from B): every interior chunk is one ds_read_b128 + one 16-byte store.
__device__ __forceinline__ void v1_tile_store(uint32_t t, uint64_t B, uint32_t total, const uint64_t* win,
                                              uint32_t* __restrict__ out32, uint32_t ntiles)
{
  const uint32_t* win32 = (const uint32_t*)win;
  const uint32_t tid = threadIdx.x;
  const uint32_t lb = (uint32_t)(B & 127u);
  // ---- store the window: 16-byte chunks of stream words from word g0 = (B >> 7) * 4, coalesced. The tile owns
  // words kf .. kl; the first / last chunk holds words of the neighbouring tiles and the two words it shares with
  // them (atomicOr), so those two chunks go word by word, every other chunk is one ds_read_b128 + one 16-byte store.
  const uint64_t g0 = (B >> 7) << 2;
  const uint32_t kf = lb >> 5, kl = (lb + total - 1u) >> 5;
  const bool head_shared = (lb & 31u) != 0;
  const bool last_tile = t == ntiles - 1;
  const bool tail_shared = ((lb + total) & 31u) != 0 && !last_tile;
  const uint32_t nch = (V1_ABLATE & 4) ? 0u : (kl >> 2) + 1u;
  const bool wide = (((uintptr_t)out32) & 15u) == 0;
  for (uint32_t c = tid; c < nch; c += V1T) {
    if (wide && c != 0 && c != nch - 1) *(uint4*)(out32 + g0 + 4u * c) = *(const uint4*)(win32 + 4u * c);
    else v1_edge_chunk(c, win32, out32, g0, kf, kl, head_shared, tail_shared);
  }
  if (last_tile && tid == 0) {
    const uint64_t endw = (B + total + 31) >> 5;
    if (endw & 1) out32[endw] = 0u;  // stream_flush: zero-pad to a 64-bit boundary (stream.c:132-138)
  }
}

// Load, code and store one tile.
template <int DT>
__device__ __forceinline__ void v1_tile(const FieldDesc& F, const Params& p, uint32_t t, uint64_t B, uint32_t total,
                                        const uint32_t* __restrict__ lens8, uint32_t* __restrict__ out32,
                                        uint64_t* __restrict__ index, uint32_t index_shift, uint32_t ntiles,
                                        const uint32_t* tab, const uint32_t* rs, uint64_t* win, uint32_t* scan_sh,
                                        uint32_t* s_special)
{
  const bool wide_ok = F.vec && (((uintptr_t)F.data) & 15u) == 0;
  V1Raw<DT> raw;
  uint32_t lw;
  if constexpr ((V1_ABLATE & 64) != 0) {  // measurement builds: no input or length loads (words from the tile index)
    const uint32_t h = (t * 2654435761u) ^ (threadIdx.x * 40503u);
#pragma unroll
    for (int i = 0; i < V1Raw<DT>::N; i++)  // normal values near 5e-4 (bf16 / fp32 halves: sign, exponent 0x74)
      raw.w[i] = make_uint4((h & 0x807f807fu) | 0x3a003a00u, ((h * 3u) & 0x807f807fu) | 0x3a003a00u,
                            ((h * 5u) & 0x807f807fu) | 0x3a003a00u, ((h * 7u) & 0x807f807fu) | 0x3a003a00u);
    lw = 0x3a3a3a3au;
  } else {
    raw.load(F, t, wide_ok);
    lw = lens8[(size_t)t * V1T + threadIdx.x];
  }
  v1_tile_code<DT>(F, p, t, B, raw, lw, index, index_shift, tab, rs, win, scan_sh, s_special);
  v1_tile_store(t, B, total, win, out32, ntiles);
}

// qwords of window a tile needs: its bits from bit B & 127 of the window (the 16-byte stream boundary below B), plus
// the two qwords the accumulator may touch past its last bit (a special block's zero third word)
__device__ __forceinline__ uint32_t v1_tile_qwords(uint64_t B, uint32_t total)
{
  return ((uint32_t)(B & 127u) + total + 63u) / 64u + 2u;
}

template <int DT>
__global__ __launch_bounds__(V1T) void k_encode1d_var_tile(FieldDesc F, Params p, const uint64_t* __restrict__ rbase,
                                                           const uint32_t* __restrict__ lens8,
                                                           uint32_t* __restrict__ out32, uint64_t* __restrict__ index,
                                                           uint32_t index_shift, uint32_t ntiles,
                                                           uint32_t* __restrict__ over)
{
  __shared__ __attribute__((aligned(16))) uint32_t tab[V1TAB];  // pair table rows 0..3 (lean-5 entries, row 3 empty)
  __shared__ uint32_t rs[1024];    // window spread tables
  __shared__ __attribute__((aligned(16))) uint64_t win[V1QS];  // the tile's code from bit base & 127 of its window
  __shared__ uint32_t scan_sh[V1T / 64];
  __shared__ uint32_t s_special;
  const uint32_t t = blockIdx.x;
  // every load the tile needs is issued before anything waits (one memory round trip per workgroup): the input rows,
  // the lane's byte lengths, the pair table, the tile's stream offsets
  V1Raw<DT> raw;
  raw.load(F, t, F.vec && (((uintptr_t)F.data) & 15u) == 0);
  const uint32_t lw = lens8[(size_t)t * V1T + threadIdx.x];
  stage_table<V1T, V1TAB>(tab, g_plane_tab_var.v);
#pragma unroll
  for (uint32_t i = 0; i < 1024 / V1T; i++) rs[threadIdx.x + V1T * i] = rspread_entry(threadIdx.x + V1T * i);
  const uint64_t B = rbase[t];
  const uint32_t total = (uint32_t)(rbase[t + 1] - B);
  if (v1_tile_qwords(B, total) > V1QS) {  // oversized: listed for k_encode1d_var_tile_big (over[0] = count)
    if (threadIdx.x == 0) over[1 + atomicAdd(over, 1u)] = t;
    return;
  }
  v1_tile_code<DT>(F, p, t, B, raw, lw, index, index_shift, tab, rs, win, scan_sh, &s_special);
  v1_tile_store(t, B, total, win, out32, ntiles);
}

template <int DT>
__global__ __launch_bounds__(V1T) void k_encode1d_var_tile_big(FieldDesc F, Params p,
                                                               const uint64_t* __restrict__ rbase,
                                                               const uint32_t* __restrict__ lens8,
                                                               uint32_t* __restrict__ out32,
                                                               uint64_t* __restrict__ index, uint32_t index_shift,
                                                               uint32_t ntiles, const uint32_t* __restrict__ over)
{
  __shared__ __attribute__((aligned(16))) uint32_t tab[V1TAB];
  __shared__ uint32_t rs[1024];
  __shared__ __attribute__((aligned(16))) uint64_t win[V1Q + 2];
  __shared__ uint32_t scan_sh[V1T / 64];
  __shared__ uint32_t s_special;
  const uint32_t n = over[0];
  if (blockIdx.x >= n) return;
  stage_table<V1T, V1TAB>(tab, g_plane_tab_var.v);
#pragma unroll
  for (uint32_t i = 0; i < 1024 / V1T; i++) rs[threadIdx.x + V1T * i] = rspread_entry(threadIdx.x + V1T * i);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t t = over[1 + i];
    const uint64_t B = rbase[t];
    const uint32_t total = (uint32_t)(rbase[t + 1] - B);
    v1_tile<DT>(F, p, t, B, total, lens8, out32, index, index_shift, ntiles, tab, rs, win, scan_sh, &s_special);
    __syncthreads();  // the window and scan slots are reused by the next tile
  }
}

// The tile form's workspace: sums[ntiles], base[ntiles + 1] (uint64), the oversized-tile list (count + ntiles
// uint32, rounded to 8 bytes), the byte lengths of whole tiles, then the totals of groups of 8 tiles.
static inline uint64_t v1_list_words(uint64_t ntiles) { return (ntiles + 2) / 2; }  // uint64 words

size_t var1d_tile_workspace_bytes(uint64_t nblocks)
{
  const uint64_t ntiles = (nblocks + V1TILE - 1) / V1TILE;
  return (size_t)((2 * ntiles + 2 + v1_list_words(ntiles) + (ntiles + V1CT - 1) / V1CT) * 8 + ntiles * V1TILE);
}

hipError_t launch_encode1d_var_tile(const FieldDesc& F, const Params& p, uint32_t* out32, uint64_t* ws,
                                    uint64_t* d_total, uint64_t* index, uint32_t index_shift, const uint64_t* d_base,
                                    void* stream)
{
  hipStream_t st = (hipStream_t)stream;
  const uint32_t ntiles = (uint32_t)((F.nblocks + V1TILE - 1) / V1TILE);
  uint64_t* sums = ws;
  uint64_t* base = ws + ntiles;
  uint32_t* over = (uint32_t*)(ws + 2 * (size_t)ntiles + 2);
  uint32_t* lens8 = (uint32_t*)(ws + 2 * (size_t)ntiles + 2 + v1_list_words(ntiles));
  uint64_t* gsums = (uint64_t*)(lens8 + (size_t)ntiles * V1T);
  const uint32_t ncw = (ntiles + V1CT - 1) / V1CT;
  if (F.dtype == DT_BF16) k_count1d_var_tile<DT_BF16><<<ncw, V1T, 0, st>>>(F, p, ntiles, sums, lens8, over, gsums);
  else k_count1d_var_tile<DT_F32><<<ncw, V1T, 0, st>>>(F, p, ntiles, sums, lens8, over, gsums);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_scan_ranges(sums, ntiles, base, d_total, out32, d_base, st, gsums);
  if (e != hipSuccess) return e;
  const uint32_t nbig = std::min(ntiles, 1280u);  // grid-stride workgroups of the oversized-tile pass (5 per CU)
  if (F.dtype == DT_BF16) {
    k_encode1d_var_tile<DT_BF16><<<ntiles, V1T, 0, st>>>(F, p, base, lens8, out32, index, index_shift, ntiles, over);
    k_encode1d_var_tile_big<DT_BF16><<<nbig, V1T, 0, st>>>(F, p, base, lens8, out32, index, index_shift, ntiles,
                                                           over);
  } else {
    k_encode1d_var_tile<DT_F32><<<ntiles, V1T, 0, st>>>(F, p, base, lens8, out32, index, index_shift, ntiles, over);
    k_encode1d_var_tile_big<DT_F32><<<nbig, V1T, 0, st>>>(F, p, base, lens8, out32, index, index_shift, ntiles, over);
  }
  return hipGetLastError();
}

}  // namespace gcow
