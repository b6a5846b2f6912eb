// Historical 1-D fixed-rate encoder variants (lean / lean-2 / lean-3 coders, per-lane, lockstep, persistent and
// non-persistent kernels) kept for the ablation microbenchmark only; the product uses the one-shot
// k_encode_fixed1d_np with the lean-5 coder (gcow_amd/csrc/gcow_kernels.hip). Included by ablate.hip after
// gcow_kernels.hip.
namespace gcow {

// ---- the persistent grid-stride lean-5 encoder (the product kernel before the one-shot grid)
// Persistent grid-stride encoder with NB rotating register buffers (prefetch depth NB): each step codes buffer k,
// stores the block, then refills buffer k with the block NB strides ahead. In steady state the block coded next was
// loaded NB steps ago and 2 (NB - 1) memory ops were issued after it, hence vmcnt(2 (NB - 1)). The caller keeps
// (nfull + NB * stride) * bytes-per-block below 2^32 (chunked launches).
template <int DT, uint32_t WB, int NB>
__global__ __launch_bounds__(256) void k_encode_fixed1d_pipe(const void* __restrict__ in, uint32_t nfull, Params p,
                                                             void* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
#pragma unroll
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab5.v[t];
  __syncthreads();
  constexpr uint32_t IB = DT == DT_BF16 ? 8u : 16u;  // input bytes per block
  const pipe_v4i rin = buf_rsrc(in, nfull * IB), rout = buf_rsrc(out, nfull * (WB / 8));
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  uint32_t bw = __builtin_amdgcn_readfirstlane(blockIdx.x * 256u + (threadIdx.x & ~63u));  // wave's first block
  if (bw >= nfull) return;
  typename PipeRow<DT>::T r[NB];
#pragma unroll
  for (int d = 0; d < NB; d++) r[d] = PipeRow<DT>::load((b + d * stride) * IB, rin);
#pragma unroll
  for (int d = 0; d < NB; d++) pipe_wait<0>(r[d]);
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      pipe_wait<2 * (NB - 1)>(r[k]);
      float f[4];
      PipeRow<DT>::unpack(r[k], f);
      bool special;
      uint64_t w = encode_block1d_lean5<WB>(f, tab2, special);
      if (special) {
        RegWriter64 rw{0ull, 0u};
        encode_block<1>(rw, f, p);
        w = WB == 64 ? rw.acc : (rw.acc & ((1ull << WB) - 1ull));
      }
      pipe_store<WB>(b * (WB / 8), rout, w);
      r[k] = PipeRow<DT>::load((b + NB * stride) * IB, rin);
      b += stride;
      bw += stride;
      if (bw >= nfull) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
      }
    }
  }
}


// ---- lean-4 coder and its pair table (the product default before the lean-5 coder)
__host__ __device__ constexpr PlaneTab2 make_plane_tab2()
{
  PlaneTab2 T{};
  for (uint32_t t = 0; t < 1280; t++) {
    const uint32_t n = t >> 8, b = t & 255u;
    const uint32_t e1 = plane_entry4_cx((n << 4) | (b & 15u));
    const uint32_t c1 = e1 & 127u, l1 = (e1 >> 7) & 7u, n1 = e1 >> 10;
    const uint32_t e2 = plane_entry4_cx((n1 << 4) | (b >> 4));
    const uint32_t c2 = e2 & 127u, l2 = (e2 >> 7) & 7u, n2 = e2 >> 10;
    T.v[t] = (c1 | (c2 << l1)) | ((l1 + l2) << 14) | (n2 << 18);
  }
  return T;
}

__device__ const PlaneTab2 g_plane_tab2 = make_plane_tab2();

// Lean-4 block. Two facts shorten the wave-uniform group-test loop of lean-3:
//  * with three coefficients significant (n = 3) a plane's code is its nibble verbatim: the three known bits, then
//    the group test for coefficient 3 -- which is that coefficient's bit, its own 1 being implied (encode.c:318-333);
//    so the group phase ends at plane T2 = max(L2, L3), not at L3;
//  * lanes whose group phase is over keep looking up plane pairs: rows n >= 3 of the pair table are verbatim, so the
//    extra iterations emit tail nibbles and the loop needs no per-lane activity masks; the tail then starts at the
//    same (wave-uniform) window nibble for every lane.
template <uint32_t WB>
__device__ __forceinline__ uint64_t encode_block1d_lean4(const float* f, const uint32_t* tab2, bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = m >= 0x7f800000u;  // Inf or NaN present
  const bool zero = m == 0;
  const uint32_t E = special ? 150u : (m >> 23);
  const bool tiny = E < 29u;
  const float s = __uint_as_float((283u - (tiny ? 150u : E)) << 23);
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = tiny ? (int32_t)0x80000000 : (int32_t)(f[i] * s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  uint64_t acc = 2ull * E + 3ull;
  const uint32_t o23 = u[2] | u[3];
  const int M0 = 31 - (int)__builtin_clz(u[0] | u[1] | o23 | 1u);
  const int T2 = o23 ? 31 - (int)__builtin_clz(o23) : 0;  // group phase: planes M0 .. max(T2, 0)
  uint32_t pos = 9 + (uint32_t)(31 - M0);
  const uint64_t Y = plane_window(u, (uint32_t)(31 - M0));
  const int jg = M0 - T2;
  uint32_t n = 0;
  int j = 0;
#pragma unroll
  for (; j < 16; j += 2) {
    if (!__any(j <= jg)) break;
    const uint32_t e = tab2[(n << 8) | ((uint32_t)(Y >> (4 * j)) & 255u)];
    const uint32_t code = pos < WB ? (e & 0x3fffu) : 0u;  // 64-bit shifts wrap: nothing past the budget
    acc |= (uint64_t)code << pos;
    pos += (e >> 14) & 15u;
    n = e >> 18;
  }
  special = special || (jg >= 16 && pos < WB);  // group phase runs past the 16-plane window (generic coder)
  if (j < 16 && pos < WB) acc |= (Y >> (4 * j)) << pos;  // rest of the window, verbatim
  const uint32_t p2 = pos + 4u * (uint32_t)(16 - j);        // where plane M0 - 16 lands
  if (__any(p2 < WB && M0 >= 16)) {
    const uint64_t Y2 = plane_window(u, (uint32_t)max(47 - M0, 0));  // planes M0 - 16 .. M0 - 31
    if (p2 < WB && M0 >= 16) acc |= Y2 << p2;
  }
  acc = zero ? 0ull : acc;
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}



// Lean 1-D fixed-rate block for parameters where every nonzero block has prec >= 32 (kmin = 0; the fixed-rate
// default maxprec 64 / minexp -1074). "Normal" blocks (biased exponent of max|x| in [29, 254], no NaN/Inf) take a
// straight path: the scale 2^(30 - emax) is finite and |x * scale| < 2^30, so the x86 INT_MIN corner cannot occur
// and the cast is a plain multiply + convert. Tiny / subnormal-max / NaN / Inf blocks return `special` and are
// coded by the generic per-block coder.
template <uint32_t WB>
__device__ __forceinline__ uint64_t encode_block1d_lean(const float* f, const uint16_t* tab, bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = (m - (29u << 23)) >= (0x7f800000u - (29u << 23));
  if (special) return 0;
  const uint32_t E = m >> 23;                      // emax = E - 126
  const float s = __uint_as_float((283u - E) << 23);  // 2^(30 - emax)
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = (int32_t)(f[i] * s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  uint64_t acc = 2ull * E + 3ull;  // 2 * (emax + 127) + 1
  const int M0 = 31 - (int)__builtin_clz(u[0] | u[1] | u[2] | u[3]);  // nonzero: max|q| >= 2^29
  const int L3 = u[3] ? 31 - (int)__builtin_clz(u[3]) : -1;
  uint32_t pos = 9 + (uint32_t)(31 - M0);  // empty planes above M0
  const uint64_t Y = plane_window(u, (uint32_t)(31 - M0));
  // group tests while n < 4: planes M0 .. max(L3, 0), i.e. window nibbles j = 0 .. M0 - max(L3, 0)
  const int jg = M0 - max(L3, 0);
  uint32_t n = 0;
  int j = 0;
  for (; j <= jg && pos < WB; ++j) {
    uint32_t x;
    if (j < 16) {
      x = (uint32_t)(Y >> (4 * j)) & 15u;
    } else {
      const int k = M0 - j;
      x = ((u[0] >> k) & 1u) | (((u[1] >> k) & 1u) << 1) | (((u[2] >> k) & 1u) << 2) | (((u[3] >> k) & 1u) << 3);
    }
    const uint32_t e = tab[(n << 4) | x];
    acc |= (uint64_t)(e & 127u) << pos;
    pos += (e >> 7) & 7u;
    n = e >> 10;
  }
  // all four significant (n = 4) from plane L3 - 1 down: verbatim nibbles, a contiguous run of the window
  if (pos < WB && L3 >= 0) {
    uint64_t field = j < 16 ? (Y >> (4 * j)) : 0ull;
    if (4u * (uint32_t)(16 - min(j, 16)) < WB - pos && M0 >= 16) {
      const uint64_t Y2 = plane_window(u, (uint32_t)(31 - M0 + 16));  // planes M0 - 16 .. M0 - 31
      field |= j <= 16 ? (Y2 << (64 - 4 * j)) : (Y2 >> (4 * (j - 16)));  // j >= 1 here
    }
    acc |= field << pos;
  }
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}

// Two-plane code table: entry (n, b) for b = nibble(plane k) | nibble(plane k-1) << 4 is the concatenated plane
// codes of both planes starting from significance count n: code[0:14) | len[14:18) | n'[18:21).
__device__ __forceinline__ uint32_t plane_entry4x2(uint32_t t)
{
  const uint32_t n = t >> 8, b = t & 255u;
  const uint32_t e1 = plane_entry4((n << 4) | (b & 15u));
  const uint32_t c1 = e1 & 127u, l1 = (e1 >> 7) & 7u, n1 = e1 >> 10;
  const uint32_t e2 = plane_entry4((n1 << 4) | (b >> 4));
  const uint32_t c2 = e2 & 127u, l2 = (e2 >> 7) & 7u, n2 = e2 >> 10;
  return (c1 | (c2 << l1)) | ((l1 + l2) << 14) | (n2 << 18);
}

// Lean block with the group phase run as a wave-uniform, predicated loop over plane pairs (no divergent exits).
template <uint32_t WB>
__device__ __forceinline__ uint64_t encode_block1d_lean2(const float* f, const uint32_t* tab2, bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = (m - (29u << 23)) >= (0x7f800000u - (29u << 23));
  const uint32_t E = special ? 150u : (m >> 23);  // special lanes run the arithmetic on a harmless exponent
  const float s = __uint_as_float((283u - E) << 23);
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = special ? 0 : (int32_t)(f[i] * s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  uint64_t acc = 2ull * E + 3ull;
  const uint32_t o = u[0] | u[1] | u[2] | u[3] | 1u;
  const int M0 = 31 - (int)__builtin_clz(o);
  const int L3 = u[3] ? 31 - (int)__builtin_clz(u[3]) : -1;
  uint32_t pos = 9 + (uint32_t)(31 - M0);
  const uint64_t Y = plane_window(u, (uint32_t)(31 - M0));
  const int jg = M0 - max(L3, 0);
  uint32_t n = 0;
  int jend = 0;
  uint64_t Y2 = 0;
  bool have2 = false;
#pragma unroll
  for (int j = 0; j < 32; j += 2) {
    const bool act = (j <= jg) && (pos < WB);
    if (!__any(act)) break;
    uint32_t b;
    if (j < 16) {
      b = (uint32_t)(Y >> (4 * j)) & 255u;
    } else {
      if (!have2) {
        Y2 = plane_window(u, (uint32_t)min(31 - M0 + 16, 31));
        have2 = true;
      }
      b = (M0 >= 16) ? ((uint32_t)(Y2 >> (4 * (j - 16))) & 255u) : 0u;
    }
    const uint32_t e = tab2[(n << 8) | b];
    const uint32_t len = act ? ((e >> 14) & 15u) : 0u;
    const uint64_t code = act ? (uint64_t)(e & 0x3fffu) : 0ull;
    acc |= code << pos;
    pos += len;
    n = act ? (e >> 18) : n;
    jend = act ? j + 2 : jend;
  }
  // all four significant from window nibble jend on: verbatim run of the window
  if (pos < WB && L3 >= 0) {
    uint64_t field;
    if (jend < 16) {
      field = Y >> (4 * jend);
      if (4u * (uint32_t)(16 - jend) < WB - pos && M0 >= 16) {
        if (!have2) Y2 = plane_window(u, (uint32_t)(31 - M0 + 16));
        field |= jend > 0 ? (Y2 << (64 - 4 * jend)) : 0ull;
      }
    } else {
      if (!have2) Y2 = M0 >= 16 ? plane_window(u, (uint32_t)(31 - M0 + 16)) : 0ull;
      field = M0 >= 16 ? (Y2 >> (4 * (jend - 16))) : 0ull;
    }
    acc |= field << pos;
  }
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}

// Persistent fixed-rate 1-D encoder: grid-stride over full blocks with the next block's load in flight while the
// current one is coded; the 2-plane table lives in LDS for the whole launch.
template <int DT, uint32_t WB>
__global__ __launch_bounds__(256) void k_encode_fixed1d_p(const void* __restrict__ in, uint32_t nfull, Params p,
                                                          void* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  __shared__ uint16_t tab[80];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = plane_entry4x2(t);
  if (threadIdx.x < 80) tab[threadIdx.x] = plane_entry4(threadIdx.x);
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float cur[4], nxt[4];
  if (b < nfull) load_row4<DT>(in, 4ll * b, cur);
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + stride;
    if (bn < nfull) load_row4<DT>(in, 4ll * bn, nxt);
    bool special;
    uint64_t w = encode_block1d_lean2<WB>(cur, tab2, special);
    if (special) w = encode_block1d_fixed<WB, 1>(cur, p, tab);
    if constexpr (WB == 64) ((uint64_t*)out)[b] = w;
    else ((uint32_t*)out)[b] = (uint32_t)w;
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = nxt[i];
  }
}

// U blocks per lane coded in lockstep: the per-block setup is straight-line and independent (ILP across blocks), the
// plane-pair loop advances all U blocks per iteration under one wave-uniform exit test, tails are O(1).
template <uint32_t WB, int U>
__device__ __forceinline__ void encode_blocks1d_lockstep(const float (*f)[4], const uint32_t* tab2, uint64_t* outw,
                                                         bool* special)
{
  uint32_t u[U][4];
  uint64_t acc[U], Y[U];
  uint32_t pos[U], n[U];
  int M0[U], L3[U], jg[U], jend[U];
#pragma unroll
  for (int t = 0; t < U; t++) {
    const uint32_t a0 = __float_as_uint(f[t][0]) & 0x7fffffffu, a1 = __float_as_uint(f[t][1]) & 0x7fffffffu;
    const uint32_t a2 = __float_as_uint(f[t][2]) & 0x7fffffffu, a3 = __float_as_uint(f[t][3]) & 0x7fffffffu;
    const uint32_t m = max(max(a0, a1), max(a2, a3));
    special[t] = (m - (29u << 23)) >= (0x7f800000u - (29u << 23));
    const uint32_t E = special[t] ? 150u : (m >> 23);
    const float s = __uint_as_float((283u - E) << 23);
    int32_t q[4];
#pragma unroll
    for (int i = 0; i < 4; i++) q[i] = special[t] ? 0 : (int32_t)(f[t][i] * s);
    fwd_lift(q[0], q[1], q[2], q[3]);
#pragma unroll
    for (int i = 0; i < 4; i++) u[t][i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
    acc[t] = 2ull * E + 3ull;
    M0[t] = 31 - (int)__builtin_clz(u[t][0] | u[t][1] | u[t][2] | u[t][3] | 1u);
    L3[t] = u[t][3] ? 31 - (int)__builtin_clz(u[t][3]) : -1;
    pos[t] = 9 + (uint32_t)(31 - M0[t]);
    Y[t] = plane_window(u[t], (uint32_t)(31 - M0[t]));
    jg[t] = M0[t] - max(L3[t], 0);
    n[t] = 0;
    jend[t] = 0;
  }
#pragma unroll
  for (int j = 0; j < 16; j += 2) {
    bool any = false;
#pragma unroll
    for (int t = 0; t < U; t++) any |= (j <= jg[t]) && (pos[t] < WB);
    if (!__any(any)) break;
#pragma unroll
    for (int t = 0; t < U; t++) {
      const bool act = (j <= jg[t]) && (pos[t] < WB);
      const uint32_t b = (uint32_t)(Y[t] >> (4 * j)) & 255u;
      const uint32_t e = tab2[(n[t] << 8) | b];
      const uint32_t len = act ? ((e >> 14) & 15u) : 0u;
      const uint64_t code = act ? (uint64_t)(e & 0x3fffu) : 0ull;
      acc[t] |= code << pos[t];
      pos[t] += len;
      n[t] = act ? (e >> 18) : n[t];
      jend[t] = act ? j + 2 : jend[t];
    }
  }
#pragma unroll
  for (int t = 0; t < U; t++) {
    // a group phase longer than the 16-plane window is left to the generic coder
    const bool deep = (jend[t] >= 16) && (jend[t] <= jg[t]) && (pos[t] < WB);
    special[t] = special[t] || deep;
    if (pos[t] < WB && L3[t] >= 0 && jend[t] < 16) {
      uint64_t field = Y[t] >> (4 * jend[t]);
      if (4u * (uint32_t)(16 - jend[t]) < WB - pos[t] && M0[t] >= 16 && jend[t] > 0) {
        const uint64_t Y2 = plane_window(u[t], (uint32_t)(31 - M0[t] + 16));
        field |= Y2 << (64 - 4 * jend[t]);
      }
      acc[t] |= field << pos[t];
    } else if (pos[t] < WB && L3[t] >= 0 && jend[t] >= 16 && M0[t] >= 16) {
      const uint64_t Y2 = plane_window(u[t], (uint32_t)(31 - M0[t] + 16));
      acc[t] |= (Y2 >> (4 * (jend[t] - 16))) << pos[t];
    }
    outw[t] = WB == 64 ? acc[t] : (acc[t] & ((1ull << WB) - 1ull));
  }
}

template <int DT, uint32_t WB, int U>
__global__ __launch_bounds__(256) void k_encode_fixed1d_u(const void* __restrict__ in, uint32_t nfull, Params p,
                                                          void* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  __shared__ uint16_t tab[80];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = plane_entry4x2(t);
  if (threadIdx.x < 80) tab[threadIdx.x] = plane_entry4(threadIdx.x);
  __syncthreads();
  // chunk c covers blocks [c * 256 * U, (c + 1) * 256 * U), lane-interleaved (coalesced); grid-stride over chunks
  const uint32_t chunk = 256u * U;
  const uint32_t nchunks = (nfull + chunk - 1) / chunk;
  uint32_t c = blockIdx.x;
  float cur[U][4], nxt[U][4];
  auto load_chunk = [&](uint32_t cc, float (*dst)[4]) {
#pragma unroll
    for (int t = 0; t < U; t++) {
      const uint32_t b = cc * chunk + 256u * t + threadIdx.x;
      if (b < nfull) load_row4<DT>(in, 4ll * b, dst[t]);
      else dst[t][0] = dst[t][1] = dst[t][2] = dst[t][3] = 0.0f;
    }
  };
  if (c < nchunks) load_chunk(c, cur);
  for (; c < nchunks; c += gridDim.x) {
    if (c + gridDim.x < nchunks) load_chunk(c + gridDim.x, nxt);
    uint64_t w[U];
    bool special[U];
    encode_blocks1d_lockstep<WB, U>(cur, tab2, w, special);
#pragma unroll
    for (int t = 0; t < U; t++) {
      const uint32_t b = c * chunk + 256u * t + threadIdx.x;
      if (b < nfull) {
        if (special[t]) w[t] = encode_block1d_fixed<WB, 1>(cur[t], p, tab);
        if constexpr (WB == 64) ((uint64_t*)out)[b] = w[t];
        else ((uint32_t*)out)[b] = (uint32_t)w[t];
      }
    }
#pragma unroll
    for (int t = 0; t < U; t++)
#pragma unroll
      for (int i = 0; i < 4; i++) cur[t][i] = nxt[t][i];
  }
}

// Lean-3 block: zero blocks and tiny blocks (emax <= -98, where sw/'s scale 2^(30 - emax) overflows to +inf and
// every x86 cast gives INT_MIN) are coded on the straight path; only blocks holding an Inf or NaN leave it.
template <uint32_t WB>
__device__ __forceinline__ uint64_t encode_block1d_lean3(const float* f, const uint32_t* tab2, bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = m >= 0x7f800000u;  // Inf or NaN present
  const bool zero = m == 0;
  const uint32_t E = special ? 150u : (m >> 23);  // biased exponent of max|x|; emax = max(E, 1) - 126
  const bool tiny = E < 29u;
  const float s = __uint_as_float((283u - (tiny ? 150u : E)) << 23);  // 2^(30 - emax) when finite
  int32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) q[i] = tiny ? (int32_t)0x80000000 : (int32_t)(f[i] * s);
  fwd_lift(q[0], q[1], q[2], q[3]);
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
  uint64_t acc = 2ull * E + 3ull;  // 2 * (emax + 127) + 1, also for subnormal maxima (E = 0 -> emax = -126)
  const int M0 = 31 - (int)__builtin_clz(u[0] | u[1] | u[2] | u[3] | 1u);
  const int L3 = u[3] ? 31 - (int)__builtin_clz(u[3]) : -1;
  uint32_t pos = 9 + (uint32_t)(31 - M0);
  const uint64_t Y = plane_window(u, (uint32_t)(31 - M0));
  const int jg = M0 - max(L3, 0);
  uint32_t n = 0;
  int jend = 0;
#pragma unroll
  for (int j = 0; j < 16; j += 2) {
    const bool act = (j <= jg) && (pos < WB);
    if (!__any(act)) break;
    const uint32_t b = (uint32_t)(Y >> (4 * j)) & 255u;
    const uint32_t e = tab2[(n << 8) | b];
    const uint32_t len = act ? ((e >> 14) & 15u) : 0u;
    const uint64_t code = act ? (uint64_t)(e & 0x3fffu) : 0ull;
    acc |= code << pos;
    pos += len;
    n = act ? (e >> 18) : n;
    jend = act ? j + 2 : jend;
  }
  special = special || ((jend >= 16) && (jend <= jg) && (pos < WB));  // group phase beyond the window
  if (pos < WB && L3 >= 0 && jend < 16) {
    uint64_t field = Y >> (4 * jend);
    if (4u * (uint32_t)(16 - jend) < WB - pos && M0 >= 16 && jend > 0)
      field |= plane_window(u, (uint32_t)(31 - M0 + 16)) << (64 - 4 * jend);
    acc |= field << pos;
  } else if (pos < WB && L3 >= 0 && jend >= 16 && M0 >= 16) {
    acc |= (plane_window(u, (uint32_t)(31 - M0 + 16)) >> (4 * (jend - 16))) << pos;
  }
  acc = zero ? 0ull : acc;  // all-zero block: a single 0 bit, padded
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}

template <uint32_t WB>
__device__ __noinline__ uint64_t encode_block1d_slow(const float* f, const Params p)
{
  RegWriter64 w{0ull, 0u};
  encode_block<1>(w, f, p);
  return WB == 64 ? w.acc : (w.acc & ((1ull << WB) - 1ull));
}

// Persistent fixed-rate 1-D encoder (lean-3): grid-stride over full blocks, next block's load in flight.
template <int DT, uint32_t WB>
__global__ __launch_bounds__(256) void k_encode_fixed1d_l3(const void* __restrict__ in, uint32_t nfull, Params p,
                                                           void* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = plane_entry4x2(t);
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float cur[4], nxt[4];
  if (b < nfull) load_row4<DT>(in, 4ll * b, cur);
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + stride;
    if (bn < nfull) load_row4<DT>(in, 4ll * bn, nxt);
    bool special;
    uint64_t w = encode_block1d_lean3<WB>(cur, tab2, special);
    if (special) w = encode_block1d_slow<WB>(cur, p);
    if constexpr (WB == 64) ((uint64_t*)out)[b] = w;
    else ((uint32_t*)out)[b] = (uint32_t)w;
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = nxt[i];
  }
}

typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef unsigned int nt_u2 __attribute__((ext_vector_type(2)));

template <int DT>
__device__ __forceinline__ void load_row4_nt(const void* base, int64_t off, float* f)
{
  if constexpr (DT == DT_BF16) {
    const nt_u2 v = __builtin_nontemporal_load((const nt_u2*)((const uint16_t*)base + off));
    f[0] = __uint_as_float(v.x << 16);
    f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16);
    f[3] = __uint_as_float(v.y & 0xffff0000u);
  } else {
    const nt_f4 v = __builtin_nontemporal_load((const nt_f4*)((const float*)base + off));
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
}

// Non-persistent fixed-rate 1-D encoder: one 4-value block per lane, non-temporal streaming loads/stores (the form
// that reached 6.06 TB/s as a pure load/store floor), lean-3 coder, inline Inf/NaN path.
template <int DT, uint32_t WB>
__global__ __launch_bounds__(256) void k_encode_fixed1d_np(const void* __restrict__ in, uint32_t nfull, Params p,
                                                           void* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  const uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float f[4] = {0, 0, 0, 0};
  if (b < nfull) load_row4_nt<DT>(in, 4ll * b, f);
#pragma unroll
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  __syncthreads();
  if (b >= nfull) return;
  bool special;
  uint64_t w = encode_block1d_lean3<WB>(f, tab2, special);
  if (special) {
    RegWriter64 rw{0ull, 0u};
    encode_block<1>(rw, f, p);
    w = WB == 64 ? rw.acc : (rw.acc & ((1ull << WB) - 1ull));
  }
  if constexpr (WB == 64) __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
  else __builtin_nontemporal_store((uint32_t)w, (uint32_t*)out + b);
}

// Persistent fixed-rate 1-D encoder (lean-3, inline Inf/NaN path, non-temporal streaming loads/stores).
template <int DT, uint32_t WB>
__global__ __launch_bounds__(256) void k_encode_fixed1d_pnt(const void* __restrict__ in, uint32_t nfull, Params p,
                                                            void* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
#pragma unroll
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float cur[4], nxt[4];
  if (b < nfull) load_row4_nt<DT>(in, 4ll * b, cur);
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + stride;
    if (bn < nfull) load_row4_nt<DT>(in, 4ll * bn, nxt);
    bool special;
    uint64_t w = encode_block1d_lean3<WB>(cur, tab2, special);
    if (special) {
      RegWriter64 rw{0ull, 0u};
      encode_block<1>(rw, cur, p);
      w = WB == 64 ? rw.acc : (rw.acc & ((1ull << WB) - 1ull));
    }
    if constexpr (WB == 64) __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
    else __builtin_nontemporal_store((uint32_t)w, (uint32_t*)out + b);
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = nxt[i];
  }
}


}  // namespace gcow
