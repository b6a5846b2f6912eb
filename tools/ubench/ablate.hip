// Ablation microbenchmark for the 1-D fixed-rate encoder (not part of libgcow.so): stage-by-stage cost of
// load/store, block setup (emax, cast, lift, negabinary), plane window transpose, group phase, tail.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../gcow_amd/csrc/gcow_kernels.hip"
#include "../../gcow_amd/csrc/gcow_blocks.hip"
#include "legacy_variants.hip"

namespace gcow {

template <int MODE>
__global__ __launch_bounds__(256) void k_ablate(const float4* __restrict__ in, uint32_t nfull, uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = plane_entry4x2(t);
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float4 cur = b < nfull ? in[b] : make_float4(0, 0, 0, 0);
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + stride;
    float4 nxt = bn < nfull ? in[bn] : make_float4(0, 0, 0, 0);
    float f[4] = {cur.x, cur.y, cur.z, cur.w};
    uint64_t w;
    if constexpr (MODE == 0) {
      w = (uint64_t)(__float_as_uint(f[0]) ^ __float_as_uint(f[1])) |
          ((uint64_t)(__float_as_uint(f[2]) ^ __float_as_uint(f[3])) << 32);
    } else if constexpr (MODE == 4) {
      bool sp;
      w = encode_block1d_lean2<64>(f, tab2, sp);
    } else {
      const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
      const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
      const uint32_t m = max(max(a0, a1), max(a2, a3));
      const bool special = (m - (29u << 23)) >= (0x7f800000u - (29u << 23));
      const uint32_t E = special ? 150u : (m >> 23);
      const float s = __uint_as_float((283u - E) << 23);
      int32_t q[4];
      for (int i = 0; i < 4; i++) q[i] = special ? 0 : (int32_t)(f[i] * s);
      fwd_lift(q[0], q[1], q[2], q[3]);
      uint32_t u[4];
      for (int i = 0; i < 4; i++) u[i] = ((uint32_t)q[i] + 0xaaaaaaaau) ^ 0xaaaaaaaau;
      if constexpr (MODE == 1) {
        w = (uint64_t)(u[0] ^ u[1]) | ((uint64_t)(u[2] ^ u[3]) << 32) | E;
      } else {
        const int M0 = 31 - (int)__builtin_clz(u[0] | u[1] | u[2] | u[3] | 1u);
        const int L3 = u[3] ? 31 - (int)__builtin_clz(u[3]) : -1;
        const uint64_t Y = plane_window(u, (uint32_t)(31 - M0));
        if constexpr (MODE == 2) {
          w = Y ^ (uint64_t)(M0 + L3);
        } else {  // MODE 3: group phase only
          uint64_t acc = 2ull * E + 3ull;
          uint32_t pos = 9 + (uint32_t)(31 - M0), n = 0;
          const int jg = M0 - max(L3, 0);
          for (int j = 0; j < 16; j += 2) {
            const bool act = (j <= jg) && (pos < 64);
            if (!__any(act)) break;
            const uint32_t bb = (uint32_t)(Y >> (4 * j)) & 255u;
            const uint32_t e = tab2[(n << 8) | bb];
            const uint32_t len = act ? ((e >> 14) & 15u) : 0u;
            const uint64_t code = act ? (uint64_t)(e & 0x3fffu) : 0ull;
            acc |= code << pos;
            pos += len;
            n = act ? (e >> 18) : n;
          }
          w = acc ^ pos;
        }
      }
    }
    out[b] = w;
    cur = nxt;
  }
}

}  // namespace gcow

typedef float nf4 __attribute__((ext_vector_type(4)));
typedef unsigned int nu4 __attribute__((ext_vector_type(4)));
typedef unsigned int nu2 __attribute__((ext_vector_type(2)));
namespace gcow {
// memory floors: 2 adjacent blocks per lane (2 x 16 B loads, one 16 B store), optionally non-temporal
template <bool NT>
__global__ __launch_bounds__(256) void k_floor2(const float4* __restrict__ in, uint32_t npairs, uint4* __restrict__ out)
{
  const uint32_t stride = gridDim.x * 256u;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < npairs; i += stride) {
    const nf4* pin = (const nf4*)in;
    nf4 a, b;
    if (NT) {
      a = __builtin_nontemporal_load(&pin[2 * i]);
      b = __builtin_nontemporal_load(&pin[2 * i + 1]);
    } else {
      a = pin[2 * i];
      b = pin[2 * i + 1];
    }
    nu4 w;
    w.x = __float_as_uint(a.x) ^ __float_as_uint(a.y); w.y = __float_as_uint(a.z) ^ __float_as_uint(a.w);
    w.z = __float_as_uint(b.x) ^ __float_as_uint(b.y); w.w = __float_as_uint(b.z) ^ __float_as_uint(b.w);
    if (NT) __builtin_nontemporal_store(w, &((nu4*)out)[i]);
    else ((nu4*)out)[i] = w;
  }
}
template <bool NT>
__global__ __launch_bounds__(256) void k_floor1(const float4* __restrict__ in, uint32_t n, uint2* __restrict__ out)
{
  const uint32_t stride = gridDim.x * 256u;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += stride) {
    const nf4* pin = (const nf4*)in;
    nf4 a = NT ? __builtin_nontemporal_load(&pin[i]) : pin[i];
    nu2 w;
    w.x = __float_as_uint(a.x) ^ __float_as_uint(a.y); w.y = __float_as_uint(a.z) ^ __float_as_uint(a.w);
    if (NT) __builtin_nontemporal_store(w, &((nu2*)out)[i]);
    else ((nu2*)out)[i] = w;
  }
}
// compute floor of the lean-3 coder: inputs re-read from a 1 MiB L2-resident window, results folded per lane
template <int K>
__global__ __launch_bounds__(256) void k_compute_floor(const float4* __restrict__ in, uint32_t nfull,
                                                       uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  uint64_t accx = 0;
  for (; b < nfull; b += stride) {
    const float4 v = in[b & 0xffffu];
    float f[4] = {v.x, v.y, v.z, v.w};
    bool sp;
    uint64_t w = encode_block1d_lean3<64>(f, tab2, sp);
    if (K == 1 && sp) {
      RegWriter64 rw{0ull, 0u};
      Params p{64, 64, 64, -1074};
      encode_block<1>(rw, f, p);
      w = rw.acc;
    }
    accx ^= w + b;
  }
  out[blockIdx.x * 256u + threadIdx.x] = accx;
}

// timing-only variants of the lean-3 coder (outputs not exact unless noted):
//   F & 1: group-phase LDS address independent of the previous lookup (latency chain removed)
//   F & 2: no second plane window (Y2)
//   F & 4: group phase skipped
template <int F>
__device__ __forceinline__ uint64_t lean3_var(const float* f, const uint32_t* tab2)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  const bool special = m >= 0x7f800000u;
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
  const int M0 = 31 - (int)__builtin_clz(u[0] | u[1] | u[2] | u[3] | 1u);
  const int L3 = u[3] ? 31 - (int)__builtin_clz(u[3]) : -1;
  uint32_t pos = 9 + (uint32_t)(31 - M0);
  const uint64_t Y = plane_window(u, (uint32_t)(31 - M0));
  const int jg = M0 - max(L3, 0);
  uint32_t n = 0;
  int jend = 0;
  if constexpr (!(F & 4)) {
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const bool act = (j <= jg) && (pos < 64);
      if (!__any(act)) break;
      const uint32_t b = (uint32_t)(Y >> (4 * j)) & 255u;
      const uint32_t e = (F & 1) ? tab2[((j & 3) << 8) | b] : tab2[(n << 8) | b];
      const uint32_t len = act ? ((e >> 14) & 15u) : 0u;
      const uint64_t code = act ? (uint64_t)(e & 0x3fffu) : 0ull;
      acc |= code << pos;
      pos += len;
      n = act ? (e >> 18) : n;
      jend = act ? j + 2 : jend;
    }
  } else {
    jend = (jg + 2) & ~1;
    pos += 2 * jend;
  }
  if (pos < 64 && L3 >= 0 && jend < 16) {
    uint64_t field = Y >> (4 * jend);
    if (!(F & 2))
      if (4u * (uint32_t)(16 - jend) < 64 - pos && M0 >= 16 && jend > 0)
        field |= plane_window(u, (uint32_t)(31 - M0 + 16)) << (64 - 4 * jend);
    acc |= field << pos;
  }
  acc = zero ? 0ull : acc;
  return special ? 0ull : acc;
}

template <int F>
__global__ __launch_bounds__(256) void k_var(const void* __restrict__ in, uint32_t nfull, uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float cur[4], nxt[4];
  if (b < nfull) load_row4_nt<DT_F32>(in, 4ll * b, cur);
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + stride;
    if (bn < nfull) load_row4_nt<DT_F32>(in, 4ll * bn, nxt);
    const uint64_t w = lean3_var<F>(cur, tab2);
    __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = nxt[i];
  }
}

// exact: two blocks per lane per iteration (b and b + stride), lean-3 coder on each
__global__ __launch_bounds__(256) void k_u2(const void* __restrict__ in, uint32_t nfull, Params p, uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  __syncthreads();
  const uint32_t stride = gridDim.x * 512u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float c0[4], c1[4], n0[4], n1[4];
  if (b < nfull) load_row4_nt<DT_F32>(in, 4ll * b, c0);
  if (b + stride / 2 < nfull) load_row4_nt<DT_F32>(in, 4ll * (b + stride / 2), c1);
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + stride, b1 = b + stride / 2;
    if (bn < nfull) load_row4_nt<DT_F32>(in, 4ll * bn, n0);
    if (bn + stride / 2 < nfull) load_row4_nt<DT_F32>(in, 4ll * (bn + stride / 2), n1);
    bool s0, s1;
    uint64_t w0 = encode_block1d_lean3<64>(c0, tab2, s0);
    uint64_t w1 = encode_block1d_lean3<64>(c1, tab2, s1);
    if (s0) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, c0, p); w0 = rw.acc; }
    if (s1) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, c1, p); w1 = rw.acc; }
    __builtin_nontemporal_store((unsigned long long)w0, (unsigned long long*)out + b);
    if (b1 < nfull) __builtin_nontemporal_store((unsigned long long)w1, (unsigned long long*)out + b1);
#pragma unroll
    for (int i = 0; i < 4; i++) { c0[i] = n0[i]; c1[i] = n1[i]; }
  }
}

struct PlaneTab1 {
  uint16_t v[80];
};
__host__ __device__ constexpr PlaneTab1 make_plane_tab1()
{
  PlaneTab1 T{};
  for (uint32_t t = 0; t < 80; t++) T.v[t] = (uint16_t)plane_entry4_cx(t);
  return T;
}
__device__ const PlaneTab1 g_plane_tab1 = make_plane_tab1();

// exact lean coder with the one-plane table (80 x u16): code[0:7) | len[7:10) | n'[10:13)
template <uint32_t WB>
__device__ __forceinline__ uint64_t lean5(const float* f, const uint16_t* tab, bool& special)
{
  const uint32_t a0 = __float_as_uint(f[0]) & 0x7fffffffu, a1 = __float_as_uint(f[1]) & 0x7fffffffu;
  const uint32_t a2 = __float_as_uint(f[2]) & 0x7fffffffu, a3 = __float_as_uint(f[3]) & 0x7fffffffu;
  const uint32_t m = max(max(a0, a1), max(a2, a3));
  special = m >= 0x7f800000u;
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
  const int M0 = 31 - (int)__builtin_clz(u[0] | u[1] | u[2] | u[3] | 1u);
  const int L3 = u[3] ? 31 - (int)__builtin_clz(u[3]) : -1;
  uint32_t pos = 9 + (uint32_t)(31 - M0);
  const uint64_t Y = plane_window(u, (uint32_t)(31 - M0));
  const int jg = M0 - max(L3, 0);
  uint32_t n = 0;
  int jend = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const bool act = (j <= jg) && (pos < WB);
    if (!__any(act)) break;
    const uint32_t x = (uint32_t)(Y >> (4 * j)) & 15u;
    const uint32_t e = tab[(n << 4) | x];
    const uint32_t len = act ? ((e >> 7) & 7u) : 0u;
    const uint64_t code = act ? (uint64_t)(e & 127u) : 0ull;
    acc |= code << pos;
    pos += len;
    n = act ? (e >> 10) : n;
    jend = act ? j + 1 : jend;
  }
  special = special || ((jend >= 16) && (jend <= jg) && (pos < WB));
  if (pos < WB && L3 >= 0 && jend < 16) {
    uint64_t field = Y >> (4 * jend);
    if (4u * (uint32_t)(16 - jend) < WB - pos && M0 >= 16 && jend > 0)
      field |= plane_window(u, (uint32_t)(31 - M0 + 16)) << (64 - 4 * jend);
    acc |= field << pos;
  } else if (pos < WB && L3 >= 0 && jend >= 16 && M0 >= 16) {
    acc |= (plane_window(u, (uint32_t)(31 - M0 + 16)) >> (4 * (jend - 16))) << pos;
  }
  acc = zero ? 0ull : acc;
  return WB == 64 ? acc : (acc & ((1ull << WB) - 1ull));
}

// non-persistent, K blocks per lane (lane t of WG g codes blocks g*256K + t + 256i), one-plane table
template <int K>
__global__ __launch_bounds__(256) void k_np1(const void* __restrict__ in, uint32_t nfull, Params p,
                                              uint64_t* __restrict__ out)
{
  __shared__ uint16_t tab[80];
  const uint32_t b0 = blockIdx.x * (256u * K) + threadIdx.x;
  float f[K][4];
#pragma unroll
  for (int i = 0; i < K; i++)
    if (b0 + 256u * i < nfull) load_row4_nt<DT_F32>(in, 4ll * (b0 + 256u * i), f[i]);
  if (threadIdx.x < 80) tab[threadIdx.x] = g_plane_tab1.v[threadIdx.x];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K; i++) {
    const uint32_t b = b0 + 256u * i;
    if (b >= nfull) break;
    bool sp;
    uint64_t w = lean5<64>(f[i], tab, sp);
    if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, f[i], p); w = rw.acc; }
    __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
  }
}

// persistent with the one-plane table (isolates the table size from the launch shape)
__global__ __launch_bounds__(256) void k_p1(const void* __restrict__ in, uint32_t nfull, Params p,
                                             uint64_t* __restrict__ out)
{
  __shared__ uint16_t tab[80];
  if (threadIdx.x < 80) tab[threadIdx.x] = g_plane_tab1.v[threadIdx.x];
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float cur[4], nxt[4];
  if (b < nfull) load_row4_nt<DT_F32>(in, 4ll * b, cur);
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + stride;
    if (bn < nfull) load_row4_nt<DT_F32>(in, 4ll * bn, nxt);
    bool sp;
    uint64_t w = lean5<64>(cur, tab, sp);
    if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, cur, p); w = rw.acc; }
    __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = nxt[i];
  }
}

// persistent, prefetch depth D (D iterations of loads in flight), lean-3 coder, exact
template <int D>
__global__ __launch_bounds__(256) void k_pd(const void* __restrict__ in, uint32_t nfull, Params p,
                                             uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  float r[D + 1][4];
#pragma unroll
  for (int d = 0; d < D; d++)
    if (b + d * stride < nfull) load_row4_nt<DT_F32>(in, 4ll * (b + d * stride), r[d]);
  __syncthreads();
  for (; b < nfull; b += stride) {
    const uint32_t bn = b + D * stride;
    if (bn < nfull) load_row4_nt<DT_F32>(in, 4ll * bn, r[D]);
    bool sp;
    uint64_t w = encode_block1d_lean3<64>(r[0], tab2, sp);
    if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, r[0], p); w = rw.acc; }
    __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
#pragma unroll
    for (int d = 0; d < D; d++)
#pragma unroll
      for (int i = 0; i < 4; i++) r[d][i] = r[d + 1][i];
  }
}

// persistent, prefetch depth D with UNCONDITIONAL (index-clamped) prefetch loads, so the waitcnt pass can keep the
// prefetches in flight (a conditional load forces s_waitcnt vmcnt(0) at the merge), lean-3 coder, exact
template <int D>
__global__ __launch_bounds__(256) void k_pdu(const void* __restrict__ in, uint32_t nfull, Params p,
                                              uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  const uint32_t last = nfull - 1;
  float r[D + 1][4];
#pragma unroll
  for (int d = 0; d < D; d++) load_row4_nt<DT_F32>(in, 4ll * min(b + d * stride, last), r[d]);
  __syncthreads();
  for (; b < nfull; b += stride) {
    load_row4_nt<DT_F32>(in, 4ll * min(b + D * stride, last), r[D]);
    bool sp;
    uint64_t w = encode_block1d_lean3<64>(r[0], tab2, sp);
    if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, r[0], p); w = rw.acc; }
    __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
#pragma unroll
    for (int d = 0; d < D; d++)
#pragma unroll
      for (int i = 0; i < 4; i++) r[d][i] = r[d + 1][i];
  }
}

// persistent, NB rotating register buffers without register moves (loop unrolled NB times), prefetch depth NB - 1
template <int NB>
__global__ __launch_bounds__(256) void k_rot(const void* __restrict__ in, uint32_t nfull, Params p,
                                              uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  const uint32_t last = nfull - 1;
  float r[NB][4];
#pragma unroll
  for (int d = 0; d < NB - 1; d++) load_row4_nt<DT_F32>(in, 4ll * min(b + d * stride, last), r[d]);
  __syncthreads();
  if (b >= nfull) return;
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      load_row4_nt<DT_F32>(in, 4ll * min(b + (NB - 1) * stride, last), r[(k + NB - 1) % NB]);
      bool sp;
      uint64_t w = encode_block1d_lean3<64>(r[k], tab2, sp);
      if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, r[k], p); w = rw.acc; }
      __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
      b += stride;
      if (b >= nfull) return;
    }
  }
}

// as k_rot, but each step refills the buffer it just coded (after its store): no load at the loop head
template <int NB>
__global__ __launch_bounds__(256) void k_rot2(const void* __restrict__ in, uint32_t nfull, Params p,
                                               uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  const uint32_t last = nfull - 1;
  float r[NB][4];
#pragma unroll
  for (int d = 0; d < NB; d++) load_row4_nt<DT_F32>(in, 4ll * min(b + d * stride, last), r[d]);
  __syncthreads();
  if (b >= nfull) return;
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      bool sp;
      uint64_t w = encode_block1d_lean3<64>(r[k], tab2, sp);
      if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, r[k], p); w = rw.acc; }
      __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
      load_row4_nt<DT_F32>(in, 4ll * min(b + NB * stride, last), r[k]);
      b += stride;
      if (b >= nfull) return;
    }
  }
}

// k_rot2 + explicit counted waits at the loop edges so that the loop header needs no wait of its own
template <int NB>
__global__ __launch_bounds__(256) void k_rot3(const void* __restrict__ in, uint32_t nfull, Params p,
                                               uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  const uint32_t last = nfull - 1;
  float r[NB][4];
#pragma unroll
  for (int d = 0; d < NB; d++) load_row4_nt<DT_F32>(in, 4ll * min(b + d * stride, last), r[d]);
  __syncthreads();
  if (b >= nfull) return;
  __builtin_amdgcn_s_waitcnt(0xF70 | (NB - 1));  // r[0] landed
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      bool sp;
      uint64_t w = encode_block1d_lean3<64>(r[k], tab2, sp);
      if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, r[k], p); w = rw.acc; }
      __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
      load_row4_nt<DT_F32>(in, 4ll * min(b + NB * stride, last), r[k]);
      b += stride;
      if (b >= nfull) return;
    }
    __builtin_amdgcn_s_waitcnt(0xF70 | (2 * (NB - 1)));  // r[0] (refilled in step 0) landed
  }
}

// k_rot2 with a wave-uniform loop exit (scalar trip test on the wave's first block), predicated store
template <int NB>
__global__ __launch_bounds__(256) void k_rot4(const void* __restrict__ in, uint32_t nfull, Params p,
                                               uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  uint32_t bw = __builtin_amdgcn_readfirstlane(blockIdx.x * 256u + (threadIdx.x & ~63u));
  const uint32_t last = nfull - 1;
  float r[NB][4];
#pragma unroll
  for (int d = 0; d < NB; d++) load_row4_nt<DT_F32>(in, 4ll * min(b + d * stride, last), r[d]);
  __syncthreads();
  if (bw >= nfull) return;
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      bool sp;
      uint64_t w = encode_block1d_lean3<64>(r[k], tab2, sp);
      if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, r[k], p); w = rw.acc; }
      if (b < nfull) __builtin_nontemporal_store((unsigned long long)w, (unsigned long long*)out + b);
      load_row4_nt<DT_F32>(in, 4ll * min(b + NB * stride, last), r[k]);
      b += stride;
      bw += stride;
      if (bw >= nfull) return;
    }
  }
}

// Hand-counted memory pipeline: buffer loads/stores issued by inline asm (invisible to the compiler's waitcnt pass)
// with explicit s_waitcnt vmcnt(2 (NB - 1)) per step; out-of-range lanes load zeros / their stores are dropped by the
// buffer range check, so the loop exit is wave-uniform and every step issues exactly one load and one store.
typedef int abl_v4i __attribute__((ext_vector_type(4)));
typedef float abl_v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ abl_v4i abl_rsrc(const void* p, uint32_t bytes)
{
  const uint64_t a = (uint64_t)p;
  abl_v4i r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((uint32_t)(a >> 32) & 0xffffu);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ abl_v4f abl_load(uint32_t off, abl_v4i rs)
{
  abl_v4f v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(rs) : "memory");
  return v;
}
__device__ __forceinline__ void abl_store(uint32_t off, abl_v4i rs, uint64_t w)
{
  asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen nt" : : "v"(w), "v"(off), "s"(rs) : "memory");
}
template <int N>
__device__ __forceinline__ void abl_wait(abl_v4f& v)
{
  asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v) : "n"(N) : "memory");
}

template <int NB, int MODE = 0>
__global__ __launch_bounds__(256) void k_asm(const void* __restrict__ in, uint32_t nfull, Params p,
                                              uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = g_plane_tab2.v[t];
  __syncthreads();
  const abl_v4i rin = abl_rsrc(in, nfull * 16u), rout = abl_rsrc(out, nfull * 8u);
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  uint32_t bw = __builtin_amdgcn_readfirstlane(blockIdx.x * 256u + (threadIdx.x & ~63u));
  if (bw >= nfull) return;
  abl_v4f r[NB];
#pragma unroll
  for (int d = 0; d < NB; d++) r[d] = abl_load((b + d * stride) * 16u, rin);
#pragma unroll
  for (int d = 0; d < NB; d++) abl_wait<0>(r[d]);
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      abl_wait<2 * (NB - 1)>(r[k]);
      float f[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
      bool sp;
      uint64_t w;
      if constexpr (MODE == 2) {
        w = (uint64_t)(__float_as_uint(f[0]) ^ __float_as_uint(f[1])) |
            ((uint64_t)(__float_as_uint(f[2]) ^ __float_as_uint(f[3])) << 32);
      } else {
        w = encode_block1d_lean3<64>(f, tab2, sp);
        if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, f, p); w = rw.acc; }
      }
      const uint32_t sb = MODE == 1 ? (b & 0xffffu) : b;  // MODE 1: L2-resident working set (compute floor)
      const uint32_t lb = MODE == 1 ? ((b + NB * stride) & 0xffffu) : (b + NB * stride);
      abl_store(sb * 8u, rout, w);
      r[k] = abl_load(lb * 16u, rin);
      b += stride;
      bw += stride;
      if (bw >= nfull) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
      }
    }
  }
}


// non-persistent lean-5: each lane codes U blocks (256 apart inside its workgroup's chunk), all loads issued first
template <int U>
__global__ __launch_bounds__(256) void k_np5(const void* __restrict__ in, uint32_t nfull, Params p, void* __restrict__ out)
{
  __shared__ uint32_t tab[1280];
  const abl_v4i rin = abl_rsrc(in, nfull * 16u), rout = abl_rsrc(out, nfull * 8u);
  const uint32_t b0 = blockIdx.x * (256u * U) + threadIdx.x;
  abl_v4f r[U];
#pragma unroll
  for (int k = 0; k < U; k++) r[k] = abl_load((b0 + 256u * k) * 16u, rin);
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab[t] = g_plane_tab5.v[t];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < U; k++) {
    abl_wait<U - 1>(r[k]);
    float f[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
    bool sp;
    uint64_t w = encode_block1d_lean5<64>(f, tab, sp);
    if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, f, p); w = rw.acc; }
    abl_store((b0 + 256u * k) * 8u, rout, w);
  }
}

// persistent lean-5 over contiguous per-workgroup chunks (stride 256 blocks) instead of a grid stride
template <int NB>
__global__ __launch_bounds__(256) void k_chunk5(const void* __restrict__ in, uint32_t nfull, Params p, void* __restrict__ out)
{
  __shared__ uint32_t tab[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab[t] = g_plane_tab5.v[t];
  __syncthreads();
  const uint32_t per = ((nfull + gridDim.x - 1) / gridDim.x + 255u) & ~255u;
  const uint32_t lo = blockIdx.x * per, hi = min(nfull, lo + per);
  const abl_v4i rin = abl_rsrc(in, hi * 16u), rout = abl_rsrc(out, hi * 8u);
  uint32_t b = lo + threadIdx.x;
  uint32_t bw = lo;
  if (bw >= hi) return;
  abl_v4f r[NB];
#pragma unroll
  for (int d = 0; d < NB; d++) r[d] = abl_load((b + d * 256u) * 16u, rin);
#pragma unroll
  for (int d = 0; d < NB; d++) abl_wait<0>(r[d]);
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      abl_wait<2 * (NB - 1)>(r[k]);
      float f[4] = {r[k].x, r[k].y, r[k].z, r[k].w};
      bool sp;
      uint64_t w = encode_block1d_lean5<64>(f, tab, sp);
      if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, f, p); w = rw.acc; }
      abl_store(b * 8u, rout, w);
      r[k] = abl_load((b + NB * 256u) * 16u, rin);
      b += 256u;
      bw += 256u;
      if (bw >= hi) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
      }
    }
  }
}

// pure compute floor: each lane loads NB blocks once and re-encodes them for the wave's whole trip count
// (same number of encodes as the real kernel, no per-iteration memory traffic), one store per lane at the end
template <int NB, int CODER = 3>
__global__ __launch_bounds__(256) void k_cfloor(const void* __restrict__ in, uint32_t nfull, Params p,
                                                 uint64_t* __restrict__ out)
{
  __shared__ uint32_t tab2[1280];
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab2[t] = CODER == 5 ? g_plane_tab5.v[t] : g_plane_tab2.v[t];
  __syncthreads();
  const uint32_t stride = gridDim.x * 256u;
  uint32_t b = blockIdx.x * 256u + threadIdx.x;
  uint32_t bw = __builtin_amdgcn_readfirstlane(blockIdx.x * 256u + (threadIdx.x & ~63u));
  if (bw >= nfull) return;
  float r[NB][4];
#pragma unroll
  for (int d = 0; d < NB; d++) load_row4_nt<DT_F32>(in, 4ll * min(b + d * stride, nfull - 1), r[d]);
  uint64_t accx = 0;
  for (;;) {
#pragma unroll
    for (int k = 0; k < NB; k++) {
      bool sp;
      uint64_t w = CODER == 5 ? encode_block1d_lean5<64>(r[k], tab2, sp)
                   : CODER == 4 ? encode_block1d_lean4<64>(r[k], tab2, sp) : encode_block1d_lean3<64>(r[k], tab2, sp);
      if (sp) { RegWriter64 rw{0ull, 0u}; encode_block<1>(rw, r[k], p); w = rw.acc; }
      accx ^= w;
      r[k][0] = __uint_as_float(__float_as_uint(r[k][0]) ^ (uint32_t)(w & 1));  // keep the loop honest
      bw += stride;
      if (bw >= nfull) {
        out[blockIdx.x * 256u + threadIdx.x] = accx;
        return;
      }
    }
  }
}

// 3-D fixed-rate split (C3, rate 8): STAGE 0 = gather + emax + cast + lift + reorder, folded into the block's words;
// STAGE 1 = + the two 32 x 32 bit transposes; (the full kernel is k_encode3d_fixed)
template <int STAGE>
__global__ __launch_bounds__(256) void k_c3_split(FieldDesc F, Params p, uint32_t* __restrict__ out32)
{
  constexpr uint32_t WPB = 16;
  extern __shared__ uint32_t lds_w[];
  const uint32_t tid = threadIdx.x;
  const uint32_t b0 = blockIdx.x * 256u;
  const uint32_t nvalid = min(256u, F.nblocks - b0);
  uint32_t* mine = lds_w + tid * (WPB + 1);
  if (tid < nvalid) {
    float f[64];
    gather_block<3, DT_F32>(F, b0 + tid, f);
    const int emax = block_emax<64>(f);
    int32_t q[64];
    const float sc = cast_scale(emax);
#pragma unroll
    for (int i = 0; i < 64; i++) q[i] = cast1(f[i], sc);
    fwd_xform<3>(q);
    uint32_t u[64];
    fwd_reorder<3>(u, q);
    if (STAGE >= 1) {
      transpose32(u);
      transpose32(u + 32);
    }
#pragma unroll
    for (int w = 0; w < 16; w++) mine[w] = u[w] ^ u[w + 16] ^ u[w + 32] ^ u[w + 48];
  }
  __syncthreads();
  uint32_t* dst = out32 + (uint64_t)b0 * WPB;
  for (uint32_t j = tid; j < nvalid * WPB; j += 256) dst[j] = lds_w[(j / WPB) * (WPB + 1) + (j % WPB)];
}

// Diagnostic build of k_encode_fixed1d_np<F32, 64, 8> (same body) with per-workgroup clock stamps: s_memtime /
// s_memrealtime at entry and after the last store, written by thread 0 with a vector store into a stamp buffer that
// no other code reads. In-kernel clock = d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md DVFS item 6).
__global__ __launch_bounds__(256) void k_np6_stamp(const void* __restrict__ in, uint32_t nfull, Params p,
                                                   void* __restrict__ out, uint64_t* __restrict__ stamps)
{
  constexpr int U = 8;
  constexpr uint32_t WB = 64;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  __shared__ uint32_t tab[1280 + 256];
  const pipe_v4i rin = buf_rsrc(in, nfull * 16u), rout = buf_rsrc(out, nfull * 8u);
  const uint32_t b0 = blockIdx.x * (256u * U) + threadIdx.x;
  typename PipeRow<DT_F32>::T r[U];
#pragma unroll
  for (int k = 0; k < U; k++) r[k] = PipeRow<DT_F32>::load((b0 + 256u * k) * 16u, rin);
#pragma unroll
  for (uint32_t t = threadIdx.x; t < 1280; t += 256) tab[t] = g_plane_tab5.v[t];
  tab[1280 + threadIdx.x] = g_rspread.v[threadIdx.x];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < U; k++) {
    pipe_wait<U - 1>(r[k]);
    float f[4];
    PipeRow<DT_F32>::unpack(r[k], f);
    bool special;
    uint64_t w = encode_block1d_lean6<WB>(f, tab, tab + 1280, special);
    if (special) {
      RegWriter64 rw{0ull, 0u};
      encode_block<1>(rw, f, p);
      w = rw.acc;
    }
    pipe_store<WB>((b0 + 256u * k) * 8u, rout, w);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint64_t* s4 = stamps + 4ull * blockIdx.x;
    s4[0] = t0; s4[1] = t1; s4[2] = r0; s4[3] = r1;
  }
}
}  // namespace gcow

static gcow::FieldDesc c3_field(const void* in)
{
  gcow::FieldDesc F{};
  F.data = in;
  F.n[0] = F.n[1] = F.n[2] = 512; F.n[3] = 1;
  F.s[0] = 1; F.s[1] = 512; F.s[2] = 512 * 512; F.s[3] = 0;
  F.bx = F.by = F.bz = 128; F.bw = 1;
  F.nblocks = 128u * 128u * 128u;
  F.dims = 3; F.dtype = gcow::DT_F32; F.vec = 1;
  return F;
}

static uint64_t* g_stamps = nullptr;
static const size_t kStampLaunches = 32, kStampWgs = 1u << 16;

// stamps of launch i of mode 90 (k_np6_stamp): 4 uint64 per workgroup, kStampWgs workgroups per launch slot
extern "C" int ablate_stamp_copy(void* host, int launch, size_t wgs)
{
  if (!g_stamps) return -1;
  return (int)hipMemcpy(host, g_stamps + (size_t)launch * kStampWgs * 4, wgs * 32, hipMemcpyDeviceToHost);
}

extern "C" int ablate_run(int mode, const void* in, uint32_t nfull, void* out, int wgs, void* stream)
{
  if (mode == 90) {  // wgs = launch slot
    if (!g_stamps && hipMalloc((void**)&g_stamps, kStampLaunches * kStampWgs * 32) != hipSuccess) return -1;
    const uint32_t g = (nfull + 2047) / 2048;
    if (g > kStampWgs || wgs < 0 || (size_t)wgs >= kStampLaunches) return -2;
    gcow::k_np6_stamp<<<g, 256, 0, (hipStream_t)stream>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out,
                                                           g_stamps + (size_t)wgs * kStampWgs * 4);
    return (int)hipGetLastError();
  }
  const uint32_t grid = min((nfull + 255) / 256, (uint32_t)(256 * wgs));
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case 91: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 8, 256><<<(nfull + 2047) / 2048, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 92: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 8, 512><<<(nfull + 4095) / 4096, 512, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 93: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 8, 1024><<<(nfull + 8191) / 8192, 1024, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 0: gcow::k_ablate<0><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 1: gcow::k_ablate<1><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 2: gcow::k_ablate<2><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 3: gcow::k_ablate<3><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 4: gcow::k_ablate<4><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 5: gcow::k_floor2<false><<<min(grid, (nfull / 2 + 255) / 256), 256, 0, st>>>((const float4*)in, nfull / 2, (uint4*)out); break;
    case 6: gcow::k_floor2<true><<<min(grid, (nfull / 2 + 255) / 256), 256, 0, st>>>((const float4*)in, nfull / 2, (uint4*)out); break;
    case 7: gcow::k_floor1<false><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint2*)out); break;
    case 8: gcow::k_floor1<true><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint2*)out); break;
    case 10: gcow::k_compute_floor<0><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 11: gcow::k_compute_floor<1><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 12: {
      gcow::Params p{64, 64, 64, -1074};
      gcow::k_encode_fixed1d_pnt<gcow::DT_F32, 64><<<grid, 256, 0, st>>>(in, nfull, p, out);
      break;
    }
    case 13: gcow::k_var<1><<<grid, 256, 0, st>>>(in, nfull, (uint64_t*)out); break;
    case 14: gcow::k_var<2><<<grid, 256, 0, st>>>(in, nfull, (uint64_t*)out); break;
    case 15: gcow::k_var<4><<<grid, 256, 0, st>>>(in, nfull, (uint64_t*)out); break;
    case 16: gcow::k_var<0><<<grid, 256, 0, st>>>(in, nfull, (uint64_t*)out); break;
    case 17: gcow::k_var<7><<<grid, 256, 0, st>>>(in, nfull, (uint64_t*)out); break;
    case 18: {
      gcow::Params p{64, 64, 64, -1074};
      gcow::k_u2<<<max(1u, grid / 2), 256, 0, st>>>(in, nfull, p, (uint64_t*)out);
      break;
    }
    case 19: gcow::k_np1<1><<<(nfull + 255) / 256, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 20: gcow::k_np1<2><<<(nfull + 511) / 512, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 21: gcow::k_np1<4><<<(nfull + 1023) / 1024, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 22: gcow::k_p1<<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 23: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 1, 256><<<(nfull + 255) / 256, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 24: gcow::k_pd<2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 25: gcow::k_pd<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 26: gcow::k_pd<4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 27: gcow::k_pd<6><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 28: gcow::k_pdu<1><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 29: gcow::k_pdu<2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 30: gcow::k_pdu<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 31: gcow::k_rot<2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 32: gcow::k_rot<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 33: gcow::k_rot<4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 34: gcow::k_rot<6><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 35: gcow::k_rot<8><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 36: gcow::k_rot2<2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 37: gcow::k_rot2<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 38: gcow::k_rot2<4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 39: gcow::k_rot3<2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 40: gcow::k_rot3<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 41: gcow::k_rot3<4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 42: gcow::k_rot4<2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 43: gcow::k_rot4<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 44: gcow::k_rot4<4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 45: gcow::k_asm<2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 46: gcow::k_asm<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 47: gcow::k_asm<4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 48: gcow::k_asm<3, 1><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 49: gcow::k_asm<3, 2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 50: gcow::k_cfloor<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 51: gcow::k_encode_fixed1d_pipe<gcow::DT_F32, 64, 3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 52: gcow::k_encode_fixed1d_pipe<gcow::DT_F32, 64, 2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 53: gcow::k_encode_fixed1d_pipe<gcow::DT_F32, 64, 4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 54: gcow::k_cfloor<3, 4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 55: gcow::k_cfloor<3, 5><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, (uint64_t*)out); break;
    case 56: gcow::k_encode_fixed1d_pipe<gcow::DT_F32, 64, 3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 57: gcow::k_encode_fixed1d_pipe<gcow::DT_F32, 64, 2><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 58: gcow::k_encode_fixed1d_pipe<gcow::DT_F32, 64, 4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 59: gcow::k_np5<2><<<(nfull + 511) / 512, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 60: gcow::k_np5<4><<<(nfull + 1023) / 1024, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 61: gcow::k_np5<8><<<(nfull + 2047) / 2048, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 62: gcow::k_chunk5<3><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 63: gcow::k_chunk5<4><<<grid, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    // k_encode_fixed1d_np prologue / second-window variants (V bit 0: table loads first; bit 1: W2 from low bytes)
    case 100: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 8, 256, 0><<<(nfull + 2047) / 2048, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 101: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 8, 256, 1><<<(nfull + 2047) / 2048, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 102: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 8, 256, 2><<<(nfull + 2047) / 2048, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 103: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 8, 256, 3><<<(nfull + 2047) / 2048, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 104: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 16, 256, 3><<<(nfull + 4095) / 4096, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 105: gcow::k_encode_fixed1d_np<gcow::DT_F32, 64, 12, 256, 3><<<(nfull + 3071) / 3072, 256, 0, st>>>(in, nfull, gcow::Params{64, 64, 64, -1074}, out); break;
    case 9: gcow::k_floor1<false><<<(nfull + 255) / 256, 256, 0, st>>>((const float4*)in, nfull, (uint2*)out); break;
    // one-shot, two blocks per lane (16-B store): the access shape a paired-store encoder would have
    case 64: gcow::k_floor2<false><<<(nfull / 2 + 255) / 256, 256, 0, st>>>((const float4*)in, nfull / 2, (uint4*)out); break;
    case 65: gcow::k_floor2<true><<<(nfull / 2 + 255) / 256, 256, 0, st>>>((const float4*)in, nfull / 2, (uint4*)out); break;
    case 70: case 71: case 72: {
      const gcow::FieldDesc F = c3_field(in);
      const gcow::Params p{512, 512, 64, -1074};
      const size_t lds = 256 * 17 * 4;
      if (mode == 70) gcow::k_encode3d_fixed<gcow::DT_F32, 16><<<F.nblocks / 256, 256, lds, st>>>(F, p, (uint32_t*)out);
      else if (mode == 71) gcow::k_c3_split<0><<<F.nblocks / 256, 256, lds, st>>>(F, p, (uint32_t*)out);
      else gcow::k_c3_split<1><<<F.nblocks / 256, 256, lds, st>>>(F, p, (uint32_t*)out);
      break;
    }
    case 66: gcow::k_floor1<true><<<(nfull + 255) / 256, 256, 0, st>>>((const float4*)in, nfull, (uint2*)out); break;
  }
  return (int)hipGetLastError();
}
