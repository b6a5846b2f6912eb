// Ablation microbenchmark for the 1-D fixed-rate encoder (not part of libgcow.so): stage-by-stage cost of
// load/store, block setup (emax, cast, lift, negabinary), plane window transpose, group phase, tail.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../gcow_amd/csrc/gcow_kernels.hip"

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
}  // namespace gcow

extern "C" int ablate_run(int mode, const void* in, uint32_t nfull, void* out, int wgs, void* stream)
{
  const uint32_t grid = min((nfull + 255) / 256, (uint32_t)(256 * wgs));
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case 0: gcow::k_ablate<0><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 1: gcow::k_ablate<1><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 2: gcow::k_ablate<2><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 3: gcow::k_ablate<3><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 4: gcow::k_ablate<4><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint64_t*)out); break;
    case 5: gcow::k_floor2<false><<<min(grid, (nfull / 2 + 255) / 256), 256, 0, st>>>((const float4*)in, nfull / 2, (uint4*)out); break;
    case 6: gcow::k_floor2<true><<<min(grid, (nfull / 2 + 255) / 256), 256, 0, st>>>((const float4*)in, nfull / 2, (uint4*)out); break;
    case 7: gcow::k_floor1<false><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint2*)out); break;
    case 8: gcow::k_floor1<true><<<grid, 256, 0, st>>>((const float4*)in, nfull, (uint2*)out); break;
    case 9: gcow::k_floor1<false><<<(nfull + 255) / 256, 256, 0, st>>>((const float4*)in, nfull, (uint2*)out); break;
  }
  return (int)hipGetLastError();
}
