// Measurement only: the store shapes a 1-D variable-rate decoder can produce for 256 Mi fp32 outputs (1 GiB), each
// lane holding 16 blocks (256 B) of output. mode 0: coalesced (16 rounds, lane-consecutive 16-B pieces);
// 1: chunk per lane, 4 rounds of 4 blocks, each block's 16 B at 256-B lane stride (the staged decoders' shape);
// 2: chunk per lane, 4 rounds, a quad-transposed store: the 4 lanes of a quad write one chunk's 64 contiguous bytes
// per instruction; 3: chunk per lane, one lane writing its 64 B of a round as 4 consecutive 16-B stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int MODE>
__global__ __launch_bounds__(128) void k_store(float4* __restrict__ out, uint32_t seed)
{
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint64_t c0 = (uint64_t)blockIdx.x * 128;
  const uint64_t c = c0 + tid;
  float v = (float)(seed ^ tid);
  if constexpr (MODE == 0) {
    float4* o = out + c0 * 16;
#pragma unroll 4
    for (int i = 0; i < 16; i++) o[i * 128 + tid] = make_float4(v, v + 1, v + 2, v + i);
  } else if constexpr (MODE == 1 || MODE == 3) {
    float4* o = out + c * 16;
    for (int r = 0; r < 4; r++) {
      float4 g[4];
#pragma unroll
      for (int k = 0; k < 4; k++) g[k] = make_float4(v + r, v + k, v, v);
#pragma unroll
      for (int k = 0; k < 4; k++) o[4 * r + k] = g[k];
      v += 1.0f;
    }
  } else if constexpr (MODE == 4 || MODE == 5) {
    // address pattern only: groups of G lanes write G x 16 contiguous bytes of one chunk per instruction
    // (G = 8: a full 128-B line, rounds of 8 blocks; G = 16: the chunk's whole 256 B)
    constexpr uint32_t G = MODE == 4 ? 8u : 16u;
    const uint32_t m = lane % G;
    const uint64_t cg = c - m;
    constexpr int R = 16 / G;  // rounds
    for (int r = 0; r < R; r++) {
#pragma unroll
      for (uint32_t i = 0; i < G; i++) out[(cg + i) * 16 + G * r + m] = make_float4(v + r, v + i, v, v);
      v += 1.0f;
    }
  } else {
    // quad q = lanes 4q .. 4q + 3 (chunks c0 + 4q + i); instruction i: lane 4q + m writes block m of chunk 4q + i
    const uint32_t m = lane & 3u;
    const uint64_t cq = c - m;  // chunk of the quad's lane 0
    for (int r = 0; r < 4; r++) {
      float4 g[4];
#pragma unroll
      for (int k = 0; k < 4; k++) g[k] = make_float4(v + r, v + k, v, v);
      // transpose within the quad: lane m needs g[m] of lane i for i = 0..3 (rotate + select, as a decoder would)
      float4 t[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t src = (lane & ~3u) | (uint32_t)i;
        float4 sel = m == 0 ? g[0] : (m == 1 ? g[1] : (m == 2 ? g[2] : g[3]));
        t[i].x = __shfl(sel.x, src, 64);
        t[i].y = __shfl(sel.y, src, 64);
        t[i].z = __shfl(sel.z, src, 64);
        t[i].w = __shfl(sel.w, src, 64);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) out[(cq + i) * 16 + 4 * r + m] = t[i];
      v += 1.0f;
    }
  }
}

int main()
{
  const size_t n4 = (size_t)64 << 20;  // float4 = 256 Mi floats
  float4* d;
  hipMalloc(&d, n4 * 16);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const uint32_t grid = (uint32_t)(n4 / 16 / 128);
  for (int mode = 0; mode < 6; mode++) {
    for (int rep = 0; rep < 3; rep++) {
      auto run = [&]() {
        if (mode == 0) k_store<0><<<grid, 128>>>(d, 1);
        else if (mode == 1) k_store<1><<<grid, 128>>>(d, 1);
        else if (mode == 2) k_store<2><<<grid, 128>>>(d, 1);
        else if (mode == 3) k_store<3><<<grid, 128>>>(d, 1);
        else if (mode == 4) k_store<4><<<grid, 128>>>(d, 1);
        else k_store<5><<<grid, 128>>>(d, 1);
      };
      for (int w = 0; w < 20; w++) run();
      hipEventRecord(a);
      for (int w = 0; w < 50; w++) run();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("mode %d: %.4f ms per 1 GiB store (%.0f GB/s)\n", mode, ms / 50, n4 * 16 / (ms / 50 * 1e-3) / 1e9);
    }
  }
  return 0;
}
