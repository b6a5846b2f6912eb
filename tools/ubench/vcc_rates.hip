// Issue cost of selects on gfx950 (not part of libgcow.so): v_cndmask_b32 reading VCC (the VOP2 form the compiler
// emits after a v_cmp_*_e32) against v_cndmask_b32_e64 reading an SGPR pair written by v_cmp_*_e64. Each lane runs
// 8 independent chains; waves per SIMD 1, 2, 8; s_memtime brackets the loop. Reports shader cycles per compare+select
// pair per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH8(INS) asm volatile(INS : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : : "vcc", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");

#define PV(x, y) "v_cmp_gt_u32_e32 vcc, " y ", " x "\nv_cndmask_b32_e32 " x ", " x ", " y ", vcc\n"
#define PS(x, y, s) "v_cmp_gt_u32_e64 " s ", " y ", " x "\nv_cndmask_b32_e64 " x ", " x ", " y ", " s "\n"
#define PC(x, y) "v_cndmask_b32_e32 " x ", " x ", " y ", vcc\n"
#define PM(x, y) "v_max_u32_e32 " x ", " x ", " y "\n"

template <int OP>
__global__ __launch_bounds__(256) void k_sel(uint32_t iters, uint64_t* out, uint32_t* sink)
{
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
           a7 = a0 * 19;
  if constexpr (OP == 3) asm volatile("s_mov_b64 vcc, 0x5555" ::: "vcc");
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; i++) {
    if constexpr (OP == 0)
      CH8(PV("%0", "%1") PV("%1", "%2") PV("%2", "%3") PV("%3", "%4") PV("%4", "%5") PV("%5", "%6") PV("%6", "%7") PV("%7", "%0"))
    if constexpr (OP == 1)
      CH8(PS("%0", "%1", "s[20:21]") PS("%1", "%2", "s[20:21]") PS("%2", "%3", "s[20:21]") PS("%3", "%4", "s[20:21]")
          PS("%4", "%5", "s[20:21]") PS("%5", "%6", "s[20:21]") PS("%6", "%7", "s[20:21]") PS("%7", "%0", "s[20:21]"))
    if constexpr (OP == 2)
      CH8(PS("%0", "%1", "s[20:21]") PS("%1", "%2", "s[22:23]") PS("%2", "%3", "s[24:25]") PS("%3", "%4", "s[26:27]")
          PS("%4", "%5", "s[20:21]") PS("%5", "%6", "s[22:23]") PS("%6", "%7", "s[24:25]") PS("%7", "%0", "s[26:27]"))
    if constexpr (OP == 3)  // selects only, VCC constant (two selects per "pair")
      CH8(PC("%0", "%1") PC("%1", "%2") PC("%2", "%3") PC("%3", "%4") PC("%4", "%5") PC("%5", "%6") PC("%6", "%7") PC("%7", "%0")
          PC("%0", "%1") PC("%1", "%2") PC("%2", "%3") PC("%3", "%4") PC("%4", "%5") PC("%5", "%6") PC("%6", "%7") PC("%7", "%0"))
    if constexpr (OP == 4)  // v_max pairs (reference: two plain VOP2 per pair)
      CH8(PM("%0", "%1") PM("%1", "%2") PM("%2", "%3") PM("%3", "%4") PM("%4", "%5") PM("%5", "%6") PM("%6", "%7") PM("%7", "%0")
          PM("%0", "%1") PM("%1", "%2") PM("%2", "%3") PM("%3", "%4") PM("%4", "%5") PM("%5", "%6") PM("%6", "%7") PM("%7", "%0"))
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

static const char* kNames[] = {"v_cmp_e32 + v_cndmask vcc", "v_cmp_e64 + v_cndmask_e64 (1 pair)",
                               "v_cmp_e64 + v_cndmask_e64 (4 pairs)", "v_cndmask vcc x2 (vcc const)",
                               "v_max_u32 x2"};

template <int OP>
static void run(int wg_per_cu, int ncu)
{
  const uint32_t iters = 4096;
  const int grid = ncu * wg_per_cu;
  uint64_t* d_out;
  uint32_t* d_sink;
  hipMalloc(&d_out, grid * 4 * sizeof(uint64_t));
  hipMalloc(&d_sink, grid * 256 * sizeof(uint32_t));
  k_sel<OP><<<grid, 256>>>(iters, d_out, d_sink);
  hipDeviceSynchronize();
  k_sel<OP><<<grid, 256>>>(iters, d_out, d_sink);
  hipDeviceSynchronize();
  uint64_t* h = (uint64_t*)malloc(grid * 4 * sizeof(uint64_t));
  hipMemcpy(h, d_out, grid * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < grid * 4; i++) avg += (double)h[i];
  avg /= grid * 4;
  const double pairs = 8.0 * iters;  // pairs per wave
  printf("%-38s waves/SIMD %d: %.2f cycles per pair per SIMD (one wave: %.2f)\n", kNames[OP], wg_per_cu,
         avg / pairs / wg_per_cu, avg / pairs);
  free(h);
  hipFree(d_out);
  hipFree(d_sink);
}

int main()
{
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  for (int w : {1, 2, 8}) {
    run<0>(w, ncu); run<1>(w, ncu); run<2>(w, ncu); run<3>(w, ncu); run<4>(w, ncu);
  }
  return 0;
}
