// Issue throughput of the integer VALU instructions the encoder uses, measured on gfx950 (not part of libgcow.so).
// Each lane runs 8 independent chains of one instruction; 8 waves per SIMD; s_memtime brackets the loop per wave.
// Reports shader cycles per wave-instruction per SIMD (= per-wave cycles / instructions / waves per SIMD).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH8(INS)                                                                                            \
  asm volatile(INS : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));

#define OP1(name) name " %0, %0, %1\n" name " %1, %1, %2\n" name " %2, %2, %3\n" name " %3, %3, %4\n" \
                  name " %4, %4, %5\n" name " %5, %5, %6\n" name " %6, %6, %7\n" name " %7, %7, %0\n"
#define OPU(name) name " %0, %0\n" name " %1, %1\n" name " %2, %2\n" name " %3, %3\n" \
                  name " %4, %4\n" name " %5, %5\n" name " %6, %6\n" name " %7, %7\n"
#define OP3(name, c) name " %0, %0, %1, " c "\n" name " %1, %1, %2, " c "\n" name " %2, %2, %3, " c "\n" \
                     name " %3, %3, %4, " c "\n" name " %4, %4, %5, " c "\n" name " %5, %5, %6, " c "\n"  \
                     name " %6, %6, %7, " c "\n" name " %7, %7, %0, " c "\n"

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t iters, uint64_t* out, uint32_t* sink)
{
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
           a7 = a0 * 19;
  uint64_t q0 = a0, q1 = a1, q2 = a2, q3 = a3;
  if constexpr (OP == 16) asm volatile("s_mov_b64 s[20:21], 0x5555" ::: "s20", "s21");
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; i++) {
    if constexpr (OP == 0) { CH8(OP1("v_add_u32")) CH8(OP1("v_add_u32")) }
    if constexpr (OP == 1) { CH8(OP1("v_xor_b32")) CH8(OP1("v_xor_b32")) }
    if constexpr (OP == 2) { CH8(OPU("v_bfrev_b32")) CH8(OPU("v_bfrev_b32")) }
    if constexpr (OP == 3) { CH8(OPU("v_ffbh_u32")) CH8(OPU("v_ffbh_u32")) }
    if constexpr (OP == 4) { CH8(OP3("v_bfe_u32", "16")) CH8(OP3("v_bfe_u32", "16")) }
    if constexpr (OP == 5) { CH8(OP3("v_alignbit_b32", "%0")) CH8(OP3("v_alignbit_b32", "%0")) }
    if constexpr (OP == 6) { CH8(OP3("v_lshl_or_b32", "%0")) CH8(OP3("v_lshl_or_b32", "%0")) }
    if constexpr (OP == 7) { CH8(OP1("v_mul_f32")) CH8(OP1("v_mul_f32")) }
    if constexpr (OP == 8) { CH8(OPU("v_cvt_i32_f32")) CH8(OPU("v_cvt_i32_f32")) }
    if constexpr (OP == 9) { CH8(OP3("v_max3_u32", "%0")) CH8(OP3("v_max3_u32", "%0")) }
    if constexpr (OP == 10) { CH8(OP1("v_cndmask_b32")) CH8(OP1("v_cndmask_b32")) }
    if constexpr (OP == 11) {
      // 64-bit shifts by a VGPR amount: 4 chains x 4 per asm
      asm volatile("v_lshlrev_b64 %0, %4, %0\nv_lshlrev_b64 %1, %4, %1\nv_lshlrev_b64 %2, %4, %2\nv_lshlrev_b64 %3, %4, %3\n"
                   "v_lshrrev_b64 %0, %4, %0\nv_lshrrev_b64 %1, %4, %1\nv_lshrrev_b64 %2, %4, %2\nv_lshrrev_b64 %3, %4, %3\n"
                   "v_lshlrev_b64 %0, %4, %0\nv_lshlrev_b64 %1, %4, %1\nv_lshlrev_b64 %2, %4, %2\nv_lshlrev_b64 %3, %4, %3\n"
                   "v_lshrrev_b64 %0, %4, %0\nv_lshrrev_b64 %1, %4, %1\nv_lshrrev_b64 %2, %4, %2\nv_lshrrev_b64 %3, %4, %3\n"
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(a0));
    }
    if constexpr (OP == 12) { CH8(OP3("v_bitop3_b32", "%0 bitop3:0x96")) CH8(OP3("v_bitop3_b32", "%0 bitop3:0x96")) }
    if constexpr (OP == 13) { CH8(OP1("v_lshlrev_b32")) CH8(OP1("v_lshlrev_b32")) }
    if constexpr (OP == 14) { CH8(OP3("v_add3_u32", "%0")) CH8(OP3("v_add3_u32", "%0")) }
    if constexpr (OP == 15) { CH8(OP3("v_perm_b32", "%0")) CH8(OP3("v_perm_b32", "%0")) }
    if constexpr (OP == 16) { CH8(OP3("v_cndmask_b32_e64", "s[20:21]")) CH8(OP3("v_cndmask_b32_e64", "s[20:21]")) }
    if constexpr (OP == 17) { CH8(OP1("v_sub_u32")) CH8(OP1("v_sub_u32")) }
    if constexpr (OP == 18) { CH8(OP1("v_ashrrev_i32")) CH8(OP1("v_ashrrev_i32")) }
    if constexpr (OP == 19) { CH8(OP3("v_and_or_b32", "%0")) CH8(OP3("v_and_or_b32", "%0")) }
    if constexpr (OP == 20) { CH8(OP3("v_or3_b32", "%0")) CH8(OP3("v_or3_b32", "%0")) }
    if constexpr (OP == 21) { CH8(OP1("v_and_b32")) CH8(OP1("v_and_b32")) }
    if constexpr (OP == 22) { CH8(OP1("v_or_b32")) CH8(OP1("v_or_b32")) }
    if constexpr (OP == 23) { CH8(OP1("v_min_u32")) CH8(OP1("v_min_u32")) }
    if constexpr (OP == 24) { CH8(OP1("v_lshrrev_b32")) CH8(OP1("v_lshrrev_b32")) }
    if constexpr (OP == 25) { CH8(OP3("v_max3_f32", "%0")) CH8(OP3("v_max3_f32", "%0")) }
    if constexpr (OP == 26) {
#define SDW(a, b) "v_lshlrev_b32_sdwa " a ", " b ", " a " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
      CH8(SDW("%0", "%1") SDW("%1", "%2") SDW("%2", "%3") SDW("%3", "%4") SDW("%4", "%5") SDW("%5", "%6") SDW("%6", "%7") SDW("%7", "%0"))
      CH8(SDW("%0", "%1") SDW("%1", "%2") SDW("%2", "%3") SDW("%3", "%4") SDW("%4", "%5") SDW("%5", "%6") SDW("%6", "%7") SDW("%7", "%0"))
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(q0 ^ q1 ^ q2 ^ q3);
}

static const char* kNames[] = {"v_add_u32", "v_xor_b32", "v_bfrev_b32", "v_ffbh_u32", "v_bfe_u32",
                               "v_alignbit_b32", "v_lshl_or_b32", "v_mul_f32", "v_cvt_i32_f32", "v_max3_u32",
                               "v_cndmask_b32", "v_lshl/rrev_b64", "v_bitop3_b32", "v_lshlrev_b32", "v_add3_u32",
                               "v_perm_b32", "v_cndmask_e64 sgpr", "v_sub_u32", "v_ashrrev_i32", "v_and_or_b32",
                               "v_or3_b32", "v_and_b32", "v_or_b32", "v_min_u32", "v_lshrrev_b32", "v_max3_f32",
                               "v_lshlrev_b32_sdwa"};

template <int OP>
static void run(int wg_per_cu, int ncu)
{
  const uint32_t iters = 4096;
  const int grid = ncu * wg_per_cu;
  uint64_t* d_out;
  uint32_t* d_sink;
  hipMalloc(&d_out, grid * 4 * sizeof(uint64_t));
  hipMalloc(&d_sink, grid * 256 * sizeof(uint32_t));
  k_rate<OP><<<grid, 256>>>(iters, d_out, d_sink);
  hipDeviceSynchronize();
  k_rate<OP><<<grid, 256>>>(iters, d_out, d_sink);
  hipDeviceSynchronize();
  uint64_t* h = (uint64_t*)malloc(grid * 4 * sizeof(uint64_t));
  hipMemcpy(h, d_out, grid * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < grid * 4; i++) avg += (double)h[i];
  avg /= grid * 4;
  const double ins = 16.0 * iters;  // instructions per wave
  // waves per SIMD = wg_per_cu (one wave of each 4-wave WG per SIMD)
  printf("%-18s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (one wave: %.2f)\n", kNames[OP],
         wg_per_cu, avg / ins / wg_per_cu, avg / ins);
  free(h);
  hipFree(d_out);
  hipFree(d_sink);
}

int main()
{
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  for (int w : {1, 2, 8}) {
    run<0>(w, ncu); run<1>(w, ncu); run<2>(w, ncu); run<3>(w, ncu); run<4>(w, ncu); run<5>(w, ncu);
    run<6>(w, ncu); run<7>(w, ncu); run<8>(w, ncu); run<9>(w, ncu); run<10>(w, ncu); run<11>(w, ncu);
    run<12>(w, ncu); run<13>(w, ncu); run<14>(w, ncu); run<15>(w, ncu); run<16>(w, ncu); run<17>(w, ncu);
    run<18>(w, ncu); run<19>(w, ncu); run<20>(w, ncu); run<21>(w, ncu); run<22>(w, ncu); run<23>(w, ncu);
    run<24>(w, ncu); run<25>(w, ncu); run<26>(w, ncu);
  }
  return 0;
}
