#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
template<int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0 = t ^ seed, x1 = t * 3u, x2 = t + 7u, x3 = t * 5u ^ seed, x4 = t+11u, x5 = t*13u, x6 = t ^ 0x55u, x7 = t + seed;
  uint64_t a0 = x0, a1 = x1, a2 = x2, a3 = x3, a4=x4, a5=x5, a6=x6, a7=x7;
  uint32_t y = seed | 1u;
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (OP == 0) { // v_add_u32 x8
      asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 1) { // v_alignbit x8
      asm volatile("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %2, %2, %2, 7\n v_alignbit_b32 %3, %3, %3, 7\n v_alignbit_b32 %4, %4, %4, 7\n v_alignbit_b32 %5, %5, %5, 7\n v_alignbit_b32 %6, %6, %6, 7\n v_alignbit_b32 %7, %7, %7, 7"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7));
    } else if constexpr (OP == 2) { // mad_u64_u32
      a0 = (uint64_t)x0 * y + a0; a1 = (uint64_t)x1 * y + a1; a2 = (uint64_t)x2 * y + a2; a3 = (uint64_t)x3 * y + a3;
      a4 = (uint64_t)x4 * y + a4; a5 = (uint64_t)x5 * y + a5; a6 = (uint64_t)x6 * y + a6; a7 = (uint64_t)x7 * y + a7;
      asm volatile("" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7));
    } else if constexpr (OP == 3) { // v_mul_lo_u32
      asm volatile("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 4) { // v_mad_u32_u24
      asm volatile("v_mad_u32_u24 %0, %0, %8, %1\n v_mad_u32_u24 %1, %1, %8, %2\n v_mad_u32_u24 %2, %2, %8, %3\n v_mad_u32_u24 %3, %3, %8, %4\n v_mad_u32_u24 %4, %4, %8, %5\n v_mad_u32_u24 %5, %5, %8, %6\n v_mad_u32_u24 %6, %6, %8, %7\n v_mad_u32_u24 %7, %7, %8, %0"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 5) { // v_mul_hi_u32
      asm volatile("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 6) { // f64 fma
      double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4=a4, d5=a5, d6=a6, d7=a7; double m = (double)y * 1e-9;
      for (int j = 0; j < 1; ++j) { d0 = fma(d0,m,d1); d1 = fma(d1,m,d2); d2=fma(d2,m,d3); d3=fma(d3,m,d4); d4=fma(d4,m,d5); d5=fma(d5,m,d6); d6=fma(d6,m,d7); d7=fma(d7,m,d0);} 
      a0 = __double_as_longlong(d0); a1 = __double_as_longlong(d1); a2=__double_as_longlong(d2); a3=__double_as_longlong(d3);
      a4 = __double_as_longlong(d4); a5 = __double_as_longlong(d5); a6=__double_as_longlong(d6); a7=__double_as_longlong(d7);
    } else if constexpr (OP == 7) { // xor x8
      asm volatile("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 8) { // v_mul_u32_u24
      asm volatile("v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 9) { // v_add3_u32
      asm volatile("v_add3_u32 %0, %0, %8, %1\n v_add3_u32 %1, %1, %8, %2\n v_add3_u32 %2, %2, %8, %3\n v_add3_u32 %3, %3, %8, %4\n v_add3_u32 %4, %4, %8, %5\n v_add3_u32 %5, %5, %8, %6\n v_add3_u32 %6, %6, %8, %7\n v_add3_u32 %7, %7, %8, %0"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 10) { // v_perm_b32
      asm volatile("v_perm_b32 %0, %0, %0, %8\n v_perm_b32 %1, %1, %1, %8\n v_perm_b32 %2, %2, %2, %8\n v_perm_b32 %3, %3, %3, %8\n v_perm_b32 %4, %4, %4, %8\n v_perm_b32 %5, %5, %5, %8\n v_perm_b32 %6, %6, %6, %8\n v_perm_b32 %7, %7, %7, %8"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    } else if constexpr (OP == 11) { // v_pk_add_u16 probe / v_lshl_add
      asm volatile("v_lshl_add_u32 %0, %0, 3, %8\n v_lshl_add_u32 %1, %1, 3, %8\n v_lshl_add_u32 %2, %2, 3, %8\n v_lshl_add_u32 %3, %3, 3, %8\n v_lshl_add_u32 %4, %4, 3, %8\n v_lshl_add_u32 %5, %5, 3, %8\n v_lshl_add_u32 %6, %6, 3, %8\n v_lshl_add_u32 %7, %7, 3, %8"
        : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7) : "v"(y));
    }
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7 ^ (uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7) ^ (uint32_t)((a0^a1^a2^a3^a4^a5^a6^a7)>>32);
  if (r == 0x12345678u) out[t] = r;
}
template<int OP> float run(uint32_t* out, int blocks) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k<OP><<<blocks,256>>>(out, 1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<OP><<<blocks,256>>>(out, 1);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); return ms / 5;
}
int main() {
  uint32_t* out; hipMalloc(&out, 1<<26);
  const char* names[] = {"v_add_u32","v_alignbit_b32","mad_u64_u32(C)","v_mul_lo_u32","v_mad_u32_u24","v_mul_hi_u32","f64 fma(C)","v_xor_b32","v_mul_u32_u24","v_add3_u32","v_perm_b32","v_lshl_add_u32"};
  int blocks = 256 * 8 * 4;
  float ms[12];
  ms[0]=run<0>(out,blocks); ms[1]=run<1>(out,blocks); ms[2]=run<2>(out,blocks); ms[3]=run<3>(out,blocks);
  ms[4]=run<4>(out,blocks); ms[5]=run<5>(out,blocks); ms[6]=run<6>(out,blocks); ms[7]=run<7>(out,blocks);
  ms[8]=run<8>(out,blocks); ms[9]=run<9>(out,blocks); ms[10]=run<10>(out,blocks); ms[11]=run<11>(out,blocks);
  double waves = blocks * 4.0;
  for (int i = 0; i < 12; ++i) {
    double winstr = waves * ITERS * 8.0;
    double rate = winstr / (ms[i] * 1e-3);  // wave-instr/s
    printf("%-16s %8.3f ms  %.3e wave-instr/s  = %.2f wave-instr/clk/CU @2.4GHz  (lane-ops %.3e/s)\n", names[i], ms[i], rate, rate / (256 * 2.4e9), rate * 64);
  }
  return 0;
}
