#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 1024
__global__ __launch_bounds__(256) void k0(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k1(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_u32_e64 %0, %0, %16\nv_add_u32_e64 %1, %1, %16\nv_add_u32_e64 %2, %2, %16\nv_add_u32_e64 %3, %3, %16\nv_add_u32_e64 %4, %4, %16\nv_add_u32_e64 %5, %5, %16\nv_add_u32_e64 %6, %6, %16\nv_add_u32_e64 %7, %7, %16\nv_add_u32_e64 %0, %0, %16\nv_add_u32_e64 %1, %1, %16\nv_add_u32_e64 %2, %2, %16\nv_add_u32_e64 %3, %3, %16\nv_add_u32_e64 %4, %4, %16\nv_add_u32_e64 %5, %5, %16\nv_add_u32_e64 %6, %6, %16\nv_add_u32_e64 %7, %7, %16\nv_add_u32_e64 %0, %0, %16\nv_add_u32_e64 %1, %1, %16\nv_add_u32_e64 %2, %2, %16\nv_add_u32_e64 %3, %3, %16\nv_add_u32_e64 %4, %4, %16\nv_add_u32_e64 %5, %5, %16\nv_add_u32_e64 %6, %6, %16\nv_add_u32_e64 %7, %7, %16\nv_add_u32_e64 %0, %0, %16\nv_add_u32_e64 %1, %1, %16\nv_add_u32_e64 %2, %2, %16\nv_add_u32_e64 %3, %3, %16\nv_add_u32_e64 %4, %4, %16\nv_add_u32_e64 %5, %5, %16\nv_add_u32_e64 %6, %6, %16\nv_add_u32_e64 %7, %7, %16" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k2(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_xor_b32_e64 %0, %0, %16\nv_xor_b32_e64 %1, %1, %16\nv_xor_b32_e64 %2, %2, %16\nv_xor_b32_e64 %3, %3, %16\nv_xor_b32_e64 %4, %4, %16\nv_xor_b32_e64 %5, %5, %16\nv_xor_b32_e64 %6, %6, %16\nv_xor_b32_e64 %7, %7, %16\nv_xor_b32_e64 %0, %0, %16\nv_xor_b32_e64 %1, %1, %16\nv_xor_b32_e64 %2, %2, %16\nv_xor_b32_e64 %3, %3, %16\nv_xor_b32_e64 %4, %4, %16\nv_xor_b32_e64 %5, %5, %16\nv_xor_b32_e64 %6, %6, %16\nv_xor_b32_e64 %7, %7, %16\nv_xor_b32_e64 %0, %0, %16\nv_xor_b32_e64 %1, %1, %16\nv_xor_b32_e64 %2, %2, %16\nv_xor_b32_e64 %3, %3, %16\nv_xor_b32_e64 %4, %4, %16\nv_xor_b32_e64 %5, %5, %16\nv_xor_b32_e64 %6, %6, %16\nv_xor_b32_e64 %7, %7, %16\nv_xor_b32_e64 %0, %0, %16\nv_xor_b32_e64 %1, %1, %16\nv_xor_b32_e64 %2, %2, %16\nv_xor_b32_e64 %3, %3, %16\nv_xor_b32_e64 %4, %4, %16\nv_xor_b32_e64 %5, %5, %16\nv_xor_b32_e64 %6, %6, %16\nv_xor_b32_e64 %7, %7, %16" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k3(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\nv_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\nv_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\nv_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k4(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_or_b32 %0, %0, %16\nv_or_b32 %1, %1, %16\nv_or_b32 %2, %2, %16\nv_or_b32 %3, %3, %16\nv_or_b32 %4, %4, %16\nv_or_b32 %5, %5, %16\nv_or_b32 %6, %6, %16\nv_or_b32 %7, %7, %16\nv_or_b32 %0, %0, %16\nv_or_b32 %1, %1, %16\nv_or_b32 %2, %2, %16\nv_or_b32 %3, %3, %16\nv_or_b32 %4, %4, %16\nv_or_b32 %5, %5, %16\nv_or_b32 %6, %6, %16\nv_or_b32 %7, %7, %16\nv_or_b32 %0, %0, %16\nv_or_b32 %1, %1, %16\nv_or_b32 %2, %2, %16\nv_or_b32 %3, %3, %16\nv_or_b32 %4, %4, %16\nv_or_b32 %5, %5, %16\nv_or_b32 %6, %6, %16\nv_or_b32 %7, %7, %16\nv_or_b32 %0, %0, %16\nv_or_b32 %1, %1, %16\nv_or_b32 %2, %2, %16\nv_or_b32 %3, %3, %16\nv_or_b32 %4, %4, %16\nv_or_b32 %5, %5, %16\nv_or_b32 %6, %6, %16\nv_or_b32 %7, %7, %16" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k5(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k6(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_alignbit_b32 %0, %0, %0, %17\nv_alignbit_b32 %1, %1, %1, %17\nv_alignbit_b32 %2, %2, %2, %17\nv_alignbit_b32 %3, %3, %3, %17\nv_alignbit_b32 %4, %4, %4, %17\nv_alignbit_b32 %5, %5, %5, %17\nv_alignbit_b32 %6, %6, %6, %17\nv_alignbit_b32 %7, %7, %7, %17\nv_alignbit_b32 %0, %0, %0, %17\nv_alignbit_b32 %1, %1, %1, %17\nv_alignbit_b32 %2, %2, %2, %17\nv_alignbit_b32 %3, %3, %3, %17\nv_alignbit_b32 %4, %4, %4, %17\nv_alignbit_b32 %5, %5, %5, %17\nv_alignbit_b32 %6, %6, %6, %17\nv_alignbit_b32 %7, %7, %7, %17\nv_alignbit_b32 %0, %0, %0, %17\nv_alignbit_b32 %1, %1, %1, %17\nv_alignbit_b32 %2, %2, %2, %17\nv_alignbit_b32 %3, %3, %3, %17\nv_alignbit_b32 %4, %4, %4, %17\nv_alignbit_b32 %5, %5, %5, %17\nv_alignbit_b32 %6, %6, %6, %17\nv_alignbit_b32 %7, %7, %7, %17\nv_alignbit_b32 %0, %0, %0, %17\nv_alignbit_b32 %1, %1, %1, %17\nv_alignbit_b32 %2, %2, %2, %17\nv_alignbit_b32 %3, %3, %3, %17\nv_alignbit_b32 %4, %4, %4, %17\nv_alignbit_b32 %5, %5, %5, %17\nv_alignbit_b32 %6, %6, %6, %17\nv_alignbit_b32 %7, %7, %7, %17" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k7(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_xor_b32_sdwa %0, %0, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %1, %1, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %2, %2, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %3, %3, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %4, %4, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %5, %5, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %6, %6, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %7, %7, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %0, %0, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %1, %1, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %2, %2, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %3, %3, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %4, %4, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %5, %5, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %6, %6, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %7, %7, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %0, %0, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %1, %1, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %2, %2, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %3, %3, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %4, %4, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %5, %5, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %6, %6, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %7, %7, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %0, %0, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %1, %1, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %2, %2, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %3, %3, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %4, %4, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %5, %5, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %6, %6, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %7, %7, %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k8(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_u32_dpp %0, %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %1, %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %2, %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %3, %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %4, %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %5, %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %6, %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %7, %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %0, %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %1, %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %2, %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %3, %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %4, %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %5, %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %6, %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %7, %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %0, %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %1, %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %2, %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %3, %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %4, %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %5, %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %6, %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %7, %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %0, %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %1, %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %2, %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %3, %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %4, %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %5, %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %6, %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_add_u32_dpp %7, %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k9(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mad_u64_u32 %8, s[20:21], %0, %16, %8\nv_mad_u64_u32 %9, s[20:21], %1, %16, %9\nv_mad_u64_u32 %10, s[20:21], %2, %16, %10\nv_mad_u64_u32 %11, s[20:21], %3, %16, %11\nv_mad_u64_u32 %12, s[20:21], %4, %16, %12\nv_mad_u64_u32 %13, s[20:21], %5, %16, %13\nv_mad_u64_u32 %14, s[20:21], %6, %16, %14\nv_mad_u64_u32 %15, s[20:21], %7, %16, %15\nv_mad_u64_u32 %8, s[20:21], %0, %16, %8\nv_mad_u64_u32 %9, s[20:21], %1, %16, %9\nv_mad_u64_u32 %10, s[20:21], %2, %16, %10\nv_mad_u64_u32 %11, s[20:21], %3, %16, %11\nv_mad_u64_u32 %12, s[20:21], %4, %16, %12\nv_mad_u64_u32 %13, s[20:21], %5, %16, %13\nv_mad_u64_u32 %14, s[20:21], %6, %16, %14\nv_mad_u64_u32 %15, s[20:21], %7, %16, %15\nv_mad_u64_u32 %8, s[20:21], %0, %16, %8\nv_mad_u64_u32 %9, s[20:21], %1, %16, %9\nv_mad_u64_u32 %10, s[20:21], %2, %16, %10\nv_mad_u64_u32 %11, s[20:21], %3, %16, %11\nv_mad_u64_u32 %12, s[20:21], %4, %16, %12\nv_mad_u64_u32 %13, s[20:21], %5, %16, %13\nv_mad_u64_u32 %14, s[20:21], %6, %16, %14\nv_mad_u64_u32 %15, s[20:21], %7, %16, %15\nv_mad_u64_u32 %8, s[20:21], %0, %16, %8\nv_mad_u64_u32 %9, s[20:21], %1, %16, %9\nv_mad_u64_u32 %10, s[20:21], %2, %16, %10\nv_mad_u64_u32 %11, s[20:21], %3, %16, %11\nv_mad_u64_u32 %12, s[20:21], %4, %16, %12\nv_mad_u64_u32 %13, s[20:21], %5, %16, %13\nv_mad_u64_u32 %14, s[20:21], %6, %16, %14\nv_mad_u64_u32 %15, s[20:21], %7, %16, %15" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k10(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_xad_u32 %0, %0, %16, %0\nv_xad_u32 %1, %1, %16, %1\nv_xad_u32 %2, %2, %16, %2\nv_xad_u32 %3, %3, %16, %3\nv_xad_u32 %4, %4, %16, %4\nv_xad_u32 %5, %5, %16, %5\nv_xad_u32 %6, %6, %16, %6\nv_xad_u32 %7, %7, %16, %7\nv_xad_u32 %0, %0, %16, %0\nv_xad_u32 %1, %1, %16, %1\nv_xad_u32 %2, %2, %16, %2\nv_xad_u32 %3, %3, %16, %3\nv_xad_u32 %4, %4, %16, %4\nv_xad_u32 %5, %5, %16, %5\nv_xad_u32 %6, %6, %16, %6\nv_xad_u32 %7, %7, %16, %7\nv_xad_u32 %0, %0, %16, %0\nv_xad_u32 %1, %1, %16, %1\nv_xad_u32 %2, %2, %16, %2\nv_xad_u32 %3, %3, %16, %3\nv_xad_u32 %4, %4, %16, %4\nv_xad_u32 %5, %5, %16, %5\nv_xad_u32 %6, %6, %16, %6\nv_xad_u32 %7, %7, %16, %7\nv_xad_u32 %0, %0, %16, %0\nv_xad_u32 %1, %1, %16, %1\nv_xad_u32 %2, %2, %16, %2\nv_xad_u32 %3, %3, %16, %3\nv_xad_u32 %4, %4, %16, %4\nv_xad_u32 %5, %5, %16, %5\nv_xad_u32 %6, %6, %16, %6\nv_xad_u32 %7, %7, %16, %7" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k11(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_bitop3_b32 %0, %0, %16, %0 bitop3:0x96\nv_bitop3_b32 %1, %1, %16, %1 bitop3:0x96\nv_bitop3_b32 %2, %2, %16, %2 bitop3:0x96\nv_bitop3_b32 %3, %3, %16, %3 bitop3:0x96\nv_bitop3_b32 %4, %4, %16, %4 bitop3:0x96\nv_bitop3_b32 %5, %5, %16, %5 bitop3:0x96\nv_bitop3_b32 %6, %6, %16, %6 bitop3:0x96\nv_bitop3_b32 %7, %7, %16, %7 bitop3:0x96\nv_bitop3_b32 %0, %0, %16, %0 bitop3:0x96\nv_bitop3_b32 %1, %1, %16, %1 bitop3:0x96\nv_bitop3_b32 %2, %2, %16, %2 bitop3:0x96\nv_bitop3_b32 %3, %3, %16, %3 bitop3:0x96\nv_bitop3_b32 %4, %4, %16, %4 bitop3:0x96\nv_bitop3_b32 %5, %5, %16, %5 bitop3:0x96\nv_bitop3_b32 %6, %6, %16, %6 bitop3:0x96\nv_bitop3_b32 %7, %7, %16, %7 bitop3:0x96\nv_bitop3_b32 %0, %0, %16, %0 bitop3:0x96\nv_bitop3_b32 %1, %1, %16, %1 bitop3:0x96\nv_bitop3_b32 %2, %2, %16, %2 bitop3:0x96\nv_bitop3_b32 %3, %3, %16, %3 bitop3:0x96\nv_bitop3_b32 %4, %4, %16, %4 bitop3:0x96\nv_bitop3_b32 %5, %5, %16, %5 bitop3:0x96\nv_bitop3_b32 %6, %6, %16, %6 bitop3:0x96\nv_bitop3_b32 %7, %7, %16, %7 bitop3:0x96\nv_bitop3_b32 %0, %0, %16, %0 bitop3:0x96\nv_bitop3_b32 %1, %1, %16, %1 bitop3:0x96\nv_bitop3_b32 %2, %2, %16, %2 bitop3:0x96\nv_bitop3_b32 %3, %3, %16, %3 bitop3:0x96\nv_bitop3_b32 %4, %4, %16, %4 bitop3:0x96\nv_bitop3_b32 %5, %5, %16, %5 bitop3:0x96\nv_bitop3_b32 %6, %6, %16, %6 bitop3:0x96\nv_bitop3_b32 %7, %7, %16, %7 bitop3:0x96" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k12(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_alignbit_b32 %5, %5, %5, 7\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_alignbit_b32 %3, %3, %3, 7\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add_u32 %7, %7, %16\nv_add_u32 %0, %0, %16\nv_alignbit_b32 %1, %1, %1, 7\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_alignbit_b32 %7, %7, %7, 7\nv_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_alignbit_b32 %5, %5, %5, 7\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k13(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mov_b32_dpp %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %0, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %4, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %6, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %16 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k14(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_pk_add_u16 %0, %0, %16\nv_pk_add_u16 %1, %1, %16\nv_pk_add_u16 %2, %2, %16\nv_pk_add_u16 %3, %3, %16\nv_pk_add_u16 %4, %4, %16\nv_pk_add_u16 %5, %5, %16\nv_pk_add_u16 %6, %6, %16\nv_pk_add_u16 %7, %7, %16\nv_pk_add_u16 %0, %0, %16\nv_pk_add_u16 %1, %1, %16\nv_pk_add_u16 %2, %2, %16\nv_pk_add_u16 %3, %3, %16\nv_pk_add_u16 %4, %4, %16\nv_pk_add_u16 %5, %5, %16\nv_pk_add_u16 %6, %6, %16\nv_pk_add_u16 %7, %7, %16\nv_pk_add_u16 %0, %0, %16\nv_pk_add_u16 %1, %1, %16\nv_pk_add_u16 %2, %2, %16\nv_pk_add_u16 %3, %3, %16\nv_pk_add_u16 %4, %4, %16\nv_pk_add_u16 %5, %5, %16\nv_pk_add_u16 %6, %6, %16\nv_pk_add_u16 %7, %7, %16\nv_pk_add_u16 %0, %0, %16\nv_pk_add_u16 %1, %1, %16\nv_pk_add_u16 %2, %2, %16\nv_pk_add_u16 %3, %3, %16\nv_pk_add_u16 %4, %4, %16\nv_pk_add_u16 %5, %5, %16\nv_pk_add_u16 %6, %6, %16\nv_pk_add_u16 %7, %7, %16" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
__global__ __launch_bounds__(256) void k15(uint32_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u;
  uint32_t x0=t^seed,x1=t*3u,x2=t+7u,x3=t*5u^seed,x4=t+11u,x5=t*13u,x6=t^0x55u,x7=t+seed;
  uint64_t a0=x0,a1=x1,a2=x2,a3=x3,a4=x4,a5=x5,a6=x6,a7=x7; uint32_t y = seed|1u; uint32_t s = seed & 31u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mul_u32_u24_e32 %0, %0, %16\nv_mul_u32_u24_e32 %1, %1, %16\nv_mul_u32_u24_e32 %2, %2, %16\nv_mul_u32_u24_e32 %3, %3, %16\nv_mul_u32_u24_e32 %4, %4, %16\nv_mul_u32_u24_e32 %5, %5, %16\nv_mul_u32_u24_e32 %6, %6, %16\nv_mul_u32_u24_e32 %7, %7, %16\nv_mul_u32_u24_e32 %0, %0, %16\nv_mul_u32_u24_e32 %1, %1, %16\nv_mul_u32_u24_e32 %2, %2, %16\nv_mul_u32_u24_e32 %3, %3, %16\nv_mul_u32_u24_e32 %4, %4, %16\nv_mul_u32_u24_e32 %5, %5, %16\nv_mul_u32_u24_e32 %6, %6, %16\nv_mul_u32_u24_e32 %7, %7, %16\nv_mul_u32_u24_e32 %0, %0, %16\nv_mul_u32_u24_e32 %1, %1, %16\nv_mul_u32_u24_e32 %2, %2, %16\nv_mul_u32_u24_e32 %3, %3, %16\nv_mul_u32_u24_e32 %4, %4, %16\nv_mul_u32_u24_e32 %5, %5, %16\nv_mul_u32_u24_e32 %6, %6, %16\nv_mul_u32_u24_e32 %7, %7, %16\nv_mul_u32_u24_e32 %0, %0, %16\nv_mul_u32_u24_e32 %1, %1, %16\nv_mul_u32_u24_e32 %2, %2, %16\nv_mul_u32_u24_e32 %3, %3, %16\nv_mul_u32_u24_e32 %4, %4, %16\nv_mul_u32_u24_e32 %5, %5, %16\nv_mul_u32_u24_e32 %6, %6, %16\nv_mul_u32_u24_e32 %7, %7, %16" : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3),"+v"(x4),"+v"(x5),"+v"(x6),"+v"(x7),"+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(y), "s"(s) : "s20","s21");
  }
  uint32_t r = x0^x1^x2^x3^x4^x5^x6^x7^(uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
  if (r == 0x12345678u) out[t] = r;
}
template<typename K> float run(K kern, uint32_t* out, int blocks) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  kern<<<blocks,256>>>(out, 1);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) kern<<<blocks,256>>>(out, 1);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); return ms / 5;
}
int main() {
  uint32_t* out; (void)hipMalloc(&out, 1<<26);
  int blocks = 256 * 8 * 4; double waves = blocks * 4.0; double winstr = waves * ITERS * 32.0; float ms;
  ms = run(k0, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_add_u32_e32", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k1, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_add_u32_e64", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k2, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_xor_b32_e64", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k3, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_lshlrev_b32", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k4, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_or_b32", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k5, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_alignbit", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k6, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_alignbit_s", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k7, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_xor_sdwa", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k8, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_add_dpp", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k9, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_mad_u64_u32", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k10, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_xad_u32", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k11, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_bitop3", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k12, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "mix_2add_1align", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k13, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_mov_dpp", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k14, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_pk_add_u16", ms, winstr/(ms*1e-3)/(256*2.4e9));
  ms = run(k15, out, blocks); printf("%-20s %8.3f ms  %.2f wave-instr/clk/CU @2.4GHz\n", "v_mul_u32_u24_e32", ms, winstr/(ms*1e-3)/(256*2.4e9));
  return 0; }