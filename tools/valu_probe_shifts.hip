// Issue probe (shifts): which shift forms issue at the full (2-cycle) rate on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 512
#define R8(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define R32(OP) R8(OP) R8(OP) R8(OP) R8(OP)
#define I0(r) "v_add_u32 " r ", " r ", %8\n"
#define I1(r) "v_lshrrev_b32 " r ", 7, " r "\n"
#define I2(r) "v_lshlrev_b32 " r ", 16, " r "\n"
#define I3(r) "v_lshrrev_b32 " r ", %9, " r "\n"
#define I4(r) "v_lshlrev_b32 " r ", %9, " r "\n"
#define I5(r) "v_ashrrev_i32 " r ", 7, " r "\n"
#define I6(r) "v_lshlrev_b32 " r ", 1, " r "\n"
#define I7(r) "v_sub_u32 " r ", " r ", %8\n"
#define I8(r) "v_mov_b32 " r ", %8\n"
#define I9(r) "v_not_b32 " r ", " r "\n"
#define I10(r) "v_or3_b32 " r ", " r ", %8, " r "\n"
#define I11(r) "v_xor_b32_e64 " r ", " r ", %8\n"
#define I12(r) "v_bfe_u32 " r ", " r ", 7, 9\n"
#define I13(r) "v_lshrrev_b32_e64 " r ", 7, " r "\n"
#define I14(r) "v_lshlrev_b32_e64 " r ", 7, " r "\n"
#define I15(r) "v_and_or_b32 " r ", " r ", %8, " r "\n"
#define I16(r) "v_min_u32 " r ", " r ", %8\n"
#define I17(r) "v_add_lshl_u32 " r ", " r ", %8, 3\n"
#define I18(r) "v_lshl_add_u32 " r ", " r ", 3, %8\n"
#define I19(r) "v_max_u32 " r ", " r ", %8\n"
#define I20(r) "v_cndmask_b32 " r ", " r ", %8, s[0:1]\n"
#define I21(r) "v_cvt_f32_u32 " r ", " r "\n"
#define I22(r) "v_xad_u32 " r ", " r ", %8, " r "\n"
#define I23(r) "v_or_b32 " r ", " r ", %8\n"
static const char* names[] = {"v_add_u32", "v_lshrrev_b32 7", "v_lshlrev_b32 16", "v_lshrrev_b32 vreg", "v_lshlrev_b32 vreg",
  "v_ashrrev_i32 7", "v_lshlrev_b32 1", "v_sub_u32", "v_mov_b32", "v_not_b32", "v_or3_b32", "v_xor_b32_e64", "v_bfe_u32",
  "v_lshrrev_b32_e64 7", "v_lshlrev_b32_e64 7", "v_and_or_b32", "v_min_u32", "v_add_lshl_u32", "v_lshl_add_u32",
  "v_max_u32", "v_cndmask s01", "v_cvt_f32_u32", "v_xad_u32", "v_or_b32"};
template <int V>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint32_t x0 = t ^ seed, x1 = t * 3u, x2 = t + 7u, x3 = t * 5u ^ seed, x4 = t + 11u, x5 = t * 13u, x6 = t ^ 0x55u, x7 = t + seed;
    const uint32_t y = seed | 1u, sh = seed & 15u;
#define A(S) asm volatile(S : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y), "v"(sh))
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (V == 0) A(R32(I0)); if constexpr (V == 1) A(R32(I1)); if constexpr (V == 2) A(R32(I2));
        if constexpr (V == 3) A(R32(I3)); if constexpr (V == 4) A(R32(I4)); if constexpr (V == 5) A(R32(I5));
        if constexpr (V == 6) A(R32(I6)); if constexpr (V == 7) A(R32(I7)); if constexpr (V == 8) A(R32(I8));
        if constexpr (V == 9) A(R32(I9)); if constexpr (V == 10) A(R32(I10)); if constexpr (V == 11) A(R32(I11));
        if constexpr (V == 12) A(R32(I12)); if constexpr (V == 13) A(R32(I13)); if constexpr (V == 14) A(R32(I14));
        if constexpr (V == 15) A(R32(I15)); if constexpr (V == 16) A(R32(I16)); if constexpr (V == 17) A(R32(I17));
        if constexpr (V == 18) A(R32(I18)); if constexpr (V == 19) A(R32(I19)); if constexpr (V == 20) A(R32(I20));
        if constexpr (V == 21) A(R32(I21)); if constexpr (V == 22) A(R32(I22)); if constexpr (V == 23) A(R32(I23));
    }
    if ((x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x12345678u) out[t] = 1;
}
// 64-bit shifts
__global__ __launch_bounds__(256) void shr64(uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint64_t a0 = t, a1 = t * 3ull, a2 = t + 7ull, a3 = t ^ seed, a4 = t + 11u, a5 = t * 13u, a6 = t ^ 0x55u, a7 = t + seed;
    for (int i = 0; i < ITERS; ++i)
        asm volatile(
#define S(r) "v_lshrrev_b64 " r ", 7, " r "\n"
            R32(S)
#undef S
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    if ((uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345678u) out[t] = 1;
}
template <typename F> static float timeit(F launch) {
    launch(); (void)hipDeviceSynchronize();
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0); launch(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1); return ms;
}
template <int V> static void run(uint32_t* out) {
    const int blocks = 256 * 16;
    float ms = timeit([&] { hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), 0, 0, out, 0x1234567u); });
    double rate = blocks * 4.0 * ITERS * 32 / (ms * 1e-3) / 1024;
    printf("%-22s %7.3f ms  %.3e instr/s/SIMD\n", names[V], ms, rate);
}
template <int... Vs> static void all(uint32_t* out, std::integer_sequence<int, Vs...>) { (run<Vs>(out), ...); }
int main() {
    uint32_t* out; (void)hipMalloc(&out, 1 << 26);
    all(out, std::make_integer_sequence<int, 24>{});
    const int blocks = 256 * 16;
    float ms = timeit([&] { hipLaunchKernelGGL(shr64, dim3(blocks), dim3(256), 0, 0, out, 1u); });
    printf("%-22s %7.3f ms  %.3e instr/s/SIMD\n", "v_lshrrev_b64", ms, blocks * 4.0 * ITERS * 32 / (ms * 1e-3) / 1024);
    return 0;
}
