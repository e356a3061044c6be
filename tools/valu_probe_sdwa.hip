// Issue probe (SDWA): SIMD cycles per wave64 instruction for the SDWA forms a
// two-instruction rot16(d ^ a) would use, next to v_xor / v_alignbit, and a
// full quarter-round group in both lowerings.  Same method as valu_probe_ops.hip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <utility>

#define ITERS 512
#define R8(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define R32(OP) R8(OP) R8(OP) R8(OP) R8(OP)
#define I_XOR(r) "v_xor_b32 " r ", " r ", %8\n"
#define I_ALN(r) "v_alignbit_b32 " r ", " r ", " r ", 16\n"
#define I_SXP(r) "v_xor_b32_sdwa " r ", " r ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define I_SXZ(r) "v_xor_b32_sdwa " r ", " r ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n"
#define I_SMV(r) "v_mov_b32_sdwa " r ", " r " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n"
#define I_ADD(r) "v_add_u32 " r ", " r ", %8\n"
// rot16(d ^ y) into t (= %9 .. ) : two SDWA xors; here written back to r through the temp %9
#define I_R16S(r) "v_xor_b32_sdwa %9, " r ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n" \
                  "v_xor_b32_sdwa %9, " r ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" \
                  "v_mov_b32 " r ", %9\n"
#define I_R16A(r) "v_xor_b32 " r ", " r ", %8\n" "v_alignbit_b32 " r ", " r ", " r ", 16\n"
#define ALT16(A, B) A("%0") B("%1") A("%2") B("%3") A("%4") B("%5") A("%6") B("%7") \
                    B("%0") A("%1") B("%2") A("%3") B("%4") A("%5") B("%6") A("%7")

struct Var { const char* name; int per_iter; };
static const Var kVars[] = {
    {"v_xor_b32", 32}, {"v_alignbit 16", 32}, {"xor_sdwa preserve", 32}, {"xor_sdwa pad", 32},
    {"mov_sdwa preserve", 32}, {"alt add/xor_sdwa", 16}, {"grp8 add|xor_sdwa", 16},
    {"rot16 sdwa x2 + mov", 24}, {"rot16 xor+alignbit", 16},
};
constexpr int kNumVars = sizeof(kVars) / sizeof(kVars[0]);

template <int V>
__device__ __forceinline__ void body(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                     uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y, uint32_t& t) {
#define SG_ASM(S) asm volatile(S : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y), "v"(t) : "vcc")
    if constexpr (V == 0) SG_ASM(R32(I_XOR));
    if constexpr (V == 1) SG_ASM(R32(I_ALN));
    if constexpr (V == 2) SG_ASM(R32(I_SXP));
    if constexpr (V == 3) SG_ASM(R32(I_SXZ));
    if constexpr (V == 4) SG_ASM(R32(I_SMV));
    if constexpr (V == 5) SG_ASM(ALT16(I_ADD, I_SXP));
    if constexpr (V == 6) SG_ASM(R8(I_ADD) R8(I_SXP));
    if constexpr (V == 7) SG_ASM(R8(I_R16S));
    if constexpr (V == 8) SG_ASM(R8(I_R16A));
#undef SG_ASM
}

template <int V>
__global__ __launch_bounds__(256) void probe(unsigned long long* cyc, uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint32_t x0 = t ^ seed, x1 = t * 3u, x2 = t + 7u, x3 = t * 5u ^ seed, x4 = t + 11u, x5 = t * 13u, x6 = t ^ 0x55u,
             x7 = t + seed, tmp = t;
    const uint32_t y = seed | 1u;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) body<V>(x0, x1, x2, x3, x4, x5, x6, x7, y, tmp);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const uint32_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ tmp;
    if (r == 0x12345678u) out[t] = r;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

static unsigned long long* g_cyc;
static uint32_t* g_out;

template <typename F>
static void measure(const char* name, double units_per_wave, int wps, F launch) {
    const int blocks = 256 * wps;
    launch(blocks);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    launch(blocks);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(blocks * 4);
    (void)hipMemcpy(c.data(), g_cyc, c.size() * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double med = (double)c[c.size() / 2];
    const double cpu = med / (units_per_wave * wps);
    const double rate = (double)blocks * 4 * units_per_wave / (ms * 1e-3) / 1024.0;
    printf("%-24s wps=%d cyc/instr/SIMD=%6.2f wall=%7.3fms clk~%.2fGHz\n", name, wps, cpu, ms, rate * cpu / 1e9);
    fflush(stdout);
}

template <int V>
static void run_var() {
    for (int wps : {1, 2, 4})
        measure(kVars[V].name, (double)ITERS * kVars[V].per_iter, wps,
                [](int blocks) { hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), 0, 0, g_cyc, g_out, 1u); });
}
template <int... Vs>
static void run_all(std::integer_sequence<int, Vs...>) { (run_var<Vs>(), ...); }

int main() {
    (void)hipMalloc(&g_cyc, 256 * 64 * 4 * 8);
    (void)hipMalloc(&g_out, 1 << 26);
    run_all(std::make_integer_sequence<int, kNumVars>{});
    return 0;
}
