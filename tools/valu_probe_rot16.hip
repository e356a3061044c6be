// Issue probe: candidate full-rate forms of the ChaCha20 rotate by 16 on gfx950.
// For each candidate: (1) bit-exactness over every 16-bit half pattern (a NaN-
// quieting or denormal-flushing f16 path would change bits), (2) SIMD cycles
// per wave64 instruction from s_memtime inside the waves, 8 independent chains,
// 1/2/4 waves per SIMD (same harness as valu_probe_ops.hip).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define ITERS 512
#define R8(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define R32(OP) R8(OP) R8(OP) R8(OP) R8(OP)

#define I_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define I_ALN(r) "v_alignbit_b32 " r ", " r ", " r ", 16\n"
#define I_PACK(r) "v_pack_b32_f16 " r ", " r ", " r " op_sel:[1,0,0]\n"
#define I_PKMAX(r) "v_pk_max_u16 " r ", " r ", " r " op_sel:[1,1] op_sel_hi:[0,0]\n"
#define I_BOP16(r) "v_bitop3_b16 " r ", " r ", " r ", " r " bitop3:0xf0 op_sel:[1,1,1,0]\n"

struct Var { const char* name; };
static const Var kVars[] = {{"v_add_u32"}, {"v_alignbit rot16"}, {"v_pack_b32_f16 rot16"}, {"v_pk_max_u16 rot16"}};
constexpr int kNumVars = sizeof(kVars) / sizeof(kVars[0]);

template <int V>
__device__ __forceinline__ void body(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                     uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y) {
#define SG_ASM(S) asm volatile(S : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y))
    if constexpr (V == 0) SG_ASM(R32(I_ADD));
    if constexpr (V == 1) SG_ASM(R32(I_ALN));
    if constexpr (V == 2) SG_ASM(R32(I_PACK));
    if constexpr (V == 3) SG_ASM(R32(I_PKMAX));
#undef SG_ASM
}

template <int V>
__global__ __launch_bounds__(256) void probe(unsigned long long* cyc, uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint32_t x0 = t ^ seed, x1 = t * 3u, x2 = t + 7u, x3 = t * 5u ^ seed, x4 = t + 11u, x5 = t * 13u, x6 = t ^ 0x55u,
             x7 = t + seed;
    const uint32_t y = seed | 1u;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) body<V>(x0, x1, x2, x3, x4, x5, x6, x7, y);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const uint32_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (r == 0x12345678u) out[t] = r;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

// rot16 of every word w = (hi << 16) | lo with hi, lo over all 2^16 patterns (pairs (i, i ^ k))
template <int V>
__global__ void check(uint32_t* bad, uint32_t k) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;  // 0 .. 2^16 - 1
    const uint32_t w = (i << 16) | ((i ^ k) & 0xffffu);
    uint32_t r = w;
    if constexpr (V == 2) asm volatile("v_pack_b32_f16 %0, %1, %1 op_sel:[1,0,0]" : "=v"(r) : "v"(w));
    if constexpr (V == 3) asm volatile("v_pk_max_u16 %0, %1, %1 op_sel:[1,1] op_sel_hi:[0,0]" : "=v"(r) : "v"(w));
    if constexpr (V == 1) asm volatile("v_alignbit_b32 %0, %1, %1, 16" : "=v"(r) : "v"(w));
    if (r != ((w << 16) | (w >> 16))) atomicAdd(bad, 1u);
}

static unsigned long long* g_cyc;
static uint32_t* g_out;

template <int V>
static void run_var() {
    uint32_t* bad;
    (void)hipMalloc(&bad, 4);
    (void)hipMemset(bad, 0, 4);
    if constexpr (V > 0)
        for (uint32_t k : {0u, 1u, 0x5555u, 0x8000u, 0x7c01u, 0xffffu, 0x0400u})
            hipLaunchKernelGGL(check<V>, dim3(256), dim3(256), 0, 0, bad, k);
    uint32_t nbad = 0;
    (void)hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost);
    (void)hipFree(bad);
    for (int wps : {1, 2, 4}) {
        const int blocks = 256 * wps;
        auto L = [&] { hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), 0, 0, g_cyc, g_out, 1u); };
        L();
        (void)hipDeviceSynchronize();
        L();
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> c(blocks * 4);
        (void)hipMemcpy(c.data(), g_cyc, c.size() * 8, hipMemcpyDeviceToHost);
        std::sort(c.begin(), c.end());
        const double cpu = (double)c[c.size() / 2] / (ITERS * 32.0 * wps);
        printf("%-22s wps=%d cyc/instr/SIMD=%6.2f bit_errors=%u\n", kVars[V].name, wps, cpu, nbad);
        fflush(stdout);
    }
}

int main() {
    (void)hipMalloc(&g_cyc, 256 * 64 * 4 * 8);
    (void)hipMalloc(&g_out, 1 << 26);
    run_var<0>();
    run_var<1>();
    run_var<2>();
    run_var<3>();
    return 0;
}
