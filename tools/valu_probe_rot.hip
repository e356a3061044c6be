// Issue probe (round 3): candidate full-rate forms of a 16-bit rotation and
// other untested VALU opcodes.  SIMD cycles per wave64 instruction with
// s_memtime inside the waves, 4 waves per SIMD (tools/valu_probe_ops.hip).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <utility>
#include <vector>

#define ITERS 512
#define R8(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define R32(OP) R8(OP) R8(OP) R8(OP) R8(OP)

#define I_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define I_ALN(r) "v_alignbit_b32 " r ", " r ", " r ", 16\n"
#define I_PACK(r) "v_pack_b32_f16 " r ", " r ", " r " op_sel:[1,0,0]\n"
#define I_SHL16(r) "v_lshlrev_b16 " r ", 3, " r "\n"
#define I_SHR16(r) "v_lshrrev_b16 " r ", 3, " r "\n"
#define I_ADD16(r) "v_add_u16 " r ", " r ", %8\n"
#define I_SDWA(r) "v_mov_b32_sdwa " r ", " r " dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n"
#define I_CND(r) "v_cndmask_b32 " r ", " r ", %8, vcc\n"
#define I_OR(r) "v_or_b32 " r ", " r ", %8\n"
#define I_SUBREV(r) "v_subrev_u32 " r ", " r ", %8\n"
#define I_MAX(r) "v_max_u32 " r ", " r ", %8\n"
#define I_LSHR(r) "v_lshrrev_b32 " r ", 7, " r "\n"
#define I_ASHR(r) "v_ashrrev_i32 " r ", 7, " r "\n"
#define I_NOT(r) "v_not_b32 " r ", " r "\n"
#define I_MULLO16(r) "v_mul_lo_u16 " r ", " r ", %8\n"
#define I_BFREV(r) "v_bfrev_b32 " r ", " r "\n"
#define I_SWAP(r) "v_swap_b32 " r ", %9\n"
#define I_XNOR(r) "v_xnor_b32 " r ", " r ", %8\n"
#define I_ALNDPP(r) "v_mov_b32_dpp " r ", " r " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define I_FADD(r) "v_add_f32 " r ", " r ", %8\n"
#define I_PKF32(r) "v_pk_add_f32 v[10:11], v[10:11], v[12:13]\n"

struct Var { const char* name; int per_iter; };
static const Var kVars[] = {
    {"v_add_u32", 32}, {"v_alignbit 16", 32}, {"v_pack_b32_f16 rot16", 32}, {"v_lshlrev_b16", 32},
    {"v_lshrrev_b16", 32}, {"v_add_u16", 32}, {"v_mov_b32_sdwa word", 32}, {"v_cndmask_b32", 32},
    {"v_or_b32", 32}, {"v_subrev_u32", 32}, {"v_max_u32", 32}, {"v_lshrrev_b32", 32}, {"v_ashrrev_i32", 32},
    {"v_not_b32", 32}, {"v_mul_lo_u16", 32}, {"v_bfrev_b32", 32}, {"v_xnor_b32", 32}, {"v_mov_b32_dpp quad", 32},
    {"v_add_f32", 32},
    {"grp8 add|pack16", 16}, {"grp8 add|aln16", 16},
};
constexpr int kNumVars = sizeof(kVars) / sizeof(kVars[0]);

template <int V>
__device__ __forceinline__ void body(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                     uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y, uint32_t& z) {
#define SG_ASM(S) asm volatile(S : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y), "v"(z) : "vcc")
    if constexpr (V == 0) SG_ASM(R32(I_ADD));
    if constexpr (V == 1) SG_ASM(R32(I_ALN));
    if constexpr (V == 2) SG_ASM(R32(I_PACK));
    if constexpr (V == 3) SG_ASM(R32(I_SHL16));
    if constexpr (V == 4) SG_ASM(R32(I_SHR16));
    if constexpr (V == 5) SG_ASM(R32(I_ADD16));
    if constexpr (V == 6) SG_ASM(R32(I_SDWA));
    if constexpr (V == 7) SG_ASM(R32(I_CND));
    if constexpr (V == 8) SG_ASM(R32(I_OR));
    if constexpr (V == 9) SG_ASM(R32(I_SUBREV));
    if constexpr (V == 10) SG_ASM(R32(I_MAX));
    if constexpr (V == 11) SG_ASM(R32(I_LSHR));
    if constexpr (V == 12) SG_ASM(R32(I_ASHR));
    if constexpr (V == 13) SG_ASM(R32(I_NOT));
    if constexpr (V == 14) SG_ASM(R32(I_MULLO16));
    if constexpr (V == 15) SG_ASM(R32(I_BFREV));
    if constexpr (V == 16) SG_ASM(R32(I_XNOR));
    if constexpr (V == 17) SG_ASM(R32(I_ALNDPP));
    if constexpr (V == 18) SG_ASM(R32(I_FADD));
    if constexpr (V == 19) SG_ASM(R8(I_ADD) R8(I_PACK));
    if constexpr (V == 20) SG_ASM(R8(I_ADD) R8(I_ALN));
#undef SG_ASM
}

template <int V>
__global__ __launch_bounds__(256) void probe(unsigned long long* cyc, uint32_t* out, uint32_t seed) {
    const uint32_t t = threadIdx.x + blockIdx.x * 256u;
    uint32_t x0 = t ^ seed, x1 = t * 3u, x2 = t + 7u, x3 = t * 5u ^ seed, x4 = t + 11u, x5 = t * 13u, x6 = t ^ 0x55u,
             x7 = t + seed, z = t;
    const uint32_t y = seed | 1u;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) body<V>(x0, x1, x2, x3, x4, x5, x6, x7, y, z);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const uint32_t r = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ z;
    if (r == 0x12345678u) out[t] = r;
    if ((threadIdx.x & 63u) == 0u) cyc[blockIdx.x * 4u + (threadIdx.x >> 6)] = c1 - c0;
}

// rot16 correctness of the v_pack_b32_f16 form
__global__ void check_pack(uint32_t* out, const uint32_t* in) {
    uint32_t x = in[threadIdx.x];
    asm volatile("v_pack_b32_f16 %0, %0, %0 op_sel:[1,0,0]" : "+v"(x));
    out[threadIdx.x] = x;
}

static unsigned long long* g_cyc;
static uint32_t* g_out;

template <int V>
static void run_var() {
    const int wps = 4, blocks = 256 * wps;
    hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), 0, 0, g_cyc, g_out, 1u);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), 0, 0, g_cyc, g_out, 1u);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> c(blocks * 4);
    (void)hipMemcpy(c.data(), g_cyc, c.size() * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double cpu = (double)c[c.size() / 2] / ((double)ITERS * kVars[V].per_iter * wps);
    printf("%-26s cyc/instr/SIMD=%6.2f\n", kVars[V].name, cpu);
    fflush(stdout);
}

template <int... Vs>
static void run_all(std::integer_sequence<int, Vs...>) {
    (run_var<Vs>(), ...);
}

int main() {
    (void)hipMalloc(&g_cyc, 256 * 64 * 4 * 8);
    (void)hipMalloc(&g_out, 1 << 26);
    uint32_t h[64], r[64];
    for (int i = 0; i < 64; ++i) h[i] = 0x12345678u * (i + 1) + 0x9abcdef0u;
    uint32_t *d_in, *d_out;
    (void)hipMalloc(&d_in, 256);
    (void)hipMalloc(&d_out, 256);
    (void)hipMemcpy(d_in, h, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check_pack, dim3(1), dim3(64), 0, 0, d_out, d_in);
    (void)hipMemcpy(r, d_out, 256, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int i = 0; i < 64; ++i) ok &= r[i] == ((h[i] << 16) | (h[i] >> 16));
    printf("v_pack_b32_f16 op_sel:[1,0,0] == rot16: %s (0x%08x -> 0x%08x)\n", ok ? "yes" : "NO", h[0], r[0]);
    run_all(std::make_integer_sequence<int, kNumVars>{});
    return 0;
}
