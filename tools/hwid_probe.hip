// Wave placement probe (round 5): which SIMD each wave of a 512-thread
// workgroup lands on when three workgroups share a CU (the packed kernel's
// launch shape: 52 KB of LDS per workgroup, grid = 3 x CUs).  Every wave reads
// its HW_ID register (simd_id bits 5:4, cu_id 11:8, sh_id 12, se_id 15:13) and
// the host prints, per wave index of the workgroup, how often it sat on each
// SIMD.  If wave 0 and wave 1 always sit on SIMDs 0 and 1, the packed
// kernel's setup (waves 0-1) loads two SIMDs of every CU and none of the
// other two.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hwid_probe tools/hwid_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kThreads = 512, kWaves = kThreads / 64;

__global__ __launch_bounds__(kThreads) void probe(uint32_t* out, uint32_t spin) {
    __shared__ uint32_t lds[13 * 1024];  // 52 KB: three workgroups per CU
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  // HW_REG_HW_ID, 32 bits
    lds[threadIdx.x] = hw;
    // stay resident for a while so that the grid's workgroups coexist
    uint32_t acc = hw;
    for (uint32_t i = 0; i < spin; ++i) acc = acc * 1664525u + 1013904223u;
    __syncthreads();
    if ((threadIdx.x & 63u) == 0u) out[blockIdx.x * kWaves + wave] = lds[threadIdx.x] ^ (acc == 1u ? 1u : 0u);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = 3 * cus;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, (size_t)grid * kWaves * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(grid), dim3(kThreads), 0, 0, d, 200000u);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<uint32_t> h((size_t)grid * kWaves);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int count[kWaves][4] = {};
    for (int b = 0; b < grid; ++b)
        for (int w = 0; w < kWaves; ++w) ++count[w][(h[(size_t)b * kWaves + w] >> 4) & 3u];
    printf("grid %d workgroups of %d threads; rows: wave index, columns: SIMD 0..3\n", grid, kThreads);
    for (int w = 0; w < kWaves; ++w)
        printf("wave %d: %6d %6d %6d %6d\n", w, count[w][0], count[w][1], count[w][2], count[w][3]);
    // how the first wave's SIMD varies across the three workgroups of one CU
    int same = 0, groups = 0;
    for (int b = 0; b < grid; ++b) {
        const uint32_t loc = h[(size_t)b * kWaves] & 0xff00u;  // cu, sh, se of wave 0
        for (int c = b + 1; c < grid; ++c)
            if ((h[(size_t)c * kWaves] & 0xff00u) == loc) {
                ++groups;
                same += ((h[(size_t)b * kWaves] >> 4) & 3u) == ((h[(size_t)c * kWaves] >> 4) & 3u);
            }
    }
    printf("pairs of workgroups on one (se, sh, cu) id: %d, wave 0 on the same SIMD: %d\n", groups, same);
    (void)hipFree(d);
    return 0;
}
