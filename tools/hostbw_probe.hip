// Round 6 probe: host-link bandwidth of (a) SDMA copies (hipMemcpyAsync) and
// (b) kernels that store to / load from registered host memory directly, one
// direction and both at once -- whether the record path's D2H could be a
// kernel's stores instead of an SDMA copy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256ull) dst[i] = src[i];
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 256ull << 20);
    const int reps = 8;
    void *h_src = aligned_alloc(4096, bytes), *h_dst = aligned_alloc(4096, bytes);
    memset(h_src, 1, bytes);
    memset(h_dst, 0, bytes);
    CK(hipHostRegister(h_src, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    CK(hipHostRegister(h_dst, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    void *dh_src = nullptr, *dh_dst = nullptr;
    CK(hipHostGetDevicePointer(&dh_src, h_src, 0));
    CK(hipHostGetDevicePointer(&dh_dst, h_dst, 0));
    void *d_a, *d_b;
    CK(hipMalloc(&d_a, bytes));
    CK(hipMalloc(&d_b, bytes));
    CK(hipMemset(d_a, 2, bytes));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t n16 = bytes / 16;
    printf("host pointers mapped: src %s, dst %s\n", dh_src == h_src ? "same VA" : "other VA", dh_dst == h_dst ? "same VA" : "other VA");
    auto run = [&](const char* name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, nullptr));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s %8.2f GB/s per direction-stream (%.3f ms per %zu MiB)\n", name, bytes * reps / (ms * 1e-3) / 1e9,
               ms / reps, bytes >> 20);
    };
    for (int grid : {cus, 4 * cus, 16 * cus}) {
        char nm[80];
        snprintf(nm, sizeof nm, "kernel D2H (device -> host stores), grid %d", grid);
        run(nm, [&] { hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s1, (const u32x4*)d_a, (u32x4*)dh_dst, n16); });
        snprintf(nm, sizeof nm, "kernel H2D (host loads -> device), grid %d", grid);
        run(nm, [&] { hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s1, (const u32x4*)dh_src, (u32x4*)d_b, n16); });
    }
    run("SDMA D2H (hipMemcpyAsync)", [&] { CK(hipMemcpyAsync(h_dst, d_a, bytes, hipMemcpyDeviceToHost, s1)); });
    run("SDMA H2D (hipMemcpyAsync)", [&] { CK(hipMemcpyAsync(d_b, h_src, bytes, hipMemcpyHostToDevice, s1)); });
    run("both: SDMA H2D (s1) + SDMA D2H (s2)", [&] {
        CK(hipMemcpyAsync(d_b, h_src, bytes, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h_dst, d_a, bytes, hipMemcpyDeviceToHost, s2));
    });
    run("both: SDMA H2D (s1) + kernel D2H (s2)", [&] {
        CK(hipMemcpyAsync(d_b, h_src, bytes, hipMemcpyHostToDevice, s1));
        hipLaunchKernelGGL(copy16, dim3(4 * cus), dim3(256), 0, s2, (const u32x4*)d_a, (u32x4*)dh_dst, n16);
    });
    // check the kernel D2H landed
    hipLaunchKernelGGL(copy16, dim3(4 * cus), dim3(256), 0, s1, (const u32x4*)d_a, (u32x4*)dh_dst, n16);
    CK(hipStreamSynchronize(s1));
    size_t bad = 0;
    for (size_t i = 0; i < bytes; ++i) bad += ((unsigned char*)h_dst)[i] != 2;
    printf("kernel D2H check: %zu bad bytes\n", bad);
    CK(hipHostUnregister(h_src));
    CK(hipHostUnregister(h_dst));
    return bad != 0;
}
