# (edits against the sources before the merge commit 620e6f4, which made pk_fork3 the product)
# packed kernel on a persistent grid (three workgroups per CU) that reads its
# population from the workspace tail and takes 128-record runs from a device
# counter; launched right after the population readback is enqueued, so the
# host's wait for the readback overlaps the packed launch instead of idling
# the GPU between classify and the keying / bucket launches
EDITS = [
    ("sg_internal.h", "constexpr uint32_t kWsTailWords = kNumLists + 1u + kWprBuckets + 1u;",
     "constexpr uint32_t kWsTailWords = kNumLists + 1u + kWprBuckets + 1u + 1u;"),
    ("sg_internal.h",
     "constexpr uint32_t kTailCtr = kNumLists + 1u;       // + b: group counter of wpr bucket b, + kWprBuckets: uniform C1 launch\n",
     "constexpr uint32_t kTailCtr = kNumLists + 1u;       // + b: group counter of wpr bucket b, + kWprBuckets: uniform C1 launch\n"
     "constexpr uint32_t kTailPackCtr = kTailCtr + kWprBuckets + 1u;  // run counter of the packed launch\n"
     "hipError_t device_cus(int* cus);  // CUs of the current device (cached)\n"),
    ("sg_internal.h",
     "hipError_t launch_pack(const KParams& p, bool open, const uint32_t* list, uint32_t count, hipStream_t s);",
     "hipError_t launch_pack(const KParams& p, bool open, const uint32_t* list, const uint32_t* cnt, uint32_t* ctr,\n"
     "                       hipStream_t s);"),
    ("sg_wpr.hip", "static hipError_t device_cus(int* cus) {", "hipError_t device_cus(int* cus) {"),
    ("sg_pack.hip", "    uint32_t nchunks, total;\n};", "    uint32_t nchunks, total;\n    uint32_t run;\n};"),
    ("sg_pack.hip", """template <bool OPEN>
__global__ __launch_bounds__(kPackThreads) void sg_pack_kernel(const KParams p, const uint32_t* __restrict__ list,
                                                               const uint32_t count) {
    __shared__ PackLds L;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uniform(tid >> 6);
    // XCD-aware run order (as the list kernels): workgroup b runs on XCD b % 8
    const uint32_t ng = gridDim.x, x8 = blockIdx.x & 7u, q8 = ng >> 3, r8 = ng & 7u;
    const uint32_t run = x8 * q8 + (x8 < r8 ? x8 : r8) + (blockIdx.x >> 3);
    const uint32_t first = run * kPackRecs;
    const uint32_t nrec = count - first < kPackRecs ? count - first : kPackRecs;
""", """template <bool OPEN>
__global__ __launch_bounds__(kPackThreads) __attribute__((amdgpu_waves_per_eu(6)))
void sg_pack_kernel(const KParams p, const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt, uint32_t* ctr) {
    __shared__ PackLds L;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uniform(tid >> 6);
    const uint32_t count = __builtin_amdgcn_readfirstlane(*cnt);
    const uint32_t nruns = (count + kPackRecs - 1u) / kPackRecs;
    for (;;) {
    if (tid == 0u) L.run = atomicAdd(ctr, 1u);
    __syncthreads();
    const uint32_t run = __builtin_amdgcn_readfirstlane(L.run);
    if (run >= nruns) break;
    const uint32_t first = run * kPackRecs;
    const uint32_t nrec = count - first < kPackRecs ? count - first : kPackRecs;
"""),
    ("sg_pack.hip", """            p.status[rec] = diff != 0u ? 1u : 0u;
        }
    }
    SG_STAMP(0u, 5);
}""", """            p.status[rec] = diff != 0u ? 1u : 0u;
        }
    }
    SG_STAMP(0u, 5);
    __syncthreads();  // the finish read the slots that the next run's setup rewrites
    }
}"""),
    ("sg_pack.hip", """hipError_t launch_pack(const KParams& p, bool open, const uint32_t* list, uint32_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (!p.tls) return hipErrorInvalidValue;  // the MAC geometry is the 13-byte TLS AD's
    const uint32_t grid = (count + kPackRecs - 1u) / kPackRecs;
""", """hipError_t launch_pack(const KParams& p, bool open, const uint32_t* list, const uint32_t* count, uint32_t* ctr,
                       hipStream_t s) {
    if (p.count == 0) return hipSuccess;
    if (!p.tls) return hipErrorInvalidValue;  // the MAC geometry is the 13-byte TLS AD's
    int cus = 0;
    hipError_t e;
    if ((e = device_cus(&cus)) != hipSuccess) return e;
    const uint32_t most = (p.count + kPackRecs - 1u) / kPackRecs;
    const uint32_t grid = 3u * (uint32_t)cus < most ? 3u * (uint32_t)cus : most;  // three workgroups per CU
"""),
    ("sg_pack.hip", "dim3(kPackThreads), 0, s, p, list, count);\n    else", "dim3(kPackThreads), 0, s, p, list, count, ctr);\n    else"),
    ("sg_pack.hip", "dim3(kPackThreads), 0, s, p, list, count);\n    return", "dim3(kPackThreads), 0, s, p, list, count, ctr);\n    return"),
    # population readback pool: a pinned buffer and an event
    ("sg_kernels.hip", """std::vector<uint32_t*> g_pop_free;
struct PinnedPop {
    uint32_t* p = nullptr;
    hipError_t acquire(size_t bytes) {
        {
            std::lock_guard<std::mutex> lk(g_pop_mu);
            if (!g_pop_free.empty()) {
                p = g_pop_free.back();
                g_pop_free.pop_back();
                return hipSuccess;
            }
        }
        return hipHostMalloc((void**)&p, bytes < 256u ? 256u : bytes, hipHostMallocDefault);
    }
    ~PinnedPop() {
        if (!p) return;
        std::lock_guard<std::mutex> lk(g_pop_mu);
        g_pop_free.push_back(p);
    }
};""", """std::vector<std::pair<uint32_t*, hipEvent_t>> g_pop_free;
struct PinnedPop {
    uint32_t* p = nullptr;
    hipEvent_t ev = nullptr;  // recorded after the readback copy
    hipError_t acquire(size_t bytes) {
        {
            std::lock_guard<std::mutex> lk(g_pop_mu);
            if (!g_pop_free.empty()) {
                p = g_pop_free.back().first;
                ev = g_pop_free.back().second;
                g_pop_free.pop_back();
                return hipSuccess;
            }
        }
        hipError_t e = hipHostMalloc((void**)&p, bytes < 256u ? 256u : bytes, hipHostMallocDefault);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) {
            (void)hipHostFree(p);
            p = nullptr;
            ev = nullptr;
        }
        return e;
    }
    ~PinnedPop() {
        if (!p) return;
        std::lock_guard<std::mutex> lk(g_pop_mu);
        g_pop_free.emplace_back(p, ev);
    }
};"""),
    ("sg_kernels.hip", """        if ((e = hipMemcpyAsync(pin.p, tail, sizeof pop, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;""",
     """        if ((e = hipMemcpyAsync(pin.p, tail, sizeof pop, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipEventRecord(pin.ev, s)) != hipSuccess)
            return e;
        // the packed records need no population on the host (persistent grid,
        // count and run counter in the tail): they run while the host waits
        // for the readback, and the batch's record window starts with them
        if ((e = mark(ev_keyed, s)) != hipSuccess || (e = mark(ev_start, s)) != hipSuccess) return e;
        ev_keyed = ev_start = nullptr;
        if (p.pack_mix && (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, tail + kPackList,
                                           tail + kTailPackCtr, s)) != hipSuccess)
            return e;
        if ((e = hipEventSynchronize(pin.ev)) != hipSuccess) return e;"""),
    ("sg_kernels.hip", """    // packed small records (keyed inside their kernel)
    if (p.pack_mix && exact &&
        (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, pop[kPackList], s)) != hipSuccess)
        return e;
""", ""),
]
