# (edits against the sources before the merge commit 620e6f4, which made pk_fork3 the product)
# pk_persist + the keying launches of a mixed batch on a side stream, beside
# the packed launch: the bucket keying (latency-bound, ~2.8 waves per SIMD)
# fills the packed launch's tail instead of running alone after it; the
# bucket kernels wait for it with an event
import runpy
from pathlib import Path

EDITS = runpy.run_path(str(Path(__file__).with_name("pk_persist.py")))["EDITS"] + [
    ("sg_kernels.hip", """template <bool OPEN>
hipError_t launch_aead_t(""", """// Side streams for the keying launches of mixed batches (per device, pooled
// like the pinned population buffers)
std::mutex g_side_mu;
std::vector<std::pair<int, std::pair<hipStream_t, hipEvent_t>>> g_side_free;
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    int dev = -1;
    hipError_t acquire() {
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        {
            std::lock_guard<std::mutex> lk(g_side_mu);
            for (size_t i = 0; i < g_side_free.size(); ++i)
                if (g_side_free[i].first == dev) {
                    s = g_side_free[i].second.first;
                    done = g_side_free[i].second.second;
                    g_side_free.erase(g_side_free.begin() + (long)i);
                    return hipSuccess;
                }
        }
        if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) {
            s = nullptr;
            return e;
        }
        if ((e = hipEventCreateWithFlags(&done, hipEventDisableTiming)) != hipSuccess) {
            (void)hipStreamDestroy(s);
            s = nullptr;
        }
        return e;
    }
    ~SideStream() {
        if (!s) return;
        std::lock_guard<std::mutex> lk(g_side_mu);
        g_side_free.push_back({dev, {s, done}});
    }
};

template <bool OPEN>
hipError_t launch_aead_t("""),
    ("sg_kernels.hip", """    const bool exact = cap_status == hipStreamCaptureStatusNone;
    if (exact) {""", """    const bool exact = cap_status == hipStreamCaptureStatusNone;
    SideStream side;  // the keying launches beside the packed one
    hipStream_t ks = s;
    if (exact) {"""),
    ("sg_kernels.hip", """        *over = pop[kTailOver];
""", """        *over = pop[kTailOver];
        if (p.pack_mix && pop[kPackList] != 0u && side.acquire() == hipSuccess) {
            ks = side.s;
            if ((e = hipStreamWaitEvent(ks, pin.ev, 0)) != hipSuccess) return e;
        }
"""),
    ("sg_kernels.hip", "        if ((e = launch_keying(p, OPEN, jobs, grid, s)) != hipSuccess) return e;",
     "        if ((e = launch_keying(p, OPEN, jobs, grid, ks)) != hipSuccess) return e;"),
    ("sg_kernels.hip", """        if ((e = launch_wpr_keying_lists(p, OPEN, wl, s)) != hipSuccess) return e;
    }
""", """        if ((e = launch_wpr_keying_lists(p, OPEN, wl, ks)) != hipSuccess) return e;
    }
    if (ks != s && ((e = hipEventRecord(side.done, ks)) != hipSuccess || (e = hipStreamWaitEvent(s, side.done, 0)) != hipSuccess))
        return e;
"""),
]
