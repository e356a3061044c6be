# (edits against the sources before the merge commit 620e6f4, which made pk_fork3 the product)
# pk_fork + the three bucket launches on three streams (J = 2 on the batch's
# stream, J = 3 on a second side stream, J = 4 after the keying on the keying
# stream), all after the keying: each persistent bucket grid takes the CU
# slots that the launches before it free, so their tails (and the packed
# launch's) overlap instead of adding up; the batch's stream joins both
import runpy
from pathlib import Path

EDITS = runpy.run_path(str(Path(__file__).with_name("pk_fork.py")))["EDITS"] + [
    ("sg_kernels.hip", """    if (ks != s && ((e = hipEventRecord(side.done, ks)) != hipSuccess || (e = hipStreamWaitEvent(s, side.done, 0)) != hipSuccess))
        return e;
""", """    SideStream side2;
    hipStream_t js[kWprBuckets] = {s, ks, ks};  // bucket b (J = 2 + b): J = 4 right after the keying
    if (ks != s) {
        if ((e = hipEventRecord(side.done, ks)) != hipSuccess || (e = hipStreamWaitEvent(s, side.done, 0)) != hipSuccess)
            return e;
        if (side2.acquire() == hipSuccess) {
            if ((e = hipStreamWaitEvent(side2.s, side.done, 0)) != hipSuccess) return e;
            js[1] = side2.s;
        }
    }
"""),
    ("sg_kernels.hip", """        for (int b = (int)kWprBuckets - 1; b >= 0; --b)
            if ((e = launch_wpr_list(p, OPEN, kWprMinJ + (uint32_t)b, wl[b], s)) != hipSuccess) return e;
    }
""", """        for (int b = (int)kWprBuckets - 1; b >= 0; --b)
            if ((e = launch_wpr_list(p, OPEN, kWprMinJ + (uint32_t)b, wl[b], js[b])) != hipSuccess) return e;
    }
    if (ks != s && ((e = hipEventRecord(side.done, ks)) != hipSuccess || (e = hipStreamWaitEvent(s, side.done, 0)) != hipSuccess))
        return e;
    if (side2.s && js[1] == side2.s &&
        ((e = hipEventRecord(side2.done, side2.s)) != hipSuccess || (e = hipStreamWaitEvent(s, side2.done, 0)) != hipSuccess))
        return e;
"""),
]
