# the mixed-batch flow of the round-4 start: no side streams, and the packed
# launch (persistent grid, count on the device) after the population wait and
# the bucket launches, where the exact-grid launch used to be (A/B control)
import runpy
from pathlib import Path

_nofork = runpy.run_path(str(Path(__file__).with_name("mix_nofork.py")))["EDITS"]
EDITS = _nofork + [
    ("sg_kernels.hip", """        if (p.pack_mix && (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, tail + kPackList,
                                           tail + kTailPackCtr, s)) != hipSuccess)
            return e;
""", ""),
    ("sg_kernels.hip", """    // one launch per populated class, largest records first
""", """    if (p.pack_mix && exact && (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, tail + kPackList,
                                                tail + kTailPackCtr, s)) != hipSuccess)
        return e;
    // one launch per populated class, largest records first
"""),
]
