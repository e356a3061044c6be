# (edits against the sources before the merge commit 620e6f4, which made pk_fork3 the product)
# pk_persist's persistent packed kernel, launched where the exact-grid one was
# (after the population readback and the bucket launches): separates the cost
# of the persistent loop from the gain of overlapping the readback wait
import runpy
from pathlib import Path

_base = runpy.run_path(str(Path(__file__).with_name("pk_persist.py")))["EDITS"]
EDITS = [e for e in _base if e[0] != "sg_kernels.hip"] + [
    ("sg_kernels.hip", """    // packed small records (keyed inside their kernel)
    if (p.pack_mix && exact &&
        (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, pop[kPackList], s)) != hipSuccess)
        return e;
""", """    // packed small records (keyed inside their kernel)
    if (p.pack_mix && exact &&
        (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, tail + kPackList, tail + kTailPackCtr, s)) !=
            hipSuccess)
        return e;
"""),
]
