# Round 6, timing only: sg_wpr_kernel as a pure data path -- tools/variants/
# wpr_noarx.py and tools/archive/variants/wpr_nomac.py together (no ARX, no
# MAC): the LDS-DMA loads, the lanes' block reads, feed-forward / XOR on zero
# keystream, staging, read-out and nt stores, prologue and epilogue.  What
# moving the record's bytes alone draws from the board.
import runpy
from pathlib import Path

_here = Path(__file__).resolve().parent
EDITS = (runpy.run_path(str(_here / "wpr_noarx.py"))["EDITS"]
         + runpy.run_path(str(_here.parent / "archive" / "variants" / "wpr_nomac.py"))["EDITS"])
