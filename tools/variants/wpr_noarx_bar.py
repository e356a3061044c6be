# Round 6, timing only: tools/variants/wpr_noarx.py with the rounds' 80
# s_barriers per chunk kept (no ARX instruction, the lock-step meetings stay)
import runpy
from pathlib import Path

EDITS = runpy.run_path(str(Path(__file__).with_name("wpr_noarx.py")), init_globals={"BAR": 1})["EDITS"]
