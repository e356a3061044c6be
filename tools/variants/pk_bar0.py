# Round 6 probe: tools/variants/pk_bar.py with BAR=0 (no barriers in the rounds)
import runpy
from pathlib import Path

EDITS = runpy.run_path(str(Path(__file__).with_name("pk_bar.py")), init_globals={"BAR": 0})["EDITS"]
