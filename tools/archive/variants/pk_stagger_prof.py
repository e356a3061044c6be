# pk_prof2 + pk_stagger (analysis only)
import runpy
from pathlib import Path

_d = Path(__file__).parent
EDITS = runpy.run_path(str(_d / "pk_prof2.py"))["EDITS"] + runpy.run_path(str(_d / "pk_stagger.py"))["EDITS"]
