# packed kernel setup: each power-table entry normalised by four
# v_mad_u64_u32 into words plus two folds of the bits >= 2^130 instead of a
# two-pass carry ripple (the product chains unchanged)
import runpy
from pathlib import Path

EDITS = runpy.run_path(str(Path(__file__).with_name("pk_setup2.py")))["EDITS"][:1]
