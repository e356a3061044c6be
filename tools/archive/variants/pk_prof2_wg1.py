# pk_prof2 with the persistent grid held to 1 workgroup(s) per CU (analysis only)
import runpy
from pathlib import Path

EDITS = runpy.run_path(str(Path(__file__).with_name("pk_prof2.py")))["EDITS"] + [
    ("sg_pack.hip",
     "const uint32_t grid = 3u * (uint32_t)cus < most ? 3u * (uint32_t)cus : most;  // three workgroups per CU",
     "const uint32_t grid = 1u * (uint32_t)cus < most ? 1u * (uint32_t)cus : most;"),
]
