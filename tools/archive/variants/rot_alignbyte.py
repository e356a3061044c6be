# the byte-granular rotations of the ChaCha20 rounds (16 and 8 bits) as
# v_alignbyte_b32 instead of v_alignbit_b32 (same values; energy A/B)
import re
from pathlib import Path

_inc = (Path(__file__).resolve().parents[2] / "suruga_amd" / "csrc" / "sg_chacha_grp.inc").read_text()
EDITS = []
for _reg in sorted(set(re.findall(r"v_alignbit_b32 (%\d+), \1, \1, (?:16|24)", _inc))):
    for _bits, _bytes in ((16, 2), (24, 3)):
        _old = f"v_alignbit_b32 {_reg}, {_reg}, {_reg}, {_bits}"
        if _old in _inc:
            EDITS.append(("sg_chacha_grp.inc", _old, f"v_alignbyte_b32 {_reg}, {_reg}, {_reg}, {_bytes}", "all"))
