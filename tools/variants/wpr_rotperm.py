"""C1 energy probe: the 16- and 8-bit rotates of the record kernel's double
rounds (9 of 10 per chunk) as v_perm_b32 byte permutes instead of
v_alignbit_b32 (same issue rate, tools/valu_probe_*; the question is the energy
per instruction at the power cap).  Bit-exact."""
import re
from pathlib import Path

_inc = (Path(__file__).resolve().parents[2] / "suruga_amd/csrc/sg_chacha_grp.inc").read_text()
_m = re.search(r'#define SG_CHACHA_DR_NB1_BAR1 (".*?")\n', _inc)
_body = _m.group(1)
_perm = re.sub(r"v_alignbit_b32 (%\d+), \1, \1, 16", r"v_perm_b32 \1, \1, \1, %[p16]", _body)
_perm = re.sub(r"v_alignbit_b32 (%\d+), \1, \1, 24", r"v_perm_b32 \1, \1, \1, %[p8]", _perm)
assert _perm.count("v_perm_b32") == 16 and _perm.count("v_alignbit_b32") == 16
_anchor = "#define SG_CHACHA_DR_NB1_BAR1_BARRIERS 8\n"
_DR = """    asm volatile(SG_WPR_DR_ASM                                                                                    \\
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \\
                   "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]),         \\
                   "+v"(x[15]))"""
_DRP = """    asm volatile(SG_WPR_DR_ASM                                                                                    \\
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \\
                   "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]),         \\
                   "+v"(x[15])                                                                                  \\
                 : [p16] "s"(0x01000302u), [p8] "s"(0x02010003u))"""
_LIVE = """                     : "s"(live0)                                                                                 \\
                     : "scc");                                                                                    \\"""
_LIVEP = """                     : "s"(live0), [p16] "s"(0x01000302u), [p8] "s"(0x02010003u)                                \\
                     : "scc");                                                                                    \\"""
EDITS = [
    ("sg_chacha_grp.inc", _anchor, _anchor + "#define SG_CHACHA_DR_NB1_PERM " + _perm + "\n"),
    ("sg_wpr.hip", "#define SG_WPR_DR_ASM SG_CHACHA_DR_NB1_BAR1", "#define SG_WPR_DR_ASM SG_CHACHA_DR_NB1_PERM"),
    ("sg_wpr.hip", _DR, _DRP),
    ("sg_wpr.hip", _LIVE, _LIVEP),
]
