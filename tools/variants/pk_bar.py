# Round 6, probe (bit-exact): the packed kernel's grouped ARX rounds with an
# s_barrier after every BAR-th rotate group (BAR=2: 4 per double round
# instead of 8; BAR=0: none -- the waves of a workgroup run their rounds
# uncoupled, a wave without a chunk skips the round)
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from gen_chacha_grp import double_round  # noqa: E402

BAR = globals().get("BAR", 2)
_lines = double_round(1, BAR)
_body = "\\n".join(_lines) + "\\n"
_nbar = sum(ln == "s_barrier" for ln in _lines)
EDITS = [
    ("sg_pack.hip", '#define SG_PACK_IDLE_BARS (10 * SG_CHACHA_DR_NB1_BAR1_BARRIERS)',
     f'#define SG_PACK_IDLE_BARS (10 * {_nbar})\n#define SG_PACK_DR_VAR "{_body}"'),
    ("sg_pack.hip", 'asm volatile("s_and_saveexec_b64 %16, %17\\n" SG_CHACHA_DR_NB1_BAR1 "s_mov_b64 exec, %16\\n"',
     'asm volatile("s_and_saveexec_b64 %16, %17\\n" SG_PACK_DR_VAR "s_mov_b64 exec, %16\\n"'),
]
