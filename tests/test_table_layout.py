"""The wave-per-record keying table's grouped layout (sg_wpr.hip,
wpr_tab_unit): restated here and checked to be a
bijection from (slot, unit, word) onto the count x 160 words the workspace
reserves, for full and partial last groups, and to give every store
instruction of the keying kernel (unit u of 64 consecutive slots) whole
128-byte rows.  Host-side model, no GPU."""
import numpy as np
import pytest

REC_WORDS = 160  # kWprRecWords
UNITS = REC_WORDS // 4


def tab_unit(count: int, slot: int, u: int) -> int:
    g, w = slot >> 3, slot & 7
    rows = 8 if g < (count >> 3) else (count & 7)
    return g * (8 * REC_WORDS) + 4 * (u * rows + w)


@pytest.mark.parametrize("count", list(range(1, 34)) + [64, 65, 1000, 8195])
def test_grouped_table_is_a_bijection(count):
    seen = np.zeros(count * REC_WORDS, dtype=np.int32)
    for slot in range(count):
        for u in range(UNITS):
            base = tab_unit(count, slot, u)
            assert base % 4 == 0 and 0 <= base and base + 4 <= count * REC_WORDS
            seen[base:base + 4] += 1
    assert (seen == 1).all()


def test_grouped_table_rows_are_whole_lines():
    count = 4096
    for slot0 in (0, 64, 1024):
        for u in (0, 17, 39):
            addrs = sorted(4 * tab_unit(count, s, u) for s in range(slot0, slot0 + 64))  # bytes
            rows = [addrs[i:i + 8] for i in range(0, 64, 8)]
            for r in rows:  # eight 16-byte units back to back, 128-byte aligned
                assert r[0] % 128 == 0 and r == list(range(r[0], r[0] + 128, 16))
