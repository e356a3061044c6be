# the packed kernel's setup and finish waves alternate between the SIMD pairs
# (waves 0-1 on even runs, waves 2-3 on odd runs) so that the setup's VALU
# does not always land on the same two SIMDs of the CU (output unchanged)
EDITS = [
("sg_pack.hip",
"""    const uint32_t m0 = tid;  // waves 0-1""",
"""    const uint32_t sw = wave ^ (((first >> 7) & 1u) << 1);
    const uint32_t m0 = (sw << 6) | lane;"""),
("sg_pack.hip",
"""    uint32_t nb = 0u, start = 0u;
    if (wave < 2u) {""",
"""    uint32_t nb = 0u, start = 0u;
    if (sw < 2u) {"""),
("sg_pack.hip",
"""        if (wave == 0u && lane == 63u) L.wtot = incl;""",
"""        if (sw == 0u && lane == 63u) L.wtot = incl;"""),
("sg_pack.hip",
"""    if (wave < 2u) {
        if (wave == 1u) start += L.wtot;""",
"""    if (sw < 2u) {
        if (sw == 1u) start += L.wtot;"""),
("sg_pack.hip",
"""    if (wave == 0u) {
        const uint32_t h0 = L.base[2u * lane]""",
"""    if (sw == 0u) {
        const uint32_t h0 = L.base[2u * lane]"""),
("sg_pack.hip",
"""    if (wave == 1u && lane == 63u) {
        const uint32_t total = start + nb;""",
"""    if (sw == 1u && lane == 63u) {
        const uint32_t total = start + nb;"""),
]
