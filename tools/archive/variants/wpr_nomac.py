# timing only (wrong tags): sg_wpr_kernel without the in-loop MFMA MAC
# (no T window reads, no v_alignbyte/merge, no i8 bias XOR, no MFMA); the
# prologue and epilogue still run (on a zero accumulator)
EDITS = [
    ("sg_wpr.hip", """        auto mac_load = [&](uint32_t jj, uint32_t i, MacRaw& R) {
""", """        auto mac_load = [&](uint32_t jj, uint32_t i, MacRaw& R) {
            return;
"""),
    ("sg_wpr.hip", """        auto mac_mfma_f = [&](const u32x4& f, const u32x4& a, bool first = false) {
""", """        auto mac_mfma_f = [&](const u32x4& f, const u32x4& a, bool first = false) {
            return;
"""),
    ("sg_wpr.hip", """        auto mac_frag = [&](const MacRaw& R) -> u32x4 {
            u32x4 f;
""", """        auto mac_frag = [&](const MacRaw& R) -> u32x4 {
            u32x4 f = {};
            return f;
"""),
]
