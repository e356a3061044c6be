# timing only (wrong tags): sg_wpr_kernel without the per-record prologue's
# field arithmetic (W = hi * lo and the digit lines r^(128k+1+d+u) are not
# computed; W is one table entry, the lines stay as the table left them)
EDITS = [
    ("sg_wpr.hip", """        const F26 W = fmul(load_f26(tab + kWHi + 20u * hh + 5u * (e >> 3)), load_f26(tab + kWLo + 5u * (e & 7u)));""",
     """        const F26 W = load_f26(tab + kWHi + 20u * hh + 5u * (e >> 3));"""),
    ("sg_wpr.hip", """        if (lane < kWprLines) {
            const uint32_t k = lane / 5u, uu = lane - 5u * k;""", """        if (false) {
            const uint32_t k = lane / 5u, uu = lane - 5u * k;"""),
    ("sg_wpr.hip", """        if (lane < kWprLines) {
            // any representative""", """        if (false) {
            // any representative"""),
]
