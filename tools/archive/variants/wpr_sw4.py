# Round 4's LDS chunk swizzle f(t) = (t >> 2) & 3 (bit-exact; its staging
# ds_write_b128 is 2-way bank-conflicted: 128 extra LDS cycles per record)
EDITS = [
    ("sg_wpr.hip", "const uint32_t wunit = (lane & ~3u) | ((lane ^ (lane >> 2) ^ (lane >> 4)) & 3u);",
     "const uint32_t wunit = (lane & ~3u) | ((lane ^ (lane >> 4)) & 3u);"),
    ("sg_wpr.hip", "const uint32_t xq = (lane ^ (lane >> 2)) & 3u;", "const uint32_t xq = (lane >> 2) & 3u;"),
]
