# timing only (wrong output): the bucket kernels (LIST) skip the ChaCha20
# rounds of each record's first, partial chunk -- the share of the bucket
# launches that a separate dense head pass would take over
EDITS = [
    ("sg_wpr.hip", "if (LIST && j == j0) SG_DR_LIVE(); else SG_DR();", "if (!(LIST && j == j0)) SG_DR();", "all"),
    ("sg_wpr.hip", """            asm volatile("s_mov_b64 exec, %7\\n" SG_CHACHA_DR1S_COL "s_mov_b64 exec, -1\\n\"""",
     """            if (!(LIST && j == j0)) asm volatile("s_mov_b64 exec, %7\\n" SG_CHACHA_DR1S_COL "s_mov_b64 exec, -1\\n\""""),
    ("sg_wpr.hip", """            asm volatile("s_mov_b64 exec, %28\\n" SG_CHACHA_DR1S_DIAG "s_mov_b64 exec, -1\\n\"""",
     """            if (!(LIST && j == j0)) asm volatile("s_mov_b64 exec, %28\\n" SG_CHACHA_DR1S_DIAG "s_mov_b64 exec, -1\\n\""""),
]
