# the i8 bias of the MFMA B operand (byte ^ 0x80) applied where the ciphertext
# registers are produced (after the feed-forward, among the full-rate XORs of
# the lock-step pair) instead of right before each MFMA
EDITS = [
    ("sg_wpr.hip", """            for (uint32_t i = 0; i < 4u; ++i) A[i] = OPEN ? D[i] : O[i];""",
     """            for (uint32_t i = 0; i < 4u; ++i) A[i] = (OPEN ? D[i] : O[i]) ^ 0x80808080u;"""),
    ("sg_wpr.hip", """                for (uint32_t i = 0; i < 4u; ++i) A[i] = u32x4{0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};""",
     """                for (uint32_t i = 0; i < 4u; ++i) A[i] = u32x4{0u, 0u, 0u, 0u};"""),
    ("sg_wpr.hip", """__builtin_bit_cast(i32x4, a ^ 0x80808080u), first ? c0 : acc,""",
     """__builtin_bit_cast(i32x4, a), first ? c0 : acc,"""),
]
