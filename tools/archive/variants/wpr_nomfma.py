# timing only (wrong tags): sg_wpr_kernel with the MAC's operand preparation
# (T window reads, v_alignbyte / merge, i8 bias XOR) but without the MFMA
# instructions themselves (the operands are consumed by an empty asm)
EDITS = [
    ("sg_wpr.hip", """            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, f),
                                                         __builtin_bit_cast(i32x4, a ^ 0x80808080u), first ? c0 : acc,
                                                         0, 0, 0);""",
     """            const u32x4 ab = a ^ 0x80808080u;
            asm volatile("" :: "v"(f), "v"(ab));
            (void)c0; (void)first;"""),
]
