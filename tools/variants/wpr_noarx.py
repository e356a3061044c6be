# Round 6, timing only (wrong output): sg_wpr_kernel without the ChaCha20 ARX
# stream -- the ten double rounds per chunk (the first one from SGPRs and the
# nine grouped asm ones) become register moves, and their s_barriers go too.
# Everything else stays: the LDS-DMA of the chunks and the keying table, the
# lanes' block reads, feed-forward and XOR, the staging write and read-out,
# the nt stores, the MFMA MAC with its T windows, prologue and epilogue.
# BAR=1 (wpr_noarx_bar.py) keeps the 80 s_barriers per chunk.
BAR = globals().get("BAR", 0)
_b4 = ".rept 4\\ns_barrier\\n.endr\\n" if BAR else ""
_b8 = ".rept 8\\ns_barrier\\n.endr\\n" if BAR else ""
EDITS = [
    ("sg_wpr.hip", "#define SG_WPR_DR_ASM SG_CHACHA_DR_NB1_BAR1", f'#define SG_WPR_DR_ASM "{_b8}"'),
    ("sg_wpr.hip", 'asm volatile("s_mov_b64 exec, %7\\n" SG_CHACHA_DR1S_COL "s_mov_b64 exec, -1\\n"',
     'asm volatile("s_mov_b64 exec, %7\\n" "v_mov_b32 %0, %4\\nv_mov_b32 %1, %5\\nv_mov_b32 %2, %6\\n' + _b4
     + '" "s_mov_b64 exec, -1\\n"'),
    ("sg_wpr.hip", 'asm volatile("s_mov_b64 exec, %28\\n" SG_CHACHA_DR1S_DIAG "s_mov_b64 exec, -1\\n"',
     'asm volatile("s_mov_b64 exec, %28\\n" "'
     + "".join(f"v_mov_b32 %{4 + i}, %{16 + i}\\n" for i in range(12)) + _b4 + '" "s_mov_b64 exec, -1\\n"'),
]
