# timing only (wrong output): the packed kernel's chunk rounds without the
# ChaCha20 ARX instructions -- every wave still meets the same 80 s_barrier per
# chunk round (lock-step kept), the keystream is the initial state
EDITS = [("sg_pack.hip",
"""            asm volatile("s_and_saveexec_b64 %16, %17\\n" SG_CHACHA_DR_NB1_BAR1 "s_mov_b64 exec, %16\\n\"""",
"""            asm volatile("s_and_saveexec_b64 %16, %17\\n" ".rept 8\\ns_barrier\\n.endr\\n" "s_mov_b64 exec, %16\\n\"""")]
