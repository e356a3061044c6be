# the double rounds at wave priority 1 (s_setprio around each round asm), the
# MAC preparation, prologue and epilogue at 0: when a SIMD has waves in both,
# the lock-step rounds issue first
EDITS = [
    ("sg_wpr.hip", """#define SG_DR()                                                                                                   \\
    asm volatile(SG_WPR_DR_ASM                                                                                    \\""",
     """#define SG_DR()                                                                                                   \\
    asm volatile("s_setprio 1\\n" SG_WPR_DR_ASM "s_setprio 0\\n"                                                   \\"""),
]
