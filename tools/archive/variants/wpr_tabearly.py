# the next record's keying table is fetched right after the last chunk's T
# fragments are in registers (after double round 8 of the last iteration)
# instead of after double round 10: two double rounds more to hide its latency
EDITS = [
    ("sg_wpr.hip", """            if (j == 3u) {
                F3[2] = mac_frag(R0);
                F3[3] = mac_frag(R1);
            }""", """            if (j == 3u) {
                F3[2] = mac_frag(R0);
                F3[3] = mac_frag(R1);
                if (next) {  // the line area is read out: the next record's table lands there
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    dma_table_of(gn * kWprWaves + wave);
                }
            }"""),
    ("sg_wpr.hip", """            if (j == 3u && next) {  // the line area is read out: the next record's table lands there
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                dma_table_of(gn * kWprWaves + wave);
            }""", ""),
]
