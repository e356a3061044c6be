# (wpr_dst with the default cache policy: L2 can merge the four pieces)
# bit-exact: the uniform 16 KiB kernel stores each lane's 64-byte output block
# straight from its registers (four 16-byte nt stores at a 64-byte lane
# stride) instead of staging it in the LDS slice and reading it out
# lane-contiguously during the next chunk: prices the staging write and the
# read-out (32 KiB of LDS traffic and 128 ds instructions per record)
EDITS = [("sg_wpr.hip",
"""#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) st16(cb + 16u * (4u * lane + (i ^ xq)), O[i]);
            pend = active;""",
"""            if constexpr (!LIST) {
                if (active) {
                    uint8_t* dd = outb + kWprChunk * j + 64u * lane;
#pragma unroll
                    for (uint32_t i = 0; i < 4u; ++i) st16(dd + 16u * i, O[i]);
                }
                pend = false;
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 4u; ++i) st16(cb + 16u * (4u * lane + (i ^ xq)), O[i]);
                pend = active;
            }"""),
]
