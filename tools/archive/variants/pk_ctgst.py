# timing only (wrong output placement): lane-contiguous 16-byte stores of the same volume
EDITS = [("sg_pack.hip",
"""            uint8_t* dst = p.out + oo + 64u * j;
            pst16(dst, o0);
            pst16(dst + 16, o1);
            pst16(dst + 32, o2);
            pst16(dst + 48, o3);
""", """            uint8_t* dst = p.out + 4096ull * ((blockIdx.x * 32u + c) & 0xffffu) + 16u * lane;
            (void)oo;
            pst16(dst, o0);
            pst16(dst + 1024, o1);
            pst16(dst + 2048, o2);
            pst16(dst + 3072, o3);
""")]
