# timing only (wrong input placement): lane-contiguous 16-byte loads of the same volume
EDITS = [("sg_pack.hip",
"""            const uint8_t* src = p.in + io + 64u * j;
            // (plain policy: the nontemporal one measured -1.3 % on C2 for this
            // kernel's 64-byte lane stride, round 3; SG_PACK_NT_LD / _ST to compare)
            d0 = pld16(src); d1 = pld16(src + 16); d2 = pld16(src + 32); d3 = pld16(src + 48);
""", """            const uint8_t* src = p.in + 4096ull * ((blockIdx.x * 32u + c) & 0xffffu) + 16u * lane;
            (void)io;
            d0 = pld16(src); d1 = pld16(src + 1024); d2 = pld16(src + 2048); d3 = pld16(src + 3072);
""")]
