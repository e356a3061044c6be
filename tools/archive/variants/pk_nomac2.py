# timing only (wrong tags): the packed kernel without its per-lane Poly1305
# share (lane_mac, the weight W, the term Q W and the LDS atomics); round 5 source
EDITS = [("sg_pack.hip",
"""            const uint32_t r0 = sl[kSR + 0], r1 = sl[kSR + 1], r2 = sl[kSR + 2], r3 = sl[kSR + 3];
            H32 h;
            lane_mac(h, cw, r0, r1, r2, r3, r1 + (r1 >> 2), r2 + (r2 >> 2), r3 + (r3 >> 2));
            const F26 Q = words_to_f26(h.h0, h.h1, h.h2, h.h3, h.h4);
            const uint32_t i = sl[kSNb] - 1u - j;
            const uint32_t* tb = L.tab + m * kTabWords;
            const F26 W = tab_weight(tb, i);
            uint32_t* ac = L.acc + kAccWords * m;
            const F26 t = fmul(Q, W);
            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 0),
                      (unsigned long long)t.v0 | ((unsigned long long)t.v2 << 32));
            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 2),
                      (unsigned long long)t.v3 | ((unsigned long long)t.v4 << 32));
            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);
""", """            asm volatile("" :: "v"(cw[0]), "v"(cw[5]), "v"(cw[10]), "v"(cw[15]));
""")]
