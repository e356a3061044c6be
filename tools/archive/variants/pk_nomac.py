# timing only (wrong tags): the packed kernel without its per-lane Poly1305 share
EDITS = [("sg_pack.hip",
"""            const uint32_t r0 = sl[kSR + 0], r1 = sl[kSR + 1], r2 = sl[kSR + 2], r3 = sl[kSR + 3];
            H32 h;
            lane_mac(h, cw, r0, r1, r2, r3, r1 + (r1 >> 2), r2 + (r2 >> 2), r3 + (r3 >> 2));
            const F26 Q = words_to_f26(h.h0, h.h1, h.h2, h.h3, h.h4);
            const uint32_t i = sl[kSNb] - 1u - j;
            const uint32_t* tb = L.tab + m * kTabWords;
            const F26 W = tab_weight(tb, i);
            const F26 t = ripple_full(fmul(Q, W));
            uint32_t* ac = L.acc + 5u * m;
            atomicAdd(ac + 0, t.v0);
            atomicAdd(ac + 1, t.v1);
            atomicAdd(ac + 2, t.v2);
            atomicAdd(ac + 3, t.v3);
            atomicAdd(ac + 4, t.v4);
""", """            (void)cw;
""")]
