# Round 6, timing only (wrong tags): the packed kernel without its in-kernel
# keying -- no keystream block 0, no weight-table products, no constant term
# (r is a constant clamped value, every table entry r, the constant zero); the
# loads of each record's list entry, length, offsets, key and nonce, the slot
# writes and the start scan stay.  The upper bound of taking the keying off the
# run's critical path, by a pre-pass (verdict r5 item 1b, before its own cost
# and traffic) or by overlapping it with the rounds (1a, before the issue slots
# its instructions still take)
EDITS = [
    ("sg_pack.hip", """            uint32_t ks[16];
            chacha_block(ks, rk.k, 0u, rk.n14, rk.n15);  // block 0 -> poly key (chacha20_poly1305.rs:50,75)""",
     """            uint32_t ks[16] = {0x0a1b2c3du, 0x04050607u, 0x08090a0bu, 0x0c0d0e0fu, rk.k[0], rk.k[1], rk.k[2], rk.k[3]};"""),
    ("sg_pack.hip", """            const F26 r = words_to_f26(r0, r1, r2w, r3, 0u);
            const F26 r2 = fmul(r, r), R = fmul(r2, r2);
            F26 y = f26_one();
            uint32_t top = 0u;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                top |= tab_put(tb, 8u + b, y);
                y = fmul(y, R);
            }
            const F26 R8 = y;  // r^32
            F26 z = r;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                top |= tab_put(tb, a, z);
                if (a < 7) z = fmul(z, R8);
            }
            tb[kTabTop] = top;""", """            const F26 r = words_to_f26(r0, r1, r2w, r3, 0u);
            const F26 R = r;
            uint32_t top = 0u;
#pragma unroll
            for (int b = 0; b < 16; ++b) top |= tab_put(tb, b, r);
            tb[kTabTop] = top;"""),
    ("sg_pack.hip", """            const F26 wl = tab_weight(tb, il);
            const F26 rB = fmul(fmul(wl, R), r);""", """            const F26 rB = f26_zero();
            (void)il;"""),
    ("sg_pack.hip", """            store_f26(sl + kSCtot, fmul_add(blk0, rB, fmul(sfx, r)));""",
     """            store_f26(sl + kSCtot, f26_add(blk0, f26_add(rB, sfx)));"""),
]
