# timing only (wrong tags): the packed kernel's setup without its field
# products (the 16 weight-table entries and the constant term; block 0, the
# loads, the slots and the scans stay)
EDITS = [("sg_pack.hip",
"""            F26 y = f26_one();
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
            tb[kTabTop] = top;""",
"""#pragma unroll
            for (int e = 0; e < 16; ++e) {
                tb[4 * e] = R.v0; tb[4 * e + 1] = R.v1; tb[4 * e + 2] = R.v2; tb[4 * e + 3] = R.v3;
            }
            tb[kTabTop] = 0u;"""),
("sg_pack.hip",
"""            const F26 wl = tab_weight(tb, il);
            const F26 rB = fmul(fmul(wl, R), r);""",
"""            const F26 rB = R; (void)il;"""),
]
