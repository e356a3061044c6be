# Round 6 (bit-exact): the packed setup's weight tables only as far as the
# record needs them -- lo[b] for b < nb, the hi chain only for records of more
# than 8 blocks (a record of nb blocks reads hi[(nb-1) >> 3] and lo[0..7] at
# most, header of sg_pack.hip); the other lanes' products run with EXEC off
# (their energy is what the power-capped batch pays for, r06p: the whole
# in-kernel keying is worth +4.4 % when removed outright)
EDITS = [
    ("sg_pack.hip", """            F26 y = f26_one();
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
            tb[kTabTop] = top;""", """            F26 y = f26_one();
            uint32_t top = 0u;
            const bool big = nb > 8u;  // the hi chain: records of more than 8 blocks only
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                if ((uint32_t)b < nb) top |= tab_put(tb, 8u + b, y);
                if ((uint32_t)b + 1u < nb) y = fmul(y, R);
            }
            top |= tab_put(tb, 0u, r);
            if (big) {
                const F26 R8 = y;  // r^32 (big: the lo chain ran to R^8)
                F26 z = r;
                const uint32_t na = (nb + 7u) >> 3;
#pragma unroll
                for (int a = 1; a < 8; ++a) {
                    if ((uint32_t)a < na) {
                        z = fmul(z, R8);
                        top |= tab_put(tb, a, z);
                    }
                }
            }
            tb[kTabTop] = top;"""),
]
