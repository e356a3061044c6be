# the MAC's T fragments read as byte-unaligned dwords straight from the digit
# lines (ds_read_b32 at the lane's own window byte) instead of aligned dwords
# shifted with v_alignbyte (TLS path: 5 reads, 1 merge, no alignbyte)
EDITS = [
    ("sg_wpr.hip", """    uint32_t mac_lo_a = (uint32_t)(uintptr_t)(mac_base - 64), mac_hi_a = (uint32_t)(uintptr_t)(mac_base + 960 - 64);""",
     """    uint32_t mac_lo_a = (uint32_t)(uintptr_t)(mac_base - 64) + (TLS ? mac_shift : 0u),
             mac_hi_a = (uint32_t)(uintptr_t)(mac_base + 960 - 64) + (TLS ? mac_shift : 0u);"""),
    ("sg_wpr.hip", """            if constexpr (TLS) {
#pragma unroll
                for (int t = 0; t < 4; ++t) R.v[t] = vb[t];
#pragma unroll
                for (int t = 2; t < 5; ++t) R.p[t] = pb[t];
            } else {""",
     """            if constexpr (TLS) {
                typedef const __attribute__((address_space(3))) uint32_t __attribute__((aligned(1))) lu32u;
                const lu32u* ub = (const lu32u*)pb;
                R.v[0] = ub[16]; R.v[1] = ub[17]; R.v[2] = ub[18];
                R.p[2] = ub[2]; R.p[3] = ub[3];
            } else {"""),
    ("sg_wpr.hip", """                f[0] = __builtin_amdgcn_alignbyte(R.v[1], R.v[0], mac_shift);
                f[1] = __builtin_amdgcn_alignbyte(R.v[2], R.v[1], mac_shift);
                const uint32_t v2 = __builtin_amdgcn_alignbyte(R.v[3], R.v[2], mac_shift);
                const uint32_t p2 = __builtin_amdgcn_alignbyte(R.p[3], R.p[2], mac_shift);
                f[2] = (v2 & 0x00ffffffu) | (p2 & 0xff000000u);
                f[3] = __builtin_amdgcn_alignbyte(R.p[4], R.p[3], mac_shift);""",
     """                f[0] = R.v[0];
                f[1] = R.v[1];
                f[2] = (R.v[2] & 0x00ffffffu) | (R.p[2] & 0xff000000u);
                f[3] = R.p[3];"""),
]
