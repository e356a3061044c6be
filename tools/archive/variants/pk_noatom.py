# timing only (wrong tags): the packed kernel's lane terms are folded into a
# register instead of the LDS accumulator (no LDS atomics in the chunk loop);
# the bound of any cheaper accumulation
EDITS = [
    ("sg_pack.hip", """                atomicAdd(ac + 0, t.v0);
                atomicAdd(ac + 1, t.v2);
                atomicAdd(ac + 2, t.v3);
                atomicAdd(ac + 3, t.v4);
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);""",
     """                fold_sink ^= t.v0 ^ t.v1 ^ t.v2 ^ t.v3 ^ t.v4 ^ (uint32_t)(uintptr_t)ac;"""),
    ("sg_pack.hip", """    const uint32_t pos = 2u * (wave & 3u) + (wave >> 2);
""", """    const uint32_t pos = 2u * (wave & 3u) + (wave >> 2);
    uint32_t fold_sink = 0u;
"""),
    ("sg_pack.hip", """    SG_STAMP(0u, 3);
    SG_STAMP(7u, 7);
""", """    SG_STAMP(0u, 3);
    SG_STAMP(7u, 7);
    if (fold_sink == 0x9e3779b9u) L.acc[0] = 1u;  // (keeps the terms live)
"""),
]
