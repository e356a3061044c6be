# packed kernel: the lane's MAC term into the record accumulator with three
# 64-bit LDS atomics instead of five (v0 | v2 << 32 and v3 | v4 << 32 side by
# side in the same words as before: each of those limbs sums below 2^32 over
# a record's at most 64 terms, so the low half never carries into the high)
EDITS = [
    ("sg_pack.hip", """                atomicAdd(ac + 0, t.v0);
                atomicAdd(ac + 1, t.v2);
                atomicAdd(ac + 2, t.v3);
                atomicAdd(ac + 3, t.v4);
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);""",
     """                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 0),
                          (unsigned long long)t.v0 | ((unsigned long long)t.v2 << 32));
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 2),
                          (unsigned long long)t.v3 | ((unsigned long long)t.v4 << 32));
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);"""),
]
