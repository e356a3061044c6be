# packed kernel: lane terms accumulated per hi index.  W(i) = hi[i >> 3] lo[i & 7]
# (hi[a] = r^(1 + 32 a)); instead of the product per lane, the lane adds
# Q lo[i & 7] into the record's accumulator a = i >> 3 (8 per record, 5 u32
# limbs each: at most 8 lane terms per accumulator), and the finish applies
# the hi factors once per record by a Horner in R8 = r^32 over the eight
# accumulators, times r.  The constant term goes in at the finish as
# coefficients: (block0 + 2^128) r^5 lo[b'] at a' ((a', b') of i = nb - 1:
# r^B = r^(4 nb + 2) = W(nb - 1) r^5) and (n 2^40 + 2^104) at a = 0.  The hi
# table goes (setup: 7 fewer products), the per-lane hi read and product go,
# the finish gains 9 products; same-address atomics drop from up to 64 lanes
# to 8 per word.
EDITS = [
    ("sg_pack.hip", """constexpr uint32_t kTabWords = 65;
constexpr uint32_t kTabTop = 64;""", """constexpr uint32_t kTabWords = 33;  // lo[8] as 128-bit words, their top bits in word 32
constexpr uint32_t kTabTop = 32;"""),
    ("sg_pack.hip", """constexpr uint32_t kAccWords = SG_PACK_ACC64 ? 6u : 5u;  // v0 v2 v3 v4 | v1 (u64)  or  v0..v4""",
     """constexpr uint32_t kAccWords = 40u;  // 8 accumulators (one per hi index) x 5 limbs"""),
    ("sg_pack.hip", """// W(i) = r^(1 + 4 i) = hi[i >> 3] lo[i & 7]
__device__ __forceinline__ F26 tab_weight(const uint32_t* tb, uint32_t i) {
    const uint32_t top = tb[kTabTop];
    return fmul(tab_get(tb, i >> 3, top), tab_get(tb, 8u + (i & 7u), top));
}""", """__device__ __forceinline__ F26 tab_lo(const uint32_t* tb, uint32_t b) { return tab_get(tb, b, tb[kTabTop]); }"""),
    ("sg_pack.hip", """            const F26 r2 = fmul(r, r), R = fmul(r2, r2);
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
            tb[kTabTop] = top;
            SG_STAMP(0u, 10);
            // constant term (header comment): r^B = r^(4 nb + 2) = W(nb - 1) R r
            const uint32_t il = nb - 1u;
            const F26 wl = tab_weight(tb, il);
            const F26 rB = fmul(fmul(wl, R), r);
""", """            const F26 r2 = fmul(r, r), R = fmul(r2, r2);
            const uint32_t il = nb - 1u, bl = il & 7u;
            F26 y = f26_one(), lob = f26_one();
            uint32_t top = 0u;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                top |= tab_put(tb, b, y);
                if ((uint32_t)b == bl) lob = y;
                if (b < 7) y = fmul(y, R);
            }
            tb[kTabTop] = top;
            SG_STAMP(0u, 10);
            // constant term: (block0 + 2^128) r^B with r^B = hi[il >> 3] lo[il & 7] r^5:
            // its hi factor comes at the finish (coefficient of accumulator il >> 3)
            const F26 rB = fmul(fmul(lob, R), r);
"""),
    ("sg_pack.hip", """            const F26 sfx = words_to_f26(0u, n << 8, 0u, 256u, 0u);      // n 2^40 + 2^104
            store_f26(sl + kSCtot, fmul_add(blk0, rB, fmul(sfx, r)));""",
     """            store_f26(sl + kSCtot, fmul(blk0, rB));"""),
    ("sg_pack.hip", """            const F26 W = tab_weight(tb, i);
            uint32_t* ac = L.acc + kAccWords * m;
            if constexpr (SG_PACK_ACC64) {
                const F26 t = fmul(Q, W);
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 0),
                          (unsigned long long)t.v0 | ((unsigned long long)t.v2 << 32));
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 2),
                          (unsigned long long)t.v3 | ((unsigned long long)t.v4 << 32));
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);
            } else {
                const F26 t = ripple_full(fmul(Q, W));
                atomicAdd(ac + 0, t.v0);
                atomicAdd(ac + 1, t.v1);
                atomicAdd(ac + 2, t.v2);
                atomicAdd(ac + 3, t.v3);
                atomicAdd(ac + 4, t.v4);
            }""", """            const F26 t = fmul(Q, tab_lo(tb, i & 7u));
            uint32_t* ac = L.acc + kAccWords * m + 5u * (i >> 3);
            atomicAdd(ac + 0, t.v0);
            atomicAdd(ac + 1, t.v1);
            atomicAdd(ac + 2, t.v2);
            atomicAdd(ac + 3, t.v3);
            atomicAdd(ac + 4, t.v4);"""),
    ("sg_pack.hip", """        const uint32_t* ac = L.acc + kAccWords * m0;
        // (ACC64: v1 = lo + hi 2^32 -> hi 2^58 = (hi << 6) 2^52 joins limb 2)
        F26 f = SG_PACK_ACC64 ? carry1(F26{ac[0], ac[4], ac[1] + (ac[5] << 6), ac[2], ac[3]})
                              : carry1(F26{ac[0], ac[1], ac[2], ac[3], ac[4]});
        f = carry1(f26_add(f, load_f26(sl + kSCtot)));""", """        const uint32_t* ac = L.acc + kAccWords * m0;
        // h = sum_a coef_a hi[a] = r sum_a coef_a R8^a (Horner in R8 = r^32 = lo[7] lo[1]);
        // coef_a = acc[a] (<= 8 lane terms), + the block-0 term at a = (nb - 1) >> 3,
        // + (n 2^40 + 2^104) at a = 0
        const uint32_t* tb = L.tab + m0 * kTabWords;
        const uint32_t r0w = sl[kSR + 0], r1w = sl[kSR + 1], r2w = sl[kSR + 2], r3w = sl[kSR + 3];
        const F26 r = words_to_f26(r0w, r1w, r2w, r3w, 0u);
        const F26 R8 = fmul(tab_lo(tb, 7u), tab_lo(tb, 1u));
        const uint32_t al = (sl[kSNb] - 1u) >> 3;
        const F26 c0 = load_f26(sl + kSCtot);
        const F26 sfx = words_to_f26(0u, n << 8, 0u, 256u, 0u);
        F26 f = f26_zero();
#pragma unroll
        for (int a = 7; a >= 0; --a) {
            F26 co = load_f26(ac + 5u * (uint32_t)a);
            if ((uint32_t)a == al) co = f26_add(co, c0);
            if (a == 0) co = f26_add(co, sfx);
            co = carry1(co);
            f = a == 7 ? co : fmul_add(f, R8, co);
        }
        f = fmul(f, r);"""),
]
