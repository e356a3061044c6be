# timing only (wrong tags): sg_wpr_kernel without the per-record epilogue's
# arithmetic (no exact assembly of the accumulator, no reduction, no W
# product, no DPP lane sum); the tag is taken from lane 63's raw entries
EDITS = [
    ("sg_wpr.hip", """#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint64_t yv = mad_i64_i32_1(acc[4 * m], kSeed);  // exact mod 2^64: the sum is positive
            yv = mad_i64_i32(acc[4 * m + 1], 256u, yv);
            yv = mad_i64_i32(acc[4 * m + 2], 65536u, yv);
            yv = mad_i64_i32(acc[4 * m + 3], 16777216u, yv);
            xw[2 * m] = (uint32_t)yv;
            xw[2 * m + 1] = (uint32_t)(yv >> 32);
        }
        F26 f = fmul(reduce_words8(xw), W);
        {""", """        (void)kSeed; (void)xw;
        F26 f = {(uint32_t)acc[0] ^ W.v0, (uint32_t)acc[1] ^ W.v1, (uint32_t)acc[2] ^ W.v2, (uint32_t)acc[3] ^ W.v3,
                 (uint32_t)acc[4] ^ W.v4};
        if (false) {"""),
]
