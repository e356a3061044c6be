# packed kernel setup with a shorter critical path: the power tables from a
# depth-3 product tree instead of two 8-long product chains, and each table
# entry normalised by four v_mad_u64_u32 into words plus two folds of the
# bits >= 2^130 (instead of a two-pass carry ripple)
EDITS = [
    ("sg_pack.hip", """// table entry e <- x (fully reduced first; top bits collected by the caller)
__device__ __forceinline__ uint32_t tab_put(uint32_t* tb, uint32_t e, F26 x) {
    x = ripple_full(x);  // limbs < 2^26: x < 2^130
    tb[4u * e + 0] = x.v0 | (x.v1 << 26);
    tb[4u * e + 1] = (x.v1 >> 6) | (x.v2 << 20);
    tb[4u * e + 2] = (x.v2 >> 12) | (x.v3 << 14);
    tb[4u * e + 3] = (x.v3 >> 18) | (x.v4 << 8);
    return (x.v4 >> 24) << (2u * e);
}""", """// a * b + c (b wave-uniform) in one v_mad_u64_u32
__device__ __forceinline__ uint64_t pk_mad(uint32_t a, uint32_t b, uint64_t c) {
    uint64_t d, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(d), "=s"(cc) : "v"(a), "s"(b), "v"(c));
    return d;
}
// table entry e <- x, a product (limbs 0, 2..4 < 2^26, limb 1 < 2^26 + 2^7):
// X = sum v_i 2^(26 i) < 2^131 as words by four v_mad_u64_u32, then the bits
// >= 2^130 folded twice (2^130 = 5 mod p; the second fold ends below 2^130)
// (top bits collected by the caller)
__device__ __forceinline__ uint32_t tab_put(uint32_t* tb, uint32_t e, F26 x) {
    uint64_t t = pk_mad(x.v1, 1u << 26, (uint64_t)x.v0);
    uint32_t w0 = (uint32_t)t;
    t = pk_mad(x.v2, 1u << 20, t >> 32);
    uint32_t w1 = (uint32_t)t;
    t = pk_mad(x.v3, 1u << 14, t >> 32);
    uint32_t w2 = (uint32_t)t;
    t = pk_mad(x.v4, 1u << 8, t >> 32);
    uint32_t w3 = (uint32_t)t, w4 = (uint32_t)(t >> 32);  // w4 < 8
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        uint32_t c;
        w0 = addc(w0, 5u * (w4 >> 2), 0u, &c);
        w1 = addc(w1, 0u, c, &c);
        w2 = addc(w2, 0u, c, &c);
        w3 = addc(w3, 0u, c, &c);
        w4 = (w4 & 3u) + c;
    }
    tb[4u * e + 0] = w0;
    tb[4u * e + 1] = w1;
    tb[4u * e + 2] = w2;
    tb[4u * e + 3] = w3;
    return w4 << (2u * e);
}"""),
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
            const F26 r2 = fmul(r, r), R = fmul(r2, r2);
            // lo[b] = R^b and hi[a] = r R^(8 a) by a product tree (depth 3 from R)
            const F26 R2 = fmul(R, R), R3 = fmul(R2, R), R4 = fmul(R2, R2);
            const F26 R5 = fmul(R4, R), R6 = fmul(R4, R2), R7 = fmul(R4, R3), R8 = fmul(R4, R4);  // R8 = r^32
            const F26 S2 = fmul(R8, R8), S3 = fmul(S2, R8), S4 = fmul(S2, S2);
            const F26 lo[8] = {f26_one(), R, R2, R3, R4, R5, R6, R7};
            const F26 hs[8] = {f26_one(), R8, S2, S3, S4, fmul(S4, R8), fmul(S4, S2), fmul(S4, S3)};
            uint32_t top = tab_put(tb, 8u, lo[0]);  // (1: its top bits are 0)
#pragma unroll
            for (int b = 1; b < 8; ++b) top |= tab_put(tb, 8u + b, lo[b]);
#pragma unroll
            for (int a = 0; a < 8; ++a) top |= tab_put(tb, a, a == 0 ? r : fmul(hs[a], r));
            tb[kTabTop] = top;"""),
]
