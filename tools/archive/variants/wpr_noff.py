# timing only (wrong output): sg_wpr_kernel without the feed-forward and
# keystream XOR (output = input; the rounds still run)
EDITS = [
    ("sg_wpr.hip", """            O[0] = D[0] ^ u32x4{x[0] + kSigma0, x[1] + kSigma1, x[2] + kSigma2, x[3] + kSigma3};
            O[1] = D[1] ^ u32x4{x[4] + kw[0], x[5] + kw[1], x[6] + kw[2], x[7] + kw[3]};
            O[2] = D[2] ^ u32x4{x[8] + kw[4], x[9] + kw[5], x[10] + kw[6], x[11] + kw[7]};
            O[3] = D[3] ^ u32x4{x[12] + ctr, x[13], x[14] + n14, x[15] + n15};""",
     """            O[0] = D[0];
            O[1] = D[1];
            O[2] = D[2];
            O[3] = D[3];"""),
]
