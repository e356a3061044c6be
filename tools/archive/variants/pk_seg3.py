# pk_seg on the three-atomic accumulator (product since fcf5645): the lane terms of one record are summed across the lanes of
# each 16-lane row first (segmented scan with DPP row shifts 1, 2, 4, 8: the
# lanes of a record are contiguous in the chunk), so only the last lane of a
# record's run in each row adds into the LDS accumulator -- fewer same-address
# LDS atomics (bank-conflict cycles ~14 % of the packed kernel's CU time, r04t)
EDITS = [
    ("sg_pack.hip", """        uint32_t m = 0u;
        if (c < nchunks) {
            const uint32_t mlo = L.bits[2u * c], mhi = L.bits[2u * c + 1u];""",
     """        uint32_t m = 0u, mlo = 0u, mhi = 0u;
        if (c < nchunks) {
            mlo = __builtin_amdgcn_readfirstlane(L.bits[2u * c]);  // (wave-uniform: SGPRs across the rounds)
            mhi = __builtin_amdgcn_readfirstlane(L.bits[2u * c + 1u]);"""),
    ("sg_pack.hip", """            uint32_t* ac = L.acc + kAccWords * m;
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
            }
        }
    }""", """            F26 t = fmul(Q, W);
            // segmented sum over the lanes of each 16-lane row: a record's lanes
            // are contiguous (the lanes without a block follow every valid one,
            // so a row shift that stays in the segment reads a valid lane); the
            // segment in the row starts at the later of the record's first lane
            // (highest start bit at or below this lane) and the row's first
            const uint64_t starts = ((uint64_t)mhi << 32) | mlo;
            const uint64_t at_or_below = starts & ((2ull << lane) - 1ull);
            const uint32_t seg0 = at_or_below ? 63u - (uint32_t)__builtin_clzll(at_or_below) : 0u;
            const uint32_t row0 = lane & ~15u;
            const uint32_t dist = lane - (seg0 > row0 ? seg0 : row0);
#define SG_SEG_STEP(D, CTRL)                                                                                  \\
            {                                                                                                 \\
                const uint32_t mk = dist >= (D) ? 0xffffffffu : 0u;                                            \\
                t.v0 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t.v0, CTRL, 0xf, 0xf, true) & mk;     \\
                t.v1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t.v1, CTRL, 0xf, 0xf, true) & mk;     \\
                t.v2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t.v2, CTRL, 0xf, 0xf, true) & mk;     \\
                t.v3 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t.v3, CTRL, 0xf, 0xf, true) & mk;     \\
                t.v4 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t.v4, CTRL, 0xf, 0xf, true) & mk;     \\
            }
            SG_SEG_STEP(1u, 0x111)
            SG_SEG_STEP(2u, 0x112)
            SG_SEG_STEP(4u, 0x114)
            SG_SEG_STEP(8u, 0x118)
#undef SG_SEG_STEP
            // the last lane of the record's run in this row adds the run's sum
            // (limbs below 16 x (2^26 + 2^7); over a record's at most 64 terms the
            // accumulator words keep the bounds of the per-lane form)
            const bool next_starts = lane < 63u && ((starts >> (lane + 1u)) & 1ull);
            const bool tail = (lane & 15u) == 15u || next_starts || b + 1u >= total;
            if (tail) {
                uint32_t* ac = L.acc + kAccWords * m;
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 0),
                          (unsigned long long)t.v0 | ((unsigned long long)t.v2 << 32));
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 2),
                          (unsigned long long)t.v3 | ((unsigned long long)t.v4 << 32));
                atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);
            }
        }
    }"""),
]
