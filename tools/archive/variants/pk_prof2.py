# analysis build (output unchanged; build with -DSG_PACK_PROFILE=1): wave 0 of
# each workgroup also sums, over the chunk rounds of its last run, the clocks
# before the ChaCha20 asm (chunk loads issued, record lookup, slot reads), in
# the asm (80 s_barrier included) and after it (feed-forward, XOR, stores,
# MAC share, LDS atomics), in stamps 12-14, and its round count in 15
# (tools/pack_phase.py prints them)
EDITS = [
("sg_pack.hip", "constexpr uint32_t kProfWgs = 8192, kProfStamps = 12;",
 "constexpr uint32_t kProfWgs = 8192, kProfStamps = 16;"),
("sg_pack.hip",
"""    const uint32_t pos = 2u * (wave & 3u) + (wave >> 2);
    for (uint32_t k = 0; k < nrounds; ++k) {
        const uint32_t c = kPackWaves * k + pos;""",
"""    const uint32_t pos = 2u * (wave & 3u) + (wave >> 2);
    uint64_t a_pre = 0, a_arx = 0, a_post = 0;
    uint32_t a_n = 0;
    for (uint32_t k = 0; k < nrounds; ++k) {
        const uint64_t q0 = __builtin_amdgcn_s_memtime();
        const uint32_t c = kPackWaves * k + pos;"""),
("sg_pack.hip",
"""        const uint64_t live = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
        for (int dr = 0; dr < 10; ++dr) {""",
"""        const uint64_t live = __builtin_amdgcn_ballot_w64(valid);
        const uint64_t q1 = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int dr = 0; dr < 10; ++dr) {"""),
("sg_pack.hip",
"""                         : "scc");
        }
        if (valid) {
            // feed-forward (chacha20.rs:104-106) and XOR (chacha20.rs:143-153)""",
"""                         : "scc");
        }
        const uint64_t q2 = __builtin_amdgcn_s_memtime();
        if (valid) {
            // feed-forward (chacha20.rs:104-106) and XOR (chacha20.rs:143-153)"""),
("sg_pack.hip",
"""            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);
        }
    }""",
"""            atomicAdd(reinterpret_cast<unsigned long long*>(ac + 4), (unsigned long long)t.v1);
        }
        const uint64_t q3 = __builtin_amdgcn_s_memtime();
        a_pre += q1 - q0;
        a_arx += q2 - q1;
        a_post += q3 - q2;
        ++a_n;
    }
    if (wave == 0u && lane == 0u && blockIdx.x < kProfWgs) {
        g_pack_prof[blockIdx.x][12] = a_pre;
        g_pack_prof[blockIdx.x][13] = a_arx;
        g_pack_prof[blockIdx.x][14] = a_post;
        g_pack_prof[blockIdx.x][15] = a_n;
    }"""),
]
