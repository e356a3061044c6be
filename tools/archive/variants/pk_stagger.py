# the three persistent workgroups of a CU start a third of a run apart (slot s
# of the CU, s = blockIdx / (grid / 3), waits s x 40 K clocks before its first
# run): tests whether the co-resident workgroups' setups, which start
# together and stay in phase, leave the CU latency-bound at the same time
# (output unchanged)
EDITS = [("sg_pack.hip",
"""    const uint32_t nruns = (count + kPackRecs - 1u) / kPackRecs;
    for (;;) {""",
"""    const uint32_t nruns = (count + kPackRecs - 1u) / kPackRecs;
    {
        const uint32_t per = gridDim.x / 3u;
        const uint32_t slot = per ? (blockIdx.x / per) % 3u : 0u;
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < 40000ull * slot) __builtin_amdgcn_s_sleep(32);
    }
    for (;;) {"""),
]
