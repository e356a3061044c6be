# Round 6 probe (bit-exact): the mixed batch's packed launch after the keying
# instead of ahead of the host's population wait -- the keying (on its side
# stream) gets the GPU first, then the packed kernel on the batch's stream and
# the J = 4 / 3 buckets on the side streams start together, so that no gap
# remains between the packed kernel's end and the buckets' start (r06o trace:
# 22-35 us per batch in which the keying runs on a nearly idle GPU)
EDITS = [
    ("sg_kernels.hip", """        if (p.pack_mix && (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, tail + kPackList,
                                           tail + kTailPackCtr, s)) != hipSuccess)
            return e;
        if ((e = hipEventSynchronize(pin.ev)) != hipSuccess) return e;""",
     """        if ((e = hipEventSynchronize(pin.ev)) != hipSuccess) return e;"""),
    ("sg_kernels.hip", """    if ((e = mark(ev_keyed, s)) != hipSuccess || (e = mark(ev_start, s)) != hipSuccess) return e;
    if (p.wpr_mix && exact) {  // most chunks first""", """    if ((e = mark(ev_keyed, s)) != hipSuccess || (e = mark(ev_start, s)) != hipSuccess) return e;
    if (exact && p.pack_mix && (e = launch_pack(p, OPEN, lists + (uint64_t)kPackList * p.count, tail + kPackList,
                                                tail + kTailPackCtr, s)) != hipSuccess)
        return e;
    if (p.wpr_mix && exact) {  // most chunks first"""),
]
