# bucket streams: all three buckets on the keying stream (J = 4, 3, 2 in
# order), overlapping only the packed launch's tail; no second side stream
EDITS = [
    ("sg_kernels.hip", "    hipStream_t js[kWprBuckets] = {s, ks, ks};  // bucket b (J = 2 + b)",
     "    hipStream_t js[kWprBuckets] = {ks, ks, ks};  // bucket b (J = 2 + b)"),
    ("sg_kernels.hip", "        if (p.wpr_mix && side[1].acquire() == hipSuccess) {", "        if (false && side[1].acquire() == hipSuccess) {"),
]
