# the final round-4 mixed-batch flow without its side streams: the persistent
# packed launch stays ahead of the population wait, the keying and every bucket
# run on the batch's stream (round 4's pk_persist configuration; A/B control)
EDITS = [
    ("sg_kernels.hip",
     "        if (((p.pack_mix && pop[kPackList] != 0u) || (p.wpr_mix && nbuckets != 0u)) && side[0].acquire() == hipSuccess) {",
     "        if (false && side[0].acquire() == hipSuccess) {"),
]
