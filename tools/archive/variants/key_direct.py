# keying pre-pass without LDS staging: every lane stores its own 640-byte record
# (flat stores at a 320-byte lane stride), so that occupancy is set by VGPRs alone
EDITS = [
("sg_wpr.hip", "    __shared__ uint32_t stage[kWprKeyThreads * kWprKeyStride];\n",
               "    __shared__ uint32_t junk[kWprKeyStride];  // inactive lanes' stores\n"),
("sg_wpr.hip", "    uint32_t* st = stage + lane * kWprKeyStride;\n", "    uint32_t* st = junk;\n"),
("sg_wpr.hip", "    // ---- second half: lo[b] = R^b, hi[h][a] = 2^(32 h) R^(8 a) (R = r^4) ----\n",
               "    st = act ? wpr_tab_half(wl, slot, 1u) : junk;\n    // ---- second half: lo[b] = R^b, hi[h][a] = 2^(32 h) R^(8 a) (R = r^4) ----\n"),
("sg_wpr.hip", "    __syncthreads();\n    wpr_flush_half(wl, slot0, 1u, stage, lane);\n    __syncthreads();\n",
               "    st = act ? wpr_tab_half(wl, slot, 0u) : junk;\n"),
("sg_wpr.hip", "    __syncthreads();\n    wpr_flush_half(wl, slot0, 0u, stage, lane);\n}\n", "}\n"),
]
