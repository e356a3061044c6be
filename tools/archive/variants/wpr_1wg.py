# residency probe (bit-exact): the 16 KiB kernel at one 512-thread workgroup per
# CU (2 waves per SIMD: one lock-step pair) instead of two -- the residency a
# two-blocks-per-lane form (8 KiB per wave iteration) would need.  The launch
# asks for 120 KiB of LDS so that a second workgroup cannot fit, and the
# persistent grid has one workgroup per CU.
EDITS = [
    ("sg_wpr.hip", "const uint32_t grid = 2u * (uint32_t)cus;", "const uint32_t grid = 1u * (uint32_t)cus;"),
    ("sg_wpr.hip",
     "#define SG_WPR_LAUNCH(O, T) hipLaunchKernelGGL((sg_wpr_kernel<O, T, 4, false>), dim3(grid), dim3(512), kWprWgLds, s, p, wl)",
     "#define SG_WPR_LAUNCH(O, T) hipLaunchKernelGGL((sg_wpr_kernel<O, T, 4, false>), dim3(grid), dim3(512), 120u * 1024u, s, p, wl)"),
]
