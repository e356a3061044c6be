# Round 6, timing only (wrong output): sg_wpr_kernel with the ChaCha20 ARX
# stream and nothing of the record's data movement or MAC: no LDS-DMA of the
# chunks or the keying table, no nt stores, no T windows / operand preparation
# / MFMA (the prologue and epilogue run on whatever the LDS holds).  What is
# left: the ten double rounds per chunk with their barriers, the lanes' LDS
# block reads, feed-forward, XOR, the staging write and read-out -- the ARX
# stream at the product's residency, priced at the power cap in-product.
EDITS = [
    ("sg_wpr.hip", """__device__ __forceinline__ void dma_sv(uint32_t l0, const void* sbase, uint32_t voff) {
    uint32_t keep;""", """__device__ __forceinline__ void dma_sv(uint32_t l0, const void* sbase, uint32_t voff) {
    return;
    uint32_t keep;"""),
    ("sg_wpr.hip", """__device__ __forceinline__ void dma_one(uint32_t l0, const void* g) {
    uint32_t keep;""", """__device__ __forceinline__ void dma_one(uint32_t l0, const void* g) {
    return;
    uint32_t keep;"""),
    ("sg_wpr.hip", """__device__ __forceinline__ void gst16_s(const void* sbase, uint32_t voff, const u32x4& v) {
    static_assert(OFF < 4096u, "global instruction offset");""", """__device__ __forceinline__ void gst16_s(const void* sbase, uint32_t voff, const u32x4& v) {
    static_assert(OFF < 4096u, "global instruction offset");
    return;"""),
    ("sg_wpr.hip", """                gst16(pend_dst + 1024u * k + 16u * ln, ld16(pb + 1024u * k + 16u * wunit));""",
     """                asm volatile("" :: "v"(ld16(pb + 1024u * k + 16u * wunit)));"""),
    ("sg_wpr.hip", """                st16(outb + n, u32x4{tw[0], tw[1], tw[2], tw[3]});  // ct || tag (chacha20_poly1305.rs:55)""",
     """                asm volatile("" :: "v"(tw[0]), "v"(tw[1]), "v"(tw[2]), "v"(tw[3]));"""),
    ("sg_wpr.hip", """                p.status[cd.rec] = diff != 0u ? 1u : 0u;""", """                asm volatile("" :: "v"(diff));"""),
    ("sg_wpr.hip", """        auto mac_load = [&](uint32_t jj, uint32_t i, MacRaw& R) {
""", """        auto mac_load = [&](uint32_t jj, uint32_t i, MacRaw& R) {
            return;
"""),
    ("sg_wpr.hip", """        auto mac_mfma_f = [&](const u32x4& f, const u32x4& a, bool first = false) {
""", """        auto mac_mfma_f = [&](const u32x4& f, const u32x4& a, bool first = false) {
            return;
"""),
    ("sg_wpr.hip", """        auto mac_frag = [&](const MacRaw& R) -> u32x4 {
            u32x4 f;
""", """        auto mac_frag = [&](const MacRaw& R) -> u32x4 {
            u32x4 f = {};
            return f;
"""),
]
