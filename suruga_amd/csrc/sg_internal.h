// sg_internal.h -- shared between the HIP kernels (sg_kernels.hip) and the
// C-ABI host layer (sg_capi.cpp).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sg {

constexpr uint32_t kThreads = 256;        // one record per 256-thread workgroup
constexpr uint32_t kKeyRecWords = 88;     // per-record keying output (u32 words, 352 B)
// keying record layout (u32 words): r[4] clamped Poly1305 r (radix 2^32),
// s[4] (second half of keystream block 0), then with R = r^k (k = MAC blocks
// per lane, see mac_geom in sg_kernels.hip) 5-limb radix-2^26 powers ordered so
// that a record with PL MAC lanes needs only a prefix (kKeyUsedWords(PL)):
//   R^0 (as hi[0]), lo[j] = R^j (j = 0..7), hi[i] = R^(8 i) (i = 1..7)
// MAC lane t scales its partial sum by R^(PL-1-t) = hi[e >> 3] lo[e & 7].
constexpr uint32_t kR32Off = 0;
constexpr uint32_t kSOff = 4;
__host__ __device__ constexpr uint32_t key_lo_off(uint32_t j) { return 13u + 5u * j; }
__host__ __device__ constexpr uint32_t key_hi_off(uint32_t i) { return i == 0u ? 8u : 48u + 5u * i; }
__host__ __device__ constexpr uint32_t key_used_words(uint32_t PL) {
    return PL <= 8u ? 13u + 5u * PL : 53u + 5u * (PL / 8u - 1u);
}
static_assert(key_used_words(64) == kKeyRecWords, "keying record layout");

// Keying record of the wave-per-record kernel (sg_wpr.hip), u32 words; F26
// entries are 5 radix-2^26 limbs.  With delta = 0/1 from the geometry
// (wpr_geom), R = r^4 and T = r^128:
//   s[4]                                    second half of keystream block 0
//   ctot[5]                                 the record's constant term
//   rd[5][5]  = r^(1 + delta + u)          u = 0..4
//   tk[8][5]  = T^k                         k = 0..7
//   lo[8][5]  = R^b                         b = 0..7
//   hi[2][4][5] = 2^(32 h) R^(8 a)          h = 0..1, a = 0..3
constexpr uint32_t kWS = 0;
constexpr uint32_t kWCtot = 4;
constexpr uint32_t kWRd = 12;
constexpr uint32_t kWTk = 40;
constexpr uint32_t kWLo = 80;
constexpr uint32_t kWHi = 120;
constexpr uint32_t kWprRecWords = 160;
// Record descriptor of a listed wave-per-record record (mixed batches), u32
// words, indexed like the keying records by the record's slot in its bucket:
//   in_off[2] out_off[2] n rec key_index n14 n15 0 0 0
constexpr uint32_t kWprDescWords = 12;

// Kernel parameters (passed by value as kernarg).
struct KParams {
    const uint8_t* keys;
    const uint32_t* key_index;
    uint32_t num_keys;       // >= 1; key indices are clamped to num_keys - 1 (no read outside the table)
    const uint64_t* seq;
    uint64_t seq0;
    const uint8_t* nonces;
    const uint8_t* ads;
    const uint8_t* in;
    const uint64_t* in_off;
    uint64_t in_stride;
    uint8_t* out;
    const uint64_t* out_off;
    uint64_t out_stride;
    const uint32_t* len;
    uint8_t* status;
    uint32_t* ws;            // count * kKeyRecWords (kWprRecWords for sg_wpr.hip) keying records
    uint32_t uniform_len;
    uint32_t count;
    uint32_t ad_len;         // explicit mode
    uint32_t ad_stride;
    uint32_t tls;            // 1 = SG_BATCH_TLS
    uint32_t tls_hdr;        // content_type | major << 8 | minor << 16
    uint32_t lds_rec_bytes;  // LDS bytes per record slot of the launched size class
    uint32_t wpr_mix;        // mixed batch: route eligible records to the wave-per-record buckets
    uint32_t pack_mix;       // mixed batch: route eligible small records to the packed kernel (sg_pack.hip)
};

// Size classes of the AEAD kernel: class c (0..7) holds records of
// n <= 128 << c bytes (class 7: the rest, up to SG_MAX_RECORD_LEN) and gives
// each record L = 2 << c lanes, one 64-byte ChaCha20 block per lane for
// c < 7; the MAC runs on PL = min(L, 64) lanes.  A 256-thread workgroup serves
// 256 / L records.  Mixed sizes are bucketed on the device (sg_classify_kernel).
constexpr uint32_t kNumClasses = 8;
// Mixed batches also route TLS records of 4 KiB < n <= 16 KiB, n a multiple of
// 64, 16-byte aligned, to the wave-per-record kernel (sg_wpr.hip): bucket
// J = ceil(n / 4096) = 2..4 (the record's chunk count), lists kNumClasses + J - 2.
constexpr uint32_t kWprBuckets = 3;
constexpr uint32_t kWprMinJ = 2;
// ... and TLS records of 64 B <= n <= 4 KiB, n a multiple of 64, 16-byte
// aligned, to the packed kernel (sg_pack.hip): list kPackList.
constexpr uint32_t kPackList = kNumClasses + kWprBuckets;
constexpr uint32_t kNumLists = kPackList + 1u;
constexpr uint32_t kListGridPerCU = 8;   // workgroups per CU for list-driven launches

__host__ __device__ inline uint32_t size_class(uint32_t n) {
    if (n <= 128u) return 0u;
    const uint32_t c = 32u - (uint32_t)__builtin_clz((n - 1u) >> 7);
    return c < 7u ? c : 7u;
}
__host__ __device__ constexpr uint32_t class_lanes(uint32_t c) { return 2u << c; }
__host__ __device__ constexpr uint32_t class_mac_lanes(uint32_t c) { return class_lanes(c) < 64u ? class_lanes(c) : 64u; }
__host__ __device__ constexpr uint32_t class_max(uint32_t c) { return c < 7u ? 128u << c : 0xffffffffu; }
// LDS bytes of one record slot: virtual-block space (16 bytes x max virtual blocks
// 2*PL) | ad || le64 (16-rounded) | ct (64-rounded) | le64(n) + zeros
__host__ __device__ inline uint32_t lds_rec_bytes(uint32_t cls, uint32_t adlen, uint32_t max_n) {
    const uint32_t PL = class_mac_lanes(cls);
    return 32u * PL + ((adlen + 8u + 15u) & ~15u) + ((max_n + 63u) & ~63u) + 64u;
}

// Wave-per-record kernel (sg_wpr.hip): uniform batches of full 16 KiB TLS
// records (n = RECORD_MAX_LEN = 2^14, tls.rs:32, the size TlsWriter::write_data
// gives every record but a stream's tail), 16-byte aligned strided layout, any
// AD length.  One wave per record, eight records per 512-thread workgroup.
constexpr uint32_t kWprN = 16384;
// Workspace (u32 words) for a batch of `count` records:
//   [0, 88 count)                   size-class keying records (by record index)
//   [88 count, 248 count)           wave-per-record keying records (by slot)
//   [248 count, 260 count)          wave-per-record descriptors (by slot)
//   [260 count, 272 count)          kNumLists record lists
//   then kNumLists populations, the over-long count, kWprBuckets + 1 group
//   counters and the packed launch's run counter
constexpr uint32_t kWsWprTab = kKeyRecWords;
constexpr uint32_t kWsWprDesc = kWsWprTab + kWprRecWords;
constexpr uint32_t kWsLists = kWsWprDesc + kWprDescWords;
constexpr uint32_t kWsRecWords = kWsLists + kNumLists;
constexpr uint32_t kWsTailWords = kNumLists + 1u + kWprBuckets + 2u;
__host__ __device__ inline uint64_t ws_words(uint32_t count) { return (uint64_t)count * kWsRecWords + kWsTailWords; }
// the counts / counters tail
__host__ __device__ inline uint32_t* ws_tail(uint32_t* ws, uint32_t count) { return ws + (uint64_t)count * kWsRecWords; }
constexpr uint32_t kTailOver = kNumLists;           // records longer than max_n
constexpr uint32_t kTailCtr = kNumLists + 1u;       // + b: group counter of wpr bucket b, + kWprBuckets: uniform C1 launch
constexpr uint32_t kTailPackCtr = kTailCtr + kWprBuckets + 1u;  // run counter of the packed launch
hipError_t device_cus(int* cus);  // CUs of the current device (cached)

// A wave-per-record bucket launch (mixed batch) or the uniform launch (list NULL).
struct WprList {
    const uint32_t* list;    // record indices (bucket list) or NULL: slot = record
    uint32_t count;          // records in the launch
    uint32_t* tab;           // keying records, kWprRecWords per slot
    uint32_t* desc;          // descriptors, kWprDescWords per slot (list launches)
    uint32_t* ctr;           // the launch's group counter (zeroed by its keying kernel)
};

// Keying jobs of the size-class keying kernel: njobs == 0 keys every record
// of the batch by index, otherwise the records of the listed size classes.
struct KeyJobs {
    const uint32_t* list[kNumClasses];
    uint32_t count[kNumClasses];
    uint32_t blk0[kNumClasses];  // first 64-record block of each job
    uint32_t njobs;
};

bool wpr_enabled();  // sg_set_lockstep / SG_LOCKSTEP environment switch
int set_wpr(int enable);
// keying pre-pass + record kernel; ev_mid (may be NULL) is recorded between them
hipError_t launch_wpr(const KParams& p, bool open, hipStream_t s, hipEvent_t ev_keyed, hipEvent_t ev_start);
// wave-per-record buckets of a mixed batch (wl[b]: J = kWprMinJ + b chunks):
// one keying launch for every bucket, then the record kernel of one bucket
hipError_t launch_wpr_keying_lists(const KParams& p, bool open, const WprList* wl, hipStream_t s);
hipError_t launch_wpr_list(const KParams& p, bool open, uint32_t J, const WprList& wl, hipStream_t s);
const char* wpr_kernel_config();
const char* class_kernel_config();

// Seal/open launch of a batch that is not a uniform 16 KiB one.  uniform:
// every record is in size_class(max_n) (keying, direct launch); otherwise
// classify into the workspace lists (kNumLists x count, populations in the
// tail), key the listed records and launch per list: the packed kernel
// (p.pack_mix) ahead of the population readback, the wave-per-record buckets
// (p.wpr_mix) and the size classes after it, on up to three streams that are
// joined into s before the call returns.  The tail's over-long count receives
// the records longer than max_n, which are skipped (open: status 3); *over
// receives that count when the populations are read back (not under capture).
// ev_keyed / ev_start (may be NULL) are recorded after the keying pre-passes
// (mixed batches: after classify, before the packed launch)
hipError_t launch_aead(const KParams& p, bool open, uint32_t max_n, bool uniform, hipStream_t s, uint32_t* over,
                       hipEvent_t ev_keyed, hipEvent_t ev_start);
// Eligibility of one record of a mixed batch for the wave-per-record buckets:
// the bucket J (kWprMinJ..4) or 0.  Shared by the classify and keying kernels.
__host__ __device__ inline uint32_t wpr_bucket_of(uint32_t n, uint64_t in_addr, uint64_t out_addr) {
    if (n <= 4096u || n > kWprN || (n & 63u) || ((in_addr | out_addr) & 15u)) return 0u;
    return (n + 4095u) >> 12;
}
// Eligibility of one record of a mixed batch for the packed small-record kernel.
__host__ __device__ inline bool pack_ok(uint32_t n, uint64_t in_addr, uint64_t out_addr) {
    return n >= 64u && n <= 4096u && (n & 63u) == 0u && ((in_addr | out_addr) & 15u) == 0u;
}
bool pack_enabled();  // sg_set_packed / SG_PACK environment switch
int set_pack(int enable);
// packed launch on a persistent grid: the list's population *cnt and the run
// counter *ctr (zero at launch) live on the device
hipError_t launch_pack(const KParams& p, bool open, const uint32_t* list, const uint32_t* cnt, uint32_t* ctr,
                       hipStream_t s);
const char* pack_kernel_config();
// zero the output of every record whose open status is 1 (wrong mac)
hipError_t launch_scrub(const KParams& p, hipStream_t s);
// record-layer framing in HBM (sg_record.cpp zero-copy path): build the wire
// image of `count` records (pitch = 5 + frag; the last record's fragment
// last_frag) from aligned fragment slots, or take the fragments of a wire
// image of equal records back into slots
hipError_t launch_frame(const uint8_t* src, uint32_t src_stride, uint8_t* dst, uint32_t pitch, uint32_t count,
                        uint32_t frag, uint32_t last_frag, uint32_t hdr, hipStream_t s);
hipError_t launch_unframe(const uint8_t* src, uint32_t pitch, uint8_t* dst, uint32_t dst_stride, uint32_t count,
                          uint32_t frag, hipStream_t s);
// dst[0, n) <- src[0, n) by a kernel (dst: the caller's registered host memory,
// written over the host link; src 4-byte aligned)
hipError_t launch_copy_out(const uint8_t* src, uint8_t* dst, uint64_t n, hipStream_t s);
hipError_t launch_fill(uint8_t* buf, uint64_t stride, uint32_t len, uint32_t count, uint64_t seed,
                       uint64_t j0, hipStream_t s);
hipError_t launch_compare(const uint8_t* a, uint64_t sa, const uint8_t* b, uint64_t sb, uint32_t len,
                          uint32_t count, unsigned long long* mism, hipStream_t s);

}  // namespace sg
