// sg_capi.cpp -- the C ABI declared in include/suruga_gpu.h.
//
// Host-side glue only: argument checking (mirroring the reference's panics /
// errors), per-device state (stream, keying workspace cache, timing events),
// staging for the single-record Encryptor/Decryptor calls, and the launches
// of the gfx950 kernels in sg_kernels.hip.  There is no CPU fallback: every
// seal/open goes through the HIP kernels or fails with an error code.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/suruga_gpu.h"
#include "sg_host.h"
#include "sg_internal.h"

namespace {
thread_local std::string g_err;
}  // namespace

namespace sg {

int fail(int code, const char* fmt, const char* detail) {
    char buf[512];
    std::snprintf(buf, sizeof buf, fmt, detail ? detail : "");
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char* where) {
    char buf[512];
    std::snprintf(buf, sizeof buf, "%s: %s", where, hipGetErrorString(e));
    g_err = buf;
    return SG_E_HIP;
}

}  // namespace sg

namespace {

using sg::fail;
using sg::hip_fail;

// A workspace of the library-owned cache.  Calls with no caller workspace
// take one that no other call is enqueuing on, make their stream wait for its
// previous user's work (`done`) and record `done` again after their launches,
// so reuse is ordered on the device even across streams and asynchronous
// calls; the host never blocks on it except to grow a buffer.
struct CachedWs {
    void* ptr = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
    bool used = false;   // `done` has been recorded
    bool held = false;   // a call is enqueuing on it
};

struct DeviceState {
    bool init = false;
    bool ok = false;
    std::vector<CachedWs*> pool;  // guarded by g_mu
};

std::mutex g_mu;  // device table, workspace pool bookkeeping (never held across a launch or a wait)
std::vector<DeviceState> g_dev;

// timing
struct TimedLaunch {
    hipEvent_t a, b;
    int kind;  // 0 keying, 1 seal, 2 open
};
std::mutex g_timing_mu;
bool g_timing = false;
std::vector<TimedLaunch> g_timed;
std::vector<hipEvent_t> g_event_pool;

hipEvent_t get_event() {  // caller holds g_timing_mu
    if (!g_event_pool.empty()) {
        hipEvent_t e = g_event_pool.back();
        g_event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Checks the device is a gfx950 part.  Caller holds g_mu.
int device_state(int dev, DeviceState** out) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(SG_E_NODEV, "no HIP device visible%s");
    if (dev < 0 || dev >= ndev) return fail(SG_E_ARG, "device ordinal out of range%s");
    if ((int)g_dev.size() < ndev) g_dev.resize(ndev);
    DeviceState& d = g_dev[dev];
    if (!d.init) {
        d.init = true;
        hipDeviceProp_t prop;
        SG_HIP(hipGetDeviceProperties(&prop, dev));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            d.ok = false;
            return fail(SG_E_NODEV, "device is %s, this library is built for gfx950 only", prop.gcnArchName);
        }
        d.ok = true;
    }
    if (!d.ok) return fail(SG_E_NODEV, "device not usable%s");
    *out = &d;
    return SG_OK;
}

// Take a cached workspace of >= need bytes for a call on stream s (the current
// device is d's).  Growing a buffer waits for its previous user only.
int ws_acquire(DeviceState* d, size_t need, hipStream_t s, CachedWs** out) {
    CachedWs* w = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (CachedWs* c : d->pool)
            if (!c->held && (!w || (c->bytes >= need && (w->bytes < need || c->bytes < w->bytes)))) w = c;
        if (!w) {
            w = new CachedWs();
            d->pool.push_back(w);
        }
        w->held = true;
    }
    auto release_on_error = [&](int rc) {
        std::lock_guard<std::mutex> lk(g_mu);
        w->held = false;
        return rc;
    };
    if (!w->done && hipEventCreateWithFlags(&w->done, hipEventDisableTiming) != hipSuccess)
        return release_on_error(fail(SG_E_HIP, "hipEventCreate failed%s"));
    if (w->bytes < need) {
        if (w->used && hipEventSynchronize(w->done) != hipSuccess)
            return release_on_error(fail(SG_E_HIP, "workspace event wait failed%s"));
        if (w->ptr) (void)hipFree(w->ptr);
        w->ptr = nullptr;
        w->bytes = 0;
        const size_t sz = need < (1u << 20) ? (1u << 20) : need;
        if (hipMalloc(&w->ptr, sz) != hipSuccess) return release_on_error(fail(SG_E_HIP, "workspace hipMalloc failed%s"));
        w->bytes = sz;
        w->used = false;
    }
    if (w->used && hipStreamWaitEvent(s, w->done, 0) != hipSuccess)
        return release_on_error(fail(SG_E_HIP, "hipStreamWaitEvent failed%s"));
    *out = w;
    return SG_OK;
}

void ws_release(CachedWs* w, hipStream_t s, bool launched) {
    if (launched && hipEventRecord(w->done, s) == hipSuccess) w->used = true;
    std::lock_guard<std::mutex> lk(g_mu);
    w->held = false;
}

int validate(const sg_batch* b, bool open) {
    if (!b) return fail(SG_E_ARG, "batch is NULL%s");
    if (b->count == 0) return SG_OK;
    if (!b->keys || !b->in || !b->out) return fail(SG_E_ARG, "keys/in/out must be non-NULL%s");
    if (((uintptr_t)b->keys & 3u) != 0) return fail(SG_E_ARG, "key table must be 4-byte aligned%s");
    if (b->num_keys == 0) return fail(SG_E_ARG, "num_keys must be >= 1%s");
    if (open && !b->status) return fail(SG_E_ARG, "open requires a status array%s");
    if (b->flags & ~(SG_BATCH_TLS | SG_BATCH_KEEP_FAILED)) return fail(SG_E_ARG, "unknown flags%s");
    if (!(b->flags & SG_BATCH_TLS)) {
        if (!b->nonces) return fail(SG_E_ARG, "explicit mode needs nonces%s");
        if (b->ad_len > SG_MAX_AD_LEN) return fail(SG_E_ARG, "ad_len exceeds SG_MAX_AD_LEN%s");
        if (b->ad_len && !b->ads) return fail(SG_E_ARG, "ad_len > 0 needs ads%s");
    }
    uint32_t maxl = b->len ? b->max_len : b->uniform_len;
    if (b->len && b->max_len == 0) return fail(SG_E_ARG, "max_len is required with len[]%s");
    uint32_t max_n = open ? (maxl >= 16 ? maxl - 16 : 0) : maxl;
    if (max_n > SG_MAX_RECORD_LEN) return fail(SG_E_ARG, "record longer than SG_MAX_RECORD_LEN%s");
    if ((b->flags & SG_BATCH_TLS) && max_n > 0xffffu)
        return fail(SG_E_ARG, "TLS mode record length must fit be16%s");
    return SG_OK;
}

// The wave-per-record kernel (sg_wpr.hip) takes uniform batches of full
// 16 KiB records in a 16-byte aligned strided layout; everything else runs on
// the size-class kernels.
bool wpr_eligible(const sg_batch* b, bool open) {
    if (!sg::wpr_enabled() || b->len || b->in_off || b->out_off) return false;
    if (b->uniform_len != (open ? sg::kWprN + SG_MAC_LEN : sg::kWprN)) return false;
    // per-record scalars are read as dwords: key index, sequence numbers, nonces
    if (((uintptr_t)b->key_index | (uintptr_t)b->seq) % 4u) return false;
    if (!(b->flags & SG_BATCH_TLS) && (uintptr_t)b->nonces % 4u) return false;
    return ((uintptr_t)b->in | (uintptr_t)b->out | b->in_stride | b->out_stride) % 16u == 0u;
}

// Keying + AEAD launches of one batch on stream s with workspace ws.
int launch_batch(const sg_batch* b, bool open, hipStream_t s, void* ws) {
    sg::KParams p;
    std::memset(&p, 0, sizeof p);
    p.keys = b->keys;
    p.key_index = b->key_index;
    p.num_keys = b->num_keys;
    p.seq = b->seq;
    p.seq0 = b->seq0;
    p.nonces = b->nonces;
    p.ads = b->ads;
    p.in = b->in;
    p.in_off = b->in_off;
    p.in_stride = b->in_stride;
    p.out = b->out;
    p.out_off = b->out_off;
    p.out_stride = b->out_stride;
    p.len = b->len;
    p.status = b->status;
    p.ws = (uint32_t*)ws;
    p.uniform_len = b->uniform_len;
    p.count = b->count;
    p.tls = (b->flags & SG_BATCH_TLS) ? 1u : 0u;
    p.ad_len = p.tls ? 13u : b->ad_len;
    p.ad_stride = b->ad_stride;
    p.tls_hdr = (uint32_t)b->content_type | ((uint32_t)b->ver_major << 8) | ((uint32_t)b->ver_minor << 16);
    const uint32_t maxl = b->len ? b->max_len : b->uniform_len;
    const uint32_t max_n = open ? (maxl >= 16u ? maxl - 16u : 0u) : maxl;
    const bool uniform = !b->len || sg::size_class(max_n) == 0u;
    const bool wpr = wpr_eligible(b, open);
    // mixed TLS batches: full-chunk records (4-16 KiB, multiples of 64 bytes)
    // go to the wave-per-record buckets; not under capture (they are launched
    // on the populations read back), and the per-record arrays are read as
    // dwords by the bucket kernels
    // (the packed kernel, sg_pack.hip, likewise takes the 64 B-4 KiB ones)
    if (!wpr && !uniform && p.tls && ((sg::wpr_enabled() && max_n > 4096u) || (sg::pack_enabled() && max_n >= 64u))) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        SG_HIP(hipStreamIsCapturing(s, &cap));
        const bool ok = cap == hipStreamCaptureStatusNone &&
                        ((uintptr_t)b->key_index | (uintptr_t)b->seq | (uintptr_t)b->len | (uintptr_t)b->in_off |
                         (uintptr_t)b->out_off) % 4u == 0u;
        p.wpr_mix = ok && sg::wpr_enabled() && max_n > 4096u;
        p.pack_mix = ok && sg::pack_enabled();
    }

    hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};
    bool timing = false;
    {
        std::lock_guard<std::mutex> lk(g_timing_mu);
        timing = g_timing;
        if (timing)
            for (auto& x : e) x = get_event();
    }
    // Every launch of the batch is enqueued before any error return: a record
    // longer than max_len only shows in the population readback, and the
    // other records' launches (and the timing bookkeeping) still follow it.
    uint32_t over = 0;
    hipError_t he = timing ? hipEventRecord(e[0], s) : hipSuccess;
    if (he == hipSuccess) {
        if (wpr)
            he = sg::launch_wpr(p, open, s, timing ? e[1] : nullptr, timing ? e[2] : nullptr);
        else
            he = sg::launch_aead(p, open, max_n, uniform, s, &over, timing ? e[1] : nullptr, timing ? e[2] : nullptr);
    }
    // failed opens hand out no plaintext (chacha20_poly1305.rs:89-93)
    if (he == hipSuccess && open && !(b->flags & SG_BATCH_KEEP_FAILED)) he = sg::launch_scrub(p, s);
    if (timing) {
        if (he == hipSuccess) he = hipEventRecord(e[3], s);
        std::lock_guard<std::mutex> lk(g_timing_mu);
        if (he == hipSuccess) {
            g_timed.push_back({e[0], e[1], 0});
            g_timed.push_back({e[2], e[3], open ? 2 : 1});
        } else {
            for (auto x : e)
                if (x) g_event_pool.push_back(x);
        }
    }
    if (he != hipSuccess) return hip_fail(he, "batch launch");
    if (over) return fail(SG_E_ARG, "records longer than max_len were not processed%s");
    return SG_OK;
}

int run_batch(const sg_batch* b, bool open) {
    int rc = validate(b, open);
    if (rc != SG_OK || b->count == 0) return rc;

    int dev = 0;
    SG_HIP(hipGetDevice(&dev));
    DeviceState* d = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        rc = device_state(dev, &d);
    }
    if (rc != SG_OK) return rc;
    // NULL = the null stream: ordered after the caller's earlier work on it
    // (torch's default stream is the null stream), and the call is synchronous
    hipStream_t s = (hipStream_t)b->stream;

    void* ws = b->workspace;
    CachedWs* cws = nullptr;
    const size_t need = sg_workspace_size(b->count);
    if (ws) {
        if (b->workspace_size < need) return fail(SG_E_ARG, "workspace too small%s");
        if ((uintptr_t)ws % 16u) return fail(SG_E_ARG, "workspace must be 16-byte aligned%s");
    } else {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        SG_HIP(hipStreamIsCapturing(s, &cap));
        if (cap != hipStreamCaptureStatusNone)
            return fail(SG_E_ARG, "a call under stream capture needs a caller workspace%s");
        if ((rc = ws_acquire(d, need, s, &cws)) != SG_OK) return rc;
        ws = cws->ptr;
    }
    rc = launch_batch(b, open, s, ws);
    if (cws) ws_release(cws, s, true);
    // NULL stream: the call returns when the batch is done, whatever it returns
    if (!b->stream) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess && rc == SG_OK) rc = hip_fail(e, "hipStreamSynchronize");
    }
    return rc;
}

}  // namespace

// ---------------------------------------------------------------------------
// single-record contexts (Encryptor / Decryptor)
// ---------------------------------------------------------------------------
using sg::fail;
using sg::hip_fail;

extern "C" {

size_t sg_key_size(void) { return SG_KEY_LEN; }
size_t sg_fixed_iv_len(void) { return 0; }
size_t sg_mac_len(void) { return SG_MAC_LEN; }
int sg_abi_version(void) { return SG_ABI_VERSION; }
const char* sg_last_error(void) { return g_err.c_str(); }
#ifndef SG_SOURCE_HASH
#define SG_SOURCE_HASH "0000000000000000"
#endif
// the hash of the sources this library was built from (suruga_amd/_build.py
// source_hash), also findable in the binary as the marker "sg-src:<hash>"
static const char kSrcMarker[] = "sg-src:" SG_SOURCE_HASH;
const char* sg_source_hash(void) { return kSrcMarker + 7; }
const char* sg_build_info(void) {
    static const std::string src = std::string(" [") + kSrcMarker + "]";
    static const std::string pk = std::string("; small records of mixed batches: ") + sg::pack_kernel_config() + src;
    static const std::string on = std::string("gfx950 ") + sg::wpr_kernel_config() + "; other batches: " +
                                  sg::class_kernel_config();
    static const std::string off = std::string("gfx950 ") + sg::class_kernel_config() + " (wave-per-record kernel off)";
    static const std::string on_pk = on + pk, off_pk = off + pk, on_s = on + src, off_s = off + src;
    const bool w = sg::wpr_enabled(), k = sg::pack_enabled();
    return w ? (k ? on_pk.c_str() : on_s.c_str()) : (k ? off_pk.c_str() : off_s.c_str());
}
size_t sg_workspace_size(uint32_t count) {
    // keying records, one list per size class, the class populations and the
    // count of records longer than max_len
    return (size_t)sg::ws_words(count) * 4u;
}

sg_ctx* sg_ctx_new(const uint8_t key[32], int device) {
    if (!key) {
        fail(SG_E_ARG, "key is NULL%s");
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> lk(g_mu);
        DeviceState* d = nullptr;
        if (device_state(device, &d) != SG_OK) return nullptr;
    }
    sg::DeviceGuard dg(device);
    if (!dg.ok) {
        fail(SG_E_HIP, "hipSetDevice failed%s");
        return nullptr;
    }
    sg_ctx* c = new sg_ctx();
    c->device = device;
    const size_t cap_in = sg::kSingleInOff + SG_MAX_RECORD_LEN + 64;
    const size_t cap_out = sg::kSingleOutOff + SG_MAX_RECORD_LEN + 64;
    bool ok = hipMalloc((void**)&c->d_key, 64) == hipSuccess &&
              hipHostMalloc((void**)&c->h_in, cap_in, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc((void**)&c->h_out, cap_out, hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&c->d_ws, sg_workspace_size(1)) == hipSuccess &&
              hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipMemcpy(c->d_key, key, 32, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {
        fail(SG_E_HIP, "context allocation failed%s");
        sg_ctx_free(c);
        return nullptr;
    }
    return c;
}

void sg_ctx_free(sg_ctx* c) {
    if (!c) return;
    sg::DeviceGuard dg(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    sg::record_staging_free(c->rec);
    (void)hipFree(c->d_key);
    (void)hipHostFree(c->h_in);
    (void)hipHostFree(c->h_out);
    (void)hipFree(c->d_ws);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static int single(sg_ctx* c, bool open, const uint8_t* nonce, size_t nonce_len, const uint8_t* in,
                  size_t in_len, const uint8_t* ad, size_t adlen, uint8_t* out) {
    if (!c) return fail(SG_E_ARG, "context is NULL%s");
    if (nonce_len != SG_NONCE_LEN || !nonce) return fail(SG_E_ARG, "nonce must be 8 bytes%s");
    if (adlen > SG_MAX_AD_LEN || (adlen && !ad)) return fail(SG_E_ARG, "bad additional data%s");
    if (in_len && !in) return fail(SG_E_ARG, "NULL buffer%s");
    if (open && in_len < SG_MAC_LEN) return SG_E_SHORT;  // chacha20_poly1305.rs:68-70
    const size_t n = open ? in_len - SG_MAC_LEN : in_len;
    if (!out && (open ? n : n + SG_MAC_LEN)) return fail(SG_E_ARG, "NULL buffer%s");  // empty pt: out may be NULL
    if (n > SG_MAX_RECORD_LEN) return fail(SG_E_ARG, "record longer than SG_MAX_RECORD_LEN%s");

    std::lock_guard<std::mutex> lk(c->mu);
    sg::DeviceGuard dg(c->device);
    if (!dg.ok) return fail(SG_E_HIP, "hipSetDevice failed%s");
    std::memcpy(c->h_in, nonce, 8);
    if (adlen) std::memcpy(c->h_in + sg::kSingleAdOff, ad, adlen);
    if (in_len) std::memcpy(c->h_in + sg::kSingleInOff, in, in_len);
    // the kernels read nonce | ad | record from the pinned block and write
    // status | output into the pinned out block over PCIe (one record is a few
    // KiB; two copy launches cost more than the transfer)
    uint8_t* src = c->h_in;
    uint8_t* dst = c->h_out;

    sg_batch b;
    std::memset(&b, 0, sizeof b);
    b.count = 1;
    b.keys = c->d_key;
    b.num_keys = 1;
    b.nonces = src;
    b.ads = src + sg::kSingleAdOff;
    b.ad_len = (uint32_t)adlen;
    b.ad_stride = (uint32_t)adlen;
    b.in = src + sg::kSingleInOff;
    b.in_stride = in_len;
    b.out = dst + sg::kSingleOutOff;
    b.out_stride = in_len + 16;
    b.uniform_len = (uint32_t)in_len;
    b.status = dst;
    b.stream = c->stream;
    b.workspace = c->d_ws;
    b.workspace_size = sg_workspace_size(1);
    // a failed open's plaintext is withheld on the host below: no device scrub
    b.flags = open ? SG_BATCH_KEEP_FAILED : 0u;
    int rc = open ? sg_open_batch(&b) : sg_seal_batch(&b);
    if (rc != SG_OK) return rc;
    const size_t out_len = open ? n : n + SG_MAC_LEN;
    SG_HIP(hipStreamSynchronize(c->stream));
    const uint8_t st = open ? c->h_out[0] : 0;
    if (open && st != 0) {
        if (n) std::memset(out, 0, n);  // the reference releases no plaintext with Err
        return st == 2 ? SG_E_SHORT : SG_E_BAD_MAC;
    }
    if (out_len) std::memcpy(out, c->h_out + sg::kSingleOutOff, out_len);
    return SG_OK;
}

int sg_seal(sg_ctx* c, const uint8_t* nonce, size_t nonce_len, const uint8_t* pt, size_t n,
            const uint8_t* ad, size_t adlen, uint8_t* out) {
    return single(c, false, nonce, nonce_len, pt, n, ad, adlen, out);
}

int sg_open(sg_ctx* c, const uint8_t* nonce, size_t nonce_len, const uint8_t* in, size_t in_len,
            const uint8_t* ad, size_t adlen, uint8_t* out) {
    return single(c, true, nonce, nonce_len, in, in_len, ad, adlen, out);
}

int sg_seal_batch(const sg_batch* b) { return run_batch(b, false); }
int sg_open_batch(const sg_batch* b) { return run_batch(b, true); }

int sg_fill_records(uint8_t* buf, uint64_t stride, uint32_t len, uint32_t count, uint64_t seed, uint64_t j0,
                    void* stream) {
    if (!buf && count) return fail(SG_E_ARG, "buf is NULL%s");
    SG_HIP(sg::launch_fill(buf, stride, len, count, seed, j0, (hipStream_t)stream));
    if (!stream) SG_HIP(hipStreamSynchronize(nullptr));
    return SG_OK;
}

int sg_compare_records(const uint8_t* a, uint64_t sa, const uint8_t* b, uint64_t sb, uint32_t len,
                       uint32_t count, unsigned long long* mism, void* stream) {
    if ((!a || !b || !mism) && count) return fail(SG_E_ARG, "NULL pointer%s");
    SG_HIP(sg::launch_compare(a, sa, b, sb, len, count, mism, (hipStream_t)stream));
    if (!stream) SG_HIP(hipStreamSynchronize(nullptr));
    return SG_OK;
}

int sg_set_lockstep(int enable) { return sg::set_wpr(enable); }
int sg_set_packed(int enable) { return sg::set_pack(enable); }

int sg_set_timing(int enable) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    for (auto& t : g_timed) {
        (void)hipEventSynchronize(t.b);
        g_event_pool.push_back(t.a);
        g_event_pool.push_back(t.b);
    }
    g_timed.clear();
    g_timing = enable != 0;
    return SG_OK;
}

int sg_timing_read(double* seal_ms, double* open_ms, double* keying_ms, uint32_t* n_seal, uint32_t* n_open,
                   uint32_t* n_keying) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    double sum[3] = {0, 0, 0};
    uint32_t cnt[3] = {0, 0, 0};
    for (auto& t : g_timed) {
        SG_HIP(hipEventSynchronize(t.b));
        float ms = 0.f;
        SG_HIP(hipEventElapsedTime(&ms, t.a, t.b));
        sum[t.kind] += ms;
        cnt[t.kind] += 1;
    }
    if (keying_ms) *keying_ms = cnt[0] ? sum[0] / cnt[0] : 0.0;
    if (seal_ms) *seal_ms = cnt[1] ? sum[1] / cnt[1] : 0.0;
    if (open_ms) *open_ms = cnt[2] ? sum[2] / cnt[2] : 0.0;
    if (n_keying) *n_keying = cnt[0];
    if (n_seal) *n_seal = cnt[1];
    if (n_open) *n_open = cnt[2];
    return SG_OK;
}

}  // extern "C"
