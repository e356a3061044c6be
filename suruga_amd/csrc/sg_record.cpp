// sg_record.cpp -- batched record layer over host memory (sg_write_records /
// sg_read_records): the throughput form of suruga's TlsWriter::write_data and
// TlsReader::read_record (src/tls.rs:99-147, 217-281).
//
// Records move through a per-context pipeline of four slots (record_slots).
// Each slot owns device buffers, a keying workspace and (staged path,
// allocated on first use) pinned host buffers.  Staged calls run the direct
// pipeline (run_direct): the host frames chunk c+1 into a slot's pinned
// staging while the kernels of chunk c read and write another slot's staging
// over the host link.  Zero-copy calls (sg_host_register'ed buffers) run the
// copy-engine pipeline (run_pipeline): while the GPU seals/opens chunk c, chunk
// c-1's output leaves and chunk c+1 comes in.  Device layout is always 16-byte
// aligned (record slot stride kSlot), so the kernels take their vector path;
// the 5-byte TLS headers are added/stripped by the CPU while copying (staged
// path) or by the frame kernels in HBM (zero-copy path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>
#include <immintrin.h>

#include "../../include/suruga_gpu.h"
#include "sg_host.h"
#include "sg_wire.h"
#include "sg_internal.h"

namespace sg {

namespace {
constexpr uint32_t kChunk = 256;                                  // records per pipeline chunk
constexpr uint32_t kSlot = ((SG_ENC_RECORD_MAX_LEN + 63u) / 64u) * 64u;  // device bytes per record
constexpr uint32_t kMetaBytes = 8u + 13u;                         // nonce + AD per record (reader)
constexpr int kMaxSlots = 8;                                      // pipeline depth (record_slots)

thread_local double t_h2d = 0, t_kernel = 0, t_d2h = 0, t_host = 0;

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

// Host threads for the framing copies (the record bytes move between the
// caller's buffers and the pinned staging at memcpy speed; one thread alone
// caps a direction near 9 GB/s).  One pool serves the whole process: it is
// created on the first call that moves more than one record and its workers
// then park on a condition variable, so N connections (two contexts each,
// cipher/mod.rs:18-23) share SG_COPY_THREADS - 1 threads instead of owning
// 7 each.  run(n, fn) calls fn(i) for every i < n on the workers and the
// calling thread and returns when all are done; concurrent callers (a
// reader and a writer thread) each queue a job and the workers take indices
// from the oldest job that still has some, so both progress.
// SG_COPY_THREADS sets the total (default 8: tools/record_path_bench.py
// measured 9.8 / 11.5 / 15.5 / 15.2 GiB/s per direction with 1 / 4 / 8 / 16
// in round 4; with round 6's direct pipeline 20.7 / 22.6 / 19.4 / 20.0 GiB/s
// write with 8 / 12 / 16 / 24, profiles/r06/record_path_ab/threads_r06.json:
// the host's memory, not the thread count, bounds it).
class CopyPool {
  public:
    static CopyPool& shared() {
        // never destroyed: parked workers must not be joined from a static
        // destructor while the runtime is tearing down
        static CopyPool* pool = new CopyPool();
        return *pool;
    }
    void run(uint32_t n, const std::function<void(uint32_t)>& fn) {
        if (n == 0) return;
        if (th_.empty() || n == 1) {
            for (uint32_t i = 0; i < n; ++i) fn(i);
            return;
        }
        Job job;
        job.fn = &fn;
        job.n = n;
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(&job);
        }
        cv_.notify_all();
        drain(job);
        std::unique_lock<std::mutex> lk(mu_);
        // no worker can pick the job up once it is off the queue; the ones that
        // did finish their last index before dropping `active`
        for (auto it = q_.begin(); it != q_.end(); ++it)
            if (*it == &job) {
                q_.erase(it);
                break;
            }
        done_.wait(lk, [&] { return job.active == 0; });
    }

  private:
    struct Job {
        const std::function<void(uint32_t)>* fn = nullptr;
        uint32_t n = 0;
        std::atomic<uint32_t> next{0};
        uint32_t active = 0;  // workers inside the job (guarded by mu_)
    };
    CopyPool() {
        const char* e = std::getenv("SG_COPY_THREADS");
        int total = e ? std::atoi(e) : 8;
        if (total < 1) total = 1;
        if (total > 32) total = 32;
        for (int i = 1; i < total; ++i) th_.emplace_back([this] { worker(); });
        for (auto& t : th_) t.detach();
    }
    static void drain(Job& j) {
        for (uint32_t i = j.next.fetch_add(1); i < j.n; i = j.next.fetch_add(1)) (*j.fn)(i);
    }
    void worker() {
        for (;;) {
            Job* j = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu_);
                for (;;) {
                    while (!q_.empty() && q_.front()->next.load() >= q_.front()->n) q_.pop_front();  // exhausted
                    if (!q_.empty()) break;
                    cv_.wait(lk);
                }
                j = q_.front();
                ++j->active;
            }
            drain(*j);
            {
                std::lock_guard<std::mutex> lk(mu_);
                --j->active;
            }
            done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::deque<Job*> q_;
};

// The framing copies of one call: inline for a single record, otherwise on
// the shared pool (created by the first call that moves more than one).
void copy_run(uint32_t n, const std::function<void(uint32_t)>& fn) {
    if (n <= 1) {
        for (uint32_t i = 0; i < n; ++i) fn(i);
        return;
    }
    CopyPool::shared().run(n, fn);
}

struct RecordStaging {
    struct Slot {
        uint8_t *h_in = nullptr, *h_out = nullptr, *h_meta = nullptr, *h_status = nullptr;
        uint32_t* h_len = nullptr;
        uint8_t *d_in = nullptr, *d_out = nullptr;
        uint8_t* d_wire = nullptr;  // the chunk's wire image (zero-copy path)
        // device addresses of the pinned blocks: the kernels read lengths,
        // nonces / AD and write statuses there over the host link, and the
        // direct pipeline's kernels read and write the record staging there
        uint8_t *dh_in = nullptr, *dh_out = nullptr, *dh_meta = nullptr, *dh_status = nullptr;
        uint32_t* dh_len = nullptr;
        void* d_ws = nullptr;
        hipStream_t st = nullptr;  // SG_COPY_STREAMS=0 only: the slot's copies and kernels
        hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // start, after H2D, after kernels, after D2H
        uint32_t nrec = 0;       // records in flight on this slot
        uint64_t first = 0;      // index of its first record in the call
        bool zc = false;         // the chunk goes the zero-copy way
        bool busy = false;
        hipStream_t kst = nullptr;  // direct pipeline: the stream of the chunk's kernels
    } slot[kMaxSlots];
    hipStream_t krn = nullptr;  // the copy-engine pipeline's kernel stream (copy-stream mode 1)
    hipStream_t kst = nullptr;  // the direct pipeline's stream
};

// Pipeline depth (SG_RECORD_SLOTS, 2..8).  Four slots (default since round 6)
// keep a chunk's H2D, another's kernels and a third's D2H in flight while the
// host-gated pipeline (run_pipeline) notices each step's end: round 5's three
// slots were enough for the device-waited form, where a chunk's whole chain was
// enqueued at once.
int record_slots() {
    static const int n = [] {
        const char* e = std::getenv("SG_RECORD_SLOTS");
        const int v = e ? std::atoi(e) : 4;
        return v < 2 ? 2 : (v > kMaxSlots ? kMaxSlots : v);
    }();
    return n;
}

// Stream layout.  Mode 1 (default): the host-link copies of every context on
// one process-wide stream per direction and each context's kernels on a stream
// of its own, so that one slot's H2D runs beside another's kernels and a
// third's D2H, the copies on different DMA engines, while a reader and a writer
// use four streams in all -- within the process's hardware queues
// (GPU_MAX_HW_QUEUES = 4: more streams than that share queues and serialise).
// Round 5, same box, 1 GiB per direction, 8 copy threads (profiles/r05g):
// registered buffers 17.4 -> 27.6 GiB/s write, 23.4 -> 25.8 read against
// per-slot streams; pageable 12.6 -> 15.2 write, 15.8 -> 14.5 read.  Round 6
// (profiles/r06/, r06d): the D2H on a stream of each context's own 14.8
// instead of 29.7 GiB/s registered read, both copy directions per context 24.2
// instead of 31.7 write -- the extra streams share hardware queues.  Mode 0
// (SG_COPY_STREAMS=0): each slot's copies and kernels on the slot's stream.
struct PipeStreams {
    hipStream_t h2d, krn, d2h;
};
int copy_streams_mode() {
    static const int m = [] {
        const char* e = std::getenv("SG_COPY_STREAMS");
        return e && e[0] == '0' ? 0 : 1;
    }();
    return m;
}
// The direct pipeline for staged calls (round 6, default; run_direct): the
// record kernels read the pinned staging and write their output into it over
// the host link themselves.  SG_RECORD_SDMA=1: the copy-engine pipeline
// (run_pipeline) for staged calls too (A/B).
bool record_direct() {
    static const bool on = [] {
        const char* e = std::getenv("SG_RECORD_SDMA");
        return !(e && e[0] == '1');
    }();
    return on;
}
// The direct pipeline's kernel stream of each context is created at the
// device's greatest stream priority: such streams draw their hardware queues
// from a pool of their own, which the process's other streams do not share,
// so a writer's and a reader's record kernels never queue behind each other or
// behind unrelated work (round 6, profiles/r06/record_path_ab/r06ps: pageable
// 22.1 / 22.2 and 20.7 / 21.6 GiB/s in the bench process against 19.8 / 20.2
// and 19.5 / 19.3, duplex standalone 28.5 / 28.2 against 25.2 / 25.0; one
// earlier default-priority run of the bench process ran the duplex at 0.91x
// the serial time, r06pr).  The same for the copy-engine pipeline's copy or
// kernel streams slowed the registered path (34.9 -> 26-27 GiB/s, r06pr), so
// those stay at the default priority.  SG_DIRECT_PRIO=0: default priority (A/B).
bool direct_stream_high() {
    static const bool on = [] {
        const char* e = std::getenv("SG_DIRECT_PRIO");
        return !(e && e[0] == '0');
    }();
    return on;
}
hipError_t make_stream(hipStream_t* s, bool high) {
    if (!high) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}
std::mutex g_cs_mu;
std::vector<std::pair<int, std::pair<hipStream_t, hipStream_t>>> g_copy_streams;  // device -> (h2d, d2h)
hipError_t process_copy_streams(int dev, hipStream_t* h2d, hipStream_t* d2h) {
    std::lock_guard<std::mutex> lk(g_cs_mu);
    for (auto& e : g_copy_streams)
        if (e.first == dev) {
            *h2d = e.second.first;
            *d2h = e.second.second;
            return hipSuccess;
        }
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(h2d, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(d2h, hipStreamNonBlocking)) != hipSuccess) return e;
    g_copy_streams.push_back({dev, {*h2d, *d2h}});
    return hipSuccess;
}

void record_staging_free(RecordStaging* rs) {
    if (!rs) return;

    for (hipStream_t t : {rs->krn, rs->kst}) {
        if (!t) continue;
        (void)hipStreamSynchronize(t);
        (void)hipStreamDestroy(t);
    }
    for (auto& s : rs->slot) {
        if (s.st) (void)hipStreamSynchronize(s.st);
        (void)hipHostFree(s.h_in);
        (void)hipHostFree(s.h_out);
        (void)hipHostFree(s.h_meta);
        (void)hipHostFree(s.h_status);
        (void)hipHostFree(s.h_len);
        (void)hipFree(s.d_in);
        (void)hipFree(s.d_out);
        (void)hipFree(s.d_wire);
        (void)hipFree(s.d_ws);
        for (auto& e : s.ev)
            if (e) (void)hipEventDestroy(e);
        if (s.st) (void)hipStreamDestroy(s.st);
    }
    delete rs;
}

namespace {

int staging(sg_ctx* c, RecordStaging** out) {
    if (!c->rec) {
        auto* rs = new RecordStaging();
        c->rec = rs;  // freed with the context even if allocation below fails
        const size_t bytes = (size_t)kChunk * kSlot;
        // Mode 1: the process's copy streams first, then the context's kernel
        // stream, and no stream that the pipeline does not use: HIP hands a
        // process's streams its hardware queues round-robin (GPU_MAX_HW_QUEUES =
        // 4), and a kernel stream that shares a queue with the D2H stream runs
        // its kernels behind the copies (round 6: the standalone write at 22.3
        // GiB/s registered with the kernels on a context stream created before
        // the copy streams, r06l, against 35.1 in a process whose other
        // streams happened to separate them)
        // (the streams are created by pipe_streams on a call's first use of them)
        for (int i = 0; i < record_slots(); ++i) {  // (h_in / h_out: host_staging, on first use)
            auto& s = rs->slot[i];
            SG_HIP(hipHostMalloc((void**)&s.h_meta, (size_t)kChunk * kMetaBytes, hipHostMallocMapped));
            SG_HIP(hipHostMalloc((void**)&s.h_status, kChunk, hipHostMallocMapped));
            SG_HIP(hipHostMalloc((void**)&s.h_len, kChunk * 4u, hipHostMallocMapped));
            SG_HIP(hipHostGetDevicePointer((void**)&s.dh_meta, s.h_meta, 0));
            SG_HIP(hipHostGetDevicePointer((void**)&s.dh_status, s.h_status, 0));
            SG_HIP(hipHostGetDevicePointer((void**)&s.dh_len, s.h_len, 0));
            SG_HIP(hipMalloc((void**)&s.d_in, bytes));
            SG_HIP(hipMalloc((void**)&s.d_out, bytes));
            SG_HIP(hipMalloc((void**)&s.d_wire, bytes + 64));
            SG_HIP(hipMalloc(&s.d_ws, sg_workspace_size(kChunk)));
            for (auto& e : s.ev) SG_HIP(hipEventCreate(&e));
        }
    }
    *out = c->rec;
    return SG_OK;
}

// The staged path's pinned blocks of a slot (the zero-copy path never needs
// them, so a context that only moves registered buffers pins no staging).
int host_staging(RecordStaging::Slot& s) {
    const size_t bytes = (size_t)kChunk * kSlot;
    if (!s.h_in) {
        SG_HIP(hipHostMalloc((void**)&s.h_in, bytes, hipHostMallocMapped));
        SG_HIP(hipHostGetDevicePointer((void**)&s.dh_in, s.h_in, 0));
    }
    if (!s.h_out) {
        SG_HIP(hipHostMalloc((void**)&s.h_out, bytes, hipHostMallocMapped));
        SG_HIP(hipHostGetDevicePointer((void**)&s.dh_out, s.h_out, 0));
    }
    return SG_OK;
}

// Account a finished slot's device times (H2D, kernels, D2H).
int account(RecordStaging::Slot& s) {
    float a = 0, b = 0, d = 0;
    SG_HIP(hipEventElapsedTime(&a, s.ev[0], s.ev[1]));
    SG_HIP(hipEventElapsedTime(&b, s.ev[1], s.ev[2]));
    SG_HIP(hipEventElapsedTime(&d, s.ev[2], s.ev[3]));
    t_h2d += a;
    t_kernel += b;
    t_d2h += d;
    return SG_OK;
}

// Leaves every pipeline slot idle on every exit path: a call that returns
// early (a launch or copy error) must not hand a half-finished slot, framed
// with its own lengths and sequence numbers, to the next call.
struct SlotReset {
    RecordStaging* rs;
    PipeStreams ps[kMaxSlots];
    explicit SlotReset(RecordStaging* r) : rs(r) {
        for (auto& p : ps) p = {nullptr, nullptr, nullptr};
        reset();
    }
    ~SlotReset() { reset(); }
    void reset() {
        for (int i = 0; i < kMaxSlots; ++i) {
            auto& s = rs->slot[i];
            if (s.busy)
                for (hipStream_t t : {ps[i].h2d, ps[i].krn, ps[i].d2h})
                    if (t) (void)hipStreamSynchronize(t);
            s.busy = false;
            s.nrec = 0;
            s.first = 0;
            s.zc = false;
        }
    }
};

// the streams of slot i for this call (mode: copy_streams_mode)
int pipe_streams(sg_ctx* c, RecordStaging* rs, int i, bool direct, PipeStreams* out) {
    if (direct) {
        if (!rs->kst) SG_HIP(make_stream(&rs->kst, direct_stream_high()));
        *out = {rs->kst, rs->kst, rs->kst};
        return SG_OK;
    }
    if (copy_streams_mode() == 0) {
        if (!rs->slot[i].st) SG_HIP(hipStreamCreateWithFlags(&rs->slot[i].st, hipStreamNonBlocking));
        *out = {rs->slot[i].st, rs->slot[i].st, rs->slot[i].st};
        return SG_OK;
    }
    // the process's copy streams first, then the context's kernel stream: HIP
    // hands a process's streams its hardware queues round-robin
    hipStream_t h = nullptr, d = nullptr;
    SG_HIP(process_copy_streams(c->device, &h, &d));
    if (!rs->krn) SG_HIP(hipStreamCreateWithFlags(&rs->krn, hipStreamNonBlocking));
    *out = {h, rs->krn, d};
    return SG_OK;
}

// The pipeline of sg_write_records / sg_read_records.  Chunk k uses slot
// k % ns and passes four steps:
//   stage    host framing copy (staged path) and the H2D, when the slot is free;
//   launch   the kernels, once the chunk's H2D has completed;
//   copy_out the D2H, once the chunk's kernels have completed;
//   finish   host framing (oldest chunk first), once the chunk's D2H has completed.
// Each step is enqueued by the calling thread when the step before it has
// completed on the device (hipEventQuery, polled every few microseconds), so
// no stream ever holds a device-side wait.  That matters once two contexts run
// at once (suruga's reader and writer, client.rs:19-24, 269-271): a copy
// enqueued ahead of its input waits inside the DMA engine's queue and holds up
// every later copy of the process on that engine and, when the process has more
// streams than hardware queues (GPU_MAX_HW_QUEUES = 4), every command of the
// streams that share its queue.  Round 5's form enqueued a chunk's whole chain
// at once with hipStreamWaitEvent between the streams: one direction at a time
// it is as fast (33.7 / 31.5 GiB/s registered, in the bench process), but a
// reader and a writer at once ran at 19.9 GiB/s together, 0.61x one after the
// other; host-gated they run at 36.4, 1.1-1.4x (profiles/r06/record_path_ab/).
// Polling back to back slowed the copies (20.6 instead of 33.5 GiB/s
// registered write, profiles/r06/record_path_hostdriven.json), so the host
// waits ~5 us between polls.
// SG_RECORD_DEVICE_WAITS=1 gives the round-5 form (A/B).  more(): whether
// another chunk is to be staged (the reader stops at a failed record).
// The direct pipeline (round 6; the staged path, record_direct): the record
// kernels read the pinned staging and write their output into it over the
// host link themselves, so no copy engine is involved and a chunk's work is
// the kernels of one stream.  The host keeps up to ns chunks in flight, fills
// the next slot's staging while the GPU works, and waits only for the oldest
// chunk before reusing its slot.  On this host link kernels move data faster
// than the copy engines (tools/hostbw_probe.hip, profiles/r06/hostbw_r06t.txt:
// kernel stores to host memory 54.8 GB/s, loads 57.3 GB/s, against 30.2 / 40.6
// GB/s for SDMA D2H / H2D, and 28.6 GB/s each with a copy in each direction at
// once).  Zero-copy calls keep the copy-engine pipeline: there the seal kernel
// reading the caller's buffer and the frame kernel writing the wire reached
// 20-23 GiB/s against 34.6 / 24.1 GiB/s write / read for SDMA copies
// (profiles/r06/record_path_ab/, r06u-r06v).
template <class More, class Stage, class Launch, class Finish>
int run_direct(RecordStaging* rs, int ns, More more, Stage stage, Launch launch, Finish finish) {
    uint64_t staged = 0, done = 0;
    auto slot = [&](uint64_t k) -> RecordStaging::Slot& { return rs->slot[k % (uint64_t)ns]; };
    int rc;
    for (;;) {
        if (staged < done + (uint64_t)ns && more()) {
            RecordStaging::Slot& s = slot(staged);
            s.busy = true;  // (before the enqueues: SlotReset then drains the streams on an error)
            s.kst = rs->kst;
            if ((rc = stage(s)) != SG_OK) return rc;
            SG_HIP(hipEventRecord(s.ev[0], s.kst));
            if ((rc = launch(s)) != SG_OK) return rc;
            SG_HIP(hipEventRecord(s.ev[3], s.kst));
            ++staged;
            continue;
        }
        if (done == staged) return SG_OK;
        RecordStaging::Slot& s = slot(done);
        SG_HIP(hipEventSynchronize(s.ev[3]));
        float ms = 0;
        SG_HIP(hipEventElapsedTime(&ms, s.ev[0], s.ev[3]));
        t_kernel += ms;  // (the chunks on the two streams overlap: device time, not wall time)
        if ((rc = finish(s)) != SG_OK) return rc;
        s.busy = false;
        ++done;
    }
}

bool record_device_waits() {
    static const bool on = [] {
        const char* e = std::getenv("SG_RECORD_DEVICE_WAITS");
        return e && e[0] == '1';
    }();
    return on;
}
template <class Streams, class More, class Stage, class Launch, class CopyOut, class Finish>
int run_pipeline(RecordStaging* rs, int ns, Streams streams, More more, Stage stage, Launch launch, CopyOut copy_out,
                 Finish finish) {
    uint64_t staged = 0, launched = 0, copied = 0, done = 0;
    auto slot = [&](uint64_t k) -> RecordStaging::Slot& { return rs->slot[k % (uint64_t)ns]; };
    auto finish_oldest = [&](RecordStaging::Slot& s) -> int {
        int r;
        if ((r = account(s)) != SG_OK) return r;
        if ((r = finish(s)) != SG_OK) return r;
        s.busy = false;
        ++done;
        return SG_OK;
    };
    int rc;
    if (record_device_waits()) {  // round 5: the chain enqueued at once, ordered on the device
        for (;;) {
            if (staged < done + (uint64_t)ns && more()) {
                RecordStaging::Slot& s = slot(staged);
                const PipeStreams& P = streams(s);
                s.busy = true;  // (before the enqueues: SlotReset then drains its streams on an error)
                if ((rc = stage(s)) != SG_OK) return rc;
                if (P.krn != P.h2d) SG_HIP(hipStreamWaitEvent(P.krn, s.ev[1], 0));
                if ((rc = launch(s)) != SG_OK) return rc;
                if (P.d2h != P.krn) SG_HIP(hipStreamWaitEvent(P.d2h, s.ev[2], 0));
                if ((rc = copy_out(s)) != SG_OK) return rc;
                ++staged;
                continue;
            }
            if (done == staged) return SG_OK;
            SG_HIP(hipEventSynchronize(slot(done).ev[3]));
            if ((rc = finish_oldest(slot(done))) != SG_OK) return rc;
        }
    }
    // 1: the step's event has completed, 0: not yet, < 0: error
    auto ready = [&](RecordStaging::Slot& s, int ev) -> int {
        const hipError_t q = hipEventQuery(s.ev[ev]);
        if (q == hipSuccess) return 1;
        if (q == hipErrorNotReady) return 0;
        return hip_fail(q, "hipEventQuery");
    };
    for (;;) {
        bool progress = false;
        if (copied > done) {
            if ((rc = ready(slot(done), 3)) < 0) return rc;
            if (rc) {
                if ((rc = finish_oldest(slot(done))) != SG_OK) return rc;
                progress = true;
            }
        }
        if (launched > copied) {
            if ((rc = ready(slot(copied), 2)) < 0) return rc;
            if (rc) {
                if ((rc = copy_out(slot(copied))) != SG_OK) return rc;
                ++copied;
                progress = true;
            }
        }
        if (staged > launched) {
            if ((rc = ready(slot(launched), 1)) < 0) return rc;
            if (rc) {
                if ((rc = launch(slot(launched))) != SG_OK) return rc;
                ++launched;
                progress = true;
            }
        }
        if (staged < done + (uint64_t)ns && more()) {
            RecordStaging::Slot& s = slot(staged);
            s.busy = true;
            if ((rc = stage(s)) != SG_OK) return rc;
            ++staged;
            progress = true;
        }
        if (done == staged && !more()) return SG_OK;
        if (!progress) {
            // ~5 us between polls: polling back to back slowed the copies
            // (20.6 instead of 33.5 GiB/s registered write, r06a), and a
            // sleep rounds up to the kernel's timer slack (~50 us)
            const auto t0 = std::chrono::steady_clock::now();
            while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(5)) _mm_pause();
        }
    }
}

inline void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
inline void put_be64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (56 - 8 * i));
}

// Caller buffers registered with sg_host_register (page-locked, device-visible
// host memory).  When a call's source and destination both lie in registered
// ranges, the record bytes move by DMA straight between them and the device
// (no framing copy through the library's pinned staging): sg_write_records
// copies the plaintext in with one contiguous H2D per chunk, builds the
// chunk's wire image (headers and fragments) in HBM and copies it out with one
// contiguous D2H; sg_read_records copies the chunk's wire image in, takes it
// apart in HBM and copies the plaintext out contiguously.
struct RegRange {
    uintptr_t lo, hi, dev;  // [lo, hi) on the host; dev: its device address (hipHostGetDevicePointer)
};
std::mutex g_reg_mu;
std::vector<RegRange> g_reg;
bool registered(const void* p, size_t n) {
    if (!p || !n) return false;
    const uintptr_t lo = (uintptr_t)p, hi = lo + n;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (const auto& r : g_reg)
        if (lo >= r.lo && hi <= r.hi) return true;
    return false;
}
// the device address of a byte of a registered range (nullptr if none)
template <class T>
T* reg_dev(T* p) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (const auto& r : g_reg)
        if (a >= r.lo && a < r.hi) return (T*)(r.dev + (a - r.lo));
    return nullptr;
}

// SG_RECORD_KD2H=1: zero-copy calls move their output by a kernel's stores
// into the caller's registered memory over the host link (the write's frame
// kernel builds the wire image straight in `wire`, the read's copy-out kernel
// moves the plaintext into `out`), after the record kernels on the same
// stream, instead of an SDMA D2H.  Round 6, same box (profiles/r06/
// record_path_ab/, r06zz-r06zy): 28.1 / 25.5 GiB/s write / read both in a
// standalone process and in the bench process, against SDMA's 21.6 / 21.0
// standalone and 35.1 / 33.9 in the bench process (the SDMA copies' rate
// depends on how the process's streams fall on the hardware queues; the
// kernel's stores serialise with the record kernels of its stream).  The same
// kernel on the D2H stream measured 21.7 / 21.4 and 25.9 / 23.9.  Default: SDMA.
bool record_kd2h() {
    static const bool on = [] {
        const char* e = std::getenv("SG_RECORD_KD2H");
        return e && e[0] == '1';
    }();
    return on;
}

// SG_ZERO_COPY=0 in the environment turns the registered-buffer path off (A/B)
bool zero_copy_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("SG_ZERO_COPY");
        return !(e && e[0] == '0');
    }();
    return on;
}

}  // namespace
}  // namespace sg

using sg::fail;

extern "C" {

size_t sg_wire_bound(size_t len) {
    const size_t recs = (len + SG_RECORD_MAX_LEN - 1) / SG_RECORD_MAX_LEN;
    return len + recs * (SG_HEADER_LEN + SG_MAC_LEN);
}

int sg_host_register(void* p, size_t len) {
    if (!p || !len) return fail(SG_E_ARG, "NULL or empty range%s");
    // mapped: the zero-copy path's output kernels write the range over the
    // host link (record_kd2h)
    hipError_t e = hipHostRegister(p, len, hipHostRegisterPortable | hipHostRegisterMapped);
    if (e != hipSuccess) return sg::hip_fail(e, "hipHostRegister");
    void* dev = nullptr;
    if ((e = hipHostGetDevicePointer(&dev, p, 0)) != hipSuccess) {
        (void)hipHostUnregister(p);
        return sg::hip_fail(e, "hipHostGetDevicePointer");
    }
    std::lock_guard<std::mutex> lk(sg::g_reg_mu);
    sg::g_reg.push_back({(uintptr_t)p, (uintptr_t)p + len, (uintptr_t)dev});
    return SG_OK;
}

int sg_host_unregister(void* p) {
    {
        std::lock_guard<std::mutex> lk(sg::g_reg_mu);
        auto it = std::find_if(sg::g_reg.begin(), sg::g_reg.end(),
                               [&](const sg::RegRange& r) { return r.lo == (uintptr_t)p; });
        if (it == sg::g_reg.end()) return fail(SG_E_ARG, "range was not registered with sg_host_register%s");
        sg::g_reg.erase(it);
    }
    const hipError_t e = hipHostUnregister(p);
    return e == hipSuccess ? SG_OK : sg::hip_fail(e, "hipHostUnregister");
}

int sg_record_timing(double* h2d_ms, double* kernel_ms, double* d2h_ms, double* host_ms) {
    if (h2d_ms) *h2d_ms = sg::t_h2d;
    if (kernel_ms) *kernel_ms = sg::t_kernel;
    if (d2h_ms) *d2h_ms = sg::t_d2h;
    if (host_ms) *host_ms = sg::t_host;
    return SG_OK;
}

int64_t sg_write_records(sg_ctx* c, uint64_t seq0, uint8_t content_type, uint8_t ver_major, uint8_t ver_minor,
                         const uint8_t* data, size_t len, uint8_t* wire, size_t wire_cap, size_t* wire_len) {
    using namespace sg;
    if (!c || (!data && len) || !wire_len) return fail(SG_E_ARG, "NULL argument%s");
    *wire_len = 0;
    t_h2d = t_kernel = t_d2h = t_host = 0;
    const uint64_t nrec = (len + SG_RECORD_MAX_LEN - 1) / SG_RECORD_MAX_LEN;
    if (nrec == 0) return 0;
    if (!wire || wire_cap < sg_wire_bound(len)) return fail(SG_E_ARG, "wire buffer too small%s");
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return fail(SG_E_HIP, "hipSetDevice failed%s");
    RecordStaging* rs = nullptr;
    int rc = staging(c, &rs);
    if (rc != SG_OK) return rc;
    size_t wpos = 0;
    // every record but the last is full, so record r starts at r * kWireRec
    constexpr size_t kWireRec = SG_HEADER_LEN + SG_RECORD_MAX_LEN + SG_MAC_LEN;
    const size_t wire_need = (size_t)(nrec - 1) * kWireRec + SG_HEADER_LEN +
                             (size_t)(len - (nrec - 1) * SG_RECORD_MAX_LEN) + SG_MAC_LEN;
    // registered caller buffers: DMA straight between them and the device
    // (the copy-engine pipeline); otherwise the pinned staging, which the
    // kernels read and write over the host link (the direct pipeline)
    const bool zc = zero_copy_enabled() && registered(data, len) && registered(wire, wire_need);
    const bool direct = record_direct() && !zc;
    // zero-copy: the frame kernel writes the wire image into `wire` itself
    // (its word stores need a 4-byte aligned wire)
    const bool kd2h = zc && ((uintptr_t)wire & 3u) == 0 && record_kd2h();
    auto rec_len = [&](uint64_t r) { return (uint32_t)std::min<uint64_t>(SG_RECORD_MAX_LEN, len - r * SG_RECORD_MAX_LEN); };
    uint64_t next = 0;  // first record of the next chunk to stage
    SlotReset slot_reset(rs);
    const int ns = record_slots();
    for (int i = 0; i < ns; ++i)
        if ((rc = pipe_streams(c, rs, i, direct, &slot_reset.ps[i])) != SG_OK) return rc;
    auto streams = [&](const RecordStaging::Slot& s) -> const PipeStreams& { return slot_reset.ps[&s - rs->slot]; };

    // host framing copy in, H2D (tls.rs:137-147: 2^14-byte fragments)
    auto stage = [&](RecordStaging::Slot& s) -> int {
        const uint32_t k = (uint32_t)std::min<uint64_t>(kChunk, nrec - next);
        const double t0 = now_ms();
        // zero-copy: the chunk's plaintext is contiguous in the caller's buffer
        // (in_stride 2^14); staged: each record in its 16-byte aligned slot
        s.zc = zc;
        if (s.zc) {
            for (uint32_t i = 0; i < k; ++i) s.h_len[i] = rec_len(next + i);
        } else {
            int r;
            if ((r = host_staging(s)) != SG_OK) return r;
            const uint64_t first = next;
            copy_run(k, [&](uint32_t i) {
                const uint64_t rr = first + i;
                std::memcpy(s.h_in + (size_t)i * kSlot, data + rr * SG_RECORD_MAX_LEN, rec_len(rr));
                s.h_len[i] = rec_len(rr);
            });
        }
        t_host += now_ms() - t0;
        s.nrec = k;
        s.first = next;
        next += k;
        if (direct) return SG_OK;  // (the kernels read the input themselves)
        bool same = true;  // every record of the chunk has the same length
        for (uint32_t i = 1; i < k; ++i) same = same && s.h_len[i] == s.h_len[0];
        const hipStream_t hs = streams(s).h2d;
        SG_HIP(hipEventRecord(s.ev[0], hs));
        if (s.zc) {
            const size_t bytes = (size_t)(k - 1) * SG_RECORD_MAX_LEN + s.h_len[k - 1];
            SG_HIP(hipMemcpyAsync(s.d_in, data + s.first * SG_RECORD_MAX_LEN, bytes, hipMemcpyHostToDevice, hs));
        } else {
            SG_HIP(hipMemcpyAsync(s.d_in, s.h_in, (size_t)k * kSlot, hipMemcpyHostToDevice, hs));
        }
        SG_HIP(hipEventRecord(s.ev[1], hs));
        return SG_OK;
    };
    // seal (and, zero-copy, the chunk's wire image: headers and fragments,
    // tls.rs:126-130, built in HBM so that it leaves in one contiguous copy --
    // a strided copy at the wire's pitch was ~50x slower on the host link)
    auto launch = [&](RecordStaging::Slot& s) -> int {
        const uint32_t k = s.nrec;
        bool same = true;
        for (uint32_t i = 1; i < k; ++i) same = same && s.h_len[i] == s.h_len[0];
        const hipStream_t ks = direct ? s.kst : streams(s).krn;
        sg_batch b;
        std::memset(&b, 0, sizeof b);
        b.count = k;
        b.flags = SG_BATCH_TLS;
        b.keys = c->d_key;
        b.num_keys = 1;
        b.seq0 = seq0 + s.first;
        b.content_type = content_type;
        b.ver_major = ver_major;
        b.ver_minor = ver_minor;
        // direct: straight from and into the pinned staging
        b.in = direct ? s.dh_in : s.d_in;
        b.in_stride = s.zc ? SG_RECORD_MAX_LEN : kSlot;
        b.out = direct ? s.dh_out : s.d_out;
        b.out_stride = kSlot;
        // a uniform chunk is a direct launch; a ragged one (the tail) is bucketed
        // the lengths of a ragged chunk are read from the pinned block over the
        // host link (a few hundred bytes: no copy of their own)
        b.len = same ? nullptr : s.dh_len;
        b.uniform_len = same ? s.h_len[0] : 0u;
        b.max_len = SG_RECORD_MAX_LEN;
        b.stream = ks;
        b.workspace = s.d_ws;
        b.workspace_size = sg_workspace_size(kChunk);
        int r;
        if ((r = sg_seal_batch(&b)) != SG_OK) return r;
        if (s.zc) {
            const uint32_t hdr = content_type | ((uint32_t)ver_major << 8) | ((uint32_t)ver_minor << 16);
            uint8_t* img = kd2h ? reg_dev(wire + s.first * kWireRec) : s.d_wire;
            SG_HIP(launch_frame(s.d_out, kSlot, img, (uint32_t)kWireRec, k, SG_RECORD_MAX_LEN + SG_MAC_LEN,
                                s.h_len[k - 1] + SG_MAC_LEN, hdr, ks));
        }
        SG_HIP(hipEventRecord(s.ev[2], ks));
        return SG_OK;
    };
    auto copy_out = [&](RecordStaging::Slot& s) -> int {
        const uint32_t k = s.nrec, last = s.h_len[k - 1] + SG_MAC_LEN;
        if (kd2h) {  // the frame kernel has written the wire already
            SG_HIP(hipEventRecord(s.ev[3], streams(s).krn));
            return SG_OK;
        }
        const hipStream_t ds = streams(s).d2h;
        if (s.zc) {
            SG_HIP(hipMemcpyAsync(wire + s.first * kWireRec, s.d_wire, (size_t)(k - 1) * kWireRec + SG_HEADER_LEN + last,
                                  hipMemcpyDeviceToHost, ds));
        } else {
            SG_HIP(hipMemcpyAsync(s.h_out, s.d_out, (size_t)k * kSlot, hipMemcpyDeviceToHost, ds));
        }
        SG_HIP(hipEventRecord(s.ev[3], ds));
        return SG_OK;
    };
    // frame the chunk's records into the wire (tls.rs:126-130): the headers and
    // (staged path) the fragments from the pinned staging
    auto finish = [&](RecordStaging::Slot& s) -> int {
        const double t0 = now_ms();
        if (!s.zc) {
            copy_run(s.nrec, [&](uint32_t i) {
                const uint64_t r = s.first + i;
                uint8_t* h = wire + r * kWireRec;
                h[0] = content_type;
                h[1] = ver_major;
                h[2] = ver_minor;
                put_be16(h + 3, rec_len(r) + SG_MAC_LEN);
                std::memcpy(h + SG_HEADER_LEN, s.h_out + (size_t)i * kSlot, rec_len(r) + SG_MAC_LEN);
            });
        }
        const uint64_t last = s.first + s.nrec - 1;
        wpos = last * kWireRec + SG_HEADER_LEN + (size_t)rec_len(last) + SG_MAC_LEN;
        t_host += now_ms() - t0;
        return SG_OK;
    };
    if (direct) rc = run_direct(rs, ns, [&] { return next < nrec; }, stage, launch, finish);
    else rc = run_pipeline(rs, ns, streams, [&] { return next < nrec; }, stage, launch, copy_out, finish);
    if (rc != SG_OK) return rc;
    *wire_len = wpos;
    return (int64_t)nrec;
}

int sg_read_records(sg_ctx* c, uint64_t seq0, const uint8_t* wire, size_t wire_len, uint8_t* out, size_t out_cap,
                    uint8_t* types, uint32_t* frag_lens, size_t max_records, sg_read_result* res) {
    using namespace sg;
    if (!c || (!wire && wire_len) || !res) return fail(SG_E_ARG, "NULL argument%s");
    std::memset(res, 0, sizeof *res);
    t_h2d = t_kernel = t_d2h = t_host = 0;

    // 1. parse complete records (tls.rs:218-238), stopping at the first bad header
    // (sg_wire.cpp: host-only, run under ASan/UBSan by tests/test_sanitizers.py)
    using Rec = WireRec;
    std::vector<Rec> recs;
    const int32_t header_error = parse_wire(wire, wire_len, max_records, recs);
    size_t need = 0;
    for (const Rec& r : recs) need += r.flen - SG_MAC_LEN;
    if (need > out_cap || (need && !out)) return fail(SG_E_ARG, "out buffer too small%s");
    if (recs.empty()) {
        res->error = header_error;
        return SG_OK;
    }

    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return fail(SG_E_HIP, "hipSetDevice failed%s");
    RecordStaging* rs = nullptr;
    int rc = staging(c, &rs);
    if (rc != SG_OK) return rc;

    const uint64_t nrec = recs.size();
    uint64_t next = 0, good = 0, opos = 0, consumed = 0;
    int32_t error = SG_OK;
    // registered caller buffers: the fragments come in by DMA from the wire and
    // the plaintext leaves by DMA into `out` at its final offset (prefix sum of
    // the plaintext lengths, as if every record opens)
    const bool zc = zero_copy_enabled() && registered(wire, wire_len) && registered(out, need);
    const bool direct = record_direct() && !zc;
    const bool kd2h = zc && record_kd2h();  // zero-copy chunks: a copy-out kernel writes `out`
    std::vector<uint64_t> pre;  // zc: plaintext offset of every record
    if (zc) {
        pre.resize(nrec + 1);
        pre[0] = 0;
        for (uint64_t i = 0; i < nrec; ++i) pre[i + 1] = pre[i] + recs[i].flen - SG_MAC_LEN;
    }
    // Zero-copy: plaintext DMA'd into `out` beyond the delivered records is
    // cleared on every exit (the reference releases none of it, tls.rs:268):
    // collect() clears it chunk by chunk, and an early return (a launch or copy
    // error) clears everything from the first undelivered record to the end of
    // the chunks issued.  Declared before the SlotReset, so that it runs after
    // the pipeline's streams have drained.
    struct ScrubOut {
        uint8_t* out;
        const std::vector<uint64_t>* pre;
        const uint64_t *good, *next;
        bool armed;
        ~ScrubOut() {
            if (armed && *next > *good) std::memset(out + (*pre)[*good], 0, (*pre)[*next] - (*pre)[*good]);
        }
    } scrub{out, &pre, &good, &next, zc};
    SlotReset slot_reset(rs);
    const int ns = record_slots();
    for (int i = 0; i < ns; ++i)
        if ((rc = pipe_streams(c, rs, i, direct, &slot_reset.ps[i])) != SG_OK) return rc;
    auto streams = [&](const RecordStaging::Slot& s) -> const PipeStreams& { return slot_reset.ps[&s - rs->slot]; };

    std::vector<uint64_t> dst_off(kChunk);
    auto collect = [&](RecordStaging::Slot& s) -> int {
        const double t0 = now_ms();
        if (error != SG_OK) {  // stopped earlier: nothing of this chunk is delivered
            if (s.zc) std::memset(out + pre[s.first], 0, pre[s.first + s.nrec] - pre[s.first]);
            return SG_OK;
        }
        // the records up to the first failing one are delivered (tls.rs:268: the
        // reader stops at its first Err); their output offsets are a prefix sum
        uint32_t ok = 0;
        for (; ok < s.nrec; ++ok) {
            if (s.h_status[ok] != 0) {  // BadRecordMac "wrong mac": deliver nothing of it
                error = s.h_status[ok] == 2 ? SG_E_SHORT : SG_E_BAD_MAC;
                break;
            }
            const Rec& R = recs[s.first + ok];
            dst_off[ok] = opos;
            opos += R.flen - SG_MAC_LEN;
            consumed += SG_HEADER_LEN + R.flen;
        }
        if (s.zc) {
            // the plaintext is in place already; from a failed record on, the
            // DMA'd bytes are cleared (the reference releases none of them)
            if (ok < s.nrec) std::memset(out + pre[s.first + ok], 0, pre[s.first + s.nrec] - pre[s.first + ok]);
            for (uint32_t i = 0; i < ok; ++i) {
                const uint64_t r = s.first + i;
                if (types) types[r] = recs[r].type;
                if (frag_lens) frag_lens[r] = recs[r].flen - SG_MAC_LEN;
            }
        } else {
            copy_run(ok, [&](uint32_t i) {
                const uint64_t r = s.first + i;
                const Rec& R = recs[r];
                const uint32_t n = R.flen - SG_MAC_LEN;
                std::memcpy(out + dst_off[i], s.h_out + (size_t)i * kSlot, n);
                if (types) types[r] = R.type;
                if (frag_lens) frag_lens[r] = n;
            });
        }
        good += ok;
        t_host += now_ms() - t0;
        return SG_OK;
    };

    // host framing copy in (staged) and the H2D of the fragments or wire image
    auto stage = [&](RecordStaging::Slot& s) -> int {
        const uint32_t k = (uint32_t)std::min<uint64_t>(kChunk, nrec - next);
        const double t0 = now_ms();
        const Rec& R0 = recs[next];
        bool same = true, tls = true, dense = true;
        for (uint32_t i = 0; i < k; ++i) {
            const Rec& R = recs[next + i];
            same = same && R.flen == R0.flen;
            tls = tls && R.type == R0.type && R.major == R0.major && R.minor == R0.minor;
            dense = dense && R.off == R0.off + (size_t)i * (SG_HEADER_LEN + R0.flen);
        }
        // zero-copy for chunks of equal, back-to-back records (a stream of
        // full records); any other chunk goes through the staging
        s.zc = zc && same && dense;
        if (!s.zc) {
            int r;
            if ((r = host_staging(s)) != SG_OK) return r;
            const uint64_t first = next;
            copy_run(k, [&](uint32_t i) {
                const Rec& R = recs[first + i];
                std::memcpy(s.h_in + (size_t)i * kSlot, wire + R.off, R.flen);
                s.h_len[i] = R.flen;
            });
        }
        // TLS mode (nonce and AD built on the device, tls.rs:250-265) when the
        // chunk's records share type and version; else explicit nonce / AD
        if (!tls) {
            for (uint32_t i = 0; i < k; ++i) {
                const Rec& R = recs[next + i];
                const uint64_t seq = seq0 + next + i;
                // nonce = be64(seq) (tls.rs:250); AD = seq || type || major || minor ||
                // be16(len - 16) (tls.rs:252-265).  Layout: nonces[kChunk][8], ads[kChunk][13]
                put_be64(s.h_meta + 8u * i, seq);
                uint8_t* m = s.h_meta + 8u * kChunk + 13u * i;
                put_be64(m, seq);
                m[8] = R.type;
                m[9] = R.major;
                m[10] = R.minor;
                put_be16(m + 11, R.flen - SG_MAC_LEN);
            }
        }
        t_host += now_ms() - t0;
        if (direct) {  // (the kernels read the staging themselves)
            s.nrec = k;
            s.first = next;
            next += k;
            return SG_OK;
        }
        const hipStream_t hs = streams(s).h2d;
        SG_HIP(hipEventRecord(s.ev[0], hs));
        if (s.zc) {  // the chunk's wire image in one contiguous copy, taken apart in HBM
            SG_HIP(hipMemcpyAsync(s.d_wire, wire + R0.off - SG_HEADER_LEN, (size_t)k * (SG_HEADER_LEN + R0.flen),
                                  hipMemcpyHostToDevice, hs));
        } else {
            SG_HIP(hipMemcpyAsync(s.d_in, s.h_in, (size_t)k * kSlot, hipMemcpyHostToDevice, hs));
        }
        SG_HIP(hipEventRecord(s.ev[1], hs));
        s.nrec = k;
        s.first = next;
        next += k;
        return SG_OK;
    };
    auto launch = [&](RecordStaging::Slot& s) -> int {
        const uint32_t k = s.nrec;
        const Rec& R0 = recs[s.first];
        bool same = true, tls = true;
        for (uint32_t i = 0; i < k; ++i) {
            const Rec& R = recs[s.first + i];
            same = same && R.flen == R0.flen;
            tls = tls && R.type == R0.type && R.major == R0.major && R.minor == R0.minor;
        }
        const hipStream_t ks = direct ? s.kst : streams(s).krn;
        if (s.zc) SG_HIP(launch_unframe(s.d_wire, SG_HEADER_LEN + R0.flen, s.d_in, kSlot, k, R0.flen, ks));
        sg_batch b;
        std::memset(&b, 0, sizeof b);
        b.count = k;
        b.keys = c->d_key;
        b.num_keys = 1;
        if (tls) {
            b.flags = SG_BATCH_TLS;
            b.seq0 = seq0 + s.first;
            b.content_type = R0.type;
            b.ver_major = R0.major;
            b.ver_minor = R0.minor;
        } else {
            uint8_t* meta = s.dh_meta;  // (read over the host link, no copy of its own)
            b.nonces = meta;
            b.ads = meta + 8u * kChunk;
            b.ad_len = 13;
            b.ad_stride = 13;
        }
        // direct: straight from and into the pinned staging
        b.in = direct ? s.dh_in : s.d_in;
        b.in_stride = kSlot;
        b.out = direct ? s.dh_out : s.d_out;
        // zero-copy: plaintext back to back, as it lands in `out`
        b.out_stride = s.zc ? (size_t)(R0.flen - SG_MAC_LEN) : kSlot;
        // lengths, nonces / AD and the per-record status go over the host link
        // in the kernels' own accesses, not in copies of their own (round 6:
        // one small D2H per chunk fewer on the copy engine)
        b.len = same ? nullptr : s.dh_len;
        b.uniform_len = same ? R0.flen : 0u;
        b.max_len = SG_ENC_RECORD_MAX_LEN;
        b.status = s.dh_status;
        b.stream = ks;
        b.workspace = s.d_ws;
        b.workspace_size = sg_workspace_size(kChunk);
        // staged: the reader delivers nothing from a failed record (it stops
        // there), so no device scrub of failed records' output; zero-copy: the
        // output goes to the caller's memory by DMA, so failed records are
        // scrubbed on the device first
        if (!s.zc) b.flags |= SG_BATCH_KEEP_FAILED;
        int r;
        if ((r = sg_open_batch(&b)) != SG_OK) return r;
        if (s.zc && kd2h)
            SG_HIP(launch_copy_out(s.d_out, reg_dev(out + pre[s.first]), pre[s.first + k] - pre[s.first], ks));
        SG_HIP(hipEventRecord(s.ev[2], ks));
        return SG_OK;
    };
    auto copy_out = [&](RecordStaging::Slot& s) -> int {
        const uint32_t k = s.nrec;
        if (s.zc && kd2h) {  // the copy-out kernel has written `out` already
            SG_HIP(hipEventRecord(s.ev[3], streams(s).krn));
            return SG_OK;
        }
        const hipStream_t ds = streams(s).d2h;
        if (s.zc) {
            SG_HIP(hipMemcpyAsync(out + pre[s.first], s.d_out, pre[s.first + k] - pre[s.first], hipMemcpyDeviceToHost,
                                  ds));
        } else {
            SG_HIP(hipMemcpyAsync(s.h_out, s.d_out, (size_t)k * kSlot, hipMemcpyDeviceToHost, ds));
        }
        SG_HIP(hipEventRecord(s.ev[3], ds));
        return SG_OK;
    };
    auto more = [&] { return next < nrec && error == SG_OK; };
    if (direct) rc = run_direct(rs, ns, more, stage, launch, collect);
    else rc = run_pipeline(rs, ns, streams, more, stage, launch, copy_out, collect);
    if (rc != SG_OK) return rc;
    scrub.armed = false;  // collect() has cleared whatever it did not deliver
    res->records = good;
    res->consumed = consumed;
    res->out_len = opos;
    res->error = error != SG_OK ? error : (good == nrec ? header_error : SG_OK);
    return SG_OK;
}

}  // extern "C"
