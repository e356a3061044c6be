// loopback_cpp.cpp -- C4 of BASELINE.json in C++: an application stream
// through the GPU record layer over a loopback TCP connection, no Python on
// the data path.  The host side is include/suruga/
// (cipher.hpp's ChaCha20Poly1305 contexts, tls.hpp's HostBuffer and
// complete_records) over the C ABI: TlsWriter::write_data's batched form
// (sg_write_records, tls.rs:137-147) on the sending side and
// RecordStreamReader's (sg_read_records, tls.rs:217-281) on the receiving side,
// with fixed keys (the handshake bypassed as in src/test.rs:29-39).
//
//   sealer thread   sg_write_records of --chunk bytes into one of 3 wire buffers
//   sender thread   send() of each sealed wire buffer, in order
//   receiver thread recv() into one of 3 receive blocks; the partial record at
//                   a block's end (complete_records) is carried to the next one
//   opener thread   sg_read_records of a block's complete records into `out`,
//                   then every delivered byte is compared with what was sent
//
// --registered: the stream's source, the wire buffers, the receive blocks and
// the output are HostBuffers registered with sg_host_register, so the record
// bytes move by DMA straight between them and the device (the zero-copy path);
// otherwise the library frames through its pinned staging.
//
// Prints one JSON line (and writes it to --json-out): end-to-end GiB/s of
// application data and, per side, the milliseconds per GiB spent in the
// socket calls, H2D copies, kernels, D2H copies and host framing
// (sg_record_timing of each call), plus the verify time.
//
// Build: g++ -O2 -std=c++17 -pthread -Iinclude tools/loopback_cpp.cpp
//        -Lsuruga_amd -lsuruga_gpu -Wl,-rpath,<repo>/suruga_amd -o tools/loopback_cpp
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/suruga/cipher.hpp"
#include "../include/suruga/tls.hpp"

using namespace suruga;

namespace {

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

template <class T>
class Queue {
public:
    void push(T v) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(v));
        }
        cv_.notify_one();
    }
    T pop() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        T v = std::move(q_.front());
        q_.pop_front();
        return v;
    }

private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<T> q_;
};

struct Side {
    double socket_s = 0, verify_s = 0, h2d_ms = 0, kernel_ms = 0, d2h_ms = 0, host_ms = 0;
    uint64_t records = 0, bytes = 0, mismatched = 0, calls = 0;
    void add_timing() {
        double a = 0, b = 0, c = 0, d = 0;
        sg_record_timing(&a, &b, &c, &d);
        h2d_ms += a;
        kernel_ms += b;
        d2h_ms += c;
        host_ms += d;
        ++calls;
    }
};

std::string json_escape(const std::string& v) {
    std::string o;
    for (char ch : v) {
        if (ch == '"' || ch == '\\') o += '\\';
        if ((unsigned char)ch >= 0x20) o += ch;
    }
    return o;
}

std::string side_json(const Side& s, double gib, bool reader) {
    char b[768];
    std::snprintf(b, sizeof b,
                  "{\"records\": %llu, \"calls\": %llu, \"socket_ms\": %.1f, \"h2d_ms\": %.1f, \"kernel_ms\": %.1f, "
                  "\"d2h_ms\": %.1f, \"host_ms\": %.1f%s, \"per_gib_ms\": {\"socket\": %.1f, \"h2d\": %.1f, "
                  "\"kernel\": %.1f, \"d2h\": %.1f, \"host\": %.1f%s}}",
                  (unsigned long long)s.records, (unsigned long long)s.calls, 1e3 * s.socket_s, s.h2d_ms, s.kernel_ms,
                  s.d2h_ms, s.host_ms,
                  reader ? (", \"verify_ms\": " + std::to_string(1e3 * s.verify_s) + ", \"bytes\": " +
                            std::to_string(s.bytes) + ", \"mismatched_bytes\": " + std::to_string(s.mismatched))
                               .c_str()
                         : "",
                  1e3 * s.socket_s / gib, s.h2d_ms / gib, s.kernel_ms / gib, s.d2h_ms / gib, s.host_ms / gib,
                  reader ? (", \"verify\": " + std::to_string(1e3 * s.verify_s / gib)).c_str() : "");
    return b;
}

}  // namespace

int main(int argc, char** argv) {
    size_t total = size_t(1) << 30, chunk = size_t(16) << 20, block = size_t(16) << 20;
    bool reg = false;
    int device = 0;
    std::string json_out;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&] { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
        if (a == "--bytes") total = std::stoull(val());
        else if (a == "--chunk") chunk = std::stoull(val());
        else if (a == "--block") block = std::stoull(val());
        else if (a == "--registered") reg = true;
        else if (a == "--device") device = std::stoi(val());
        else if (a == "--json-out") json_out = val();
        else {
            std::fprintf(stderr, "usage: %s [--bytes N] [--chunk N] [--block N] [--registered] [--json-out F]\n", argv[0]);
            return 2;
        }
    }
    // the stream: a random pattern of `chunk` bytes, repeated
    HostBuffer pattern(chunk, reg);
    uint64_t x = 0xC4C4C4C4ull;
    for (size_t i = 0; i < chunk; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        pattern.data()[i] = (uint8_t)(x >> 56);
    }
    Bytes key(32);
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)i;
    ChaCha20Poly1305 aead(device);
    auto enc_p = aead.new_encryptor(key);
    auto dec_p = aead.new_decryptor(key);
    auto* enc = dynamic_cast<ChaCha20Poly1305Encryptor*>(enc_p.get());
    auto* dec = dynamic_cast<ChaCha20Poly1305Decryptor*>(dec_p.get());

    const int srv = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    addr.sin_port = 0;
    int one = 1;
    setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (::bind(srv, (sockaddr*)&addr, sizeof addr) != 0 || ::listen(srv, 1) != 0) {
        std::perror("bind/listen");
        return 1;
    }
    socklen_t alen = sizeof addr;
    getsockname(srv, (sockaddr*)&addr, &alen);

    Side W, R;
    std::atomic<bool> failed{false};
    std::string err;
    std::mutex err_mu;
    auto fail = [&](const std::string& e) {
        std::lock_guard<std::mutex> lk(err_mu);
        if (err.empty()) err = e;
        failed = true;
    };

    // ---- writer: sealer + sender -------------------------------------------
    const size_t wcap = sg_wire_bound(chunk);
    std::vector<std::unique_ptr<HostBuffer>> wires;
    for (int i = 0; i < 3; ++i) wires.push_back(std::make_unique<HostBuffer>(wcap, reg));
    Queue<int> wfree;
    Queue<std::pair<int, size_t>> wfull;
    for (int i = 0; i < 3; ++i) wfree.push(i);
    // ---- reader: receiver + opener -------------------------------------------
    const size_t rcap = block + SG_HEADER_LEN + SG_ENC_RECORD_MAX_LEN;
    std::vector<std::unique_ptr<HostBuffer>> blocks, outs;
    for (int i = 0; i < 3; ++i) {
        blocks.push_back(std::make_unique<HostBuffer>(rcap, reg));
        outs.push_back(std::make_unique<HostBuffer>(rcap, reg));
    }
    Queue<int> rfree;
    Queue<std::pair<int, size_t>> rfull;  // block, complete bytes (-1: end)
    for (int i = 0; i < 3; ++i) rfree.push(i);

    const double t0 = now_s();
    std::thread sealer([&] {
        try {
            uint64_t seq = 0;
            for (size_t sent = 0; sent < total && !failed;) {
                const size_t n = std::min(chunk, total - sent);
                const int w = wfree.pop();
                size_t wl = 0;
                const int64_t nrec = sg_write_records(enc->handle(), seq, 23, 3, 3, pattern.data(), n,
                                                      wires[w]->data(), wcap, &wl);
                check_sg(nrec < 0 ? (int)nrec : 0);
                W.add_timing();
                seq += (uint64_t)nrec;
                sent += n;
                wfull.push({w, wl});
            }
            W.records = seq;
        } catch (const std::exception& e) {
            fail(std::string("sealer: ") + e.what());
        }
        wfull.push({-1, 0});
    });
    std::thread sender([&] {
        const int s = ::socket(AF_INET, SOCK_STREAM, 0);
        int sz = 8 << 20;
        setsockopt(s, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
        if (::connect(s, (sockaddr*)&addr, sizeof addr) != 0) {
            fail("connect");
            return;
        }
        for (;;) {
            const auto it = wfull.pop();
            if (it.first < 0) break;
            const double a = now_s();
            const uint8_t* p = wires[it.first]->data();
            for (size_t off = 0; off < it.second;) {
                const ssize_t k = ::send(s, p + off, it.second - off, 0);
                if (k <= 0) {
                    fail("send");
                    break;
                }
                off += (size_t)k;
            }
            W.socket_s += now_s() - a;
            wfree.push(it.first);
        }
        ::shutdown(s, SHUT_WR);
        ::close(s);
    });
    std::thread receiver([&] {
        const int c = ::accept(srv, nullptr, nullptr);
        int sz = 8 << 20;
        setsockopt(c, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
        std::vector<uint8_t> carry;
        bool eof = false;
        while (!eof && !failed) {
            const int b = rfree.pop();
            uint8_t* p = blocks[b]->data();
            size_t have = carry.size();
            if (have) std::memcpy(p, carry.data(), have);
            while (have < block) {
                const double a = now_s();
                const ssize_t k = ::recv(c, p + have, rcap - have, 0);
                R.socket_s += now_s() - a;
                if (k <= 0) {
                    eof = true;
                    break;
                }
                have += (size_t)k;
            }
            size_t done = 0;
            try {
                done = complete_records(p, have);
            } catch (const std::exception& e) {
                fail(std::string("receiver: ") + e.what());
                break;
            }
            carry.assign(p + done, p + have);
            rfull.push({b, done});
        }
        if (!carry.empty() && !failed) fail("trailing partial record of " + std::to_string(carry.size()) + " bytes");
        rfull.push({-1, 0});
        ::close(c);
    });
    std::thread opener([&] {
        uint64_t seq = 0, got = 0;
        for (;;) {
            const auto it = rfull.pop();
            if (it.first < 0) break;
            try {
                sg_read_result res;
                HostBuffer& out = *outs[it.first];
                check_sg(sg_read_records(dec->handle(), seq, blocks[it.first]->data(), it.second, out.data(),
                                         out.size(), nullptr, nullptr, 1u << 20, &res));
                R.add_timing();
                if (res.error != SG_OK || res.consumed != it.second) throw detail::record_error(res.error);
                const double a = now_s();
                // the stream is the pattern repeated every `chunk` bytes
                for (size_t off = 0; off < res.out_len;) {
                    const size_t po = (got + off) % chunk, n = std::min<size_t>(res.out_len - off, chunk - po);
                    if (std::memcmp(out.data() + off, pattern.data() + po, n) != 0)
                        for (size_t i = 0; i < n; ++i) R.mismatched += out.data()[off + i] != pattern.data()[po + i];
                    off += n;
                }
                R.verify_s += now_s() - a;
                got += res.out_len;
                seq += res.records;
            } catch (const std::exception& e) {
                fail(std::string("opener: ") + e.what());
            }
            rfree.push(it.first);
        }
        R.records = seq;
        R.bytes = got;
    });
    sealer.join();
    sender.join();
    receiver.join();
    opener.join();
    const double wall = now_s() - t0;
    ::close(srv);

    const double gib = (double)total / (1ull << 30);
    const bool ok = !failed && R.bytes == total && R.mismatched == 0;
    char head[512];
    std::snprintf(head, sizeof head,
                  "{\"harness\": \"tools/loopback_cpp.cpp (C++ over include/suruga, no Python on the data path)\", "
                  "\"bytes\": %zu, \"chunk\": %zu, \"block\": %zu, \"registered\": %s, \"seconds\": %.4f, "
                  "\"gibs\": %.3f, \"correct\": %s, ",
                  total, chunk, block, reg ? "true" : "false", wall, gib / wall, ok ? "true" : "false");
    std::string line = std::string(head) + "\"build\": \"" + json_escape(sg_build_info()) + "\", \"writer\": " + side_json(W, gib, false) +
                       ", \"reader\": " + side_json(R, gib, true) + (err.empty() ? "" : ", \"error\": \"" + json_escape(err) + "\"") +
                       "}";
    std::printf("%s\n", line.c_str());
    if (!json_out.empty()) {
        if (FILE* f = std::fopen(json_out.c_str(), "w")) {
            std::fprintf(f, "%s\n", line.c_str());
            std::fclose(f);
        }
    }
    return ok ? 0 : 1;
}
