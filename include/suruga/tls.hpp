// suruga/tls.hpp -- C++ host-side mirror of suruga's record layer
// (klutzy/suruga src/tls.rs TlsWriter / TlsReader) with the batched GPU path.
//
//   TlsWriter::write_record   tls.rs:99-135   seq = be64(write_count), AD =
//       seq||type||major||minor||be16(len), 5-byte header, oversize -> panic
//       (std::logic_error here)
//   TlsWriter::write_data     tls.rs:137-147  2^14-byte fragments.  With the GPU
//       encryptor the whole call is ONE sg_write_records (batched sealing with
//       pinned double-buffered staging); any other Encryptor (e.g. the null
//       cipher of test.rs) takes the reference's per-record loop.
//   TlsReader::read_record    tls.rs:217-281  header checks, AD with len-16, decrypt
//   TlsReader::read_message   tls.rs:294-348  (handshake messages returned raw:
//       the handshake is outside this path)
//   RecordStreamReader        batched read_record: one sg_read_records per buffer.
//   HostBuffer                registered (sg_host_register) caller buffers: the
//       record layer's zero-copy path; complete_records: the header walk alone.
#ifndef SURUGA_TLS_HPP
#define SURUGA_TLS_HPP

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "cipher.hpp"

namespace suruga {

constexpr uint8_t TLS_VERSION_MAJOR = 3, TLS_VERSION_MINOR = 3;  // tls.rs:17
constexpr size_t RECORD_MAX_LEN = 1u << 14;                       // tls.rs:32
constexpr size_t ENC_RECORD_MAX_LEN = (1u << 14) + 2048u;         // tls.rs:35

// tls.rs:19-29
enum class ContentType : uint8_t {
    ChangeCipherSpecTy = 20,
    AlertTy = 21,
    HandshakeTy = 22,
    ApplicationDataTy = 23,
};

inline bool content_type_from_u8(uint8_t v, ContentType* out) {
    if (v < 20 || v > 23) return false;
    *out = static_cast<ContentType>(v);
    return true;
}

// tls.rs:38-61
struct Record {
    ContentType content_type;
    uint8_t ver_major, ver_minor;
    Bytes fragment;
    Record(ContentType ty, uint8_t major, uint8_t minor, Bytes frag)
        : content_type(ty), ver_major(major), ver_minor(minor), fragment(std::move(frag)) {
        if (fragment.size() > RECORD_MAX_LEN) throw std::logic_error("Record::new: fragment too long");  // panics
    }
};

// io::Write / io::Read stand-ins: the reference is generic over them.
class Writer {
public:
    virtual ~Writer() = default;
    virtual void write_all(const uint8_t* p, size_t n) = 0;  // throws TlsError{IoFailure}
};
class Reader {
public:
    virtual ~Reader() = default;
    virtual size_t read(uint8_t* p, size_t n) = 0;  // 0 = EOF
};

class VecWriter : public Writer {
public:
    Bytes buf;
    void write_all(const uint8_t* p, size_t n) override { buf.insert(buf.end(), p, p + n); }
};
class SliceReader : public Reader {
public:
    explicit SliceReader(Bytes b) : buf_(std::move(b)) {}
    size_t read(uint8_t* p, size_t n) override {
        const size_t k = std::min(n, buf_.size() - pos_);
        std::memcpy(p, buf_.data() + pos_, k);
        pos_ += k;
        return k;
    }

private:
    Bytes buf_;
    size_t pos_ = 0;
};

namespace detail {
inline void put_be64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = static_cast<uint8_t>(v >> (56 - 8 * i));  // util.rs:43-45
}
inline TlsError record_error(int32_t code) {
    switch (code) {
        case SG_E_BAD_MAC: return TlsError(TlsErrorKind::BadRecordMac, "wrong mac");
        case SG_E_SHORT: return TlsError(TlsErrorKind::BadRecordMac, "encrypted message too short");
        case SG_E_UNEXPECTED_MESSAGE: return TlsError(TlsErrorKind::UnexpectedMessage, "unexpected ContentType");
        case SG_E_RECORD_OVERFLOW: return TlsError(TlsErrorKind::RecordOverflow, "TLSEncryptedText too long");
        default: return TlsError(TlsErrorKind::InternalError, "record status " + std::to_string(code));
    }
}
}  // namespace detail

// tls.rs:63-171
class TlsWriter {
public:
    explicit TlsWriter(Writer& w) : w_(w) {}

    void set_encryptor(std::unique_ptr<Encryptor> enc) {  // tls.rs:91-97
        if (enc_) throw std::logic_error("encryptor already set");
        enc_ = std::move(enc);
        write_count = 0;
    }
    bool has_encryptor() const { return enc_ != nullptr; }

    void write_record(const Record& record) {  // tls.rs:99-135
        Bytes fragment;
        if (enc_) {
            uint8_t seq[8];
            detail::put_be64(seq, write_count);
            uint8_t ad[13];
            std::memcpy(ad, seq, 8);
            ad[8] = static_cast<uint8_t>(record.content_type);
            ad[9] = record.ver_major;
            ad[10] = record.ver_minor;
            ad[11] = static_cast<uint8_t>(record.fragment.size() >> 8);
            ad[12] = static_cast<uint8_t>(record.fragment.size());
            fragment = enc_->encrypt(Slice(seq, 8), record.fragment, Slice(ad, 13));
        } else {
            fragment = record.fragment;
        }
        if (fragment.size() > ENC_RECORD_MAX_LEN) throw std::logic_error("record too long");  // :118-121 panics
        const uint8_t hdr[5] = {static_cast<uint8_t>(record.content_type), record.ver_major, record.ver_minor,
                                static_cast<uint8_t>(fragment.size() >> 8), static_cast<uint8_t>(fragment.size())};
        w_.write_all(hdr, 5);
        w_.write_all(fragment.data(), fragment.size());
        write_count += 1;
    }

    void write_data(ContentType ty, Slice data) {  // tls.rs:137-147
        auto* gpu = dynamic_cast<ChaCha20Poly1305Encryptor*>(enc_.get());
        if (gpu && data.size > 0) {
            wire_.resize(sg_wire_bound(data.size));
            size_t wl = 0;
            const int64_t nrec = sg_write_records(gpu->handle(), write_count, static_cast<uint8_t>(ty),
                                                  TLS_VERSION_MAJOR, TLS_VERSION_MINOR, data.data, data.size,
                                                  wire_.data(), wire_.size(), &wl);
            check_sg(static_cast<int>(nrec < 0 ? nrec : 0));
            w_.write_all(wire_.data(), wl);
            write_count += static_cast<uint64_t>(nrec);
            return;
        }
        for (size_t off = 0; off < data.size; off += RECORD_MAX_LEN) {
            const size_t n = std::min(RECORD_MAX_LEN, data.size - off);
            write_record(Record(ty, TLS_VERSION_MAJOR, TLS_VERSION_MINOR, Bytes(data.data + off, data.data + off + n)));
        }
    }

    void write_alert(uint8_t level, uint8_t description) {  // tls.rs:154-158
        const uint8_t a[2] = {level, description};
        write_data(ContentType::AlertTy, Slice(a, 2));
    }
    void write_change_cipher_spec() {  // tls.rs:160-162
        const uint8_t one = 1;
        write_data(ContentType::ChangeCipherSpecTy, Slice(&one, 1));
    }
    void write_application_data(Slice data) {  // tls.rs:164-169
        if (!enc_) throw std::logic_error("attempted to write ApplicationData before handshake");
        write_data(ContentType::ApplicationDataTy, data);
    }

    uint64_t write_count = 0;

private:
    Writer& w_;
    std::unique_ptr<Encryptor> enc_;
    Bytes wire_;
};

// read_message result (tls.rs:283-292 Message)
struct Message {
    enum Kind { Handshake, ChangeCipherSpec, Alert, ApplicationData } kind;
    Bytes payload;           // Handshake / ApplicationData
    uint8_t alert_level = 0;  // Alert
    uint8_t alert_description = 0;
};

// alert.rs:5-44: the levels and descriptions FromPrimitive accepts
inline bool known_alert(uint8_t level, uint8_t desc) {
    static const uint8_t kDesc[] = {0,  10, 20, 21, 22, 30, 40, 41, 42, 43, 44, 45, 46,
                                    47, 48, 49, 50, 51, 60, 70, 71, 80, 90, 100, 110};
    if (level != 1 && level != 2) return false;
    return std::find(std::begin(kDesc), std::end(kDesc), desc) != std::end(kDesc);
}

// tls.rs:173-380
class TlsReader {
public:
    explicit TlsReader(Reader& r) : r_(r) {}

    void set_decryptor(std::unique_ptr<Decryptor> dec) {  // tls.rs:206-212
        if (dec_) throw std::logic_error("decryptor already set");
        dec_ = std::move(dec);
        read_count = 0;
    }

    Record read_record() {  // tls.rs:217-281
        uint8_t hdr[5];
        read_exact(hdr, 1);
        ContentType ty;
        if (!content_type_from_u8(hdr[0], &ty))
            throw TlsError(TlsErrorKind::UnexpectedMessage, "unexpected ContentType: " + std::to_string(hdr[0]));
        read_exact(hdr + 1, 4);
        const size_t len = (static_cast<size_t>(hdr[3]) << 8) | hdr[4];
        if (len > ENC_RECORD_MAX_LEN)
            throw TlsError(TlsErrorKind::RecordOverflow, "TLSEncryptedText too long: " + std::to_string(len));
        Bytes fragment(len);
        read_exact(fragment.data(), len);
        if (!dec_) {
            if (len > RECORD_MAX_LEN)
                throw TlsError(TlsErrorKind::RecordOverflow, "decrypted record too long: " + std::to_string(len));
            read_count += 1;
            return Record(ty, hdr[1], hdr[2], std::move(fragment));
        }
        uint8_t seq[8];
        detail::put_be64(seq, read_count);
        const size_t mac_len = dec_->mac_len();
        if (len < mac_len)
            throw TlsError(TlsErrorKind::BadRecordMac, "encrypted message too short: " + std::to_string(len));
        const size_t plen = len - mac_len;
        uint8_t ad[13];
        std::memcpy(ad, seq, 8);
        ad[8] = hdr[0];
        ad[9] = hdr[1];
        ad[10] = hdr[2];
        ad[11] = static_cast<uint8_t>(plen >> 8);
        ad[12] = static_cast<uint8_t>(plen);
        Bytes data = dec_->decrypt(Slice(seq, 8), fragment, Slice(ad, 13));
        if (data.size() > RECORD_MAX_LEN) throw std::logic_error("decrypted record too long");  // :269-272 panics
        read_count += 1;
        return Record(ty, hdr[1], hdr[2], std::move(data));
    }

    Message read_message() {  // tls.rs:294-348
        for (;;) {
            Record rec = read_record();
            switch (rec.content_type) {
                case ContentType::ChangeCipherSpecTy:
                    if (rec.fragment.size() != 1 || rec.fragment[0] != 1)
                        throw TlsError(TlsErrorKind::UnexpectedMessage, "invalid ChangeCipherSpec arrived");
                    return Message{Message::ChangeCipherSpec, {}};
                case ContentType::AlertTy: {
                    const size_t len = rec.fragment.size();
                    if (len == 0) throw TlsError(TlsErrorKind::UnexpectedMessage, "zero-length Alert record arrived");
                    if (len < 2) throw TlsError(TlsErrorKind::UnexpectedMessage, "awkward Alert record arrived");
                    if (!known_alert(rec.fragment[0], rec.fragment[1]))
                        throw TlsError(TlsErrorKind::UnexpectedMessage, "unknown alert");
                    Message m{Message::Alert, {}};
                    m.alert_level = rec.fragment[0];
                    m.alert_description = rec.fragment[1];
                    return m;
                }
                case ContentType::HandshakeTy:
                    if (rec.fragment.empty())
                        throw TlsError(TlsErrorKind::UnexpectedMessage, "zero-length Handshake arrived");
                    return Message{Message::Handshake, std::move(rec.fragment)};
                case ContentType::ApplicationDataTy:
                    return Message{Message::ApplicationData, std::move(rec.fragment)};
            }
        }
    }

    Bytes read_application_data() {  // tls.rs:350-364
        if (!dec_) throw std::logic_error("ApplicationData called before handshake");
        Message m = read_message();
        if (m.kind != Message::ApplicationData) throw std::logic_error("unimplemented: non-application message");
        return std::move(m.payload);
    }

    uint64_t read_count = 0;

private:
    void read_exact(uint8_t* p, size_t n) {  // util.rs:97-102 ReadExt
        while (n) {
            const size_t k = r_.read(p, n);
            if (k == 0) throw TlsError(TlsErrorKind::IoFailure, "unexpected EOF");
            p += k;
            n -= k;
        }
    }
    Reader& r_;
    std::unique_ptr<Decryptor> dec_;
};

// Batched TlsReader over a byte stream: all complete records in the buffer are
// opened by one sg_read_records call; a partial record stays buffered.
class RecordStreamReader {
public:
    explicit RecordStreamReader(ChaCha20Poly1305Decryptor& dec, size_t max_records = 1u << 16)
        : dec_(dec), types_(max_records), lens_(max_records) {}

    void feed(const uint8_t* p, size_t n) { buf_.insert(buf_.end(), p, p + n); }
    size_t buffered() const { return buf_.size(); }

    // Appends the plaintext of every complete record to `out` and returns the
    // (content type, length) of each; throws the first record's TlsError after
    // delivering the records before it.
    std::vector<std::pair<ContentType, uint32_t>> drain(Bytes& out) {
        std::vector<std::pair<ContentType, uint32_t>> recs;
        if (buf_.empty()) return recs;
        const size_t base = out.size();
        out.resize(base + buf_.size());
        sg_read_result res;
        check_sg(sg_read_records(dec_.handle(), read_count, buf_.data(), buf_.size(), out.data() + base,
                                 buf_.size(), types_.data(), lens_.data(), types_.size(), &res));
        out.resize(base + res.out_len);
        for (uint64_t i = 0; i < res.records; ++i)
            recs.emplace_back(static_cast<ContentType>(types_[i]), lens_[i]);
        buf_.erase(buf_.begin(), buf_.begin() + static_cast<std::ptrdiff_t>(res.consumed));
        read_count += res.records;
        if (res.error != SG_OK) throw detail::record_error(res.error);
        return recs;
    }

    uint64_t read_count = 0;

private:
    ChaCha20Poly1305Decryptor& dec_;
    Bytes buf_;
    std::vector<uint8_t> types_;
    std::vector<uint32_t> lens_;
};

// Page-locked caller buffer for the record layer's zero-copy path: memory
// registered with sg_host_register moves by DMA straight between it and the
// device (sg_write_records' data and wire, sg_read_records' wire and out).
// register_it = false gives the same buffer unregistered (the staged path).
class HostBuffer {
public:
    HostBuffer(size_t n, bool register_it) : n_(n) {
        p_ = static_cast<uint8_t*>(std::aligned_alloc(4096, (n + 4095) / 4096 * 4096 + (n ? 0 : 4096)));
        if (!p_) throw std::bad_alloc();
        if (register_it && n_) {  // (an empty buffer stays unregistered: nothing to move)
            const int rc = sg_host_register(p_, n_);
            if (rc != SG_OK) {
                std::free(p_);
                check_sg(rc);
            }
            reg_ = true;
        }
    }
    ~HostBuffer() {
        if (reg_) (void)sg_host_unregister(p_);
        std::free(p_);
    }
    HostBuffer(const HostBuffer&) = delete;
    HostBuffer& operator=(const HostBuffer&) = delete;
    uint8_t* data() const { return p_; }
    size_t size() const { return n_; }
    bool registered() const { return reg_; }

private:
    uint8_t* p_ = nullptr;
    size_t n_ = 0;
    bool reg_ = false;
};

// Bytes of `wire` taken by its complete records (tls.rs:217-238 header checks,
// sg_parse_records; host only): the rest is a partial record to carry over.
// Throws the first bad header's TlsError.
inline size_t complete_records(const uint8_t* wire, size_t n, size_t max_records = 4096) {
    std::vector<sg_wire_record> recs(max_records);
    size_t count = 0;
    int32_t error = SG_OK;
    check_sg(sg_parse_records(wire, n, recs.size(), recs.data(), &count, &error));
    if (error != SG_OK && count == 0) throw detail::record_error(error);
    return count ? recs[count - 1].offset + recs[count - 1].frag_len : 0;
}

}  // namespace suruga

#endif  // SURUGA_TLS_HPP
