// sg_wire.cpp -- the TLS record header parser of sg_read_records and
// sg_parse_records (klutzy/suruga src/tls.rs:217-281), split out of
// sg_record.cpp so that the bytes a peer controls are parsed by code that
// builds and runs without a GPU: tests/cpp/test_host_san.cpp runs it under
// AddressSanitizer and UndefinedBehaviorSanitizer over a corpus of malformed
// and truncated headers.
#include "sg_wire.h"

#include "sg_err.h"

namespace sg {

int32_t parse_wire(const uint8_t* wire, size_t wire_len, size_t max_records, std::vector<WireRec>& recs) {
    size_t pos = 0;
    while (wire_len - pos >= SG_HEADER_LEN && recs.size() < max_records) {
        const uint8_t* h = wire + pos;
        if (h[0] < 20 || h[0] > 23)  // ContentType 20..23 (tls.rs:19-29, 218-225)
            return SG_E_UNEXPECTED_MESSAGE;
        const uint32_t flen = ((uint32_t)h[3] << 8) | h[4];
        if (flen > SG_ENC_RECORD_MAX_LEN)  // tls.rs:232-234
            return SG_E_RECORD_OVERFLOW;
        if (wire_len - pos - SG_HEADER_LEN < flen) break;  // incomplete: wait for more bytes
        if (flen < SG_MAC_LEN)  // tls.rs:258-262 "encrypted message too short"
            return SG_E_SHORT;
        if (flen - SG_MAC_LEN > SG_RECORD_MAX_LEN)  // tls.rs:269-272 (the reference panics)
            return SG_E_RECORD_OVERFLOW;
        recs.push_back({pos + SG_HEADER_LEN, flen, h[0], h[1], h[2]});
        pos += SG_HEADER_LEN + flen;
    }
    return SG_OK;
}

}  // namespace sg

extern "C" int sg_parse_records(const uint8_t* wire, size_t wire_len, size_t max_records, sg_wire_record* recs,
                                size_t* count, int32_t* error) {
    if ((!wire && wire_len) || !count || !error || (max_records && !recs))
        return sg::fail(SG_E_ARG, "NULL argument%s");
    std::vector<sg::WireRec> v;
    *error = sg::parse_wire(wire, wire_len, max_records, v);
    for (size_t i = 0; i < v.size(); ++i)
        recs[i] = {(uint64_t)v[i].off, v[i].flen, v[i].type, v[i].major, v[i].minor, 0};
    *count = v.size();
    return SG_OK;
}
