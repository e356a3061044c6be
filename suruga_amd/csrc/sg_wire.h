// sg_wire.h -- the record layer's wire parser (host only, no HIP).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace sg {

struct WireRec {
    size_t off;      // wire offset of the fragment (after the 5-byte header)
    uint32_t flen;   // fragment length (ct || tag)
    uint8_t type, major, minor;
};

// The complete records at the start of `wire` (at most max_records), header
// checks in TlsReader::read_record's order (tls.rs:217-238, 258-262, 269-272).
// Returns SG_OK when parsing stopped at the end of the complete records (or at
// max_records), else the error of the first bad header; `recs` holds the
// records before it.  Reads no byte outside [wire, wire + wire_len).
int32_t parse_wire(const uint8_t* wire, size_t wire_len, size_t max_records, std::vector<WireRec>& recs);

}  // namespace sg
