// sg_host.h -- private host-side declarations shared by the C-ABI translation
// units (sg_capi.cpp, sg_record.cpp).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>

#include "../../include/suruga_gpu.h"
#include "sg_err.h"

namespace sg {

int hip_fail(hipError_t e, const char* where);

struct RecordStaging;                   // sg_record.cpp
void record_staging_free(RecordStaging* rs);

// Makes `dev` the calling thread's current HIP device for a scope and restores
// the previous one on exit, so a context call never leaves the caller's thread
// on another device.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

}  // namespace sg

#define SG_HIP(call)                                                \
    do {                                                            \
        hipError_t e_ = (call);                                     \
        if (e_ != hipSuccess) return sg::hip_fail(e_, #call);       \
    } while (0)

// One context per direction (Aead::new_encryptor / new_decryptor): the key on
// the device, staging for single records, and (lazily) the record-layer
// pipeline of sg_write_records / sg_read_records.
// Single-record staging (sg_seal / sg_open): one pinned host block per
// direction that the kernels read and write over the host link, so a call is
// the keying and AEAD launches and one stream sync:
//   in  block: nonce @0 | ad @kSingleAdOff | record @kSingleInOff
//   out block: status @0 | output @kSingleOutOff
namespace sg {
constexpr size_t kSingleAdOff = 16;
constexpr size_t kSingleInOff = 512;
constexpr size_t kSingleOutOff = 64;
}  // namespace sg
struct sg_ctx {
    int device = 0;
    uint8_t* d_key = nullptr;      // 32 B
    uint8_t* h_in = nullptr;       // pinned blocks the kernels read and write directly:
                                   // kSingleInOff / kSingleOutOff + SG_MAX_RECORD_LEN + 64
    uint8_t* h_out = nullptr;
    void* d_ws = nullptr;
    hipStream_t stream = nullptr;
    sg::RecordStaging* rec = nullptr;
    std::mutex mu;
};
