// sg_err.h -- the library's error reporting, without HIP: the host-only
// translation units (sg_wire.cpp, sg_keysched.cpp) include this alone, so they
// build with a plain host compiler (the sanitizer test, tests/cpp/test_host_san.cpp).
#pragma once

#include "../../include/suruga_gpu.h"

namespace sg {
// thread-local last-error message (sg_last_error); returns `code`
int fail(int code, const char* fmt, const char* detail = nullptr);
}  // namespace sg
