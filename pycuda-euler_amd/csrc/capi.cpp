// capi.cpp -- error state and version of the libeulerhip C ABI (include/eulerhip.h).
#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace ec {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}
}  // namespace ec

extern "C" const char *ec_last_error(void) { return ec::g_err; }
extern "C" int ec_version(void) { return 100; /* 0.1.0 */ }
