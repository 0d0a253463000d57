// Test infrastructure: the two error-reporting symbols hier_io.cpp and spt_build.cpp take from capi.hip, so that the
// host C++ of libhlgs.so can be built on its own with gcc under AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/sanitize/build.py).  Same behaviour as capi.hip's: the last message per thread.
#include <string>

#include "../../include/hlgs.h"

static thread_local std::string g_err;

namespace hlgs {
int fail_msg(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}
}  // namespace hlgs

extern "C" const char* hlgs_last_error(void) { return g_err.c_str(); }
