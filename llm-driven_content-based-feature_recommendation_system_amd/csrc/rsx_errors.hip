// Error reporting and library identity for the C-ABI (see include/recsys_amd.h).
#include "rsx_common.h"
#include <stdarg.h>
#include <stdio.h>

namespace rsx {
static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace rsx

RSX_API const char* rsx_last_error(void) { return rsx::g_err; }

RSX_API int rsx_abi_version(void) { return 5; }

// Device the library's kernels were compiled for; callers compare against the
// running device's gcnArchName before the first launch.
RSX_API const char* rsx_target_arch(void) { return "gfx950"; }

#ifndef RSX_SRC_HASH
#define RSX_SRC_HASH "unknown"
#endif
// sha256 (first 16 hex digits) of the sources this library was built from (csrc/Makefile)
RSX_API const char* rsx_build_hash(void) { return RSX_SRC_HASH; }
