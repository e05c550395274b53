// Library-level entry points: version and thread-local error reporting.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace {
thread_local char g_err[512] = "";
}

namespace p6 {
int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace p6

extern "C" int pose6d_version(void) { return 1; }
extern "C" const char* pose6d_last_error(void) { return g_err; }
