// C-ABI plumbing: thread-local error string, version.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace mmr {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  // a failed HIP call (e.g. an out-of-memory hipMalloc) leaves a sticky per-thread error that the NEXT
  // call's launch check would report as its own: the failing call reports it here, then clears it
  (void)hipGetLastError();
}
void clear_error() { g_err[0] = 0; }
}  // namespace mmr

extern "C" {
const char* mmr_last_error(void) { return mmr::g_err; }
int mmr_version(void) { return 1; }
}
