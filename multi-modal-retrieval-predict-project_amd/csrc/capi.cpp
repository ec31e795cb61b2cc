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
std::atomic<int> pin_gemm_bf16{-1};
std::atomic<int> pin_x3_waves{-1};
std::atomic<int> pin_x3_mlp{-1};
}  // namespace mmr

extern "C" {
const char* mmr_last_error(void) { return mmr::g_err; }
int mmr_version(void) { return 1; }

mmr_status mmr_pin_variant(int32_t which, int32_t value) {
  mmr::clear_error();
  if (which == MMR_PIN_GEMM_BF16) {
    const int nv = mmr_linear_bf16_n_variants();
    MMR_REQUIRE(value >= -1 && value < nv, "mmr_pin_variant: gemm variant %d (-1 or 0..%d)", value, nv - 1);
    mmr::pin_gemm_bf16.store(value);
    return MMR_OK;
  }
  if (which == MMR_PIN_X3_WAVES) {
    MMR_REQUIRE(value == -1 || value == 4 || value == 8, "mmr_pin_variant: x3 waves %d (-1, 4, 8)", value);
    mmr::pin_x3_waves.store(value);
    return MMR_OK;
  }
  if (which == MMR_PIN_X3_MLP) {
    MMR_REQUIRE(value >= -1 && value <= 1, "mmr_pin_variant: x3 mlp form %d (-1, 0, 1)", value);
    mmr::pin_x3_mlp.store(value);
    return MMR_OK;
  }

  mmr::set_error("mmr_pin_variant: unknown pin %d", which);
  return MMR_ERR_INVALID;
}
}
