// Inner-product cost volume on the matrix cores (v_mfma_f32_16x16x4_f32).  Placeholder:
// not yet enabled, the dispatcher falls through to the VALU kernel.
#include "common.h"

namespace smcv {
int ip_mfma_entry(const void*, const void*, void*, int, int64_t, int64_t, int64_t, int64_t,
                  int64_t, const int64_t*, const int64_t*, void*, bool* handled) {
  *handled = false;
  return SM_OK;
}
}  // namespace smcv
