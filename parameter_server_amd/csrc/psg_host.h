// psg_host.h -- host-side helpers shared by the C-ABI translation units
// (psg_runtime.hip, psg_exchange.hip): the thread-local last-error text
// behind psg_last_error() and the HIP error check.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/psg.h"

namespace psg {
// Records the message for psg_last_error() and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}  // namespace psg

#define HIP_TRY(expr)                                                            \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess)                                                        \
      return ::psg::fail(_e == hipErrorOutOfMemory ? PSG_ERR_OOM : PSG_ERR_DEVICE, \
                         "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                              \
  } while (0)
