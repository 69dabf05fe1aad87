// Host-side helpers shared by the C-ABI launchers (error reporting, streams).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/ghm_hip.h"

void ghm_set_error(const char* msg, const char* file, int line);

#define GHM_CHECK(cond, msg)                              \
  do {                                                    \
    if (!(cond)) {                                        \
      ghm_set_error(msg, __FILE__, __LINE__);         \
      return GHM_EINVAL;                                  \
    }                                                     \
  } while (0)

inline hipStream_t ghm_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

int ghm_launch_status();
