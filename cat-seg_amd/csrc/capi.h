// Internal helpers for the extern "C" entry points (error state, checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "catseg_hip.h"

void catseg_set_error(const char* fmt, ...);

// Compute units of the current device (hipDeviceAttributeMultiprocessorCount, cached per device):
// persistent grids are sized from it, never from a literal 256 (partitioned parts expose fewer)
int catseg_device_cus();

// A/B knob registration (tuning.hip, include/catseg_hip_tuning.h): a process-wide int read at
// launch, settable by name through catseg_tuning_set; not part of the product ABI.
struct CatsegKnobReg { CatsegKnobReg(const char* name, int* value); };
#define CATSEG_KNOB(var, name) static CatsegKnobReg var##_knob_reg(name, &(var))

#define CATSEG_CHECK(cond, msg)                      \
  do {                                               \
    if (!(cond)) {                                   \
      catseg_set_error("%s", msg);                   \
      return CATSEG_ERR_ARG;                         \
    }                                                \
  } while (0)

#define CATSEG_FAIL(msg)        \
  do {                          \
    catseg_set_error("%s", msg);\
    return CATSEG_ERR_ARG;      \
  } while (0)

static inline int catseg_launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    catseg_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return CATSEG_ERR_HIP;
  }
  return CATSEG_OK;
}
