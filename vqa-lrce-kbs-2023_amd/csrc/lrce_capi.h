// Internal helpers shared by the C-ABI entry points (error reporting).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/lrce_hip.h"

int lrce_fail(int code, const char* fmt, ...);
int lrce_check_launch(const char* what);
const uint64_t* lrce_rng_offset();  // registered device RNG offset (or nullptr)
