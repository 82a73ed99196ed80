// gs_internal.h -- shared by the library's .hip files; not part of the C ABI.
#pragma once
#include "gsplat_mi355x.h"

// set gs_last_error() (fmt has one %s, filled with `what`) and return s
__attribute__((visibility("hidden"))) gs_status gs_internal_fail(gs_status s, const char *fmt, const char *what);
// GS_ERR_LAUNCH with the HIP error text if the last launch failed, else GS_OK
__attribute__((visibility("hidden"))) gs_status gs_internal_check_launch(const char *what);
