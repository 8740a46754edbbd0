// ecamd_internal.hpp -- helpers ecamd_device.hip shares with the other launch files.
#pragma once

namespace ecamd {

int dev_ensure(int* dev_out);                       // 0, or ECAMD_ENODEV / ECAMD_EHIP
int dev_cu_count(int dev);
int dev_fail(int code, const char* fmt, ...);       // sets ecamd_last_error(), returns code
int dev_tune(const char* key);                      // current value of an ecamd_tune() knob

}  // namespace ecamd
