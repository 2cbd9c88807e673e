// Library-level entry points of libdauc.so (version, status text).
#include "dauc_internal.h"

extern "C" {

int dauc_version(void) { return 100; }  // 1.00

const char* dauc_strerror(int status) {
    if (status == DAUC_OK) return "success";
    if (status == DAUC_EINVAL) return "invalid argument";
    if (status < 0 && status > DAUC_EINVAL) return hipGetErrorString(static_cast<hipError_t>(-status));
    return "unknown status";
}

}  // extern "C"
