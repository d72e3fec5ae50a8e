// Library-level entry points of liblrspnp_hip.so (see include/lrspnp.h).
#include <string.h>

#include "lrs_common.h"

extern "C" const char *lrs_version(void) { return "lrspnp-hip 0.1.0 (gfx950)"; }

extern "C" int lrs_check_device(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return LRS_E_NODEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return LRS_E_NODEVICE;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? LRS_OK : LRS_E_NODEVICE;
}
