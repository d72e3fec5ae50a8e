// Library-level entry points of liblrspnp_hip.so (see include/lrspnp.h).
#include <string.h>

#include <vector>

#include "lrs_common.h"

extern "C" const char *lrs_version(void) { return "lrspnp-hip 0.1.0 (gfx950)"; }

extern "C" int lrs_check_device(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return LRS_E_NODEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return LRS_E_NODEVICE;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? LRS_OK : LRS_E_NODEVICE;
}

// waiter's later work runs after signaler's work so far: an event with a device-scope release (the
// two streams' kernels are on one device; nothing on the host waits on it).  One event per thread
// and device, re-recorded per call: a wait takes the event's state when it is enqueued.
extern "C" int lrs_stream_wait(void *waiter, void *signaler) {
    int dev = 0;   // the signalling stream's device (the event is created there)
    hipError_t e = hipStreamGetDevice((hipStream_t)signaler, &dev);
    if (e != hipSuccess) return (int)e;
    thread_local std::vector<hipEvent_t> evs;
    if ((int)evs.size() <= dev) evs.resize(dev + 1, nullptr);
    if (!evs[dev]) {
        int cur = 0;
        e = hipGetDevice(&cur);
        if (e == hipSuccess && cur != dev) e = hipSetDevice(dev);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&evs[dev], hipEventDisableTiming | hipEventDisableSystemFence);
        if (cur != dev) (void)hipSetDevice(cur);
        if (e != hipSuccess) {
            evs[dev] = nullptr;
            return (int)e;
        }
    }
    e = hipEventRecord(evs[dev], (hipStream_t)signaler);
    if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)waiter, evs[dev], 0);
    return (int)e;
}
