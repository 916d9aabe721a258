// hq_launch.h -- host side of the kernel launchers (one per .hip translation
// unit of libhq).  Not part of the public ABI (include/hq.h).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace hq {

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

// Profiling: the next launches carry start/stop events in their dispatch packet
// (hipExtLaunchKernel), so timing a kernel adds no marker packet between kernels
// (each hipEventRecord between two kernels left the GPU idle ~5 us).  Set by
// set_launch_events (hq_search.hip), read by HQ_LAUNCH in every launcher.
extern thread_local hipEvent_t t_ev_start, t_ev_stop;
void set_launch_events(hipEvent_t start, hipEvent_t stop);

// Dynamic LDS of `bytes` for kernel `fn` (static + dynamic may pass 64 KiB, up to
// the CU's 160 KiB on gfx950): raised once per kernel (each template instance is
// its own function; the largest size granted so far is kept per function
// pointer, a refused raise is retried at the next call).  False if the runtime
// refused it: the launcher then returns an error instead of launching.
bool allow_dyn_lds(const void* fn, size_t bytes);

#define HQ_LAUNCH(K, G, B, S, STREAM, ...)                                                   \
    do {                                                                                     \
        if (t_ev_start || t_ev_stop)                                                         \
            hipExtLaunchKernelGGL(K, G, B, S, STREAM, t_ev_start, t_ev_stop, 0, __VA_ARGS__); \
        else                                                                                 \
            hipLaunchKernelGGL(K, G, B, S, STREAM, __VA_ARGS__);                             \
    } while (0)

}  // namespace hq
