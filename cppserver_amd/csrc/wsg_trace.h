// wsg_trace.h — roctx ranges around the host-side phases of the library
// (tracing): a host-staged batch, its segments' H2D / decode /
// D2H enqueue, a session batch's flush, a multi-GPU run.  `rocprofv3
// --marker-trace` shows them next to the kernel and copy trace; without a
// tool attached a range costs a call into an empty stub.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace wsg {

struct TraceRange {
    explicit TraceRange(const char* name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

} // namespace wsg
