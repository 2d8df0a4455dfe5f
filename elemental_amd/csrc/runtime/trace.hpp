// Host-side trace ranges: the role of the reference's AUTO_PROFILE_REGION
// (include/El/core/Profiling.hpp:143-264, NVTX / VTune ranges at every SUMMA
// entry, NN.hpp:115-118, and in Gemm_impl, Gemm.cpp:148,170).  Here they are
// roctx ranges: `rocprofv3 --marker-trace` shows them on the host timeline next
// to the kernels each range launched; with no tool attached a push/pop is a
// few nanoseconds.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace elx {

class TraceRange {
public:
    explicit TraceRange(const char* name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace elx

#define ELX_TRACE_CAT2(a, b) a##b
#define ELX_TRACE_CAT(a, b) ELX_TRACE_CAT2(a, b)
#define ELX_TRACE(name) ::elx::TraceRange ELX_TRACE_CAT(elx_trace_, __LINE__)(name)
