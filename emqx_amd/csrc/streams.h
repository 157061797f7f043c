// Stream ordering shared by the C-ABI entry points.
#pragma once
#include <hip/hip_runtime.h>

namespace emqx {

// A device call given no stream runs on a library-owned stream, created non-blocking (so it
// never serialises with unrelated work).  Such a stream is not ordered after the device's null
// stream, where a caller that passes no stream (PyTorch's default stream, plain hipMemcpy)
// produced the inputs: wait for the work already enqueued there first.
inline hipError_t after_null_stream(hipStream_t own) {
  hipEvent_t ev = nullptr;
  hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) return e;
  e = hipEventRecord(ev, nullptr);
  if (e == hipSuccess) e = hipStreamWaitEvent(own, ev, 0);
  const hipError_t d = hipEventDestroy(ev);  // released once the wait has been satisfied
  return e != hipSuccess ? e : d;
}

}  // namespace emqx
