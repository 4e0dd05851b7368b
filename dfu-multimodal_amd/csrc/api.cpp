// Library-level entry points of libdfu_hip.so: error string, version, zero fill.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include <atomic>
#include <mutex>
#include "../../include/dfu_hip.h"

static thread_local char g_err[1024] = "";

extern "C" void dfu_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* dfu_last_error_string(void) { return g_err; }

extern "C" int dfu_version(void) { return 1; }

extern "C" int dfu_zero(void* ptr, int64_t bytes, void* stream) {
  if (bytes == 0) return DFU_OK;
  hipError_t e = hipMemsetAsync(ptr, 0, (size_t)bytes, (hipStream_t)stream);
  if (e != hipSuccess) {
    dfu_set_error("dfu_zero: %s", hipGetErrorString(e));
    return (int)e;
  }
  return DFU_OK;
}

extern "C" int dfu_stream_capture_status(void* stream, int32_t* status) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hipError_t e = hipStreamIsCapturing((hipStream_t)stream, &st);
  if (e != hipSuccess) {
    dfu_set_error("dfu_stream_capture_status: %s", hipGetErrorString(e));
    return (int)e;
  }
  if (status) *status = (int32_t)st;
  return DFU_OK;
}

// Recovery after a failed HIP-graph capture (dfu_hip.graphs): when the origin stream's
// hipStreamEndCapture fails on unjoined work, the capture is NOT ended -- the origin and every
// stream forked into it stay in capture mode, and the next eager call that touches the legacy
// stream (an allocation, an event) fails.  Join every capturing stream into every other one
// (events recorded inside the capture), then end the capture on each (only the origin's end
// succeeds; the others return hipErrorStreamCaptureUnmatched) and drop the partial graphs.
extern "C" int dfu_streams_abort_capture(void* const* streams, int32_t n,
                                         int32_t* still_capturing) {
  if (still_capturing) *still_capturing = 0;
  if (n <= 0 || streams == nullptr) return DFU_OK;
  if (n > 64) {
    dfu_set_error("dfu_streams_abort_capture: at most 64 streams");
    return DFU_E_INVALID;
  }
  hipStream_t cap[64];
  int m = 0;
  for (int i = 0; i < n; ++i) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)streams[i], &st) == hipSuccess &&
        st != hipStreamCaptureStatusNone)
      cap[m++] = (hipStream_t)streams[i];
  }
  hipEvent_t ev[64];
  for (int i = 0; i < m; ++i) {
    ev[i] = nullptr;
    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) == hipSuccess)
      (void)hipEventRecord(ev[i], cap[i]);
  }
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j)
      if (i != j && ev[j] != nullptr) (void)hipStreamWaitEvent(cap[i], ev[j], 0);
  for (int pass = 0; pass < 2; ++pass)
    for (int i = 0; i < m; ++i) {
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(cap[i], &st) != hipSuccess || st == hipStreamCaptureStatusNone)
        continue;
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(cap[i], &g);
      if (g != nullptr) (void)hipGraphDestroy(g);
    }
  for (int i = 0; i < m; ++i)
    if (ev[i] != nullptr) (void)hipEventDestroy(ev[i]);
  int left = 0;
  for (int i = 0; i < m; ++i) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(cap[i], &st) == hipSuccess && st != hipStreamCaptureStatusNone)
      ++left;
  }
  (void)hipGetLastError();  // the failed ends above are the expected outcome
  if (still_capturing) *still_capturing = left;
  return DFU_OK;
}

// Library-owned streams (the encoder side stream, the ViT weight-gradient stream, graph-capture
// streams): non-blocking, so they never take part in the legacy stream's implicit
// synchronisation, and owned here rather than by torch's stream pool, so one left capturing by a
// failed capture (HIP cannot end it: dfu_streams_abort_capture) can be retired for good instead
// of being handed out again by the pool's round robin.
extern "C" int dfu_stream_create(int32_t priority, void** stream) {
  if (stream == nullptr) {
    dfu_set_error("dfu_stream_create: null output");
    return DFU_E_INVALID;
  }
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
  if (e != hipSuccess) {
    dfu_set_error("dfu_stream_create: %s", hipGetErrorString(e));
    return (int)e;
  }
  *stream = (void*)s;
  return DFU_OK;
}

// Stream-to-stream ordering without a torch Event object per call (torch's Stream.wait_stream
// builds one, records it and destroys it: ~6.5 us of host time against ~2 us here, and the
// library's two-stream step joins streams ~100 times a step).  A per-device ring of events
// created once: hipStreamWaitEvent waits for the record that is current when it is called, so
// an event re-recorded 256 joins later leaves the earlier waits intact; inside a graph capture
// the record / wait pair becomes the same dependency edge torch's events would make.
namespace {
constexpr int kWaitRing = 256;
constexpr int kWaitDevices = 64;
struct WaitRing {
  std::atomic<hipEvent_t*> ev{nullptr};
  std::atomic<uint32_t> next{0};
};
WaitRing g_wait[kWaitDevices];
std::mutex g_wait_mu;
}  // namespace

extern "C" int dfu_stream_wait(void* waiter, void* producer) {
  if (waiter == producer) return DFU_OK;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess || dev < 0 || dev >= kWaitDevices) {
    dfu_set_error("dfu_stream_wait: no current device (%d)", dev);
    return e != hipSuccess ? (int)e : DFU_E_INVALID;
  }
  WaitRing& r = g_wait[dev];
  hipEvent_t* ev = r.ev.load(std::memory_order_acquire);
  if (ev == nullptr) {
    std::lock_guard<std::mutex> lock(g_wait_mu);
    ev = r.ev.load(std::memory_order_relaxed);
    if (ev == nullptr) {
      hipEvent_t* fresh = new hipEvent_t[kWaitRing];
      for (int i = 0; i < kWaitRing; ++i) {
        e = hipEventCreateWithFlags(&fresh[i], hipEventDisableTiming);
        if (e != hipSuccess) {
          for (int j = 0; j < i; ++j) (void)hipEventDestroy(fresh[j]);
          delete[] fresh;
          dfu_set_error("dfu_stream_wait: %s", hipGetErrorString(e));
          return (int)e;
        }
      }
      r.ev.store(fresh, std::memory_order_release);
      ev = fresh;
    }
  }
  hipEvent_t x = ev[r.next.fetch_add(1, std::memory_order_relaxed) % kWaitRing];
  e = hipEventRecord(x, (hipStream_t)producer);
  if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)waiter, x, 0);
  if (e != hipSuccess) {
    dfu_set_error("dfu_stream_wait: %s", hipGetErrorString(e));
    return (int)e;
  }
  return DFU_OK;
}

extern "C" int dfu_stream_destroy(void* stream) {
  hipError_t e = hipStreamDestroy((hipStream_t)stream);
  if (e != hipSuccess) {
    dfu_set_error("dfu_stream_destroy: %s", hipGetErrorString(e));
    return (int)e;
  }
  return DFU_OK;
}
