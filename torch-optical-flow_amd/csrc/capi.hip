// Version / status entry points of liboflow_hip.so (include/oflow.h).
#include "oflow_internal.h"

extern "C" int oflow_abi_version(void) { return OFLOW_ABI_VERSION; }

// every translation unit that writes or stages split-fp16 operands gets the flag pointer (for the current device)
extern "C" int oflow_set_range_flag(unsigned int* d_flag) {
  using namespace oflow;
  int st = range_flag_set_conv(d_flag);
  if (st == 0) st = range_flag_set_encoder(d_flag);
  if (st == 0) st = range_flag_set_s32io(d_flag);
  if (st == 0) st = range_flag_set_convc1(d_flag);
  return st;  // OFLOW_OK or a HIP error code (positive)
}

namespace {
__global__ void range_flag_exchange_kernel(unsigned int* flag, unsigned int* out) {
  if (threadIdx.x == 0) *out = atomicExch(flag, 0u);
}
}  // namespace

extern "C" int oflow_range_flag_exchange(unsigned int* d_flag, unsigned int* d_out, void* stream) {
  if (!d_flag || !d_out) return OFLOW_E_NULL;
  hipLaunchKernelGGL(range_flag_exchange_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), d_flag, d_out);
  return oflow::launch_status();
}

// Instrumentation (bench.py's per-kernel timings; not a reference interface): HIP timing events that can also be
// recorded inside a stream capture as external event-record nodes, so that every replay of the graph re-records them
// (torch.cuda.Event refuses external records on ROCm). Status: OFLOW_OK or a HIP error code.
extern "C" int oflow_timing_event_create(void** ev) {
  if (!ev) return OFLOW_E_NULL;
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreate(&e);
  *ev = e;
  return static_cast<int>(r);
}
extern "C" int oflow_timing_event_destroy(void* ev) { return static_cast<int>(hipEventDestroy(static_cast<hipEvent_t>(ev))); }
extern "C" int oflow_timing_event_record(void* ev, void* stream, int external) {
  hipEvent_t e = static_cast<hipEvent_t>(ev);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!external) return static_cast<int>(hipEventRecord(e, s));
  // during a capture: an event-record node appended to the stream's capture dependencies (ROCm 7.2 rejects
  // hipEventRecordWithFlags(hipEventRecordExternal) on a capturing stream with "invalid argument")
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  hipError_t r = hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &nd);
  if (r != hipSuccess) return static_cast<int>(r);
  if (cs != hipStreamCaptureStatusActive) return static_cast<int>(hipEventRecord(e, s));
  hipGraphNode_t node = nullptr;
  r = hipGraphAddEventRecordNode(&node, g, deps, nd, e);
  if (r != hipSuccess) return static_cast<int>(r);
  return static_cast<int>(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
}
extern "C" int oflow_timing_event_elapsed_ms(void* start, void* end, float* ms) {
  if (!ms) return OFLOW_E_NULL;
  return static_cast<int>(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(end)));
}

extern "C" const char* oflow_status_string(int status) {
  switch (status) {
    case OFLOW_OK: return "ok";
    case OFLOW_E_NULL: return "null pointer argument";
    case OFLOW_E_SHAPE: return "invalid or inconsistent size";
    case OFLOW_E_LEVELS: return "num_levels outside [1, 8]";
    case OFLOW_E_TINY:
      return "a correlation pyramid level is smaller than 2 pixels in H or W (the reference divides by "
             "W_l-1 / H_l-1 there and returns NaN); pad the input images to at least 128x128";
    case OFLOW_E_RADIUS: return "radius outside [0, 7]";
    case OFLOW_E_MODE: return "unknown interpolation or padding mode";
    case OFLOW_E_ALIGN: return "device pointer is not 4-byte aligned";
    default:
      if (status > 0) return hipGetErrorString(static_cast<hipError_t>(status));
      return "unknown oflow status";
  }
}
