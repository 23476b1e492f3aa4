// Stream plumbing of the iteration pipeline: HIP streams restricted to a subset of
// the CUs (hipExtStreamCreateWithCUMask).  The latency-bound rollout occupies one
// block per CU on a few dozen CUs; a CU-masked stream pair lets the value-function
// fit of the previous iteration run on the remaining CUs at the same time without
// its blocks taking the rollout's CUs (core.run_policy_gradient_algorithm, pipelined).
#include "../../include/mrl_hip.h"
#include "mrl_common.h"

using namespace mrl;

extern "C" {

int mrl_device_cu_count(int32_t* out) {
  if (!out) return fail(E_ARG, "null pointer");
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_check(e, "mrl_device_cu_count");
  int n = 0;
  e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return hip_check(e, "mrl_device_cu_count");
  *out = n;
  return OK;
}

int mrl_stream_create_cu_mask(const uint32_t* mask, int32_t words, void** stream_out) {
  if (!mask || !stream_out || words <= 0) return fail(E_ARG, "mrl_stream_create_cu_mask: bad arguments");
  hipStream_t s = nullptr;
  hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return hip_check(e, "hipExtStreamCreateWithCUMask");
  *stream_out = (void*)s;
  return OK;
}

int mrl_stream_get_cu_mask(void* stream, int32_t words, uint32_t* mask) {
  if (!stream || !mask || words <= 0) return fail(E_ARG, "mrl_stream_get_cu_mask: bad arguments");
  return hip_check(hipExtStreamGetCUMask((hipStream_t)stream, (uint32_t)words, mask), "hipExtStreamGetCUMask");
}

int mrl_stream_destroy(void* stream) {
  if (!stream) return OK;
  return hip_check(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
}

// Cross-stream ordering on a memory value (tools/xstream_probe.py: 5.6 us per hop against
// 15.7 with an event): the producer's stream writes `value` to `flag` after its prior work,
// the consumer's stream waits until flag >= value before its later work.
int mrl_stream_signal(void* stream, uint32_t* flag, uint32_t value) {
  if (!flag) return fail(E_ARG, "mrl_stream_signal: null flag");
  return hip_check(hipStreamWriteValue32((hipStream_t)stream, flag, value, 0), "hipStreamWriteValue32");
}

int mrl_stream_wait(void* stream, uint32_t* flag, uint32_t value) {
  if (!flag) return fail(E_ARG, "mrl_stream_wait: null flag");
  return hip_check(hipStreamWaitValue32((hipStream_t)stream, flag, value, hipStreamWaitValueGte, 0xFFFFFFFFu),
                   "hipStreamWaitValue32");
}

}  // extern "C"
