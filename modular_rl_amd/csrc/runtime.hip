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

}  // extern "C"
