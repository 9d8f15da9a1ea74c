// gtf_mem.hip -- device memory for hosts without a framework allocator.
//
// The drop-in CLIs (extrapolate / clustering / update: one process per stage and
// iteration, run_gnn_trackml_mod.sh:61-146) spend most of an invocation bringing up a
// framework: on the MI355X box `import torch` + its first device tensor take 1.9-2.0 s
// of a 2.3 s extrapolation CLI, against 0.25-0.45 s for the HIP runtime itself
// (tools/cold_start.py). These entry points give such a host plain allocations and copies
// from the runtime libgtf is linked against, so it never loads a second one.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gtf.h"

namespace gtf {
void set_error(const char* msg);
}

namespace {
int fail(const char* what, hipError_t e) {
    char msg[256];
    snprintf(msg, sizeof(msg), "%s: %s", what, hipGetErrorString(e));
    gtf::set_error(msg);
    return -1;
}
}  // namespace

extern "C" {

int gtf_device_init(int32_t device) {
    const hipError_t e = hipSetDevice(device);
    return e == hipSuccess ? 0 : fail("gtf_device_init", e);
}

int gtf_malloc(void** ptr, size_t bytes) {
    if (!ptr) return fail("gtf_malloc", hipErrorInvalidValue);
    *ptr = nullptr;
    const hipError_t e = hipMalloc(ptr, bytes ? bytes : 256);   // never a null device pointer
    return e == hipSuccess ? 0 : fail("gtf_malloc", e);
}

int gtf_free(void* ptr) {
    const hipError_t e = hipFree(ptr);
    return e == hipSuccess ? 0 : fail("gtf_free", e);
}

int gtf_memcpy_htod(void* dst, const void* src, size_t bytes, gtf_stream_t stream) {
    if (!bytes) return 0;
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
    return e == hipSuccess ? 0 : fail("gtf_memcpy_htod", e);
}

int gtf_memcpy_dtoh(void* dst, const void* src, size_t bytes, gtf_stream_t stream) {
    if (!bytes) return 0;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? 0 : fail("gtf_memcpy_dtoh", e);
}

int gtf_memcpy_dtod(void* dst, const void* src, size_t bytes, gtf_stream_t stream) {
    if (!bytes) return 0;
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    return e == hipSuccess ? 0 : fail("gtf_memcpy_dtod", e);
}

int gtf_memset(void* dst, int32_t value, size_t bytes, gtf_stream_t stream) {
    if (!bytes) return 0;
    const hipError_t e = hipMemsetAsync(dst, value, bytes, (hipStream_t)stream);
    return e == hipSuccess ? 0 : fail("gtf_memset", e);
}

int gtf_stream_synchronize(gtf_stream_t stream) {
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? 0 : fail("gtf_stream_synchronize", e);
}

}  // extern "C"
