// Calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths this
// repository's kernels use (8-byte and 1-byte per lane, plus a 16-byte reference):
// each kernel streams a known number of bytes once from HBM (buffers >> L2+MALL).
// Build: hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o calib_fetch
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void rd8(const double* __restrict__ a, double* out, size_t n) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.678) out[0] = s;
}
__global__ void rd16(const double2* __restrict__ a, double* out, size_t n) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i].x + a[i].y;
    if (s == 12345.678) out[0] = s;
}
__global__ void rd1(const uint8_t* __restrict__ a, double* out, size_t n) {
    unsigned s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 1234567u) out[0] = s;
}
__global__ void wr8(double* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}

int main() {
    const size_t bytes = (size_t)1 << 30;  // 1 GiB: far beyond L2 + Infinity Cache
    void *a, *out;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(rd8, dim3(4096), dim3(256), 0, 0, (const double*)a, (double*)out, bytes / 8);
        hipLaunchKernelGGL(rd16, dim3(4096), dim3(256), 0, 0, (const double2*)a, (double*)out, bytes / 16);
        hipLaunchKernelGGL(rd1, dim3(4096), dim3(256), 0, 0, (const uint8_t*)a, (double*)out, bytes);
        hipLaunchKernelGGL(wr8, dim3(4096), dim3(256), 0, 0, (double*)a, bytes / 8);
    }
    (void)hipDeviceSynchronize();
    printf("streamed %zu bytes per kernel (FETCH/WRITE_SIZE are in KiB: expect %zu)\n", bytes, bytes / 1024);
    return 0;
}
