// hw_sqrt.hip -- TEST INFRASTRUCTURE ONLY: the device's square-root instruction
// (v_sqrt_f32) evaluated on the GPU for the CPU oracle.
//
// The reference's distance() on gfx950 (CL:179-192 as its OpenCL build
// compiles it) takes v_sqrt_f32 of the d^2 it computes.  That
// instruction is monotone and within 1 ulp but not correctly rounded (1 ulp off
// on 15.1% of the normal floats: scripts/mb/sqrt_probe.hip), and its exact
// values have no published definition, so the oracle's argmin (hq_oracle.c
// ref_len, oracle.py ref_len) takes it as a parameter: the GPU tests hand it
// these functions (tests/conftest.py); without them the oracle uses the
// correctly rounded sqrtf.  Never linked into the product.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>

namespace {

__global__ void sqrt_kernel(const float* x, float* y, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __builtin_amdgcn_sqrtf(x[i]);
}

std::mutex g_mu;
float* g_buf = nullptr;  // device scratch for one value (hqhw_sqrt1)

}  // namespace

extern "C" {

// y[i] = v_sqrt_f32(x[i]), i < n.  0 on success, else the HIP error code.
int hqhw_sqrt_n(const float* x, float* y, long long n) {
    if (n <= 0) return 0;
    float* d = nullptr;
    hipError_t e = hipMalloc(&d, 2 * (size_t)n * sizeof(float));
    if (e != hipSuccess) return (int)e;
    e = hipMemcpy(d, x, (size_t)n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        sqrt_kernel<<<(unsigned)((n + 255) / 256), 256>>>(d, d + n, n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(y, d + n, (size_t)n * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return (int)e;
}

// One value (the C oracle's callback; serialised).  NaN if the device fails.
float hqhw_sqrt1(float x) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_buf && hipMalloc(&g_buf, 2 * sizeof(float)) != hipSuccess) {
        g_buf = nullptr;
        return __builtin_nanf("");
    }
    float y = __builtin_nanf("");
    if (hipMemcpy(g_buf, &x, sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return y;
    sqrt_kernel<<<1, 64>>>(g_buf, g_buf + 1, 1);
    if (hipGetLastError() != hipSuccess) return y;
    if (hipMemcpy(&y, g_buf + 1, sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return __builtin_nanf("");
    return y;
}

}  // extern "C"
