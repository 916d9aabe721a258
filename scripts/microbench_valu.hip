// microbench_valu.hip -- FP32 FMA issue rates on gfx950 (scalar v_fma_f32 vs packed
// v_pk_fma_f32) at 1..8 waves per SIMD.  Calibration for the cost-kernel design.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mb scripts/microbench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int NACC>
__global__ void fma_scalar(float* out, float a, float b, int iters) {
    float acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(acc[i], a, b);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NACC>
__global__ void fma_packed(float* out, float a, float b, int iters) {
    f2 acc[NACC];
    const f2 av = {a, a}, bv = {b, b};
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = f2{threadIdx.x * 1e-3f + i, i * 0.5f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_elementwise_fma(acc[i], av, bv);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i].x + acc[i].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
    float* out;
    (void)hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 4096;
    int ncu = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) ncu = prop.multiProcessorCount;
    for (int waves_per_simd : {1, 2, 4, 8}) {
        const int blocks = ncu * waves_per_simd;  // 256-thread blocks = 1 wave per SIMD each
        for (int packed = 0; packed < 2; ++packed) {
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(e0);
                if (packed)
                    hipLaunchKernelGGL(fma_packed<8>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f, iters);
                else
                    hipLaunchKernelGGL(fma_scalar<16>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f, iters);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                const double fmas = (double)blocks * 256 * iters * 16;  // 16 fp32 FMAs per thread-iter
                if (rep == 1)
                    printf("waves/SIMD=%d %s: %.3f ms  %.1f TFLOP/s (fp32 FMA=2 flop)\n", waves_per_simd,
                           packed ? "v_pk_fma_f32" : "v_fma_f32   ", ms, 2 * fmas / ms / 1e9);
            }
        }
    }
    return 0;
}
