// microbench_mix.hip -- gfx950 issue interaction of MFMA and VALU, and the cost
// of transcendentals, at 4 waves per SIMD (the cost kernel's occupancy).
//   A: NV v_pk_fma_f32 per iteration           B: NM v_mfma_f32_16x16x16_f16
//   C: both in one wave (independent chains)    D: v_exp_f32 stream
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mbm scripts/microbench_mix.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

template <int NV, int NM, int NT>
__global__ void mix(float* out, float a, float b, int iters) {
    f2 acc[NV > 0 ? NV : 1];
    f4 d[NM > 0 ? NM : 1];
    float t[NT > 0 ? NT : 1];
    const f2 av = {a, a}, bv = {b, b};
    h4 x = {(_Float16)(threadIdx.x * 1e-3f), (_Float16)a, (_Float16)b, (_Float16)1.f};
#pragma unroll
    for (int i = 0; i < (NV > 0 ? NV : 1); ++i) acc[i] = f2{threadIdx.x * 1e-3f + i, i * 0.5f};
#pragma unroll
    for (int i = 0; i < (NM > 0 ? NM : 1); ++i) d[i] = f4{0.f, 0.f, 0.f, (float)i};
#pragma unroll
    for (int i = 0; i < (NT > 0 ? NT : 1); ++i) t[i] = threadIdx.x * 1e-6f + i * 1e-3f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
#pragma unroll
            for (int i = 0; i < NM; ++i) d[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(x, x, d[i], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < NV; ++i) acc[i] = __builtin_elementwise_fma(acc[i], av, bv);
#pragma unroll
            for (int i = 0; i < NT; ++i) t[i] = __builtin_amdgcn_exp2f(t[i]);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += acc[i].x + acc[i].y;
#pragma unroll
    for (int i = 0; i < NM; ++i) s += d[i][0] + d[i][3];
#pragma unroll
    for (int i = 0; i < NT; ++i) s += t[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NV, int NM, int NT>
void run(const char* name, float* out, int ncu) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2048, blocks = ncu * 4;  // 256-thread blocks: 4 waves per SIMD
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((mix<NV, NM, NT>), dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    // cycles per wave-iteration-step on one SIMD: 4 waves share it
    const double clk = 2.4e9, steps = (double)iters * 8;
    printf("%-28s %8.3f ms  %7.2f SIMD cycles per step (4 waves)\n", name, best, best * 1e-3 * clk / steps);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 4096);
    int ncu = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) ncu = prop.multiProcessorCount;
    run<8, 0, 0>("A  8 pk_fma", out, ncu);
    run<16, 0, 0>("A 16 pk_fma", out, ncu);
    run<0, 4, 0>("B  4 mfma16x16x16", out, ncu);
    run<0, 8, 0>("B  8 mfma16x16x16", out, ncu);
    run<8, 4, 0>("C  8 pk_fma + 4 mfma", out, ncu);
    run<16, 4, 0>("C 16 pk_fma + 4 mfma", out, ncu);
    run<16, 8, 0>("C 16 pk_fma + 8 mfma", out, ncu);
    run<0, 0, 8>("D  8 exp2", out, ncu);
    run<8, 0, 8>("E  8 pk_fma + 8 exp2", out, ncu);
    return 0;
}
