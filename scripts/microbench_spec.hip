// microbench_spec.hip -- gfx950: do an MFMA-only wave and a VALU-only wave on
// the same SIMD overlap?  512-thread workgroups (8 waves, two per SIMD: wave w
// and w + 4 share SIMD w & 3), 2 workgroups per CU = 4 waves per SIMD, the
// cost kernel's occupancy.  Per iteration a wave issues either NM
// v_mfma_f32_16x16x32_f16 (the cost kernel's vertical pass) or NV v_pk_fma_f32
// (its horizontal pass), by role:
//   role 0: every wave VALU              role 1: every wave MFMA
//   role 2: waves 0-3 MFMA, waves 4-7 VALU (each SIMD: one of each per workgroup)
//   role 3: every wave both, in one instruction stream (independent chains)
// If the pipes overlap across waves, role 2 takes ~max(role 0, role 1) / 2 per
// unit of work while role 3 takes ~their sum / 2.
// build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o scripts/mbs scripts/microbench_spec.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

// VALU work of one unit: VK 0 = one v_pk_fma_f32, 1 = two v_fma_f32, 2 = two v_exp_f32
template <int VK>
__device__ __forceinline__ f2 valu_op(f2 x, f2 a, f2 b) {
    if constexpr (VK == 0) return __builtin_elementwise_fma(x, a, b);
    else if constexpr (VK == 1) return f2{__builtin_fmaf(x.x, a.x, b.x), __builtin_fmaf(x.y, a.y, b.y)};
    else return f2{__builtin_amdgcn_exp2f(x.x) * 0.5f, __builtin_amdgcn_exp2f(x.y) * 0.5f};
}
template <int NV, int NM, int ROLE, int VK = 0>
__global__ __launch_bounds__(512) void spec(float* out, float a, float b, int iters) {
    const int w = threadIdx.x >> 6;
    const bool do_m = ROLE == 1 || ROLE == 3 || (ROLE == 2 && w < 4);
    const bool do_v = ROLE == 0 || ROLE == 3 || (ROLE == 2 && w >= 4);
    f2 acc[NV];
    f4 d[NM];
    const f2 av = {a, a}, bv = {b, b};
    h8 x;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (_Float16)(threadIdx.x * 1e-3f + i);
#pragma unroll
    for (int i = 0; i < NV; ++i) acc[i] = f2{threadIdx.x * 1e-3f + i, i * 0.5f};
#pragma unroll
    for (int i = 0; i < NM; ++i) d[i] = f4{0.f, 0.f, 0.f, (float)i};
    if (do_m && do_v) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
#pragma unroll
                for (int i = 0; i < NM; ++i) d[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, d[i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < NV; ++i) acc[i] = valu_op<VK>(acc[i], av, bv);
            }
        }
    } else if (do_m) {
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int i = 0; i < NM; ++i) d[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, d[i], 0, 0, 0);
    } else {
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int i = 0; i < NV; ++i) acc[i] = valu_op<VK>(acc[i], av, bv);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += acc[i].x + acc[i].y;
#pragma unroll
    for (int i = 0; i < NM; ++i) s += d[i][0] + d[i][3];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NV, int NM, int ROLE, int VK = 0>
void run(const char* name, float* out, int ncu) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 4096, blocks = ncu * 2;
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((spec<NV, NM, ROLE, VK>), dim3(blocks), dim3(512), 0, 0, out, 0.999f, 1e-3f, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
    }
    // SIMD cycles per iteration step (4 waves per SIMD) at 2.4 GHz
    const double steps = (double)iters * 4;
    printf("%-44s %8.3f ms  %8.1f SIMD cycles/step\n", name, best, best * 1e-3 * 2.4e9 / steps);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 4096);
    int ncu = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) ncu = prop.multiProcessorCount;
    printf("CUs %d\n", ncu);
    run<16, 4, 0>("role0 all VALU   (16 pk_fma)", out, ncu);
    run<16, 4, 1>("role1 all MFMA   (4 mfma 16x16x32)", out, ncu);
    run<16, 4, 2>("role2 split: MFMA waves 0-3, VALU waves 4-7", out, ncu);
    run<16, 4, 3>("role3 both in every wave", out, ncu);
    run<32, 4, 0>("role0 all VALU   (32 pk_fma)", out, ncu);
    run<32, 4, 2>("role2 split 32 pk_fma / 4 mfma", out, ncu);
    run<32, 4, 3>("role3 both 32 pk_fma + 4 mfma", out, ncu);
    run<8, 4, 0>("role0 all VALU   (8 pk_fma)", out, ncu);
    run<8, 4, 2>("role2 split 8 pk_fma / 4 mfma", out, ncu);
    run<8, 4, 3>("role3 both 8 pk_fma + 4 mfma", out, ncu);
    // plain (unpacked) FMAs and transcendentals against the same MFMA stream
    run<8, 4, 0, 1>("role0 all VALU   (16 v_fma_f32)", out, ncu);
    run<8, 4, 2, 1>("role2 split 16 v_fma_f32 / 4 mfma", out, ncu);
    run<8, 4, 3, 1>("role3 both 16 v_fma_f32 + 4 mfma", out, ncu);
    run<4, 4, 0, 2>("role0 all VALU   (8 v_exp_f32 + 8 mul)", out, ncu);
    run<4, 4, 2, 2>("role2 split 8 v_exp_f32 + 8 mul / 4 mfma", out, ncu);
    run<4, 4, 3, 2>("role3 both 8 v_exp_f32 + 8 mul + 4 mfma", out, ncu);
    return 0;
}
