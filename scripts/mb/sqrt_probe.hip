// Exhaustive check of the hardware square root (v_sqrt_f32) over every normal
// positive float: is it correctly rounded, and is it monotone?  The reference's
// distance() on gfx950 (its OpenCL build) ranks colours by v_sqrt_f32 of the
// fma-chain d^2 (for d^2 >= FLT_MIN), so the CPU oracle can restate it with a
// correctly rounded sqrtf only if the hardware's result is correctly rounded.
//
// CR test, exact in fp64: y = v_sqrt_f32(x) is correctly rounded iff
// m_lo^2 <= x <= m_hi^2 with m_lo, m_hi the midpoints between y and its
// neighbours (25 significant bits, so their squares are exact doubles).
//
// Build: hipcc --offload-arch=gfx950 -O2 -o sqrt_probe sqrt_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

struct Out {
    unsigned long long not_cr, not_mono, checked, beyond_1ulp;
    unsigned int n_ex;
    unsigned int ex_x[64], ex_y[64];
};

__global__ void probe(uint32_t base, uint32_t n, Out* o) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t bits = base + i;
    const float x = __uint_as_float(bits);
    const float y = __builtin_amdgcn_sqrtf(x);
    const float yn = __builtin_amdgcn_sqrtf(__uint_as_float(bits + 1));
    const uint32_t yb = __float_as_uint(y);
    const double dy = (double)y;
    const double lo = 0.5 * (dy + (double)__uint_as_float(yb - 1));
    const double hi = 0.5 * (dy + (double)__uint_as_float(yb + 1));
    const double dx = (double)x;
    const bool cr = lo * lo <= dx && dx <= hi * hi;
    // 1 ulp off: the correctly rounded value is a neighbour of y
    auto is_cr = [&](uint32_t cb) {
        const double c = (double)__uint_as_float(cb);
        const double l = 0.5 * (c + (double)__uint_as_float(cb - 1)), u = 0.5 * (c + (double)__uint_as_float(cb + 1));
        return l * l <= dx && dx <= u * u;
    };
    const bool off1 = !cr && (is_cr(yb - 1) || is_cr(yb + 1));
    const bool mono = bits + 1 >= 0x7f800000u || yn >= y;
    unsigned long long bad = 0, bm = 0, b1 = (!cr && !off1) ? 1 : 0;
    if (!cr) {
        bad = 1;
        const unsigned int k = atomicAdd(&o->n_ex, 1u);
        if (k < 64) {
            o->ex_x[k] = bits;
            o->ex_y[k] = yb;
        }
    }
    if (!mono) bm = 1;
    // wave totals, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        bad += __shfl_down(bad, off, 64);
        bm += __shfl_down(bm, off, 64);
        b1 += __shfl_down(b1, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (bad) atomicAdd(&o->not_cr, bad);
        if (bm) atomicAdd(&o->not_mono, bm);
        if (b1) atomicAdd(&o->beyond_1ulp, b1);
        atomicAdd(&o->checked, 64ull);
    }
}

int main() {
    Out* d = nullptr;
    if (hipMalloc(&d, sizeof(Out)) != hipSuccess) return 1;
    hipMemset(d, 0, sizeof(Out));
    const uint32_t lo = 0x00800000u, hi = 0x7f800000u;  // FLT_MIN .. inf (exclusive)
    const uint32_t chunk = 1u << 28;
    for (uint32_t b = lo; b < hi;) {
        const uint32_t n = (hi - b) < chunk ? (hi - b) : chunk;
        probe<<<(n + 255) / 256, 256>>>(b, n, d);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        b += n;
    }
    Out h;
    hipMemcpy(&h, d, sizeof(Out), hipMemcpyDeviceToHost);
    printf("{\"range\": [\"0x%08x\", \"0x%08x\"], \"checked_approx\": %llu, \"not_correctly_rounded\": %llu, "
           "\"not_monotone\": %llu, \"beyond_1ulp\": %llu, \"examples\": [",
           lo, hi, h.checked, h.not_cr, h.not_mono, h.beyond_1ulp);
    const unsigned int ne = h.n_ex < 64 ? h.n_ex : 64;
    for (unsigned int k = 0; k < ne && k < 16; ++k)
        printf("%s[\"0x%08x\", \"0x%08x\"]", k ? ", " : "", h.ex_x[k], h.ex_y[k]);
    printf("]}\n");
    hipFree(d);
    return 0;
}
