// hq_setup.hip -- once-per-search and output kernels: the S-CIELAB of the
// original image (LabRef, IM:100-153 + IM:285-370 with CL:2-145), the final
// quantize (CL:147-170, IM:770-798) and the error image (CL:201-231,
// IM:858-894).
#include "hq_device.h"
#include "hq_launch.h"

namespace hq {

// ----------------------------------------------------------------------------
// Packed 8-bit copy of the image (assign's U8 path): pixel q -> R | G << 8 |
// B << 16 when every channel is exactly k/255 (IM:100's int-RGB source, bit
// for bit: u8_unit); any other value (off the lattice, outside [0, 1], -0,
// NaN) sets *not_u8, and the host then drops the copy.  One pass on the
// device instead of a host scan of every pixel.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_u8_kernel(const float* R, const float* G, const float* B,
                                                      uint32_t* out, int* not_u8, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool bad = false;
    if (q < n) {
        const float f[3] = {R[q], G[q], B[q]};
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const bool in = f[j] >= 0.f && f[j] <= 1.f;
            const uint32_t k = in ? (uint32_t)__builtin_rintf(f[j] * 255.0f) : 0u;
            bad |= !in || __float_as_uint(u8_unit(k, 0)) != __float_as_uint(f[j]);
            v |= k << (8 * j);
        }
        out[q] = v;
    }
    if (__ballot(bad) && __lane_id() == 0) *not_u8 = 1;  // idempotent plain store
}

// ----------------------------------------------------------------------------
// LabRef (setup, once per search): IM:100-153 + IM:285-370 on the device.
// ----------------------------------------------------------------------------
// planar R,G,B -> Opp float4 (CL:79-90 then CL:111-116)
__global__ __launch_bounds__(256) void labref_opp_kernel(const float* R, const float* G,
                                                         const float* B, float4* opp, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float lr = srgb_lin(R[q]), lg = srgb_lin(G[q]), lb = srgb_lin(B[q]);
    const float X = dot3(lr, lg, lb, c_RGB2XYZ + 0);
    const float Y = dot3(lr, lg, lb, c_RGB2XYZ + 3);
    const float Z = dot3(lr, lg, lb, c_RGB2XYZ + 6);
    opp[q] = make_float4(dot3(X, Y, Z, c_XYZ2Opp + 0), dot3(X, Y, Z, c_XYZ2Opp + 3),
                         dot3(X, Y, Z, c_XYZ2Opp + 6), 0.f);
}

// inline XYZ float4 -> Opp float4 (CL:111-116), for hq_xyz_to_scielab
__global__ __launch_bounds__(256) void xyz_to_opp_kernel(const float4* xyz, float4* opp, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 v = xyz[q];
    opp[q] = make_float4(dot3(v.x, v.y, v.z, c_XYZ2Opp + 0), dot3(v.x, v.y, v.z, c_XYZ2Opp + 3),
                         dot3(v.x, v.y, v.z, c_XYZ2Opp + 6), 0.f);
}

// planar R,G,B -> inline XYZ float4 (CL:79-90), for hq_rgb_to_xyz
__global__ __launch_bounds__(256) void rgb_to_xyz_kernel(const float* R, const float* G,
                                                         const float* B, float4* xyz, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float lr = srgb_lin(R[q]), lg = srgb_lin(G[q]), lb = srgb_lin(B[q]);
    xyz[q] = make_float4(dot3(lr, lg, lb, c_RGB2XYZ + 0), dot3(lr, lg, lb, c_RGB2XYZ + 3),
                         dot3(lr, lg, lb, c_RGB2XYZ + 6), 0.f);
}

// Horizontal 1-D pass of convolve4Channels / convolve1Channel (CL:2-74) on the
// extended rows: out = sum_t fma(in[refl], k[t], acc), chans 3 (.xyz) or 1 (.x).
__global__ __launch_bounds__(256) void labref_hconv_kernel(const float4* in, float4* out,
                                                           const float* k, int half, int chans,
                                                           int W, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const int ly = (int)(q / W), x = (int)(q % W);
    const float4* row = in + (int64_t)ly * W;
    float ax = 0.f, ay = 0.f, az = 0.f;
    for (int i = -half, t = 0; i <= half; ++i, ++t) {
        const float4 v = row[reflect_only(x + i, W)];
        ax = fmaf(v.x, k[4 * t + 0], ax);
        if (chans == 3) {
            ay = fmaf(v.y, k[4 * t + 1], ay);
            az = fmaf(v.z, k[4 * t + 2], az);
        }
    }
    out[q] = make_float4(ax, ay, az, 0.f);
}

// Vertical pass over the owned rows reading the extended rows; update = 1
// accumulates into conv like the `update` flag of CL:30-36 / CL:67-73.
__global__ __launch_bounds__(256) void labref_vconv_kernel(const float4* in, float4* conv,
                                                           const float* k, int half, int chans,
                                                           int update, Geom g) {
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n_own) return;
    const int y = g.r0 + (int)(q / g.W), x = (int)(q % g.W);
    float ax = 0.f, ay = 0.f, az = 0.f;
    for (int i = -half, t = 0; i <= half; ++i, ++t) {
        const float4 v = in[(int64_t)(reflect_only(y + i, g.H) - g.e0) * g.W + x];
        ax = fmaf(v.x, k[4 * t + 0], ax);
        if (chans == 3) {
            ay = fmaf(v.y, k[4 * t + 1], ay);
            az = fmaf(v.z, k[4 * t + 2], az);
        }
    }
    float4 o = conv[q];
    if (update) {
        o.x += ax;
        if (chans == 3) { o.y += ay; o.z += az; }
    } else {
        o.x = ax;
        if (chans == 3) { o.y = ay; o.z = az; }
    }
    conv[q] = o;
}

// conv (Opp) -> Lab (CL:124-145, true division) -> planar L,A,B (pitch) and
// optional inline float4 copy.
__global__ __launch_bounds__(256) void labref_lab_kernel(const float4* conv, float* L, float* A,
                                                         float* B, float4* inline4, int W,
                                                         int64_t n, int pitch, float ilx,
                                                         float ily, float ilz) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 o = conv[q];
    const float il[3] = {ilx, ily, ilz};
    const float3 lab = opp2lab_ref(o.x, o.y, o.z, il);
    if (L) {
        const int64_t off = (q / W) * pitch + (q % W);
        L[off] = lab.x; A[off] = lab.y; B[off] = lab.z;
    }
    if (inline4) inline4[q] = make_float4(lab.x, lab.y, lab.z, 0.f);
}

// inline float4 Lab (owned rows) -> planar with pitch
__global__ __launch_bounds__(256) void lab_to_planar_kernel(const float4* lab4, float* L, float* A,
                                                            float* B, int W, int64_t n, int pitch) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 v = lab4[q];
    const int64_t off = (q / W) * pitch + (q % W);
    L[off] = v.x; A[off] = v.y; B[off] = v.z;
}

// ----------------------------------------------------------------------------
// Final quantize (CL:147-170): exhaustive argmin, any K, chosen colour out.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void quantize_kernel(const float4* in, const float4* colors,
                                                       int K, int* used, float4* out, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const float4 px = in[q];
    float4 bc = colors[0];
    float best = ref_dist4(px, bc);
    int bi = 0;
    for (int i = 1; i < K; ++i) {
        const float4 c = colors[i];
        const float d = ref_dist4(px, c);
        if (d < best) { best = d; bc = c; bi = i; }
    }
    out[q] = bc;
    if (used[bi] == 0) atomicOr(&used[bi], 1);
}

// CIEDE (CL:201-231) + error image of IM:886-893, fp64 block partials.
template <int DE>
__global__ __launch_bounds__(256) void error_image_kernel(const float4* orig, const float4* quant,
                                                          float4* err_img, double* partial,
                                                          int64_t n) {
    __shared__ double s_red[4];
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double v = 0.0;
    if (q < n) {
        const float4 a = orig[q], b = quant[q];
        const float e = delta_e<DE>(a.x, a.y, a.z, b.x, b.y, b.z);
        const float im = ((255.f - e) * (255.f - e)) / (255.f * 255.f);
        if (err_img) err_img[q] = make_float4(im, im, im, 0.f);
        v = e;
    }
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// ----------------------------------------------------------------------------
// Launchers
// ----------------------------------------------------------------------------
hipError_t launch_pack_u8(const float* R, const float* G, const float* B, uint32_t* out, int* not_u8,
                          int64_t n, hipStream_t s) {
    HQ_LAUNCH(pack_u8_kernel, dim3(blocks_for(n)), dim3(256), 0, s, R, G, B, out, not_u8, n);
    return hipGetLastError();
}

hipError_t launch_labref_opp(const float* R, const float* G, const float* B, float4* opp,
                             int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(labref_opp_kernel, dim3(blocks_for(n)), dim3(256), 0, s, R, G, B, opp, n);
    return hipGetLastError();
}

hipError_t launch_xyz_to_opp(const float4* xyz, float4* opp, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(xyz_to_opp_kernel, dim3(blocks_for(n)), dim3(256), 0, s, xyz, opp, n);
    return hipGetLastError();
}

hipError_t launch_rgb_to_xyz(const float* R, const float* G, const float* B, float4* xyz,
                             int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(rgb_to_xyz_kernel, dim3(blocks_for(n)), dim3(256), 0, s, R, G, B, xyz, n);
    return hipGetLastError();
}

hipError_t launch_labref_hconv(const float4* in, float4* out, const float* k, int half,
                               int chans, int W, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(labref_hconv_kernel, dim3(blocks_for(n)), dim3(256), 0, s, in, out, k,
                       half, chans, W, n);
    return hipGetLastError();
}

hipError_t launch_labref_vconv(const float4* in, float4* conv, const float* k, int half,
                               int chans, int update, const Geom& g, hipStream_t s) {
    const int64_t n_own = (int64_t)g.W * (g.r1 - g.r0);
    hipLaunchKernelGGL(labref_vconv_kernel, dim3(blocks_for(n_own)), dim3(256), 0, s, in, conv,
                       k, half, chans, update, g);
    return hipGetLastError();
}

hipError_t launch_labref_lab(const float4* conv, float* L, float* A, float* B, float4* inline4,
                             int W, int64_t n, int pitch, const float* illum, hipStream_t s) {
    hipLaunchKernelGGL(labref_lab_kernel, dim3(blocks_for(n)), dim3(256), 0, s, conv, L, A, B,
                       inline4, W, n, pitch, illum[0], illum[1], illum[2]);
    return hipGetLastError();
}

hipError_t launch_lab_to_planar(const float4* lab4, float* L, float* A, float* B, int W,
                                int64_t n, int pitch, hipStream_t s) {
    hipLaunchKernelGGL(lab_to_planar_kernel, dim3(blocks_for(n)), dim3(256), 0, s, lab4, L, A, B,
                       W, n, pitch);
    return hipGetLastError();
}

hipError_t launch_quantize(const float4* in, const float4* colors, int K, int* used, float4* out,
                           int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(quantize_kernel, dim3(blocks_for(n)), dim3(256), 0, s, in, colors, K,
                       used, out, n);
    return hipGetLastError();
}

hipError_t launch_error_image(const float4* orig, const float4* quant, float4* err_img,
                              double* partial, int64_t n, int de, hipStream_t s) {
    if (de == 0)
        hipLaunchKernelGGL(error_image_kernel<0>, dim3(blocks_for(n)), dim3(256), 0, s, orig,
                           quant, err_img, partial, n);
    else
        hipLaunchKernelGGL(error_image_kernel<1>, dim3(blocks_for(n)), dim3(256), 0, s, orig,
                           quant, err_img, partial, n);
    return hipGetLastError();
}

}  // namespace hq
