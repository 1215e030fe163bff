// Shared helpers for the gfx950 kernels of libnps_hip.so (see include/nps.h).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdarg>
#include <cmath>

#include "../../include/nps.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace nps {

void set_error(const char* fmt, ...);

#define NPS_CHECK_ARG(cond, ...)            \
    do {                                    \
        if (!(cond)) {                      \
            ::nps::set_error(__VA_ARGS__);  \
            return -1;                      \
        }                                   \
    } while (0)

#define NPS_CHECK_LAUNCH(what)                                                          \
    do {                                                                                \
        hipError_t e_ = hipGetLastError();                                              \
        if (e_ != hipSuccess) {                                                         \
            ::nps::set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e_)); \
            return -2;                                                                  \
        }                                                                               \
    } while (0)

// nn.GELU() default (approximate='none'): 0.5 x (1 + erf(x / sqrt 2))
__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// The same GELU with a branch-free erfc (Numerical Recipes' Chebyshev-fitted erfcc: fractional error < 1.2e-7
// for every argument, so GELU keeps ~1e-7 relative accuracy on both tails): 0.5 x erfc(|x|/sqrt 2) for x < 0,
// x - 0.5 x erfc(x/sqrt 2) otherwise; ~15 VALU (one v_rcp, one v_exp) instead of erff's branchy polynomial —
// for the fused GroupNorm+GELU prologue of the conv producers, which applies it to every staged element.
__device__ __forceinline__ float gelu_fast(float x) {
    const float z = fabsf(x) * 0.70710678118654752440f;
    // v_rcp_f32 (1 ulp): __frcp_rn expands to a ~10-instruction IEEE division sequence, which made this the
    // costliest part of the conv producers' GroupNorm+GELU prologue; the 1-ulp reciprocal moves the result by
    // < 3e-8 relative (the polynomial's own error is 1.2e-7)
    const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
    float p = fmaf(t, 0.17087277f, -0.82215223f);
    p = fmaf(t, p, 1.48851587f);
    p = fmaf(t, p, -1.13520398f);
    p = fmaf(t, p, 0.27886807f);
    p = fmaf(t, p, -0.18628806f);
    p = fmaf(t, p, 0.09678418f);
    p = fmaf(t, p, 0.37409196f);
    p = fmaf(t, p, 1.00002368f);
    p = fmaf(t, p, -1.26551223f);
    const float erfc = t * __expf(fmaf(-z, z, p));
    const float h = 0.5f * x * erfc;
    return x < 0.f ? h : x - h;
}

// gelu_fast on two values at once: the same operations in the same order (so bit-identical per element), written
// on float2 so the polynomial runs as packed v_pk_fma_f32 / v_pk_mul_f32 (one instruction per pair)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
    const f32x2 z = f32x2{fabsf(x[0]), fabsf(x[1])} * 0.70710678118654752440f;
    const f32x2 d = z * 0.5f + 1.0f;
    const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    f32x2 p = t * 0.17087277f + -0.82215223f;
    p = t * p + 1.48851587f;
    p = t * p + -1.13520398f;
    p = t * p + 0.27886807f;
    p = t * p + -0.18628806f;
    p = t * p + 0.09678418f;
    p = t * p + 0.37409196f;
    p = t * p + 1.00002368f;
    p = t * p + -1.26551223f;
    const f32x2 q = -z * z + p;
    const f32x2 erfc = t * f32x2{__expf(q[0]), __expf(q[1])};
    const f32x2 h = 0.5f * x * erfc;
    return f32x2{x[0] < 0.f ? h[0] : x[0] - h[0], x[1] < 0.f ? h[1] : x[1] - h[1]};
}

__device__ __forceinline__ int wrap_mod(int v, int n) {
    int r = v % n;
    return r < 0 ? r + n : r;
}

// wave64 sum of a double
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum of a double into lane 0 of wave 0 (blockDim.x multiple of 64, <= 1024).
__device__ __forceinline__ double block_sum(double v, double* scratch) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x < 64) {
        const int nw = blockDim.x >> 6;
        r = (lane < nw) ? scratch[lane] : 0.0;
        r = wave_sum(r);
    }
    __syncthreads();
    return r;
}

// ---- range tags (include/nps.h NPS_TAG_*): an upper bound of |x| over a tensor, kept as the max of
// NPS_TAG_SUB sub-slots so the writers' atomics spread over many addresses.
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Value of a tag (0 for NULL).  Wave-collective: all 64 lanes must be active (lane l reads sub-slot l).
__device__ __forceinline__ float tag_read(const float* tag) {
    if (tag == nullptr) return 0.f;
    const int lane = threadIdx.x & 63;
    return wave_max(tag[lane * NPS_TAG_STRIDE]);
}

// Raise a tag to cover m (>= 0) of every lane.  Wave-collective (all 64 lanes active); one atomic per
// wave, into the sub-slot picked by `salt` (e.g. the wave's global index).  Non-negative floats order
// like their bit patterns, so an unsigned atomic max is a float max.
__device__ __forceinline__ void tag_publish(float* tag, float m, unsigned salt) {
    if (tag == nullptr) return;
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0 && m > 0.f)
        atomicMax(reinterpret_cast<unsigned int*>(tag + (salt % NPS_TAG_SUB) * NPS_TAG_STRIDE), __float_as_uint(m));
}

// a globally unique-ish wave number of the calling wave (sub-slot salt)
__device__ __forceinline__ unsigned wave_salt() {
    return ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
}

}  // namespace nps
