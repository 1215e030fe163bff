// Grid encoder input packing, TimeConvDense decoder, activation_wrapper
// post-processing, reductions and layout transforms for gfx950 (see include/nps.h).
#include "nps_common.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace nps {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace nps

extern "C" const char* nps_last_error(void) { return nps::g_err; }
extern "C" const char* nps_version(void) { return "nps_hip 0.1 gfx950"; }

namespace {

// ---------------------------------------------------------------- encoder input
// One block = 64 pixels of one sample; channels staged through LDS so both the
// planar reads of u and the NHWC writes are coalesced.
__global__ void pack_grid_kernel(const float* __restrict__ u, const float* __restrict__ pos,
                                 const float* __restrict__ cond, const float* __restrict__ sc, float* __restrict__ xin,
                                 float* __restrict__ vb, int CT, int HW, int K, int S, int Cp) {
    extern __shared__ float tile[];  // [Cp][65]
    const int b = blockIdx.y;
    const int p0 = blockIdx.x * 64;
    const int np = min(64, HW - p0);
    const int KS = K + S;
    for (int i = threadIdx.x; i < Cp * 64; i += blockDim.x) {
        const int ch = i / 64, p = i % 64;
        float v = 0.f;
        if (p < np) {
            const int pix = p0 + p;
            if (ch < CT)
                v = u[((size_t)b * CT + ch) * HW + pix];
            else if (ch < CT + 2)
                v = pos[((size_t)b * HW + pix) * 2 + (ch - CT)];
            else if (ch < CT + 2 + K)
                v = cond[b * K + (ch - CT - 2)];
            else if (ch < CT + 2 + KS)
                v = sc[((size_t)b * S + (ch - CT - 2 - K)) * HW + pix];
        }
        tile[ch * 65 + p] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < np * Cp; i += blockDim.x) {
        const int p = i / Cp, ch = i % Cp;
        xin[((size_t)b * HW + p0 + p) * Cp + ch] = tile[ch * 65 + p];
    }
    if (vb != nullptr) {
        for (int i = threadIdx.x; i < np * KS; i += blockDim.x) {
            const int p = i / KS, ch = i % KS;
            vb[((size_t)b * HW + p0 + p) * KS + ch] = tile[(CT + 2 + ch) * 65 + p];
        }
    }
}

// ---------------------------------------------------------------- TimeConvDense
// One block = 64 pixels x 4 slots.  Phase 1: d1[o][t1] = GELU(conv1d_k1,s2(pre)) into
// LDS; phase 2: d2 = conv1d_k2(d1), then add_delta, tanh, spatial-cond mask.
__global__ void timeconv_kernel(const float* __restrict__ pre, const float* __restrict__ u,
                                const float* __restrict__ w1, const float* __restrict__ b1,
                                const float* __restrict__ w2, const float* __restrict__ b2,
                                const float* __restrict__ dtcum, const float* __restrict__ mask, int mask_S,
                                int mask_ch, float* __restrict__ out, int nc, int tw, int HW, int ka, int kb, int L1,
                                int act_tanh) {
    extern __shared__ float d1s[];  // [2nc][L1][64]
    const int b = blockIdx.y;
    const int p = threadIdx.x & 63, slot = threadIdx.x >> 6;
    const int pix = blockIdx.x * 64 + p;
    const bool valid = pix < HW;
    const int L = 3 * tw;
    const int c2 = 2 * nc;
    const float* pb = pre + (size_t)b * nc * L * HW + pix;
    for (int o = slot; o < c2; o += 4) {
        for (int t1 = 0; t1 < L1; ++t1) {
            float acc = b1[o];
            if (valid) {
                for (int ci = 0; ci < nc; ++ci) {
                    const float* src = pb + (size_t)(ci * L + 2 * t1) * HW;
                    const float* wr = w1 + (o * nc + ci) * ka;
                    for (int k = 0; k < ka; ++k) acc = fmaf(wr[k], src[(size_t)k * HW], acc);
                }
            }
            d1s[(o * L1 + t1) * 64 + p] = nps::gelu_erf(acc);
        }
    }
    __syncthreads();
    if (!valid) return;
    const float* mrow = mask ? mask + ((size_t)b * mask_S + mask_ch) * HW + pix : nullptr;
    const float m = mrow ? *mrow : 0.f;
    for (int o2 = slot; o2 < nc; o2 += 4) {
        const float ulast = u[(((size_t)b * nc + o2) * tw + (tw - 1)) * HW + pix];
        for (int t2 = 0; t2 < tw; ++t2) {
            float acc = b2[o2];
            for (int o = 0; o < c2; ++o) {
                const float* wr = w2 + (o2 * c2 + o) * kb;
                for (int k = 0; k < kb; ++k) acc = fmaf(wr[k], d1s[(o * L1 + t2 + k) * 64 + p], acc);
            }
            float v = ulast + dtcum[t2] * acc;
            if (act_tanh) v = tanhf(v);
            if (mrow) v = v - m * v;
            out[(((size_t)b * nc + o2) * tw + t2) * HW + pix] = v;
        }
    }
}


// Specialised TimeConvDense for a compile-time (num_c, tw): the block's PX pixels of the planar
// pre-decoder output are staged in LDS once (coalesced), both conv1d layers run from LDS with fully
// unrolled taps and the weights read as wave-uniform (scalar-cache) loads.  PX sets the LDS per block
// (4 * PX * NC * (3 TW + 2 L1) bytes): 64 pixels at NC = 3 is 107 KB, one block (4 waves) per CU;
// 16 pixels lets 5 blocks share a CU.
template <int NC, int TW, int PX>
__global__ __launch_bounds__(256) void timeconv_fast_kernel(const float* __restrict__ pre, const float* __restrict__ u,
                                                            const float* __restrict__ w1, const float* __restrict__ b1,
                                                            const float* __restrict__ w2, const float* __restrict__ b2,
                                                            const float* __restrict__ dtcum, const float* __restrict__ mask,
                                                            int mask_S, int mask_ch, float* __restrict__ out, int HW,
                                                            int act_tanh) {
    constexpr int L = 3 * TW;
    constexpr int KA = (TW + 1) / 2;
    constexpr int KB = (TW + 3) / 4 + 1 + (TW % 4 == 0 ? 1 : 0);
    constexpr int L1 = (L - KA) / 2 + 1;
    constexpr int C2 = 2 * NC;
    static_assert(L1 - KB + 1 == TW, "TimeConvDense kernel sizes");
    extern __shared__ float lds[];
    constexpr int NSLOT = 256 / PX;
    constexpr int PP = PX + 1;       // row pitch: the NSLOT / 4 slots of a wave read rows 16 apart
    float* xs = lds;                 // [NC*L][PP]
    float* d1 = lds + NC * L * PP;   // [C2][L1][PP]
    const int b = blockIdx.y;
    const int p = threadIdx.x % PX, slot = threadIdx.x / PX;
    const int p0 = blockIdx.x * PX;
    const int np = min(PX, HW - p0);
    const float* src = pre + (size_t)b * NC * L * HW + p0;
    for (int i = threadIdx.x; i < NC * L * PX; i += 256) {
        const int r = i / PX, q = i % PX;
        xs[r * PP + q] = q < np ? src[(size_t)r * HW + q] : 0.f;
    }
    __syncthreads();
    // conv1 (stride 2) + GELU: each work item = one output channel x R1 consecutive positions, the
    // input window held in registers (R1*KA FMAs per 2*R1+KA-2 LDS reads)
    constexpr int R1 = 8;
    static_assert(L1 % R1 == 0, "conv1 run length");
    for (int j = slot; j < C2 * (L1 / R1); j += NSLOT) {
        const int o = j / (L1 / R1), t0 = (j - o * (L1 / R1)) * R1;
        float acc[R1];
#pragma unroll
        for (int r = 0; r < R1; ++r) acc[r] = b1[o];
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) {
            float xw[2 * (R1 - 1) + KA];
            const float* xr = xs + (ci * L + 2 * t0) * PP + p;
#pragma unroll
            for (int k = 0; k < 2 * (R1 - 1) + KA; ++k) xw[k] = xr[k * PP];
            const float* wr = w1 + (o * NC + ci) * KA;
#pragma unroll
            for (int k = 0; k < KA; ++k) {
                const float wk = wr[k];
#pragma unroll
                for (int r = 0; r < R1; ++r) acc[r] = fmaf(wk, xw[2 * r + k], acc[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < R1; ++r) d1[(o * L1 + t0 + r) * PP + p] = nps::gelu_erf(acc[r]);
    }
    __syncthreads();
    if (p >= np) return;
    const int pix = p0 + p;
    const float m = mask ? mask[((size_t)b * mask_S + mask_ch) * HW + pix] : 0.f;
    constexpr int R2 = 5;
    static_assert(TW % R2 == 0, "conv2 run length");
    for (int j = slot; j < NC * (TW / R2); j += NSLOT) {
        const int o2 = j / (TW / R2), t0 = (j - o2 * (TW / R2)) * R2;
        float acc[R2];
#pragma unroll
        for (int r = 0; r < R2; ++r) acc[r] = b2[o2];
#pragma unroll
        for (int o = 0; o < C2; ++o) {
            float dw[R2 - 1 + KB];
            const float* dr = d1 + (o * L1 + t0) * PP + p;
#pragma unroll
            for (int k = 0; k < R2 - 1 + KB; ++k) dw[k] = dr[k * PP];
            const float* wr = w2 + (o2 * C2 + o) * KB;
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const float wk = wr[k];
#pragma unroll
                for (int r = 0; r < R2; ++r) acc[r] = fmaf(wk, dw[r + k], acc[r]);
            }
        }
        const float ulast = u[(((size_t)b * NC + o2) * TW + (TW - 1)) * HW + pix];
#pragma unroll
        for (int r = 0; r < R2; ++r) {
            float v = ulast + dtcum[t0 + r] * acc[r];
            if (act_tanh) v = tanhf(v);
            if (mask) v = v - m * v;
            out[(((size_t)b * NC + o2) * TW + t0 + r) * HW + pix] = v;
        }
    }
}

// sums[p] = sum of plane p (fp64)
__global__ void plane_sums_kernel(const float* __restrict__ base, long plane_stride, int plane_size,
                                  double* __restrict__ sums) {
    __shared__ double red[16];
    const float* pl = base + (size_t)blockIdx.y * plane_stride;
    double s = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < plane_size; i += gridDim.x * blockDim.x) s += pl[i];
    s = nps::block_sum(s, red);
    if (threadIdx.x == 0) atomicAdd(&sums[blockIdx.y], s);
}

// activation_wrapper.py:80-105 'individual_static', element-wise in place
__global__ void volume_rescale_kernel(float* __restrict__ u, const double* __restrict__ new_tot,
                                      const double* __restrict__ prev_tot, const float* __restrict__ mpdcum,
                                      const float* __restrict__ mask, int mask_S, int mask_ch, int nc, int tw, int HW) {
    const int plane = blockIdx.y;  // (b, c, t)
    const int t = plane % tw;
    const int bc = plane / tw;
    const int b = bc / nc;
    const float newt = (float)new_tot[plane];
    const float prev = (float)prev_tot[bc];
    const float mpd = mpdcum[t];
    float dif = (1.f - newt / prev) * 100.f;
    dif = tanhf(dif / mpd) / 100.f * mpd;
    const float resc = 1.f - dif;
    const float f = resc * prev;
    float* pl = u + (size_t)plane * HW;
    const float* mk = mask ? mask + ((size_t)b * mask_S + mask_ch) * HW : nullptr;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += gridDim.x * blockDim.x) {
        float v = (pl[i] / newt) * f;
        if (mk) v = v - mk[i] * v;
        pl[i] = v;
    }
}

__global__ void sq_err_kernel(const float* __restrict__ a, const float* __restrict__ b, long n,
                              double* __restrict__ out) {
    __shared__ double red[16];
    double s = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float d = a[i] - b[i];
        s += (double)d * d;
    }
    s = nps::block_sum(s, red);
    if (threadIdx.x == 0) atomicAdd(out, s);
}

// [B][R][Cc] -> [B][Cc][R] tile transpose (R = H*W pixels, Cc channels)
__global__ void transpose_kernel(const float* __restrict__ in, float* __restrict__ out, int R, int Cc) {
    __shared__ float t[32][33];
    const int b = blockIdx.z;
    const int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
    const float* ib = in + (size_t)b * R * Cc;
    float* ob = out + (size_t)b * R * Cc;
    for (int i = threadIdx.y; i < 32; i += blockDim.y) {
        const int r = r0 + i, c = c0 + threadIdx.x;
        if (r < R && c < Cc) t[i][threadIdx.x] = ib[(size_t)r * Cc + c];
    }
    __syncthreads();
    for (int i = threadIdx.y; i < 32; i += blockDim.y) {
        const int c = c0 + i, r = r0 + threadIdx.x;
        if (r < R && c < Cc) ob[(size_t)c * R + r] = t[threadIdx.x][i];
    }
}


// ---------------------------------------------------------------- TimeConvDense backward
// One wave = 64 pixels, one pixel per lane; the forward chain is recomputed per pixel
// (dec_grid.py:126-146 + add_delta :8-31 + tanh + mask), then back-propagated:
//   gpre[b][ci*L + j][pix]  (planar, like the forward's pre-decoder output)
//   ws[block][w1 | b1 | w2 | b2]  per-block parameter-gradient partials (summed by nps_channel_sums).
// NC_ > 0: the loop bounds (num_c, tw and the derived kernel sizes) are compile-time, so the inner
// reductions unroll (their LDS reads issue back to back instead of one latency per FMA) and the weights
// become scalar loads; NC_ == 0 is the generic form (the arguments decide).
template <int NC_, int TW_>
__global__ __launch_bounds__(64) void timeconv_bwd_kernel(
    const float* __restrict__ pre, const float* __restrict__ u, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    const float* __restrict__ dtcum, const float* __restrict__ mask, int mask_S, int mask_ch,
    const float* __restrict__ gout, float* __restrict__ gpre, float* __restrict__ ws, int nc_, int tw_, int HW,
    int ka_, int kb_, int L1_, int act_tanh, int nparams) {
    extern __shared__ float lds[];
    constexpr bool CT = NC_ > 0;
    constexpr int KA_C = (TW_ + 1) / 2, KB_C = (TW_ + 3) / 4 + 1 + (TW_ % 4 == 0 ? 1 : 0);
    constexpr int L1_C = (3 * TW_ - KA_C) / 2 + 1;
    const int nc = CT ? NC_ : nc_, tw = CT ? TW_ : tw_;
    const int ka = CT ? KA_C : ka_, kb = CT ? KB_C : kb_, L1 = CT ? L1_C : L1_;
    const int C2 = 2 * nc, L = 3 * tw;
    float* d1 = lds;                       // [C2*L1][64]  GELU(conv1)
    float* gd = lds + C2 * L1 * 64;        // [C2*L1][64]  GELU'(conv1) -> grad of conv1 pre-activation
    float* gd2 = gd + C2 * L1 * 64;        // [nc*tw][64]  grad of conv2 output
    const int b = blockIdx.y, p = threadIdx.x;
    const int pix = blockIdx.x * 64 + p;
    const bool valid = pix < HW;
    const int pc = valid ? pix : 0;
    const float* xb = pre + (size_t)b * nc * L * HW + pc;
    const size_t blk = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    // 1. conv1 (stride 2) pre-activation
    for (int o = 0; o < C2; ++o)
        for (int t1 = 0; t1 < L1; ++t1) {
            float acc = b1[o];
#pragma unroll
            for (int ci = 0; ci < nc; ++ci)
#pragma unroll
                for (int k = 0; k < ka; ++k) acc = fmaf(w1[(o * nc + ci) * ka + k], xb[(size_t)(ci * L + 2 * t1 + k) * HW], acc);
            const float z = acc;
            d1[(o * L1 + t1) * 64 + p] = nps::gelu_erf(z);
            gd[(o * L1 + t1) * 64 + p] = 0.5f * (1.0f + erff(z * 0.70710678118654752440f)) +
                                         z * 0.39894228040143267794f * expf(-0.5f * z * z);
        }
    // 2. conv2, add_delta, tanh, mask -> gradient of conv2's output
    const float m = (mask && valid) ? mask[((size_t)b * mask_S + mask_ch) * HW + pix] : 0.f;
    for (int o2 = 0; o2 < nc; ++o2) {
        const float ulast = u[(((size_t)b * nc + o2) * tw + (tw - 1)) * HW + pc];
        for (int t = 0; t < tw; ++t) {
            float acc = b2[o2];
#pragma unroll
            for (int o = 0; o < C2; ++o)
#pragma unroll
                for (int k = 0; k < kb; ++k) acc = fmaf(w2[(o2 * C2 + o) * kb + k], d1[(o * L1 + t + k) * 64 + p], acc);
            float g = valid ? gout[(((size_t)b * nc + o2) * tw + t) * HW + pix] : 0.f;
            if (mask) g = g - m * g;
            if (act_tanh) {
                const float y = tanhf(ulast + dtcum[t] * acc);
                g *= 1.f - y * y;
            }
            gd2[(o2 * tw + t) * 64 + p] = g * dtcum[t];
        }
    }
    // 3. parameter partials of conv2: w2[o2][o][k], b2[o2]
    const int ow1 = 0, ob1 = C2 * nc * ka, ow2 = ob1 + C2, ob2 = ow2 + nc * C2 * kb;
    for (int o2 = 0; o2 < nc; ++o2) {
        float sb = 0.f;
#pragma unroll
        for (int t = 0; t < tw; ++t) sb += gd2[(o2 * tw + t) * 64 + p];
        sb = nps::wave_sum((double)sb);
        if (p == 0) ws[blk * nparams + ob2 + o2] = sb;
        for (int o = 0; o < C2; ++o)
            for (int k = 0; k < kb; ++k) {
                float s2 = 0.f;
#pragma unroll
                for (int t = 0; t < tw; ++t) s2 = fmaf(gd2[(o2 * tw + t) * 64 + p], d1[(o * L1 + t + k) * 64 + p], s2);
                s2 = (float)nps::wave_sum((double)s2);
                if (p == 0) ws[blk * nparams + ow2 + (o2 * C2 + o) * kb + k] = s2;
            }
    }
    // 4. gradient of conv1's pre-activation (in place over GELU')
    for (int o = 0; o < C2; ++o)
        for (int t1 = 0; t1 < L1; ++t1) {
            float g = 0.f;
#pragma unroll
            for (int o2 = 0; o2 < nc; ++o2)
#pragma unroll
                for (int k = 0; k < kb; ++k) {
                    const int t = t1 - k;
                    if (t >= 0 && t < tw) g = fmaf(gd2[(o2 * tw + t) * 64 + p], w2[(o2 * C2 + o) * kb + k], g);
                }
            gd[(o * L1 + t1) * 64 + p] *= g;
        }
    // 5. parameter partials of conv1: w1[o][ci][k], b1[o]
    for (int o = 0; o < C2; ++o) {
        float sb = 0.f;
#pragma unroll
        for (int t1 = 0; t1 < L1; ++t1) sb += gd[(o * L1 + t1) * 64 + p];
        sb = (float)nps::wave_sum((double)sb);
        if (p == 0) ws[blk * nparams + ob1 + o] = sb;
        for (int ci = 0; ci < nc; ++ci)
            for (int k = 0; k < ka; ++k) {
                float s1 = 0.f;
#pragma unroll
                for (int t1 = 0; t1 < L1; ++t1)
                    s1 = fmaf(gd[(o * L1 + t1) * 64 + p], xb[(size_t)(ci * L + 2 * t1 + k) * HW], s1);
                s1 = (float)nps::wave_sum((double)s1);
                if (p == 0) ws[blk * nparams + ow1 + (o * nc + ci) * ka + k] = s1;
            }
    }
    // 6. gradient of the pre-decoder output
    if (!valid) return;
    float* gb = gpre + (size_t)b * nc * L * HW + pix;
    for (int ci = 0; ci < nc; ++ci)
        for (int j = 0; j < L; ++j) {
            float g = 0.f;
#pragma unroll
            for (int k = 0; k < ka; ++k) {   // 2 t1 + k = j
                const int t1 = (j - k) >> 1;
                if (((j - k) & 1) || j - k < 0 || t1 >= L1) continue;
#pragma unroll
                for (int o = 0; o < C2; ++o) g = fmaf(gd[(o * L1 + t1) * 64 + p], w1[(o * nc + ci) * ka + k], g);
            }
            gb[(size_t)(ci * L + j) * HW] = g;
        }
}

// GELU and its derivative from one branch-free erfc (nps_common.hpp gelu_fast's Numerical Recipes
// polynomial, < 1.2e-7 relative): Phi(z) = 0.5 erfc(-z / sqrt 2), GELU = z Phi, GELU' = Phi + z phi(z).
__device__ __forceinline__ void gelu_and_grad(float z, float& g, float& gp) {
    const float x = fabsf(z) * 0.70710678118654752440f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, x, 1.0f));
    float p = fmaf(t, 0.17087277f, -0.82215223f);
    p = fmaf(t, p, 1.48851587f);
    p = fmaf(t, p, -1.13520398f);
    p = fmaf(t, p, 0.27886807f);
    p = fmaf(t, p, -0.18628806f);
    p = fmaf(t, p, 0.09678418f);
    p = fmaf(t, p, 0.37409196f);
    p = fmaf(t, p, 1.00002368f);
    p = fmaf(t, p, -1.26551223f);
    const float hx2 = -x * x;  // -z^2 / 2
    const float half_erfc = 0.5f * t * __expf(hx2 + p);
    const float phi = z < 0.f ? half_erfc : 1.0f - half_erfc;
    g = z * phi;
    gp = fmaf(z * 0.39894228040143267794f, __expf(hx2), phi);
}

// TimeConvDense backward for a compile-time (num_c, tw) — the twophase cfgs (tw = 25).  Same chain as
// timeconv_bwd_kernel (dec_grid.py:126-146 + add_delta :8-31 + tanh + mask), laid out for throughput:
//  * a block of 256 threads walks pixel groups of PX pixels (grid-stride, so a block keeps its parameter-
//    gradient accumulators in registers over many groups and writes ONE ws row at the end);
//  * thread = (slot, pixel): the PX lanes of a slot are PX pixels, the NSLOT = 256 / PX slots split each
//    phase's work items (an output channel x a run of positions), so every LDS row read is PX consecutive
//    floats and every item keeps its input window in registers;
//  * LDS per block: the group's planar `pre` rows, GELU(conv1), GELU' -> conv1 gradient (rows zero-padded
//    so the stride-2 transpose in the `pre` gradient needs no bounds tests), the conv2-output gradient
//    (zero-padded for the conv2 transpose) and the weights.
// Phases per group (barrier between): stage pre | A conv1 -> GELU, GELU' | B conv2 -> tanh', mask, dt ->
// g2 | C conv2^T(g2) * GELU' -> gz, D w2/b2 partials | E w1/b1 partials, F conv1^T(gz) -> gpre.
template <int NC, int TW, int PX>
__global__ __launch_bounds__(256, 2) void timeconv_bwd_fast_kernel(
    const float* __restrict__ pre, const float* __restrict__ u, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    const float* __restrict__ dtcum, const float* __restrict__ mask, int mask_S, int mask_ch,
    const float* __restrict__ gout, float* __restrict__ gpre, float* __restrict__ ws, int HW, int ngroups,
    int nrows, int act_tanh) {
    constexpr int L = 3 * TW;
    constexpr int KA = (TW + 1) / 2;
    constexpr int KB = (TW + 3) / 4 + 1 + (TW % 4 == 0 ? 1 : 0);
    constexpr int L1 = (L - KA) / 2 + 1;
    constexpr int C2 = 2 * NC;
    constexpr int NSLOT = 256 / PX, PP = PX + 1;
    constexpr int RA = 4, RB = 5, RM = 4;          // run lengths: conv1 / conv2 positions, gpre pairs
    constexpr int QN = (KA + 1) / 2;               // taps of one parity
    constexpr int GZ0 = QN - 1;                    // left zero pad of a gz row
    constexpr int MR = ((L + 1) / 2 + RM - 1) / RM * RM;
    constexpr int GZW = MR + GZ0;                  // padded gz row (t1 = m - q over m < MR, q < QN)
    constexpr int G2W = TW + 2 * (KB - 1);         // padded g2 row
    constexpr int KH = KB / 2, KAH = (KA + 1) / 2; // tap halves of the w2 / w1 partial items
    constexpr int NW1 = C2 * NC * KA, NW2 = NC * C2 * KB;
    constexpr int NPAR = NW1 + C2 + NW2 + NC;
    static_assert(L1 - KB + 1 == TW && L1 % RA == 0 && TW % RB == 0 && KB % 2 == 0, "TimeConvDense sizes");
    static_assert(GZW >= GZ0 + L1, "gz padding");
    constexpr int NA = C2 * (L1 / RA), NB = NC * (TW / RB), ND = NC * C2 * 2, NE = C2 * NC * 2,
                  NF = NC * (MR / RM);
    constexpr int NDI = (ND + NSLOT - 1) / NSLOT, NEI = (NE + NSLOT - 1) / NSLOT;

    extern __shared__ float lds[];
    float* xs = lds;                    // [NC*L][PP]
    float* d1 = xs + NC * L * PP;       // [C2*L1][PP]
    float* gz = d1 + C2 * L1 * PP;      // [C2*GZW][PP]   GELU' then the conv1 pre-activation gradient
    float* g2 = gz + C2 * GZW * PP;     // [NC*G2W][PP]
    float* w1s = g2 + NC * G2W * PP;    // [C2][NC][KA]
    float* w2s = w1s + NW1;             // [NC][C2][KB]
    float* b1s = w2s + NW2;
    float* b2s = b1s + C2;
    float* dts = b2s + NC;

    const int tid = threadIdx.x;
    const int p = tid % PX, slot = tid / PX;
    for (int i = tid; i < C2 * GZW * PP + NC * G2W * PP; i += 256) gz[i] = 0.f;  // gz and g2 (pads stay 0)
    for (int i = tid; i < NW1; i += 256) w1s[i] = w1[i];
    for (int i = tid; i < NW2; i += 256) w2s[i] = w2[i];
    if (tid < C2) b1s[tid] = b1[tid];
    if (tid < NC) b2s[tid] = b2[tid];
    if (tid < TW) dts[tid] = dtcum[tid];

    double accD[NDI][KH], accE[NEI][KAH], accb2[NDI], accb1[NEI];
#pragma unroll
    for (int i = 0; i < NDI; ++i)
#pragma unroll
        for (int k = 0; k < KH; ++k) accD[i][k] = accb2[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NEI; ++i)
#pragma unroll
        for (int k = 0; k < KAH; ++k) accE[i][k] = accb1[i] = 0.0;

    const int gpb = (HW + PX - 1) / PX;  // groups per sample
    for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const int b = grp / gpb;
        const int p0 = (grp - b * gpb) * PX;
        const int np = min(PX, HW - p0);
        const bool valid = p < np;
        const int pix = p0 + (valid ? p : 0);
        __syncthreads();  // previous group's readers of xs / gz / g2 are done
        {
            const float* src = pre + (size_t)b * NC * L * HW + p0;
            for (int i = tid; i < NC * L * PX; i += 256) {
                const int r = i / PX, q = i % PX;
                xs[r * PP + q] = q < np ? src[(size_t)r * HW + q] : 0.f;
            }
        }
        __syncthreads();
        // A. conv1 (stride 2) -> GELU into d1, GELU' into gz
        for (int j = slot; j < NA; j += NSLOT) {
            const int o = j / (L1 / RA), t0 = (j - o * (L1 / RA)) * RA;
            float acc[RA];
#pragma unroll
            for (int r = 0; r < RA; ++r) acc[r] = b1s[o];
#pragma unroll
            for (int ci = 0; ci < NC; ++ci) {
                float xw[2 * (RA - 1) + KA];
                const float* xr = xs + (ci * L + 2 * t0) * PP + p;
#pragma unroll
                for (int k = 0; k < 2 * (RA - 1) + KA; ++k) xw[k] = xr[k * PP];
                const float* wr = w1s + (o * NC + ci) * KA;
#pragma unroll
                for (int k = 0; k < KA; ++k) {
                    const float wk = wr[k];
#pragma unroll
                    for (int r = 0; r < RA; ++r) acc[r] = fmaf(wk, xw[2 * r + k], acc[r]);
                }
            }
#pragma unroll
            for (int r = 0; r < RA; ++r) {
                float g, gp;
                gelu_and_grad(acc[r], g, gp);
                d1[(o * L1 + t0 + r) * PP + p] = g;
                gz[(o * GZW + GZ0 + t0 + r) * PP + p] = gp;
            }
        }
        __syncthreads();
        // B. conv2, add_delta, tanh, mask -> g2 = d loss / d conv2 output (x dt)
        {
            const float m = (mask && valid) ? mask[((size_t)b * mask_S + mask_ch) * HW + pix] : 0.f;
            for (int j = slot; j < NB; j += NSLOT) {
                const int o2 = j / (TW / RB), t0 = (j - o2 * (TW / RB)) * RB;
                float acc[RB];
#pragma unroll
                for (int r = 0; r < RB; ++r) acc[r] = b2s[o2];
#pragma unroll
                for (int o = 0; o < C2; ++o) {
                    float dw[RB - 1 + KB];
                    const float* dr = d1 + (o * L1 + t0) * PP + p;
#pragma unroll
                    for (int k = 0; k < RB - 1 + KB; ++k) dw[k] = dr[k * PP];
                    const float* wr = w2s + (o2 * C2 + o) * KB;
#pragma unroll
                    for (int k = 0; k < KB; ++k) {
                        const float wk = wr[k];
#pragma unroll
                        for (int r = 0; r < RB; ++r) acc[r] = fmaf(wk, dw[r + k], acc[r]);
                    }
                }
                const float ulast = u[(((size_t)b * NC + o2) * TW + (TW - 1)) * HW + pix];
                const float* gr = gout + (((size_t)b * NC + o2) * TW + t0) * HW + pix;
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const float dt = dts[t0 + r];
                    float g = valid ? gr[(size_t)r * HW] : 0.f;
                    if (mask) g = g - m * g;
                    if (act_tanh) {
                        const float y = tanhf(ulast + dt * acc[r]);
                        g *= 1.f - y * y;
                    }
                    g2[(o2 * G2W + KB - 1 + t0 + r) * PP + p] = g * dt;
                }
            }
        }
        __syncthreads();
        // C. gz = GELU' * conv2^T(g2)   (in place over GELU')
        for (int j = slot; j < NA; j += NSLOT) {
            const int o = j / (L1 / RA), t0 = (j - o * (L1 / RA)) * RA;
            float acc[RA];
#pragma unroll
            for (int r = 0; r < RA; ++r) acc[r] = 0.f;
#pragma unroll
            for (int o2 = 0; o2 < NC; ++o2) {
                // t1 - k + KB - 1 over t1 in [t0, t0 + RA), k < KB: padded g2 index t0 .. t0 + RA + KB - 2
                float gw[RA + KB - 1];
                const float* gr = g2 + (o2 * G2W + t0) * PP + p;
#pragma unroll
                for (int i = 0; i < RA + KB - 1; ++i) gw[i] = gr[i * PP];
                const float* wr = w2s + (o2 * C2 + o) * KB;
#pragma unroll
                for (int k = 0; k < KB; ++k) {
                    const float wk = wr[k];
#pragma unroll
                    for (int r = 0; r < RA; ++r) acc[r] = fmaf(wk, gw[r - k + KB - 1], acc[r]);
                }
            }
#pragma unroll
            for (int r = 0; r < RA; ++r) gz[(o * GZW + GZ0 + t0 + r) * PP + p] *= acc[r];
        }
        // D. w2 / b2 partials: item (o2, o, tap half); b2 rides on (o2, 0, 0)
#pragma unroll
        for (int ii = 0; ii < NDI; ++ii) {
            const int j = slot + ii * NSLOT;
            if (j < ND) {
                const int o2 = j / (2 * C2), o = (j / 2) % C2, kh = j & 1;
                const float* gr = g2 + (o2 * G2W + KB - 1) * PP + p;
                const float* dr = d1 + (o * L1 + kh * KH) * PP + p;
                float acc[KH], sb = 0.f;
#pragma unroll
                for (int k = 0; k < KH; ++k) acc[k] = 0.f;
#pragma unroll
                for (int t = 0; t < TW; ++t) {
                    const float g = gr[t * PP];
                    sb += g;
#pragma unroll
                    for (int k = 0; k < KH; ++k) acc[k] = fmaf(g, dr[(t + k) * PP], acc[k]);
                }
#pragma unroll
                for (int k = 0; k < KH; ++k) accD[ii][k] += (double)acc[k];
                if (o == 0 && kh == 0) accb2[ii] += (double)sb;
            }
        }
        __syncthreads();
        // E. w1 / b1 partials: item (o, ci, tap half); b1 rides on (o, 0, 0)
#pragma unroll
        for (int ii = 0; ii < NEI; ++ii) {
            const int j = slot + ii * NSLOT;
            if (j < NE) {
                const int o = j / (2 * NC), ci = (j / 2) % NC, kh = j & 1;
                const float* gr = gz + (o * GZW + GZ0) * PP + p;
                const float* xr = xs + (ci * L + kh * KAH) * PP + p;
                float acc[KAH], sb = 0.f;
#pragma unroll
                for (int k = 0; k < KAH; ++k) acc[k] = 0.f;
#pragma unroll 8
                for (int t1 = 0; t1 < L1; ++t1) {
                    const float g = gr[t1 * PP];
                    sb += g;
#pragma unroll
                        for (int k = 0; k < KAH; ++k)  // (KA odd: the second half's tap KA is unused; it reads
                        acc[k] = fmaf(g, xr[(2 * t1 + k) * PP], acc[k]);  // at most one row past xs, into d1)
                }
#pragma unroll
                for (int k = 0; k < KAH; ++k) accE[ii][k] += (double)acc[k];
                if (ci == 0 && kh == 0) accb1[ii] += (double)sb;
            }
        }
        // F. gpre[ci][2m + par] = sum_o sum_q gz[o][m - q] w1[o][ci][2q + par]
        for (int j = slot; j < NF; j += NSLOT) {
            const int ci = j / (MR / RM), m0 = (j - ci * (MR / RM)) * RM;
            float acc[RM][2];
#pragma unroll
            for (int r = 0; r < RM; ++r) acc[r][0] = acc[r][1] = 0.f;
#pragma unroll
            for (int o = 0; o < C2; ++o) {
                float gw[RM + QN - 1];  // padded gz index m0 + i  <->  t1 = m0 + i - GZ0
                const float* gr = gz + (o * GZW + m0) * PP + p;
#pragma unroll
                for (int i = 0; i < RM + QN - 1; ++i) gw[i] = gr[i * PP];
                const float* wr = w1s + (o * NC + ci) * KA;
#pragma unroll
                for (int q = 0; q < QN; ++q)
#pragma unroll
                    for (int par = 0; par < 2; ++par) {
                        if (2 * q + par >= KA) continue;
                        const float wk = wr[2 * q + par];
#pragma unroll
                        for (int r = 0; r < RM; ++r) acc[r][par] = fmaf(wk, gw[r - q + QN - 1], acc[r][par]);
                    }
            }
            if (valid) {
                float* gp = gpre + ((size_t)b * NC * L + ci * L) * HW + pix;
#pragma unroll
                for (int r = 0; r < RM; ++r)
#pragma unroll
                    for (int par = 0; par < 2; ++par) {
                        const int jo = 2 * (m0 + r) + par;
                        if (jo < L) gp[(size_t)jo * HW] = acc[r][par];
                    }
            }
        }
    }
    // one ws row per block: each parameter has exactly one owning slot; sum its PX lanes
    float* row = ws + (size_t)blockIdx.x * NPAR;
    constexpr int OB1 = NW1, OW2 = OB1 + C2, OB2 = OW2 + NW2;
    auto lane_sum = [](double v) {
#pragma unroll
        for (int o = PX / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        return v;
    };
#pragma unroll
    for (int ii = 0; ii < NDI; ++ii) {
        const int j = slot + ii * NSLOT;
        if (j < ND) {  // slot-uniform: the PX lanes of the shuffle take the branch together
            const int o2 = j / (2 * C2), o = (j / 2) % C2, kh = j & 1;
#pragma unroll
            for (int k = 0; k < KH; ++k) {
                const double s = lane_sum(accD[ii][k]);
                if (p == 0) row[OW2 + (o2 * C2 + o) * KB + kh * KH + k] = (float)s;
            }
            if (o == 0 && kh == 0) {
                const double s = lane_sum(accb2[ii]);
                if (p == 0) row[OB2 + o2] = (float)s;
            }
        }
    }
#pragma unroll
    for (int ii = 0; ii < NEI; ++ii) {
        const int j = slot + ii * NSLOT;
        if (j < NE) {
            const int o = j / (2 * NC), ci = (j / 2) % NC, kh = j & 1;
#pragma unroll
            for (int k = 0; k < KAH; ++k) {
                const double s = lane_sum(accE[ii][k]);
                if (p == 0 && kh * KAH + k < KA) row[(o * NC + ci) * KA + kh * KAH + k] = (float)s;
            }
            if (ci == 0 && kh == 0) {
                const double s = lane_sum(accb1[ii]);
                if (p == 0) row[OB1 + o] = (float)s;
            }
        }
    }
    // rows past the grid (the ABI sizes ws for one row per 64 pixels) are zero
    for (int r = gridDim.x + blockIdx.x; r < nrows; r += gridDim.x)
        for (int i = tid; i < NPAR; i += 256) ws[(size_t)r * NPAR + i] = 0.f;
}

// D[plane] = sum_hw g*(1-m) * u   (planes (b, c, t); m = spatial-cond mask of sample b or none)
__global__ void plane_dot_kernel(const float* __restrict__ g, const float* __restrict__ u,
                                 const float* __restrict__ mask, int mask_S, int mask_ch, int nct, int HW,
                                 double* __restrict__ D) {
    __shared__ double red[16];
    const int plane = blockIdx.y;
    const int b = plane / nct;
    const float* gp = g + (size_t)plane * HW;
    const float* up = u + (size_t)plane * HW;
    const float* mk = mask ? mask + ((size_t)b * mask_S + mask_ch) * HW : nullptr;
    double s = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += gridDim.x * blockDim.x) {
        float gg = gp[i];
        if (mk) gg = gg - mk[i] * gg;
        s += (double)(gg * up[i]);
    }
    s = nps::block_sum(s, red);
    if (threadIdx.x == 0) atomicAdd(&D[plane], s);
}

// backward of volume_rescale_kernel (activation_wrapper.py:80-105):
//   v = (u / s) * f(s), f = resc(s) * prev;  df/ds = 1 - tanh^2;  out = v - m v
//   gu = g1 f / s + D ((1 - tanh^2) / s - f / s^2),   g1 = g (1 - m),  D = sum_plane g1 u
__global__ void volume_rescale_bwd_kernel(const float* __restrict__ g,
                                          const double* __restrict__ new_tot, const double* __restrict__ prev_tot,
                                          const float* __restrict__ mpdcum, const float* __restrict__ mask,
                                          int mask_S, int mask_ch, const double* __restrict__ D, int nc, int tw,
                                          int HW, float* __restrict__ gu) {
    const int plane = blockIdx.y;
    const int t = plane % tw;
    const int bc = plane / tw;
    const int b = bc / nc;
    const float newt = (float)new_tot[plane];
    const float prev = (float)prev_tot[bc];
    const float mpd = mpdcum[t];
    const float th = tanhf((1.f - newt / prev) * 100.f / mpd);
    const float f = (1.f - th / 100.f * mpd) * prev;
    const float coef = (float)D[plane] * ((1.f - th * th) / newt - f / (newt * newt));
    const float* gp = g + (size_t)plane * HW;
    float* op = gu + (size_t)plane * HW;
    const float* mk = mask ? mask + ((size_t)b * mask_S + mask_ch) * HW : nullptr;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < HW; i += gridDim.x * blockDim.x) {
        float gg = gp[i];
        if (mk) gg = gg - mk[i] * gg;
        op[i] = gg * f / newt + coef;
    }
}

}  // namespace

extern "C" int nps_pack_grid_input(const float* u, const float* pos, const float* cond, const float* sc, float* xin,
                                   float* vb, int B, int CT, int H, int W, int K, int S, int Cp, void* stream) {
    NPS_CHECK_ARG(u && pos && xin && B > 0 && CT > 0 && H > 0 && W > 0 && K >= 0 && S >= 0 && Cp >= CT + 2 + K + S,
                  "pack_grid_input: bad args");
    NPS_CHECK_ARG((K == 0 || cond) && (S == 0 || sc), "pack_grid_input: missing cond/spatial cond");
    const size_t lds = sizeof(float) * Cp * 65;
    NPS_CHECK_ARG(lds <= 64 * 1024, "pack_grid_input: Cp=%d too large", Cp);
    const int HW = H * W;
    pack_grid_kernel<<<dim3((HW + 63) / 64, B), 256, lds, (hipStream_t)stream>>>(u, pos, cond, sc, xin,
                                                                                 (K + S) ? vb : nullptr, CT, HW, K, S,
                                                                                 Cp);
    NPS_CHECK_LAUNCH("pack_grid_input");
    return 0;
}

extern "C" int nps_timeconv_decode(const float* pre, const float* u, const float* w1, const float* b1, const float* w2,
                                   const float* b2, const float* dtcum, const float* mask, int mask_S, int mask_ch,
                                   float* out, int B, int num_c, int tw, int H, int W, int act_tanh, void* stream) {
    NPS_CHECK_ARG(pre && u && w1 && b1 && w2 && b2 && dtcum && out && B > 0 && num_c > 0 && tw > 0 && H > 0 && W > 0,
                  "timeconv_decode: bad args");
    // dec_grid.py:117-124 kernel sizes
    const int ka = (tw + 1) / 2;
    const int kb = (tw + 3) / 4 + 1 + (tw % 4 == 0 ? 1 : 0);
    const int L1 = (3 * tw - ka) / 2 + 1;
    NPS_CHECK_ARG(L1 - kb + 1 == tw, "timeconv_decode: kernel sizes do not reproduce tw=%d", tw);
    const size_t lds = sizeof(float) * 2 * num_c * L1 * 64;
    NPS_CHECK_ARG(lds <= 96 * 1024, "timeconv_decode: num_c=%d too large", num_c);
    const int HW = H * W;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)timeconv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        attr_set = true;
    }
    if (tw == 25 && (num_c == 1 || num_c == 3)) {
        constexpr int PX = 16;
        const size_t lds2 = sizeof(float) * (PX + 1) * num_c * (3 * 25 + 2 * L1);
        hipStream_t st = (hipStream_t)stream;
        if (num_c == 1) {
            static bool set1 = false;
            if (!set1) {
                (void)hipFuncSetAttribute((const void*)timeconv_fast_kernel<1, 25, PX>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                set1 = true;
            }
            timeconv_fast_kernel<1, 25, PX><<<dim3((HW + PX - 1) / PX, B), 256, lds2, st>>>(
                pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, out, HW, act_tanh);
        } else {
            static bool set3 = false;
            if (!set3) {
                (void)hipFuncSetAttribute((const void*)timeconv_fast_kernel<3, 25, PX>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                set3 = true;
            }
            timeconv_fast_kernel<3, 25, PX><<<dim3((HW + PX - 1) / PX, B), 256, lds2, st>>>(
                pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, out, HW, act_tanh);
        }
        NPS_CHECK_LAUNCH("timeconv_decode");
        return 0;
    }
    timeconv_kernel<<<dim3((HW + 63) / 64, B), 256, lds, (hipStream_t)stream>>>(
        pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, out, num_c, tw, HW, ka, kb, L1, act_tanh);
    NPS_CHECK_LAUNCH("timeconv_decode");
    return 0;
}

extern "C" int nps_plane_sums(const float* base, long plane_stride, int plane_size, int nplanes, double* sums,
                              void* stream) {
    NPS_CHECK_ARG(base && sums && plane_size > 0 && nplanes > 0, "plane_sums: bad args");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(sums, 0, sizeof(double) * nplanes, s) != hipSuccess) {
        nps::set_error("plane_sums: memset failed");
        return -2;
    }
    int nb = (plane_size + 256 * 8 - 1) / (256 * 8);
    nb = nb < 1 ? 1 : (nb > 64 ? 64 : nb);
    plane_sums_kernel<<<dim3(nb, nplanes), 256, 0, s>>>(base, plane_stride, plane_size, sums);
    NPS_CHECK_LAUNCH("plane_sums");
    return 0;
}

extern "C" int nps_volume_rescale(float* u, const double* new_tot, const double* prev_tot, const float* mpdcum,
                                  const float* mask, int mask_S, int mask_ch, int B, int num_c, int tw, int H, int W,
                                  void* stream) {
    NPS_CHECK_ARG(u && new_tot && prev_tot && mpdcum && B > 0 && num_c > 0 && tw > 0, "volume_rescale: bad args");
    const int HW = H * W;
    int nb = (HW + 256 * 4 - 1) / (256 * 4);
    nb = nb < 1 ? 1 : (nb > 64 ? 64 : nb);
    volume_rescale_kernel<<<dim3(nb, B * num_c * tw), 256, 0, (hipStream_t)stream>>>(u, new_tot, prev_tot, mpdcum, mask,
                                                                                     mask_S, mask_ch, num_c, tw, HW);
    NPS_CHECK_LAUNCH("volume_rescale");
    return 0;
}

extern "C" int nps_sq_err_sum(const float* a, const float* b, long n, double* out, void* stream) {
    NPS_CHECK_ARG(a && b && out && n > 0, "sq_err_sum: bad args");
    long nb = (n + 256 * 16 - 1) / (256 * 16);
    nb = nb < 1 ? 1 : (nb > 1024 ? 1024 : nb);
    sq_err_kernel<<<(unsigned)nb, 256, 0, (hipStream_t)stream>>>(a, b, n, out);
    NPS_CHECK_LAUNCH("sq_err_sum");
    return 0;
}

extern "C" int nps_nchw_to_nhwc(const float* in, float* out, int B, int C, int H, int W, void* stream) {
    NPS_CHECK_ARG(in && out && B > 0 && C > 0 && H > 0 && W > 0, "nchw_to_nhwc: bad args");
    // in: [B][C][HW] = [B][R=C][Cc=HW] -> out [B][HW][C]
    const int R = C, Cc = H * W;
    transpose_kernel<<<dim3((R + 31) / 32, (Cc + 31) / 32, B), dim3(32, 8), 0, (hipStream_t)stream>>>(in, out, R, Cc);
    NPS_CHECK_LAUNCH("nchw_to_nhwc");
    return 0;
}

extern "C" int nps_nhwc_to_nchw(const float* in, float* out, int B, int C, int H, int W, void* stream) {
    NPS_CHECK_ARG(in && out && B > 0 && C > 0 && H > 0 && W > 0, "nhwc_to_nchw: bad args");
    const int R = H * W, Cc = C;
    transpose_kernel<<<dim3((R + 31) / 32, (Cc + 31) / 32, B), dim3(32, 8), 0, (hipStream_t)stream>>>(in, out, R, Cc);
    NPS_CHECK_LAUNCH("nhwc_to_nchw");
    return 0;
}

namespace {
template <int NC, int TW, int PX>
constexpr size_t tc_bwd_lds() {
    constexpr int L = 3 * TW, KA = (TW + 1) / 2, KB = (TW + 3) / 4 + 1 + (TW % 4 == 0 ? 1 : 0);
    constexpr int L1 = (L - KA) / 2 + 1, C2 = 2 * NC, PP = PX + 1, QN = (KA + 1) / 2, RM = 4;
    constexpr int MR = ((L + 1) / 2 + RM - 1) / RM * RM, GZW = MR + QN - 1, G2W = TW + 2 * (KB - 1);
    return sizeof(float) * ((size_t)(NC * L + C2 * L1 + C2 * GZW + NC * G2W) * PP + C2 * NC * KA + NC * C2 * KB +
                            C2 + NC + TW);
}

// resident blocks of the tw = 25 backward kernel over the whole device (its grid: one pass, no tail)
template <int NC, int PX>
int tc_bwd_blocks() {
    static int n = 0;
    if (n == 0) {
        const void* f = (const void*)timeconv_bwd_fast_kernel<NC, 25, PX>;
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        int per_cu = 0, dev = 0, ncu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 256, tc_bwd_lds<NC, 25, PX>());
        n = std::max(1, per_cu) * std::max(1, ncu);
    }
    return n;
}

// NPS_TC_BWD_GENERIC=1 routes every shape through the one-wave generic kernel (A/B and parity checks)
bool tc_bwd_generic() {
    static const int g = [] {
        const char* e = std::getenv("NPS_TC_BWD_GENERIC");
        return e && e[0] == '1' ? 1 : 0;
    }();
    return g != 0;
}
}  // namespace

extern "C" int nps_timeconv_decode_bwd(const float* pre, const float* u, const float* w1, const float* b1,
                                       const float* w2, const float* b2, const float* dtcum, const float* mask,
                                       int mask_S, int mask_ch, const float* gout, float* gpre, float* ws, int B,
                                       int num_c, int tw, int H, int W, int act_tanh, void* stream) {
    NPS_CHECK_ARG(pre && u && w1 && b1 && w2 && b2 && dtcum && gout && gpre && ws && B > 0 && num_c > 0 && tw > 0 &&
                      H > 0 && W > 0,
                  "timeconv_decode_bwd: bad args");
    const int ka = (tw + 1) / 2;
    const int kb = (tw + 3) / 4 + 1 + (tw % 4 == 0 ? 1 : 0);
    const int L1 = (3 * tw - ka) / 2 + 1;
    NPS_CHECK_ARG(L1 - kb + 1 == tw, "timeconv_decode_bwd: kernel sizes do not reproduce tw=%d", tw);
    const int nparams = 2 * num_c * num_c * ka + 2 * num_c + num_c * 2 * num_c * kb + num_c;
    const size_t lds = sizeof(float) * 64 * (2 * 2 * num_c * L1 + num_c * tw);
    NPS_CHECK_ARG(lds <= 160 * 1024, "timeconv_decode_bwd: num_c=%d tw=%d too large", num_c, tw);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)timeconv_bwd_kernel<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void*)timeconv_bwd_kernel<3, 25>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void*)timeconv_bwd_kernel<1, 25>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    const int HW = H * W;
    const dim3 grid((HW + 63) / 64, B);
    hipStream_t s = (hipStream_t)stream;
    if ((num_c == 3 || num_c == 1) && tw == 25 && !tc_bwd_generic()) {  // the twophase cfgs
        constexpr int PX = 16;
        const int ngroups = B * ((HW + PX - 1) / PX);
        const int nrows = B * ((HW + 63) / 64);
        const int par = num_c == 3 ? tc_bwd_blocks<3, PX>() : tc_bwd_blocks<1, PX>();
        const int G = std::min(std::min(ngroups, nrows), par);
        if (num_c == 3)
            timeconv_bwd_fast_kernel<3, 25, PX><<<G, 256, tc_bwd_lds<3, 25, PX>(), s>>>(
                pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, gout, gpre, ws, HW, ngroups, nrows, act_tanh);
        else
            timeconv_bwd_fast_kernel<1, 25, PX><<<G, 256, tc_bwd_lds<1, 25, PX>(), s>>>(
                pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, gout, gpre, ws, HW, ngroups, nrows, act_tanh);
    } else if (num_c == 3 && tw == 25)
        timeconv_bwd_kernel<3, 25><<<grid, 64, lds, s>>>(pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, gout,
                                                         gpre, ws, num_c, tw, HW, ka, kb, L1, act_tanh, nparams);
    else if (num_c == 1 && tw == 25)
        timeconv_bwd_kernel<1, 25><<<grid, 64, lds, s>>>(pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, gout,
                                                         gpre, ws, num_c, tw, HW, ka, kb, L1, act_tanh, nparams);
    else
        timeconv_bwd_kernel<0, 0><<<grid, 64, lds, s>>>(pre, u, w1, b1, w2, b2, dtcum, mask, mask_S, mask_ch, gout,
                                                        gpre, ws, num_c, tw, HW, ka, kb, L1, act_tanh, nparams);
    NPS_CHECK_LAUNCH("timeconv_decode_bwd");
    return 0;
}

extern "C" int nps_plane_dot(const float* g, const float* u, const float* mask, int mask_S, int mask_ch, int B,
                             int nct, int H, int W, double* D, void* stream) {
    NPS_CHECK_ARG(g && u && D && B > 0 && nct > 0 && H > 0 && W > 0, "plane_dot: bad args");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(D, 0, sizeof(double) * B * nct, s) != hipSuccess) {
        nps::set_error("plane_dot: memset failed");
        return -2;
    }
    const int HW = H * W;
    int nb = (HW + 256 * 8 - 1) / (256 * 8);
    nb = nb < 1 ? 1 : (nb > 64 ? 64 : nb);
    plane_dot_kernel<<<dim3(nb, B * nct), 256, 0, s>>>(g, u, mask, mask_S, mask_ch, nct, HW, D);
    NPS_CHECK_LAUNCH("plane_dot");
    return 0;
}

extern "C" int nps_volume_rescale_bwd(const float* g, const double* new_tot, const double* prev_tot,
                                      const float* mpdcum, const float* mask, int mask_S, int mask_ch,
                                      const double* D, float* gu, int B, int num_c, int tw, int H, int W,
                                      void* stream) {
    NPS_CHECK_ARG(g && new_tot && prev_tot && mpdcum && D && gu && B > 0 && num_c > 0 && tw > 0,
                  "volume_rescale_bwd: bad args");
    const int HW = H * W;
    int nb = (HW + 256 * 4 - 1) / (256 * 4);
    nb = nb < 1 ? 1 : (nb > 64 ? 64 : nb);
    volume_rescale_bwd_kernel<<<dim3(nb, B * num_c * tw), 256, 0, (hipStream_t)stream>>>(
        g, new_tot, prev_tot, mpdcum, mask, mask_S, mask_ch, D, num_c, tw, HW, gu);
    NPS_CHECK_LAUNCH("volume_rescale_bwd");
    return 0;
}
