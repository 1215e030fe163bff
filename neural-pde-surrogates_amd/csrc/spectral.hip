// SpectralConv2d forward for gfx950 (proc_fno.py:257-288): truncated DFT analysis,
// per-mode complex channel mixing, truncated inverse DFT + c2r synthesis.
//
// Only the retained 2*m1 x m2 modes exist on device: the forward W-transform
// keeps m2 of W/2+1 bins, the H-transform keeps R = min(H, 2*m1) rows, so the
// input is read exactly once and nothing of size B*C*H*(W/2+1) is formed.
// Every stage streams NHWC activations with C on consecutive lanes (coalesced)
// and reads twiddles from LDS tables built in-kernel from sincospif of the exact
// integer phase (k*n mod N)/N.
#include "nps_common.hpp"

#include <cstdlib>
#include <type_traits>

namespace {

constexpr int R_CHUNK = 8;     // retained rows per pass in dft_h
constexpr int MAXR = 32;       // max retained rows in idft_h (m1 <= 16)
constexpr int MAXB = 8;        // batch rows held in registers by the mixer per pass
constexpr int WB = 16;         // pixels per batch of independent loads in the W-transforms

// retained row r -> frequency k1 (proc_fno.py:266-269: rows [:m1] and [-m1:])
__device__ __forceinline__ int row_k1(int r, int H, int R, int m1) { return r < m1 ? r : H - R + r; }

// e^{-2 pi i k n / N} = (cos, -sin)
__device__ __forceinline__ float2 twiddle(int k, int n, int N) {
    const int ph = (int)(((long)k * n) % N);
    float s, c;
    sincospif(2.0f * (float)ph / (float)N, &s, &c);
    return make_float2(c, s);  // (cos theta, sin theta), theta = 2 pi k n / N
}

// Activation element types of the spectral passes: fp32, or bf16 stored as its 16 bits (the bf16 3-D path,
// BASELINE config C5: bf16 storage, fp32 arithmetic).
typedef unsigned short bf16_t;
__device__ __forceinline__ float ld_f(float v) { return v; }
__device__ __forceinline__ float ld_f(bf16_t v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ void st_f(float* p, float v) { *p = v; }
__device__ __forceinline__ void st_f(bf16_t* p, float v) { *p = __builtin_bit_cast(bf16_t, (__bf16)v); }

// X1[b][h][k2][c] = sum_w x[b][h][w][c] e^{-2 pi i k2 w / W}
// With c2r_adj != 0 this is the adjoint of the c2r synthesis (backward of idft_w): every bin is scaled
// by `scale` and, except DC / Nyquist, doubled (torch irfft backward: rfft(g)/N, columns 1..W-(W//2+1) x2).
// KC bins per pass (a multiple of 4 >= the retained bins where possible): the twiddle table is laid out
// [w][KC] so one pixel's KC twiddles are KC/2 broadcast ds_read_b128, and bins past m2 carry zero
// twiddles (no per-bin branches in the inner loop).
template <int KC, typename TIn = float>
__global__ void dft_w_kernel(nps_conv2d_t a, int m2, float2* __restrict__ X1, float scale, int c2r_adj) {
    extern __shared__ __attribute__((aligned(16))) float2 tw[];  // [W][KC]
    const int h = blockIdx.x, b = blockIdx.y;
    const int W = a.Win, H = a.Hin, C = a.Cin;
    for (int kb = 0; kb < m2; kb += KC) {
        const int nk = min(KC, m2 - kb);
        __syncthreads();
        for (int i = threadIdx.x; i < KC * W; i += blockDim.x) {
            const int w = i / KC, k = i - (i / KC) * KC;
            tw[i] = k < nk ? twiddle(kb + k, w, W) : make_float2(0.f, 0.f);
        }
        __syncthreads();
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            // locate the source of channel c
            const TIn* base = nullptr;
            int sc = 0, sC = 1;
            int c0 = 0;
            for (int s = 0; s < a.nsrc; ++s) {
                if (c >= c0 && c < c0 + a.src[s].C) {
                    base = reinterpret_cast<const TIn*>(a.src[s].ptr);
                    sc = c - c0;
                    sC = a.src[s].C;
                }
                c0 += a.src[s].C;
            }
            const TIn* row = base + ((size_t)(b * H + h) * W) * sC + sc;
            float re[KC], im[KC];
#pragma unroll
            for (int k = 0; k < KC; ++k) re[k] = im[k] = 0.f;
            // WB independent row loads are issued before their FMAs: one (b, h) row per work-group
            // leaves too few waves per CU to cover HBM latency one load at a time
            auto bins = [&](float v, int w) {
                const f32x4* t4 = reinterpret_cast<const f32x4*>(tw + w * KC);
#pragma unroll
                for (int q = 0; q < KC / 2; ++q) {
                    const f32x4 t = t4[q];  // (cos, sin) of bins 2q, 2q + 1
                    re[2 * q] = fmaf(v, t[0], re[2 * q]);
                    im[2 * q] = fmaf(-v, t[1], im[2 * q]);
                    re[2 * q + 1] = fmaf(v, t[2], re[2 * q + 1]);
                    im[2 * q + 1] = fmaf(-v, t[3], im[2 * q + 1]);
                }
            };
            int w0 = 0;
            for (; w0 + WB <= W; w0 += WB) {
                float v[WB];
#pragma unroll
                for (int j = 0; j < WB; ++j) v[j] = ld_f(row[(size_t)(w0 + j) * sC]);
#pragma unroll
                for (int j = 0; j < WB; ++j) bins(v[j], w0 + j);
            }
            for (; w0 < W; ++w0) bins(ld_f(row[(size_t)w0 * sC]), w0);
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                if (k < nk) {
                    float f = scale;
                    const int kk = kb + k;
                    if (c2r_adj && !((kk == 0) || (2 * kk == W))) f *= 2.f;
                    X1[((size_t)(b * H + h) * m2 + kk) * C + c] = make_float2(re[k] * f, im[k] * f);
                }
            }
        }
    }
}

// The W-pass DFT as an exact-fp32 MFMA GEMM per image row (b, h): X1[k][c] = sum_w T[k][w] x[w][c], M = the 32 rows
// [cos 2 pi k w / W (k < m2) | sin ... at row 16 + k] (zero past m2), N = 32 channels, K = 2 pixels per
// v_mfma_f32_32x32x2_f32.  The VALU kernel above reads its twiddles as LDS broadcasts (6 ds_read_b128 per pixel for
// 24 FMAs per channel), which bound it near 3 TB/s; here each lane reads ONE twiddle float per 2 pixels and reuses it
// for 4 MFMAs.  A wave owns (row, 128-channel group): lane l loads the 16-B channel quad 4 (l % 32) .. +3 of pixel
// w0 + l / 32 (two 512-B runs per load), and element i of the quad is column l % 32 of accumulator block i — block i
// holds channels 4 n + i, a channel permutation undone at the store.  Persistent work-groups build the [W][32] table
// once.  Same exact-fp32 products as the VALU chain (MI355X_MICROARCH: f32-input MFMA is bit-exact fmaf), another
// summation order.  Accumulator lane l, register r: column l % 32, row 8 (r / 4) + 4 (l / 32) + r % 4 — bin k's cos
// row k and sin row 16 + k sit in the same lane (registers r and r + 8).
__global__ __launch_bounds__(256) void dft_w_mfma_kernel(nps_conv2d_t a, int m2, float2* __restrict__ X1, float scale,
                                                         int c2r_adj, int nrows) {
    extern __shared__ __attribute__((aligned(16))) float twm[];  // [W][32]
    const int W = a.Win, H = a.Hin, C = a.Cin;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    for (int i = threadIdx.x; i < W * 32; i += 256) {
        const int w = i >> 5, m = i & 31;
        const int k = m & 15;
        float v = 0.f;
        if (k < m2) {
            const float2 t = twiddle(k, w, W);  // (cos, sin)
            v = m < 16 ? t.x : t.y;
        }
        twm[i] = v;
    }
    __syncthreads();
    const int ng = (C + 127) / 128;
    const int ntask = nrows * ng;
    for (int task = blockIdx.x * 4 + wave; task < ntask; task += gridDim.x * 4) {
        const int row = task / ng, g = task - (task / ng) * ng;
        const int b = row / H, hh = row - (row / H) * H;
        // this lane's channel quad: source pointer at pixel 0 and the source's pixel stride (sources are 4-aligned)
        const int c0 = g * 128 + 4 * l32;
        const float* base = nullptr;
        int sC = 0, lo = 0;
        for (int si = 0; si < a.nsrc; ++si) {
            if (c0 >= lo && c0 < lo + a.src[si].C) {
                sC = a.src[si].C;
                base = a.src[si].ptr + ((size_t)(b * H + hh) * W) * sC + (c0 - lo);
            }
            lo += a.src[si].C;
        }
        const bool ok = c0 < C && base != nullptr;
        f32x16 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
        constexpr int U = 8;  // K-steps (2 pixels each) per batch of independent loads
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        int w0 = 0;
        for (; w0 + 2 * U <= W; w0 += 2 * U) {
            f32x4 xv[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                xv[u] = ok ? *reinterpret_cast<const f32x4*>(base + (size_t)(w0 + 2 * u + h) * sC) : z;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float t = twm[(w0 + 2 * u + h) * 32 + l32];
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(t, xv[u][j], acc[j], 0, 0, 0);
            }
        }
        for (; w0 < W; w0 += 2) {  // (W % 2 == 0: host-checked)
            const float t = twm[(w0 + h) * 32 + l32];
            const f32x4 xq = ok ? *reinterpret_cast<const f32x4*>(base + (size_t)(w0 + h) * sC) : z;
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(t, xq[j], acc[j], 0, 0, 0);
        }
        float2* dst = X1 + (size_t)(b * H + hh) * m2 * C;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = g * 128 + 4 * l32 + j;  // block j, column l32
            if (c >= C) continue;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int k = 8 * (r >> 2) + 4 * h + (r & 3);  // bin of cos row k / sin row 16 + k
                if (k < m2) {
                    float f = scale;
                    if (c2r_adj && !((k == 0) || (2 * k == W))) f *= 2.f;
                    dst[(size_t)k * C + c] = make_float2(acc[j][r] * f, -acc[j][r + 8] * f);
                }
            }
        }
    }
}

// bins per pass for m2 retained bins: the smallest multiple of 4 covering them (16 and chunked above)
inline int kc_for(int m2) { return m2 <= 4 ? 4 : (m2 <= 8 ? 8 : (m2 <= 12 ? 12 : 16)); }

// X2[b][r][k2][c] = sum_h X1[b][h][k2][c] e^{-2 pi i k1(r) h / H}
__global__ void dft_h_kernel(const float2* __restrict__ X1, float2* __restrict__ X2, int H, int R, int m1, int m2,
                             int C) {
    extern __shared__ float2 tw[];  // [R_CHUNK][H]
    const int b = blockIdx.z, r0 = blockIdx.y * R_CHUNK;
    const int nr = min(R_CHUNK, R - r0);
    for (int i = threadIdx.x; i < nr * H; i += blockDim.x) tw[i] = twiddle(row_k1(r0 + i / H, H, R, m1), i % H, H);
    __syncthreads();
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // (k2, c)
    if (idx >= m2 * C) return;
    float2 acc[R_CHUNK];
#pragma unroll
    for (int r = 0; r < R_CHUNK; ++r) acc[r] = make_float2(0.f, 0.f);
    const float2* src = X1 + (size_t)b * H * m2 * C + idx;
    for (int hh = 0; hh < H; ++hh) {
        const float2 v = src[(size_t)hh * m2 * C];
#pragma unroll
        for (int r = 0; r < R_CHUNK; ++r) {
            if (r < nr) {
                const float2 t = tw[r * H + hh];  // e^{-i th} = (c, -s)
                acc[r].x = fmaf(v.x, t.x, fmaf(v.y, t.y, acc[r].x));
                acc[r].y = fmaf(v.y, t.x, fmaf(-v.x, t.y, acc[r].y));
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R_CHUNK; ++r)
        if (r < nr) X2[((size_t)(b * R + r0 + r) * m2) * C + idx] = acc[r];
}

// H-pass of the forward DFT, split over the work-group: X2[b][r][col] = sum_h X1[b][h][col] e^{-2 pi i k1(r) h / H}
// for every column col = (k2, c).  Work-group = 64 columns x 4 h-slices (wave s sums h = s, s + 4, ...: a
// wave reads one 512-B row segment per h, coalesced), all RC retained rows in registers (rows past R have
// zero twiddles), partial sums reduced through LDS.  The single-thread-per-column form left ~2 waves per
// CU each walking H serially (latency-bound, 0.5 TB/s at C3).
template <int RC>
__global__ __launch_bounds__(256) void dft_h2_kernel(const float2* __restrict__ X1, float2* __restrict__ X2, int H,
                                                     int R, int m1, int NC) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];  // tw [H][RC], then partials [4][RC][64]
    const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, hs = tid >> 6;
    const int col = blockIdx.x * 64 + lane;
    for (int i = tid; i < H * RC; i += 256) {
        const int h = i / RC, r = i - (i / RC) * RC;
        sm[i] = r < R ? twiddle(row_k1(r, H, R, m1), h, H) : make_float2(0.f, 0.f);
    }
    __syncthreads();
    float2 acc[RC];
#pragma unroll
    for (int r = 0; r < RC; ++r) acc[r] = make_float2(0.f, 0.f);
    const bool ok = col < NC;
    const float2* src = X1 + (size_t)b * H * NC + (ok ? col : 0);
    constexpr int U = 4;  // independent row loads issued before their FMAs
    for (int h0 = hs; h0 < H; h0 += 4 * U) {
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int h = h0 + 4 * u;
            v[u] = (ok && h < H) ? src[(size_t)h * NC] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int h = min(h0 + 4 * u, H - 1);  // (v is 0 past H)
            const f32x4* t4 = reinterpret_cast<const f32x4*>(sm + h * RC);
#pragma unroll
            for (int q = 0; q < RC / 2; ++q) {
                const f32x4 t = t4[q];  // (c, s) of rows 2q, 2q + 1; e^{-i th} = (c, -s)
                acc[2 * q].x = fmaf(v[u].x, t[0], fmaf(v[u].y, t[1], acc[2 * q].x));
                acc[2 * q].y = fmaf(v[u].y, t[0], fmaf(-v[u].x, t[1], acc[2 * q].y));
                acc[2 * q + 1].x = fmaf(v[u].x, t[2], fmaf(v[u].y, t[3], acc[2 * q + 1].x));
                acc[2 * q + 1].y = fmaf(v[u].y, t[2], fmaf(-v[u].x, t[3], acc[2 * q + 1].y));
            }
        }
    }
    __syncthreads();  // the twiddle table is dead: its LDS takes the partial sums
#pragma unroll
    for (int r = 0; r < RC; ++r) sm[(hs * RC + r) * 64 + lane] = acc[r];
    __syncthreads();
    for (int r = hs; r < R; r += 4) {
        float2 t = sm[r * 64 + lane];
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            const float2 u = sm[(k * RC + r) * 64 + lane];
            t.x += u.x;
            t.y += u.y;
        }
        if (ok) X2[((size_t)b * R + r) * NC + col] = t;
    }
}

// H-pass of the inverse DFT: Z[b][h][col] = sum_r Y[b][r][col] e^{+2 pi i k1(r) h / H}.  Work-group = 64
// columns x IH_HB rows h (4 waves, wave s taking h = h0 + s, + 4, ...), the column's RC retained values in
// registers, the twiddles of the block's rows in LDS; same r order and fma form as the one-thread-per-column
// kernel it replaces (bit-identical results, 16x the work-groups).
constexpr int IH_HB = 64;
template <int RC>
__global__ __launch_bounds__(256) void idft_h2_kernel(const float2* __restrict__ Y, float2* __restrict__ Z, int H,
                                                      int R, int m1, int NC) {
    __shared__ __attribute__((aligned(16))) float2 tw[IH_HB][RC];
    const int b = blockIdx.z, h0 = blockIdx.y * IH_HB, tid = threadIdx.x, lane = tid & 63, hs = tid >> 6;
    const int col = blockIdx.x * 64 + lane;
    const bool ok = col < NC;
    for (int i = tid; i < IH_HB * RC; i += 256) {
        const int hh = i / RC, r = i - (i / RC) * RC;
        tw[hh][r] = (r < R && h0 + hh < H) ? twiddle(row_k1(r, H, R, m1), h0 + hh, H) : make_float2(0.f, 0.f);
    }
    float2 y[RC];
#pragma unroll
    for (int r = 0; r < RC; ++r) y[r] = (ok && r < R) ? Y[((size_t)b * R + r) * NC + col] : make_float2(0.f, 0.f);
    __syncthreads();
    for (int hh = hs; hh < IH_HB && h0 + hh < H; hh += 4) {
        float re = 0.f, im = 0.f;
        const f32x4* t4 = reinterpret_cast<const f32x4*>(&tw[hh][0]);
#pragma unroll
        for (int q = 0; q < RC / 2; ++q) {
            const f32x4 t = t4[q];  // e^{+i th} = (c, s) of rows 2q, 2q + 1
            re = fmaf(y[2 * q].x, t[0], fmaf(-y[2 * q].y, t[1], re));
            im = fmaf(y[2 * q].x, t[1], fmaf(y[2 * q].y, t[0], im));
            re = fmaf(y[2 * q + 1].x, t[2], fmaf(-y[2 * q + 1].y, t[3], re));
            im = fmaf(y[2 * q + 1].x, t[3], fmaf(y[2 * q + 1].y, t[2], im));
        }
        if (ok) Z[((size_t)b * H + h0 + hh) * NC + col] = make_float2(re, im);
    }
}

inline int rc_for(int R) { return R <= 8 ? 8 : (R <= 16 ? 16 : (R <= 24 ? 24 : 32)); }

// wpack[r][k2][i][o] from weights1/weights2 [Cin][Cout][m1][m2] (complex64)
__global__ void spec_pack_kernel(const float2* __restrict__ w1, const float2* __restrict__ w2, float2* __restrict__ wp,
                                 int Cin, int Cout, int H, int R, int m1, int m2) {
    const size_t n = (size_t)R * m2 * Cin * Cout;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int o = i % Cout;
    size_t t = i / Cout;
    const int ci = t % Cin;
    t /= Cin;
    const int k2 = t % m2;
    const int r = (int)(t / m2);
    const int k1 = row_k1(r, H, R, m1);
    // the [-m1:] write happens second and wins where the corners overlap
    if (k1 >= H - m1)
        wp[i] = w2[(((size_t)ci * Cout + o) * m1 + (k1 - (H - m1))) * m2 + k2];
    else
        wp[i] = w1[(((size_t)ci * Cout + o) * m1 + k1) * m2 + k2];
}

// Y[b][mode][o] = sum_i X2[b][mode][i] * wp[mode][i][o]   (complex; mode = (r, k2))
__global__ void mix_kernel(const float2* __restrict__ X2, const float2* __restrict__ wp, float2* __restrict__ Y, int B,
                           int nmodes, int Cin, int Cout) {
    extern __shared__ float2 xs[];  // [MAXB][Cin]
    const int mode = blockIdx.x;
    const int o = blockIdx.y * blockDim.x + threadIdx.x;
    for (int b0 = 0; b0 < B; b0 += MAXB) {
        const int nb = min(MAXB, B - b0);
        __syncthreads();
        for (int i = threadIdx.x; i < nb * Cin; i += blockDim.x)
            xs[i] = X2[((size_t)(b0 + i / Cin) * nmodes + mode) * Cin + i % Cin];
        __syncthreads();
        if (o < Cout) {
            float2 acc[MAXB];
#pragma unroll
            for (int bb = 0; bb < MAXB; ++bb) acc[bb] = make_float2(0.f, 0.f);
            const float2* w = wp + (size_t)mode * Cin * Cout + o;
            for (int i = 0; i < Cin; ++i) {
                const float2 wv = w[(size_t)i * Cout];
#pragma unroll
                for (int bb = 0; bb < MAXB; ++bb) {
                    if (bb < nb) {
                        const float2 xv = xs[bb * Cin + i];
                        acc[bb].x = fmaf(xv.x, wv.x, fmaf(-xv.y, wv.y, acc[bb].x));
                        acc[bb].y = fmaf(xv.x, wv.y, fmaf(xv.y, wv.x, acc[bb].y));
                    }
                }
            }
#pragma unroll
            for (int bb = 0; bb < MAXB; ++bb)
                if (bb < nb) Y[((size_t)(b0 + bb) * nmodes + mode) * Cout + o] = acc[bb];
        }
    }
}

// Y[b][mode][o] = sum_i X2[b][mode][i] * wp[mode][i][o] on the matrix cores (v_mfma_f32_16x16x4_f32: exact
// fp32 products, fp32 accumulation — the per-mode complex GEMM of proc_fno.py:253-255).  The complex product
// is the real GEMM Y'^T = W'^T X'^T with (re, im) interleaved on both sides: output row 2o + p (p = 0 re,
// 1 im), K index 2i + q (q = 0 re, 1 im of X), W'^T[2o+p][2i+q] = Re W if p == q, -Im W if (p, q) = (0, 1),
// +Im W if (1, 0).  So a 16x16x4 MFMA covers 8 output channels x 16 batch rows x 2 input channels.
// Work-group (256 threads) = one mode x 64 output channels; wave w owns channels [16w, 16w + 16) of them
// (two 16x16 tiles); the batch is processed 16 * NBC rows at a time against the same LDS weight chunk, so
// the weights stream from HBM once for any B <= 16 * NBC.  Weight chunks of MIX_IC input channels
// ([i][64 o] complex, fp32 in LDS; WT = float2 for the fp32 path, uint32 = packed bf16 (re, im) for the
// bf16 path) are double-buffered through registers: chunk c + 1 is in flight while chunk c is multiplied.
constexpr int MIX_IC = 32;   // input channels per weight chunk
constexpr int MIX_OC = 64;   // output channels per work-group

__device__ __forceinline__ float2 bf16x2_to_float2(unsigned v) {
    return make_float2(__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u));
}

template <typename WT, int NBC>
__global__ __launch_bounds__(256) void mix_mfma_kernel(const float2* __restrict__ X2, const WT* __restrict__ wp,
                                                       float2* __restrict__ Y, int B, int nmodes, int Cin, int Cout) {
    constexpr int WPT = MIX_IC * MIX_OC * (int)sizeof(WT) / (256 * 16);  // 16-B weight pieces per thread
    static_assert(WPT >= 1 && MIX_IC * MIX_OC * sizeof(WT) % (256 * 16) == 0, "weight chunk split");
    __shared__ float2 Ws[2][MIX_IC][MIX_OC];          // weight chunk, fp32 complex
    __shared__ float2 Xs[MIX_IC][16 * NBC + 1];       // X chunk [i][b] (+1: bank offset between rows)
    const int mode = blockIdx.x;
    const int o0 = blockIdx.y * MIX_OC;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nchunks = (Cin + MIX_IC - 1) / MIX_IC;
    const WT* wmode = wp + (size_t)mode * Cin * Cout;
    // weight piece k of this thread: chunk-local input channel ci, output channel co .. co + 16/sizeof(WT) - 1
    constexpr int PER_ROW = MIX_OC * (int)sizeof(WT) / 16;  // 16-B pieces per chunk row
    f32x4 wr[WPT];
    auto wfetch = [&](int c) {
#pragma unroll
        for (int k = 0; k < WPT; ++k) {
            const int piece = k * 256 + tid;
            const int ci = piece / PER_ROW, cp = piece - ci * PER_ROW;
            const int i = c * MIX_IC + ci;
            const int co = o0 + cp * (16 / (int)sizeof(WT));
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            // Cout % 4 == 0 (host-checked): a piece is either wholly inside [0, Cout) or wholly outside
            wr[k] = (i < Cin && co < Cout) ? *reinterpret_cast<const f32x4*>(wmode + (size_t)i * Cout + co) : z;
        }
    };
    auto wstore = [&](int buf) {
#pragma unroll
        for (int k = 0; k < WPT; ++k) {
            const int piece = k * 256 + tid;
            const int ci = piece / PER_ROW, cp = piece - ci * PER_ROW;
            if constexpr (sizeof(WT) == 8) {
                *reinterpret_cast<f32x4*>(&Ws[buf][ci][cp * 2]) = wr[k];
            } else {  // 4 packed bf16 complex -> fp32 complex
#pragma unroll
                for (int e = 0; e < 4; ++e) Ws[buf][ci][cp * 4 + e] = bf16x2_to_float2(__float_as_uint(wr[k][e]));
            }
        }
    };
    // MFMA lane roles (16x16x4): A row r = lane & 15 -> (o = 2 per-tile pairs: r >> 1, p = r & 1); K index
    // k = lane >> 4 -> (input channel ic = k >> 1 of the step, q = k & 1); B column = batch b = lane & 15
    const int r = lane & 15, p = r & 1, k = lane >> 4, ic = k >> 1, q = k & 1;
    for (int b0 = 0; b0 < B; b0 += 16 * NBC) {
        f32x4 acc[NBC][2];
#pragma unroll
        for (int n = 0; n < NBC; ++n)
#pragma unroll
            for (int t = 0; t < 2; ++t) acc[n][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        wfetch(0);
        for (int c = 0; c < nchunks; ++c) {
            const int buf = c & 1;
            __syncthreads();  // buffer `buf` and Xs are free (their readers passed the previous chunk)
            wstore(buf);
            for (int e = tid; e < MIX_IC * 16 * NBC; e += 256) {  // X chunk: [i][b]
                const int ci = e % MIX_IC, bb = e / MIX_IC;
                const int i = c * MIX_IC + ci, b = b0 + bb;
                Xs[ci][bb] = (i < Cin && b < B) ? X2[((size_t)b * nmodes + mode) * Cin + i] : make_float2(0.f, 0.f);
            }
            if (c + 1 < nchunks) wfetch(c + 1);  // next chunk in flight during this chunk's MFMAs
            __syncthreads();
#pragma unroll 4
            for (int s = 0; s < MIX_IC / 2; ++s) {
                const int ci = 2 * s + ic;
                float a[2];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const float2 w = Ws[buf][ci][wave * 16 + t * 8 + (r >> 1)];
                    a[t] = p == q ? w.x : (p == 0 ? -w.y : w.y);
                }
#pragma unroll
                for (int n = 0; n < NBC; ++n) {
                    const float2 x = Xs[ci][n * 16 + r];
                    const float bv = q ? x.y : x.x;
#pragma unroll
                    for (int t = 0; t < 2; ++t) acc[n][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], bv, acc[n][t], 0, 0, 0);
                }
            }
        }
        // D: column = batch b0 + 16n + (lane & 15); rows (lane >> 4) * 4 + reg = (re, im) of channels
        // 2 (lane >> 4) and 2 (lane >> 4) + 1 of the tile
#pragma unroll
        for (int n = 0; n < NBC; ++n) {
            const int b = b0 + n * 16 + (lane & 15);
            if (b >= B) continue;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int o = o0 + wave * 16 + t * 8 + 2 * (lane >> 4);
                float2* y = Y + ((size_t)b * nmodes + mode) * Cout;
                if (o < Cout) y[o] = make_float2(acc[n][t][0], acc[n][t][1]);
                if (o + 1 < Cout) y[o + 1] = make_float2(acc[n][t][2], acc[n][t][3]);
            }
        }
    }
}

// Z[b][h][k2][o] = sum_r Y[b][r][k2][o] e^{+2 pi i k1(r) h / H}
__global__ void idft_h_kernel(const float2* __restrict__ Y, float2* __restrict__ Z, int H, int R, int m1, int m2,
                              int Cout) {
    extern __shared__ float2 tw[];  // [R][H]
    const int b = blockIdx.z;
    for (int i = threadIdx.x; i < R * H; i += blockDim.x) tw[i] = twiddle(row_k1(i / H, H, R, m1), i % H, H);
    __syncthreads();
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // (k2, o)
    if (idx >= m2 * Cout) return;
    float2 y[MAXR];
#pragma unroll
    for (int r = 0; r < MAXR; ++r) y[r] = (r < R) ? Y[((size_t)(b * R + r) * m2) * Cout + idx] : make_float2(0.f, 0.f);
    for (int hh = 0; hh < H; ++hh) {
        float re = 0.f, im = 0.f;
#pragma unroll
        for (int r = 0; r < MAXR; ++r) {
            if (r < R) {
                const float2 t = tw[r * H + hh];  // e^{+i th} = (c, s)
                re = fmaf(y[r].x, t.x, fmaf(-y[r].y, t.y, re));
                im = fmaf(y[r].x, t.y, fmaf(y[r].y, t.x, im));
            }
        }
        Z[((size_t)(b * H + hh) * m2) * Cout + idx] = make_float2(re, im);
    }
}

// out[b][h][w][o] (=|+=) act( sum_k c_k Re(Z[b][h][k][o] e^{2 pi i k w / W}) / (H W) [+ addend] )
// doubling = 0, scale = 1 is the adjoint of the truncated real-input DFT (backward of dft_w):
// gx[w] = sum_k Re(gX[k] e^{+2 pi i k w / W}).
template <int KC, typename TOut = float>
__global__ void idft_w_kernel(const float2* __restrict__ Z, TOut* __restrict__ out, int H, int W, int m2, int Cout,
                              int accumulate, const TOut* __restrict__ addend, int act, float scale_arg,
                              int doubling, float* __restrict__ out_tag) {
    extern __shared__ __attribute__((aligned(16))) float2 tw[];  // [chunk][W][KC], zero past m2
    const int h = blockIdx.x, b = blockIdx.y;
    const int nch = (m2 + KC - 1) / KC;
    for (int i = threadIdx.x; i < nch * W * KC; i += blockDim.x) {
        const int ch = i / (W * KC), r = i - ch * (W * KC);
        const int w = r / KC, k = ch * KC + (r - (r / KC) * KC);
        tw[i] = k < m2 ? twiddle(k, w, W) : make_float2(0.f, 0.f);
    }
    __syncthreads();
    const float scale = scale_arg;
    float amax = 0.f;  // max |written value| of the final chunk (the output's range tag)
    for (int o = threadIdx.x; o < Cout; o += blockDim.x) {
        float zr[KC], zi[KC];
        for (int kb = 0; kb < m2; kb += KC) {
            const int nk = min(KC, m2 - kb);
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                float2 z = make_float2(0.f, 0.f);
                if (k < nk) {
                    const int kk = kb + k;
                    z = Z[((size_t)(b * H + h) * m2 + kk) * Cout + o];
                    // one-sided c2r: DC and (even W) Nyquist count once, with Im discarded
                    const bool self_conj = (kk == 0) || (2 * kk == W);
                    const float cm = (self_conj || !doubling) ? 1.f : 2.f;
                    z.x *= cm;
                    z.y = self_conj ? 0.f : z.y * cm;
                }
                zr[k] = z.x;
                zi[k] = z.y;
            }
            const float2* twc = tw + (size_t)(kb / KC) * W * KC;
            // the read-modify-write stream of out / addend is batched WB pixels at a time (loads first)
            const bool last_chunk = kb + KC >= m2;
            const bool rd_out = kb > 0 || accumulate;
            const bool rd_add = last_chunk && addend != nullptr;
            const size_t rowo = (size_t)(b * H + h) * W;
            auto pixel = [&](int w, float prev, float add) {
                const f32x4* t4 = reinterpret_cast<const f32x4*>(twc + w * KC);
                float v = 0.f;
#pragma unroll
                for (int q = 0; q < KC / 2; ++q) {
                    const f32x4 t = t4[q];  // (cos, sin) of bins 2q, 2q + 1 (zero past m2)
                    v = fmaf(zr[2 * q], t[0], fmaf(-zi[2 * q], t[1], v));
                    v = fmaf(zr[2 * q + 1], t[2], fmaf(-zi[2 * q + 1], t[3], v));
                }
                // same float order as the unbatched form: v*scale (+ out) (+ addend), GELU
                v = kb == 0 ? (accumulate ? v * scale + prev : v * scale) : prev + v * scale;
                if (last_chunk) {
                    if (addend) v += add;
                    if (act == 1) v = nps::gelu_erf(v);
                    amax = fmaxf(amax, fabsf(v));
                }
                st_f(out + (rowo + w) * Cout + o, v);
            };
            int w0 = 0;
            for (; w0 + WB <= W; w0 += WB) {
                float prev[WB], add[WB];
                if (rd_out) {  // uniform branches around straight-line batches of loads
#pragma unroll
                    for (int j = 0; j < WB; ++j) prev[j] = ld_f(out[(rowo + w0 + j) * Cout + o]);
                } else {
#pragma unroll
                    for (int j = 0; j < WB; ++j) prev[j] = 0.f;
                }
                if (rd_add) {
#pragma unroll
                    for (int j = 0; j < WB; ++j) add[j] = ld_f(addend[(rowo + w0 + j) * Cout + o]);
                } else {
#pragma unroll
                    for (int j = 0; j < WB; ++j) add[j] = 0.f;
                }
#pragma unroll
                for (int j = 0; j < WB; ++j) pixel(w0 + j, prev[j], add[j]);
            }
            for (; w0 < W; ++w0)
                pixel(w0, rd_out ? ld_f(out[(rowo + w0) * Cout + o]) : 0.f,
                      rd_add ? ld_f(addend[(rowo + w0) * Cout + o]) : 0.f);
        }
    }
    nps::tag_publish(out_tag, amax, nps::wave_salt());
}


// Backward of mix_kernel for one mode per block (weights streamed once):
//   gX2[b][mode][i] = sum_o gY[b][mode][o] * conj(wp[mode][i][o])
//   gwp[mode][i][o] = sum_b conj(X2[b][mode][i]) * gY[b][mode][o]
// One wave per input channel row i: lanes sweep o (coalesced), the gX2 sums are wave reductions.
__global__ void mix_bwd_kernel(const float2* __restrict__ X2, const float2* __restrict__ wp,
                               const float2* __restrict__ gY, float2* __restrict__ gX2, float2* __restrict__ gwp,
                               int B, int nmodes, int Cin, int Cout) {
    extern __shared__ float2 gys[];  // [B][Cout]
    const int mode = blockIdx.x;
    for (int i = threadIdx.x; i < B * Cout; i += blockDim.x)
        gys[i] = gY[((size_t)(i / Cout) * nmodes + mode) * Cout + i % Cout];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int i = blockIdx.y * nw + wave; i < Cin; i += gridDim.y * nw) {
        for (int b0 = 0; b0 < B; b0 += MAXB) {
            const int nb = min(MAXB, B - b0);
            float2 xv[MAXB];
#pragma unroll
            for (int bb = 0; bb < MAXB; ++bb)
                xv[bb] = bb < nb ? X2[((size_t)(b0 + bb) * nmodes + mode) * Cin + i] : make_float2(0.f, 0.f);
            float2 gx[MAXB];
#pragma unroll
            for (int bb = 0; bb < MAXB; ++bb) gx[bb] = make_float2(0.f, 0.f);
            for (int o = lane; o < Cout; o += 64) {
                const size_t wi = ((size_t)mode * Cin + i) * Cout + o;
                const float2 w = wp[wi];
                float2 gw = b0 == 0 ? make_float2(0.f, 0.f) : gwp[wi];
#pragma unroll
                for (int bb = 0; bb < MAXB; ++bb) {
                    if (bb < nb) {
                        const float2 g = gys[(b0 + bb) * Cout + o];
                        // g * conj(w)
                        gx[bb].x = fmaf(g.x, w.x, fmaf(g.y, w.y, gx[bb].x));
                        gx[bb].y = fmaf(g.y, w.x, fmaf(-g.x, w.y, gx[bb].y));
                        // conj(x) * g
                        gw.x = fmaf(xv[bb].x, g.x, fmaf(xv[bb].y, g.y, gw.x));
                        gw.y = fmaf(xv[bb].x, g.y, fmaf(-xv[bb].y, g.x, gw.y));
                    }
                }
                gwp[wi] = gw;
            }
#pragma unroll
            for (int bb = 0; bb < MAXB; ++bb) {
                if (bb < nb) {
                    float re = gx[bb].x, im = gx[bb].y;
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) {
                        re += __shfl_xor(re, off, 64);
                        im += __shfl_xor(im, off, 64);
                    }
                    if (lane == 0) gX2[((size_t)(b0 + bb) * nmodes + mode) * Cin + i] = make_float2(re, im);
                }
            }
        }
    }
}

// The same backward on the matrix cores (v_mfma_f32_16x16x4f32, exact fp32, complex as interleaved real
// rows / columns as in mix_mfma_kernel), for B <= 16 * NBC.  Work-group = one mode x 64 input channels
// (wave w: channels [16w, +16), two 16-row tiles of 8 complex channels); the output channels are walked
// in chunks of 32 with the chunk's weights [64 i][32 o] and gY [32 o][B] in LDS (weights double-buffered
// through registers), and each chunk does both products:
//   gX2[b][i]  += sum_o conj(W[i][o]) gY[b][o]      A = conj(W) [(i,p)][(o,q)], B = gY [(o,q)][b]
//   gW[i][o]    = sum_b conj(X2[b][i]) gY[b][o]     A = conj(X2) [(i,p)][(b,q)] (registers), B = gY [(b,q)][o]
// so the weights stream from HBM once and the weight gradient is written once.
constexpr int MIXB_OC = 32;  // output channels per chunk
template <int NBC>
__global__ __launch_bounds__(256) void mix_bwd_mfma_kernel(const float2* __restrict__ X2, const float2* __restrict__ wp,
                                                           const float2* __restrict__ gY, float2* __restrict__ gX2,
                                                           float2* __restrict__ gwp, int B, int nmodes, int Cin,
                                                           int Cout) {
    constexpr int NB = 16 * NBC;          // batch columns
    constexpr int WPT = 64 * MIXB_OC * 8 / (256 * 16);  // 16-B weight pieces per thread per chunk (4)
    __shared__ float2 Ws[2][64][MIXB_OC + 1];  // [i][o] (+1: bank offset between rows)
    __shared__ float2 Gs[MIXB_OC][NB + 1];     // [o][b]
    const int mode = blockIdx.x;
    const int i0 = blockIdx.y * 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nchunks = (Cout + MIXB_OC - 1) / MIXB_OC;
    const float2* wmode = wp + (size_t)mode * Cin * Cout;
    f32x4 wr[WPT];
    auto wfetch = [&](int c) {
#pragma unroll
        for (int k = 0; k < WPT; ++k) {
            const int piece = k * 256 + tid;
            const int row = piece / (MIXB_OC / 2), cp = piece - row * (MIXB_OC / 2);
            const int i = i0 + row, o = c * MIXB_OC + 2 * cp;
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            // Cout % 4 == 0 (host-checked): a 2-channel piece is wholly inside [0, Cout) or wholly outside
            wr[k] = (i < Cin && o < Cout) ? *reinterpret_cast<const f32x4*>(wmode + (size_t)i * Cout + o) : z;
        }
    };
    auto wstore = [&](int buf) {
#pragma unroll
        for (int k = 0; k < WPT; ++k) {
            const int piece = k * 256 + tid;
            const int row = piece / (MIXB_OC / 2), cp = piece - row * (MIXB_OC / 2);
            Ws[buf][row][2 * cp] = make_float2(wr[k][0], wr[k][1]);
            Ws[buf][row][2 * cp + 1] = make_float2(wr[k][2], wr[k][3]);
        }
    };
    // lane roles (16x16x4): row r = lane & 15 -> (complex row r >> 1 of the tile, p = r & 1); k = lane >> 4
    // -> (pair member k >> 1, q = k & 1)
    const int r = lane & 15, p = r & 1, k = lane >> 4, kh = k >> 1, q = k & 1;
    // conj(X2) A fragments of this wave's rows, one per K step of 2 batch entries
    float xa[2][NB / 2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int i = i0 + wave * 16 + t * 8 + (r >> 1);
#pragma unroll
        for (int kk = 0; kk < NB / 2; ++kk) {
            const int b = 2 * kk + kh;
            const float2 x = (i < Cin && b < B) ? X2[((size_t)b * nmodes + mode) * Cin + i] : make_float2(0.f, 0.f);
            xa[t][kk] = p == q ? x.x : (p == 0 ? x.y : -x.y);
        }
    }
    f32x4 gx[NBC][2];
#pragma unroll
    for (int n = 0; n < NBC; ++n)
#pragma unroll
        for (int t = 0; t < 2; ++t) gx[n][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nks = (B + 1) / 2;  // K steps of the weight-gradient product
    wfetch(0);
    for (int c = 0; c < nchunks; ++c) {
        const int buf = c & 1;
        __syncthreads();  // buffer `buf` and Gs are free
        wstore(buf);
        for (int e = tid; e < MIXB_OC * NB; e += 256) {  // gY chunk: [o][b]
            const int oc = e % MIXB_OC, b = e / MIXB_OC;
            const int o = c * MIXB_OC + oc;
            Gs[oc][b] = (o < Cout && b < B) ? gY[((size_t)b * nmodes + mode) * Cout + o] : make_float2(0.f, 0.f);
        }
        if (c + 1 < nchunks) wfetch(c + 1);
        __syncthreads();
        // gX2: K = this chunk's 32 output channels, 2 per step
#pragma unroll 4
        for (int s2 = 0; s2 < MIXB_OC / 2; ++s2) {
            const int oc = 2 * s2 + kh;
            float a[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const float2 w = Ws[buf][wave * 16 + t * 8 + (r >> 1)][oc];
                a[t] = p == q ? w.x : (p == 0 ? w.y : -w.y);  // conj(W)
            }
#pragma unroll
            for (int n = 0; n < NBC; ++n) {
                const float2 g = Gs[oc][n * 16 + r];
                const float bv = q ? g.y : g.x;
#pragma unroll
                for (int t = 0; t < 2; ++t) gx[n][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], bv, gx[n][t], 0, 0, 0);
            }
        }
        // gW for this chunk: 2 row tiles x 2 column tiles of 16 output channels, K = batch (2 per step)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
            f32x4 gw[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            for (int kk = 0; kk < nks; ++kk) {
                const float2 g = Gs[cc * 16 + r][2 * kk + kh];
                const float bv = q ? g.y : g.x;
#pragma unroll
                for (int t = 0; t < 2; ++t) gw[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[t][kk], bv, gw[t], 0, 0, 0);
            }
            // D: column = output channel (lane & 15); rows (lane >> 4) * 4 + reg = (re, im) of complex rows
            // 2 (lane >> 4) and 2 (lane >> 4) + 1 of the tile
            const int o = c * MIXB_OC + cc * 16 + (lane & 15);
            if (o < Cout) {
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int i = i0 + wave * 16 + t * 8 + 2 * (lane >> 4);
                    if (i < Cin) gwp[((size_t)mode * Cin + i) * Cout + o] = make_float2(gw[t][0], gw[t][1]);
                    if (i + 1 < Cin) gwp[((size_t)mode * Cin + i + 1) * Cout + o] = make_float2(gw[t][2], gw[t][3]);
                }
            }
        }
    }
    // gX2: D column = batch 16n + (lane & 15); rows = (re, im) of complex rows 2 (lane >> 4) + {0, 1}
#pragma unroll
    for (int n = 0; n < NBC; ++n) {
        const int b = n * 16 + (lane & 15);
        if (b >= B) continue;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int i = i0 + wave * 16 + t * 8 + 2 * (lane >> 4);
            float2* g = gX2 + ((size_t)b * nmodes + mode) * Cin;
            if (i < Cin) g[i] = make_float2(gx[n][t][0], gx[n][t][1]);
            if (i + 1 < Cin) g[i + 1] = make_float2(gx[n][t][2], gx[n][t][3]);
        }
    }
}

// gw1/gw2 [Cin][Cout][m1][m2] from gwp[r][k2][i][o] (adjoint of spec_pack_kernel: a weights1 row that
// the weights2 corner overwrites in the forward gets zero gradient)
__global__ void spec_unpack_grad_kernel(const float2* __restrict__ gwp, float2* __restrict__ gw1,
                                        float2* __restrict__ gw2, int Cin, int Cout, int H, int R, int m1, int m2) {
    const size_t n = (size_t)Cin * Cout * m1 * m2;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int k2 = idx % m2;
    size_t t = idx / m2;
    const int j = t % m1;
    t /= m1;
    const int o = t % Cout;
    const int ci = (int)(t / Cout);
    auto row_of = [&](int k1) { return k1 < m1 ? k1 : k1 - (H - R); };
    // weights1 row j -> frequency k1 = j, unless the [-m1:] corner covers it
    float2 g1 = make_float2(0.f, 0.f);
    if (j < H - m1) g1 = gwp[(((size_t)row_of(j) * m2 + k2) * Cin + ci) * Cout + o];
    gw1[idx] = g1;
    const int k1b = H - m1 + j;
    gw2[idx] = gwp[(((size_t)row_of(k1b) * m2 + k2) * Cin + ci) * Cout + o];
}


size_t dft_w_lds(int m2, int W) { return sizeof(float2) * kc_for(m2) * W; }
size_t idft_w_lds(int m2, int W) {
    const int kc = kc_for(m2);
    return sizeof(float2) * ((m2 + kc - 1) / kc) * kc * W;
}

template <typename TIn = float>
void launch_dft_w(dim3 grid, int bs, size_t lds, hipStream_t s, const nps_conv2d_t& a, int m2, float2* X1, float scale,
                  int c2r_adj) {
    static int mfma = -1;  // dev knob NPS_DFTW_MFMA=0: the VALU W-pass
    if (mfma < 0) {
        const char* e = getenv("NPS_DFTW_MFMA");
        mfma = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    bool quads = true;  // every source 4-channel aligned: a lane's 16-B quad lies in one source
    for (int i = 0; i < a.nsrc; ++i) quads = quads && (a.src[i].C & 3) == 0;
    if (std::is_same<TIn, float>::value && mfma && quads && m2 <= 16 && (a.Win & 1) == 0 &&
        a.Win * 32 * 4 <= 64 * 1024) {
        static int ncu = 0;
        if (ncu == 0) {
            int dev = 0, n = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
                n = 256;
            ncu = n;
        }
        const int nrows = (int)(grid.x * grid.y);  // (H, B) rows
        const long tasks = (long)nrows * ((a.Cin + 127) / 128);
        const int g = (int)((tasks + 3) / 4 < 2 * ncu ? (tasks + 3) / 4 : 2 * ncu);  // persistent, every WG resident
        dft_w_mfma_kernel<<<g, 256, (size_t)a.Win * 32 * 4, s>>>(a, m2, X1, scale, c2r_adj, nrows);
        return;
    }
    switch (kc_for(m2)) {
        case 4: dft_w_kernel<4, TIn><<<grid, bs, lds, s>>>(a, m2, X1, scale, c2r_adj); break;
        case 8: dft_w_kernel<8, TIn><<<grid, bs, lds, s>>>(a, m2, X1, scale, c2r_adj); break;
        case 12: dft_w_kernel<12, TIn><<<grid, bs, lds, s>>>(a, m2, X1, scale, c2r_adj); break;
        default: dft_w_kernel<16, TIn><<<grid, bs, lds, s>>>(a, m2, X1, scale, c2r_adj); break;
    }
}

template <int KC, typename TOut>
void launch_idft_w_kc(dim3 grid, int bs, size_t lds, hipStream_t s, const float2* Z, TOut* out, int H, int W, int m2,
                      int C, int accumulate, const TOut* addend, int act, float scale, int doubling, float* tag) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)idft_w_kernel<KC, TOut>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  96 * 1024);
        attr_set = true;
    }
    idft_w_kernel<KC, TOut><<<grid, bs, lds, s>>>(Z, out, H, W, m2, C, accumulate, addend, act, scale, doubling, tag);
}

template <typename TOut = float>
void launch_idft_w(dim3 grid, int bs, size_t lds, hipStream_t s, const float2* Z, TOut* out, int H, int W, int m2,
                   int C, int accumulate, const TOut* addend, int act, float scale, int doubling,
                   float* tag = nullptr) {
    switch (kc_for(m2)) {
        case 4: launch_idft_w_kc<4, TOut>(grid, bs, lds, s, Z, out, H, W, m2, C, accumulate, addend, act, scale, doubling, tag); break;
        case 8: launch_idft_w_kc<8, TOut>(grid, bs, lds, s, Z, out, H, W, m2, C, accumulate, addend, act, scale, doubling, tag); break;
        case 12: launch_idft_w_kc<12, TOut>(grid, bs, lds, s, Z, out, H, W, m2, C, accumulate, addend, act, scale, doubling, tag); break;
        default: launch_idft_w_kc<16, TOut>(grid, bs, lds, s, Z, out, H, W, m2, C, accumulate, addend, act, scale, doubling, tag); break;
    }
}

}  // namespace

extern "C" int nps_spectral_dft_w(const nps_src_t* src, int nsrc, int B, int H, int W, int C, int m2, float* X1,
                                  void* stream) {
    NPS_CHECK_ARG(src && nsrc >= 1 && nsrc <= NPS_MAX_SRC && X1 && B > 0 && H > 0 && W > 0 && m2 > 0 &&
                      m2 <= W / 2 + 1,
                  "spectral_dft_w: bad args (m2=%d W=%d)", m2, W);
    nps_conv2d_t a = {};
    a.nsrc = nsrc;
    int cs = 0;
    for (int i = 0; i < nsrc; ++i) {
        NPS_CHECK_ARG(src[i].H == H && src[i].W == W && src[i].off_y == 0 && src[i].off_x == 0,
                      "spectral_dft_w: sources must cover the frame");
        a.src[i] = src[i];
        cs += src[i].C;
    }
    NPS_CHECK_ARG(cs == C, "spectral_dft_w: channel mismatch");
    a.Hin = H;
    a.Win = W;
    a.Cin = C;
    const size_t lds = dft_w_lds(m2, W);
    NPS_CHECK_ARG(lds <= 64 * 1024, "spectral_dft_w: W=%d too large", W);
    const int bs = C >= 256 ? 256 : ((C + 63) / 64) * 64;
    launch_dft_w(dim3(H, B), bs, lds, (hipStream_t)stream, a, m2, reinterpret_cast<float2*>(X1), 1.f, 0);
    NPS_CHECK_LAUNCH("spectral_dft_w");
    return 0;
}

extern "C" int nps_spectral_dft_h(const float* X1, float* X2, int B, int H, int m1, int m2, int C, void* stream) {
    NPS_CHECK_ARG(X1 && X2 && B > 0 && H > 0 && m1 > 0 && m1 <= H && m2 > 0 && C > 0, "spectral_dft_h: bad args");
    const int R = H < 2 * m1 ? H : 2 * m1;
    hipStream_t s = (hipStream_t)stream;
    const int RC = rc_for(R);
    const size_t lds2 = sizeof(float2) * RC * (H > 256 ? H : 256);  // max(twiddles, 4 x RC x 64 partials)
    if (R <= 32 && lds2 <= 96 * 1024) {
        const int NC = m2 * C;
        const dim3 grid((NC + 63) / 64, B);
        const auto* x = reinterpret_cast<const float2*>(X1);
        auto* y = reinterpret_cast<float2*>(X2);
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)dft_h2_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
            (void)hipFuncSetAttribute((const void*)dft_h2_kernel<24>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
            attr = true;
        }
        switch (RC) {
            case 8: dft_h2_kernel<8><<<grid, 256, lds2, s>>>(x, y, H, R, m1, NC); break;
            case 16: dft_h2_kernel<16><<<grid, 256, lds2, s>>>(x, y, H, R, m1, NC); break;
            case 24: dft_h2_kernel<24><<<grid, 256, lds2, s>>>(x, y, H, R, m1, NC); break;
            default: dft_h2_kernel<32><<<grid, 256, lds2, s>>>(x, y, H, R, m1, NC); break;
        }
        NPS_CHECK_LAUNCH("spectral_dft_h");
        return 0;
    }
    const size_t lds = sizeof(float2) * R_CHUNK * H;
    NPS_CHECK_ARG(lds <= 64 * 1024, "spectral_dft_h: H=%d too large", H);
    dim3 grid((m2 * C + 255) / 256, (R + R_CHUNK - 1) / R_CHUNK, B);
    dft_h_kernel<<<grid, 256, lds, s>>>(reinterpret_cast<const float2*>(X1), reinterpret_cast<float2*>(X2), H, R, m1,
                                        m2, C);
    NPS_CHECK_LAUNCH("spectral_dft_h");
    return 0;
}

extern "C" int nps_spectral_pack_weights(const float* w1, const float* w2, float* wpack, int Cin, int Cout, int H,
                                         int m1, int m2, void* stream) {
    NPS_CHECK_ARG(w1 && w2 && wpack && Cin > 0 && Cout > 0 && m1 > 0 && m1 <= H && m2 > 0,
                  "spectral_pack_weights: bad args");
    const int R = H < 2 * m1 ? H : 2 * m1;
    const size_t n = (size_t)R * m2 * Cin * Cout;
    spec_pack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        reinterpret_cast<const float2*>(w1), reinterpret_cast<const float2*>(w2), reinterpret_cast<float2*>(wpack),
        Cin, Cout, H, R, m1, m2);
    NPS_CHECK_LAUNCH("spectral_pack_weights");
    return 0;
}

extern "C" int nps_spectral_mix(const float* X2, const float* wpack, float* Y, int B, int R, int m2, int Cin, int Cout,
                                void* stream) {
    NPS_CHECK_ARG(X2 && wpack && Y && B > 0 && R > 0 && m2 > 0 && Cin > 0 && Cout > 0, "spectral_mix: bad args");
    hipStream_t s = (hipStream_t)stream;
    static int use_valu = -1;  // dev knob NPS_MIX_VALU=1: the scalar-FMA mixer (A/B reference)
    if (use_valu < 0) {
        const char* e = getenv("NPS_MIX_VALU");
        use_valu = (e != nullptr && e[0] == '1') ? 1 : 0;
    }
    const int nmodes = R * m2;
    if (!use_valu && (Cout & 3) == 0) {
        const dim3 grid(nmodes, (Cout + MIX_OC - 1) / MIX_OC);
        const auto* x = reinterpret_cast<const float2*>(X2);
        const auto* w = reinterpret_cast<const float2*>(wpack);
        auto* y = reinterpret_cast<float2*>(Y);
        if (B <= 16)
            mix_mfma_kernel<float2, 1><<<grid, 256, 0, s>>>(x, w, y, B, nmodes, Cin, Cout);
        else
            mix_mfma_kernel<float2, 2><<<grid, 256, 0, s>>>(x, w, y, B, nmodes, Cin, Cout);
        NPS_CHECK_LAUNCH("spectral_mix (MFMA)");
        return 0;
    }
    const size_t lds = sizeof(float2) * MAXB * Cin;
    NPS_CHECK_ARG(lds <= 64 * 1024, "spectral_mix: Cin=%d too large", Cin);
    const int bs = Cout >= 256 ? 256 : ((Cout + 63) / 64) * 64;
    dim3 grid(nmodes, (Cout + bs - 1) / bs);
    mix_kernel<<<grid, bs, lds, s>>>(reinterpret_cast<const float2*>(X2), reinterpret_cast<const float2*>(wpack),
                                     reinterpret_cast<float2*>(Y), B, nmodes, Cin, Cout);
    NPS_CHECK_LAUNCH("spectral_mix");
    return 0;
}

extern "C" int nps_spectral_idft_h(const float* Y, float* Z, int B, int H, int m1, int m2, int Cout, void* stream) {
    NPS_CHECK_ARG(Y && Z && B > 0 && H > 0 && m1 > 0 && m1 <= H && m2 > 0 && Cout > 0, "spectral_idft_h: bad args");
    const int R = H < 2 * m1 ? H : 2 * m1;
    NPS_CHECK_ARG(R <= MAXR, "spectral_idft_h: %d retained rows > %d", R, MAXR);
    {
        const int NC = m2 * Cout;
        const dim3 g2((NC + 63) / 64, (H + IH_HB - 1) / IH_HB, B);
        hipStream_t s = (hipStream_t)stream;
        const auto* y = reinterpret_cast<const float2*>(Y);
        auto* z = reinterpret_cast<float2*>(Z);
        switch (rc_for(R)) {
            case 8: idft_h2_kernel<8><<<g2, 256, 0, s>>>(y, z, H, R, m1, NC); break;
            case 16: idft_h2_kernel<16><<<g2, 256, 0, s>>>(y, z, H, R, m1, NC); break;
            case 24: idft_h2_kernel<24><<<g2, 256, 0, s>>>(y, z, H, R, m1, NC); break;
            default: idft_h2_kernel<32><<<g2, 256, 0, s>>>(y, z, H, R, m1, NC); break;
        }
        NPS_CHECK_LAUNCH("spectral_idft_h");
        return 0;
    }
    const size_t lds = sizeof(float2) * R * H;
    NPS_CHECK_ARG(lds <= 96 * 1024, "spectral_idft_h: H=%d too large", H);
    dim3 grid((m2 * Cout + 255) / 256, 1, B);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)idft_h_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        attr_set = true;
    }
    idft_h_kernel<<<grid, 256, lds, (hipStream_t)stream>>>(reinterpret_cast<const float2*>(Y),
                                                           reinterpret_cast<float2*>(Z), H, R, m1, m2, Cout);
    NPS_CHECK_LAUNCH("spectral_idft_h");
    return 0;
}

extern "C" int nps_spectral_idft_w(const float* Z, float* out, int B, int H, int W, int m2, int Cout, int accumulate,
                                   const float* addend, int act, float* out_tag, void* stream) {
    NPS_CHECK_ARG(Z && out && B > 0 && H > 0 && W > 0 && m2 > 0 && m2 <= W / 2 + 1 && Cout > 0,
                  "spectral_idft_w: bad args");
    const size_t lds = idft_w_lds(m2, W);
    NPS_CHECK_ARG(lds <= 96 * 1024, "spectral_idft_w: m2*W too large");
    const int bs = Cout >= 256 ? 256 : ((Cout + 63) / 64) * 64;
    launch_idft_w(dim3(H, B), bs, lds, (hipStream_t)stream, reinterpret_cast<const float2*>(Z), out, H, W, m2, Cout,
                  accumulate, addend, act, 1.0f / ((float)H * (float)W), 1, out_tag);
    NPS_CHECK_LAUNCH("spectral_idft_w");
    return 0;
}

// ---- bf16 storage variants (BASELINE config C5: 3-D rFFT spectral conv in bf16) ------------------------
// Same transforms with bf16 activations in HBM (read / written as bf16, every sum in fp32) and the packed
// weights as bf16 complex (re, im) pairs, so the dominant HBM streams — activations and, at small batch,
// the per-mode weights — move half the bytes.
extern "C" int nps_spectral_dft_w_bf16(const nps_src_t* src, int nsrc, int B, int H, int W, int C, int m2, float* X1,
                                       void* stream) {
    NPS_CHECK_ARG(src && nsrc >= 1 && nsrc <= NPS_MAX_SRC && X1 && B > 0 && H > 0 && W > 0 && m2 > 0 &&
                      m2 <= W / 2 + 1,
                  "spectral_dft_w_bf16: bad args (m2=%d W=%d)", m2, W);
    nps_conv2d_t a = {};
    a.nsrc = nsrc;
    int cs = 0;
    for (int i = 0; i < nsrc; ++i) {
        NPS_CHECK_ARG(src[i].H == H && src[i].W == W && src[i].off_y == 0 && src[i].off_x == 0,
                      "spectral_dft_w_bf16: sources must cover the frame");
        a.src[i] = src[i];
        cs += src[i].C;
    }
    NPS_CHECK_ARG(cs == C, "spectral_dft_w_bf16: channel mismatch");
    a.Hin = H;
    a.Win = W;
    a.Cin = C;
    const size_t lds = dft_w_lds(m2, W);
    NPS_CHECK_ARG(lds <= 64 * 1024, "spectral_dft_w_bf16: W=%d too large", W);
    const int bs = C >= 256 ? 256 : ((C + 63) / 64) * 64;
    launch_dft_w<bf16_t>(dim3(H, B), bs, lds, (hipStream_t)stream, a, m2, reinterpret_cast<float2*>(X1), 1.f, 0);
    NPS_CHECK_LAUNCH("spectral_dft_w_bf16");
    return 0;
}

extern "C" int nps_spectral_idft_w_bf16(const float* Z, void* out, int B, int H, int W, int m2, int Cout,
                                        int accumulate, const void* addend, int act, void* stream) {
    NPS_CHECK_ARG(Z && out && B > 0 && H > 0 && W > 0 && m2 > 0 && m2 <= W / 2 + 1 && Cout > 0,
                  "spectral_idft_w_bf16: bad args");
    const size_t lds = idft_w_lds(m2, W);
    NPS_CHECK_ARG(lds <= 96 * 1024, "spectral_idft_w_bf16: m2*W too large");
    const int bs = Cout >= 256 ? 256 : ((Cout + 63) / 64) * 64;
    launch_idft_w<bf16_t>(dim3(H, B), bs, lds, (hipStream_t)stream, reinterpret_cast<const float2*>(Z),
                          reinterpret_cast<bf16_t*>(out), H, W, m2, Cout, accumulate,
                          reinterpret_cast<const bf16_t*>(addend), act, 1.0f / ((float)H * (float)W), 1);
    NPS_CHECK_LAUNCH("spectral_idft_w_bf16");
    return 0;
}

extern "C" int nps_spectral_mix_bf16(const float* X2, const void* wpack, float* Y, int B, int R, int m2, int Cin,
                                     int Cout, void* stream) {
    NPS_CHECK_ARG(X2 && wpack && Y && B > 0 && R > 0 && m2 > 0 && Cin > 0 && Cout > 0 && (Cout & 3) == 0,
                  "spectral_mix_bf16: bad args (Cout %% 4 == 0 required)");
    const int nmodes = R * m2;
    const dim3 grid(nmodes, (Cout + MIX_OC - 1) / MIX_OC);
    const auto* x = reinterpret_cast<const float2*>(X2);
    const auto* w = reinterpret_cast<const unsigned*>(wpack);
    auto* y = reinterpret_cast<float2*>(Y);
    if (B <= 16)
        mix_mfma_kernel<unsigned, 1><<<grid, 256, 0, (hipStream_t)stream>>>(x, w, y, B, nmodes, Cin, Cout);
    else
        mix_mfma_kernel<unsigned, 2><<<grid, 256, 0, (hipStream_t)stream>>>(x, w, y, B, nmodes, Cin, Cout);
    NPS_CHECK_LAUNCH("spectral_mix_bf16");
    return 0;
}

// ---- SpectralConv2d backward (autograd conventions of torch.fft) ----------------
extern "C" int nps_spectral_idft_w_bwd(const float* gy, float* gZ, int B, int H, int W, int m2, int Cout,
                                       void* stream) {
    NPS_CHECK_ARG(gy && gZ && B > 0 && H > 0 && W > 0 && m2 > 0 && m2 <= W / 2 + 1 && Cout > 0,
                  "spectral_idft_w_bwd: bad args");
    nps_conv2d_t a = {};
    a.nsrc = 1;
    a.src[0].ptr = gy;
    a.src[0].C = Cout;
    a.src[0].H = H;
    a.src[0].W = W;
    a.Hin = H;
    a.Win = W;
    a.Cin = Cout;
    const size_t lds = dft_w_lds(m2, W);
    NPS_CHECK_ARG(lds <= 64 * 1024, "spectral_idft_w_bwd: W=%d too large", W);
    const int bs = Cout >= 256 ? 256 : ((Cout + 63) / 64) * 64;
    launch_dft_w(dim3(H, B), bs, lds, (hipStream_t)stream, a, m2, reinterpret_cast<float2*>(gZ),
                 1.0f / ((float)H * (float)W), 1);
    NPS_CHECK_LAUNCH("spectral_idft_w_bwd");
    return 0;
}

extern "C" int nps_spectral_dft_w_bwd(const float* gX1, float* gx, int B, int H, int W, int m2, int Cin,
                                      void* stream) {
    NPS_CHECK_ARG(gX1 && gx && B > 0 && H > 0 && W > 0 && m2 > 0 && m2 <= W / 2 + 1 && Cin > 0,
                  "spectral_dft_w_bwd: bad args");
    const size_t lds = idft_w_lds(m2, W);
    NPS_CHECK_ARG(lds <= 96 * 1024, "spectral_dft_w_bwd: m2*W too large");
    const int bs = Cin >= 256 ? 256 : ((Cin + 63) / 64) * 64;
    launch_idft_w<float>(dim3(H, B), bs, lds, (hipStream_t)stream, reinterpret_cast<const float2*>(gX1), gx, H, W, m2,
                         Cin, 0, nullptr, 0, 1.0f, 0);
    NPS_CHECK_LAUNCH("spectral_dft_w_bwd");
    return 0;
}

extern "C" int nps_spectral_mix_bwd(const float* X2, const float* wpack, const float* gY, float* gX2, float* gwpack,
                                    int B, int R, int m2, int Cin, int Cout, void* stream) {
    NPS_CHECK_ARG(X2 && wpack && gY && gX2 && gwpack && B > 0 && R > 0 && m2 > 0 && Cin > 0 && Cout > 0,
                  "spectral_mix_bwd: bad args");
    static int use_valu = -1;  // dev knob NPS_MIX_VALU=1: the scalar-FMA backward (A/B reference)
    if (use_valu < 0) {
        const char* e = getenv("NPS_MIX_VALU");
        use_valu = (e != nullptr && e[0] == '1') ? 1 : 0;
    }
    if (!use_valu && (Cout & 3) == 0 && B <= 32) {
        const dim3 grid(R * m2, (Cin + 63) / 64);
        const auto* x = reinterpret_cast<const float2*>(X2);
        const auto* w = reinterpret_cast<const float2*>(wpack);
        const auto* gy = reinterpret_cast<const float2*>(gY);
        auto* gx = reinterpret_cast<float2*>(gX2);
        auto* gw = reinterpret_cast<float2*>(gwpack);
        if (B <= 16)
            mix_bwd_mfma_kernel<1><<<grid, 256, 0, (hipStream_t)stream>>>(x, w, gy, gx, gw, B, R * m2, Cin, Cout);
        else
            mix_bwd_mfma_kernel<2><<<grid, 256, 0, (hipStream_t)stream>>>(x, w, gy, gx, gw, B, R * m2, Cin, Cout);
        NPS_CHECK_LAUNCH("spectral_mix_bwd (MFMA)");
        return 0;
    }
    const size_t lds = sizeof(float2) * B * Cout;
    NPS_CHECK_ARG(lds <= 64 * 1024, "spectral_mix_bwd: B*Cout=%d too large", B * Cout);
    const int ychunks = (Cin + 31) / 32;
    mix_bwd_kernel<<<dim3(R * m2, ychunks), 256, lds, (hipStream_t)stream>>>(
        reinterpret_cast<const float2*>(X2), reinterpret_cast<const float2*>(wpack),
        reinterpret_cast<const float2*>(gY), reinterpret_cast<float2*>(gX2), reinterpret_cast<float2*>(gwpack), B,
        R * m2, Cin, Cout);
    NPS_CHECK_LAUNCH("spectral_mix_bwd");
    return 0;
}

extern "C" int nps_spectral_unpack_grad(const float* gwpack, float* gw1, float* gw2, int Cin, int Cout, int H, int m1,
                                        int m2, void* stream) {
    NPS_CHECK_ARG(gwpack && gw1 && gw2 && Cin > 0 && Cout > 0 && m1 > 0 && m1 <= H && m2 > 0,
                  "spectral_unpack_grad: bad args");
    const int R = H < 2 * m1 ? H : 2 * m1;
    const size_t n = (size_t)Cin * Cout * m1 * m2;
    spec_unpack_grad_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        reinterpret_cast<const float2*>(gwpack), reinterpret_cast<float2*>(gw1), reinterpret_cast<float2*>(gw2), Cin,
        Cout, H, R, m1, m2);
    NPS_CHECK_LAUNCH("spectral_unpack_grad");
    return 0;
}
