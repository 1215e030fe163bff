// Backward (training) kernels of the grid hot path for gfx950 (MI355X): weight gradients of every
// conv on fp32 MFMA, GroupNorm+GELU frame backward, and the element-wise / reduction pieces the
// pushforward train_step (trainers/autoregressivepushforwardtrainer.py:43-163) differentiates through.
// Input gradients of convs are NOT here: they are forward convs of dy with re-packed weights
// (nps_conv2d_fwd), see nps_hip/autograd.py.
#include "nps_common.hpp"
#include <cstdlib>

namespace {

// ------------------------------------------------------------------------------ weight gradient
// G[m][n][tap] += sum_{b, p} A[b][p][m] * Xext[b][p + tap*dil - pad][n]
// GEMM view: M = A channels, N = X channels, K = pixels of A (split over work-groups).
// Work-group (4 waves) = 64 m x 64 n x up to 9 taps; wave = 32 m x 32 n x taps, one
// v_mfma_f32_32x32x2_f32 accumulator per tap (exact f32).  Per pixel tile (TH x TW A pixels on the
// dilation lattice) A is staged transposed as [m][px] (px contiguous: one ds_read_b128 feeds 4
// MFMAs) and the X patch as [n][patch px]; the A fragment is reused across every tap.
constexpr int WG_TH = 4, WG_TW = 16, WG_PX = WG_TH * WG_TW;  // 64 A pixels per tile
constexpr int WG_TAPS = 9;
constexpr int WG_APITCH = WG_PX + 4;                         // 16-B aligned rows, conflict-free b128 reads

__host__ __device__ inline int wg_patch_px(int KH, int KW) { return (WG_TH + KH - 1) * (WG_TW + KW - 1); }
__host__ __device__ inline int wg_bpitch(int KH, int KW) { return wg_patch_px(KH, KW) | 1; }  // odd: b32 reads conflict-free

__device__ __forceinline__ f32x4 ld4(const float* p, int C, int c) {  // channels [c, c+4) of one pixel row
    if ((C & 3) == 0 && c + 4 <= C) return *reinterpret_cast<const f32x4*>(p + c);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (c + e < C) v[e] = p[c + e];
    return v;
}

__global__ __launch_bounds__(256) void wgrad_kernel(const nps_wgrad_t p, int ntiles, int tiles_per_split, int n_mt,
                                                    int n_nt, int ntap_groups) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1, h = lane >> 5;
    int r = blockIdx.x;
    const int tg = r % ntap_groups;
    r /= ntap_groups;
    const int nt = r % n_nt, mt = r / n_nt;
    const int m0 = mt * 64, n0 = nt * 64;
    const int ntaps_all = p.KH * p.KW;
    const int tap0 = tg * WG_TAPS;
    const int ntap = min(WG_TAPS, ntaps_all - tap0);
    const int T = p.dil;                       // lattice step (A pixels sampled every T rows/cols)
    const int PW = WG_TW + p.KW - 1, PH = WG_TH + p.KH - 1;
    const int npatch = PH * PW;
    const int BP = wg_bpitch(p.KH, p.KW);
    float* As = smem;                          // [64 m][WG_APITCH]
    float* Bs = smem + 64 * WG_APITCH;         // [64 n][BP]
    const int ny = (p.Ha + T - 1) / T, nx = (p.Wa + T - 1) / T;
    const int tiles_y = T * ((ny + WG_TH - 1) / WG_TH), tiles_x = T * ((nx + WG_TW - 1) / WG_TW);
    const int Hext = p.Hx + 2 * p.circ, Wext = p.Wx + 2 * p.circ;

    const int t_begin = blockIdx.y * tiles_per_split;
    const int t_end = min(ntiles, t_begin + tiles_per_split);
    if (t_begin >= t_end) return;

    // register prefetch of one tile's A (4 float4 / thread) and X patch (<= 10 float4 / thread)
    constexpr int NA = WG_PX * 16 / 256;
    constexpr int NB = (8 * 20 * 16 + 255) / 256;  // 5x5 patch
    f32x4 ra[NA], rb[NB];
    auto tile_origin = [&](int t, int& b, int& oy0, int& ox0) {
        b = t / (tiles_y * tiles_x);
        const int rr = t - b * tiles_y * tiles_x;
        const int ty = rr / tiles_x, tx = rr - (rr / tiles_x) * tiles_x;
        oy0 = (ty % T) + (ty / T) * WG_TH * T;
        ox0 = (tx % T) + (tx / T) * WG_TW * T;
    };
    auto issue = [&](int t) {
        int b, oy0, ox0;
        tile_origin(t, b, oy0, ox0);
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const int idx = tid + k * 256;
            const int px = idx >> 4, mq = idx & 15;
            const int oy = oy0 + (px / WG_TW) * T, ox = ox0 + (px % WG_TW) * T;
            const int m = m0 + mq * 4;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (oy < p.Ha && ox < p.Wa && m < p.M) v = ld4(p.a + ((size_t)(b * p.Ha + oy) * p.Wa + ox) * p.M, p.M, m);
            ra[k] = v;
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int idx = tid + k * 256;
            const int pp = idx >> 4, nq = idx & 15;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (pp < npatch) {
                const int pr = pp / PW, pc = pp - (pp / PW) * PW;
                const int ye = oy0 + pr * T - p.pad_y, xe = ox0 + pc * T - p.pad_x;
                const int n = n0 + nq * 4;
                if (ye >= 0 && ye < Hext && xe >= 0 && xe < Wext && n < p.N) {
                    const int y = p.circ ? nps::wrap_mod(ye - p.circ, p.Hx) : ye;
                    const int x = p.circ ? nps::wrap_mod(xe - p.circ, p.Wx) : xe;
                    v = ld4(p.x + ((size_t)(b * p.Hx + y) * p.Wx + x) * p.N, p.N, n);
                }
            }
            rb[k] = v;
        }
    };
    auto commit = [&]() {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const int idx = tid + k * 256;
            const int px = idx >> 4, mq = idx & 15;
#pragma unroll
            for (int e = 0; e < 4; ++e) As[(mq * 4 + e) * WG_APITCH + px] = ra[k][e];
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int idx = tid + k * 256;
            const int pp = idx >> 4, nq = idx & 15;
            if (pp < npatch) {
#pragma unroll
                for (int e = 0; e < 4; ++e) Bs[(nq * 4 + e) * BP + pp] = rb[k][e];
            }
        }
    };

    f32x16 acc[WG_TAPS];
#pragma unroll
    for (int i = 0; i < WG_TAPS; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;

    // per-tap patch offsets of this thread's (ky, kx)
    int toff[WG_TAPS];
#pragma unroll
    for (int i = 0; i < WG_TAPS; ++i) {
        const int tap = tap0 + (i < ntap ? i : 0);
        toff[i] = (tap / p.KW) * PW + (tap % p.KW);
    }
    const float* arow = As + (wm * 32 + (lane & 31)) * WG_APITCH + h * 4;
    const float* brow = Bs + (wn * 32 + (lane & 31)) * BP;

    issue(t_begin);
    for (int t = t_begin; t < t_end; ++t) {
        __syncthreads();
        commit();
        __syncthreads();
        if (t + 1 < t_end) issue(t + 1);
#pragma unroll
        for (int gi = 0; gi < WG_PX / 8; ++gi) {
            const f32x4 av = *reinterpret_cast<const f32x4*>(arow + gi * 8);
            // A pixels gi*8 + h*4 + e (e < 4) lie in tile row gi/2, columns (gi&1)*8 + h*4 + e
            const int pbase = (gi >> 1) * PW + (gi & 1) * 8 + h * 4;
#pragma unroll
            for (int i = 0; i < WG_TAPS; ++i) {
                if (i < ntap) {
                    const float* bp = brow + pbase + toff[i];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bp[e], acc[i], 0, 0, 0);
                }
            }
        }
    }

    // accumulate this split's partial into G: lane holds rows (r/4)*8 + h*4 + r%4, column lane%32
    const int n = n0 + wn * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < WG_TAPS; ++i) {
        if (i >= ntap) continue;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
            const int m = m0 + wm * 32 + (rr >> 2) * 8 + h * 4 + (rr & 3);
            if (m < p.M && n < p.N) atomicAdd(p.g + ((size_t)m * p.N + n) * ntaps_all + tap0 + i, acc[i][rr]);
        }
    }
}

// ------------------------------------------------------------------------------ channel sums
// out[c] += sum over rows of x[row][c]  (bias gradients: rows = B*H*W pixels of an NHWC tensor)
__global__ void channel_sums_kernel(const float* __restrict__ x, long rows, int C, int rows_per_block,
                                    float* __restrict__ out) {
    extern __shared__ float part[];  // [C]
    for (int c = threadIdx.x; c < C; c += blockDim.x) part[c] = 0.f;
    __syncthreads();
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(rows, r0 + rows_per_block);
    // each thread owns channel c = tid % C ... swept over rows in strides of (blockDim / C)
    if (C <= (int)blockDim.x) {
        const int per = blockDim.x / C;
        const int c = threadIdx.x % C, lr = threadIdx.x / C;
        if (lr < per) {
            float s = 0.f;
            for (long rr = r0 + lr; rr < r1; rr += per) s += x[rr * C + c];
            atomicAdd(&part[c], s);
        }
    } else {
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            float s = 0.f;
            for (long rr = r0; rr < r1; ++rr) s += x[rr * C + c];
            part[c] += s;
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&out[c], part[c]);
}

// The same for C % 4 == 0, C <= 1024: thread = one channel quad (fixed) x rows lr, lr + per, ... of the
// block's range, summed in registers from 16-B loads; one LDS add per channel per thread at the end.
__global__ void channel_sums4_kernel(const float* __restrict__ x, long rows, int C, int rows_per_block,
                                     float* __restrict__ out) {
    extern __shared__ float part[];  // [C]
    for (int c = threadIdx.x; c < C; c += blockDim.x) part[c] = 0.f;
    __syncthreads();
    const int Q = C >> 2, per = blockDim.x / Q;
    const int q = threadIdx.x % Q, lr = threadIdx.x / Q;
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(rows, r0 + rows_per_block);
    if (lr < per) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        const f32x4* xp = reinterpret_cast<const f32x4*>(x) + q;
#pragma unroll 4
        for (long rr = r0 + lr; rr < r1; rr += per) s += xp[rr * Q];
#pragma unroll
        for (int e = 0; e < 4; ++e) atomicAdd(&part[4 * q + e], s[e]);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&out[c], part[c]);
}

// ------------------------------------------------------------------------------ element-wise
__device__ __forceinline__ float gelu_grad(float z) {
    // d/dz [0.5 z (1 + erf(z/sqrt2))] = Phi(z) + z phi(z)
    return 0.5f * (1.0f + erff(z * 0.70710678118654752440f)) + z * 0.39894228040143267794f * expf(-0.5f * z * z);
}

__global__ void gelu_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = nps::gelu_erf(x[i]);
}

__global__ void gelu_bwd_kernel(const float* __restrict__ x, const float* __restrict__ gy, float* __restrict__ gx,
                                long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        gx[i] = gy[i] * gelu_grad(x[i]);
}

// out[b][y + oy][x + ox][c] += src[b][y][x][c] for the positions that land inside out
__global__ void add_at_kernel(float* __restrict__ out, const float* __restrict__ src, int Ho, int Wo, int Hs, int Ws,
                              int C, int oy, int ox) {
    const int b = blockIdx.y;
    const long n = (long)Hs * Ws * C;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long pix = i / C;
        const int y = (int)(pix / Ws), x = (int)(pix - (long)y * Ws);
        const int yy = y + oy, xx = x + ox;
        if (yy >= 0 && yy < Ho && xx >= 0 && xx < Wo)
            out[(((size_t)b * Ho + yy) * Wo + xx) * C + c] += src[((size_t)b * Hs * Ws + pix) * C + c];
    }
}

// out = base + crop_Nd(src) at (oy, ox) in one pass (4-channel quads; the residual of proc_unet_modern.py:250 in the
// differentiable path): out pixel (Y, X) adds src pixel (Y - oy, X - ox) where that lies inside src — instead of
// clone(base) + add_at (5 tensor streams -> 3)
// out = base + crop_Nd(src) in one pass; STATS: also ADDS out's per-sample (sum, sum of squares) into
// out_stats[b][blockIdx.x % NPS_STATS_SUB] (fp64; one atomic pair per work-group after an LDS reduction)
template <bool STATS>
__global__ __launch_bounds__(256) void add_at_copy4_kernel(float* __restrict__ out, const float* __restrict__ base,
                                                           const float* __restrict__ src, int Ho, int Wo, int Hs,
                                                           int Ws, int C, int oy, int ox, double* out_stats) {
    const int b = blockIdx.y;
    const int Q = C >> 2;
    const long n = (long)Ho * Wo * Q;
    const f32x4* bq = reinterpret_cast<const f32x4*>(base) + (size_t)b * n;
    f32x4* oq = reinterpret_cast<f32x4*>(out) + (size_t)b * n;
    const f32x4* sq = reinterpret_cast<const f32x4*>(src) + (size_t)b * Hs * Ws * Q;
    double s1 = 0.0, s2 = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int q = (int)(i % Q);
        const long pix = i / Q;
        const int Y = (int)(pix / Wo), X = (int)(pix - (long)Y * Wo);
        const int y = Y - oy, x = X - ox;
        f32x4 v = bq[i];
        if (y >= 0 && y < Hs && x >= 0 && x < Ws) v += sq[((size_t)y * Ws + x) * Q + q];
        oq[i] = v;
        if constexpr (STATS) {
            // (the 4 lanes' partials in fp32 as the conv epilogues' store_tile_s, then fp64)
            s1 += (double)((v[0] + v[1]) + (v[2] + v[3]));
            s2 += (double)((v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]));
        }
    }
    if constexpr (STATS) {
        __shared__ double red[2 * 4];
        s1 = nps::wave_sum(s1);
        s2 = nps::wave_sum(s2);
        const int w = (int)(threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0) {
            red[2 * w] = s1;
            red[2 * w + 1] = s2;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double* p = out_stats + ((size_t)b * NPS_STATS_SUB + blockIdx.x % NPS_STATS_SUB) * 2;
            atomicAdd(p, ((red[0] + red[2]) + (red[4] + red[6])));
            atomicAdd(p + 1, ((red[1] + red[3]) + (red[5] + red[7])));
        }
    }
}

// out[b][Y][X][c] = x[b][(Y - pad) mod H][(X - pad) mod W][c]   (circular_pad_2d, common.py:61-90)
__global__ void circ_pad_kernel(const float* __restrict__ x, float* __restrict__ out, int H, int W, int C, int pad) {
    const int b = blockIdx.y;
    const int Ho = H + 2 * pad, Wo = W + 2 * pad;
    const long n = (long)Ho * Wo * C;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long pix = i / C;
        const int Y = (int)(pix / Wo), X = (int)(pix - (long)Y * Wo);
        const int y = nps::wrap_mod(Y - pad, H), xx = nps::wrap_mod(X - pad, W);
        out[(size_t)b * n + i] = x[(((size_t)b * H + y) * W + xx) * C + c];
    }
}

// adjoint of circ_pad: gx[b][y][x][c] = sum of gp over the padded positions that wrap to (y, x)
__global__ void circ_fold_kernel(const float* __restrict__ gp, float* __restrict__ gx, int H, int W, int C, int pad) {
    const int b = blockIdx.y;
    const int Hp = H + 2 * pad, Wp = W + 2 * pad;
    const long n = (long)H * W * C;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long pix = i / C;
        const int y = (int)(pix / W), x = (int)(pix - (long)y * W);
        float s = 0.f;
        for (int Y = y + pad - ((y + pad) / H) * H; Y < Hp; Y += H)      // smallest Y >= 0 with Y = y + pad (mod H)
            for (int X = x + pad - ((x + pad) / W) * W; X < Wp; X += W)
                s += gp[(((size_t)b * Hp + Y) * Wp + X) * C + c];
        gx[(size_t)b * n + i] = s;
    }
}

// out[i] = (*scale) * (a[i] - b[i])   (gradient of sqrt(MSE_sum), scale = g / sqrt(L) on the device)
__global__ void scaled_diff_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                   const double* __restrict__ scale, float* __restrict__ out, long n) {
    const float s = (float)scale[0];
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        out[i] = s * (a[i] - b[i]);
}

// ------------------------------------------------------------------------------ frame (GN + GELU) backward
// Forward (nps_frame_pack): per frame element x (0 where no source covers it),
//   xhat = (x - mu[b,g]) * rstd[b,g];  z = gamma_c xhat + beta_c;  y = act(z).
// Pass 1: P[b][c] += sum_pix gz, Q[b][c] += sum_pix gz * xhat   (gz = gy * act'(z)).
// Pass 2: dgamma_c = sum_b Q, dbeta_c = sum_b P;  S1[b,g] = sum_{c in g} gamma_c P, S2 = sum gamma_c Q;
//   dx = rstd (gamma_c gz - S1/N - xhat S2/N) at covered positions (N = elements of the group).
__device__ __forceinline__ void gn_tab_fill(const nps_conv2d_t& a, int b, float2* tab) {
    if (a.gn_stats != nullptr && threadIdx.x < a.gn_groups) {
        const double cnt = (double)(a.Cin / a.gn_groups) * a.Hin * a.Win;
        const double s1 = a.gn_stats[(b * a.gn_groups + threadIdx.x) * 2];
        const double s2 = a.gn_stats[(b * a.gn_groups + threadIdx.x) * 2 + 1];
        const double mean = s1 / cnt;
        double var = s2 / cnt - mean * mean;
        var = var < 0.0 ? 0.0 : var;
        tab[threadIdx.x] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.gn_eps)));
    }
}

__device__ __forceinline__ float frame_val(const nps_conv2d_t& a, int b, int y, int x, int c) {
    int lo = 0;
#pragma unroll
    for (int si = 0; si < NPS_MAX_SRC; ++si) {
        if (si < a.nsrc) {
            const nps_src_t S = si == 0 ? a.src[0] : (si == 1 ? a.src[1] : a.src[2]);
            if (c >= lo && c < lo + S.C) {
                const int yy = y - S.off_y, xx = x - S.off_x;
                if (yy >= 0 && yy < S.H && xx >= 0 && xx < S.W)
                    return S.ptr[((size_t)(b * S.H + yy) * S.W + xx) * S.C + (c - lo)];
                return 0.f;
            }
            lo += S.C;
        }
    }
    return 0.f;
}

__global__ void frame_bwd_reduce_kernel(nps_conv2d_t a, const float* __restrict__ gy, double* __restrict__ PQ) {
    extern __shared__ float part[];  // [2][Cin]
    __shared__ float2 tab[16];
    const int b = blockIdx.y;
    gn_tab_fill(a, b, tab);
    for (int c = threadIdx.x; c < 2 * a.Cin; c += blockDim.x) part[c] = 0.f;
    __syncthreads();
    const int cpg = a.gn_stats ? a.Cin / a.gn_groups : 1;
    const long n = (long)a.Hin * a.Win * a.Cin;
    const float* g = gy + (size_t)b * n;
    // each thread keeps a fixed channel when the grid stride is a multiple of Cin
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int c = (int)(i % a.Cin);
        const long pix = i / a.Cin;
        const int y = (int)(pix / a.Win), x = (int)(pix - (long)y * a.Win);
        float v = frame_val(a, b, y, x, c);
        float xh = v;
        if (a.gn_stats) {
            const float2 mr = tab[c / cpg];
            xh = (v - mr.x) * mr.y;
            v = xh * a.gn_gamma[c] + a.gn_beta[c];
        }
        float gz = g[i];
        if (a.pre_act == 1) gz *= gelu_grad(v);
        atomicAdd(&part[c], gz);
        atomicAdd(&part[a.Cin + c], gz * xh);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.Cin; c += blockDim.x) {
        atomicAdd(&PQ[(b * 2) * a.Cin + c], (double)part[c]);
        atomicAdd(&PQ[(b * 2 + 1) * a.Cin + c], (double)part[a.Cin + c]);
    }
}

// s12[g] = (sum over the group's channels of gamma[c] * (P, Q)[b][c]) / N, the GroupNorm backward's two group
// means, computed by the whole work-group (every thread a strided share of its group's channels, wave sums,
// fp64 LDS adds), written to s12 by threads < G.  It ends WITHOUT a barrier after those writes: the caller must
// __syncthreads before any thread reads s12 (both callers do, behind their own table setup).  (Was one thread per
// group walking Cin / groups channels of L2 loads while the work-group's other waves waited: with GroupNorm(1),
// 2 x Cin dependent-issue loads before any pixel.)
__device__ __forceinline__ void frame_bwd_s12(const nps_conv2d_t& a, const double* __restrict__ PQ, int b, int cpg,
                                              float (*s12)[2]) {
    __shared__ double acc[16][2];
    const int G = a.gn_groups;
    if (threadIdx.x < 2 * G) (&acc[0][0])[threadIdx.x] = 0.0;
    __syncthreads();
    const int tpg = (int)blockDim.x / G;  // (G <= 16: >= 16 threads per group)
    const int g = (int)threadIdx.x / tpg, j = (int)threadIdx.x - g * tpg;
    const double* P = PQ + (size_t)(b * 2) * a.Cin;
    const double* Q = P + a.Cin;
    double s1 = 0.0, s2 = 0.0;
    if (g < G)
        for (int c = g * cpg + j; c < (g + 1) * cpg; c += tpg) {
            const double ga = (double)a.gn_gamma[c];
            s1 += ga * P[c];
            s2 += ga * Q[c];
        }
    const int wg0 = __shfl(g, 0), wg1 = __shfl(g, 63);
    if (wg0 == wg1) {  // the whole wave in one group: one LDS add pair per wave
        s1 = nps::wave_sum(s1);
        s2 = nps::wave_sum(s2);
        if ((threadIdx.x & 63) == 0 && g < G) {
            atomicAdd(&acc[g][0], s1);
            atomicAdd(&acc[g][1], s2);
        }
    } else if (g < G) {
        atomicAdd(&acc[g][0], s1);
        atomicAdd(&acc[g][1], s2);
    }
    __syncthreads();
    if ((int)threadIdx.x < G) {
        const double N = (double)cpg * a.Hin * a.Win;
        s12[threadIdx.x][0] = (float)(acc[threadIdx.x][0] / N);
        s12[threadIdx.x][1] = (float)(acc[threadIdx.x][1] / N);
    }
}

__global__ void frame_bwd_apply_kernel(nps_conv2d_t a, const float* __restrict__ gy, const double* __restrict__ PQ,
                                       float* d0, float* d1, float* d2, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, const float* __restrict__ gy2) {
    __shared__ float2 tab[16];
    __shared__ float s12[16][2];
    const int b = blockIdx.y, si = blockIdx.z;
    gn_tab_fill(a, b, tab);
    const int cpg = a.gn_stats ? a.Cin / a.gn_groups : 1;
    if (a.gn_stats) frame_bwd_s12(a, PQ, b, cpg, s12);
    if (a.gn_stats && b == 0 && si == 0 && blockIdx.x == 0 && dgamma) {
        for (int c = threadIdx.x; c < a.Cin; c += blockDim.x) {
            double sg = 0.0, sb = 0.0;
            for (int bb = 0; bb < a.B; ++bb) {
                sb += PQ[(bb * 2) * a.Cin + c];
                sg += PQ[(bb * 2 + 1) * a.Cin + c];
            }
            dgamma[c] = (float)sg;
            dbeta[c] = (float)sb;
        }
    }
    __syncthreads();
    float* dst = si == 0 ? d0 : (si == 1 ? d1 : d2);
    if (dst == nullptr) return;
    const nps_src_t S = si == 0 ? a.src[0] : (si == 1 ? a.src[1] : a.src[2]);
    const int lo = si == 0 ? 0 : (si == 1 ? a.src[0].C : a.src[0].C + a.src[1].C);
    const long n = (long)S.H * S.W * S.C;
    const float* g = gy + (size_t)b * a.Hin * a.Win * a.Cin;
    const float* g2 = gy2 != nullptr ? gy2 + (size_t)b * a.Hin * a.Win * a.Cin : nullptr;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int cs = (int)(i % S.C);
        const long pix = i / S.C;
        const int ys = (int)(pix / S.W), xs = (int)(pix - (long)ys * S.W);
        const int y = ys + S.off_y, x = xs + S.off_x;
        float d = 0.f;
        if (y >= 0 && y < a.Hin && x >= 0 && x < a.Win) {
            const int c = lo + cs;
            const float v = S.ptr[(size_t)b * n + i];
            float gz = g[((size_t)y * a.Win + x) * a.Cin + c];
            if (a.gn_stats) {
                const int gidx = c / cpg;
                const float2 mr = tab[gidx];
                const float xh = (v - mr.x) * mr.y;
                const float ga = a.gn_gamma[c];
                if (a.pre_act == 1) gz *= gelu_grad(xh * ga + a.gn_beta[c]);
                d = mr.y * (ga * gz - s12[gidx][0] - xh * s12[gidx][1]);
            } else {
                if (a.pre_act == 1) gz *= gelu_grad(v);
                d = gz;
            }
            if (g2 != nullptr) d += g2[((size_t)y * a.Win + x) * a.Cin + c];  // the plain frame's gradient
        }
        dst[(size_t)b * n + i] = d;
    }
}

// Quad forms of the frame backward (every source's C, Cin and the GroupNorm group size multiples of 4, so
// a channel quad lies in one source and one group): thread = one fixed channel quad x pixels lr, lr + per,
// ... of the block's pixel range (row / column stepped, no per-element division), 16-B loads and stores,
// the reduce pass's sums in registers until one LDS add per channel per thread.
#ifndef FB_U
#define FB_U 4  // pixels per loop step of the quad frame-backward kernels
#endif
struct FrameQuad {  // the source, GroupNorm operands and source origin of a thread's channel quad
    const float* ptr;
    int C, H, W, oy, ox, cs;
    f32x4 gam, bet;
    float2 mr;
};
__device__ __forceinline__ FrameQuad frame_quad(const nps_conv2d_t& a, int c0, const float2* tab, int cpg) {
    FrameQuad f;
    int lo = 0, si = 0, base = 0;
#pragma unroll
    for (int k = 0; k < NPS_MAX_SRC; ++k)
        if (k < a.nsrc) {
            const int C = k == 0 ? a.src[0].C : (k == 1 ? a.src[1].C : a.src[2].C);
            if (c0 >= lo && c0 < lo + C) {
                si = k;
                base = lo;
            }
            lo += C;
        }
    const nps_src_t S = si == 0 ? a.src[0] : (si == 1 ? a.src[1] : a.src[2]);
    f.ptr = S.ptr;
    f.C = S.C;
    f.H = S.H;
    f.W = S.W;
    f.oy = S.off_y;
    f.ox = S.off_x;
    f.cs = c0 - base;
    if (a.gn_stats) {
        f.gam = *reinterpret_cast<const f32x4*>(a.gn_gamma + c0);
        f.bet = *reinterpret_cast<const f32x4*>(a.gn_beta + c0);
        f.mr = tab[c0 / cpg];
    } else {
        f.gam = f32x4{1.f, 1.f, 1.f, 1.f};
        f.bet = f32x4{0.f, 0.f, 0.f, 0.f};
        f.mr = make_float2(0.f, 1.f);
    }
    return f;
}

__global__ void frame_bwd_reduce4_kernel(nps_conv2d_t a, const float* __restrict__ gy, double* __restrict__ PQ,
                                         int px_per_block) {
    extern __shared__ float part[];  // [2][Cin]
    __shared__ float2 tab[16];
    const int b = blockIdx.y;
    gn_tab_fill(a, b, tab);
    for (int c = threadIdx.x; c < 2 * a.Cin; c += blockDim.x) part[c] = 0.f;
    __syncthreads();
    const int Q = a.Cin >> 2, per = blockDim.x / Q;
    const int q = threadIdx.x % Q, lr = threadIdx.x / Q;
    const int npix = a.Hin * a.Win;
    const int p0 = blockIdx.x * px_per_block, p1 = min(npix, p0 + px_per_block);
    if (lr < per && p0 + lr < p1) {
        const int cpg = a.gn_stats ? a.Cin / a.gn_groups : 1;
        const FrameQuad f = frame_quad(a, 4 * q, tab, cpg);
        const float* sb = f.ptr + (size_t)b * f.H * f.W * f.C + f.cs;
        const float* g = gy + (size_t)b * npix * a.Cin + 4 * q;
        f32x4 P = {0.f, 0.f, 0.f, 0.f}, Qs = {0.f, 0.f, 0.f, 0.f};
        int pix = p0 + lr;
        int y = pix / a.Win, x = pix - y * a.Win;
        const int dy = per / a.Win, dx = per - dy * a.Win;
        // FB_U pixels per step: all their loads issue before the first use (memory-level parallelism)
        for (; pix < p1; pix += FB_U * per) {
            f32x4 v[FB_U], gz[FB_U];
#pragma unroll
            for (int k = 0; k < FB_U; ++k) {
                const int pk = pix + k * per;
                const int yy = y - f.oy, xx = x - f.ox;
                v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
                gz[k] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (pk < p1) {
                    if (yy >= 0 && yy < f.H && xx >= 0 && xx < f.W)
                        v[k] = *reinterpret_cast<const f32x4*>(sb + ((size_t)yy * f.W + xx) * f.C);
                    gz[k] = *reinterpret_cast<const f32x4*>(g + (size_t)pk * a.Cin);
                }
                x += dx;
                y += dy;
                if (x >= a.Win) {
                    x -= a.Win;
                    ++y;
                }
            }
#pragma unroll
            for (int k = 0; k < FB_U; ++k) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {  // (a pixel past p1 has gz = 0: adds nothing)
                    const float xh = a.gn_stats ? (v[k][e] - f.mr.x) * f.mr.y : v[k][e];
                    const float z = a.gn_stats ? xh * f.gam[e] + f.bet[e] : v[k][e];
                    float gk = gz[k][e];
                    if (a.pre_act == 1) gk *= gelu_grad(z);
                    P[e] += gk;
                    Qs[e] = fmaf(gk, xh, Qs[e]);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            atomicAdd(&part[4 * q + e], P[e]);
            atomicAdd(&part[a.Cin + 4 * q + e], Qs[e]);
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.Cin; c += blockDim.x) {
        atomicAdd(&PQ[(b * 2) * a.Cin + c], (double)part[c]);
        atomicAdd(&PQ[(b * 2 + 1) * a.Cin + c], (double)part[a.Cin + c]);
    }
}

// dtag[i] (or NULL): a range tag raised to cover |dsrc[i]| (one atomic per wave), so the conv backward that reads
// the source gradient as its dy needs no absmax pass (nps_hip autograd: range tags)
__global__ void frame_bwd_apply4_kernel(nps_conv2d_t a, const float* __restrict__ gy, const double* __restrict__ PQ,
                                        float* d0, float* d1, float* d2, float* __restrict__ dgamma,
                                        float* __restrict__ dbeta, int px_per_block, float* t0, float* t1,
                                        float* t2, const float* __restrict__ gy2) {
    __shared__ float2 tab[16];
    __shared__ float s12[16][2];
    const int b = blockIdx.y, si = blockIdx.z;
    gn_tab_fill(a, b, tab);
    const int cpg = a.gn_stats ? a.Cin / a.gn_groups : 1;
    if (a.gn_stats) frame_bwd_s12(a, PQ, b, cpg, s12);
    if (a.gn_stats && b == 0 && si == 0 && blockIdx.x == 0 && dgamma) {
        for (int c = threadIdx.x; c < a.Cin; c += blockDim.x) {
            double sg = 0.0, sb = 0.0;
            for (int bb = 0; bb < a.B; ++bb) {
                sb += PQ[(bb * 2) * a.Cin + c];
                sg += PQ[(bb * 2 + 1) * a.Cin + c];
            }
            dgamma[c] = (float)sg;
            dbeta[c] = (float)sb;
        }
    }
    __syncthreads();
    float* dst = si == 0 ? d0 : (si == 1 ? d1 : d2);
    if (dst == nullptr) return;
    const nps_src_t S = si == 0 ? a.src[0] : (si == 1 ? a.src[1] : a.src[2]);
    const int lo = si == 0 ? 0 : (si == 1 ? a.src[0].C : a.src[0].C + a.src[1].C);
    const int Q = S.C >> 2, per = blockDim.x / Q;
    const int q = threadIdx.x % Q, lr = threadIdx.x / Q;
    const int npix = S.H * S.W;
    const int p0 = blockIdx.x * px_per_block, p1 = min(npix, p0 + px_per_block);
    float amax = 0.f;
    if (!(lr >= per || p0 + lr >= p1)) {  // (no early return: the tag publish below is wave-collective)
    const int c0 = lo + 4 * q;
    const int gidx = c0 / cpg;
    const float2 mr = a.gn_stats ? tab[gidx] : make_float2(0.f, 1.f);
    const float t1 = a.gn_stats ? s12[gidx][0] : 0.f, t2 = a.gn_stats ? s12[gidx][1] : 0.f;
    f32x4 gam = {1.f, 1.f, 1.f, 1.f}, bet = {0.f, 0.f, 0.f, 0.f};
    if (a.gn_stats) {
        gam = *reinterpret_cast<const f32x4*>(a.gn_gamma + c0);
        bet = *reinterpret_cast<const f32x4*>(a.gn_beta + c0);
    }
    const float* sp = S.ptr + (size_t)b * npix * S.C + 4 * q;
    float* dp = dst + (size_t)b * npix * S.C + 4 * q;
    const float* g = gy + (size_t)b * a.Hin * a.Win * a.Cin + c0;
    // gy2 (or NULL): the gradient of the same frame from a second consumer of the plain concatenation (the
    // ResidualBlock's shortcut / identity path), added here instead of by autograd's accumulation pass
    const float* g2 = gy2 != nullptr ? gy2 + (size_t)b * a.Hin * a.Win * a.Cin + c0 : nullptr;
    int pix = p0 + lr;
    int ys = pix / S.W, xs = pix - ys * S.W;
    const int dy = per / S.W, dx = per - dy * S.W;
    for (; pix < p1; pix += FB_U * per) {
        f32x4 v[FB_U], gz[FB_U], gp[FB_U];
        bool in[FB_U];
#pragma unroll
        for (int k = 0; k < FB_U; ++k) {  // FB_U pixels' loads first, then their math and stores
            const int pk = pix + k * per;
            const int y = ys + S.off_y, x = xs + S.off_x;
            in[k] = pk < p1 && y >= 0 && y < a.Hin && x >= 0 && x < a.Win;
            v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            gz[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            gp[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (in[k]) {
                v[k] = *reinterpret_cast<const f32x4*>(sp + (size_t)pk * S.C);
                gz[k] = *reinterpret_cast<const f32x4*>(g + ((size_t)y * a.Win + x) * a.Cin);
                if (g2 != nullptr) gp[k] = *reinterpret_cast<const f32x4*>(g2 + ((size_t)y * a.Win + x) * a.Cin);
            }
            xs += dx;
            ys += dy;
            if (xs >= S.W) {
                xs -= S.W;
                ++ys;
            }
        }
#pragma unroll
        for (int k = 0; k < FB_U; ++k) {
            const int pk = pix + k * per;
            if (pk >= p1) break;
            f32x4 d = {0.f, 0.f, 0.f, 0.f};
            if (in[k]) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (a.gn_stats) {
                        const float xh = (v[k][e] - mr.x) * mr.y;
                        float gk = gz[k][e];
                        if (a.pre_act == 1) gk *= gelu_grad(xh * gam[e] + bet[e]);
                        d[e] = mr.y * (gam[e] * gk - t1 - xh * t2);
                    } else {
                        float gk = gz[k][e];
                        if (a.pre_act == 1) gk *= gelu_grad(v[k][e]);
                        d[e] = gk;
                    }
                    d[e] += gp[k][e];
                }
            }
            *reinterpret_cast<f32x4*>(dp + (size_t)pk * S.C) = d;
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(d[0]), fabsf(d[1])), fmaxf(fabsf(d[2]), fabsf(d[3]))));
        }
    }
    }
    nps::tag_publish(si == 0 ? t0 : (si == 1 ? t1 : t2), amax, nps::wave_salt());
}

inline int grid_for(long n, int per_block = 256 * 8, int cap = 4096) {
    long nb = (n + per_block - 1) / per_block;
    return (int)(nb < 1 ? 1 : (nb > cap ? cap : nb));
}

}  // namespace

// ================================================================================ C ABI
extern "C" size_t nps_wgrad_lds_bytes(int KH, int KW) {
    return sizeof(float) * (64 * WG_APITCH + 64 * wg_bpitch(KH, KW));
}

extern "C" int nps_conv2d_wgrad(const nps_wgrad_t* pp, void* stream) {
    NPS_CHECK_ARG(pp != nullptr, "conv2d_wgrad: null");
    const nps_wgrad_t& p = *pp;
    NPS_CHECK_ARG(p.a && p.x && p.g && p.B > 0 && p.Ha > 0 && p.Wa > 0 && p.M > 0 && p.Hx > 0 && p.Wx > 0 && p.N > 0,
                  "conv2d_wgrad: bad shape");
    NPS_CHECK_ARG(p.KH >= 1 && p.KH <= 5 && p.KW >= 1 && p.KW <= 5 && p.dil >= 1 && p.circ >= 0,
                  "conv2d_wgrad: kernel %dx%d dil %d unsupported", p.KH, p.KW, p.dil);
    NPS_CHECK_ARG(p.db == nullptr, "conv2d_wgrad: the bias gradient (db) is computed by the split-fp16 entry points only");
    const int T = p.dil;
    const int ny = (p.Ha + T - 1) / T, nx = (p.Wa + T - 1) / T;
    const long tiles_y = (long)T * ((ny + WG_TH - 1) / WG_TH), tiles_x = (long)T * ((nx + WG_TW - 1) / WG_TW);
    const long ntiles = (long)p.B * tiles_y * tiles_x;
    NPS_CHECK_ARG(ntiles < (1L << 30), "conv2d_wgrad: too many tiles");
    const int n_mt = (p.M + 63) / 64, n_nt = (p.N + 63) / 64;
    const int ntg = (p.KH * p.KW + WG_TAPS - 1) / WG_TAPS;
    const long base = (long)n_mt * n_nt * ntg;
    // split K (pixel tiles) so the grid puts ~4 work-groups on each of the 256 CUs, >= 8 tiles each
    long splits = (1024 + base - 1) / base;
    const long max_splits = (ntiles + 7) / 8;
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    const int per = (int)((ntiles + splits - 1) / splits);
    splits = (ntiles + per - 1) / per;
    NPS_CHECK_ARG(base * 1 < (1L << 31) && splits < 65536, "conv2d_wgrad: grid too large");
    const size_t lds = nps_wgrad_lds_bytes(p.KH, p.KW);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    wgrad_kernel<<<dim3((unsigned)base, (unsigned)splits), 256, lds, (hipStream_t)stream>>>(p, (int)ntiles, per, n_mt,
                                                                                         n_nt, ntg);
    NPS_CHECK_LAUNCH("conv2d_wgrad");
    return 0;
}

extern "C" int nps_channel_sums(const float* x, long rows, int C, float* out, void* stream) {
    NPS_CHECK_ARG(x && out && rows > 0 && C > 0 && C <= 8192, "channel_sums: bad args");
    const int rpb = 256;
    const long nb = (rows + rpb - 1) / rpb;
    NPS_CHECK_ARG(nb < (1L << 31), "channel_sums: too many rows");
    if ((C & 3) == 0 && C <= 1024 && (reinterpret_cast<size_t>(x) & 15) == 0)
        channel_sums4_kernel<<<(unsigned)nb, 256, sizeof(float) * C, (hipStream_t)stream>>>(x, rows, C, rpb, out);
    else
        channel_sums_kernel<<<(unsigned)nb, 256, sizeof(float) * C, (hipStream_t)stream>>>(x, rows, C, rpb, out);
    NPS_CHECK_LAUNCH("channel_sums");
    return 0;
}

extern "C" int nps_gelu(const float* x, float* y, long n, void* stream) {
    NPS_CHECK_ARG(x && y && n > 0, "gelu: bad args");
    gelu_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(x, y, n);
    NPS_CHECK_LAUNCH("gelu");
    return 0;
}

extern "C" int nps_gelu_bwd(const float* x, const float* gy, float* gx, long n, void* stream) {
    NPS_CHECK_ARG(x && gy && gx && n > 0, "gelu_bwd: bad args");
    gelu_bwd_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(x, gy, gx, n);
    NPS_CHECK_LAUNCH("gelu_bwd");
    return 0;
}

extern "C" int nps_add_at(float* out, const float* src, int B, int Ho, int Wo, int Hs, int Ws, int C, int off_y,
                          int off_x, void* stream) {
    NPS_CHECK_ARG(out && src && B > 0 && Ho > 0 && Wo > 0 && Hs > 0 && Ws > 0 && C > 0, "add_at: bad args");
    add_at_kernel<<<dim3(grid_for((long)Hs * Ws * C, 256 * 8, 2048), B), 256, 0, (hipStream_t)stream>>>(
        out, src, Ho, Wo, Hs, Ws, C, off_y, off_x);
    NPS_CHECK_LAUNCH("add_at");
    return 0;
}

extern "C" int nps_add_at_copy(float* out, const float* base, const float* src, int B, int Ho, int Wo, int Hs, int Ws,
                               int C, int off_y, int off_x, double* out_stats, void* stream) {
    NPS_CHECK_ARG(out && base && src && B > 0 && Ho > 0 && Wo > 0 && Hs > 0 && Ws > 0 && C > 0 && (C & 3) == 0 &&
                      ((reinterpret_cast<size_t>(out) | reinterpret_cast<size_t>(base) |
                        reinterpret_cast<size_t>(src)) & 15) == 0,
                  "add_at_copy: bad args (C %% 4 == 0, 16-B aligned tensors)");
    const dim3 grid(grid_for((long)Ho * Wo * (C / 4), 256 * 4, 2048), B);
    if (out_stats)
        add_at_copy4_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(out, base, src, Ho, Wo, Hs, Ws, C, off_y,
                                                                          off_x, out_stats);
    else
        add_at_copy4_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(out, base, src, Ho, Wo, Hs, Ws, C, off_y,
                                                                           off_x, nullptr);
    NPS_CHECK_LAUNCH("add_at_copy");
    return 0;
}

extern "C" int nps_circular_pad(const float* x, float* out, int B, int H, int W, int C, int pad, void* stream) {
    NPS_CHECK_ARG(x && out && B > 0 && H > 0 && W > 0 && C > 0 && pad >= 0 && pad <= H && pad <= W,
                  "circular_pad: bad args");
    circ_pad_kernel<<<dim3(grid_for((long)(H + 2 * pad) * (W + 2 * pad) * C, 256 * 8, 2048), B), 256, 0,
                      (hipStream_t)stream>>>(x, out, H, W, C, pad);
    NPS_CHECK_LAUNCH("circular_pad");
    return 0;
}

extern "C" int nps_circular_fold(const float* gp, float* gx, int B, int H, int W, int C, int pad, void* stream) {
    NPS_CHECK_ARG(gp && gx && B > 0 && H > 0 && W > 0 && C > 0 && pad >= 0, "circular_fold: bad args");
    circ_fold_kernel<<<dim3(grid_for((long)H * W * C, 256 * 8, 2048), B), 256, 0, (hipStream_t)stream>>>(gp, gx, H, W,
                                                                                                         C, pad);
    NPS_CHECK_LAUNCH("circular_fold");
    return 0;
}

extern "C" int nps_scaled_diff(const float* a, const float* b, const double* scale, float* out, long n, void* stream) {
    NPS_CHECK_ARG(a && b && scale && out && n > 0, "scaled_diff: bad args");
    scaled_diff_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(a, b, scale, out, n);
    NPS_CHECK_LAUNCH("scaled_diff");
    return 0;
}

extern "C" int nps_frame_pack_bwd(const nps_conv2d_t* ap, const float* gy, float* const* dsrc, float* dgamma,
                                  float* dbeta, double* work, void* stream) {
    return nps_frame_pack_bwd_tagged(ap, gy, dsrc, nullptr, dgamma, dbeta, work, stream);
}

namespace {
int frame_pack_bwd_impl(const nps_conv2d_t* ap, const float* gy, const float* gy_plain, float* const* dsrc,
                        float* const* dtag, float* dgamma, float* dbeta, double* work, bool work_zeroed, void* stream);
}  // namespace

extern "C" int nps_frame_pack_bwd_tagged(const nps_conv2d_t* ap, const float* gy, float* const* dsrc,
                                         float* const* dtag, float* dgamma, float* dbeta, double* work,
                                         void* stream) {
    return frame_pack_bwd_impl(ap, gy, nullptr, dsrc, dtag, dgamma, dbeta, work, false, stream);
}

extern "C" int nps_frame_pack_bwd2(const nps_conv2d_t* ap, const float* gy, const float* gy_plain, float* const* dsrc,
                                   float* const* dtag, float* dgamma, float* dbeta, double* work, void* stream) {
    return frame_pack_bwd_impl(ap, gy, gy_plain, dsrc, dtag, dgamma, dbeta, work, true, stream);
}

namespace {
int frame_pack_bwd_impl(const nps_conv2d_t* ap, const float* gy, const float* gy_plain, float* const* dsrc,
                        float* const* dtag, float* dgamma, float* dbeta, double* work, bool work_zeroed, void* stream) {
    NPS_CHECK_ARG(ap && gy && dsrc, "frame_pack_bwd: null");
    const nps_conv2d_t& a = *ap;
    NPS_CHECK_ARG(a.nsrc >= 1 && a.nsrc <= NPS_MAX_SRC && a.B > 0 && a.Hin > 0 && a.Win > 0 && a.Cin > 0,
                  "frame_pack_bwd: bad frame");
    int csum = 0;
    for (int i = 0; i < a.nsrc; ++i) csum += a.src[i].C;
    NPS_CHECK_ARG(csum == a.Cin, "frame_pack_bwd: Cin mismatch");
    NPS_CHECK_ARG(!a.gn_stats || (a.gn_groups > 0 && a.gn_groups <= 16 && a.Cin % a.gn_groups == 0 && a.gn_gamma &&
                                  a.gn_beta && work),
                  "frame_pack_bwd: bad GroupNorm");
    hipStream_t s = (hipStream_t)stream;
    // quad kernels: every channel count a multiple of 4 (so is the GroupNorm group), 16-B aligned tensors
    bool quad = (a.Cin & 3) == 0 && a.Cin <= 1024 && (reinterpret_cast<size_t>(gy) & 15) == 0 &&
                (!a.gn_stats || ((a.Cin / a.gn_groups) & 3) == 0);
    quad = quad && (reinterpret_cast<size_t>(gy_plain) & 15) == 0;
    for (int i = 0; i < a.nsrc; ++i)
        quad = quad && (a.src[i].C & 3) == 0 && (reinterpret_cast<size_t>(a.src[i].ptr) & 15) == 0 &&
               (dsrc[i] == nullptr || (reinterpret_cast<size_t>(dsrc[i]) & 15) == 0);
    const int npix = a.Hin * a.Win;
    // pixels per block of the quad kernels: 256, halved (down to 64) while the grid has < ~4 blocks per CU — at the
    // per-GPU batch of the 8-GPU run (B = 2) the 256-pixel blocks left the CUs 2 blocks each and the frame
    // backward latency-bound (training B = 2: 66.0 -> 64.7 ms per step at 128 / 64 pixels, same box;
    // profiles/r6/experiments/train_b2_knob_sweep.jsonl); B = 16 keeps 256
    int PXB = 256;
    while (PXB > 64 && (long)((npix + PXB - 1) / PXB) * a.B < 1000) PXB >>= 1;
    if (a.gn_stats) {
        NPS_CHECK_ARG(a.Cin <= 4096, "frame_pack_bwd: Cin too large");
        if (!work_zeroed && hipMemsetAsync(work, 0, sizeof(double) * 2 * a.B * a.Cin, s) != hipSuccess) {
            nps::set_error("frame_pack_bwd: memset failed");
            return -2;
        }
        const long n = (long)npix * a.Cin;
        if (quad)
            frame_bwd_reduce4_kernel<<<dim3((npix + PXB - 1) / PXB, a.B), 256, sizeof(float) * 2 * a.Cin, s>>>(
                a, gy, work, PXB);
        else
            frame_bwd_reduce_kernel<<<dim3(grid_for(n, 256 * 16, 1024), a.B), 256, sizeof(float) * 2 * a.Cin, s>>>(
                a, gy, work);
        NPS_CHECK_LAUNCH("frame_pack_bwd reduce");
    }
    long nmax = 1, pmax = 1;
    for (int i = 0; i < a.nsrc; ++i) {
        nmax = std::max(nmax, (long)a.src[i].H * a.src[i].W * a.src[i].C);
        pmax = std::max(pmax, (long)a.src[i].H * a.src[i].W);
    }
    float* d[3] = {dsrc[0], a.nsrc > 1 ? dsrc[1] : nullptr, a.nsrc > 2 ? dsrc[2] : nullptr};
    float* t[3] = {nullptr, nullptr, nullptr};
    for (int i = 0; dtag != nullptr && i < a.nsrc; ++i) t[i] = d[i] != nullptr ? dtag[i] : nullptr;
    if (quad) {
        frame_bwd_apply4_kernel<<<dim3((unsigned)((pmax + PXB - 1) / PXB), a.B, a.nsrc), 256, 0, s>>>(
            a, gy, work, d[0], d[1], d[2], dgamma, dbeta, PXB, t[0], t[1], t[2], gy_plain);
        NPS_CHECK_LAUNCH("frame_pack_bwd apply");
        return 0;
    }
    frame_bwd_apply_kernel<<<dim3(grid_for(nmax, 256 * 8, 2048), a.B, a.nsrc), 256, 0, s>>>(a, gy, work, d[0], d[1],
                                                                                           d[2], dgamma, dbeta, gy_plain);
    NPS_CHECK_LAUNCH("frame_pack_bwd apply");
    for (int i = 0; i < a.nsrc; ++i)  // (the element-wise kernel publishes no tags: one absmax pass per source)
        if (t[i] != nullptr && nps_absmax(d[i], (long)a.B * a.src[i].H * a.src[i].W * a.src[i].C, t[i], stream) != 0)
            return -2;
    return 0;
}
}  // namespace
