// Split-fp16 (3-pass) weight gradient for gfx950 (MI355X): the NPS_PREC_X3F16 arithmetic of the
// forward convs applied to G[m][n][tap] += sum_{b,p} A[b][p][m] * Xext[b][p + tap - pad][n]
// (nps_conv2d_wgrad_x3, include/nps.h) — the weight output of aten convolution_backward for the
// stride-1 undilated 1x1 / 2x2 / 3x3 convs of models/common.py:37-47, 93-120 (and the space-to-depth /
// phase forms of the stride-2 and transposed ones).  The fp32 wgrad_kernel (backward.hip) stays the
// path for dilated and 5x5 convs.
//
// GEMM view: M = A channels, N = X channels, K = A pixels.  v_mfma_f32_32x32x16_f16 takes 8 consecutive
// K values per lane, i.e. 8 consecutive pixels of one row: the A tile is staged transposed, [m][px], and
// the X patch [n][patch row][col].  A tap (ky, kx) shifts the X run by kx pixels, which breaks the 16-B
// alignment of the run; each lane reads 12 halves (b128 + b64) of its patch row once per (row, ky) and
// builds the KW shifted runs in registers (even shifts: dword renaming, odd: v_alignbyte).
// Operands are range-scaled by exact powers of two (max |a|, max |x| -> [2^13, 2^14), from range tags
// computed by nps_absmax) and split hi + lo; every product is hi*hi + hi*lo + lo*hi in one fp32
// accumulator (~2^-21 relative per product, the fp32 class of the reference's FMA chain).
#include "conv2d_common.hpp"

#include <type_traits>

namespace {

constexpr int WX_TH = 4, WX_TW = 16, WX_PX = WX_TH * WX_TW;  // 64 A pixels per tile (4 rows of 16)
constexpr int WX_APITCH = WX_PX + 8;                         // halves per A row: 144 B, conflict-free b128
constexpr int WX_PROW = 24;                                  // halves per staged patch row (16 + KW - 1 <= 24)

__host__ __device__ constexpr int wx_prows(int KH) { return WX_TH + KH - 1; }
// halves per patch channel: rows x 24 (+8 so consecutive channels start 16 B apart mod 256 B: conflict-free)
__host__ __device__ constexpr int wx_bpitch(int KH) { return wx_prows(KH) * WX_PROW + 8; }
__host__ __device__ constexpr size_t wx_lds_bytes(int KH) {
    return (size_t)2 * 2 * (64 * WX_APITCH + 64 * wx_bpitch(KH));  // [hi | lo] x (A + patch), fp16
}

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (N > 0) {
        static_for<N - 1>(f);
        f(std::integral_constant<int, N - 1>{});
    }
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// halves [s, s + 8) of the 12-half run d[0..5] (s compile-time, 0 <= s <= 4)
template <int S>
__device__ __forceinline__ f16x8 shifted_run(const unsigned (&d)[6]) {
    u32x4 r;
    if constexpr ((S & 1) == 0) {
        r = u32x4{d[S / 2], d[S / 2 + 1], d[S / 2 + 2], d[S / 2 + 3]};
    } else {
        constexpr int k = S / 2;
        r = u32x4{__builtin_amdgcn_alignbyte(d[k + 1], d[k], 2), __builtin_amdgcn_alignbyte(d[k + 2], d[k + 1], 2),
                  __builtin_amdgcn_alignbyte(d[k + 3], d[k + 2], 2), __builtin_amdgcn_alignbyte(d[k + 4], d[k + 3], 2)};
    }
    return __builtin_bit_cast(f16x8, r);
}

__device__ __forceinline__ f32x4 ld4c(const float* p, int C, int c) {  // channels [c, c+4) of one pixel row
    if ((C & 3) == 0 && c + 4 <= C) return *reinterpret_cast<const f32x4*>(p + c);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (c + e < C) v[e] = p[c + e];
    return v;
}

// Work-group (4 waves, 256 threads) = 64 m x 64 n x KH*KW taps over a range of pixel tiles (split K);
// wave (wm, wn) owns 32 m x 32 n x taps, one 32x32 accumulator per tap.  Per tile every thread fetches
// 2 pixels x 4 channels of A (pixel pairs along a row) and of the patch into registers, then splits them
// into the LDS planes with packed 2-pixel writes.
template <int KH, int KW>
__global__ __launch_bounds__(256, 2) void wgrad_x3_kernel(const nps_wgrad_t p, const float* a_range,
                                                          const float* x_range, int ntiles, int tiles_per_split,
                                                          int n_nt) {
    constexpr int NT = KH * KW;
    constexpr int PR = wx_prows(KH), PC = WX_TW + KW - 1;  // patch rows / useful columns
    constexpr int PCE = (PC + 1) & ~1;                       // fetched columns (pixel pairs)
    constexpr int BP = wx_bpitch(KH);
    constexpr int NA = WX_PX / 2 * 16 / 256;                 // A pixel-pair quads per thread (2)
    constexpr int NB = (PR * PCE / 2 * 16 + 255) / 256;      // patch pixel-pair quads per thread
    extern __shared__ __attribute__((aligned(16))) _Float16 wsm[];
    _Float16* Ah = wsm;
    _Float16* Al = Ah + 64 * WX_APITCH;
    _Float16* Bh = Al + 64 * WX_APITCH;
    _Float16* Bl = Bh + 64 * BP;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1, h = lane >> 5;
    const int nt = blockIdx.x % n_nt, mt = blockIdx.x / n_nt;
    const int m0 = mt * 64, n0 = nt * 64;
    const int tiles_x = (p.Wa + WX_TW - 1) / WX_TW, tiles_y = (p.Ha + WX_TH - 1) / WX_TH;
    const int Hext = p.Hx + 2 * p.circ, Wext = p.Wx + 2 * p.circ;
    const int t_begin = blockIdx.y * tiles_per_split;
    const int t_end = min(ntiles, t_begin + tiles_per_split);
    if (t_begin >= t_end) return;
    const float sa = pow2_scale_for(nps::tag_read(a_range));
    const float sx = pow2_scale_for(nps::tag_read(x_range));

    f32x4 ra[NA][2], rb[NB][2];
    auto issue = [&](int t) {
        const int b = t / (tiles_y * tiles_x);
        const int rr = t - b * tiles_y * tiles_x;
        const int oy0 = (rr / tiles_x) * WX_TH, ox0 = (rr % tiles_x) * WX_TW;
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const int idx = tid + k * 256;
            const int pp = idx >> 4, mq = idx & 15;  // pixel pair pp: pixels 2pp, 2pp + 1 (one row)
            const int oy = oy0 + (2 * pp) / WX_TW, ox = ox0 + (2 * pp) % WX_TW;
            const int m = m0 + mq * 4;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (oy < p.Ha && ox + j < p.Wa && m < p.M)
                    v = ld4c(p.a + ((size_t)(b * p.Ha + oy) * p.Wa + ox + j) * p.M, p.M, m);
                ra[k][j] = v;
            }
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int idx = tid + k * 256;
            const int pp = idx >> 4, nq = idx & 15;
            const int pr = (2 * pp) / PCE, pc = (2 * pp) % PCE;
            const int n = n0 + nq * 4;
            const int ye = oy0 + pr - p.pad_y;
            const bool rok = pr < PR && ye >= 0 && ye < Hext && n < p.N;
            const int y = p.circ ? nps::wrap_mod(ye - p.circ, p.Hx) : ye;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int xe = ox0 + pc + j - p.pad_x;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (rok && pc + j < PC && xe >= 0 && xe < Wext) {
                    const int x = p.circ ? nps::wrap_mod(xe - p.circ, p.Wx) : xe;
                    v = ld4c(p.x + ((size_t)(b * p.Hx + y) * p.Wx + x) * p.N, p.N, n);
                }
                rb[k][j] = v;
            }
        }
    };
    // split a pixel pair's 4 channels into (hi, lo) fp16 and write each channel's 2 pixels as one b32
    auto put = [&](_Float16* H, _Float16* L, int base, int pitch, const f32x4& v0, const f32x4& v1, float s) {
        f16x4 h0, l0, h1, l1;
        split4(v0 * s, h0, l0);
        split4(v1 * s, h1, l1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            *reinterpret_cast<h2f*>(H + base + e * pitch) = h2f{h0[e], h1[e]};
            *reinterpret_cast<h2f*>(L + base + e * pitch) = h2f{l0[e], l1[e]};
        }
    };
    auto commit = [&]() {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const int idx = tid + k * 256;
            const int pp = idx >> 4, mq = idx & 15;
            put(Ah, Al, mq * 4 * WX_APITCH + 2 * pp, WX_APITCH, ra[k][0], ra[k][1], sa);
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int idx = tid + k * 256;
            const int pp = idx >> 4, nq = idx & 15;
            const int pr = (2 * pp) / PCE, pc = (2 * pp) % PCE;
            if (pr < PR) put(Bh, Bl, nq * 4 * BP + pr * WX_PROW + pc, BP, rb[k][0], rb[k][1], sx);
        }
    };

    f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
    const int arow = (wm * 32 + (lane & 31)) * WX_APITCH + h * 8;
    const int brow = (wn * 32 + (lane & 31)) * BP + h * 8;

    // the fetch registers are dead during the MFMA loop (register budget: 144 accumulators); the second
    // work-group of the CU computes while this one fetches
    for (int t = t_begin; t < t_end; ++t) {
        issue(t);
        __syncthreads();  // the previous tile's reads of the LDS planes are done
        commit();
        __syncthreads();
#pragma unroll
        for (int r = 0; r < WX_TH; ++r) {
            const f16x8 ah = *reinterpret_cast<const f16x8*>(Ah + arow + r * WX_TW);
            const f16x8 al = *reinterpret_cast<const f16x8*>(Al + arow + r * WX_TW);
#pragma unroll
            for (int ky = 0; ky < KH; ++ky) {
                unsigned dh[6], dl[6];
                {
                    const _Float16* ph = Bh + brow + (r + ky) * WX_PROW;
                    const _Float16* pl = Bl + brow + (r + ky) * WX_PROW;
                    const u32x4 h4 = *reinterpret_cast<const u32x4*>(ph);
                    const u32x4 l4 = *reinterpret_cast<const u32x4*>(pl);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        dh[e] = h4[e];
                        dl[e] = l4[e];
                    }
                    if constexpr (KW > 1) {
                        const u32x2 h2 = *reinterpret_cast<const u32x2*>(ph + 8);
                        const u32x2 l2 = *reinterpret_cast<const u32x2*>(pl + 8);
                        dh[4] = h2[0];
                        dh[5] = h2[1];
                        dl[4] = l2[0];
                        dl[5] = l2[1];
                    } else {
                        dh[4] = dh[5] = dl[4] = dl[5] = 0u;
                    }
                }
                static_for<KW>([&](auto kxc) {
                    constexpr int kx = decltype(kxc)::value;
                    const f16x8 bh = shifted_run<kx>(dh), bl = shifted_run<kx>(dl);
                    f32x16& c = acc[ky * KW + kx];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
                });
            }
        }
    }

    // this split's partial into G: lane holds rows (r/4)*8 + h*4 + r%4, column lane%32
    const float inv = 1.f / (sa * sx);
    const int n = n0 + wn * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
            const int m = m0 + wm * 32 + (rr >> 2) * 8 + h * 4 + (rr & 3);
            if (m < p.M && n < p.N) atomicAdd(p.g + ((size_t)m * p.N + n) * NT + i, acc[i][rr] * inv);
        }
    }
}

template <int KH, int KW>
int launch_wgrad_x3(const nps_wgrad_t& p, const float* ar, const float* xr, hipStream_t s) {
    const long tiles_x = (p.Wa + WX_TW - 1) / WX_TW, tiles_y = (p.Ha + WX_TH - 1) / WX_TH;
    const long ntiles = (long)p.B * tiles_y * tiles_x;
    NPS_CHECK_ARG(ntiles < (1L << 30), "conv2d_wgrad_x3: too many tiles");
    const int n_mt = (p.M + 63) / 64, n_nt = (p.N + 63) / 64;
    const long base = (long)n_mt * n_nt;
    // split K (pixel tiles) so the grid puts ~4 work-groups on each of the 256 CUs, >= 8 tiles each
    long splits = (1024 + base - 1) / base;
    const long max_splits = (ntiles + 7) / 8;
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    const int per = (int)((ntiles + splits - 1) / splits);
    splits = (ntiles + per - 1) / per;
    NPS_CHECK_ARG(base < (1L << 31) && splits < 65536, "conv2d_wgrad_x3: grid too large");
    const size_t lds = wx_lds_bytes(KH);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)wgrad_x3_kernel<KH, KW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr_set = true;
    }
    wgrad_x3_kernel<KH, KW><<<dim3((unsigned)base, (unsigned)splits), 256, lds, s>>>(p, ar, xr, (int)ntiles, per, n_nt);
    NPS_CHECK_LAUNCH("conv2d_wgrad_x3");
    return 0;
}

}  // namespace

extern "C" int nps_conv2d_wgrad_x3(const nps_wgrad_t* pp, const float* a_range, const float* x_range, void* stream) {
    NPS_CHECK_ARG(pp != nullptr && a_range != nullptr && x_range != nullptr, "conv2d_wgrad_x3: null");
    const nps_wgrad_t& p = *pp;
    NPS_CHECK_ARG(p.a && p.x && p.g && p.B > 0 && p.Ha > 0 && p.Wa > 0 && p.M > 0 && p.Hx > 0 && p.Wx > 0 && p.N > 0,
                  "conv2d_wgrad_x3: bad shape");
    NPS_CHECK_ARG(p.dil == 1 && p.circ >= 0 && p.KH == p.KW && (p.KH == 1 || p.KH == 2 || p.KH == 3),
                  "conv2d_wgrad_x3: kernel %dx%d dil %d unsupported (1x1 / 2x2 / 3x3, undilated)", p.KH, p.KW, p.dil);
    hipStream_t s = (hipStream_t)stream;
    switch (p.KH) {
        case 1: return launch_wgrad_x3<1, 1>(p, a_range, x_range, s);
        case 2: return launch_wgrad_x3<2, 2>(p, a_range, x_range, s);
        default: return launch_wgrad_x3<3, 3>(p, a_range, x_range, s);
    }
}
