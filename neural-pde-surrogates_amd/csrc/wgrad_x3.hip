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

#include <cstdlib>
#include <type_traits>

namespace {

constexpr int WX_TH = 4, WX_TW = 16, WX_PX = WX_TH * WX_TW;  // 64 A pixels per tile (4 rows of 16)
constexpr int WX_APITCH = WX_PX + 8;                         // halves per A row: 144 B, conflict-free b128
constexpr int WX_PROW = 24;                                  // halves per staged patch row (16 + KW - 1 <= 24)

__host__ __device__ constexpr int wx_prows(int KH) { return WX_TH + KH - 1; }
// halves per patch channel: rows x 24 (+8 so consecutive channels start 16 B apart mod 256 B: conflict-free)
__host__ __device__ constexpr int wx_bpitch(int KH) { return wx_prows(KH) * WX_PROW + 8; }
__host__ __device__ constexpr size_t wx_lds_bytes(int KH) {
    return (size_t)2 * 2 * 2 * (64 * WX_APITCH + 64 * wx_bpitch(KH));  // 2 buffers x [hi | lo] x (A + patch)
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

// 16 zero bytes: the fetch address of every slot outside the tile / frame / channel range, so the producers'
// loads are unconditional and the compiler's in-order vmcnt waits stay exact (a load skipped on one path
// makes them drain the newest loads too)
__device__ __attribute__((aligned(16))) float wx_zero4[4];

// Bias gradient beside the weight gradient (nps_wgrad_t.db, a = dy): the A staging threads of the work-groups of
// n-tile 0 (each A element is staged once per n-tile) sum the raw values they stage, per channel quad, over their
// split; the 16 lanes of a quarter-wave that stage one quad combine their sums, and one lane adds each channel into
// the workspace's bias row wsb[M] (zeroed with the partials, stored into db by the fold) — the separate
// nps_channel_sums pass over dy and its zero-fill are gone.
__device__ __forceinline__ void db_flush(float* wsb, int m, int M, f32x4 s) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += __shfl_xor(s[e], o);
    if ((threadIdx.x & 15) == 0)
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (m + e < M) atomicAdd(wsb + m + e, s[e]);
}

// Work-group (8 waves, 512 threads, one per CU) = 64 m x 64 n x KH*KW taps over a range of pixel tiles
// (split K).  Wave w owns 32 m x 32 n (wm = w & 1, wn = (w >> 1) & 1) and half the taps: waves 0-3 taps
// [0, NT0), waves 4-7 taps [NT0, NT) — one 32x32 accumulator per tap; waves w and w + 4 share a SIMD, so
// every SIMD carries all the taps of one (m, n) block.  A 1x1 conv splits the tile's pixel rows instead
// (both halves add into the same G entries).  Every wave also stages: each lane fetches pixel pairs (2
// pixels along a row x 4 channels per slot) two tiles ahead into one of two register sets, and after its
// MFMAs of tile i splits tile i + 1 into the other LDS buffer (VALU beside the partner wave's MFMAs); one
// barrier per tile.  Lanes 0-15 of a wave-quarter take 16 consecutive pixel pairs, so the packed 2-pixel
// b32 writes of one instruction hit distinct banks.
// Grid: base = n_mt * n_nt (m, n) tiles x splits pixel ranges, 1-D.  With splits % 8 == 0 the (tile, split) of
// work-group l is XCD-aware: work-groups are dealt to the 8 XCDs round-robin (l % 8), and the `base` tiles of
// one split — which read the same A and X pixels (each tile its own 64-channel slices) — are consecutive
// work-groups of ONE XCD, so the pixels come from HBM once and from that XCD's L2 for the other tiles (for a
// 1x1 conv the kernel is bound by those reads: 3 m-tiles x 3 n-tiles read every byte 3 times).
template <int KH, int KW>
__global__ __launch_bounds__(512) void wgrad_x3_kernel(const nps_wgrad_t p, const float* a_range,
                                                       const float* x_range, float* __restrict__ ws, int ntiles,
                                                       int tiles_per_split, int n_nt, int base, int xcd_remap,
                                                       float* wsb) {
    constexpr int NT = KH * KW;
    constexpr bool ROWSPLIT = NT == 1;
    constexpr int NT0 = ROWSPLIT ? 1 : (NT + 1) / 2;       // taps of waves 0-3
    constexpr int NTW = NT0;                                 // accumulators per wave (max over the halves)
    constexpr int PR = wx_prows(KH), PC = WX_TW + KW - 1;  // patch rows / useful columns
    constexpr int PCE = (PC + 1) & ~1;                       // fetched columns (pixel pairs)
    constexpr int PPR = PCE / 2;                             // pixel pairs per patch row
    constexpr int BP = wx_bpitch(KH);
    constexpr int NPA = WX_PX / 2;                           // A pixel pairs (32)
    constexpr int NPB = PR * PPR;                            // patch pixel pairs
    constexpr int GA = (NPA + 15) / 16, GB = (NPB + 15) / 16;  // groups of 16 pixel pairs
    constexpr int NA = (GA * 4 * 64 + 511) / 512;            // slots per lane (x 4 channel quads)
    constexpr int NB = (GB * 4 * 64 + 511) / 512;
    constexpr int BUF = 2 * (64 * WX_APITCH + 64 * BP);      // halves per LDS buffer
    extern __shared__ __attribute__((aligned(16))) _Float16 wsm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int tile, split;
    if (xcd_remap) {
        const int j = blockIdx.x >> 3;  // this work-group's rank on its XCD
        tile = j % base;
        split = (j / base) * 8 + (blockIdx.x & 7);
    } else {
        tile = blockIdx.x % base;
        split = blockIdx.x / base;
    }
    const int nt = tile % n_nt, mt = tile / n_nt;
    const int m0 = mt * 64, n0 = nt * 64;
    const int tiles_x = (p.Wa + WX_TW - 1) / WX_TW, tiles_y = (p.Ha + WX_TH - 1) / WX_TH;
    const int t_begin = split * tiles_per_split;
    const int t_end = min(ntiles, t_begin + tiles_per_split);
    if (t_begin >= t_end) return;
    const int nloc = t_end - t_begin;
    const float sa = pow2_scale_for(nps::tag_read(a_range));
    const float sx = pow2_scale_for(nps::tag_read(x_range));
    const int Hext = p.Hx + 2 * p.circ, Wext = p.Wx + 2 * p.circ;

    // ---- staging: per-slot geometry, fixed for the work-group (only the tile origin changes): slot k of
    // this lane is group-of-16 g = (tid + 512 k) >> 6 — pair block g % G, channel block g / G — so the
    // per-tile address arithmetic is a few adds and compares (no integer division)
    int a_r[NA], a_c[NA], a_m[NA], a_lds[NA];
    bool a_ok[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        const int idx = tid + k * 512, l = idx & 63, g = idx >> 6;
        const int pp = (l & 15) + 16 * (g % GA), mq = (l >> 4) + 4 * (g / GA);
        const bool in = g < GA * 4 && pp < NPA;
        a_r[k] = (2 * pp) / WX_TW;
        a_c[k] = (2 * pp) % WX_TW;
        a_m[k] = m0 + mq * 4;
        a_ok[k] = in && a_m[k] < p.M;
        a_lds[k] = in ? mq * 4 * WX_APITCH + 2 * pp : -1;
    }
    int b_r[NB], b_c[NB], b_n[NB], b_lds[NB];
    bool b_ok[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const int idx = tid + k * 512, l = idx & 63, g = idx >> 6;
        const int pp = (l & 15) + 16 * (g % GB), nq = (l >> 4) + 4 * (g / GB);
        const bool in = g < GB * 4 && pp < NPB;
        b_r[k] = pp / PPR;
        b_c[k] = 2 * (pp % PPR);
        b_n[k] = n0 + nq * 4;
        b_ok[k] = in && b_n[k] < p.N;
        b_lds[k] = in ? nq * 4 * BP + b_r[k] * WX_PROW + b_c[k] : -1;
    }
    // frame coordinate of an extended-frame coordinate e (0 <= e < H + 2 circ), without a division
    auto wrap = [&](int e, int H) {
        int v = e - p.circ;
        v = v < 0 ? v + H : v;
        return v >= H ? v - H : v;
    };
    auto issue = [&](int t, f32x4 (&ra)[NA][2], f32x4 (&rb)[NB][2]) {
        const int b = t / (tiles_y * tiles_x);
        const int rr = t - b * tiles_y * tiles_x;
        const int oy0 = (rr / tiles_x) * WX_TH, ox0 = (rr % tiles_x) * WX_TW;
        const float* ab = p.a + (size_t)b * p.Ha * p.Wa * p.M;
        const float* xb = p.x + (size_t)b * p.Hx * p.Wx * p.N;
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const int oy = oy0 + a_r[k], ox = ox0 + a_c[k];
            const bool ok = a_ok[k] && oy < p.Ha;
#pragma unroll
            for (int j = 0; j < 2; ++j) {  // unconditional loads (zero page outside): exact vmcnt waits
                const float* src = (ok && ox + j < p.Wa) ? ab + ((size_t)oy * p.Wa + ox + j) * p.M + a_m[k] : wx_zero4;
                ra[k][j] = *reinterpret_cast<const f32x4*>(src);
            }
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int ye = oy0 + b_r[k] - p.pad_y;
            const bool rok = b_ok[k] && ye >= 0 && ye < Hext;
            const int y = wrap(ye, p.Hx);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int xe = ox0 + b_c[k] + j - p.pad_x;
                const bool ok = rok && b_c[k] + j < PC && xe >= 0 && xe < Wext;
                const float* src = ok ? xb + ((size_t)y * p.Wx + wrap(xe, p.Wx)) * p.N + b_n[k] : wx_zero4;
                rb[k][j] = *reinterpret_cast<const f32x4*>(src);
            }
        }
    };
    // split a pixel pair's 4 channels into (hi, lo) fp16; each channel's 2 pixels are one b32 write
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
    const bool dbo = wsb != nullptr && nt == 0;  // bias-gradient partials (db_flush)
    f32x4 dbs[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) dbs[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto commit = [&](int i, const f32x4 (&ra)[NA][2], const f32x4 (&rb)[NB][2]) {
        _Float16* Ah = wsm + (i & 1) * BUF;
        _Float16* Al = Ah + 64 * WX_APITCH;
        _Float16* Bh = Al + 64 * WX_APITCH;
        _Float16* Bl = Bh + 64 * BP;
#pragma unroll
        for (int k = 0; k < NA; ++k)
            if (a_lds[k] >= 0) {
                put(Ah, Al, a_lds[k], WX_APITCH, ra[k][0], ra[k][1], sa);
                if (dbo) dbs[k] += ra[k][0] + ra[k][1];
            }
#pragma unroll
        for (int k = 0; k < NB; ++k)
            if (b_lds[k] >= 0) put(Bh, Bl, b_lds[k], BP, rb[k][0], rb[k][1], sx);
    };

    // ---- MFMA part
    const int wm = wave & 1, wn = (wave >> 1) & 1, half = wave >> 2, h = lane >> 5;
    f32x16 acc[NTW];
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
    const int arow = (wm * 32 + (lane & 31)) * WX_APITCH + h * 8;
    const int brow = (wn * 32 + (lane & 31)) * BP + h * 8;
    // tap (ky, kx) of this wave's half -> its accumulator; the half's taps are a compile-time range per branch
    auto compute_half = [&](const _Float16* Ah, const _Float16* Al, const _Float16* Bh, const _Float16* Bl,
                            auto T0c, auto T1c, auto R0c, auto R1c) {
        constexpr int T0 = decltype(T0c)::value, T1 = decltype(T1c)::value;
        constexpr int R0 = decltype(R0c)::value, R1 = decltype(R1c)::value;
        static_for<R1 - R0>([&](auto rc) {
            constexpr int r = R0 + decltype(rc)::value;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(Ah + arow + r * WX_TW);
            const f16x8 al = *reinterpret_cast<const f16x8*>(Al + arow + r * WX_TW);
            static_for<KH>([&](auto kyc) {
                constexpr int ky = decltype(kyc)::value;
                if constexpr (ky * KW + KW > T0 && ky * KW < T1) {  // this row of taps meets [T0, T1)
                    unsigned dh[6], dl[6];
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
                    static_for<KW>([&](auto kxc) {
                        constexpr int kx = decltype(kxc)::value;
                        constexpr int tap = ky * KW + kx;
                        if constexpr (tap >= T0 && tap < T1) {
                            const f16x8 bh = shifted_run<kx>(dh), bl = shifted_run<kx>(dl);
                            f32x16& c = acc[tap - T0];
                            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
                            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
                            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
                        }
                    });
                }
            });
        });
    };
    auto compute = [&](int i) {
        const _Float16* Ah = wsm + (i & 1) * BUF;
        const _Float16* Al = Ah + 64 * WX_APITCH;
        const _Float16* Bh = Al + 64 * WX_APITCH;
        const _Float16* Bl = Bh + 64 * BP;
        using I = std::integral_constant<int, 0>;
        if constexpr (ROWSPLIT) {
            if (half == 0)
                compute_half(Ah, Al, Bh, Bl, I{}, std::integral_constant<int, 1>{}, I{},
                             std::integral_constant<int, WX_TH / 2>{});
            else
                compute_half(Ah, Al, Bh, Bl, I{}, std::integral_constant<int, 1>{},
                             std::integral_constant<int, WX_TH / 2>{}, std::integral_constant<int, WX_TH>{});
        } else {
            if (half == 0)
                compute_half(Ah, Al, Bh, Bl, I{}, std::integral_constant<int, NT0>{}, I{},
                             std::integral_constant<int, WX_TH>{});
            else
                compute_half(Ah, Al, Bh, Bl, std::integral_constant<int, NT0>{}, std::integral_constant<int, NT>{},
                             I{}, std::integral_constant<int, WX_TH>{});
        }
    };

    // ---- pipeline: local tile i is fetched into set i & 1 two tiles ahead, split into buffer i & 1 after
    // the MFMAs of tile i - 1 (buffer (i - 1) & 1), computed after the next barrier
    f32x4 a0[NA][2], b0[NB][2], a1[NA][2], b1[NB][2];
    issue(t_begin, a0, b0);
    if (nloc > 1) issue(t_begin + 1, a1, b1);
    commit(0, a0, b0);
    __syncthreads();  // tile 0 staged
    for (int i = 0; i < nloc; i += 2) {
        if (i + 2 < nloc) issue(t_begin + i + 2, a0, b0);
        compute(i);
        if (i + 1 < nloc) commit(i + 1, a1, b1);
        __syncthreads();  // tile i read (buffer free), tile i + 1 staged
        if (i + 1 >= nloc) break;
        if (i + 3 < nloc) issue(t_begin + i + 3, a1, b1);
        compute(i + 1);
        if (i + 2 < nloc) commit(i + 2, a0, b0);
        __syncthreads();
    }

    if (dbo) {
#pragma unroll
        for (int k = 0; k < NA; ++k)
            if (a_lds[k] >= 0) db_flush(wsb, a_m[k], p.M, dbs[k]);  // (a_lds: uniform per 16-lane group)
    }
    // this split's partial into the tap-major workspace W[tap][m][n]: lane holds rows (r/4)*8 + h*4 + r%4,
    // column lane%32, so one atomic wave-instruction covers two 128-B runs (the full-rate shape; the
    // [m][n][tap] order of G would scatter the 64 lanes 36 B apart)
    const float inv = 1.f / (sa * sx);
    const int n = n0 + wn * 32 + (lane & 31);
    const int tbase = ROWSPLIT ? 0 : half * NT0;
    const int ntw = ROWSPLIT ? 1 : (half == 0 ? NT0 : NT - NT0);
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
        if (i >= ntw) continue;
        float* wt = ws + (size_t)(tbase + i) * p.M * p.N;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
            const int m = m0 + wm * 32 + (rr >> 2) * 8 + h * 4 + (rr & 3);
            if (m < p.M && n < p.N) atomicAdd(wt + (size_t)m * p.N + n, acc[i][rr] * inv);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// 1x1 weight gradient with 192 x 192 work-group tiles: G[m][n] += sum_p A[p][m] X[p][n] over the flat pixel
// range (a 1x1 conv's dy and input share their pixels).  The 64 x 64 tiles of wgrad_x3_kernel stage every
// pixel for only 64 x 64 MACs and re-stage it once per (m, n) tile (3 x 3 tiles at M = N = 192), which left the
// 1x1 class at 0.09 of 833 TF/s; here one work-group covers up to 192 m x 192 n, so each staged pixel feeds
// 192 x 192 MACs and A, X are read once per m-tile / n-tile pair.
//   * 512 threads: threads 0-255 stage A, 256-511 stage X — 32-pixel tiles, each thread 3 items of (pixel pair,
//     channel quad): two 16-B loads, split hi + lo, four packed 2-pixel b32 writes per half into [channel][pixel]
//     LDS rows (80-B pitch: the MFMA operand reads are conflict-free ds_read_b128), two LDS buffers;
//   * wave w computes m [96 (w & 1), +96) x n [96 ((w >> 1) & 1), +96) (3 x 3 accumulators of 32 x 32) over
//     pixels [16 (w >> 2), +16) of each tile: one K-step of v_mfma_f32_32x32x16_f16, 27 MFMAs (3 passes) per
//     tile; the two pixel halves add into the same G entries;
//   * split K over pixel tiles (XCD-aware order as wgrad_x3_kernel), fp32 atomics into W[m][n], fold into G.
constexpr int W1_TP = 32;              // pixels per tile
constexpr int W1_PITCH = W1_TP + 8;    // halves per LDS channel row
constexpr int W1_ROWS = 192;           // channel rows per operand (the work-group's m or n range)
constexpr int W1_BUF = 2 * 2 * W1_ROWS * W1_PITCH;  // halves per buffer: [A | X] x [hi | lo]
constexpr size_t W1_LDS = (size_t)2 * W1_BUF * 2;   // two buffers, bytes

__global__ __launch_bounds__(512) void wgrad1_wide_kernel(const nps_wgrad_t p, const float* a_range,
                                                          const float* x_range, float* __restrict__ ws,
                                                          long npix, int ntiles, int tiles_per_split, int n_nt,
                                                          int base, int xcd_remap, float* wsb) {
    extern __shared__ __attribute__((aligned(16))) _Float16 w1sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int tile, split;
    if (xcd_remap) {
        const int j = blockIdx.x >> 3;
        tile = j % base;
        split = (j / base) * 8 + (blockIdx.x & 7);
    } else {
        tile = blockIdx.x % base;
        split = blockIdx.x / base;
    }
    const int mt = tile / n_nt, nt = tile % n_nt;
    const int m0 = mt * W1_ROWS, n0 = nt * W1_ROWS;
    const int t_begin = split * tiles_per_split;
    const int t_end = min(ntiles, t_begin + tiles_per_split);
    if (t_begin >= t_end) return;
    const float sa = pow2_scale_for(nps::tag_read(a_range));
    const float sx = pow2_scale_for(nps::tag_read(x_range));

    // ---- staging role: threads 0-255 A (channels m0..), 256-511 X (channels n0..)
    const bool isx = tid >= 256;
    const int st = tid & 255;
    const float* src = isx ? p.x : p.a;
    const int C = isx ? p.N : p.M;
    const int c0 = isx ? n0 : m0;
    const float scale = isx ? sx : sa;
    int it_pp[3], it_c[3];
    bool it_ok[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // item = (pixel pair pp of 16, channel quad cq of 48)
        const int i = st + 256 * k;
        it_pp[k] = i & 15;
        it_c[k] = (i >> 4) * 4;  // channel offset in the 192-row block
        it_ok[k] = c0 + it_c[k] < C;
    }
    auto issue = [&](int t, f32x4 (&r)[3][2]) {
        const long pbase = (long)t * W1_TP;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const long px = pbase + 2 * it_pp[k] + j;
                const float* q = (it_ok[k] && px < npix) ? src + px * C + c0 + it_c[k] : wx_zero4;
                r[k][j] = *reinterpret_cast<const f32x4*>(q);
            }
    };
    const bool dbo = wsb != nullptr && nt == 0 && !isx;  // bias-gradient partials of the A stagers (db_flush)
    f32x4 dbs[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    auto commit = [&](int i, const f32x4 (&r)[3][2]) {
        _Float16* H = w1sm + (i & 1) * W1_BUF + (isx ? 2 * W1_ROWS * W1_PITCH : 0);
        _Float16* L = H + W1_ROWS * W1_PITCH;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (dbo) dbs[k] += r[k][0] + r[k][1];
            f16x4 h0, l0, h1, l1;
            split4(r[k][0] * scale, h0, l0);
            split4(r[k][1] * scale, h1, l1);
            const int base_o = it_c[k] * W1_PITCH + 2 * it_pp[k];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                *reinterpret_cast<h2f*>(H + base_o + e * W1_PITCH) = h2f{h0[e], h1[e]};
                *reinterpret_cast<h2f*>(L + base_o + e * W1_PITCH) = h2f{l0[e], l1[e]};
            }
        }
    };

    // ---- MFMA role
    const int wm = wave & 1, wn = (wave >> 1) & 1, half = wave >> 2, h = lane >> 5;
    f32x16 acc[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int koff = 16 * half + 8 * h;  // this lane's 8 pixels of the tile
    auto compute = [&](int i) {
        const _Float16* Ah = w1sm + (i & 1) * W1_BUF;
        const _Float16* Al = Ah + W1_ROWS * W1_PITCH;
        const _Float16* Xh = Al + W1_ROWS * W1_PITCH;
        const _Float16* Xl = Xh + W1_ROWS * W1_PITCH;
        f16x8 ah[3], al[3], bh[3], bl[3];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const int ra = (wm * 96 + b * 32 + (lane & 31)) * W1_PITCH + koff;
            const int rb = (wn * 96 + b * 32 + (lane & 31)) * W1_PITCH + koff;
            ah[b] = *reinterpret_cast<const f16x8*>(Ah + ra);
            al[b] = *reinterpret_cast<const f16x8*>(Al + ra);
            bh[b] = *reinterpret_cast<const f16x8*>(Xh + rb);
            bl[b] = *reinterpret_cast<const f16x8*>(Xl + rb);
        }
#pragma unroll
        for (int bm = 0; bm < 3; ++bm)
#pragma unroll
            for (int bn = 0; bn < 3; ++bn) {
                f32x16& c = acc[bm][bn];
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bm], bh[bn], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bm], bl[bn], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[bm], bh[bn], c, 0, 0, 0);
            }
    };

    // ---- pipeline: tile i + 1 fetched into registers while tile i is computed, then split into the other buffer
    const int nloc = t_end - t_begin;
    f32x4 r[3][2];
    issue(t_begin, r);
    commit(0, r);
    __syncthreads();
    for (int i = 0; i < nloc; ++i) {
        if (i + 1 < nloc) issue(t_begin + i + 1, r);
        compute(i);
        if (i + 1 < nloc) commit(i + 1, r);
        __syncthreads();
    }

    if (dbo) {
#pragma unroll
        for (int k = 0; k < 3; ++k) db_flush(wsb, m0 + it_c[k], p.M, dbs[k]);
    }
    // ---- partial into W[m][n]: lane holds rows (rr/4)*8 + h*4 + rr%4 of each block, column lane%32
    const float inv = 1.f / (sa * sx);
#pragma unroll
    for (int bm = 0; bm < 3; ++bm)
#pragma unroll
        for (int bn = 0; bn < 3; ++bn) {
            const int n = n0 + wn * 96 + bn * 32 + (lane & 31);
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                const int m = m0 + wm * 96 + bm * 32 + (rr >> 2) * 8 + h * 4 + (rr & 3);
                if (m < p.M && n < p.N) atomicAdd(ws + (size_t)m * p.N + n, acc[bm][bn][rr] * inv);
            }
        }
}

// ---------------------------------------------------------------------------------------------
// 2x2 weight gradient with 128 m x 128 n work-group tiles (the space-to-depth Downsample and the transposed
// conv's phase form: M = 192, N = 4 x 192).  wgrad_x3_kernel's 64 x 64 tiles use each staged pixel for 64 x 64
// MACs per tap and re-stage it per (m, n) tile; here a 32-pixel tile (2 rows x 16) of A [m][px] and its 3 x 18
// patch of X [n][row][col] feed 128 x 128 x 4 taps.  Wave w: m [64 (w & 1), +64) x n [64 ((w >> 1) & 1), +64)
// (2 x 2 accumulators of 32 x 32) for the taps of kernel row ky = w >> 2 (both kx: the patch row is read once,
// the kx = 1 run built in registers as in wgrad_x3_kernel); one K-step (16 pixels = one row) per MFMA.
constexpr int W2_TH = 2, W2_TW = 16, W2_TP = W2_TH * W2_TW;
constexpr int W2_APITCH = W2_TP + 8;              // halves per A row
constexpr int W2_PROW = 24;                        // halves per patch row (17 used)
constexpr int W2_PR = W2_TH + 1;                   // patch rows
constexpr int W2_BPITCH = W2_PR * W2_PROW + 8;     // halves per patch channel
constexpr int W2_ROWS = 128;
constexpr int W2_BUF = 2 * W2_ROWS * W2_APITCH + 2 * W2_ROWS * W2_BPITCH;  // halves per buffer
constexpr size_t W2_LDS = (size_t)2 * W2_BUF * 2;

__global__ __launch_bounds__(512) void wgrad2_wide_kernel(const nps_wgrad_t p, const float* a_range,
                                                          const float* x_range, float* __restrict__ ws, int ntiles,
                                                          int tiles_per_split, int n_nt, int base, int xcd_remap,
                                                          float* wsb) {
    constexpr int PC = W2_TW + 1, PPR = (PC + 1) / 2;  // useful patch columns, pixel pairs per patch row (9)
    constexpr int NPB = W2_PR * PPR;                    // patch pixel pairs (27)
    extern __shared__ __attribute__((aligned(16))) _Float16 w2sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int tile, split;
    if (xcd_remap) {
        const int j = blockIdx.x >> 3;
        tile = j % base;
        split = (j / base) * 8 + (blockIdx.x & 7);
    } else {
        tile = blockIdx.x % base;
        split = blockIdx.x / base;
    }
    const int mt = tile / n_nt, nt = tile % n_nt;
    const int m0 = mt * W2_ROWS, n0 = nt * W2_ROWS;
    const int tiles_x = (p.Wa + W2_TW - 1) / W2_TW, tiles_y = (p.Ha + W2_TH - 1) / W2_TH;
    const int t_begin = split * tiles_per_split;
    const int t_end = min(ntiles, t_begin + tiles_per_split);
    if (t_begin >= t_end) return;
    const float sa = pow2_scale_for(nps::tag_read(a_range));
    const float sx = pow2_scale_for(nps::tag_read(x_range));
    const int Hext = p.Hx + 2 * p.circ, Wext = p.Wx + 2 * p.circ;

    // staging slots: A item = (pixel pair pp of 16, channel quad of 32): one per thread; B items = (patch pair of
    // 27, channel quad of 32): two per thread (864 of 1024 used).  Lanes 0-15 of a wave-quarter take 16
    // consecutive pairs, so the packed 2-pixel b32 writes of one instruction hit distinct banks.
    const int a_pp = tid & 15, a_q = tid >> 4;
    const int a_r = (2 * a_pp) / W2_TW, a_c = (2 * a_pp) % W2_TW, a_m = m0 + 4 * a_q;
    const bool a_ok = a_m < p.M;
    const int a_lds = 4 * a_q * W2_APITCH + 2 * a_pp;
    int b_r[2], b_c[2], b_n[2], b_lds[2];
    bool b_ok[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int idx = tid + 512 * k, l = idx & 15, g = idx >> 4;  // g: group of 16 pairs
        const int ngrp = (NPB + 15) / 16;                          // 2 pair-groups per channel quad
        const int pp = l + 16 * (g % ngrp), nq = g / ngrp;
        const bool in = nq < W2_ROWS / 4 && pp < NPB;
        b_r[k] = pp / PPR;
        b_c[k] = 2 * (pp % PPR);
        b_n[k] = n0 + 4 * nq;
        b_ok[k] = in && b_n[k] < p.N;
        b_lds[k] = in ? 4 * nq * W2_BPITCH + b_r[k] * W2_PROW + b_c[k] : -1;
    }
    auto wrap = [&](int e, int H) {
        int v = e - p.circ;
        v = v < 0 ? v + H : v;
        return v >= H ? v - H : v;
    };
    auto issue = [&](int t, f32x4 (&ra)[2], f32x4 (&rb)[2][2]) {
        const int b = t / (tiles_y * tiles_x);
        const int rr = t - b * tiles_y * tiles_x;
        const int oy0 = (rr / tiles_x) * W2_TH, ox0 = (rr % tiles_x) * W2_TW;
        const float* ab = p.a + (size_t)b * p.Ha * p.Wa * p.M;
        const float* xb = p.x + (size_t)b * p.Hx * p.Wx * p.N;
        {
            const int oy = oy0 + a_r, ox = ox0 + a_c;
            const bool ok = a_ok && oy < p.Ha;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float* src = (ok && ox + j < p.Wa) ? ab + ((size_t)oy * p.Wa + ox + j) * p.M + a_m : wx_zero4;
                ra[j] = *reinterpret_cast<const f32x4*>(src);
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int ye = oy0 + b_r[k] - p.pad_y;
            const bool rok = b_ok[k] && ye >= 0 && ye < Hext;
            const int y = wrap(ye, p.Hx);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int xe = ox0 + b_c[k] + j - p.pad_x;
                const bool ok = rok && b_c[k] + j < PC && xe >= 0 && xe < Wext;
                const float* src = ok ? xb + ((size_t)y * p.Wx + wrap(xe, p.Wx)) * p.N + b_n[k] : wx_zero4;
                rb[k][j] = *reinterpret_cast<const f32x4*>(src);
            }
        }
    };
    auto put = [&](_Float16* H, _Float16* L, int base_o, int pitch, const f32x4& v0, const f32x4& v1, float sc) {
        f16x4 h0, l0, h1, l1;
        split4(v0 * sc, h0, l0);
        split4(v1 * sc, h1, l1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            *reinterpret_cast<h2f*>(H + base_o + e * pitch) = h2f{h0[e], h1[e]};
            *reinterpret_cast<h2f*>(L + base_o + e * pitch) = h2f{l0[e], l1[e]};
        }
    };
    const bool dbo = wsb != nullptr && nt == 0;  // bias-gradient partials (db_flush)
    f32x4 dbs = {0.f, 0.f, 0.f, 0.f};
    auto commit = [&](int i, const f32x4 (&ra)[2], const f32x4 (&rb)[2][2]) {
        _Float16* Ah = w2sm + (i & 1) * W2_BUF;
        _Float16* Al = Ah + W2_ROWS * W2_APITCH;
        _Float16* Bh = Al + W2_ROWS * W2_APITCH;
        _Float16* Bl = Bh + W2_ROWS * W2_BPITCH;
        put(Ah, Al, a_lds, W2_APITCH, ra[0], ra[1], sa);
        if (dbo) dbs += ra[0] + ra[1];
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (b_lds[k] >= 0) put(Bh, Bl, b_lds[k], W2_BPITCH, rb[k][0], rb[k][1], sx);
    };

    // MFMA role
    const int wm = wave & 1, wn = (wave >> 1) & 1, ky = wave >> 2, h = lane >> 5;
    f32x16 acc[2][2][2];  // [kx][m block][n block]
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[x][i][j][r] = 0.f;
    auto compute = [&](int i) {
        const _Float16* Ah = w2sm + (i & 1) * W2_BUF;
        const _Float16* Al = Ah + W2_ROWS * W2_APITCH;
        const _Float16* Bh = Al + W2_ROWS * W2_APITCH;
        const _Float16* Bl = Bh + W2_ROWS * W2_BPITCH;
#pragma unroll
        for (int r = 0; r < W2_TH; ++r) {
            f16x8 ah[2], al[2];
#pragma unroll
            for (int bm = 0; bm < 2; ++bm) {
                const int ra = (wm * 64 + bm * 32 + (lane & 31)) * W2_APITCH + r * W2_TW + 8 * h;
                ah[bm] = *reinterpret_cast<const f16x8*>(Ah + ra);
                al[bm] = *reinterpret_cast<const f16x8*>(Al + ra);
            }
#pragma unroll
            for (int bn = 0; bn < 2; ++bn) {
                const int rb = (wn * 64 + bn * 32 + (lane & 31)) * W2_BPITCH + (r + ky) * W2_PROW + 8 * h;
                unsigned dh[6], dl[6];
                const u32x4 h4 = *reinterpret_cast<const u32x4*>(Bh + rb);
                const u32x4 l4 = *reinterpret_cast<const u32x4*>(Bl + rb);
                const u32x2 h2 = *reinterpret_cast<const u32x2*>(Bh + rb + 8);
                const u32x2 l2 = *reinterpret_cast<const u32x2*>(Bl + rb + 8);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    dh[e] = h4[e];
                    dl[e] = l4[e];
                }
                dh[4] = h2[0];
                dh[5] = h2[1];
                dl[4] = l2[0];
                dl[5] = l2[1];
                static_for<2>([&](auto kxc) {
                    constexpr int kx = decltype(kxc)::value;
                    const f16x8 bh = shifted_run<kx>(dh), bl = shifted_run<kx>(dl);
#pragma unroll
                    for (int bm = 0; bm < 2; ++bm) {
                        f32x16& c = acc[kx][bm][bn];
                        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bm], bh, c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bm], bl, c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[bm], bh, c, 0, 0, 0);
                    }
                });
            }
        }
    };

    const int nloc = t_end - t_begin;
    f32x4 ra[2], rb[2][2];
    issue(t_begin, ra, rb);
    commit(0, ra, rb);
    __syncthreads();
    for (int i = 0; i < nloc; ++i) {
        if (i + 1 < nloc) issue(t_begin + i + 1, ra, rb);
        compute(i);
        if (i + 1 < nloc) commit(i + 1, ra, rb);
        __syncthreads();
    }

    if (dbo) db_flush(wsb, a_m, p.M, dbs);
    const float inv = 1.f / (sa * sx);
#pragma unroll
    for (int kx = 0; kx < 2; ++kx) {
        float* wt = ws + (size_t)(ky * 2 + kx) * p.M * p.N;
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int bn = 0; bn < 2; ++bn) {
                const int n = n0 + wn * 64 + bn * 32 + (lane & 31);
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) {
                    const int m = m0 + wm * 64 + bm * 32 + (rr >> 2) * 8 + h * 4 + (rr & 3);
                    if (m < p.M && n < p.N) atomicAdd(wt + (size_t)m * p.N + n, acc[kx][bm][bn][rr] * inv);
                }
            }
    }
}

// G[m][n][tap] += W[tap][m][n] (acc), or = (nps_conv2d_wgrad_x3_set: G need not be zeroed first); the same for
// the bias row (db += / = wsb) when the launch computed one
__global__ void wgrad_fold_kernel(const float* __restrict__ w, float* __restrict__ g, int MN, int nt, int acc,
                                  const float* __restrict__ wsb, float* __restrict__ db, int M) {
    const long total = (long)MN * nt;
    for (long o = (long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (long)gridDim.x * blockDim.x) {
        const long mn = o / nt;
        const int t = (int)(o - mn * nt);
        const float v = w[(size_t)t * MN + mn];
        g[o] = acc ? g[o] + v : v;
    }
    if (db != nullptr)
        for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < M; m += gridDim.x * blockDim.x)
            db[m] = acc ? db[m] + wsb[m] : wsb[m];
}

// Work-groups of the split-K grid: 2 per CU in turn (the first one's atomics overlap the second one's tiles), but 1
// per CU for small pixel counts (the per-GPU batch of the 8-GPU run, B = 2 at <= 260^2): there each work-group's
// split was only 26-90 tiles, and the per-split fixed costs (prologue, 36 K partial atomics) halved with half the
// splits — x3w_1tap 4.57 -> 3.61 ms, x3w_9tap 12.16 -> 11.43 ms per training step at B = 2 (same box;
// profiles/r6/experiments/train_b2_knob_sweep.jsonl; 1024 and a larger minimum split were slower)
inline long wx_wgs(const nps_wgrad_t& p) { return (long)p.B * p.Ha * p.Wa <= 200000 ? 256 : 512; }
constexpr long WX_MINT = 8;  // minimum pixel tiles per split
// dev knob NPS_WX_REMAP=0: the plain (tile-fastest) work-group order
const int g_wx_remap = [] {
    const char* e = std::getenv("NPS_WX_REMAP");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
}();

template <int KH, int KW>
int launch_wgrad_x3(const nps_wgrad_t& p, const float* ar, const float* xr, float* ws, hipStream_t s,
                       int acc) {
    const long tiles_x = (p.Wa + WX_TW - 1) / WX_TW, tiles_y = (p.Ha + WX_TH - 1) / WX_TH;
    const long ntiles = (long)p.B * tiles_y * tiles_x;
    NPS_CHECK_ARG(ntiles < (1L << 30), "conv2d_wgrad_x3: too many tiles");
    const int n_mt = (p.M + 63) / 64, n_nt = (p.N + 63) / 64;
    const long base = (long)n_mt * n_nt;
    // split K (pixel tiles): at most 2 work-groups in turn per CU (the first one's atomics overlap the
    // second one's tiles; a grid just past a multiple of 256 would add a nearly empty round), >= 8 tiles each
    long splits = wx_wgs(p) / base;
    const long max_splits = (ntiles + WX_MINT - 1) / WX_MINT;
    if (splits > max_splits) splits = max_splits;
    if (splits >= 16) splits &= ~7L;  // a multiple of 8: the XCD-aware tile order (kernel comment)
    if (splits < 1) splits = 1;
    const int per = (int)((ntiles + splits - 1) / splits);
    const long used = (ntiles + per - 1) / per;  // splits that own tiles (the rest exit at once)
    const int remap = (splits % 8 == 0 && g_wx_remap) ? 1 : 0;
    if (!remap) splits = used;
    NPS_CHECK_ARG(base * splits < (1L << 31), "conv2d_wgrad_x3: grid too large");
    const size_t lds = wx_lds_bytes(KH);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)wgrad_x3_kernel<KH, KW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr_set = true;
    }
    const size_t MN = (size_t)p.M * p.N;
    float* wsb = p.db != nullptr ? ws + MN * KH * KW : nullptr;  // bias row behind the partials (db_flush)
    if (hipMemsetAsync(ws, 0, sizeof(float) * (MN * KH * KW + (wsb ? p.M : 0)), s) != hipSuccess) {
        nps::set_error("conv2d_wgrad_x3: workspace memset failed");
        return -2;
    }
    wgrad_x3_kernel<KH, KW><<<(unsigned)(base * splits), 512, lds, s>>>(p, ar, xr, ws, (int)ntiles, per, n_nt,
                                                                         (int)base, remap, wsb);
    NPS_CHECK_LAUNCH("conv2d_wgrad_x3");
    const long total = (long)MN * KH * KW;
    const long nb = (total + 255) / 256;
    wgrad_fold_kernel<<<(unsigned)(nb < 2048 ? nb : 2048), 256, 0, s>>>(ws, p.g, (int)MN, KH * KW, acc, wsb, p.db, p.M);
    NPS_CHECK_LAUNCH("conv2d_wgrad_x3 (fold)");
    return 0;
}

// 1x1 weight gradient on wgrad1_wide_kernel (dy and x on the same pixels: no padding / circular extension)
int launch_wgrad1_wide(const nps_wgrad_t& p, const float* ar, const float* xr, float* ws, hipStream_t s,
                       int acc) {
    const long npix = (long)p.B * p.Ha * p.Wa;
    const long ntiles = (npix + W1_TP - 1) / W1_TP;
    NPS_CHECK_ARG(ntiles < (1L << 30), "conv2d_wgrad_x3 (1x1): too many tiles");
    const int n_mt = (p.M + W1_ROWS - 1) / W1_ROWS, n_nt = (p.N + W1_ROWS - 1) / W1_ROWS;
    const long base = (long)n_mt * n_nt;
    long splits = wx_wgs(p) / base;  // two work-groups per CU in turn (LDS: 120 KiB each, one resident)
    const long max_splits = (ntiles + WX_MINT - 1) / WX_MINT;
    if (splits > max_splits) splits = max_splits;
    if (splits >= 16) splits &= ~7L;
    if (splits < 1) splits = 1;
    const int per = (int)((ntiles + splits - 1) / splits);
    const long used = (ntiles + per - 1) / per;
    const int remap = (splits % 8 == 0 && g_wx_remap) ? 1 : 0;
    if (!remap) splits = used;
    NPS_CHECK_ARG(base * splits < (1L << 31), "conv2d_wgrad_x3 (1x1): grid too large");
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)wgrad1_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)W1_LDS);
        attr_set = true;
    }
    const size_t MN = (size_t)p.M * p.N;
    float* wsb = p.db != nullptr ? ws + MN : nullptr;
    if (hipMemsetAsync(ws, 0, sizeof(float) * (MN + (wsb ? p.M : 0)), s) != hipSuccess) {
        nps::set_error("conv2d_wgrad_x3: workspace memset failed");
        return -2;
    }
    wgrad1_wide_kernel<<<(unsigned)(base * splits), 512, W1_LDS, s>>>(p, ar, xr, ws, npix, (int)ntiles, per, n_nt,
                                                                       (int)base, remap, wsb);
    NPS_CHECK_LAUNCH("conv2d_wgrad_x3 (1x1 wide)");
    const long nb = ((long)MN + 255) / 256;
    wgrad_fold_kernel<<<(unsigned)(nb < 2048 ? nb : 2048), 256, 0, s>>>(ws, p.g, (int)MN, 1, acc, wsb, p.db, p.M);
    NPS_CHECK_LAUNCH("conv2d_wgrad_x3 (fold)");
    return 0;
}

// 2x2 weight gradient on wgrad2_wide_kernel (128 x 128 work-group tiles)
int launch_wgrad2_wide(const nps_wgrad_t& p, const float* ar, const float* xr, float* ws, hipStream_t s,
                       int acc) {
    const long tiles_x = (p.Wa + W2_TW - 1) / W2_TW, tiles_y = (p.Ha + W2_TH - 1) / W2_TH;
    const long ntiles = (long)p.B * tiles_y * tiles_x;
    NPS_CHECK_ARG(ntiles < (1L << 30), "conv2d_wgrad_x3 (2x2): too many tiles");
    const int n_mt = (p.M + W2_ROWS - 1) / W2_ROWS, n_nt = (p.N + W2_ROWS - 1) / W2_ROWS;
    const long base = (long)n_mt * n_nt;
    long splits = wx_wgs(p) / base;
    const long max_splits = (ntiles + WX_MINT - 1) / WX_MINT;
    if (splits > max_splits) splits = max_splits;
    if (splits >= 16) splits &= ~7L;
    if (splits < 1) splits = 1;
    const int per = (int)((ntiles + splits - 1) / splits);
    const long used = (ntiles + per - 1) / per;
    const int remap = (splits % 8 == 0 && g_wx_remap) ? 1 : 0;
    if (!remap) splits = used;
    NPS_CHECK_ARG(base * splits < (1L << 31), "conv2d_wgrad_x3 (2x2): grid too large");
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)wgrad2_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)W2_LDS);
        attr_set = true;
    }
    const size_t MN = (size_t)p.M * p.N;
    float* wsb = p.db != nullptr ? ws + MN * 4 : nullptr;
    if (hipMemsetAsync(ws, 0, sizeof(float) * (MN * 4 + (wsb ? p.M : 0)), s) != hipSuccess) {
        nps::set_error("conv2d_wgrad_x3: workspace memset failed");
        return -2;
    }
    wgrad2_wide_kernel<<<(unsigned)(base * splits), 512, W2_LDS, s>>>(p, ar, xr, ws, (int)ntiles, per, n_nt, (int)base,
                                                                       remap, wsb);
    NPS_CHECK_LAUNCH("conv2d_wgrad_x3 (2x2 wide)");
    const long nb = ((long)MN * 4 + 255) / 256;
    wgrad_fold_kernel<<<(unsigned)(nb < 2048 ? nb : 2048), 256, 0, s>>>(ws, p.g, (int)MN, 4, acc, wsb, p.db, p.M);
    NPS_CHECK_LAUNCH("conv2d_wgrad_x3 (fold)");
    return 0;
}

// dev knob NPS_WX_WIDE1=0: 1x1 weight gradients on the 64 x 64 tiles of wgrad_x3_kernel
const int g_wx_wide1 = [] {
    const char* e = std::getenv("NPS_WX_WIDE1");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
}();
// dev knob NPS_WX_WIDE2=0: 2x2 weight gradients on the 64 x 64 tiles of wgrad_x3_kernel
const int g_wx_wide2 = [] {
    const char* e = std::getenv("NPS_WX_WIDE2");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
}();

}  // namespace

// partials [KH*KW][M][N] + the bias row [M] (nps_wgrad_t.db)
extern "C" size_t nps_wgrad_x3_ws_floats(int M, int N, int KH, int KW) { return (size_t)M * N * KH * KW + M; }

namespace {
int wgrad_x3_dispatch(const nps_wgrad_t* pp, const float* a_range, const float* x_range, float* ws, void* stream,
                      int acc) {
    NPS_CHECK_ARG(pp != nullptr && a_range != nullptr && x_range != nullptr && ws != nullptr, "conv2d_wgrad_x3: null");
    const nps_wgrad_t& p = *pp;
    NPS_CHECK_ARG(p.a && p.x && p.g && p.B > 0 && p.Ha > 0 && p.Wa > 0 && p.M > 0 && p.Hx > 0 && p.Wx > 0 && p.N > 0,
                  "conv2d_wgrad_x3: bad shape");
    NPS_CHECK_ARG(p.dil == 1 && p.circ >= 0 && p.KH == p.KW && (p.KH == 1 || p.KH == 2 || p.KH == 3),
                  "conv2d_wgrad_x3: kernel %dx%d dil %d unsupported (1x1 / 2x2 / 3x3, undilated)", p.KH, p.KW, p.dil);
    NPS_CHECK_ARG((p.M & 3) == 0 && (p.N & 3) == 0 && (reinterpret_cast<size_t>(p.a) & 15) == 0 &&
                      (reinterpret_cast<size_t>(p.x) & 15) == 0,
                  "conv2d_wgrad_x3: channel counts %d, %d must be multiples of 4 (16-B pixel quads)", p.M, p.N);
    hipStream_t s = (hipStream_t)stream;
    switch (p.KH) {
        case 1:
            if (g_wx_wide1 && p.pad_y == 0 && p.pad_x == 0 && p.circ == 0 && p.Ha == p.Hx && p.Wa == p.Wx)
                return launch_wgrad1_wide(p, a_range, x_range, ws, s, acc);
            return launch_wgrad_x3<1, 1>(p, a_range, x_range, ws, s, acc);
        case 2:
            // (the wide kernel needs M, N > 64 to beat the 64 x 64 tiles)
            if (g_wx_wide2 && p.M > 64 && p.N > 64) return launch_wgrad2_wide(p, a_range, x_range, ws, s, acc);
            return launch_wgrad_x3<2, 2>(p, a_range, x_range, ws, s, acc);
        default: return launch_wgrad_x3<3, 3>(p, a_range, x_range, ws, s, acc);
    }
}
}  // namespace

extern "C" int nps_conv2d_wgrad_x3(const nps_wgrad_t* pp, const float* a_range, const float* x_range, float* ws,
                                   void* stream) {
    return wgrad_x3_dispatch(pp, a_range, x_range, ws, stream, 1);
}

extern "C" int nps_conv2d_wgrad_x3_set(const nps_wgrad_t* pp, const float* a_range, const float* x_range, float* ws,
                                       void* stream) {
    return wgrad_x3_dispatch(pp, a_range, x_range, ws, stream, 0);
}
