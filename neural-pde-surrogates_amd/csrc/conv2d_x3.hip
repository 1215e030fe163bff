// Split-fp16 (3-pass) implicit-GEMM 2-D convolution for gfx950 (MI355X), NHWC activations:
// the NPS_PREC_X3F16 arithmetic of nps_conv2d_fwd (include/nps.h) for every stride-1, undilated
// 1x1 / 2x2 / 3x3 conv of the reference's grid path (models/common.py:37-47, 93-120;
// proc_unet_modern.py, proc_fno.py:114-117, enc_grid.py, dec_grid.py).
#include "conv2d_common.hpp"

#include <cstdlib>
#include <type_traits>

namespace {

// ---------------------------------------------------------------------------------------------
// Split-fp16 producer/consumer conv (NPS_PREC_X3F16) for stride-1, undilated 1x1 / 2x2 / 3x3 convs.
// 512 threads.  Work-group = 64 output channels x TILE_PX = 4*PB*32 output pixels (TH x TW) of one
// sample; consumer wave w (0-3) owns 64 co x PB*32 px (2 x PB accumulators of 32x32, one per tile).
//   * LDS holds only the input patch: a ring of NST = 3 stages of 16 channels, each pixel as
//     [16 hi | 16 lo] fp16 + 16 B pad (80 B), patch rows padded to x3_row_bytes so the B-operand
//     ds_read_b128 are bank-conflict-free.  Producer waves 4-7 fetch
//     stage s+4 while stage s+2 is being committed (two register sets), so each global load has two
//     consumer stages to land; one s_barrier per stage.
//   * The weight fragments (2 KiB per (chunk, tap, 32-co block): [hi | lo] x 64 lanes x 16 B) are read
//     by the consumer waves straight from global memory (L2/L1-resident: all 4 waves read the same
//     bytes), two K-groups ahead in a 3-slot register ring, so LDS never carries the 9x-larger A tile.
//   * K-group = (stage, tap): 24 v_mfma_f32_32x32x16_f16 per wave (2 co x PB px tiles x 3 passes),
//     passes ordered hi*lo, hi*hi, lo*hi so the B registers are reloaded for the next group right
//     after their last use (lo after pass 1, hi after pass 3) — one B register set.
//   * Work-groups are numbered co-block fastest and remapped so consecutive numbers share an XCD
//     (the 3 co-blocks of a tile and neighbouring tiles read the same patch bytes from one L2).
__host__ __device__ constexpr int x3_patch_px_max(int ntaps, int tile_px) {
    // largest (TH + k - 1) * (TW + k - 1) over the tile shapes nps_conv2d_plan uses for tile_px
    // (25 taps: 5x5, 256-pixel tiles only — a 512-pixel 5x5 patch ring does not fit LDS; 128-pixel tiles:
    // the wide kernel, 8x16 / 4x32 / 16x8)
    return ntaps == 1      ? tile_px
           : ntaps == 25   ? (tile_px == 512 ? 12 * 68 : 12 * 36)
           : tile_px == 128 ? (ntaps == 4 ? 5 * 33 : 6 * 34)
                            : (tile_px == 512 ? (ntaps == 4 ? 9 * 65 : 10 * 66) : (ntaps == 4 ? 9 * 33 : 10 * 34));
}

#define X3_MFMA __builtin_amdgcn_mfma_f32_32x32x16_f16
// Producer slot -> patch pixel (slot idx holds channel quad idx & 3 of pixel idx >> 2)
__device__ __forceinline__ int x3_slot_px(int idx) { return idx >> 2; }

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (N > 0) {
        static_for<N - 1>(f);
        f(std::integral_constant<int, N - 1>{});
    }
}

// store target of the out-of-range items of the LDS store phase (never read)
__device__ __attribute__((aligned(64))) float x3_sink[256];
// 64 zero bytes: the fetch address of B elements outside the frame or past the channel tail, so the
// stage loop needs no masks (PMC: the 1x1 kernel issues 3-4k VALU instructions per wave)
__device__ __attribute__((aligned(64))) float x3_zero16[16];

// NHWC output with 4-aligned channels: the epilogue goes through LDS (x3_store_phase)
__host__ __device__ __forceinline__ bool x3_lds_epilogue(const nps_conv2d_t& a) {
    return !a.out_nchw && (a.out_C & 3) == 0 && (a.Cout & 3) == 0;
}

// All 512 threads store the work-group's NCO-channel x TILE_PX tile from LDS (T[pixel][NCO + 4]):
// NCO/4 consecutive threads cover one pixel's NCO channels (one contiguous run of the NHWC output), with
// the fused bias / addends / GELU / accumulate of store_tile, in the same float order.
template <int TILE_PX, int NCO>
__device__ __forceinline__ void x3_store_phase(const nps_conv2d_t& a, int b, int cob, int oy0, int ox0, int lat,
                                               int ph, const float* T, const float* btab, int tid, float& amax,
                                               double* red) {
    const int poy = a.out_off_y + (ph >> 1), pox = a.out_off_x + (ph & 1);  // transposed-conv phase offset
    constexpr int Q = NCO / 4;
    const bool st = a.out_stats != nullptr;
    double s1 = 0.0, s2 = 0.0;  // out_stats: fp64 sum / sum of squares of the stored values
    if (!a.accumulate && a.addend0 == nullptr && a.addend1 == nullptr) {
        // No operand to read: the bias comes from the LDS table and out-of-range items store to a sink, so the
        // loop holds no global load and no branch around a store.  (vmcnt retires loads and stores in one
        // in-order queue; with a conditional store per item the compiler waited vmcnt(0) at every item —
        // one store round trip each, 13-15k of a tile's ~115k cycles: DESIGN.md § Round 3.)
#pragma unroll 4
        for (int i = tid; i < TILE_PX * Q; i += 512) {
            const int P = i / Q, q = i - (i / Q) * Q;
            const int co0 = cob * NCO + q * 4;
            const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
            const int oy = oy0 + ti * lat, ox = ox0 + tj * lat;
            const int dy = oy * a.out_os + poy, dx = ox * a.out_os + pox;
            const bool ok = !(co0 >= a.Cout || oy >= a.Hout || ox >= a.Wout || dy < 0 || dy >= a.out_H || dx < 0 ||
                              dx >= a.out_W);
            const f32x4 acc = *reinterpret_cast<const f32x4*>(T + P * (NCO + 4) + q * 4);
            const f32x4 bi = *reinterpret_cast<const f32x4*>(btab + (ok ? co0 : 0));
            f32x4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = acc[e] + bi[e];
                if (a.act == 1) v = nps::gelu_erf(v);
                r[e] = v;
                amax = ok ? fmaxf(amax, fabsf(v)) : amax;
            }
            float* dst = ok ? a.out + ((((size_t)b * a.out_H + dy) * a.out_W + dx) * a.out_C + co0)
                            : x3_sink + 4 * (tid & 63);
            *reinterpret_cast<f32x4*>(dst) = r;
            if (st) {
                float f1 = 0.f, f2 = 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    f1 += r[e];
                    f2 += r[e] * r[e];
                }
                s1 += ok ? (double)f1 : 0.0;
                s2 += ok ? (double)f2 : 0.0;
            }
        }
        stats_publish_wg(a, b, s1, s2, red);
        return;
    }
#pragma unroll 4
    for (int i = tid; i < TILE_PX * Q; i += 512) {
        const int P = i / Q, q = i - (i / Q) * Q;
        const int co0 = cob * NCO + q * 4;
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        const int oy = oy0 + ti * lat, ox = ox0 + tj * lat;  // lat: dilation-lattice step (1 unless dilated)
        const int dy = oy * a.out_os + poy, dx = ox * a.out_os + pox;
        if (co0 >= a.Cout || oy >= a.Hout || ox >= a.Wout || dy < 0 || dy >= a.out_H || dx < 0 || dx >= a.out_W)
            continue;
        const f32x4 acc = *reinterpret_cast<const f32x4*>(T + P * (NCO + 4) + q * 4);
        const size_t o = (((size_t)b * a.out_H + dy) * a.out_W + dx) * a.out_C + co0;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 bi = *reinterpret_cast<const f32x4*>(btab + co0);
        const f32x4 a0 = a.addend0 ? *reinterpret_cast<const f32x4*>(a.addend0 + o) : z;
        const f32x4 a1 = a.addend1 ? *reinterpret_cast<const f32x4*>(a.addend1 + o) : z;
        const f32x4 ov = a.accumulate ? *reinterpret_cast<const f32x4*>(a.out + o) : z;
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v = acc[e] + bi[e];
            if (!a.add_after_act) v = v + a0[e] + a1[e];
            if (a.act == 1) v = nps::gelu_erf(v);
            if (a.add_after_act) v = v + a0[e] + a1[e];
            if (a.accumulate) v += ov[e];
            r[e] = v;
            amax = fmaxf(amax, fabsf(v));
        }
        *reinterpret_cast<f32x4*>(a.out + o) = r;
        if (st) {  // fp32 partials of the quad (as store_tile_s), one pair of fp64 adds per quad
            float f1 = 0.f, f2 = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                f1 += a.accumulate ? r[e] - ov[e] : r[e];
                f2 += a.accumulate ? (r[e] - ov[e]) * (r[e] + ov[e]) : r[e] * r[e];
            }
            s1 += (double)f1;
            s2 += (double)f2;
        }
    }
    stats_publish_wg(a, b, s1, s2, red);  // the next GroupNorm(1)'s moments of this sample: one pair per tile
}

// PRO: the frame prologue (GroupNorm affine and/or GELU, proc_unet_modern.py:62-99) is applied by the
// producers while staging, instead of a frame_pack pass in front of the conv.
// WIDE: the work-group covers 192 output channels x 128 pixels instead of 64 x 4*PB*32: consumer wave w
// owns channels [96 (w & 1), +96) (3 co blocks) x pixels [64 (w >> 1), +64) (2 pixel blocks).  The staged
// patch then feeds all 192 channels: 3x less producer work (fetch, split, prologue) and patch traffic per
// MFMA than three 64-channel work-groups re-staging the same patch.
template <int NTAPS, int PB, bool PRO, bool WIDE = false>
__global__ __launch_bounds__(512) void conv2d_x3_kernel(const nps_conv2d_t a) {
    constexpr int KWT = NTAPS == 25 ? 5 : (NTAPS == 9 ? 3 : (NTAPS == 4 ? 2 : 1));
    constexpr int CBW = WIDE ? 3 : 2;          // 32-channel co blocks per consumer wave
    constexpr int PBW = WIDE ? 2 : PB;         // 32-pixel blocks per consumer wave
    constexpr int NCO = WIDE ? 192 : 64;       // output channels per work-group
    constexpr int TILE_PX = WIDE ? 128 : 4 * PB * 32;
    constexpr int MAXP = (x3_patch_px_max(NTAPS, TILE_PX) * 4 + 255) / 256;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const Geo g = make_geo(a);
    const int ncob = (a.Cout + NCO - 1) / NCO;
    const int ntiles = g.tiles_x * g.tiles_y;
    const int nph = a.nphase > 1 ? a.nphase : 1;  // transposed-conv phases in this launch
    const int nwg = ntiles * a.B * ncob * nph;  // work-group tiles of the launch (the grid is persistent)
    // tile l -> (co block, sample, output origin): co block fastest; consecutive tiles of one XCD's
    // work-groups (l = i, i + G, ... with G % 8 == 0 stay on XCD i % 8) get consecutive numbers, so the 3
    // co-blocks of a tile and neighbouring tiles read the same patch bytes from that XCD's L2
    auto decode = [&](int l, int& cob, int& b, int& oy0, int& ox0, int& ph) {
        const int full = nwg & ~7;
        const int L0 = l < full ? (l & 7) * (full >> 3) + (l >> 3) : l;
        ph = L0 % nph;  // phase fastest: the phases of a tile share its patch bytes in one L2
        const int L = L0 / nph;
        cob = L % ncob;
        const int rest = L / ncob;
        const int tile = rest % ntiles;
        b = rest / ntiles;
        const int ty = tile / g.tiles_x, tx = tile - (tile / g.tiles_x) * g.tiles_x;
        // dilated convs tile on the dilation lattice (g.T = dil): tile (ty, tx) is lattice phase
        // (ty % T, tx % T), block (ty / T, tx / T); its pixels are oy0 + ti * T, ox0 + tj * T
        oy0 = (ty % g.T) + (ty / g.T) * a.TH * g.T;
        ox0 = (tx % g.T) + (tx / g.T) * a.TW * g.T;
    };
    const int npix = g.PH * g.PW;
    const int rowb = x3_row_bytes(a.TW, g.PW);  // LDS bytes per patch row (bank-conflict-free B reads)
    const int stage_b = g.PH * rowb;
    char* ring = reinterpret_cast<char*>(smem) + 128;
    // bias table of the LDS store phase, behind the ring / tile region (x3_lds_bytes); first read after the
    // first barrier of the tile loop
    float* btab = reinterpret_cast<float*>(ring + x3_region_bytes(a));
    for (int c = tid; c < a.Cout; c += 512) btab[c] = a.bias != nullptr ? a.bias[c] : 0.f;
    const int nstages = (a.Cin + CK - 1) / CK;
    const int last = nstages - 1;
    const bool lds_epi = WIDE || x3_lds_epilogue(a);  // wide tiles: always (x3_wide_eligible)
    auto barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

    // static priority for the producer half (MI355X_MICROARCH 'Two waves per SIMD' item 4): they win the
    // VALU arbitration against their SIMD partner's MFMA stream; same-box A/B: 3x3 class -1.7 % per call
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    if (wave >= 4) {
        // ------------------------------------------------------------------ producers: patch only
        const int ptid = tid - 256;
        const int Hext = a.Hin + 2 * a.circ, Wext = a.Win + 2 * a.circ;
        const float xs = (PRO && a.gn_stats != nullptr) ? gn_prologue_scale(a) : in_scale_of(a);
        // 1 / (elements per GroupNorm group), once per launch
        const double gn_icnt = (PRO && a.gn_stats != nullptr) ? 1.0 / ((double)(a.Cin / a.gn_groups) * a.Hin * a.Win) : 0.0;
        // a register set: MAXP patch slots, then (PRO) the stage's GroupNorm operands gamma[4], beta[4]
        // and the group's (sum, sum of squares) as two doubles, fetched with the patch
        constexpr int NR = MAXP + (PRO ? 3 : 0);
        f32x4 r0[NR], r1[NR];
        // Per-slot source addresses: the patch pixel of slot k is fixed for a tile, so its address in the
        // current source (and whether it lies inside it) is computed only when a stage's source (or the
        // tile) changes; a stage then costs one add + one load per slot.  Slot k holds channels
        // [4*gq, 4*gq + 4) of the stage, gq = ptid & 3 for every k.
        const int gq = ptid & 3;
        const float* sbase[MAXP];
        int soff[MAXP];  // LDS byte offset of each slot inside a stage (fixed for the launch)
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            const int idx = ptid + k * 256;
            const int p = x3_slot_px(idx);
            const int pr = p / g.PW, pc = p - pr * g.PW;
            soff[k] = pr * rowb + pc * X3_PIXB + (idx & 3) * 8;
        }
        unsigned pixm = 0;  // slots whose pixel lies inside the current source
        unsigned finm = 0;  // slots whose pixel lies inside the (circularly extended) frame
        int cur_src = -1;
        int fb = 0, fy0 = 0, fx0 = 0, fcob = 0, fph = 0;  // tile being fetched
        auto locate = [&](int sidx) {
            const nps_src_t S0 = a.src[0], S1 = a.src[1], S2 = a.src[2];
            const int si = a.s2d ? 0 : sidx;  // (the view's parities all read src[0])
            const float* sptr = si == 0 ? S0.ptr : (si == 1 ? S1.ptr : S2.ptr);
            const int sC = si == 0 ? S0.C : (si == 1 ? S1.C : S2.C);
            const int sH = si == 0 ? S0.H : (si == 1 ? S1.H : S2.H);
            const int sW = si == 0 ? S0.W : (si == 1 ? S1.W : S2.W);
            const int soy = si == 0 ? S0.off_y : (si == 1 ? S1.off_y : S2.off_y);
            const int sox = si == 0 ? S0.off_x : (si == 1 ? S1.off_x : S2.off_x);
            const int ybase = fy0 - a.pad_y, xbase = fx0 - a.pad_x;
            // space-to-depth view (a.s2d): sidx is the view's parity p, the source is src[0] at (2 y + (p >> 1)
            // - s2d_pad, 2 x + (p & 1) - s2d_pad)
            const int s2m = a.s2d ? 2 : 1;
            const int s2y = a.s2d ? (sidx >> 1) - a.s2d_pad : 0, s2x = a.s2d ? (sidx & 1) - a.s2d_pad : 0;
            pixm = 0;
            finm = 0;
#pragma unroll
            for (int k = 0; k < MAXP; ++k) {
                const int idx = ptid + k * 256;
                const int p = x3_slot_px(idx);
                const int pr = p / g.PW, pc = p - pr * g.PW;
                const int ye = ybase + pr * g.rstep, xe = xbase + pc * g.rstep;
                bool ok = p < npix && ye >= 0 && ye < Hext && xe >= 0 && xe < Wext;
                finm = ok ? (finm | (1u << k)) : finm;
                const int fy = a.circ ? nps::wrap_mod(ye - a.circ, a.Hin) : ye;
                const int fx = a.circ ? nps::wrap_mod(xe - a.circ, a.Win) : xe;
                const int yy = fy * s2m + s2y - soy, xx = fx * s2m + s2x - sox;
                ok = ok && yy >= 0 && yy < sH && xx >= 0 && xx < sW;
                sbase[k] = sptr + (ok ? ((size_t)(fb * sH + yy) * sW + xx) * sC : (size_t)fb * sH * sW * sC);
                pixm = ok ? (pixm | (1u << k)) : pixm;
            }
        };
        // issue() returns the mask of slots holding in-frame data; commit() zeroes the others
        auto issue = [&](int st, f32x4 (&rp)[NR]) -> unsigned {
            const int c0 = st * CK;
            const int cend = min(c0 + CK, a.Cin);
            int sidx = 0, cbase = 0;
            if (a.s2d) {  // space-to-depth view: the stage's parity (C % 16 == 0: one parity per stage)
                sidx = c0 / a.src[0].C;
                cbase = sidx * a.src[0].C;
            } else {
                int lo = 0;
#pragma unroll
                for (int si = 0; si < NPS_MAX_SRC; ++si) {  // unrolled: static kernarg indexing
                    if (si < a.nsrc) {
                        const int hi = lo + a.src[si].C;
                        if (c0 >= lo && cend <= hi) {  // host-checked (x3_sources_aligned): one source per stage
                            sidx = si;
                            cbase = lo;
                        }
                        lo = hi;
                    }
                }
            }
            if (sidx != cur_src) {  // uniform
                locate(sidx);
                cur_src = sidx;
            }
            // this lane's channel offset in the source pixel; lanes past the channel tail of the last stage
            // read the pixel's first channels instead (in bounds; zeroed at commit)
            const bool chok = c0 + gq * 4 < cend;
            const unsigned chm = chok ? ~0u : 0u;
            const int cs = chok ? c0 - cbase + gq * 4 : 0;
#pragma unroll
            for (int k = 0; k < MAXP; ++k)  // compiler-visible loads: waited before first use, spill-safe
                rp[k] = *reinterpret_cast<const f32x4*>(sbase[k] + cs);
            if constexpr (PRO) {
                // this lane's 4 frame channels share one group (host-checked: channels per group % 4 == 0);
                // without GroupNorm (or past the channel tail) the loads read the packed weights instead
                const int c = chok ? c0 + gq * 4 : 0;
                const bool gn = a.gn_stats != nullptr;
                const float* pg = gn ? a.gn_gamma + c : reinterpret_cast<const float*>(a.wpack);
                const float* pb = gn ? a.gn_beta + c : reinterpret_cast<const float*>(a.wpack);
                const double* ps = gn ? a.gn_stats + ((size_t)fb * a.gn_groups + c / (a.Cin / a.gn_groups)) * 2
                                      : reinterpret_cast<const double*>(a.wpack);
                rp[MAXP] = *reinterpret_cast<const f32x4*>(pg);
                rp[MAXP + 1] = *reinterpret_cast<const f32x4*>(pb);
                rp[MAXP + 2] = *reinterpret_cast<const f32x4*>(ps);
            }
            // bits 0-15: slot data lies inside the source; bits 16-31: slot pixel lies inside the frame
            return (pixm & chm) | ((finm & chm) << 16);
        };
        auto commit = [&](int st, const f32x4 (&rp)[NR], unsigned okm) {
            char* Pt = ring + (st % X3_NST) * stage_b;
            // GroupNorm as one FMA per element, y = x * gs + gb with gs = rstd * gamma, gb = beta - mean * gs
            // (the form PyTorch's GroupNorm kernel evaluates): the group moments -> (mean, rstd) once per stage
            // and lane (fp64 moments, one fp64 reciprocal of the count per launch, v_rsq_f32), not per element
            f32x4 gs = {1.f, 1.f, 1.f, 1.f}, gb = {0.f, 0.f, 0.f, 0.f};
            if constexpr (PRO) {
                if (a.gn_stats != nullptr) {  // as frame_pack_kernel / the reference's GroupNorm
                    const f32x4 sv = rp[MAXP + 2];
                    double s1, s2;
                    __builtin_memcpy(&s1, &sv, 8);
                    __builtin_memcpy(&s2, reinterpret_cast<const char*>(&sv) + 8, 8);
                    const double mu = s1 * gn_icnt;
                    double var = fma(s2, gn_icnt, -mu * mu);
                    var = var < 0.0 ? 0.0 : var;
                    const float mean = (float)mu;
                    const float rstd = __builtin_amdgcn_rsqf((float)(var + (double)a.gn_eps));
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        gs[e] = rstd * rp[MAXP][e];
                        gb[e] = fmaf(-mean, gs[e], rp[MAXP + 1][e]);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < MAXP; ++k) {
                const int idx = ptid + k * 256;
                if (x3_slot_px(idx) < npix) {
                    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                    f16x4 hi, lo;
                    f32x4 v = ((okm >> k) & 1u) ? rp[k] : z;
                    if constexpr (PRO) {
                        if ((okm >> (16 + k)) & 1u) {
                            if (a.gn_stats != nullptr) {
#pragma unroll
                                for (int e = 0; e < 4; ++e) v[e] = fmaf(v[e], gs[e], gb[e]);
                            }
                            if (a.pre_act == 1) {
#pragma unroll
                                for (int e = 0; e < 4; ++e) v[e] = nps::gelu_fast(v[e]);
                            }
                        } else {
                            v = z;  // the conv's own zero padding (and channels past Cin)
                        }
                    }
                    split4(v * xs, hi, lo);
                    char* base = Pt + soff[k];
                    *reinterpret_cast<f16x4*>(base) = hi;
                    *reinterpret_cast<f16x4*>(base + 32) = lo;
                }
            }
        };
        // Per tile: the first two stages (fetched during the previous tile's epilogue) are split into
        // ring slots 0 / 1, then iteration st (while the consumers compute stage st) waits for stage
        // st + 2's fetch (issued one iteration earlier), splits it into slot (st + 2) % 3 (released at
        // the last barrier) and fetches stage st + 3.  The fetches are ordinary (compiler-visible) loads:
        // the compiler waits for them before their first use, across the raw barriers, and a spill of a
        // register set waits for its loads first (an inline-asm load protocol is not spill-safe);
        // stage indices past the end are clamped (fetched anyway: the loads in flight are the same on
        // every path), commits past the end skipped.  Barriers per tile: 1 + nstages + 2, as consumers.
        int l = blockIdx.x;
        float pmax = 0.f;  // max |stored value| of this thread's share of the store phases (out_tag)
        decode(l, fcob, fb, fy0, fx0, fph);
        unsigned m0 = issue(0, r0);
        unsigned m1 = issue(min(1, last), r1);
        for (;;) {
            const int scob = fcob, sb = fb, soy0 = fy0, sox0 = fx0, sph = fph;  // tile being computed / stored
            commit(0, r0, m0);
            if (nstages > 1) commit(1, r1, m1);
            unsigned m = issue(min(2, last), r0);
            barrier();
            for (int st = 0; st < nstages; ++st) {
                if (st + 2 < nstages) commit(st + 2, r0, m);
                m = issue(min(st + 3, last), r0);
                barrier();
            }
            const int ln = l + (int)gridDim.x;
            const bool more = ln < nwg;
            if (more) {  // the next tile's first two stages load while this tile is stored
                decode(ln, fcob, fb, fy0, fx0, fph);
                cur_src = -1;
                m0 = issue(0, r0);
                m1 = issue(min(1, last), r1);
            }
            barrier();  // the consumers' tile is in LDS
            if (lds_epi)
                x3_store_phase<TILE_PX, NCO>(a, sb, scob, soy0, sox0, g.T, sph, reinterpret_cast<const float*>(ring), btab, tid,
                                             pmax, reinterpret_cast<double*>(smem));  // (red: the unused 128-B header)
            barrier();  // every read of the staged tile is done: the ring may be refilled
            if (!more) break;
            l = ln;
        }
        nps::tag_publish(a.out_tag, pmax, nps::wave_salt());
        return;
    }

    // ---------------------------------------------------------------------- consumers
    int boff[PBW];
    const int px0 = WIDE ? (wave >> 1) * 64 : wave * 32 * PB;  // this wave's first tile pixel
    const int cw0 = WIDE ? (wave & 1) * 96 : 0;                // this wave's first channel in the co group
#pragma unroll
    for (int pb = 0; pb < PBW; ++pb) {
        const int P = px0 + pb * 32 + (lane & 31);
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        boff[pb] = ti * rowb + tj * X3_PIXB + (lane >> 5) * 16;
    }
    f32x16 acc[CBW][PBW];
    const int ncb = packed_ncb(a.Cout);
    const size_t gstride = (size_t)ncb * 2048;  // bytes per K-group (chunk, tap) of the packed weight
    const int G = nstages * NTAPS;
    const char* wbase = nullptr;
    // weight fragments: a ring of AR K-groups, loaded AR - 1 K-groups ahead (wide tiles: two ahead, 3x3 class
    // -3.5 %, profiles/r4/experiments/x3_valu_diet_and_aring3_ab.txt)
    constexpr int AR = WIDE ? 3 : 2;
    f16x8 Aw[AR][CBW][2];
    f16x8 Bh[2][PBW], Bl[2][PBW];
    auto loadA = [&](int gg, f16x8 (&d)[CBW][2]) {
        const char* p = wbase + (size_t)gg * gstride;
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb) {
            d[cb][0] = *reinterpret_cast<const f16x8*>(p + cb * 2048);
            d[cb][1] = *reinterpret_cast<const f16x8*>(p + cb * 2048 + 1024);
        }
    };
    auto boffs = [&](int gg) {  // byte offset of K-group gg's patch window in the LDS ring
        const int st = gg / NTAPS, tap = gg - (gg / NTAPS) * NTAPS;
        return (st % X3_NST) * stage_b + (tap / KWT) * rowb + (tap % KWT) * X3_PIXB;
    };
    auto loadB = [&](int gg, f16x8 (&d)[PBW], int half) {
        const char* p = ring + boffs(gg) + half * 32;
#pragma unroll
        for (int pb = 0; pb < PBW; ++pb) d[pb] = *reinterpret_cast<const f16x8*>(p + boff[pb]);
    };
    // K-group gg uses weight slot gg & 1 and patch slot gg & 1; the loads of group gg + 1 (weights from
    // global memory, patch from LDS) go to the other slots, interleaved one per MFMA gap.  Loads are
    // never skipped (index clamped to the last group): a skipped load on one path makes the compiler's
    // in-order vmcnt wait drain the newest loads.
    auto gclamp = [&](int x) { return x < G ? x : G - 1; };
    auto group = [&](int gg, const int ra, const int r) __attribute__((always_inline)) {  // ra: weight slot of K-group gg, r: patch slot
        loadA(gclamp(gg + AR - 1), Aw[(ra + AR - 1) % AR]);
        loadB(gclamp(gg + 1), Bh[r ^ 1], 0);
        loadB(gclamp(gg + 1), Bl[r ^ 1], 1);
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
            for (int pb = 0; pb < PBW; ++pb) acc[cb][pb] = X3_MFMA(Aw[ra][cb][0], Bh[r][pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
            for (int pb = 0; pb < PBW; ++pb) acc[cb][pb] = X3_MFMA(Aw[ra][cb][0], Bl[r][pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
            for (int pb = 0; pb < PBW; ++pb) acc[cb][pb] = X3_MFMA(Aw[ra][cb][1], Bh[r][pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 2 * CBW; ++i) {  // weights first: the longest latency gets the most cover
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 VMEM read
        }
#pragma unroll
        for (int i = 0; i < 2 * PBW; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * CBW * PBW - 2 * PBW - 2 * CBW, 0);
        __builtin_amdgcn_sched_barrier(0);
        if ((gg + 1) % NTAPS == 0) barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // epilogue scale: undo the power-of-2 scale of the input and of the phase's packed weight (its trailer)
    const float xsc = (PRO && a.gn_stats != nullptr) ? gn_prologue_scale(a) : in_scale_of(a);
    const size_t wbody = packed_body(a.Cout, a.Cin, NTAPS);
    const int h = lane >> 5;
    float amax = 0.f;  // max |stored value| over this thread's tiles (out_tag)
    for (int l = blockIdx.x; l < nwg; l += gridDim.x) {
        int cob, b, oy0, ox0;
        int ph;
        decode(l, cob, b, oy0, ox0, ph);
        const float* wph = a.wpack + (size_t)ph * a.phase_wstride;
        const float inv = 1.f / (pow2_scale_for(wph[wbody]) * xsc);
        wbase = reinterpret_cast<const char*>(wph) + (size_t)(cob * (NCO / 32) + cw0 / 32) * 2048 + lane * 16;
#pragma unroll
        for (int i = 0; i < CBW; ++i)
#pragma unroll
            for (int j = 0; j < PBW; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        loadA(0, Aw[0]);
        if constexpr (AR == 3) loadA(gclamp(1), Aw[1]);
        barrier();
        loadB(0, Bh[0], 0);
        loadB(0, Bl[0], 1);
        int g0 = 0;
        if constexpr (AR == 2) {
            for (; g0 + 2 <= G; g0 += 2) {
                group(g0, 0, 0);
                group(g0 + 1, 1, 1);
            }
            if (g0 < G) group(g0, 0, 0);
        } else {  // slots (gg % 3, gg % 2): 6 K-groups per iteration, the tail continues the same pattern
            for (; g0 + 6 <= G; g0 += 6) {
                static_for<6>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    group(g0 + j, j % 3, j % 2);
                });
            }
            static_for<6>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if (g0 + j < G) group(g0 + j, j % 3, j % 2);
            });
        }
        if (lds_epi) {
            // the ring is free (every read of it completed before the last stage barrier): the consumers
            // drop the 64 x TILE_PX tile into LDS, then all 8 waves store it with coalesced 16-B accesses
            float* T = reinterpret_cast<float*>(ring);
#pragma unroll
            for (int pb = 0; pb < PBW; ++pb) {
                const int P = px0 + pb * 32 + (lane & 31);
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const f32x4 v = {acc[cb][pb][4 * m] * inv, acc[cb][pb][4 * m + 1] * inv,
                                         acc[cb][pb][4 * m + 2] * inv, acc[cb][pb][4 * m + 3] * inv};
                        *reinterpret_cast<f32x4*>(T + P * (NCO + 4) + cw0 + cb * 32 + 8 * m + 4 * h) = v;
                    }
            }
            barrier();
            x3_store_phase<TILE_PX, NCO>(a, b, cob, oy0, ox0, g.T, ph, T, btab, tid, amax, reinterpret_cast<double*>(smem));
        } else if constexpr (!WIDE) {
            static_for<PBW>([&](auto pbc) {  // compile-time pb: acc stays in registers
                constexpr int pb = decltype(pbc)::value;
                const int P = px0 + pb * 32 + (lane & 31);
                const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
                const int oy = oy0 + ti * g.T, ox = ox0 + tj * g.T;
                if (oy >= a.Hout || ox >= a.Wout) return;
                const int dy = oy * a.out_os + a.out_off_y + (ph >> 1), dx = ox * a.out_os + a.out_off_x + (ph & 1);
                if (dy < 0 || dy >= a.out_H || dx < 0 || dx >= a.out_W) return;
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb) {
                    f32x16 v = acc[cb][pb];
#pragma unroll
                    for (int r = 0; r < 16; ++r) v[r] *= inv;
                    store_tile(a, b, cob * NCO + cw0 + cb * 32, h, v, dy, dx, amax);
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
            barrier();
        }
        barrier();  // the staged tile is fully read: the producers may refill the ring
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}


// ---------------------------------------------------------------------------------------------
// Split-fp16 1x1 conv without a patch ring: every wave is its own producer.  A 1x1 stage has 9x less
// MFMA work per staged byte than a 3x3 one, so the ring kernel's single fetch in flight per work-group
// leaves it bound by HBM latency.  Here a work-group is up to 8 waves over the same PB * 32 output
// pixels (wave w: output channels [co_lo + 64w, + 64), co_lo = 512 * blockIdx.z), each wave streaming
// its B fragments straight from HBM into a D-deep register ring with no barrier; the co-block waves of
// a work-group read the same bytes (one HBM fetch, L1/L2 hits).  A stage is 32 channels: lane half h
// fetches the contiguous run [32s + 16h, + 16) of its pixel (64 B, four 16-B loads), which feeds two
// K-groups — the packing (pack_weights_x3_kernel, ntaps == 1) orders the weights to match.  The
// weights stream from L2 one stage ahead.  MFMA passes hi*hi, hi*lo, lo*hi as the ring kernel; the
// epilogue goes through LDS (one contiguous channel run per pixel) or store_tile.

template <int PB, int D>
__global__ __launch_bounds__(512) void conv1x1_x3_kernel(const nps_conv2d_t a) {
    constexpr int CBW = 2;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int co_lo = blockIdx.z * 512;
    const int cob = (co_lo >> 6) + wv;  // global 64-channel block of this wave
    const int b = blockIdx.y;
    const int h = lane >> 5;
    const int npx = a.Hout * a.Wout;
    const int P0 = blockIdx.x * (PB * 32);
    const float xs = in_scale_of(a);
    const bool scaled = has_in_scale(a);  // range-scaled input (xs != 1 possible)
    // this lane's output pixel of each pixel block -> its (circularly extended) frame position
    int fy[PB], fx[PB];
    unsigned pin = 0;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
        const int P = P0 + pb * 32 + (lane & 31);
        const int oy = P / a.Wout, ox = P - (P / a.Wout) * a.Wout;
        const int ye = oy - a.pad_y, xe = ox - a.pad_x;
        const bool ok = P < npx && ye >= 0 && ye < a.Hin + 2 * a.circ && xe >= 0 && xe < a.Win + 2 * a.circ;
        fy[pb] = a.circ ? nps::wrap_mod(ye - a.circ, a.Hin) : ye;
        fx[pb] = a.circ ? nps::wrap_mod(xe - a.circ, a.Win) : xe;
        pin = ok ? (pin | (1u << pb)) : pin;
    }
    const float* sp[PB];  // this lane's pixel in its current source (x3_zero16 when outside it)
    int cur_src = -1;     // per lane: the two lane halves may read different sources
    int cbase = 0;
    auto locate = [&](int sidx) {
        const nps_src_t S0 = a.src[0], S1 = a.src[1], S2 = a.src[2];
        const float* sptr = sidx == 0 ? S0.ptr : (sidx == 1 ? S1.ptr : S2.ptr);
        const int sC = sidx == 0 ? S0.C : (sidx == 1 ? S1.C : S2.C);
        const int sH = sidx == 0 ? S0.H : (sidx == 1 ? S1.H : S2.H);
        const int sW = sidx == 0 ? S0.W : (sidx == 1 ? S1.W : S2.W);
        const int soy = sidx == 0 ? S0.off_y : (sidx == 1 ? S1.off_y : S2.off_y);
        const int sox = sidx == 0 ? S0.off_x : (sidx == 1 ? S1.off_x : S2.off_x);
#pragma unroll
        for (int pb = 0; pb < PB; ++pb) {
            const int yy = fy[pb] - soy, xx = fx[pb] - sox;
            const bool ok = ((pin >> pb) & 1u) && yy >= 0 && yy < sH && xx >= 0 && xx < sW;
            sp[pb] = ok ? sptr + ((size_t)(b * sH + yy) * sW + xx) * sC : nullptr;
        }
    };
    const int nstages = (a.Cin + 2 * CK - 1) / (2 * CK);  // 32-channel stages
    const int last = nstages - 1;
    f32x4 raw[D][PB][4];  // register ring of B stages (fp32, as loaded; zeros outside the frame)
    auto issue = [&](int st, bool live, f32x4 (&r)[PB][4]) {
        const int c0 = st * 2 * CK + h * CK;  // this lane half's 16-channel run (inside one source:
        int sidx = 0, lo = 0, sb = 0;         // sources are 16-aligned, host-checked)
#pragma unroll
        for (int si = 0; si < NPS_MAX_SRC; ++si) {
            if (si < a.nsrc) {
                const int hi = lo + a.src[si].C;
                if (c0 >= lo && c0 < hi) {
                    sidx = si;
                    sb = lo;
                }
                lo = hi;
            }
        }
        if (sidx != cur_src) {  // per lane (the halves of a wave may differ)
            locate(sidx);
            cur_src = sidx;
            cbase = sb;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool chok = live && c0 + q * 4 < a.Cin;  // past the channel tail (or a padded stage): zeros
#pragma unroll
            for (int pb = 0; pb < PB; ++pb) {
                const float* src = (chok && sp[pb] != nullptr) ? sp[pb] + (c0 - cbase + q * 4) : x3_zero16;
                r[pb][q] = *reinterpret_cast<const f32x4*>(src);
            }
        }
    };
    const int ncb = packed_ncb(a.Cout);
    const size_t gstride = (size_t)ncb * 2048;  // bytes per chunk of the packed weight
    // the last 512-channel group's waves past the packed blocks (Cout = 600: 12 packed 64-channel blocks, waves
    // of blocks 12-15) read the last packed block instead of bytes past the buffer; they store nothing
    // (co >= Cout in either epilogue)
    const int wcob = cob < ncb / CBW ? cob : ncb / CBW - 1;
    const char* wbase = reinterpret_cast<const char*>(a.wpack) + (size_t)wcob * CBW * 2048 + lane * 16;
    f16x8 Aw[2][2][CBW][2];  // [slot][chunk of the pair][cb][hi, lo]
    auto loadA = [&](int st, f16x8 (&d)[2][CBW][2]) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const char* p = wbase + (size_t)(2 * st + k) * gstride;
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb) {
                d[k][cb][0] = *reinterpret_cast<const f16x8*>(p + cb * 2048);
                d[k][cb][1] = *reinterpret_cast<const f16x8*>(p + cb * 2048 + 1024);
            }
        }
    };
    f32x16 acc[CBW][PB];
#pragma unroll
    for (int i = 0; i < CBW; ++i)
#pragma unroll
        for (int j = 0; j < PB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // the stage loop runs a multiple of D stages so its body is straight-line (a per-stage guard makes the
    // compiler's wait at the guard's join vmcnt(0)); padded stages fetch the last stage again with an
    // all-zero mask, so their MFMAs add exact zeros
    static_for<D - 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        issue(min(j, last), j <= last, raw[j]);
    });
    loadA(0, Aw[0]);
    const int npad = (nstages + D - 1) / D * D;
    for (int s0 = 0; s0 < npad; s0 += D) {
        static_for<D>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            constexpr int jn = (j + D - 1) % D;
            const int st = s0 + j;
            issue(min(st + D - 1, last), st + D - 1 <= last, raw[jn]);
            loadA(min(st + 1, last), Aw[(j + 1) & 1]);
            // keep the new fetches ahead of this stage's MFMAs: sunk below them, the MFMAs' wait for
            // this stage's operands would become vmcnt(0) and drain the whole ring every stage
            __builtin_amdgcn_sched_barrier(0);
            constexpr int r = j & 1;  // D is even: the weight slot parity is static
#pragma unroll
            for (int k = 0; k < 2; ++k) {  // the two K-groups of the stage: floats [8k, 8k + 8) of the run
                f16x8 Bh[PB], Bl[PB];
#pragma unroll
                for (int pb = 0; pb < PB; ++pb) {
                    f16x4 h0, l0, h1, l1;
                    f32x4 v0 = raw[j][pb][2 * k], v1 = raw[j][pb][2 * k + 1];
                    if (scaled) {
                        v0 *= xs;
                        v1 *= xs;
                    }
                    split4(v0, h0, l0);
                    split4(v1, h1, l1);
                    Bh[pb] = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
                    Bl[pb] = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
                }
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                    for (int pb = 0; pb < PB; ++pb)
                        acc[cb][pb] = X3_MFMA(Aw[r][k][cb][0], Bh[pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                    for (int pb = 0; pb < PB; ++pb)
                        acc[cb][pb] = X3_MFMA(Aw[r][k][cb][0], Bl[pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                    for (int pb = 0; pb < PB; ++pb)
                        acc[cb][pb] = X3_MFMA(Aw[r][k][cb][1], Bh[pb], acc[cb][pb], 0, 0, 0);
            }
        });
    }
    const float inv = 1.f / (pow2_scale_for(a.wpack[packed_body(a.Cout, a.Cin, 1)]) * xs);
    if (x3_lds_epilogue(a)) {
        // the work-group's (waves*64) x PB*32 tile goes through LDS (pitch = waves*64 + 4 floats: conflict-
        // free 16-B writes) and is stored pixel by pixel, each pixel's channels one contiguous run
        extern __shared__ __attribute__((aligned(16))) float T[];
        const int pitch = (int)(blockDim.x) + 4;  // blockDim.x = 64 * waves
#pragma unroll
        for (int pb = 0; pb < PB; ++pb) {
            const int P = pb * 32 + (lane & 31);
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const f32x4 v = {acc[cb][pb][4 * m] * inv, acc[cb][pb][4 * m + 1] * inv,
                                     acc[cb][pb][4 * m + 2] * inv, acc[cb][pb][4 * m + 3] * inv};
                    *reinterpret_cast<f32x4*>(T + P * pitch + wv * 64 + cb * 32 + 8 * m + 4 * h) = v;
                }
        }
        __syncthreads();
        const int nco = min(a.Cout - co_lo, (int)blockDim.x);
        const int C4 = nco >> 2;
        // item i = (pixel p, channel quad): when C4 divides the block, a thread keeps one channel quad
        // and steps pixels by blockDim / C4 (no per-item divisions)
        const bool fixq = ((int)blockDim.x % C4) == 0;
        const int pstep = fixq ? (int)blockDim.x / C4 : 0;
        int fp = fixq ? (int)threadIdx.x / C4 : 0;
        const int fcl = fixq ? ((int)threadIdx.x - fp * C4) * 4 : 0;
        int foy = (P0 + fp) / a.Wout, fox = (P0 + fp) - ((P0 + fp) / a.Wout) * a.Wout;
        float amax = 0.f;
        for (int i = threadIdx.x; i < PB * 32 * C4; i += blockDim.x) {
            int p, cl, oy, ox;
            if (fixq) {
                p = fp;
                cl = fcl;
                oy = foy;
                ox = fox;
                fp += pstep;
                fox += pstep;
                while (fox >= a.Wout) {
                    fox -= a.Wout;
                    ++foy;
                }
            } else {
                p = i / C4;
                cl = (i - (i / C4) * C4) * 4;
                oy = (P0 + p) / a.Wout;
                ox = (P0 + p) - ((P0 + p) / a.Wout) * a.Wout;
            }
            const int co0 = co_lo + cl;
            const int P = P0 + p;
            if (P >= npx) continue;
            const int dy = oy * a.out_os + a.out_off_y, dx = ox * a.out_os + a.out_off_x;
            if (dy < 0 || dy >= a.out_H || dx < 0 || dx >= a.out_W) continue;
            const f32x4 accv = *reinterpret_cast<const f32x4*>(T + p * pitch + cl);
            const size_t o = (((size_t)b * a.out_H + dy) * a.out_W + dx) * a.out_C + co0;
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            const f32x4 bi = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + co0) : z;
            const f32x4 a0 = a.addend0 ? *reinterpret_cast<const f32x4*>(a.addend0 + o) : z;
            const f32x4 a1 = a.addend1 ? *reinterpret_cast<const f32x4*>(a.addend1 + o) : z;
            const f32x4 ov = a.accumulate ? *reinterpret_cast<const f32x4*>(a.out + o) : z;
            f32x4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // as store_tile / x3_store_phase
                float v = accv[e] + bi[e];
                if (!a.add_after_act) v = v + a0[e] + a1[e];
                if (a.act == 1) v = nps::gelu_erf(v);
                if (a.add_after_act) v = v + a0[e] + a1[e];
                if (a.accumulate) v += ov[e];
                r[e] = v;
                amax = fmaxf(amax, fabsf(v));
            }
            *reinterpret_cast<f32x4*>(a.out + o) = r;
        }
        nps::tag_publish(a.out_tag, amax, nps::wave_salt());
        return;
    }
    float amax = 0.f;
    static_for<PB>([&](auto pbc) {  // compile-time pb: acc stays in registers
        constexpr int pb = decltype(pbc)::value;
        const int P = P0 + pb * 32 + (lane & 31);
        if (P >= npx) return;
        const int oy = P / a.Wout, ox = P - (P / a.Wout) * a.Wout;
        const int dy = oy * a.out_os + a.out_off_y, dx = ox * a.out_os + a.out_off_x;
        if (dy < 0 || dy >= a.out_H || dx < 0 || dx >= a.out_W) return;
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb) {
            const int co = cob * 64 + cb * 32;
            if (co >= a.Cout) continue;
            f32x16 v = acc[cb][pb];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] *= inv;
            store_tile(a, b, co, h, v, dy, dx, amax);
        }
    });
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}

// 1x1 with the weights staged in LDS: a wave covers ALL output channels (NCB 32-channel blocks) of its
// 32 pixels, so a work-group of 4 waves (128 pixels) fetches its input once per CU instead of once per
// co-block wave.  Per 32-channel stage the 4 waves copy the stage's weight fragments (2 chunks x NCB
// blocks x 2 KB) into one of two LDS buffers (fetched one stage ahead into registers, compiler-managed
// loads), one barrier per stage; B as in conv1x1_x3_kernel (per-lane 64-B runs in a D-deep register
// ring, zero page outside the frame).  Epilogue: store_tile per 32-channel block.
// PRO: the frame prologue act(GroupNorm(frame)) (the U-Net's final GN(8) + GELU before its 1x1 conv,
// proc_unet_modern.py:191-196) applied to each loaded input element before the split, instead of a frame_pack
// pass: per-channel affine (scale, shift) of this work-group's sample in an LDS table built at kernel start from the
// fp64 moments, then GELU; frame pixels no source covers get act(GN(0)), the conv's own zero padding stays 0.
// Cout > NCB * 32 (the input-gradient convs 192 -> 388 / 196 of the shortcut and FNO 1x1s): channel groups of
// NCB * 32, group g = work-group index / 8 % ng, pixel tile = the rest (nps_launch_conv2d_x3: the ng groups of one
// tile are 8 work-groups apart, so they run on one XCD and the later ones read the tile's input from its L2);
// a group's blocks past Cout skip their MFMAs (the 4-channel tail group of 388 costs 1 block of 6).
template <int NCB, int D, bool PRO = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv1x1_wl_kernel(const nps_conv2d_t a,
                                                                                                  int ng) {
    constexpr int WSTAGE = 2 * NCB * 2048;       // bytes of one stage's weight fragments
    constexpr int WPT = WSTAGE / (256 * 16);     // 16-B pieces per thread per stage
    static_assert(WSTAGE % (256 * 16) == 0, "weight stage split");
    extern __shared__ __attribute__((aligned(16))) char wl[];  // [2][2 chunks][NCB][hi|lo][64][16 B]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.y;
    const int h = lane >> 5;
    const int npx = a.Hout * a.Wout;
    int tile = (int)blockIdx.x, grp = 0;
    if (ng > 1) {
        const int r = (int)blockIdx.x >> 3;
        grp = r % ng;
        tile = (r / ng) * 8 + ((int)blockIdx.x & 7);
        if (tile * 128 >= npx) return;  // (the tile count is padded to a multiple of 8)
    }
    const int cob = grp * NCB * 32;                       // this group's first output channel
    const int nact = min(NCB, (a.Cout - cob + 31) / 32);  // its blocks that hold output channels
    const int P = tile * 128 + wv * 32 + (lane & 31);
    const float xs = PRO ? gn_prologue_scale(a) : in_scale_of(a);
    const bool scaled = PRO || has_in_scale(a);
    int fy, fx;
    bool pin;
    {
        const int oy = P / a.Wout, ox = P - (P / a.Wout) * a.Wout;
        const int ye = oy - a.pad_y, xe = ox - a.pad_x;
        pin = P < npx && ye >= 0 && ye < a.Hin + 2 * a.circ && xe >= 0 && xe < a.Win + 2 * a.circ;
        fy = a.circ ? nps::wrap_mod(ye - a.circ, a.Hin) : ye;
        fx = a.circ ? nps::wrap_mod(xe - a.circ, a.Win) : xe;
    }
    const float* sp = nullptr;
    int cur_src = -1, cbase = 0;
    auto locate = [&](int sidx) {
        const nps_src_t S0 = a.src[0], S1 = a.src[1], S2 = a.src[2];
        const float* sptr = sidx == 0 ? S0.ptr : (sidx == 1 ? S1.ptr : S2.ptr);
        const int sC = sidx == 0 ? S0.C : (sidx == 1 ? S1.C : S2.C);
        const int sH = sidx == 0 ? S0.H : (sidx == 1 ? S1.H : S2.H);
        const int sW = sidx == 0 ? S0.W : (sidx == 1 ? S1.W : S2.W);
        const int yy = fy - (sidx == 0 ? S0.off_y : (sidx == 1 ? S1.off_y : S2.off_y));
        const int xx = fx - (sidx == 0 ? S0.off_x : (sidx == 1 ? S1.off_x : S2.off_x));
        const bool ok = pin && yy >= 0 && yy < sH && xx >= 0 && xx < sW;
        sp = ok ? sptr + ((size_t)(b * sH + yy) * sW + xx) * sC : nullptr;
    };
    const int nstages = (a.Cin + 2 * CK - 1) / (2 * CK);
    const int last = nstages - 1;
    f32x4 raw[D][4];
    auto issue = [&](int st, bool live, f32x4 (&r)[4]) {
        const int c0 = st * 2 * CK + h * CK;
        int sidx = 0, lo = 0, sb = 0;
#pragma unroll
        for (int si = 0; si < NPS_MAX_SRC; ++si) {
            if (si < a.nsrc) {
                const int hi = lo + a.src[si].C;
                if (c0 >= lo && c0 < hi) {
                    sidx = si;
                    sb = lo;
                }
                lo = hi;
            }
        }
        if (sidx != cur_src) {
            locate(sidx);
            cur_src = sidx;
            cbase = sb;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool chok = live && c0 + q * 4 < a.Cin;
            const float* src = (chok && sp != nullptr) ? sp + (c0 - cbase + q * 4) : x3_zero16;
            r[q] = *reinterpret_cast<const f32x4*>(src);
        }
    };
    // weight stage st: chunks 2st, 2st + 1, blocks [0, NCB) of each (the packed chunk holds packed_ncb blocks)
    const size_t gstride = (size_t)packed_ncb(a.Cout) * 2048;
    const char* wg = reinterpret_cast<const char*>(a.wpack) + (size_t)grp * NCB * 2048;
    f32x4 wr[WPT];
    auto wfetch = [&](int st) {
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
            const int off = (i * 256 + (int)threadIdx.x) * 16;  // byte offset inside the stage
            const int k = off / (NCB * 2048), rem = off - k * (NCB * 2048);
            wr[i] = *reinterpret_cast<const f32x4*>(wg + (size_t)(2 * st + k) * gstride + rem);
        }
    };
    auto wstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < WPT; ++i)
            *reinterpret_cast<f32x4*>(wl + buf * WSTAGE + (i * 256 + (int)threadIdx.x) * 16) = wr[i];
    };
    if ((int)threadIdx.x < NCB * 32)  // the epilogue's bias table (zero past Cout), behind the first barrier
        reinterpret_cast<float*>(wl + 2 * WSTAGE)[threadIdx.x] =
            (a.bias != nullptr && cob + (int)threadIdx.x < a.Cout) ? a.bias[cob + threadIdx.x] : 0.f;
    // PRO: per-channel GroupNorm affine of sample b, y = x * gs[c] + gb[c] (gs = rstd * gamma, gb = beta - mean * gs, the
    // producers' form in conv2d_x3_kernel), zero past Cin (GELU(0) = 0 against zero weights)
    float* gtab = reinterpret_cast<float*>(wl + 2 * WSTAGE + NCB * 32 * 4);  // [2][nstages * 32]
    if constexpr (PRO) {
        const int ncp = ((a.Cin + 2 * CK - 1) / (2 * CK)) * 2 * CK;
        const bool gn = a.gn_stats != nullptr;
        const double icnt = gn ? 1.0 / ((double)(a.Cin / a.gn_groups) * a.Hin * a.Win) : 0.0;
        for (int c = threadIdx.x; c < ncp; c += 256) {
            float gs = 1.f, gb = 0.f;
            if (c >= a.Cin) {
                gs = 0.f;
            } else if (gn) {
                const double* st = a.gn_stats + ((size_t)b * a.gn_groups + c / (a.Cin / a.gn_groups)) * 2;
                const double mu = st[0] * icnt;
                double var = fma(st[1], icnt, -mu * mu);
                var = var < 0.0 ? 0.0 : var;
                const float rstd = __builtin_amdgcn_rsqf((float)(var + (double)a.gn_eps));
                gs = rstd * a.gn_gamma[c];
                gb = fmaf(-(float)mu, gs, a.gn_beta[c]);
            }
            gtab[c] = gs;
            gtab[ncp + c] = gb;
        }
    }
    f32x16 acc[NCB];
#pragma unroll
    for (int i = 0; i < NCB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    static_for<D - 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        issue(min(j, last), j <= last, raw[j]);
    });
    wfetch(0);
    wstore(0);
    wfetch(min(1, last));
    __syncthreads();
    const int npad = (nstages + D - 1) / D * D;
    for (int s0 = 0; s0 < npad; s0 += D) {
        static_for<D>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            constexpr int jn = (j + D - 1) % D;
            const int st = s0 + j;
            // weights of stage st + 1 (fetched last stage) -> the other buffer (its readers passed the
            // previous barrier); then fetch stage st + 2's
            wstore((st + 1) & 1);
            wfetch(min(st + 2, last));
            issue(min(st + D - 1, last), st + D - 1 <= last, raw[jn]);
            __builtin_amdgcn_sched_barrier(0);
            const char* wb = wl + (st & 1) * WSTAGE + lane * 16;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                f16x4 h0, l0, h1, l1;
                f32x4 v0 = raw[j][2 * k], v1 = raw[j][2 * k + 1];
                if constexpr (PRO) {  // channels st * 32 + h * 16 + 8 k + [0, 8) of this lane's pixel
                    // (the padded iterations of the ring, st > last, read no table: their input must stay 0)
                    const int ncp = ((a.Cin + 2 * CK - 1) / (2 * CK)) * 2 * CK;
                    const bool live = pin && st <= last;
                    const int c = min(st, last) * 2 * CK + h * CK + 8 * k;
                    const f32x4 s0 = *reinterpret_cast<const f32x4*>(gtab + c);
                    const f32x4 s1 = *reinterpret_cast<const f32x4*>(gtab + c + 4);
                    const f32x4 b0 = *reinterpret_cast<const f32x4*>(gtab + ncp + c);
                    const f32x4 b1 = *reinterpret_cast<const f32x4*>(gtab + ncp + c + 4);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float y0 = fmaf(v0[e], s0[e], b0[e]), y1 = fmaf(v1[e], s1[e], b1[e]);
                        if (a.pre_act == 1) {
                            y0 = nps::gelu_fast(y0);
                            y1 = nps::gelu_fast(y1);
                        }
                        v0[e] = live ? y0 : 0.f;  // (outside the frame: the conv's zero padding)
                        v1[e] = live ? y1 : 0.f;
                    }
                }
                if (scaled) {
                    v0 *= xs;
                    v1 *= xs;
                }
                split4(v0, h0, l0);
                split4(v1, h1, l1);
                const f16x8 Bh = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
                const f16x8 Bl = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb) {
                    if (cb >= nact) break;  // (uniform: a tail group's empty blocks)
                    const f16x8 Ah = *reinterpret_cast<const f16x8*>(wb + (k * NCB + cb) * 2048);
                    const f16x8 Al = *reinterpret_cast<const f16x8*>(wb + (k * NCB + cb) * 2048 + 1024);
                    acc[cb] = X3_MFMA(Ah, Bh, acc[cb], 0, 0, 0);
                    acc[cb] = X3_MFMA(Ah, Bl, acc[cb], 0, 0, 0);
                    acc[cb] = X3_MFMA(Al, Bh, acc[cb], 0, 0, 0);
                }
            }
            __syncthreads();
        });
    }
    const float inv = 1.f / (pow2_scale_for(a.wpack[packed_body(a.Cout, a.Cin, 1)]) * xs);
    if constexpr (!PRO) {
        if (a.spec_z != nullptr) {
            // FNO layer fusion (nps_conv2d_t.spec_z): the c2r W pass of the spectral conv on the same accumulators,
            // out[co][px] += sum_k' Z'[k'][co] T[k'][px] on exact-fp32 v_mfma_f32_32x32x2f32 (one K-step per bin:
            // k' = 2k Re Z c_k against cos 2 pi k x / W, 2k + 1 Im Z c_k against -sin), Z' pre-scaled by
            // spec_scale / inv (exact powers of 2 both), so the epilogue's acc * inv + bias carries it.  The
            // work-group's 128 pixels lie in one row (Wout % 128 == 0, host-checked): Z' of that row and the
            // pixels' twiddles are staged in the (free) weight buffers, behind the exchange slot at their start.
            const int m2 = a.spec_m2, K2 = 2 * m2;
            const int t0 = tile * 128, y0 = t0 / a.Wout, x0 = t0 - y0 * a.Wout;  // (Cout <= NCB * 32: one group)
            float* zs = reinterpret_cast<float*>(wl + 256);                 // [K2][NCB * 32]
            float* ts = zs + K2 * NCB * 32;                                   // [128][K2]
            const float fac = a.spec_scale / inv;
            const float2* zrow = reinterpret_cast<const float2*>(a.spec_z) + ((size_t)b * a.Hout + y0) * m2 * a.Cout;
            for (int i = threadIdx.x; i < m2 * NCB * 32; i += 256) {
                const int k = i / (NCB * 32), o = i - k * (NCB * 32);
                const bool self_conj = (k == 0) || (2 * k == a.Wout);
                const float cm = self_conj ? 1.f : 2.f;
                float2 z = make_float2(0.f, 0.f);
                if (o < a.Cout) z = zrow[(size_t)k * a.Cout + o];
                zs[(2 * k) * NCB * 32 + o] = z.x * cm * fac;
                zs[(2 * k + 1) * NCB * 32 + o] = self_conj ? 0.f : z.y * cm * fac;
            }
            for (int i = threadIdx.x; i < 128 * m2; i += 256) {
                const int p = i / m2, k = i - (i / m2) * m2;
                const int ph = (int)(((long)k * (x0 + p)) % a.Wout);
                float sn, cs;
                sincospif(2.0f * (float)ph / (float)a.Wout, &sn, &cs);
                ts[p * K2 + 2 * k] = cs;
                ts[p * K2 + 2 * k + 1] = -sn;
            }
            __syncthreads();
            const float* tl = ts + (wv * 32 + (lane & 31)) * K2 + h;  // B: pixel lane % 32, k' parity lane / 32
            for (int k = 0; k < m2; ++k) {
                const float bt = tl[2 * k];
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb)
                    acc[cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(zs[(2 * k + h) * NCB * 32 + cb * 32 + (lane & 31)], bt,
                                                                  acc[cb], 0, 0, 0);
            }
        }
    }
    const int oy = P / a.Wout, ox = P - (P / a.Wout) * a.Wout;
    const int dy = oy * a.out_os + a.out_off_y, dx = ox * a.out_os + a.out_off_x;
    float amax = 0.f;
    const bool pout = P < npx && dy >= 0 && dy < a.out_H && dx >= 0 && dx < a.out_W;
    if (x3_lds_epilogue(a) && a.addend1 == nullptr && !a.accumulate) {
        // The fused epilogue in store_tile's float order (acc*inv + bias [+ a0 + a1] [GELU] [+ a0 + a1]
        // [+ out]), the bias from the LDS table, every operand load issued before the stores it would
        // otherwise queue behind, and no branch around a store (out-of-range quads go to a sink).  vmcnt
        // retires loads and stores in one in-order queue, so a load issued after a store waits for it
        // (DESIGN.md § Round 3); store_tile's per-block loads did exactly that.
        const float* btab = reinterpret_cast<const float*>(wl + 2 * WSTAGE);
        const size_t base = pout ? (((size_t)b * a.out_H + dy) * a.out_W + dx) * a.out_C : 0;
        // per 32-channel block: apply the epilogue (its addend was loaded before the previous block's stores),
        // load the next block's addend, store this block.  (Two addends or accumulate: store_tile below.)
        double s1 = 0.0, s2 = 0.0;
        auto epi = [&](auto opc) {
            constexpr bool OP = decltype(opc)::value;
            f32x4 a0[4];
            auto load = [&](int cb) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int co0 = cob + cb * 32 + 8 * m + 4 * h;
                    const bool ok = pout && co0 < a.Cout;
                    a0[m] = *reinterpret_cast<const f32x4*>(ok ? a.addend0 + base + co0 : x3_zero16);
                }
            };
            if constexpr (OP) load(0);
            static_for<NCB>([&](auto cbc) {
                constexpr int cb = decltype(cbc)::value;
                float f1 = 0.f, f2 = 0.f;  // out_stats (plain epilogue, host-checked): this block's moments
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int co0 = cb * 32 + 8 * m + 4 * h;
                    const bool ok = pout && cob + co0 < a.Cout;
                    const f32x4 bi = *reinterpret_cast<const f32x4*>(btab + co0);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float v = acc[cb][4 * m + e] * inv + bi[e];
                        if constexpr (OP) {  // + a1 (0) as store_tile: v + a0 + 0 == v + a0
                            if (!a.add_after_act) v = v + a0[m][e];
                        }
                        if (a.act == 1) v = nps::gelu_erf(v);
                        if constexpr (OP) {
                            if (a.add_after_act) v = v + a0[m][e];
                        }
                        acc[cb][4 * m + e] = v;
                        amax = ok ? fmaxf(amax, fabsf(v)) : amax;
                        f1 += ok ? v : 0.f;
                        f2 += ok ? v * v : 0.f;
                    }
                }
                s1 += (double)f1;
                s2 += (double)f2;
                if constexpr (OP && cb + 1 < NCB) {
                    __builtin_amdgcn_sched_barrier(0);
                    load(cb + 1);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int co0 = cob + cb * 32 + 8 * m + 4 * h;
                    const bool ok = pout && co0 < a.Cout;
                    const f32x4 r = {acc[cb][4 * m], acc[cb][4 * m + 1], acc[cb][4 * m + 2], acc[cb][4 * m + 3]};
                    *reinterpret_cast<f32x4*>(ok ? a.out + base + co0 : x3_sink + 4 * lane) = r;
                }
                __builtin_amdgcn_sched_barrier(0);
            });
        };
        if (a.addend0 != nullptr)
            epi(std::true_type{});
        else
            epi(std::false_type{});
        // range tag + moments, once per work-group (every LDS read of the main loop is behind its last barrier:
        // the weight buffers hold the exchange)
        publish_wg(a, b, amax, s1, s2, reinterpret_cast<double*>(wl));
        return;
    }
    if (pout) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
            if (cob + cb * 32 >= a.Cout) continue;
            f32x16 v = acc[cb];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] *= inv;
            store_tile(a, b, cob + cb * 32, h, v, dy, dx, amax);
        }
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
    if (a.out_stats != nullptr) {
        // moments of the stored values, recomputed from the accumulators (out_stats on a 1x1 conv:
        // plain epilogue only — bias, no addends / act / accumulate, host-checked); kept out of the store
        // loop, where the extra live values made this kernel spill
        double s1 = 0.0, s2 = 0.0;
        if (pout) {
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                if (cob + cb * 32 >= a.Cout) continue;
                float f1 = 0.f, f2 = 0.f;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int co0 = cob + cb * 32 + 8 * m + 4 * h;
                    if (co0 >= a.Cout) continue;
                    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                    const f32x4 bi = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + co0) : z;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float r = acc[cb][4 * m + e] * inv + bi[e];
                        f1 += r;
                        f2 += r * r;
                    }
                }
                s1 += (double)f1;
                s2 += (double)f2;
            }
        }
        stats_publish(a, b, s1, s2);
    }
}

template <int NT, int PB, bool PRO = false, bool WIDE = false>
void launch_x3_one(const nps_conv2d_t& a, unsigned nwg, int lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv2d_x3_kernel<NT, PB, PRO, WIDE>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    conv2d_x3_kernel<NT, PB, PRO, WIDE><<<nwg, 512, lds, s>>>(a);
}



}  // namespace


// dev knob NPS_X1_GROUPS=0: 1x1 convs with Cout > 192 on the co-block kernel (conv1x1_x3_kernel) instead of the
// LDS-weight kernel's channel groups
static const int g_x1_groups = [] {
    const char* e = getenv("NPS_X1_GROUPS");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
}();

// test hook (nps_x3_set_grid): persistent-grid size override (> 0)
static long g_x3_grid_override = 0;

extern "C" int nps_x3_set_grid(long wgs) {
    g_x3_grid_override = wgs > 0 ? wgs : 0;
    return 0;
}

int nps_launch_conv2d_x3(const nps_conv2d_t& a, int lds, hipStream_t s) {
    const Geo g = make_geo(a);
    const bool wide = x3_wide_tile(a);  // 192-channel x 128-pixel work-groups (nps_conv2d_plan)
    const long nwg = (long)g.tiles_x * g.tiles_y * a.B * ((a.Cout + (wide ? 191 : 63)) / (wide ? 192 : 64)) *
                     (a.nphase > 1 ? a.nphase : 1);
    NPS_CHECK_ARG(a.nphase <= 1 || (a.nphase == 4 && a.KH * a.KW == 4 && a.out_os == 2 && a.phase_wstride > 0),
                  "conv2d_fwd (split-fp16): nphase = 4 is the k4/s2 transposed conv (2x2 phases, out_os 2)");
    NPS_CHECK_ARG(nwg < (1L << 31), "conv2d_fwd: grid too large");
    // persistent grid: one 512-thread work-group per CU (the LDS ring takes most of a CU), each walking
    // the tiles l = blockIdx.x, + gridDim.x, ...; a multiple of 8 keeps every work-group's tiles on one XCD
    static int ncu = 0;
    if (ncu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        ncu = n;
    }
    static long per = -1;
    if (per < 0) {
        per = (ncu & ~7) > 0 ? (ncu & ~7) : ncu;
        const char* e = getenv("NPS_X3_GRID");  // dev knob: work-groups of the persistent grid
        if (e != nullptr && atol(e) > 0) per = atol(e);
    }
    const long pw = g_x3_grid_override > 0 ? g_x3_grid_override : per;
    const bool lds_epi = !a.out_nchw && (a.out_C & 3) == 0 && (a.Cout & 3) == 0;  // == x3_lds_epilogue
    const unsigned grid = (unsigned)(pw < nwg ? pw : nwg);  // either epilogue walks tiles (tests: many per WG)
    const bool p512 = a.TH * a.TW == 512;
    const bool pro = a.gn_stats != nullptr || a.pre_act != 0;  // fused frame prologue: 3x3 only (host-checked)
    // 1x1 convs (never with a prologue: x3_eligible) run on the ring-free kernel, whose 32-channel
    // stages match the 1x1 weight packing; work-group = min(ncob, 8) waves, blockIdx.z = 512-channel group
    if (a.KH * a.KW == 1) {
        NPS_CHECK_ARG(!pro || a.Cout <= 192, "conv2d_fwd (split-fp16): a 1x1 prologue needs the LDS-weight kernel "
                      "(Cout <= 192)");
        NPS_CHECK_ARG(a.spec_z == nullptr || a.Cout <= 192,
                      "conv2d_fwd (split-fp16 1x1): the fused c2r term needs the LDS-weight kernel");
        const int ncob = (a.Cout + 63) / 64;
        // out_stats: the LDS-weight kernel's fused register epilogue takes the moments of the values it stores
        // (after the addend and the activation); its store_tile fallback (two addends, accumulate) cannot
        NPS_CHECK_ARG(a.out_stats == nullptr || (a.Cout <= 192 && !a.accumulate && a.addend1 == nullptr && lds_epi),
                      "conv2d_fwd (split-fp16 1x1): out_stats needs the LDS-weight kernel (Cout <= 192), an NHWC "
                      "4-aligned output and at most one addend, no accumulate");
        static int res_on = -1;  // dev knob NPS_X1_RES=1: resident-weight kernel for every 1x1 (default: only the
        if (res_on < 0) {        // planar decoder shape; at par or slower on the others, profiles/r5/experiments/x1_resident_weights_ab.txt)
            const char* e = getenv("NPS_X1_RES");
            res_on = (e != nullptr && e[0] == '1') ? 1 : 0;
        }
        if (pro) {  // fused GroupNorm + GELU prologue: the LDS-weight kernel with the per-channel affine table
            const long nb = ((long)a.Hout * a.Wout + 127) / 128;
            NPS_CHECK_ARG(nb < (1L << 31) && a.B < 65536, "conv2d_fwd: grid too large");
            const int ncp = ((a.Cin + 31) / 32) * 32;
            conv1x1_wl_kernel<6, 2, true><<<dim3((unsigned)nb, a.B), 256, 2 * 2 * 6 * 2048 + 6 * 32 * 4 + 2 * ncp * 4, s>>>(a, 1);
            NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16 1x1, LDS weights, GroupNorm prologue)");
            return 0;
        }
        if (nps_launch_conv1x1_res(a, res_on, s)) return 0;  // resident weights (conv1x1_res.hip)
        if (a.Cout <= 192 || g_x1_groups) {
            // Cout > 192: channel groups of 192 (the input-gradient convs 192 -> 388 / 196), the ng groups of a pixel
            // tile 8 work-groups apart (one XCD: the later groups read the tile from L2), tiles padded to 8
            const int ng = (a.Cout + 191) / 192;
            long nb = ((long)a.Hout * a.Wout + 127) / 128;
            if (ng > 1) nb = (nb + 7) / 8 * 8 * ng;
            NPS_CHECK_ARG(nb < (1L << 31) && a.B < 65536, "conv2d_fwd: grid too large");
            // B-ring depth 2: measured fastest on every rollout shape (profiles/r1_conv_shapes_1x1_wl_depth.log)
            conv1x1_wl_kernel<6, 2><<<dim3((unsigned)nb, a.B), 256, 2 * 2 * 6 * 2048 + 6 * 32 * 4, s>>>(a, ng);
            NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16 1x1, LDS weights)");
            return 0;
        }
        const int waves = ncob < 8 ? ncob : 8;
        const long nblk = ((long)a.Hout * a.Wout + 63) / 64;
        NPS_CHECK_ARG(nblk < (1L << 31) && a.B < 65536, "conv2d_fwd: grid too large");
        const dim3 grid1((unsigned)nblk, a.B, (ncob + 7) / 8);
        const int lds1 = lds_epi ? 64 * (64 * waves + 4) * 4 : 0;
        conv1x1_x3_kernel<2, 2><<<grid1, 64 * waves, lds1, s>>>(a);
        NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16 1x1)");
        return 0;
    }
    if (wide) {
        if (a.KH * a.KW == 9)
            pro ? launch_x3_one<9, 2, true, true>(a, grid, lds, s) : launch_x3_one<9, 2, false, true>(a, grid, lds, s);
        else if (a.KH * a.KW == 4)
            launch_x3_one<4, 2, false, true>(a, grid, lds, s);
        else
            NPS_CHECK_ARG(false, "conv2d_fwd (split-fp16): wide tiles are 2x2 / 3x3 only");
        NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16, wide)");
        return 0;
    }
    switch (a.KH * a.KW) {
        case 9:
            if (pro)
                p512 ? launch_x3_one<9, 4, true>(a, grid, lds, s) : launch_x3_one<9, 2, true>(a, grid, lds, s);
            else
                p512 ? launch_x3_one<9, 4>(a, grid, lds, s) : launch_x3_one<9, 2>(a, grid, lds, s);
            break;
        case 25:  // 5x5 (DRN, dilated on the lattice): 256-pixel tiles only (host-checked by the LDS budget)
            NPS_CHECK_ARG(!p512, "conv2d_fwd (split-fp16): 5x5 needs a 256-pixel tile");
            launch_x3_one<25, 2>(a, grid, lds, s);
            break;
        case 4: p512 ? launch_x3_one<4, 4>(a, grid, lds, s) : launch_x3_one<4, 2>(a, grid, lds, s); break;
        default: NPS_CHECK_ARG(false, "conv2d_fwd (split-fp16): unsupported tap count"); break;
    }
    NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16)");
    return 0;
}

// Highest byte (exclusive) of the packed weight that the split-fp16 launch of *a (after nps_conv2d_plan) reads, from
// the index arithmetic of the kernel the launcher picks for it (an over-read must be caught by a
// host check, not by allocation luck).  tests/test_cabi.py sweeps shapes against nps_conv2d_packed_size.
extern "C" long nps_conv2d_x3_weight_span(const nps_conv2d_t* ap) {
    NPS_CHECK_ARG(ap != nullptr && ap->precision == NPS_PREC_X3F16, "conv2d_x3_weight_span: split-fp16 args only");
    const nps_conv2d_t& a = *ap;
    const int nt = a.KH * a.KW;
    const long ncb = packed_ncb(a.Cout);      // 32-channel blocks per (chunk, tap) group: a multiple of 6
    const long gstride = ncb * 2048;          // bytes per (chunk, tap) group
    long span = (long)(packed_body(a.Cout, a.Cin, nt) + 1) * 4;  // the trailer's max|w| (weight scale)
    auto top = [&](long v) { span = v > span ? v : span; };
    if (nt == 1) {
        const long nst = (a.Cin + 2 * CK - 1) / (2 * CK);  // 32-channel stages: chunks 2 st, 2 st + 1
        const char* e = getenv("NPS_X1_RES");
        const int all = (e != nullptr && e[0] == '1') ? 1 : 0;
        int rncb = 0, rng = 0, rnres = 0;
        const bool pro = a.gn_stats != nullptr || a.pre_act != 0;
        if (!pro && nps_conv1x1_res_plan(a, all, &rncb, &rng, &rnres)) {
            // conv1x1_res_kernel: chunks [0, nres), blocks [0, ng * NCB) (group grp at grp * NCB)
            top((rnres - 1) * gstride + (long)rng * rncb * 2048);
        } else if (a.Cout <= 192 || g_x1_groups) {
            // conv1x1_wl_kernel<6, *>: wfetch(min(st + 2, last)) -> chunks 2 last + 1, 6 blocks of the chunk at
            // its group's offset (ng groups of 6 blocks)
            top((2 * nst - 1) * gstride + (long)((a.Cout + 191) / 192) * 6 * 2048);
        } else {
            // conv1x1_x3_kernel: wave block min(cob, ncb / 2 - 1) x 2 blocks, chunks 2 st + k
            top((2 * nst - 1) * gstride + ncb * 2048);
        }
    } else {
        const long nstages = (a.Cin + CK - 1) / CK;
        const long G = nstages * nt;                  // K-groups; loads clamp to G - 1 (gclamp)
        const bool wide = x3_wide_tile(a);
        const long nco = wide ? 192 : 64;             // channels per work-group tile
        const long ncob = (a.Cout + nco - 1) / nco;
        top((G - 1) * gstride + ncob * (nco / 32) * 2048);
    }
    if (a.nphase > 1) span += (long)(a.nphase - 1) * a.phase_wstride * 4;  // phase p's weight at p * phase_wstride floats
    return span;
}
