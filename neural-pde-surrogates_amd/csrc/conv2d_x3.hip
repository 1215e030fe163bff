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
//     [16 hi | 16 lo] fp16 + 16 B pad (80 B, conflict-free ds_read_b128).  Producer waves 4-7 fetch
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
#define X3_MFMA16 __builtin_amdgcn_mfma_f32_16x16x32_f16
#ifndef NPS_X3_M16
#define NPS_X3_M16 0  // 1: wide tiles on tap-paired 16x16x32 consumers (x3_consume_m16; dev variant, 3 % slower:
                      // profiles/r5/experiments/x3_m16_tap_paired_ab.txt); 0 = the 32x32x16 consumers
#endif
#ifndef NPS_X3_PRIO
#define NPS_X3_PRIO 1
#endif
#ifndef NPS_X3_REMAP
#define NPS_X3_REMAP 0
#endif
#ifndef NPS_X3_ARING
#define NPS_X3_ARING 2  // weight-fragment ring depth of the 64-channel tiles
#endif
#ifndef NPS_X3_ARING_WIDE
#define NPS_X3_ARING_WIDE 3  // ... of the wide tiles: two K-groups ahead (3x3 class -3.5 %, profiles/r4/experiments)
#endif
#ifndef NPS_X3F_ABL
#define NPS_X3F_ABL 0  // dev ablations of conv2d_x3f_kernel (speed only): 1 no patch fetch, 2 no spread stores,
                       // 3 no producer units, 4 = 1 + 2
#endif
#ifndef NPS_X3_ABL
#define NPS_X3_ABL 0  // dev ablations of the 3x3 main loop; 0 in every shipped build
#endif
// Producer slot -> (patch pixel, channel quad).  REMAP: the 16 lanes of one ds_write_b64 group take
// pixels {0, 2, 4, 6} (lanes 16-31: {1, 3, 5, 7}) of a run of 8, whose 32-B [hi] / [lo] runs at the 80-B
// pixel pitch land on disjoint banks (consecutive pixels collide: 20 p mod 32 repeats within 4).
__device__ __forceinline__ int x3_slot_px(int idx) {
#if NPS_X3_REMAP
    const int j = idx & 31;
    return ((idx >> 5) << 3) + ((j >> 2) & 3) * 2 + (j >> 4);
#else
    return idx >> 2;
#endif
}

#ifdef NPS_X3_STAMP  // dev diagnostic: per-work-group s_memtime stamps of consumer wave 0
__device__ unsigned long long x3_stamps[1 << 20];
#define X3_STAMP(i) \
    if (wave == 0 && lane == 0 && l < (1 << 16)) x3_stamps[l * 16 + (i)] = __builtin_amdgcn_s_memtime()
#define X3_RSTAMP(i) \
    if (wave == 0 && lane == 0 && l < (1 << 16)) x3_stamps[l * 16 + (i)] = __builtin_amdgcn_s_memrealtime()
#else
#define X3_STAMP(i)
#define X3_RSTAMP(i)
#endif

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

// Wide-tile consumers on v_mfma_f32_16x16x32_f16 with TAP-PAIRED K (NPS_X3_M16, default).  Under the DVFS
// clock the 16x16x32 shape delivers 1.12-1.15x the FLOP/s of 32x32x16 on random operands at equal cycles
// per FLOP (MI355X_MICROARCH "DVFS give-back" item 7), and this kernel is clock-held (0.55 of 833 TF/s on
// zero operands, 0.40 on random ones: DESIGN.md § Round 4).  K of one MFMA = 16 channels of tap t (k 0-15)
// + the same 16 channels of tap t + 1 (k 16-31), so the split-fp16 passes stay three per 16 input channels
// and tap (hi*lo, hi*hi, lo*hi over a PAIR of taps: 3 MFMAs of 16 cycles per 16x16 block = the 96 cycles per
// 32x32 block and tap of the 32x32x16 form) and neither operand is duplicated:
//   * A (weights) reads the existing packing: lane l = (co row l & 15, channel half (l >> 4) & 1, tap half
//     l >> 5) takes the 16-B piece that lane (co & 31) + 32 * half of the 32x32x16 fragment of its tap holds;
//     the two tap halves are two K-groups of the packed weight (per-lane addresses, 256-B runs);
//   * B (patch) reads 16 B per lane from LDS: pixel l & 15 of the block, channel half, tap half — a pair may
//     straddle two stages (tap 8 of stage s, tap 0 of s + 1): both are in the ring (stage s + 1 is committed
//     one stage ahead), and the stage barrier follows the group holding the stage's last tap;
//   * a flattened K-group count G = nstages * NTAPS that is odd ends with a half-empty pair: its second half
//     reads zero weights (x3_zero_w) against a re-read of the real patch window.
// A wave owns 96 channels (6 blocks of 16) x 64 pixels (4 blocks of 16): 24 f32x4 accumulators, as before.
// MFMA order co-block outer: a block's weight fragments are dead after its 12 MFMAs of the pair, and the next
// pair's fragments of that block load into the same registers (one pair = 72 MFMAs of cover, as the 32x32x16
// consumers' 3-slot ring), while the patch operands are double-buffered (the next pair's 8 reads issued at the
// top of this one).  Epilogue: the tile into LDS and x3_store_phase, as the 32x32x16 consumers.
__device__ __attribute__((aligned(64))) float x3_zero_w[1536];  // 6 KiB of zero weights (the odd tail's empty half)

template <int NTAPS, int NCO, int TILE_PX, bool PRO, typename Decode, typename Barrier>
__device__ __forceinline__ void x3_consume_m16(const nps_conv2d_t& a, const Geo& g, const char* ring, const float* btab,
                                               int stage_b, int nstages, int nwg, Decode& decode, Barrier& barrier) {
    constexpr int KWT = NTAPS == 9 ? 3 : 2;
    constexpr int CB = 6, PBn = 4;  // 16-channel co blocks x 16-pixel blocks of a wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int px0 = (wave >> 1) * 64, cw0 = (wave & 1) * 96;
    const int l16 = lane & 15, kb = lane >> 4, kh = kb & 1, th = kb >> 1;
    int boff[PBn];
#pragma unroll
    for (int pb = 0; pb < PBn; ++pb) {
        const int P = px0 + pb * 16 + l16;
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        boff[pb] = (ti * g.PW + tj) * X3_PIXB + kh * 16;
    }
    f32x4 acc[CB][PBn];
    const int ncb = packed_ncb(a.Cout);         // 6: wide tiles are Cout == 192 (x3_wide_eligible)
    const size_t gstride = (size_t)ncb * 2048;  // bytes per K-group (chunk, tap) of the packed weight
    const int G = nstages * NTAPS;
    const int GP = (G + 1) >> 1;                // tap pairs
    // this lane's byte offset inside a 32-co block fragment: row l16 (+256 B for the odd 16-co block), channel
    // half kh (the 32x32x16 fragment's lanes 32-63); 16-co block b of the wave at ((b >> 1) * 2048 + (b & 1) * 256)
    const int loff = (l16 + 32 * kh) * 16;
    const char* wbase = nullptr;
    f16x8 Aw[CB][2];
    f16x8 Bh[2][PBn], Bl[2][PBn];
    auto apair = [&](int gp) {  // this lane's weight row of pair gp (the odd tail's empty half: zeros)
        const int t = 2 * gp + th;
        return t < G ? wbase + (size_t)t * gstride : reinterpret_cast<const char*>(x3_zero_w) + loff;
    };
    auto boffs = [&](int t) {  // byte offset of flattened tap t's patch window in the LDS ring
        const int st = t / NTAPS, tap = t - (t / NTAPS) * NTAPS;
        return (st % X3_NST) * stage_b + ((tap / KWT) * g.PW + tap % KWT) * X3_PIXB;
    };
    auto bsel = [&](int gp) {  // this lane's tap of pair gp (the odd tail's empty half re-reads the real tap)
        const int t = 2 * gp + th;
        return boffs(t < G ? t : 2 * gp);
    };
    auto loadB = [&](int gp, f16x8 (&dh)[PBn], f16x8 (&dl)[PBn]) __attribute__((always_inline)) {
        const char* p = ring + bsel(gp);
#pragma unroll
        for (int pb = 0; pb < PBn; ++pb) {
            dl[pb] = *reinterpret_cast<const f16x8*>(p + boff[pb] + 32);
            dh[pb] = *reinterpret_cast<const f16x8*>(p + boff[pb]);
        }
    };
    const float xsc = (PRO && a.gn_stats != nullptr) ? gn_prologue_scale(a) : in_scale_of(a);
    const size_t wbody = packed_body(a.Cout, a.Cin, NTAPS);
    float amax = 0.f;
    for (int l = blockIdx.x; l < nwg; l += gridDim.x) {
        int cob, b, oy0, ox0, ph;
        decode(l, cob, b, oy0, ox0, ph);
        const float* wph = a.wpack + (size_t)ph * a.phase_wstride;
        const float inv = 1.f / (pow2_scale_for(wph[wbody]) * xsc);
        wbase = reinterpret_cast<const char*>(wph) + (size_t)cob * (NCO / 32) * 2048 + (cw0 >> 5) * 2048 + loff;
#pragma unroll
        for (int i = 0; i < CB; ++i)
#pragma unroll
            for (int j = 0; j < PBn; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
            const char* p = apair(0);
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
                Aw[cb][0] = *reinterpret_cast<const f16x8*>(p + (cb >> 1) * 2048 + (cb & 1) * 256);
                Aw[cb][1] = *reinterpret_cast<const f16x8*>(p + (cb >> 1) * 2048 + (cb & 1) * 256 + 1024);
            }
        }
        barrier();
        loadB(0, Bh[0], Bl[0]);
        // pair gp: patch operands in slot r, the next pair's into r ^ 1; each co block's next weights load
        // right after that block's last MFMA (hi after the hi*lo and hi*hi passes, lo after lo*hi)
        auto group = [&](int gp, const int r) __attribute__((always_inline)) {
            const int gn = gp + 1 < GP ? gp + 1 : gp;
            loadB(gn, Bh[r ^ 1], Bl[r ^ 1]);
            const char* pa = apair(gn);
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
#pragma unroll
                for (int pb = 0; pb < PBn; ++pb)
                    acc[cb][pb] = X3_MFMA16(Aw[cb][0], Bl[r][pb], acc[cb][pb], 0, 0, 0);  // hi * lo
#pragma unroll
                for (int pb = 0; pb < PBn; ++pb)
                    acc[cb][pb] = X3_MFMA16(Aw[cb][0], Bh[r][pb], acc[cb][pb], 0, 0, 0);  // hi * hi
                Aw[cb][0] = *reinterpret_cast<const f16x8*>(pa + (cb >> 1) * 2048 + (cb & 1) * 256);
#pragma unroll
                for (int pb = 0; pb < PBn; ++pb)
                    acc[cb][pb] = X3_MFMA16(Aw[cb][1], Bh[r][pb], acc[cb][pb], 0, 0, 0);  // lo * hi
                Aw[cb][1] = *reinterpret_cast<const f16x8*>(pa + (cb >> 1) * 2048 + (cb & 1) * 256 + 1024);
            }
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
                if (cb < 2) {  // the next pair's 8 patch reads, one per MFMA gap in the first two blocks
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                } else {
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // next hi fragment of block cb
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // next lo fragment of block cb
            }
            __builtin_amdgcn_sched_barrier(0);
            const int t0 = 2 * gp;
            if (t0 % NTAPS == NTAPS - 1 || (t0 + 1 < G && (t0 + 1) % NTAPS == NTAPS - 1)) barrier();
            __builtin_amdgcn_sched_barrier(0);
        };
        int gp = 0;
        for (; gp + 2 <= GP; gp += 2) {
            group(gp, 0);
            group(gp + 1, 1);
        }
        if (gp < GP) group(gp, 0);
        // the ring is free (every read of it completed before the last stage barrier): the tile goes to LDS
        // (16x16 accumulator: lane holds pixel l16, channels 4 kb + [0, 4) of its block), then all 8 waves store it
        float* T = reinterpret_cast<float*>(const_cast<char*>(ring));
#pragma unroll
        for (int pb = 0; pb < PBn; ++pb) {
            const int P = px0 + pb * 16 + l16;
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
                const f32x4 v = acc[cb][pb] * inv;
                *reinterpret_cast<f32x4*>(T + P * (NCO + 4) + cw0 + cb * 16 + 4 * kb) = v;
            }
        }
        barrier();
        x3_store_phase<TILE_PX, NCO>(a, b, cob, oy0, ox0, g.T, ph, T, btab, tid, amax,
                                     reinterpret_cast<double*>(const_cast<char*>(ring) - 128));
        barrier();  // the staged tile is fully read: the producers may refill the ring
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}

// PRO: the frame prologue (GroupNorm affine and/or GELU, proc_unet_modern.py:62-99) is applied by the
// producers while staging, instead of a frame_pack pass in front of the conv.
// WIDE: the work-group covers 192 output channels x 128 pixels instead of 64 x 4*PB*32: consumer wave w
// owns channels [96 (w & 1), +96) (3 co blocks) x pixels [64 (w >> 1), +64) (2 pixel blocks).  The staged
// patch then feeds all 192 channels: 3x less producer work (fetch, split, prologue) and patch traffic per
// MFMA than three 64-channel work-groups re-staging the same patch.
template <int NTAPS, int PB, bool PRO, bool WIDE = false, bool PST = false>
__global__ __launch_bounds__(512) void conv2d_x3_kernel(const nps_conv2d_t a) {
    constexpr int KWT = NTAPS == 25 ? 5 : (NTAPS == 9 ? 3 : (NTAPS == 4 ? 2 : 1));
    constexpr int CBW = WIDE ? 3 : 2;          // 32-channel co blocks per consumer wave
    constexpr int PBW = WIDE ? 2 : PB;         // 32-pixel blocks per consumer wave
    constexpr int NCO = WIDE ? 192 : 64;       // output channels per work-group
    constexpr int TILE_PX = WIDE ? 128 : 4 * PB * 32;
    constexpr int MAXP = (x3_patch_px_max(NTAPS, TILE_PX) * 4 + 255) / 256;
    constexpr bool SPREAD = WIDE && NPS_X3_SPREAD;  // wide tiles: spread store (dev knob: the store phase)
    constexpr bool M16 = WIDE && !SPREAD && NPS_X3_M16;  // wide tiles: tap-paired 16x16x32 consumers
    static_assert(!PST || (WIDE && !SPREAD && !M16), "producer-side store: wide 32x32x16 tiles only");
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
    const int stage_b = (npix * X3_PIXB + 15) & ~15;
    char* ring = reinterpret_cast<char*>(smem) + 128;
    // bias table of the LDS store phase, behind the ring / tile region (x3_lds_bytes); first read after the
    // first barrier of the tile loop
    float* btab = reinterpret_cast<float*>(ring + x3_region_bytes(a));
    for (int c = tid; c < a.Cout; c += 512) btab[c] = a.bias != nullptr ? a.bias[c] : 0.f;
#if NPS_X3_ABL == 9
    // dev ablation (wrong results, speed only): the wide consumers read their weight fragments from LDS — 3 K-groups
    // (36 KiB of real packed weight bits, so the MFMA operands toggle as in the real stream) behind the store-phase
    // tile, in the part of the wide-tile region nothing else touches — the ceiling of a weights-through-LDS design
    // without its producer-side copy
    if constexpr (WIDE) {
        for (int i = tid; i < 3 * 12288 / 16; i += 512)
            *reinterpret_cast<f32x4*>(ring + 100352 + i * 16) =
                *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(a.wpack) + i * 16);
    }
#endif
    const int nstages = (a.Cin + CK - 1) / CK;
    const int last = nstages - 1;
    const bool lds_epi = WIDE || x3_lds_epilogue(a);  // wide tiles: always (x3_wide_eligible)
    auto barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

    // static priority for the producer half (MI355X_MICROARCH 'Two waves per SIMD' item 4): they win the
    // VALU arbitration against their SIMD partner's MFMA stream; same-box A/B: 3x3 class -1.7 % per call
    // (NPS_X3_PRIO=0 / 2: none / the consumers instead)
#if NPS_X3_PRIO == 1
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#elif NPS_X3_PRIO == 2
    if (wave < 4) __builtin_amdgcn_s_setprio(1);
#endif
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
                    char* base = Pt + x3_slot_px(idx) * X3_PIXB + (idx & 3) * 8;
#if NPS_X3_ABL == 7  // dev ablation: the commit's arithmetic without its LDS writes (values kept live)
                    {
                        typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
                        const u32x2_t hb = __builtin_bit_cast(u32x2_t, hi), lb = __builtin_bit_cast(u32x2_t, lo);
                        asm volatile("" ::"v"(hb[0] ^ lb[0]), "v"(hb[1] ^ lb[1]));
                    }
#elif NPS_X3_ABL == 8  // dev ablation: the LDS writes of constant data (no fetch wait, no arithmetic)
                    *reinterpret_cast<f16x4*>(base) = f16x4{0, 0, 0, 0};
                    *reinterpret_cast<f16x4*>(base + 32) = f16x4{0, 0, 0, 0};
#else
                    *reinterpret_cast<f16x4*>(base) = hi;
                    *reinterpret_cast<f16x4*>(base + 32) = lo;
#endif
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
        if constexpr (PST) {
            // Producer-side store (wide tiles): the consumers drop tile t into the tile region Tw (its own LDS
            // region behind the ring) and go straight on to tile t + 1; the producers store tile t from Tw during
            // tile t + 1's stage iterations, in NCH chunks of 4 items per thread (item = one pixel's 4 channels,
            // 16 B; consecutive threads walk a pixel's NCO channels: x3_store_phase's coalesced order and float
            // order).  Chunk c's operand loads (addends, the accumulated output) are issued at stage s(c), after
            // that stage's patch fetch, and the chunk is finished at the next stage iteration, after the commit —
            // so no wait of the in-order vmcnt queue stalls a patch fetch.  The last chunk finishes before the
            // tile's last stage barrier, after which the consumers overwrite Tw.  No store phase: per tile
            // 1 + nstages barriers on both sides (the consumers' MFMAs run while the tile is stored).
            constexpr int PQ = NCO / 4;                  // channel quads per pixel
            constexpr int PITEMS = TILE_PX * PQ / 256;  // items per producer thread and tile (24)
            static_assert(PITEMS % 4 == 0, "4-item chunks");
            constexpr int NCH = PITEMS / 4;
            const float* Tw = reinterpret_cast<const float*>(ring + x3_ring_bytes(a));
            // (host-checked: at most one operand, the accumulated output or addend0)
            const float* opp = a.accumulate ? a.out : a.addend0;
            const bool oper = opp != nullptr;
            const bool pipe = nstages > NCH;  // one chunk per stage, loads a stage ahead
            int p_b = 0, p_cob = 0, p_oy0 = 0, p_ox0 = 0, p_ph = 0;  // the tile being stored
            bool pend = false;
            int fl_c = -1;  // chunk whose operand loads are in flight
            double ps1 = 0.0, ps2 = 0.0;
            f32x4 iop[4];
            auto item_at = [&](int k, int& P, int& q, size_t& off, bool& ok) {
                const int i = ptid + 256 * k;
                P = i / PQ;
                q = i - P * PQ;
                const int co0 = p_cob * NCO + q * 4;
                const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
                const int oy = p_oy0 + ti * g.T, ox = p_ox0 + tj * g.T;
                const int dy = oy * a.out_os + a.out_off_y + (p_ph >> 1), dx = ox * a.out_os + a.out_off_x + (p_ph & 1);
                ok = co0 < a.Cout && oy < a.Hout && ox < a.Wout && dy >= 0 && dy < a.out_H && dx >= 0 && dx < a.out_W;
                off = ok ? (((size_t)p_b * a.out_H + dy) * a.out_W + dx) * a.out_C + co0 : 0;
            };
            auto chunk_issue = [&](int c) {
                if (!oper) return;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    int P, q;
                    size_t off;
                    bool ok;
                    item_at(4 * c + j, P, q, off, ok);
                    // out-of-range items read the zero page (no branch around a load)
                    iop[j] = *reinterpret_cast<const f32x4*>(ok ? opp + off : x3_zero16);
                }
            };
            auto chunk_finish = [&](int c) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    int P, q;
                    size_t off;
                    bool ok;
                    item_at(4 * c + j, P, q, off, ok);
                    const f32x4 acc = *reinterpret_cast<const f32x4*>(Tw + P * (NCO + 4) + q * 4);
                    const f32x4 bi = *reinterpret_cast<const f32x4*>(btab + (ok ? p_cob * NCO + q * 4 : 0));
                    f32x4 r;
                    float f1 = 0.f, f2 = 0.f;
                    if (!oper) {  // x3_store_phase's operand-free form
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float v = acc[e] + bi[e];
                            if (a.act == 1) v = nps::gelu_erf(v);
                            r[e] = v;
                            pmax = ok ? fmaxf(pmax, fabsf(v)) : pmax;
                            f1 += v;
                            f2 += v * v;
                        }
                    } else if (a.accumulate) {  // x3_store_phase's float order with zero addends
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float v = acc[e] + bi[e];
                            if (!a.add_after_act) v = v + 0.f + 0.f;
                            if (a.act == 1) v = nps::gelu_erf(v);
                            if (a.add_after_act) v = v + 0.f + 0.f;
                            v += iop[j][e];
                            r[e] = v;
                            pmax = ok ? fmaxf(pmax, fabsf(v)) : pmax;
                            f1 += v - iop[j][e];
                            f2 += (v - iop[j][e]) * (v + iop[j][e]);
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float v = acc[e] + bi[e];
                            if (!a.add_after_act) v = v + iop[j][e] + 0.f;
                            if (a.act == 1) v = nps::gelu_erf(v);
                            if (a.add_after_act) v = v + iop[j][e] + 0.f;
                            r[e] = v;
                            pmax = ok ? fmaxf(pmax, fabsf(v)) : pmax;
                            f1 += v;
                            f2 += v * v;
                        }
                    }
                    float* dst = ok ? a.out + off : x3_sink + 4 * (tid & 63);
                    *reinterpret_cast<f32x4*>(dst) = r;
                    ps1 += ok ? (double)f1 : 0.0;
                    ps2 += ok ? (double)f2 : 0.0;
                }
            };
            auto tile_done = [&]() {
                stats_publish(a, p_b, ps1, ps2);  // the tile's moments: one pair per wave (no-op without out_stats)
                ps1 = ps2 = 0.0;
                pend = false;
            };
            for (;;) {
                const int tcob = fcob, tb = fb, ty0 = fy0, tx0 = fx0, tph = fph;  // tile computed now
                commit(0, r0, m0);
                if (nstages > 1) commit(1, r1, m1);
                unsigned m = issue(min(2, last), r0);
                barrier();  // (the consumers' previous tile is in Tw)
                const int ln = l + (int)gridDim.x;
                const bool more = ln < nwg;
                bool got0 = false, got1 = false;
                for (int st = 0; st < nstages; ++st) {
                    if (st + 2 < nstages) commit(st + 2, r0, m);
                    if (pend) {
                        if (pipe) {
                            if (fl_c >= 0) chunk_finish(fl_c);
                            fl_c = -1;
                        } else {
                            for (int c = 0; c < NCH; ++c)
                                if ((c * nstages) / NCH == st) {
                                    chunk_issue(c);
                                    chunk_finish(c);
                                }
                        }
                    }
                    // the next patch stage, or the next tile's first two (as the spread-store loop below)
                    if (st + 3 <= last) {
                        m = issue(st + 3, r0);
                    } else if (more && st == last - 2) {
                        decode(ln, fcob, fb, fy0, fx0, fph);
                        cur_src = -1;
                        m0 = issue(0, r0);
                        got0 = true;
                    } else if (got0 && st == last - 1) {
                        m1 = issue(min(1, last), r1);
                        got1 = true;
                    }
                    if (pend && pipe) {
#pragma unroll 1
                        for (int c = 0; c < NCH; ++c)
                            if ((c * (nstages - 1)) / NCH == st) {
                                chunk_issue(c);
                                fl_c = c;
                            }
                    }
                    if (pend && st == last) tile_done();
                    barrier();
                }
                p_b = tb;
                p_cob = tcob;
                p_oy0 = ty0;
                p_ox0 = tx0;
                p_ph = tph;
                pend = true;
                if (!more) break;
                if (!got0) {
                    decode(ln, fcob, fb, fy0, fx0, fph);
                    cur_src = -1;
                    m0 = issue(0, r0);
                }
                if (!got1) m1 = issue(min(1, last), r1);
                l = ln;
            }
            barrier();  // the last tile is in Tw
#pragma unroll 1
            for (int c = 0; c < NCH; ++c) {
                chunk_issue(c);
                chunk_finish(c);
            }
            tile_done();
            nps::tag_publish(a.out_tag, pmax, nps::wave_salt());
            return;
        }
        if constexpr (SPREAD) {
            // Wide tiles: the consumers store each tile during the next one's main loop, so the producers have
            // no store phase: per tile 1 + nstages barriers, and the next tile's first two stages are fetched
            // into r0 / r1 by the last stage iterations of this one (where the fetch of stage st + 3 would run
            // past the end), then committed as soon as the last stage's barrier frees the ring.
            for (;;) {
                commit(0, r0, m0);
                if (nstages > 1) commit(1, r1, m1);
                unsigned m = issue(min(2, last), r0);
                barrier();
                const int ln = l + (int)gridDim.x;
                const bool more = ln < nwg;
                bool got0 = false, got1 = false;
                for (int st = 0; st < nstages; ++st) {
                    if (st + 2 < nstages) commit(st + 2, r0, m);
                    if (st + 3 <= last) {
                        m = issue(st + 3, r0);
                    } else if (more && st == last - 2) {  // r0 is free after the commit of stage `last`
                        decode(ln, fcob, fb, fy0, fx0, fph);
                        cur_src = -1;
                        m0 = issue(0, r0);
                        got0 = true;
                    } else if (got0 && st == last - 1) {  // r1 has been free since this tile's top
                        m1 = issue(min(1, last), r1);
                        got1 = true;
                    }
                    barrier();
                }
                if (!more) break;
                if (!got0) {
                    decode(ln, fcob, fb, fy0, fx0, fph);
                    cur_src = -1;
                    m0 = issue(0, r0);
                }
                if (!got1) m1 = issue(min(1, last), r1);
                l = ln;
            }
            return;
        }
        for (;;) {
            const int scob = fcob, sb = fb, soy0 = fy0, sox0 = fx0, sph = fph;  // tile being computed / stored
            commit(0, r0, m0);
            if (nstages > 1) commit(1, r1, m1);
            unsigned m = issue(min(2, last), r0);
            barrier();
            for (int st = 0; st < nstages; ++st) {
#if NPS_X3_ABL == 4  // dev ablation: the producers only keep the barriers (stale patch)
                barrier();
                continue;
#elif NPS_X3_ABL == 5  // dev ablation: fetch only (no GroupNorm/GELU/split/LDS commit)
                m = issue(min(st + 3, last), r0);
                barrier();
                continue;
#elif NPS_X3_ABL == 6 || NPS_X3_ABL == 7 || NPS_X3_ABL == 8  // dev ablations: commit only (stale registers, no
                if (st + 2 < nstages) commit(st + 2, r0, m);                      // fetch); 7, 8: see commit
                barrier();
                continue;
#endif
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
    if constexpr (M16) {
        x3_consume_m16<NTAPS, NCO, TILE_PX, PRO>(a, g, ring, btab, stage_b, nstages, nwg, decode, barrier);
        return;
    }
    int boff[PBW];
    const int px0 = WIDE ? (wave >> 1) * 64 : wave * 32 * PB;  // this wave's first tile pixel
    const int cw0 = WIDE ? (wave & 1) * 96 : 0;                // this wave's first channel in the co group
#pragma unroll
    for (int pb = 0; pb < PBW; ++pb) {
        const int P = px0 + pb * 32 + (lane & 31);
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        boff[pb] = (ti * g.PW + tj) * X3_PIXB + (lane >> 5) * 16;
    }
    f32x16 acc[CBW][PBW];
    const int ncb = packed_ncb(a.Cout);
    const size_t gstride = (size_t)ncb * 2048;  // bytes per K-group (chunk, tap) of the packed weight
    const int G = nstages * NTAPS;
    const char* wbase = nullptr;
    // weight fragments: a ring of NPS_X3_ARING K-groups (2: loaded one K-group ahead; 3: two ahead)
    constexpr int AR = WIDE ? NPS_X3_ARING_WIDE : NPS_X3_ARING;
    f16x8 Aw[AR][CBW][2];
    f16x8 Bh[2][PBW], Bl[2][PBW];
    auto loadA = [&](int gg, f16x8 (&d)[CBW][2]) {
#if NPS_X3_ABL == 9
        if constexpr (WIDE) {
            const char* q = ring + 100352 + (gg % 3) * 12288 + (cw0 / 32) * 2048 + lane * 16;
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb) {
                d[cb][0] = *reinterpret_cast<const f16x8*>(q + cb * 2048);
                d[cb][1] = *reinterpret_cast<const f16x8*>(q + cb * 2048 + 1024);
            }
            return;
        }
#endif
        const char* p = wbase + (size_t)gg * gstride;
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb) {
            d[cb][0] = *reinterpret_cast<const f16x8*>(p + cb * 2048);
            d[cb][1] = *reinterpret_cast<const f16x8*>(p + cb * 2048 + 1024);
        }
    };
    auto boffs = [&](int gg) {  // byte offset of K-group gg's patch window in the LDS ring
        const int st = gg / NTAPS, tap = gg - (gg / NTAPS) * NTAPS;
        return (st % X3_NST) * stage_b + ((tap / KWT) * g.PW + tap % KWT) * X3_PIXB;
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
#ifdef NPS_X3_STAMP
    unsigned long long bar_cycles = 0;  // consumer wave 0: cycles spent in the stage barriers
#endif
    // Spread store (wide tiles): wave w drops its own 96-channel x 64-pixel block of tile t into the epilogue
    // tile region Tw (behind the ring), then stores that block during tile t + 1's main loop, one 64-lane item
    // (16 B per lane: one pixel's 4 channels) every sp_every K-groups — no store phase, no barrier (a wave only
    // ever reads back the block it wrote), and the output write stream is spread over the main loop instead of
    // every CU bursting 96 KiB at once.  The item's epilogue is x3_store_phase's (bias from the LDS table,
    // addends, GELU, accumulate, range tag, GroupNorm moments, same float order); its operand loads are issued
    // before the K-group's MFMAs and consumed after them.
    constexpr int SPQ = 24;                  // channel quads of a wave's 96-channel block
    constexpr int SP_ITEMS = 64 * SPQ / 64;  // 64 pixels x 24 quads / 64 lanes
    float* Tw = reinterpret_cast<float*>(ring + x3_ring_bytes(a));
    const int tw_sh = __builtin_ctz((unsigned)a.TW);  // wide tiles: TW in {4, 8, 16, 32}
    const bool sp_oper = a.accumulate || a.addend0 != nullptr || a.addend1 != nullptr;
    int sp_n = 0, sp_next = 0, sp_every = 1;  // items left of the pending tile, next K-group with an item
    int sp_b = 0, sp_cob = 0, sp_oy0 = 0, sp_ox0 = 0, sp_ph = 0;
    double sp_s1 = 0.0, sp_s2 = 0.0;
    float sp_amax = 0.f;
    f32x4 sp_v, sp_a0, sp_a1, sp_ov;
    size_t sp_off = 0;
    int sp_co0 = 0;
    bool sp_ok = false;
    auto sp_issue = [&]() __attribute__((always_inline)) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const int i = (SP_ITEMS - sp_n) * 64 + lane;
        const int Pl = i / SPQ, q = i - (i / SPQ) * SPQ;
        const int P = px0 + Pl, col = cw0 + 4 * q;
        sp_co0 = sp_cob * NCO + col;
        const int oy = sp_oy0 + (P >> tw_sh), ox = sp_ox0 + (P & (a.TW - 1));
        const int dy = oy * a.out_os + a.out_off_y + (sp_ph >> 1), dx = ox * a.out_os + a.out_off_x + (sp_ph & 1);
        sp_ok = sp_co0 < a.Cout && oy < a.Hout && ox < a.Wout && dy >= 0 && dy < a.out_H && dx >= 0 && dx < a.out_W;
        sp_off = sp_ok ? (((size_t)sp_b * a.out_H + dy) * a.out_W + dx) * a.out_C + sp_co0 : 0;
        sp_v = *reinterpret_cast<const f32x4*>(Tw + P * (NCO + 4) + col);
        sp_a0 = z;
        sp_a1 = z;
        sp_ov = z;
        if (sp_oper) {  // out-of-range lanes read the zero page
            if (a.addend0 != nullptr)
                sp_a0 = *reinterpret_cast<const f32x4*>(sp_ok ? a.addend0 + sp_off : x3_zero16);
            if (a.addend1 != nullptr)
                sp_a1 = *reinterpret_cast<const f32x4*>(sp_ok ? a.addend1 + sp_off : x3_zero16);
            if (a.accumulate) sp_ov = *reinterpret_cast<const f32x4*>(sp_ok ? a.out + sp_off : x3_zero16);
        }
    };
    auto sp_finish = [&]() __attribute__((always_inline)) {
        const f32x4 bi = *reinterpret_cast<const f32x4*>(btab + (sp_ok ? sp_co0 : 0));
        f32x4 r;
        float f1 = 0.f, f2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // x3_store_phase's float order
            float v = sp_v[e] + bi[e];
            if (!a.add_after_act) v = v + sp_a0[e] + sp_a1[e];
            if (a.act == 1) v = nps::gelu_erf(v);
            if (a.add_after_act) v = v + sp_a0[e] + sp_a1[e];
            if (a.accumulate) v += sp_ov[e];
            r[e] = v;
            sp_amax = sp_ok ? fmaxf(sp_amax, fabsf(v)) : sp_amax;
            f1 += a.accumulate ? v - sp_ov[e] : v;
            f2 += a.accumulate ? (v - sp_ov[e]) * (v + sp_ov[e]) : v * v;
        }
        if (a.out_stats != nullptr) {
            sp_s1 += sp_ok ? (double)f1 : 0.0;
            sp_s2 += sp_ok ? (double)f2 : 0.0;
        }
        float* dst = sp_ok ? a.out + sp_off : x3_sink + 4 * lane;
        *reinterpret_cast<f32x4*>(dst) = r;
        if (--sp_n == 0) stats_publish(a, sp_b, sp_s1, sp_s2);  // the tile's moments: one pair per wave
    };
    auto group = [&](int gg, const int ra, const int r) __attribute__((always_inline)) {  // ra: weight slot of K-group gg, r: patch slot
        bool sp = false;
        if constexpr (SPREAD) {
            sp = sp_n > 0 && gg >= sp_next;  // uniform
            if (sp) sp_issue();
            __builtin_amdgcn_sched_barrier(0);
        }
#if NPS_X3_ABL == 1  // dev ablation (wrong results, speed only): every K-group reads group 0's weights (L1-hot)
        loadA(0, Aw[(ra + AR - 1) % AR]);
#elif NPS_X3_ABL == 2  // dev ablation: waves 2, 3 read group 0's weights (L1-hot), waves 0, 1 the real stream
        loadA(wave >= 2 ? 0 : gclamp(gg + AR - 1), Aw[(ra + AR - 1) % AR]);
#else
        loadA(gclamp(gg + AR - 1), Aw[(ra + AR - 1) % AR]);
#endif
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
            __builtin_amdgcn_sched_group_barrier((NPS_X3_ABL == 9 && WIDE) ? 0x100 : 0x020, 1, 0);  // 1 VMEM read
        }
#pragma unroll
        for (int i = 0; i < 2 * PBW; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * CBW * PBW - 2 * PBW - 2 * CBW, 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SPREAD) {
            if (sp) {
                sp_finish();
                sp_next += sp_every;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if ((gg + 1) % NTAPS == 0) {
#ifdef NPS_X3_STAMP
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            barrier();
            bar_cycles += __builtin_amdgcn_s_memtime() - t0;
#else
            barrier();
#endif
        }
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
        X3_STAMP(0);
        X3_RSTAMP(4);
        loadA(0, Aw[0]);
        if constexpr (AR == 3) loadA(gclamp(1), Aw[1]);
        barrier();
        loadB(0, Bh[0], 0);
        loadB(0, Bl[0], 1);
        X3_STAMP(1);
        int g0 = 0;
        if constexpr (AR == 2) {
            for (; g0 + 2 <= G; g0 += 2) {
                group(g0, 0, 0);
                group(g0 + 1, 1, 1);
#ifdef NPS_X3_STAMP
                if (g0 == 0) X3_STAMP(7);  // first two K-groups done (the first operand waits)
#endif
            }
            if (g0 < G) group(g0, 0, 0);
        } else {  // slots (gg % 3, gg % 2): 6 K-groups per iteration, the tail continues the same pattern
            for (; g0 + 6 <= G; g0 += 6) {
                static_for<6>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    group(g0 + j, j % 3, j % 2);
                });
#ifdef NPS_X3_STAMP
                if (g0 == 0) X3_STAMP(7);
#endif
            }
            static_for<6>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if (g0 + j < G) group(g0 + j, j % 3, j % 2);
            });
        }
        X3_STAMP(2);
#ifdef NPS_X3_STAMP
        if (wave == 0 && lane == 0 && l < (1 << 16)) x3_stamps[l * 16 + 6] = bar_cycles;
        bar_cycles = 0;
#endif
        if constexpr (PST) {
            // the tile into Tw (the producers store it during the next tile's stages, or after the last one);
            // no barrier: the next tile's first barrier publishes it
#pragma unroll
            for (int pb = 0; pb < PBW; ++pb) {
                const int P = px0 + pb * 32 + (lane & 31);
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const f32x4 v = {acc[cb][pb][4 * m] * inv, acc[cb][pb][4 * m + 1] * inv,
                                         acc[cb][pb][4 * m + 2] * inv, acc[cb][pb][4 * m + 3] * inv};
                        *reinterpret_cast<f32x4*>(Tw + P * (NCO + 4) + cw0 + cb * 32 + 8 * m + 4 * h) = v;
                    }
            }
            X3_STAMP(3);
            X3_RSTAMP(5);
            continue;
        }
        if constexpr (SPREAD) {
            // items of the previous tile the main loop had no K-group for (small Cin), then this tile's block
            // into Tw: the wave's own block only, which it alone reads back — no barrier
            while (sp_n > 0) {
                sp_issue();
                sp_finish();
            }
#pragma unroll
            for (int pb = 0; pb < PBW; ++pb) {
                const int P = px0 + pb * 32 + (lane & 31);
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const f32x4 v = {acc[cb][pb][4 * m] * inv, acc[cb][pb][4 * m + 1] * inv,
                                         acc[cb][pb][4 * m + 2] * inv, acc[cb][pb][4 * m + 3] * inv};
                        *reinterpret_cast<f32x4*>(Tw + P * (NCO + 4) + cw0 + cb * 32 + 8 * m + 4 * h) = v;
                    }
            }
            sp_n = SP_ITEMS;
            sp_b = b;
            sp_cob = cob;
            sp_oy0 = oy0;
            sp_ox0 = ox0;
            sp_ph = ph;
            sp_s1 = sp_s2 = 0.0;
            sp_next = 0;
            // the next tile (same Cin, so the same G) stores one item every sp_every K-groups
            sp_every = G > SP_ITEMS ? (G - 1) / (SP_ITEMS - 1) : 1;
            X3_STAMP(3);
            X3_RSTAMP(5);
            continue;
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
            X3_STAMP(8);
            x3_store_phase<TILE_PX, NCO>(a, b, cob, oy0, ox0, g.T, ph, T, btab, tid, amax, reinterpret_cast<double*>(smem));
            X3_STAMP(9);
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
        X3_STAMP(3);
        X3_RSTAMP(5);
    }
    if constexpr (PST) barrier();  // the last tile is in Tw: the producers store it
    if constexpr (SPREAD) {  // the last tile: no next main loop to spread it over
        while (sp_n > 0) {
            sp_issue();
            sp_finish();
        }
        amax = fmaxf(amax, sp_amax);
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}


#ifdef NPS_X3F_KERNEL  // dev build only (tools/build_variant.sh -DNPS_X3F_KERNEL): not in the default library
// tile coordinates of conv2d_x3f_kernel
struct X3Tile {
    int cob, b, oy0, ox0, ph;
};

// ---------------------------------------------------------------------------------------------
// Wide split-fp16 2x2 / 3x3 conv with fused roles: conv2d_x3f_kernel<NTAPS, PRO>.  The same 192-channel x
// 128-pixel tiles, patch ring, weight stream and spread store as conv2d_x3_kernel<NTAPS, 2, PRO, true>, but
// 4 waves (one per SIMD, up to 512 registers each) that are producers AND consumers: every wave stages a
// quarter of the patch and computes its 96-channel x 64-pixel block.  In the 8-wave kernel the producer wave
// and the MFMA wave of a SIMD compete for its instruction issue (the producer's fetch / GroupNorm / GELU /
// split / LDS-write stream costs the MFMA stream 17-24 %: dev ablation NPS_X3_ABL=4, profiles/r4); here the
// producer work of a stage is cut into NU units (half a patch slot each) placed inside the stage's K-groups,
// each unit's ~50 VALU between that group's 18 MFMAs (`sched_group_barrier`: 1 MFMA, 3 VALU), where a wave's
// own VALU issues in the MFMA pipe's shadow.  The stage stream runs across tiles: ring slot = stream stage %
// 3, so the next tile's first stages are fetched and committed during this tile's last ones (no per-tile
// producer prologue).  Three register sets, set = stream stage % 3: during stage s the units commit stage s + 2
// and the last K-group fetches stage s + 4 (a full stage of lead); the fetch goes out after that group's
// weight loads, because vmcnt retires in order and every weight load issued after it waits for it too.  The
// loop body is three stages, so the sets are compile-time.
template <int NTAPS, bool PRO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void conv2d_x3f_kernel(
    const nps_conv2d_t a) {
    constexpr int KWT = NTAPS == 9 ? 3 : 2;
    constexpr int CBW = 3, PBW = 2, NCO = 192;
    constexpr int MAXP = (x3_patch_px_max(NTAPS, 128) * 4 + 255) / 256;  // patch slots per thread per stage
    constexpr int RG = NTAPS == 9 ? 3 : 2;  // operand ring depth in K-groups (divides NTAPS)
    constexpr int NU = 2 * MAXP;            // producer units per stage
    static_assert(NTAPS % RG == 0 && (NTAPS == 9 || NTAPS == 4), "conv2d_x3f: 2x2 / 3x3");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const Geo g = make_geo(a);
    const int ncob = (a.Cout + NCO - 1) / NCO;
    const int ntiles = g.tiles_x * g.tiles_y;
    const int nph = a.nphase > 1 ? a.nphase : 1;
    const int nwg = ntiles * a.B * ncob * nph;
    auto decode = [&](int l, int& cob, int& b, int& oy0, int& ox0, int& ph) {  // as conv2d_x3_kernel
        const int full = nwg & ~7;
        const int L0 = l < full ? (l & 7) * (full >> 3) + (l >> 3) : l;
        ph = L0 % nph;
        const int L = L0 / nph;
        cob = L % ncob;
        const int rest = L / ncob;
        const int tile = rest % ntiles;
        b = rest / ntiles;
        const int ty = tile / g.tiles_x, tx = tile - (tile / g.tiles_x) * g.tiles_x;
        oy0 = ty * a.TH;
        ox0 = tx * a.TW;
    };
    const int npix = g.PH * g.PW;
    const int stage_b = (npix * X3_PIXB + 15) & ~15;
    char* ring = reinterpret_cast<char*>(smem) + 128;
    float* btab = reinterpret_cast<float*>(ring + x3_region_bytes(a));
    for (int c = tid; c < a.Cout; c += 256) btab[c] = a.bias != nullptr ? a.bias[c] : 0.f;
    const int nstages = (a.Cin + CK - 1) / CK;
    const int last = nstages - 1;
    const int mytiles = (int)blockIdx.x < nwg ? (nwg - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const int total = mytiles * nstages;  // stream stages of this work-group
    auto barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

    // ------------------------------------------------------------------ producer state (all 256 threads)
    const int Hext = a.Hin + 2 * a.circ, Wext = a.Win + 2 * a.circ;
    // PRO: GroupNorm + GELU (host-checked: the fused kernel runs no other prologue), compile-time so the producer
    // units are branch-free and share the MFMAs' basic block
    const float xs = PRO ? gn_prologue_scale(a) : in_scale_of(a);
    const double gn_icnt = PRO ? 1.0 / ((double)(a.Cin / a.gn_groups) * a.Hin * a.Win) : 0.0;
    constexpr int NR = MAXP + (PRO ? 3 : 0);
    f32x4 rS[3][NR];
    unsigned mS[3] = {0u, 0u, 0u};
    const int gq = tid & 3;
    const float* sbase[MAXP];
    unsigned pixm = 0, finm = 0;
    int cur_src = -1;
    int ftile = -1;                       // tile (of this work-group) the fetch cursor is in
    int fb = 0, fy0 = 0, fx0 = 0;
    auto locate = [&](int sidx) __attribute__((always_inline)) {
        const nps_src_t S0 = a.src[0], S1 = a.src[1], S2 = a.src[2];
        const int si = a.s2d ? 0 : sidx;
        const float* sptr = si == 0 ? S0.ptr : (si == 1 ? S1.ptr : S2.ptr);
        const int sC = si == 0 ? S0.C : (si == 1 ? S1.C : S2.C);
        const int sH = si == 0 ? S0.H : (si == 1 ? S1.H : S2.H);
        const int sW = si == 0 ? S0.W : (si == 1 ? S1.W : S2.W);
        const int soy = si == 0 ? S0.off_y : (si == 1 ? S1.off_y : S2.off_y);
        const int sox = si == 0 ? S0.off_x : (si == 1 ? S1.off_x : S2.off_x);
        const int ybase = fy0 - a.pad_y, xbase = fx0 - a.pad_x;
        const int s2m = a.s2d ? 2 : 1;
        const int s2y = a.s2d ? (sidx >> 1) - a.s2d_pad : 0, s2x = a.s2d ? (sidx & 1) - a.s2d_pad : 0;
        pixm = 0;
        finm = 0;
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            const int p = x3_slot_px(tid + k * 256);
            const int pr = p / g.PW, pc = p - pr * g.PW;
            const int ye = ybase + pr, xe = xbase + pc;
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
    // fetch stream stage s (tile s / nstages of this work-group) into rp; returns the slot masks (bits 0-15:
    // data inside the source, 16-31: pixel inside the frame)
    auto issue = [&](int s, f32x4 (&rp)[NR]) __attribute__((always_inline)) -> unsigned {
        const int k = s / nstages, st = s - (s / nstages) * nstages;
        if (k != ftile) {  // uniform
            int fcob, fph;
            decode((int)blockIdx.x + k * (int)gridDim.x, fcob, fb, fy0, fx0, fph);
            ftile = k;
            cur_src = -1;
        }
        const int c0 = st * CK;
        const int cend = min(c0 + CK, a.Cin);
        int sidx = 0, cbase = 0;
        if (a.s2d) {
            sidx = c0 / a.src[0].C;
            cbase = sidx * a.src[0].C;
        } else {
            int lo = 0;
#pragma unroll
            for (int si = 0; si < NPS_MAX_SRC; ++si) {
                if (si < a.nsrc) {
                    const int hi = lo + a.src[si].C;
                    if (c0 >= lo && cend <= hi) {
                        sidx = si;
                        cbase = lo;
                    }
                    lo = hi;
                }
            }
        }
        if (sidx != cur_src) {
            locate(sidx);
            cur_src = sidx;
        }
        const bool chok = c0 + gq * 4 < cend;
        const unsigned chm = chok ? ~0u : 0u;
        const int cs = chok ? c0 - cbase + gq * 4 : 0;
#pragma unroll
        for (int q = 0; q < MAXP; ++q) rp[q] = *reinterpret_cast<const f32x4*>(sbase[q] + cs);
        if constexpr (PRO) {
            const int c = chok ? c0 + gq * 4 : 0;
            rp[MAXP] = *reinterpret_cast<const f32x4*>(a.gn_gamma + c);
            rp[MAXP + 1] = *reinterpret_cast<const f32x4*>(a.gn_beta + c);
            rp[MAXP + 2] = *reinterpret_cast<const f32x4*>(
                a.gn_stats + ((size_t)fb * a.gn_groups + c / (a.Cin / a.gn_groups)) * 2);
        }
        return (pixm & chm) | ((finm & chm) << 16);
    };
    // commit of a stream stage, unit u (slot u / 2, elements 2 (u & 1) .. +2): GroupNorm (one FMA, gs / gb
    // derived at unit 0), GELU, then at the slot's second unit the scale, the hi / lo split and one LDS write
    f32x4 gs = {1.f, 1.f, 1.f, 1.f}, gb = {0.f, 0.f, 0.f, 0.f};
    f32x4 cv = {0.f, 0.f, 0.f, 0.f};
    auto commit_unit = [&](int s, const f32x4 (&rp)[NR], unsigned okm, int u) __attribute__((always_inline)) {
        const int k = u >> 1, hh = u & 1;
        if constexpr (PRO) {
            if (u == 0) {
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
        const bool dat = (okm >> k) & 1u, inf = (okm >> (16 + k)) & 1u;
#pragma unroll
        for (int e = 2 * hh; e < 2 * hh + 2; ++e) {
            float v = dat ? rp[k][e] : 0.f;
            if constexpr (PRO) {
                v = nps::gelu_fast(fmaf(v, gs[e], gb[e]));
                v = inf ? v : 0.f;  // the conv's own zero padding (and channels past Cin)
            }
            cv[e] = v;
        }
        if (hh == 1) {
            f16x4 hi, lo;
            split4(cv * xs, hi, lo);
            const int idx = tid + k * 256;
            const int p = x3_slot_px(idx);
            // a slot past the patch writes into the (unused) 128-B header instead: no branch around the writes
            const bool inp = p < npix;
            char* base = inp ? ring + (s % X3_NST) * stage_b + p * X3_PIXB + (idx & 3) * 8
                             : reinterpret_cast<char*>(smem) + (lane & 3) * 32;
            *reinterpret_cast<f16x4*>(base) = hi;
            *reinterpret_cast<f16x4*>(base + (inp ? 32 : 16)) = lo;
        }
    };

    // ------------------------------------------------------------------ consumer state
    int boff[PBW];
    const int px0 = (wave >> 1) * 64;
    const int cw0 = (wave & 1) * 96;
#pragma unroll
    for (int pb = 0; pb < PBW; ++pb) {
        const int P = px0 + pb * 32 + (lane & 31);
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        boff[pb] = (ti * g.PW + tj) * X3_PIXB + (lane >> 5) * 16;
    }
    f32x16 acc[CBW][PBW];
    const int ncb = packed_ncb(a.Cout);
    const size_t gstride = (size_t)ncb * 2048;
    const int G = nstages * NTAPS;
    const char* wbase = nullptr;
    f16x8 Aw[RG][CBW][2];
    f16x8 Bh[RG][PBW], Bl[RG][PBW];
    auto loadA = [&](int gg, f16x8 (&d)[CBW][2]) __attribute__((always_inline)) {
        const char* p = wbase + (size_t)gg * gstride;
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb) {
            d[cb][0] = *reinterpret_cast<const f16x8*>(p + cb * 2048);
            d[cb][1] = *reinterpret_cast<const f16x8*>(p + cb * 2048 + 1024);
        }
    };
    // K-group gg of the tile whose stage 0 is stream stage s0: patch window in ring slot (s0 + gg / NTAPS) % 3
    auto loadB = [&](int s0, int gg, f16x8 (&dh)[PBW], f16x8 (&dl)[PBW]) __attribute__((always_inline)) {
        const int st = gg / NTAPS, tap = gg - (gg / NTAPS) * NTAPS;
        const char* p = ring + ((s0 + st) % X3_NST) * stage_b + ((tap / KWT) * g.PW + tap % KWT) * X3_PIXB;
#pragma unroll
        for (int pb = 0; pb < PBW; ++pb) {
            dh[pb] = *reinterpret_cast<const f16x8*>(p + boff[pb]);
            dl[pb] = *reinterpret_cast<const f16x8*>(p + boff[pb] + 32);
        }
    };
    auto gclamp = [&](int x) { return x < G ? x : G - 1; };
    const float xsc = xs;
    const size_t wbody = packed_body(a.Cout, a.Cin, NTAPS);
    const int h = lane >> 5;
    float amax = 0.f;
    float inv = 0.f;
    int s0 = 0;  // stream stage of the current tile's stage 0
    // spread store (as conv2d_x3_kernel's wide path)
    constexpr int SPQ = 24;
    constexpr int SP_ITEMS = 64 * SPQ / 64;
    float* Tw = reinterpret_cast<float*>(ring + x3_ring_bytes(a));
    const int tw_sh = __builtin_ctz((unsigned)a.TW);
    const bool sp_oper = a.accumulate || a.addend0 != nullptr || a.addend1 != nullptr;
    int sp_n = 0, sp_next = 0, sp_every = 1;
    int sp_b = 0, sp_cob = 0, sp_oy0 = 0, sp_ox0 = 0, sp_ph = 0;
    double sp_s1 = 0.0, sp_s2 = 0.0;
    f32x4 sp_v, sp_a0, sp_a1, sp_ov;
    size_t sp_off = 0;
    int sp_co0 = 0;
    bool sp_ok = false;
    auto sp_issue = [&]() __attribute__((always_inline)) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const int i = (SP_ITEMS - sp_n) * 64 + lane;
        const int Pl = i / SPQ, q = i - (i / SPQ) * SPQ;
        const int P = px0 + Pl, col = cw0 + 4 * q;
        sp_co0 = sp_cob * NCO + col;
        const int oy = sp_oy0 + (P >> tw_sh), ox = sp_ox0 + (P & (a.TW - 1));
        const int dy = oy * a.out_os + a.out_off_y + (sp_ph >> 1), dx = ox * a.out_os + a.out_off_x + (sp_ph & 1);
        sp_ok = sp_co0 < a.Cout && oy < a.Hout && ox < a.Wout && dy >= 0 && dy < a.out_H && dx >= 0 && dx < a.out_W;
        sp_off = sp_ok ? (((size_t)sp_b * a.out_H + dy) * a.out_W + dx) * a.out_C + sp_co0 : 0;
        sp_v = *reinterpret_cast<const f32x4*>(Tw + P * (NCO + 4) + col);
        sp_a0 = z;
        sp_a1 = z;
        sp_ov = z;
        if (sp_oper) {
            if (a.addend0 != nullptr) sp_a0 = *reinterpret_cast<const f32x4*>(sp_ok ? a.addend0 + sp_off : x3_zero16);
            if (a.addend1 != nullptr) sp_a1 = *reinterpret_cast<const f32x4*>(sp_ok ? a.addend1 + sp_off : x3_zero16);
            if (a.accumulate) sp_ov = *reinterpret_cast<const f32x4*>(sp_ok ? a.out + sp_off : x3_zero16);
        }
    };
    auto sp_finish = [&]() __attribute__((always_inline)) {
        const f32x4 bi = *reinterpret_cast<const f32x4*>(btab + (sp_ok ? sp_co0 : 0));
        f32x4 r;
        float f1 = 0.f, f2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v = sp_v[e] + bi[e];
            if (!a.add_after_act) v = v + sp_a0[e] + sp_a1[e];
            if (a.act == 1) v = nps::gelu_erf(v);
            if (a.add_after_act) v = v + sp_a0[e] + sp_a1[e];
            if (a.accumulate) v += sp_ov[e];
            r[e] = v;
            amax = sp_ok ? fmaxf(amax, fabsf(v)) : amax;
            f1 += a.accumulate ? v - sp_ov[e] : v;
            f2 += a.accumulate ? (v - sp_ov[e]) * (v + sp_ov[e]) : v * v;
        }
        if (a.out_stats != nullptr) {
            sp_s1 += sp_ok ? (double)f1 : 0.0;
            sp_s2 += sp_ok ? (double)f2 : 0.0;
        }
        float* dst = sp_ok ? a.out + sp_off : x3_sink + 4 * lane;
#if NPS_X3F_ABL != 2 && NPS_X3F_ABL != 4
        *reinterpret_cast<f32x4*>(dst) = r;
#else
        (void)dst;
#endif
        if (--sp_n == 0) stats_publish(a, sp_b, sp_s1, sp_s2);
    };
    // a tile starts (its stage 0 is stream stage s): decode, zero the accumulators, first operands
    auto tile_start = [&](int s) __attribute__((always_inline)) {
        int cob, b, oy0, ox0, ph;
        decode((int)blockIdx.x + (s / nstages) * (int)gridDim.x, cob, b, oy0, ox0, ph);
        const float* wph = a.wpack + (size_t)ph * a.phase_wstride;
        inv = 1.f / (pow2_scale_for(wph[wbody]) * xsc);
        wbase = reinterpret_cast<const char*>(wph) + (size_t)(cob * (NCO / 32) + cw0 / 32) * 2048 + lane * 16;
        s0 = s;
#pragma unroll
        for (int i = 0; i < CBW; ++i)
#pragma unroll
            for (int j = 0; j < PBW; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        static_for<RG - 1>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            loadA(gclamp(i), Aw[i]);
        });
        loadB(s0, 0, Bh[0], Bl[0]);
        return X3Tile{cob, b, oy0, ox0, ph};
    };
    // a tile ends: the previous tile's leftover items, then this tile's block into Tw and the spread state
    auto tile_end = [&](const X3Tile& t) __attribute__((always_inline)) {
        while (sp_n > 0) {
            sp_issue();
            sp_finish();
        }
#pragma unroll
        for (int pb = 0; pb < PBW; ++pb) {
            const int P = px0 + pb * 32 + (lane & 31);
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const f32x4 v = {acc[cb][pb][4 * m] * inv, acc[cb][pb][4 * m + 1] * inv,
                                     acc[cb][pb][4 * m + 2] * inv, acc[cb][pb][4 * m + 3] * inv};
                    *reinterpret_cast<f32x4*>(Tw + P * (NCO + 4) + cw0 + cb * 32 + 8 * m + 4 * h) = v;
                }
        }
        sp_n = SP_ITEMS;
        sp_cob = t.cob;
        sp_b = t.b;
        sp_oy0 = t.oy0;
        sp_ox0 = t.ox0;
        sp_ph = t.ph;
        sp_s1 = sp_s2 = 0.0;
        sp_next = 0;
        sp_every = G > SP_ITEMS ? (G - 1) / (SP_ITEMS - 1) : 1;
    };

    // ------------------------------------------------------------------ prologue: stream stages 0 .. 3
    if (total > 0) {
        mS[0] = issue(0, rS[0]);
        if (total > 1) mS[1] = issue(1, rS[1]);
        static_for<NU>([&](auto uc) { commit_unit(0, rS[0], mS[0], decltype(uc)::value); });
        if (total > 1) static_for<NU>([&](auto uc) { commit_unit(1, rS[1], mS[1], decltype(uc)::value); });
        if (total > 2) mS[2] = issue(2, rS[2]);
        if (total > 3) mS[0] = issue(3, rS[0]);
    }
    barrier();
    X3Tile cur{0, 0, 0, 0, 0};
    // stream stage s (s % 3 == P): the consumers compute it (tile s / nstages, stage s - s0); the producer units
    // commit stage s + 2 from set (P + 2) % 3 and the last K-group fetches stage s + 4 into set (P + 1) % 3
    auto stage = [&](int s, auto Pc) __attribute__((always_inline)) {
        constexpr int P = decltype(Pc)::value;
        constexpr int SC = (P + 2) % 3, SF = (P + 1) % 3;
        const int st = s - s0;
        const bool do_fetch = s + 4 < total;
        static_for<NTAPS>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            const int gg = st * NTAPS + j;
            const bool sp = sp_n > 0 && gg >= sp_next;
            if (sp) sp_issue();
            __builtin_amdgcn_sched_barrier(0);
            // one basic block per K-group: loads, the producer units and the MFMAs are all unconditional (a
            // branch would split the block, and sched_group_barrier only interleaves inside one): the operand
            // indices clamp, and past the end of the stream the units commit stale registers into the ring slot
            // of stage s + 2, which nothing reads any more
            loadA(gclamp(gg + RG - 1), Aw[(j + RG - 1) % RG]);
            loadB(s0, gclamp(gg + 1), Bh[(j + 1) % RG], Bl[(j + 1) % RG]);
            // this group's producer units (unit u runs in group u * NTAPS / NU)
            static_for<NU>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                if constexpr (u * NTAPS / NU == j && NPS_X3F_ABL != 3) commit_unit(s + 2, rS[SC], mS[SC], u);
            });
            constexpr int ra = j % RG;
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                for (int pb = 0; pb < PBW; ++pb)
                    acc[cb][pb] = X3_MFMA(Aw[ra][cb][0], Bh[ra][pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                for (int pb = 0; pb < PBW; ++pb)
                    acc[cb][pb] = X3_MFMA(Aw[ra][cb][0], Bl[ra][pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                for (int pb = 0; pb < PBW; ++pb)
                    acc[cb][pb] = X3_MFMA(Aw[ra][cb][1], Bh[ra][pb], acc[cb][pb], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 2 * CBW; ++i) {  // weights first, then the patch, VALU in every gap
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
#pragma unroll
            for (int i = 0; i < 2 * PBW; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
#pragma unroll
            for (int i = 0; i < 3 * CBW * PBW - 2 * PBW - 2 * CBW; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (j == NTAPS - 1 && NPS_X3F_ABL != 1 && NPS_X3F_ABL != 4) {  // after this group's weight loads
                if (do_fetch) mS[SF] = issue(s + 4, rS[SF]);
            }
            if (sp) {
                sp_finish();
                sp_next += sp_every;
            }
            __builtin_amdgcn_sched_barrier(0);
        });
        barrier();  // stage s + 2 committed by every wave; every read of stage s's slot done
    };
    auto step = [&](int s, auto Pc) __attribute__((always_inline)) {
        if (s >= total) return;
        if (s == 0 || s - s0 == nstages) {
            if (s > 0) tile_end(cur);
            cur = tile_start(s);
        }
        stage(s, Pc);
    };
    for (int s = 0; s < total; s += 3) {
        step(s, std::integral_constant<int, 0>{});
        step(s + 1, std::integral_constant<int, 1>{});
        step(s + 2, std::integral_constant<int, 2>{});
    }
    if (total > 0) tile_end(cur);
    while (sp_n > 0) {
        sp_issue();
        sp_finish();
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}

#endif  // NPS_X3F_KERNEL

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
template <int NCB, int D, bool PRO = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv1x1_wl_kernel(const nps_conv2d_t a) {
    constexpr int WSTAGE = 2 * NCB * 2048;       // bytes of one stage's weight fragments
    constexpr int WPT = WSTAGE / (256 * 16);     // 16-B pieces per thread per stage
    static_assert(WSTAGE % (256 * 16) == 0, "weight stage split");
    extern __shared__ __attribute__((aligned(16))) char wl[];  // [2][2 chunks][NCB][hi|lo][64][16 B]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.y;
#ifdef NPS_X3_STAMP  // dev diagnostic (tools/x1_stamps.py): per-work-group stamps of wave 0
    const int l = blockIdx.y * gridDim.x + blockIdx.x;
    const int wave = wv;
    X3_STAMP(0);
    X3_RSTAMP(4);
#endif
    const int h = lane >> 5;
    const int npx = a.Hout * a.Wout;
    const int P = blockIdx.x * 128 + wv * 32 + (lane & 31);
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
    const char* wg = reinterpret_cast<const char*>(a.wpack);
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
            (a.bias != nullptr && (int)threadIdx.x < a.Cout) ? a.bias[threadIdx.x] : 0.f;
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
#ifdef NPS_X3_STAMP
    X3_STAMP(1);
#endif
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
#ifdef NPS_X3_STAMP
    X3_STAMP(2);
#endif
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
            const int t0 = (int)blockIdx.x * 128, y0 = t0 / a.Wout, x0 = t0 - y0 * a.Wout;
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
                    const int co0 = cb * 32 + 8 * m + 4 * h;
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
                    const bool ok = pout && co0 < a.Cout;
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
                    const int co0 = cb * 32 + 8 * m + 4 * h;
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
            if (cb * 32 >= a.Cout) continue;
            f32x16 v = acc[cb];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] *= inv;
            store_tile(a, b, cb * 32, h, v, dy, dx, amax);
        }
    }
#ifdef NPS_X3_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores have left this wave
    X3_STAMP(3);
    X3_RSTAMP(5);
#endif
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
    if (a.out_stats != nullptr) {
        // moments of the stored values, recomputed from the accumulators (out_stats on a 1x1 conv:
        // plain epilogue only — bias, no addends / act / accumulate, host-checked); kept out of the store
        // loop, where the extra live values made this kernel spill
        double s1 = 0.0, s2 = 0.0;
        if (pout) {
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                if (cb * 32 >= a.Cout) continue;
                float f1 = 0.f, f2 = 0.f;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int co0 = cb * 32 + 8 * m + 4 * h;
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

#ifdef NPS_X1_DMA_KERNEL  // dev build only (tools/build_variant.sh -DNPS_X1_DMA_KERNEL): not in the default library
// ---------------------------------------------------------------------------------------------
// 1x1 as a persistent HBM stream: conv1x1_dma_kernel<NCB>.  A 1x1 conv moves (Cin + Cout) x 4 B per pixel
// for 2 Cin Cout flops, so it is bound by how many bytes each CU keeps in flight, not by the MFMAs; the
// register-staged kernels above hold one 32-channel stage per wave in flight and stall at every
// work-group's prologue and store drain.  Here one 512-thread work-group per CU walks 128-pixel tiles:
//   * waves 4-7 (loaders) copy each 32-channel stage of the tile's input (128 px x 128 B) and of the packed
//     weights (2 chunks x NCB blocks x 2 KiB) HBM/L2 -> LDS with global_load_lds_dwordx4 (no VGPR round
//     trip), input IA = NS - 1 = 4 stages and weights 2 stages ahead of the MFMA waves, across tile
//     boundaries; a loader wave only ever issues DMAs, so one counted vmcnt per stage retires them;
//   * waves 0-3 (MFMA) own 32 pixels x all NCB*32 output channels each: per 16-channel K-group a lane reads
//     its pixel's 8 channels (2 ds_read_b128), splits them hi/lo and runs 3 MFMAs per 32-channel block
//     against the weight fragments read from LDS; the tile's last stage is followed by the fused epilogue
//     (store_tile: bias, addends, GELU, accumulate, range tag, GroupNorm moments) straight from the
//     accumulators while the loaders' DMAs for the next tile are already in flight.
// Input image per slot: [pixel][8 x 16-B chunks]; chunk c of pixel p lives at chunk c ^ ((p >> 1) & 7)
// (the DMA writes lane-linearly, so the swizzle is on the source address): the 16 lanes of a
// ds_read_b128 group read 16 distinct bank quads.
__host__ __device__ constexpr int x1d_ns(int ncb) { return 5; }  // input ring slots (16 KiB)
constexpr int X1D_NW = 3;                 // weight ring slots (NCB x 4 KiB)
constexpr int X1D_ISLOT = 128 * 128;      // bytes of one input stage: 128 px x 32 ch x 4 B

__host__ __device__ constexpr int x1d_lds_bytes(int ncb) {
    return x1d_ns(ncb) * X1D_ISLOT + X1D_NW * ncb * 4096 + ncb * 32 * 4;
}

__device__ __forceinline__ void x1d_dma16(const void* g, void* lds) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const unsigned*>(g),
                                     (__attribute__((address_space(3))) unsigned*)(lds), 16, 0, 0);
}

// Epilogue of one 32-channel accumulator block of a lane (channels co_base + 8m + 4h + [0, 4), m < 4) at
// NHWC element offset `base` (4-aligned channels), whose accumulator started from bias x (weight scale x
// input scale) — an exact power-of-2 multiple, so acc * inv is the conv plus the bias, rounded once: acc :=
// the stored values (scale, addends, GELU, accumulate, as store_tile_s), max |value| into amax, their moments
// (or, accumulating, the change they make) into (s1, s2).  epi_store writes them; no load follows it.
__device__ __forceinline__ void epi_finish(const nps_conv2d_t& a, size_t base, int co_base, int h, float inv,
                                           f32x16& acc, float& amax, double& s1, double& s2) {
    const bool st = a.out_stats != nullptr;
    float f1 = 0.f, f2 = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int co0 = co_base + 8 * m + 4 * h;
        if (co0 >= a.Cout) continue;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 a0 = a.addend0 ? *reinterpret_cast<const f32x4*>(a.addend0 + base + co0) : z;
        const f32x4 a1 = a.addend1 ? *reinterpret_cast<const f32x4*>(a.addend1 + base + co0) : z;
        const f32x4 o = a.accumulate ? *reinterpret_cast<const f32x4*>(a.out + base + co0) : z;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v = acc[4 * m + e] * inv;  // (the bias is in the accumulator: conv1x1_dma_kernel)
            if (!a.add_after_act) v = v + a0[e] + a1[e];
            if (a.act == 1) v = nps::gelu_erf(v);
            if (a.add_after_act) v = v + a0[e] + a1[e];
            if (a.accumulate) v += o[e];
            acc[4 * m + e] = v;
            amax = fmaxf(amax, fabsf(v));
            if (st) {
                f1 += a.accumulate ? v - o[e] : v;
                f2 += a.accumulate ? (v - o[e]) * (v + o[e]) : v * v;
            }
        }
    }
    if (st) {
        s1 += (double)f1;
        s2 += (double)f2;
    }
}
__device__ __forceinline__ void epi_store(const nps_conv2d_t& a, size_t base, int co_base, int h, const f32x16& v) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int co0 = co_base + 8 * m + 4 * h;
        if (co0 >= a.Cout) continue;
        *reinterpret_cast<f32x4*>(a.out + base + co0) = f32x4{v[4 * m], v[4 * m + 1], v[4 * m + 2], v[4 * m + 3]};
    }
}

template <int NCB>
__global__ __launch_bounds__(512) void conv1x1_dma_kernel(const nps_conv2d_t a) {
    constexpr int WSLOT = NCB * 4096;          // 2 chunks x NCB blocks x (hi, lo) x 1 KiB
    constexpr int NS = x1d_ns(NCB), IA = NS - 1;  // input slots; input stages issued ahead
    constexpr int VMC = NCB + 8;               // loader DMAs allowed in flight at a stage barrier (below)
    static_assert(IA >= 3 && 2 * NCB * 2 % 4 == 0, "conv1x1_dma pipeline");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* iring = reinterpret_cast<char*>(smem);
    char* wring = iring + NS * X1D_ISLOT;
    float* btab = reinterpret_cast<float*>(wring + X1D_NW * WSLOT);  // [NCB * 32] bias x scale (0 past Cout)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int npx = a.Hout * a.Wout;
    const int ptiles = (npx + 127) / 128;      // 128-pixel tiles per sample
    const int ntiles = ptiles * a.B;
    const int nst = (a.Cin + 31) / 32;         // 32-channel stages per tile
    const int mytiles = blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const int U = mytiles * nst;               // stages this work-group runs (every wave: U + 1 barriers)
    auto barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

    if (wave >= 4) {
        // -------------------------------------------------------------- loaders: DMA only
        const int pw = wave - 4;
        const int lo1 = a.src[0].C, lo2 = a.src[0].C + (a.nsrc > 1 ? a.src[1].C : 0);
        const size_t gstride = (size_t)packed_ncb(a.Cout) * 2048;  // bytes per packed 16-channel chunk
        const char* wg = reinterpret_cast<const char*>(a.wpack);
        // Input cursor (next stage to fetch; past the end it re-fetches the last stage into the freed slot,
        // bytes nobody reads).  Per tile, each lane's 4 pixels (DMA instruction i: tile pixels
        // 32 pw + 8 i + lane / 8) are located once in every source; a stage then selects the source of the
        // lane's swizzled 16-B chunk (4 channels, inside one source: host-checked 4-aligned sources).
        const float* pp[4][3];
        int ki = 0, sti = 0, uin = 0;
        auto locate = [&](int k) {
            const int t = (int)blockIdx.x + k * (int)gridDim.x;
            const int b = t / ptiles, P0 = (t - b * ptiles) * 128;
            const nps_src_t S0 = a.src[0], S1 = a.src[1], S2 = a.src[2];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int P = P0 + 32 * pw + 8 * i + (lane >> 3);
                const int oy = P / a.Wout, ox = P - (P / a.Wout) * a.Wout;
                const int ye = oy - a.pad_y, xe = ox - a.pad_x;
                const bool ok = P < npx && ye >= 0 && ye < a.Hin + 2 * a.circ && xe >= 0 && xe < a.Win + 2 * a.circ;
                const int fy = a.circ ? nps::wrap_mod(ye - a.circ, a.Hin) : ye;
                const int fx = a.circ ? nps::wrap_mod(xe - a.circ, a.Win) : xe;
                auto at = [&](const nps_src_t& S) -> const float* {
                    const int yy = fy - S.off_y, xx = fx - S.off_x;
                    return (ok && yy >= 0 && yy < S.H && xx >= 0 && xx < S.W)
                               ? S.ptr + ((size_t)(b * S.H + yy) * S.W + xx) * S.C
                               : nullptr;
                };
                pp[i][0] = at(S0);
                pp[i][1] = a.nsrc > 1 ? at(S1) : nullptr;
                pp[i][2] = a.nsrc > 2 ? at(S2) : nullptr;
            }
        };
        auto issue_in = [&](int u) {  // stage at the cursor -> the ring slot iteration u frees
            if (uin < U && sti == 0) locate(ki);
            char* dst = iring + (u % NS) * X1D_ISLOT;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int px = 32 * pw + 8 * i + (lane >> 3);
                const int ch = sti * 32 + 4 * ((lane & 7) ^ ((px >> 1) & 7));  // the swizzled chunk's channels
                const int si = (ch >= lo1 ? 1 : 0) + (ch >= lo2 ? 1 : 0);
                const float* base = si == 0 ? pp[i][0] : (si == 1 ? pp[i][1] : pp[i][2]);
                const int cl = ch - (si == 0 ? 0 : (si == 1 ? lo1 : lo2));
                const float* src = (base != nullptr && ch < a.Cin) ? base + cl : x3_zero16;
                x1d_dma16(src, dst + (32 * pw + 8 * i) * 128);
            }
            if (uin < U) {
                ++uin;
                if (++sti == nst) {
                    sti = 0;
                    ++ki;
                }
            }
        };
        int stw = 0, uw = 0;  // weight cursor
        auto issue_w = [&](int u) {
            char* dst = wring + (u % X1D_NW) * WSLOT;
#pragma unroll
            for (int j = 0; j < NCB; ++j) {
                const int q = pw * NCB + j;                     // 1-KiB piece of the stage
                const int k = q / (2 * NCB), rem = q - k * (2 * NCB);
                x1d_dma16(wg + (size_t)(2 * stw + k) * gstride + rem * 1024 + lane * 16, dst + q * 1024);
            }
            if (uw < U) {
                ++uw;
                if (++stw == nst) stw = 0;
                if (uw == U) stw = (U - 1) % nst;  // past the end: the last stage again
            }
        };
        // Pipeline: before barrier B_u (after which the MFMA waves compute stage u + 1) stage u + 1's input
        // and weights have landed.  Iteration u issues W(u + 2) then I(u + IA) into the slots stage u - 1
        // freed at B_{u-1}; W(u + 1), the newest DMA group B_u depends on, was issued first in iteration
        // u - 1, so at most (4) + (NCB + 4) = VMC DMAs issued after it may still be in flight; I(u + 1) is
        // older.  The prologue I(0) .. I(IA - 3), W(0), I(IA - 2), W(1), I(IA - 1) keeps that shape, so one
        // counted wait fits every barrier (4 input DMAs and NCB weight DMAs per loader wave and stage).
        if (U > 0) {
#pragma unroll
            for (int i = 0; i + 2 < IA; ++i) issue_in(i);
            issue_w(0);
            issue_in(IA - 2);
            issue_w(1);
            issue_in(IA - 1);
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
        barrier();
#ifdef NPS_X3_STAMP  // dev (tools/x1d_stamps.py): loader wave 4's cycles in its vmcnt waits and barriers
        unsigned long long tv = 0, tb = 0;
#endif
        for (int u = 0; u < U; ++u) {
            issue_w(u + 2);
            issue_in(u + IA);
#ifdef NPS_X3_STAMP
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            barrier();
            tv += t1 - t0;
            tb += __builtin_amdgcn_s_memtime() - t1;
#else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
            barrier();
#endif
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the work-group's LDS
#ifdef NPS_X3_STAMP
        {
            const int l = blockIdx.x;
            if (wave == 4 && lane == 0 && l < (1 << 16)) {
                x3_stamps[l * 16 + 5] = tv;
                x3_stamps[l * 16 + 6] = tb;
                x3_stamps[l * 16 + 7] = U;
            }
        }
#endif
        return;
    }

    // ------------------------------------------------------------------ MFMA waves
    const float xs = in_scale_of(a);
    const bool scaled = has_in_scale(a);
    const float inv = 1.f / (pow2_scale_for(a.wpack[packed_body(a.Cout, a.Cin, 1)]) * xs);
    const int h = lane >> 5;
    const int px = 32 * wave + (lane & 31);                      // this lane's tile pixel
    const int sw = (px >> 1) & 7;
    for (int c = tid; c < NCB * 32; c += 256)
        btab[c] = (a.bias != nullptr && c < a.Cout) ? a.bias[c] / inv : 0.f;
    f32x16 acc[NCB];
    float amax = 0.f;
#ifdef NPS_X3_STAMP  // dev (tools/x1d_stamps.py): MFMA wave 0's cycles at barriers and in epilogues
    const int l = blockIdx.x;
    unsigned long long tbar = 0, tepi = 0;
    X3_STAMP(0);
    X3_RSTAMP(8);
#endif
    barrier();  // B_{-1}: stage 0 landed (and the bias table written)
#ifdef NPS_X3_STAMP
    X3_STAMP(1);
#endif
    for (int u = 0; u < U; ++u) {
        const int k = u / nst, st = u - (u / nst) * nst;
        if (st == 0) {  // accumulators start from the scaled bias (lane element r: co 8 (r / 4) + 4 h + r % 4)
#pragma unroll
            for (int i = 0; i < NCB; ++i)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const f32x4 bv = *reinterpret_cast<const f32x4*>(btab + i * 32 + 8 * m + 4 * h);
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[i][4 * m + e] = bv[e];
                }
        }
        const char* ib = iring + (u % NS) * X1D_ISLOT + px * 128;
        const char* wb = wring + (u % X1D_NW) * WSLOT + lane * 16;
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) {
            // K-group kg of the stage: lane half h holds channels 16 h + 8 kg + [0, 8) (the 1x1 packing)
            const int c0 = 4 * h + 2 * kg;
            f32x4 v0 = *reinterpret_cast<const f32x4*>(ib + ((c0 ^ sw) << 4));
            f32x4 v1 = *reinterpret_cast<const f32x4*>(ib + (((c0 + 1) ^ sw) << 4));
            if (scaled) {
                v0 *= xs;
                v1 *= xs;
            }
            // the K-group's weight fragments, all issued before the first MFMA (LDS returns in order: the
            // MFMAs of block cb wait only for its own pair)
            f16x8 Ah[NCB], Al[NCB];
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                Ah[cb] = *reinterpret_cast<const f16x8*>(wb + (kg * NCB + cb) * 2048);
                Al[cb] = *reinterpret_cast<const f16x8*>(wb + (kg * NCB + cb) * 2048 + 1024);
            }
            f16x4 h0, l0, h1, l1;
            split4(v0, h0, l0);
            split4(v1, h1, l1);
            const f16x8 Bh = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
            const f16x8 Bl = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                acc[cb] = X3_MFMA(Ah[cb], Bh, acc[cb], 0, 0, 0);
                acc[cb] = X3_MFMA(Ah[cb], Bl, acc[cb], 0, 0, 0);
                acc[cb] = X3_MFMA(Al[cb], Bh, acc[cb], 0, 0, 0);
            }
        }
#ifdef NPS_X3_STAMP
        const unsigned long long tb0 = __builtin_amdgcn_s_memtime();
        barrier();  // B_u
        const unsigned long long tb1 = __builtin_amdgcn_s_memtime();
        tbar += tb1 - tb0;
#else
        barrier();  // B_u: every read of stage u's slots is done; stage u + 1 has landed
#endif
        if (st == nst - 1) {
            // the tile's epilogue, from the accumulators (the loaders' DMAs for the next stages are in flight).
            // Two passes: every load (bias, addends, accumulate) and the arithmetic first, the stores last —
            // vmcnt counts loads and stores in one in-order queue, so a load behind a store would wait for
            // that store to reach memory.
            const int t = (int)blockIdx.x + k * (int)gridDim.x;
            const int b = t / ptiles, P = (t - b * ptiles) * 128 + px;
            double s1 = 0.0, s2 = 0.0;
            if (P < npx) {
                const int oy = P / a.Wout, ox = P - (P / a.Wout) * a.Wout;
                const int dy = oy * a.out_os + a.out_off_y, dx = ox * a.out_os + a.out_off_x;
                if (dy >= 0 && dy < a.out_H && dx >= 0 && dx < a.out_W) {  // NHWC, 4-aligned (x1_dma_ok)
                    const size_t base = (((size_t)b * a.out_H + dy) * a.out_W + dx) * a.out_C;
                    static_for<NCB>([&](auto cbc) {  // compile-time cb: acc stays in registers
                        constexpr int cb = decltype(cbc)::value;
                        epi_finish(a, base, cb * 32, h, inv, acc[cb], amax, s1, s2);
                        if (cb & 1) __builtin_amdgcn_sched_barrier(0);  // loads hoisted 2 blocks at most
                    });
                    static_for<NCB>([&](auto cbc) {
                        constexpr int cb = decltype(cbc)::value;
                        epi_store(a, base, cb * 32, h, acc[cb]);
                    });
                }
            }
            stats_publish(a, b, s1, s2);
#ifdef NPS_X3_STAMP
            tepi += __builtin_amdgcn_s_memtime() - tb1;
#endif
        }
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
#ifdef NPS_X3_STAMP
    if (wave == 0 && lane == 0 && l < (1 << 16)) {
        x3_stamps[l * 16 + 2] = tbar;
        x3_stamps[l * 16 + 3] = tepi;
    }
    X3_STAMP(4);
    X3_RSTAMP(9);
#endif
}
#endif  // NPS_X1_DMA_KERNEL

template <int NT, int PB, bool PRO = false, bool WIDE = false, bool PST = false>
void launch_x3_one(const nps_conv2d_t& a, unsigned nwg, int lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv2d_x3_kernel<NT, PB, PRO, WIDE, PST>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    conv2d_x3_kernel<NT, PB, PRO, WIDE, PST><<<nwg, 512, lds, s>>>(a);
}

#ifdef NPS_X3F_KERNEL
template <int NT, bool PRO>
void launch_x3f_one(const nps_conv2d_t& a, unsigned nwg, int lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv2d_x3f_kernel<NT, PRO>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    conv2d_x3f_kernel<NT, PRO><<<nwg, 256, lds, s>>>(a);
}
#endif

#ifdef NPS_X1_DMA_KERNEL
template <int NCB>
void launch_x1d(const nps_conv2d_t& a, unsigned grid, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv1x1_dma_kernel<NCB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  x1d_lds_bytes(NCB));
        attr_set = true;
    }
    conv1x1_dma_kernel<NCB><<<grid, 512, x1d_lds_bytes(NCB), s>>>(a);
}
#endif

}  // namespace

// The DMA-stream 1x1 (conv1x1_dma_kernel) can take every split-fp16 1x1 with Cout <= 192 whose sources are
// 4-channel aligned (16-B DMA pieces) and whose output is NHWC with 4-aligned channels.  Opt-in (a dev build
// with -DNPS_X1_DMA_KERNEL, then the knob NPS_X1_DMA=1): measured at par with conv1x1_wl_kernel on the C3 shapes, slower with an addend epilogue
// (profiles/r3/experiments/x1dma_*); both are bound by the epilogue's store issue.
static bool x1_dma_on() {
#ifndef NPS_X1_DMA_KERNEL
    return false;  // the kernel is not in this build
#endif
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("NPS_X1_DMA");
        on = (e != nullptr && e[0] == '1') ? 1 : 0;
    }
    return on == 1;
}
bool x1_dma_ok(const nps_conv2d_t& a) {
    if (!x1_dma_on() || a.KH * a.KW != 1 || a.stride != 1 || a.dil != 1 || a.Cout > 192 || !x3_lds_epilogue(a))
        return false;
    for (int i = 0; i < a.nsrc; ++i)
        if ((a.src[i].C & 3) != 0) return false;
    return true;
}
extern "C" int nps_conv2d_x1_dma(const nps_conv2d_t* a) { return a != nullptr && x1_dma_ok(*a) ? 1 : 0; }

// test hook (nps_x3_set_grid): persistent-grid size override (> 0)
static long g_x3_grid_override = 0;

static bool wl_on() {  // 1x1 convs with Cout <= 192 on the LDS-weight kernel (dev knob NPS_X3_1X1_WL=0: off)
    static int wl = -1;
    if (wl < 0) {
        const char* e = getenv("NPS_X3_1X1_WL");
        wl = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    return wl == 1;
}
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
        NPS_CHECK_ARG(a.spec_z == nullptr || (wl_on() && a.Cout <= 192),
                      "conv2d_fwd (split-fp16 1x1): the fused c2r term needs the LDS-weight kernel");
#ifdef NPS_X1_DMA_KERNEL
        if (x1_dma_ok(a) && a.spec_z == nullptr) {
            const int ncb = (a.Cout + 31) / 32;
            const long ntiles = (((long)a.Hout * a.Wout + 127) / 128) * a.B;
            NPS_CHECK_ARG(ntiles < (1L << 31), "conv2d_fwd: grid too large");
            const unsigned g1 = (unsigned)(ntiles < ncu ? ntiles : ncu);  // persistent: one work-group per CU
            if (ncb <= 2)
                launch_x1d<2>(a, g1, s);
            else if (ncb <= 4)
                launch_x1d<4>(a, g1, s);
            else
                launch_x1d<6>(a, g1, s);
            NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16 1x1, DMA stream)");
            return 0;
        }
#endif
        static int cfg = -1;  // dev knob NPS_X3_1X1_CFG: 0 = (PB 2, D 2), 1 = (1, 4), 2 = (1, 2)
        if (cfg < 0) {
            const char* e = getenv("NPS_X3_1X1_CFG");
            cfg = e != nullptr ? atoi(e) % 3 : 0;
        }
        const int ncob = (a.Cout + 63) / 64;
        const int wl = wl_on() ? 1 : 0;  // dev knob NPS_X3_1X1_WL=0: co-block waves instead of LDS-staged weights
        // out_stats: the LDS-weight kernel's fused register epilogue takes the moments of the values it stores
        // (after the addend and the activation); its store_tile fallback (two addends, accumulate) cannot
        NPS_CHECK_ARG(a.out_stats == nullptr || (wl && a.Cout <= 192 && !a.accumulate && a.addend1 == nullptr && lds_epi),
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
            conv1x1_wl_kernel<6, 2, true><<<dim3((unsigned)nb, a.B), 256, 2 * 2 * 6 * 2048 + 6 * 32 * 4 + 2 * ncp * 4, s>>>(a);
            NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16 1x1, LDS weights, GroupNorm prologue)");
            return 0;
        }
        if (nps_launch_conv1x1_res(a, res_on, s)) return 0;  // resident weights (conv1x1_res.hip)
        if (wl && a.Cout <= 192) {  // (Cout 193..256 measured slower with 8 blocks per wave: co-block waves)
            const long nb = ((long)a.Hout * a.Wout + 127) / 128;
            NPS_CHECK_ARG(nb < (1L << 31) && a.B < 65536, "conv2d_fwd: grid too large");
            static int wd = -1;  // dev knob NPS_X3_WL_D: B-ring depth 2 / 3 / 4 (default 2: measured fastest
            if (wd < 0) {        // on every rollout shape, profiles/r1_conv_shapes_1x1_wl_depth.log)
                const char* e = getenv("NPS_X3_WL_D");
                wd = (e != nullptr && (atoi(e) == 3 || atoi(e) == 4)) ? atoi(e) : 2;
            }
            const dim3 gw((unsigned)nb, a.B);
            if (wd == 2)
                conv1x1_wl_kernel<6, 2><<<gw, 256, 2 * 2 * 6 * 2048 + 6 * 32 * 4, s>>>(a);
            else if (wd == 3)
                conv1x1_wl_kernel<6, 3><<<gw, 256, 2 * 2 * 6 * 2048 + 6 * 32 * 4, s>>>(a);
            else
                conv1x1_wl_kernel<6, 4><<<gw, 256, 2 * 2 * 6 * 2048 + 6 * 32 * 4, s>>>(a);
            NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16 1x1, LDS weights)");
            return 0;
        }
        const int pb1 = cfg >= 1 ? 1 : 2;
        const int waves = ncob < 8 ? ncob : 8;
        const long nblk = ((long)a.Hout * a.Wout + pb1 * 32 - 1) / (pb1 * 32);
        NPS_CHECK_ARG(nblk < (1L << 31) && a.B < 65536, "conv2d_fwd: grid too large");
        const dim3 grid1((unsigned)nblk, a.B, (ncob + 7) / 8);
        const int lds1 = lds_epi ? pb1 * 32 * (64 * waves + 4) * 4 : 0;
        if (cfg == 1)
            conv1x1_x3_kernel<1, 4><<<grid1, 64 * waves, lds1, s>>>(a);
        else if (cfg == 2)
            conv1x1_x3_kernel<1, 2><<<grid1, 64 * waves, lds1, s>>>(a);
        else
            conv1x1_x3_kernel<2, 2><<<grid1, 64 * waves, lds1, s>>>(a);
        NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16 1x1)");
        return 0;
    }
#ifdef NPS_X3F_KERNEL
    static int fused = -1;  // dev build knob NPS_X3_FUSED=1: the fused-role kernel for wide tiles
    if (fused < 0) {
        const char* e = getenv("NPS_X3_FUSED");
        fused = (e != nullptr && e[0] == '1') ? 1 : 0;
    }
    // (the fused kernel's prologue is GroupNorm + GELU or none)
    if (wide && fused && (!pro || (a.gn_stats != nullptr && a.pre_act == 1))) {
        if (a.KH * a.KW == 9)
            pro ? launch_x3f_one<9, true>(a, grid, lds, s) : launch_x3f_one<9, false>(a, grid, lds, s);
        else if (a.KH * a.KW == 4)
            launch_x3f_one<4, false>(a, grid, lds, s);
        else
            NPS_CHECK_ARG(false, "conv2d_fwd (split-fp16): wide tiles are 2x2 / 3x3 only");
        NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16, wide, fused roles)");
        return 0;
    }
#endif
    static int pst = -1;  // dev knob NPS_X3_PSTORE=1: wide tiles stored by the producers during the next tile
    if (pst < 0) {        // instead of the store phase (5 % slower: profiles/r5/experiments/x3_producer_store_ab.txt)
        const char* e = getenv("NPS_X3_PSTORE");
        pst = (e != nullptr && e[0] == '1') ? 1 : 0;
    }
    // (the producer-side store takes at most one epilogue operand: the accumulated output or addend0)
    if (wide && pst && !NPS_X3_SPREAD && !NPS_X3_M16 && a.addend1 == nullptr && !(a.accumulate && a.addend0 != nullptr)) {
        if (a.KH * a.KW == 9)
            pro ? launch_x3_one<9, 2, true, true, true>(a, grid, lds, s)
                : launch_x3_one<9, 2, false, true, true>(a, grid, lds, s);
        else if (a.KH * a.KW == 4)
            launch_x3_one<4, 2, false, true, true>(a, grid, lds, s);
        else
            NPS_CHECK_ARG(false, "conv2d_fwd (split-fp16): wide tiles are 2x2 / 3x3 only");
        NPS_CHECK_LAUNCH("conv2d_fwd (split-fp16, wide, producer-side store)");
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

#ifdef NPS_X3_STAMP
extern "C" int nps_x3_stamps(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(x3_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif

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
        } else if (a.Cout <= 192) {
            // conv1x1_wl_kernel<6, *>: wfetch(min(st + 2, last)) -> chunks 2 last + 1, 6 blocks of the chunk
            top((2 * nst - 1) * gstride + 6 * 2048);
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
