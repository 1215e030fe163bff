// Implicit-GEMM 2-D convolution on fp32 MFMA for gfx950 (MI355X), NHWC activations.
//
// Replaces every nn.Conv2d / nn.ConvTranspose2d forward on the reference's grid
// path (models/common.py:37-47, 93-120; proc_unet_modern.py, proc_dilatedresnet.py,
// proc_fno.py:114-117, enc_grid.py:234-243, dec_grid.py:365-368), see include/nps.h.
//
// GEMM view: D[co][px] = sum_k A[co][k] * B[k][px], k = (chunk of 16 input
// channels, tap).  One workgroup = WAVES wavefronts = 64 output channels x
// 64*WAVES output pixels (a TH x TW pixel tile of one sample); each wave owns
// 64 co x 64 px = 2 x 2 tiles of v_mfma_f32_32x32x2_f32 (exact f32, the only
// f32 matrix path on gfx950).
//   * B (input patch of the tile incl. halo, 16 channels) is staged global ->
//     registers -> LDS once per channel chunk and read by every tap: 9x fewer
//     global reads than im2col for a 3x3 conv.  The prologue (crop_Nd zero
//     fill, channel concat, circular wrap, GroupNorm affine, GELU) is applied
//     while staging, so none of those ever round-trips through HBM.
//   * A (weights) is pre-packed in MFMA-fragment order so every wave load is
//     one contiguous 1 KiB dwordx4 burst straight into VGPRs (L2 resident),
//     prefetched one tap ahead.
//   * Dilated convs tile the output on the dilation lattice ("lattice" mode),
//     so the LDS patch is (TH+KH-1) x (TW+KW-1) instead of growing with d.
//   * Patch double-buffered in LDS; one barrier per 16-channel chunk.

#include "conv2d_common.hpp"

namespace {

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void conv2d_fwd_kernel(const nps_conv2d_t a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NT = WAVES * 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.z, cob = blockIdx.y;
    const Geo g = make_geo(a);
    const int ty = blockIdx.x / g.tiles_x, tx = blockIdx.x % g.tiles_x;
    const int oy0 = (ty % g.T) + (ty / g.T) * a.TH * g.T;
    const int ox0 = (tx % g.T) + (tx / g.T) * a.TW * g.T;
    const int ybase = oy0 * a.stride - a.pad_y, xbase = ox0 * a.stride - a.pad_x;
    const int Hext = a.Hin + 2 * a.circ, Wext = a.Win + 2 * a.circ;
    const int npix = g.PH * g.PW;
    const int NG = npix * (CK / 4);
    const int bufsz = ((npix * PIXS + 3) & ~3);
    float2* gn_tab = reinterpret_cast<float2*>(smem);          // [gn_groups <= 16] (mean, rstd)
    float* pbuf = smem + 32;                                   // 2 patch buffers (128 B header keeps 16-B alignment)
    const int nchunks = (a.Cin + CK - 1) / CK;
    const int ntaps = a.KH * a.KW;
    const int ncb = packed_ncb(a.Cout);

    if (a.gn_stats != nullptr && tid < a.gn_groups) {
        const double cnt = (double)(a.Cin / a.gn_groups) * a.Hin * a.Win;
        const double s = a.gn_stats[(b * a.gn_groups + tid) * 2], ss = a.gn_stats[(b * a.gn_groups + tid) * 2 + 1];
        const double mean = s / cnt;
        double var = ss / cnt - mean * mean;
        var = var < 0.0 ? 0.0 : var;
        gn_tab[tid] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.gn_eps)));
    }
    __syncthreads();
    const int cpg = a.gn_stats ? a.Cin / a.gn_groups : 1;

    // Patch element idx of chunk ch = 4 channels of one patch pixel.  Loading is split from the
    // prologue transform so the global loads of chunk ch+1 stay in flight under chunk ch's MFMAs.
    auto elem_valid = [&](int ch, int idx, int& yv, int& xv, int& c) -> bool {
        const int p = idx >> 2, gq = idx & 3;
        const int pr = p / g.PW, pc = p - pr * g.PW;
        const int ye = ybase + pr * g.rstep, xe = xbase + pc * g.rstep;
        c = ch * CK + gq * 4;
        if (!(ye >= 0 && ye < Hext && xe >= 0 && xe < Wext && c < a.Cin)) return false;
        yv = a.circ ? nps::wrap_mod(ye - a.circ, a.Hin) : ye;
        xv = a.circ ? nps::wrap_mod(xe - a.circ, a.Win) : xe;
        return true;
    };
    auto load_raw = [&](int ch, int idx) -> f32x4 {
        int yv, xv, c;
        if (!elem_valid(ch, idx, yv, xv, c)) return f32x4{0.f, 0.f, 0.f, 0.f};
        return fetch4(a, b, yv, xv, c);
    };
    auto transform = [&](int ch, int idx, f32x4 v) -> f32x4 {
        if (a.gn_stats == nullptr && !a.pre_act) return v;
        int yv, xv, c;
        if (!elem_valid(ch, idx, yv, xv, c)) return v;  // conv zero padding stays 0
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (c + e < a.Cin) {
                float t = v[e];
                if (a.gn_stats != nullptr) {
                    const float2 mr = gn_tab[(c + e) / cpg];
                    t = (t - mr.x) * mr.y * a.gn_gamma[c + e] + a.gn_beta[c + e];
                }
                if (a.pre_act == 1) t = nps::gelu_erf(t);
                v[e] = t;
            }
        }
        return v;
    };
    // register-prefetch staging (patch fits MAXL float4 per thread) or direct staging
    const bool prefetch = NG <= MAXL * NT;
    f32x4 pre[MAXL];
    auto load_patch = [&](int ch) {
#pragma unroll
        for (int k = 0; k < MAXL; ++k) {
            const int idx = tid + k * NT;
            pre[k] = (idx < NG) ? load_raw(ch, idx) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto store_patch = [&](int ch, int buf) {
        float* dst = pbuf + buf * bufsz;
#pragma unroll
        for (int k = 0; k < MAXL; ++k) {
            const int idx = tid + k * NT;
            if (idx < NG) {
                const int p = idx >> 2, gq = idx & 3;
                *reinterpret_cast<f32x4*>(dst + p * PIXS + gq * 4) = transform(ch, idx, pre[k]);
            }
        }
    };
    auto stage_direct = [&](int ch, int buf) {
        float* dst = pbuf + buf * bufsz;
        for (int idx = tid; idx < NG; idx += NT) {
            const int p = idx >> 2, gq = idx & 3;
            *reinterpret_cast<f32x4*>(dst + p * PIXS + gq * 4) = transform(ch, idx, load_raw(ch, idx));
        }
    };

    // per-lane B (patch) base offsets for this wave's two 32-pixel blocks
    int boff[2];
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
        const int P = wave * 64 + pb * 32 + (lane & 31);
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        boff[pb] = ((ti * g.ri) * g.PW + tj * g.ri) * PIXS + (lane >> 5) * 8;
    }

    const f32x4* wp = reinterpret_cast<const f32x4*>(a.wpack);
    auto load_A = [&](f32x4 (&dst)[2][2], int ch, int tap) {
        const size_t base = ((size_t)(ch * ntaps + tap) * ncb + cob * 2) * 2;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int q = 0; q < 2; ++q) dst[cb][q] = wp[(base + cb * 2 + q) * 64 + lane];
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    f32x4 a_cur[2][2], a_nxt[2][2];
    load_A(a_cur, 0, 0);
    if (prefetch) {
        load_patch(0);
        store_patch(0, 0);
    } else {
        stage_direct(0, 0);
    }
    __syncthreads();

    for (int ch = 0; ch < nchunks; ++ch) {
        const bool more = ch + 1 < nchunks;
        if (more && prefetch) load_patch(ch + 1);
        const float* buf = pbuf + (ch & 1) * bufsz;
        for (int tap = 0; tap < ntaps; ++tap) {
            int nch = ch, ntap = tap + 1;
            if (ntap == ntaps) { ntap = 0; nch = ch + 1; }
            if (nch < nchunks) load_A(a_nxt, nch, ntap);
            const int ky = tap / a.KW, kx = tap - (tap / a.KW) * a.KW;
            const int toff = (ky * g.rk * g.PW + kx * g.rk) * PIXS;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                f32x4 bv[2];
#pragma unroll
                for (int pb = 0; pb < 2; ++pb) bv[pb] = *reinterpret_cast<const f32x4*>(buf + boff[pb] + toff + q * 4);
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                        for (int pb = 0; pb < 2; ++pb)
                            acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[cb][q][e], bv[pb][e], acc[cb][pb], 0, 0, 0);
            }
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                for (int q = 0; q < 2; ++q) a_cur[cb][q] = a_nxt[cb][q];
        }
        if (more) {
            if (prefetch)
                store_patch(ch + 1, (ch + 1) & 1);
            else
                stage_direct(ch + 1, (ch + 1) & 1);
        }
        __syncthreads();
    }

    // ---------------- epilogue ----------------
    const int h = lane >> 5;
    float amax = 0.f;
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
        const int P = wave * 64 + pb * 32 + (lane & 31);
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        const int oy = oy0 + ti * g.T, ox = ox0 + tj * g.T;
        if (ti >= a.TH || oy >= a.Hout || ox >= a.Wout) continue;
        const int dy = oy * a.out_os + a.out_off_y, dx = ox * a.out_os + a.out_off_x;
        if (dy < 0 || dy >= a.out_H || dx < 0 || dx >= a.out_W) continue;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) store_tile(a, b, cob * 64 + cb * 32, h, acc[cb][pb], dy, dx, amax);
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}

// ---------------------------------------------------------------------------------------------
// Producer/consumer variant for stride-1, undilated convs with 1, 4 or 9 taps (every U-Net conv,
// the transposed-conv phases, all 1x1s).  512 threads: waves 0-3 are MFMA consumers that only
// read LDS (no global loads, no VALU beyond address math), waves 4-7 are producers that stage
// the next K-stage (weights + input patch with the crop/concat/wrap/GN/GELU prologue) while the
// consumers run the current one.  Producers hold stage s+2's global loads in registers across
// the barrier (raw s_barrier, only lgkmcnt drained) so their HBM/L2 latency overlaps two stages.
// Wave tile = CBW*32 output channels x PB*32 pixels; the 4 consumer waves are WCO (channel) x
// 4/WCO (pixel); a work-group covers WCO*CBW*32 channels x (4/WCO)*PB*32 pixels.
__host__ __device__ constexpr int pc_patch_px_max(int ntaps, int tile_px) {
    return ntaps == 1 ? tile_px : (tile_px == 256 ? (ntaps == 4 ? 297 : 340) : (ntaps == 4 ? 153 : 180));
}

// Exact-fp32 producer/consumer kernel (v_mfma_f32_32x32x2_f32): the 1x1 / 2x2 / 3x3 convs under
// NPS_PREC_F32.
template <int NTAPS, int CKB, int PB, int CBW, int WCO>
__global__ __launch_bounds__(512) void conv2d_pc_kernel(const nps_conv2d_t a) {
    constexpr int KWT = NTAPS == 9 ? 3 : (NTAPS == 4 ? 2 : 1);
    constexpr int SUB = CKB / CK;                       // 16-channel sub-chunks per stage
    constexpr int PIXSB = CKB + 4;                      // LDS floats per patch pixel
    constexpr int NCBG = WCO * CBW;                     // 32-channel output blocks per work-group
    constexpr int WPX = 4 / WCO;
    constexpr int TILE_PX = WPX * PB * 32;
    constexpr int AROW = NCBG * 2 * 64;                 // float4 of A per (sub, tap)
    constexpr int AFL = SUB * NTAPS * AROW * 4;         // floats of the A (weight) tile per stage
    constexpr int NAP = SUB * NTAPS * AROW / 256;       // A float4 per producer thread per stage
    constexpr int MAXP = (pc_patch_px_max(NTAPS, TILE_PX) * (CKB / 4) + 255) / 256;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool producer = wave >= 4;
    const int b = blockIdx.z, cob = blockIdx.y;
    const Geo g = make_geo(a);
    const int ty = blockIdx.x / g.tiles_x, tx = blockIdx.x % g.tiles_x;
    const int oy0 = ty * a.TH, ox0 = tx * a.TW;
    const int ybase = oy0 - a.pad_y, xbase = ox0 - a.pad_x;
    const int Hext = a.Hin + 2 * a.circ, Wext = a.Win + 2 * a.circ;
    const int npix = g.PH * g.PW;
    const int NG = npix * (CKB / 4);
    const int patch_fl = (npix * PIXSB + 3) & ~3;
    const int stage_fl = AFL + patch_fl;
    float* ring = smem + 32;
    const int n16 = (a.Cin + CK - 1) / CK;              // 16-channel chunks of the packed weight
    const int nstages = (n16 + SUB - 1) / SUB;
    const int ncb = packed_ncb(a.Cout);

    if (producer) {
        // ------------------------------------------------------------------ producers
        // Pure data movement (the GroupNorm/GELU prologue is materialised by nps_frame_pack when
        // this kernel is used): on gfx950 f32 MFMA and VALU share the FP32 datapath, so every
        // producer VALU instruction is MFMA time lost.  Slot geometry is computed once.
        const int ptid = tid - 256;
        const f32x4* wp = reinterpret_cast<const f32x4*>(a.wpack);
        f32x4 ra[NAP], rp[MAXP];
        int sy[MAXP], sx[MAXP];  // virtual-frame pixel of each slot (after circular wrap); sy = -1: zero pad
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            const int idx = ptid + k * 256;
            const int p = idx / (CKB / 4);
            const int pr = p / g.PW, pc = p - pr * g.PW;
            const int ye = ybase + pr, xe = xbase + pc;
            const bool ok = idx < NG && ye >= 0 && ye < Hext && xe >= 0 && xe < Wext;
            sy[k] = ok ? (a.circ ? nps::wrap_mod(ye - a.circ, a.Hin) : ye) : -1;
            sx[k] = ok ? (a.circ ? nps::wrap_mod(xe - a.circ, a.Win) : xe) : 0;
        }
        // two register sets: stage s is loaded into set s & 1, two stages ahead of its LDS commit, so
        // every global load has two consumer stages of time to land (more bytes in flight per CU)
        f32x4 ra1[NAP], rp1[MAXP];
        auto issue = [&](int st, f32x4 (&ra)[NAP], f32x4 (&rp)[MAXP]) {  // global loads of stage st
#pragma unroll
            for (int k = 0; k < NAP; ++k) {
                const int e = k * 256 + ptid;
                const int stp = (k * 256) / AROW;                 // (sub, tap) of this float4 (static)
                const int rem = e - stp * AROW;
                const int sub = stp / NTAPS, tap = stp - sub * NTAPS;
                const int ch16 = st * SUB + sub;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (ch16 < n16) v = wp[(((size_t)ch16 * NTAPS + tap) * ncb + cob * NCBG) * 2 * 64 + rem];
                ra[k] = v;
            }
            // source holding this stage's channels (uniform); fast path when one 4-aligned source covers it
            const int c0 = st * CKB;
            const int cend = min(c0 + CKB, a.Cin);
            int sidx = -1, cbase = 0;
            {
                int lo = 0;
#pragma unroll
                for (int si = 0; si < NPS_MAX_SRC; ++si) {  // unrolled: static kernarg indexing
                    if (si < a.nsrc) {
                        const int hi = lo + a.src[si].C;
                        if (c0 >= lo && cend <= hi && (a.src[si].C & 3) == 0 && ((c0 - lo) & 3) == 0) {
                            sidx = si;
                            cbase = lo;
                        }
                        lo = hi;
                    }
                }
            }
            if (sidx >= 0) {
                // scalar selects over per-source locals (an indexed kernarg struct would go to scratch)
                const nps_src_t S0 = a.src[0], S1 = a.src[1], S2 = a.src[2];
                const float* sptr = sidx == 0 ? S0.ptr : (sidx == 1 ? S1.ptr : S2.ptr);
                const int sC = sidx == 0 ? S0.C : (sidx == 1 ? S1.C : S2.C);
                const int sH = sidx == 0 ? S0.H : (sidx == 1 ? S1.H : S2.H);
                const int sW = sidx == 0 ? S0.W : (sidx == 1 ? S1.W : S2.W);
                const int soy = sidx == 0 ? S0.off_y : (sidx == 1 ? S1.off_y : S2.off_y);
                const int sox = sidx == 0 ? S0.off_x : (sidx == 1 ? S1.off_x : S2.off_x);
                const int cs = c0 - cbase;
#pragma unroll
                for (int k = 0; k < MAXP; ++k) {
                    const int idx = ptid + k * 256;
                    const int gq = idx % (CKB / 4);
                    const int yy = sy[k] - soy, xx = sx[k] - sox;
                    f32x4 v = {0.f, 0.f, 0.f, 0.f};
                    if (sy[k] >= 0 && yy >= 0 && yy < sH && xx >= 0 && xx < sW && c0 + gq * 4 < cend)
                        v = *reinterpret_cast<const f32x4*>(sptr + ((size_t)(b * sH + yy) * sW + xx) * sC + cs + gq * 4);
                    rp[k] = v;
                }
            } else {
#pragma unroll
                for (int k = 0; k < MAXP; ++k) {
                    const int idx = ptid + k * 256;
                    const int gq = idx % (CKB / 4);
                    f32x4 v = {0.f, 0.f, 0.f, 0.f};
                    if (sy[k] >= 0 && c0 + gq * 4 < a.Cin) v = fetch4(a, b, sy[k], sx[k], c0 + gq * 4);
                    rp[k] = v;
                }
            }
        };
        auto commit = [&](int buf, const f32x4 (&ra)[NAP], const f32x4 (&rp)[MAXP]) {  // LDS store of a stage
            float* A = ring + buf * stage_fl;
            float* Pt = A + AFL;
#pragma unroll
            for (int k = 0; k < NAP; ++k) *reinterpret_cast<f32x4*>(A + (k * 256 + ptid) * 4) = ra[k];
#pragma unroll
            for (int k = 0; k < MAXP; ++k) {
                const int idx = ptid + k * 256;
                if (idx < NG) {
                    const int p = idx / (CKB / 4), gq = idx - p * (CKB / 4);
                    *reinterpret_cast<f32x4*>(Pt + p * PIXSB + gq * 4) = rp[k];
                }
            }
        };
        issue(0, ra, rp);
        commit(0, ra, rp);
        if (nstages > 1) issue(1, ra1, rp1);
        if (nstages > 2) issue(2, ra, rp);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (int st = 0; st < nstages; ++st) {
            if (st + 1 < nstages) {
                if ((st + 1) & 1) {
                    commit(1, ra1, rp1);
                    if (st + 3 < nstages) issue(st + 3, ra1, rp1);
                } else {
                    commit(0, ra, rp);
                    if (st + 3 < nstages) issue(st + 3, ra, rp);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        return;
    }

    // ---------------------------------------------------------------------- consumers
    const int wco = wave % WCO, wpx = wave / WCO;
    int boff[PB];
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
        const int P = wpx * 32 * PB + pb * 32 + (lane & 31);
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        boff[pb] = (ti * g.PW + tj) * PIXSB + (lane >> 5) * 8;
    }
    f32x16 acc[CBW][PB];
#pragma unroll
    for (int i = 0; i < CBW; ++i)
#pragma unroll
        for (int j = 0; j < PB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // Operands of K-group gi = (sub, tap, q) are read one group ahead into a second register set,
    // so every group's 8*PB MFMAs (>= 512 cycles) cover the LDS latency of the next group's reads.
    constexpr int G = SUB * NTAPS * 2;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int st = 0; st < nstages; ++st) {
        const float* A = ring + (st & 1) * stage_fl;
        const float* Pt = A + AFL;
        f32x4 av[2][CBW], bv[2][PB];
        auto load_group = [&](int gi, f32x4 (&ad)[CBW], f32x4 (&bd)[PB]) {
            const int q = gi & 1, tq = gi >> 1;
            const int sub = tq / NTAPS, tap = tq - sub * NTAPS;
            const int ky = tap / KWT, kx = tap % KWT;
            const int toff = (ky * g.PW + kx) * PIXSB + sub * CK;
#pragma unroll
            for (int cb = 0; cb < CBW; ++cb)
                ad[cb] = *reinterpret_cast<const f32x4*>(
                    A + (((sub * NTAPS + tap) * NCBG + wco * CBW + cb) * 2 + q) * 256 + lane * 4);
#pragma unroll
            for (int pb = 0; pb < PB; ++pb) bd[pb] = *reinterpret_cast<const f32x4*>(Pt + boff[pb] + toff + q * 4);
        };
        load_group(0, av[0], bv[0]);
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
            const int cur = gi & 1;
            if (gi + 1 < G) load_group(gi + 1, av[cur ^ 1], bv[cur ^ 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
                    for (int pb = 0; pb < PB; ++pb)
                        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][cb][e], bv[cur][pb][e], acc[cb][pb], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }

    // epilogue
    const int h = lane >> 5;
    float amax = 0.f;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
        const int P = wpx * 32 * PB + pb * 32 + (lane & 31);
        const int ti = P / a.TW, tj = P - (P / a.TW) * a.TW;
        const int oy = oy0 + ti, ox = ox0 + tj;
        if (oy >= a.Hout || ox >= a.Wout) continue;
        const int dy = oy * a.out_os + a.out_off_y, dx = ox * a.out_os + a.out_off_x;
        if (dy < 0 || dy >= a.out_H || dx < 0 || dx >= a.out_W) continue;
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb) {
            store_tile(a, b, (cob * NCBG + wco * CBW + cb) * 32, h, acc[cb][pb], dy, dx, amax);
            __builtin_amdgcn_sched_barrier(0);  // keep each tile's epilogue loads local (register pressure)
        }
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}

// Weight element (co, ci, tap) of the conv being packed, from w in the layout the mode implies.
__device__ __forceinline__ float weight_elem(const float* __restrict__ w, int Cout, int Cin, int KH, int KW, int tphase,
                                             int co, int ci, int tap) {
    if (co >= Cout || ci >= Cin) return 0.f;
    const int ky = tap / KW, kx = tap % KW;
    if (tphase == -2) {
        // 3x3 / stride-2 conv as a 2x2 conv over the space-to-depth input: channel
        // ci = (dy*2 + dx)*C + c, tap (ky, kx) -> kernel element (2ky + dy, 2kx + dx) of w[Cout][C][3][3]
        const int C = Cin / 4, par = ci / C, c = ci - par * C;
        const int kyy = 2 * ky + (par >> 1), kxx = 2 * kx + (par & 1);
        return (kyy < 3 && kxx < 3) ? w[(((size_t)co * C + c) * 3 + kyy) * 3 + kxx] : 0.f;
    }
    if (tphase == -3)  // input-gradient conv of w[Cin][Cout][KH][KW] (the forward conv's): transposed, flipped
        return w[(((size_t)ci * Cout + co) * KH + (KH - 1 - ky)) * KW + (KW - 1 - kx)];
    if (tphase < 0) return w[(((size_t)co * Cin + ci) * KH + ky) * KW + kx];
    // 4x4 / stride-2 transposed conv, output phase (py, px): tap (ty, tx) uses
    // kernel element (py + 2(1-ty), px + 2(1-tx)) of w[Cin][Cout][4][4]
    const int py = tphase >> 1, px = tphase & 1;
    const int kyy = py + 2 * (1 - ky), kxx = px + 2 * (1 - kx);
    return w[(((size_t)ci * Cout + co) * 4 + kyy) * 4 + kxx];
}

// Packed layout (fp32): [chunk][tap][cb (32-co block, padded to a multiple of 6)][q (2)][lane (64)][4]
// element = w[co = cb*32 + (lane&31)][ci = chunk*16 + (lane>>5)*8 + q*4 + e][tap]
__global__ void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ wp, int Cout, int Cin, int KH,
                                    int KW, int tphase, size_t total) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int ntaps = KH * KW;
    const int ncb = packed_ncb(Cout);
    const int e = i & 3;
    size_t r = i >> 2;
    const int lane = r & 63; r >>= 6;
    const int q = r & 1; r >>= 1;
    const int cb = r % ncb; r /= ncb;
    const int tap = r % ntaps; r /= ntaps;
    const int chunk = (int)r;
    wp[i] = weight_elem(w, Cout, Cin, KH, KW, tphase, cb * 32 + (lane & 31), chunk * CK + (lane >> 5) * 8 + q * 4 + e,
                        tap);
}

// Packed layout (3-pass split fp16, same bytes): [chunk][tap][cb][hl (2)][lane (64)][8 halves]
// element j of lane = (hi | lo) of s * w[co = cb*32 + (lane&31)][ci = chunk*16 + (lane>>5)*8 + j][tap],
// s = pow2_scale_for(max|w|): max|w| from the per-work-group partials nps_absmax_parts left in trailer[1 ..],
// written back to trailer[0] (where the conv kernels read it)
// pair i of one weight's split-fp16 packing, given max|w| = m
__device__ __forceinline__ void pack_x3_pair(const float* __restrict__ w, _Float16* __restrict__ wp, int Cout, int Cin,
                                             int KH, int KW, int tphase, size_t i, float m) {
    const int ntaps = KH * KW;
    const int ncb = packed_ncb(Cout);
    const int j = i & 7;
    size_t r = i >> 3;
    const int lane = r & 63; r >>= 6;
    const int cb = r % ncb; r /= ncb;
    const int tap = r % ntaps; r /= ntaps;
    const int chunk = (int)r;
    // 1x1: chunk pair (2s, 2s + 1) covers channels [32s, 32s + 32) with lane half h holding the contiguous
    // run [32s + 16h, 32s + 16h + 16): chunk 2s its first 8, chunk 2s + 1 its last 8 (conv1x1_x3_kernel
    // fetches 64 contiguous bytes per lane); other tap counts: chunk c = channels [16c, 16c + 16)
    const int ci = ntaps == 1 && (tphase == -1 || tphase == -3) ? (chunk >> 1) * 32 + (lane >> 5) * 16 + (chunk & 1) * 8 + j
                                              : chunk * CK + (lane >> 5) * 8 + j;
    const float v = pow2_scale_for(m) * weight_elem(w, Cout, Cin, KH, KW, tphase, cb * 32 + (lane & 31), ci, tap);
    const size_t frag = i >> 9;  // (chunk, tap, cb) fragment of 64 lanes x 8
    const size_t o = frag * 1024 + (size_t)lane * 8 + j;
    const h2f hv = pkrtz(v, 0.f);
    const h2f lv = pkrtz(v - (float)hv[0], 0.f);
    wp[o] = hv[0];
    wp[o + 512] = lv[0];
}

// max|w| from the absmax partials in trailer[1 .. nparts] (wave 0 reduces them, LDS broadcast)
__device__ __forceinline__ float pack_x3_max(const float* __restrict__ wmax, int nparts) {
    __shared__ float s_max;
    if (threadIdx.x < 64) {
        const float p = (int)threadIdx.x < nparts ? wmax[1 + threadIdx.x] : 0.f;
        const float mw = nps::wave_max(p);
        if (threadIdx.x == 0) s_max = mw;
    }
    __syncthreads();
    return s_max;
}

__global__ void pack_weights_x3_kernel(const float* __restrict__ w, _Float16* __restrict__ wp, int Cout, int Cin,
                                       int KH, int KW, int tphase, size_t total_pairs, float* __restrict__ wmax,
                                       int nparts) {
    const float m = pack_x3_max(wmax, nparts);
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // (hi, lo) pair index
    if (i >= total_pairs) return;
    if (i == 0) wmax[0] = m;  // the first thread of the launch publishes it as trailer[0]
    pack_x3_pair(w, wp, Cout, Cin, KH, KW, tphase, i, m);
}

// ---- batched packing (nps_conv2d_pack_weights_x3_batch): up to PACK_BATCH weights per launch pair, the jobs passed
// by value; work-group b belongs to the job whose block range [start[j], start[j + 1]) holds it (uniform scan)
constexpr int PACK_BATCH = 48;
struct PackBatch {
    nps_pack_job_t job[PACK_BATCH];
    int start[PACK_BATCH + 1];  // prefix sums of the jobs' work-group counts
    int n;
};
__device__ __forceinline__ int batch_job(const PackBatch& pb, int blk) {
    int j = 0;
    while (j + 1 < pb.n && pb.start[j + 1] <= blk) ++j;
    return j;
}
__host__ __device__ inline long pack_job_nw(const nps_pack_job_t& J) {  // weight elements the job reads
    return J.transposed_phase == -1 || J.transposed_phase == -3
               ? (long)J.Cout * J.Cin * J.KH * J.KW
               : (J.transposed_phase == -2 ? (long)J.Cout * (J.Cin / 4) * 9 : (long)J.Cout * J.Cin * 16);
}
__host__ __device__ inline int pack_job_nparts(const nps_pack_job_t& J) {  // = nps_absmax_parts' partial count
    long nb = (pack_job_nw(J) + 1024 * 16 - 1) / (1024 * 16);
    return (int)(nb < 1 ? 1 : (nb > PACK_TRAILER - 1 ? PACK_TRAILER - 1 : nb));
}
// one partial max |w| per work-group of 1024 threads (absmax_parts_kernel's form), into the job's trailer[1 + k]
__global__ __launch_bounds__(1024) void absmax_parts_batch_kernel(const PackBatch pb) {
    const int j = batch_job(pb, blockIdx.x);
    const nps_pack_job_t& J = pb.job[j];
    const int k = blockIdx.x - pb.start[j], nb = pb.start[j + 1] - pb.start[j];
    const long n = pack_job_nw(J);
    const float* x = J.w;
    __shared__ float wm[16];
    float m = 0.f;
    const long t0 = (long)k * blockDim.x + threadIdx.x, step = (long)nb * blockDim.x;
    long tail = 0;
    if ((reinterpret_cast<size_t>(x) & 15) == 0) {
        const long n4 = n >> 2;
        const float4* x4 = reinterpret_cast<const float4*>(x);
        for (long i = t0; i < n4; i += step) {
            const float4 v = x4[i];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
        tail = n4 << 2;
    }
    for (long i = tail + t0; i < n; i += step) m = fmaxf(m, fabsf(x[i]));
    m = nps::wave_max(m);
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x < 64) {
        float v = (int)threadIdx.x < (int)(blockDim.x >> 6) ? wm[threadIdx.x] : 0.f;
        v = nps::wave_max(v);
        if (threadIdx.x == 0)
            J.wpack[packed_body(J.Cout, J.Cin, J.KH * J.KW) + 1 + k] = v;
    }
}
__global__ void pack_weights_x3_batch_kernel(const PackBatch pb) {
    const int j = batch_job(pb, blockIdx.x);
    const nps_pack_job_t& J = pb.job[j];
    const size_t pairs = packed_body(J.Cout, J.Cin, J.KH * J.KW);
    float* wmax = J.wpack + pairs;
    const float m = pack_x3_max(wmax, pack_job_nparts(J));
    const size_t i = (size_t)(blockIdx.x - pb.start[j]) * blockDim.x + threadIdx.x;
    if (i >= pairs) return;
    if (i == 0) wmax[0] = m;
    pack_x3_pair(J.w, reinterpret_cast<_Float16*>(J.wpack), J.Cout, J.Cin, J.KH, J.KW, J.transposed_phase, i, m);
}

size_t packed_size(int Cout, int Cin, int ntaps) { return packed_body(Cout, Cin, ntaps) + PACK_TRAILER; }

bool pc_eligible(const nps_conv2d_t& a) {
    const int nt = a.KH * a.KW;
    // the producer/consumer kernel does no prologue (callers materialise it with nps_frame_pack)
    return a.stride == 1 && a.dil == 1 && a.KH == a.KW && (nt == 1 || nt == 4 || nt == 9) && a.gn_stats == nullptr &&
           a.pre_act == 0;
}

// 3-pass split-fp16 kernel: every stride-1 undilated 1x1 / 2x2 / 3x3 conv and the (dilated) 5x5 convs of
// the dilated ResNet.  A frame prologue (GroupNorm affine and/or GELU) is fused into the 3x3 kernel's
// producers when each 16-B channel quad lies in one group; other prologue convs are fed by nps_frame_pack.
bool x3_eligible(const nps_conv2d_t& a) {
    const int nt = a.KH * a.KW;
    // 1x1 / 2x2 / 3x3 undilated; 5x5 at any dilation (DRN, proc_dilatedresnet.py: tiled on the lattice)
    const bool geo = a.stride == 1 && a.KH == a.KW &&
                     ((a.dil == 1 && (nt == 1 || nt == 4 || nt == 9)) || (nt == 25 && a.dil >= 1));
    if (a.gn_stats == nullptr && a.pre_act == 0) return geo;
    // fused prologue: the 3x3 producers, and the 1x1 LDS-weight kernel (its launcher checks Cout <= 192)
    return geo && (nt == 9 || nt == 1) && (a.pre_act == 0 || a.pre_act == 1) &&
           (a.gn_stats == nullptr || (a.gn_groups > 0 && a.Cin % a.gn_groups == 0 && (a.Cin / a.gn_groups) % 4 == 0));
}


// producer/consumer variant per tap count: 1x1 convs use 192-channel x 128-pixel work-groups
// (the input is streamed once); 2x2 / 3x3 use 64 x 256 (or 64 x 128) so the weight tile of a
// 16-channel stage fits LDS twice
inline int pc_ncbg(int nt) { return nt == 1 ? 6 : 2; }

int pc_lds_bytes(const nps_conv2d_t& a) {
    const Geo g = make_geo(a);
    const int nt = a.KH * a.KW;
    const int ckb = nt == 1 ? 32 : 16;
    const int afl = (ckb / CK) * nt * pc_ncbg(nt) * 2 * 64 * 4;
    const int patch = (g.PH * g.PW * (ckb + 4) + 3) & ~3;
    return (32 + 2 * (afl + patch)) * 4;
}

int lds_bytes(const nps_conv2d_t& a) {
    if (a.waves == 8) return a.precision == NPS_PREC_X3F16 ? x3_lds_bytes(a) : pc_lds_bytes(a);
    const Geo g = make_geo(a);
    const int bufsz = ((g.PH * g.PW * PIXS + 3) & ~3);
    return (32 + 2 * bufsz) * 4;
}

}  // namespace

extern "C" size_t nps_conv2d_packed_size(int Cout, int Cin, int ntaps) { return packed_size(Cout, Cin, ntaps); }

extern "C" int nps_conv2d_pack_weights(const float* w, float* wpack, int Cout, int Cin, int KH, int KW,
                                       int transposed_phase, void* stream) {
    NPS_CHECK_ARG(w && wpack && Cout > 0 && Cin > 0 && KH > 0 && KW > 0, "conv2d_pack_weights: bad args");
    NPS_CHECK_ARG(transposed_phase == -1 || transposed_phase == -3 ||
                      ((transposed_phase == -2 || (transposed_phase >= 0 && transposed_phase < 4)) && KH == 2 &&
                       KW == 2 && (transposed_phase != -2 || Cin % 4 == 0)),
                  "conv2d_pack_weights: phase / space-to-depth packing needs KH=KW=2");
    const size_t total = packed_body(Cout, Cin, KH * KW);
    const int bs = 256;
    pack_weights_kernel<<<(unsigned)((total + bs - 1) / bs), bs, 0, (hipStream_t)stream>>>(w, wpack, Cout, Cin, KH, KW,
                                                                                        transposed_phase, total);
    NPS_CHECK_LAUNCH("conv2d_pack_weights");
    return 0;
}

extern "C" int nps_conv2d_pack_weights_x3(const float* w, float* wpack, int Cout, int Cin, int KH, int KW,
                                          int transposed_phase, void* stream) {
    NPS_CHECK_ARG(w && wpack && Cout > 0 && Cin > 0 && KH > 0 && KW > 0, "conv2d_pack_weights_x3: bad args");
    NPS_CHECK_ARG(transposed_phase == -1 || transposed_phase == -3 ||
                      ((transposed_phase == -2 || (transposed_phase >= 0 && transposed_phase < 4)) && KH == 2 &&
                       KW == 2 && (transposed_phase != -2 || Cin % 4 == 0)),
                  "conv2d_pack_weights_x3: phase / space-to-depth packing needs KH=KW=2");
    const size_t pairs = packed_body(Cout, Cin, KH * KW);  // one (hi, lo) pair per fp32 slot
    float* wmax = wpack + pairs;                             // trailer[0]
    const long nw = transposed_phase == -1 || transposed_phase == -3 ? (long)Cout * Cin * KH * KW
                                           : (transposed_phase == -2 ? (long)Cout * (Cin / 4) * 9 : (long)Cout * Cin * 16);
    const int nparts = nps_absmax_parts(w, nw, wmax + 1, PACK_TRAILER - 1, (hipStream_t)stream);
    if (nparts <= 0) return -2;
    const int bs = 256;
    pack_weights_x3_kernel<<<(unsigned)((pairs + bs - 1) / bs), bs, 0, (hipStream_t)stream>>>(
        w, reinterpret_cast<_Float16*>(wpack), Cout, Cin, KH, KW, transposed_phase, pairs, wmax, nparts);
    NPS_CHECK_LAUNCH("conv2d_pack_weights_x3");
    return 0;
}

extern "C" int nps_conv2d_pack_weights_x3_batch(const nps_pack_job_t* jobs, int n, void* stream) {
    NPS_CHECK_ARG(jobs != nullptr && n >= 0, "conv2d_pack_weights_x3_batch: bad args");
    hipStream_t s = (hipStream_t)stream;
    for (int c0 = 0; c0 < n; c0 += PACK_BATCH) {
        PackBatch pa = {}, pp = {};
        pa.n = pp.n = n - c0 < PACK_BATCH ? n - c0 : PACK_BATCH;
        for (int k = 0; k < pa.n; ++k) {
            const nps_pack_job_t& J = jobs[c0 + k];
            const int tp = J.transposed_phase;
            NPS_CHECK_ARG(J.w && J.wpack && J.Cout > 0 && J.Cin > 0 && J.KH > 0 && J.KW > 0, "conv2d_pack_weights_x3_batch: "
                          "job %d: bad args", c0 + k);
            NPS_CHECK_ARG(tp == -1 || tp == -3 || ((tp == -2 || (tp >= 0 && tp < 4)) && J.KH == 2 && J.KW == 2 &&
                                                   (tp != -2 || J.Cin % 4 == 0)),
                          "conv2d_pack_weights_x3_batch: job %d: phase / space-to-depth packing needs KH=KW=2", c0 + k);
            pa.job[k] = pp.job[k] = J;
            const long pairs = (long)packed_body(J.Cout, J.Cin, J.KH * J.KW);
            pa.start[k + 1] = pa.start[k] + pack_job_nparts(J);
            pp.start[k + 1] = pp.start[k] + (int)((pairs + 255) / 256);
            NPS_CHECK_ARG(pp.start[k + 1] < (1 << 30), "conv2d_pack_weights_x3_batch: too large");
        }
        if (pa.n == 0) break;
        absmax_parts_batch_kernel<<<(unsigned)pa.start[pa.n], 1024, 0, s>>>(pa);
        NPS_CHECK_LAUNCH("conv2d_pack_weights_x3_batch (absmax)");
        pack_weights_x3_batch_kernel<<<(unsigned)pp.start[pp.n], 256, 0, s>>>(pp);
        NPS_CHECK_LAUNCH("conv2d_pack_weights_x3_batch");
    }
    return 0;
}

extern "C" int nps_conv2d_x3_sources_ok(const nps_src_t* src, int nsrc) {
    nps_conv2d_t t = {};
    t.nsrc = nsrc;
    for (int i = 0; i < nsrc && i < NPS_MAX_SRC; ++i) t.src[i] = src[i];
    return nsrc >= 1 && nsrc <= NPS_MAX_SRC && x3_sources_aligned(t) ? 1 : 0;
}

extern "C" int nps_conv2d_x3_prologue_ok(int KH, int KW, int Cin, int gn_groups, int pre_act) {
    nps_conv2d_t t = {};
    t.KH = KH;
    t.KW = KW;
    t.stride = 1;
    t.dil = 1;
    t.Cin = Cin;
    static const double dummy[2] = {0.0, 0.0};
    t.gn_stats = gn_groups > 0 ? dummy : nullptr;
    t.gn_groups = gn_groups;
    t.pre_act = pre_act;
    return x3_eligible(t) ? 1 : 0;
}

extern "C" int nps_conv2d_x3_eligible(int KH, int KW, int stride, int dil) {
    nps_conv2d_t t = {};
    t.KH = KH;
    t.KW = KW;
    t.stride = stride;
    t.dil = dil;
    return x3_eligible(t) ? 1 : 0;
}

extern "C" int nps_conv2d_plan(nps_conv2d_t* a) {
    NPS_CHECK_ARG(a != nullptr, "conv2d_plan: null");
    // dilated stride-1 convs tile on the dilation lattice (patch independent of d)
    a->lattice = (a->dil > 1 && a->stride == 1) ? 1 : 0;
    const long units_co = (a->Cout + 63) / 64;
    if (a->precision == NPS_PREC_X3F16 && x3_eligible(*a)) {
        // split-fp16 kernel: 512-pixel tiles (16x32, 32x16, 8x64) or 256-pixel ones (16x16, 8x32),
        // scored by the useful fraction of the launched pixels x the fill of the last round of
        // work-groups over the 256 CUs; 256-pixel tiles carry a 10 % penalty (half the reuse of
        // each weight fragment per global load)
        // Wide tiles (16x8, 8x16, 4x32 pixels x 192 channels) replace them for 2x2 / 3x3 convs with
        // 128 < Cout <= 192: one staged patch feeds all the output channels (dev knob NPS_X3_WIDE=0: off).
        static int wide_on = -1;
        if (wide_on < 0) {
            const char* e = getenv("NPS_X3_WIDE");
            wide_on = (e != nullptr && e[0] == '0') ? 0 : 1;
        }
        const bool wide = wide_on && x3_wide_eligible(*a);
        // wide candidates in preference order: 16x8 first (same-box A/B at C3: 3x3 class -1.7 % against 8x16,
        // equal FETCH_SIZE; profiles/r2s2/tile_ab)
        const int cand[9][2] = {{16, 32}, {32, 16}, {8, 64}, {16, 16}, {8, 32}, {16, 8}, {8, 16}, {4, 32}, {32, 4}};
        const long units = wide ? (a->Cout + 191) / 192 : units_co;
        static int wide_tile = -2;  // dev knob NPS_X3_WIDE_TILE=0/1/2/3: force 16x8 / 8x16 / 4x32 / 32x4 wide tiles
        if (wide_tile == -2) {
            const char* e = getenv("NPS_X3_WIDE_TILE");
            wide_tile = (e != nullptr && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : -1;
        }
        int best = -1;
        double best_eff = -1.0;
        for (int i = wide ? 5 : 0; i < (wide ? (wide_tile == 3 ? 9 : 8) : 5); ++i) {
            if (wide && wide_tile >= 0 && i != 5 + wide_tile) continue;
            nps_conv2d_t t = *a;
            t.waves = 8;
            t.TH = cand[i][0];
            t.TW = cand[i][1];
            if (x3_lds_bytes(t) > 160 * 1024) continue;
            const Geo g = make_geo(t);
            const long wgs = (long)g.tiles_x * g.tiles_y * a->B * units;
            const double useful = (double)a->Hout * a->Wout * a->B * units / ((double)wgs * t.TH * t.TW);
            const long rounds = (wgs + 255) / 256;
            const double fill = (double)wgs / (double)(rounds * 256);
            const double eff = useful * fill * (t.TH * t.TW == 256 ? 0.9 : 1.0);
            if (eff > best_eff) {
                best_eff = eff;
                best = i;
            }
        }
        a->waves = 8;
        a->TH = cand[best][0];
        a->TW = cand[best][1];
        return x3_lds_bytes(*a);
    }
    if (pc_eligible(*a)) {
        // producer/consumer kernel: 256-pixel tiles (16x16 or 8x32, whichever wastes less of the
        // output edge); 128-pixel 8x16 tiles only when the 256-pixel grid cannot give every CU a
        // work-group (the 8x16 tile does half the MFMAs per LDS byte).
        const int nt = a->KH * a->KW;
        const long units = (a->Cout + pc_ncbg(nt) * 32 - 1) / (pc_ncbg(nt) * 32);
        const int cand[3][2] = {{16, 16}, {8, 32}, {8, 16}};
        int best = -1;
        double best_eff = -1.0;
        long best_wgs = 0;
        for (int i = 0; i < 3; ++i) {
            nps_conv2d_t t = *a;
            t.waves = 8;
            t.TH = cand[i][0];
            t.TW = cand[i][1];
            const bool pb2 = t.TH * t.TW == 256;
            if (nt == 1 && pb2) continue;  // 1x1: 192 x 128 work-groups only
            if (pc_lds_bytes(t) > 160 * 1024) continue;
            const Geo g = make_geo(t);
            const long wgs = (long)g.tiles_x * g.tiles_y * a->B * units;
            if (!pb2 && nt != 1 && best >= 0 && best_wgs >= 256) continue;  // 256-pixel tiles already fill the chip
            const double useful = (double)a->Hout * a->Wout * a->B * units;
            const double eff = useful / ((double)wgs * t.TH * t.TW) * (wgs < 256 ? (double)wgs / 256.0 : 1.0) *
                               (pb2 || nt == 1 ? 1.0 : 0.8);
            if (eff > best_eff) {
                best_eff = eff;
                best = i;
                best_wgs = wgs;
            }
        }
        if (best >= 0) {
            a->waves = 8;
            a->TH = cand[best][0];
            a->TW = cand[best][1];
            return pc_lds_bytes(*a);
        }
    }
    // candidate tiles (waves, TH, TW), largest first: take the first one whose grid
    // puts >= 8 waves on each of the 256 CUs, else the one with the most waves.
    const int cand[5][3] = {{4, 16, 16}, {4, 8, 32}, {2, 8, 16}, {1, 8, 8}, {1, 4, 16}};
    int best = -1;
    long best_waves = -1;
    for (int i = 0; i < 5; ++i) {
        nps_conv2d_t t = *a;
        t.waves = cand[i][0];
        t.TH = cand[i][1];
        t.TW = cand[i][2];
        if (t.stride > 1 && t.TH * t.TW > 128) continue;  // stride-2 patches grow 4x
        if (lds_bytes(t) > 160 * 1024) continue;
        const Geo g = make_geo(t);
        const long waves = (long)g.tiles_x * g.tiles_y * a->B * units_co * t.waves;
        if (waves > best_waves) {
            best_waves = waves;
            best = i;
        }
        if (waves >= 256 * 8) break;
    }
    NPS_CHECK_ARG(best >= 0, "conv2d_plan: no tile fits (KH=%d KW=%d stride=%d dil=%d)", a->KH, a->KW, a->stride,
                  a->dil);
    a->waves = cand[best][0];
    a->TH = cand[best][1];
    a->TW = cand[best][2];
    return lds_bytes(*a);
}

namespace {
template <int NT, int CKB, int PB, int CBW, int WCO>
void launch_pc_one(const nps_conv2d_t& a, dim3 grid, int lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv2d_pc_kernel<NT, CKB, PB, CBW, WCO>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    conv2d_pc_kernel<NT, CKB, PB, CBW, WCO><<<grid, 512, lds, s>>>(a);
}

void launch_pc_taps(const nps_conv2d_t& a, dim3 grid, int lds, hipStream_t s, int nt, bool pb2) {
    if (nt == 9) {
        if (pb2) launch_pc_one<9, 16, 2, 2, 1>(a, grid, lds, s); else launch_pc_one<9, 16, 1, 2, 1>(a, grid, lds, s);
    } else {
        if (pb2) launch_pc_one<4, 16, 2, 2, 1>(a, grid, lds, s); else launch_pc_one<4, 16, 1, 2, 1>(a, grid, lds, s);
    }
}

int launch_pc(const nps_conv2d_t& a, dim3 grid, int lds, hipStream_t s) {
    const int nt = a.KH * a.KW;
    const bool pb2 = a.TH * a.TW == 256;
    grid.y = (a.Cout + pc_ncbg(nt) * 32 - 1) / (pc_ncbg(nt) * 32);
    if (nt == 1)
        launch_pc_one<1, 32, 2, 3, 2>(a, grid, lds, s);
    else
        launch_pc_taps(a, grid, lds, s, nt, pb2);
    NPS_CHECK_LAUNCH("conv2d_fwd (producer/consumer)");
    return 0;
}

}  // namespace

extern "C" int nps_conv2d_fwd(const nps_conv2d_t* ap, void* stream) {
    NPS_CHECK_ARG(ap != nullptr, "conv2d_fwd: null args");
    const nps_conv2d_t& a = *ap;
    NPS_CHECK_ARG(a.nsrc >= 1 && a.nsrc <= NPS_MAX_SRC, "conv2d_fwd: nsrc=%d", a.nsrc);
    int csum = 0;
    for (int s = 0; s < a.nsrc; ++s) {
        NPS_CHECK_ARG(a.src[s].ptr && a.src[s].C > 0 && a.src[s].H > 0 && a.src[s].W > 0, "conv2d_fwd: bad src %d", s);
        csum += a.src[s].C;
    }
    NPS_CHECK_ARG(csum * (a.s2d ? 4 : 1) == a.Cin, "conv2d_fwd: Cin=%d != sum of source channels %d%s", a.Cin, csum,
                  a.s2d ? " x 4 (space-to-depth view)" : "");
    NPS_CHECK_ARG(!a.s2d || (a.precision == NPS_PREC_X3F16 && a.nsrc == 1 && a.KH == 2 && a.KW == 2 && a.stride == 1 &&
                             a.dil == 1 && a.circ == 0 && !a.gn_stats && !a.pre_act && (a.src[0].C & 15) == 0 &&
                             a.src[0].off_y == 0 && a.src[0].off_x == 0 && a.nphase <= 1),
                  "conv2d_fwd: the space-to-depth view is for split-fp16 2x2 convs of one 16-channel-aligned source");
    NPS_CHECK_ARG(a.B > 0 && a.Hout > 0 && a.Wout > 0 && a.Cout > 0 && a.wpack && a.out, "conv2d_fwd: bad shape");
    NPS_CHECK_ARG(a.KH > 0 && a.KW > 0 && a.stride > 0 && a.dil > 0, "conv2d_fwd: bad kernel geometry");
    NPS_CHECK_ARG(!a.gn_stats || (a.gn_groups > 0 && a.gn_groups <= 16 && a.Cin % a.gn_groups == 0 && a.gn_gamma &&
                                  a.gn_beta),
                  "conv2d_fwd: bad GroupNorm prologue");
    NPS_CHECK_ARG(a.circ == 0 || (a.Hin > 0 && a.Win > 0), "conv2d_fwd: circular padding of empty frame");
    NPS_CHECK_ARG(a.spec_z == nullptr ||
                      (a.precision == NPS_PREC_X3F16 && a.KH == 1 && a.KW == 1 && a.stride == 1 && a.Cout <= 192 &&
                       !a.gn_stats && !a.pre_act && !a.accumulate && !a.addend0 && !a.addend1 && !a.out_nchw &&
                       (a.out_C & 3) == 0 && (a.Cout & 3) == 0 && a.spec_m2 > 0 && a.spec_m2 <= 16 &&
                       (a.Wout & 127) == 0 && a.pad_y == 0 && a.pad_x == 0 && a.circ == 0 && a.out_os == 1 &&
                       a.out_off_y == 0 && a.out_off_x == 0 && a.out_H == a.Hout && a.out_W == a.Wout),
                  "conv2d_fwd: the fused c2r term (spec_z) needs a plain split-fp16 1x1 on the LDS-weight kernel "
                  "(Cout <= 192, no prologue / addend / accumulate, Wout %% 128 == 0, m2 <= 16)");
    NPS_CHECK_ARG(a.waves == 1 || a.waves == 2 || a.waves == 4 || a.waves == 8, "conv2d_fwd: call nps_conv2d_plan first");
    NPS_CHECK_ARG(a.precision == NPS_PREC_F32 || x3_sources_aligned(a),
                  "conv2d_fwd: split-fp16 conv needs sources on 16-channel boundaries with C %% 4 == 0 (frame_pack first)");
    NPS_CHECK_ARG(a.precision == NPS_PREC_F32 || (a.precision == NPS_PREC_X3F16 && x3_eligible(a) && a.waves == 8),
                  "conv2d_fwd: precision %d not available for this conv (KH=%d stride=%d dil=%d)", a.precision, a.KH,
                  a.stride, a.dil);
    NPS_CHECK_ARG(a.precision == NPS_PREC_X3F16
                      ? ((a.TH * a.TW == 512 || a.TH * a.TW == 256) && (a.TW == 16 || a.TW == 32 || a.TW == 64)) ||
                            (a.TH * a.TW == 128 && x3_wide_eligible(a) && (a.TW == 4 || a.TW == 8 || a.TW == 16 || a.TW == 32))
                      : (a.waves == 8 ? (a.TH * a.TW == 256 || a.TH * a.TW == 128) && pc_eligible(a) &&
                                            (a.KH * a.KW != 1 || a.TH * a.TW == 128)
                                      : a.TH * a.TW == 64 * a.waves),
                  "conv2d_fwd: tile %dx%d does not match waves=%d", a.TH, a.TW, a.waves);
    NPS_CHECK_ARG(a.out_stats == nullptr || (a.precision == NPS_PREC_X3F16 && (a.KH * a.KW != 1 || a.Cout <= 192) &&
                                             !a.out_nchw && (a.out_C & 3) == 0 && (a.Cout & 3) == 0),
                  "conv2d_fwd: out_stats needs a split-fp16 conv (1x1: Cout <= 192) with an NHWC, 4-aligned output");
    NPS_CHECK_ARG(a.nphase <= 1 || a.precision == NPS_PREC_X3F16,
                  "conv2d_fwd: merged transposed-conv phases (nphase > 1) need the split-fp16 kernel");
    const Geo g = make_geo(a);
    const int lds = lds_bytes(a);
    NPS_CHECK_ARG(lds <= 160 * 1024, "conv2d_fwd: LDS %d B too large", lds);
    dim3 grid((unsigned)(g.tiles_x * g.tiles_y), (unsigned)((a.Cout + 63) / 64), (unsigned)a.B);
    hipStream_t s = (hipStream_t)stream;
    if (a.precision == NPS_PREC_X3F16) return nps_launch_conv2d_x3(a, lds, s);
    if (a.waves == 8) return launch_pc(a, grid, lds, s);
    static bool attr_set = false;  // allow > 64 KiB dynamic LDS (gfx950 has 160 KiB per CU)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv2d_fwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)conv2d_fwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)conv2d_fwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    switch (a.waves) {
        case 4: conv2d_fwd_kernel<4><<<grid, 256, lds, s>>>(a); break;
        case 2: conv2d_fwd_kernel<2><<<grid, 128, lds, s>>>(a); break;
        default: conv2d_fwd_kernel<1><<<grid, 64, lds, s>>>(a); break;
    }
    NPS_CHECK_LAUNCH("conv2d_fwd");
    return 0;
}

// ------------------------------------------------------------------ GroupNorm statistics
namespace {
// One (group, sample) pair per blockIdx.(y,z); the frame is swept as contiguous 16-B runs per source
// with 32-bit index math; per-thread fp32 partials over each float4, fp64 above that.
__device__ __forceinline__ void gn_accum_src(const nps_src_t& S, int lo, int g0, int g1, int b, int Hin, int Win,
                                             double& s, double& ss) {
    const int clo = max(lo, g0), chi = min(lo + S.C, g1);
    if (clo >= chi) return;
    const int nc = chi - clo, lc0 = clo - lo;
    const int y0 = max(0, S.off_y), y1 = min(Hin, S.off_y + S.H);
    const int x0 = max(0, S.off_x), x1 = min(Win, S.off_x + S.W);
    if (y0 >= y1 || x0 >= x1) return;
    const int wi = x1 - x0;
    const int stride = gridDim.x * blockDim.x;
    if (nc == S.C && wi == S.W && (S.C & 3) == 0) {
        // whole rows of the source, all channels: one contiguous run, no index math
        const int n = (y1 - y0) * S.W * (S.C >> 2);
        const f32x4* p = reinterpret_cast<const f32x4*>(S.ptr + ((size_t)(b * S.H + (y0 - S.off_y)) * S.W) * S.C);
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            const f32x4 v = p[i];
            s += (double)((v[0] + v[1]) + (v[2] + v[3]));
            ss += (double)((v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]));
        }
        return;
    }
    if ((nc & 3) == 0 && (lc0 & 3) == 0 && (S.C & 3) == 0) {
        const int nq = nc >> 2;
        const int n = (y1 - y0) * wi * nq;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            const int pix = i / nq, q = i - pix * nq;
            const int y = pix / wi, x = pix - y * wi;
            const f32x4 v = *reinterpret_cast<const f32x4*>(
                S.ptr + ((size_t)(b * S.H + (y + y0 - S.off_y)) * S.W + (x + x0 - S.off_x)) * S.C + lc0 + q * 4);
            s += (double)((v[0] + v[1]) + (v[2] + v[3]));
            ss += (double)((v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]));
        }
    } else {
        const int n = (y1 - y0) * wi * nc;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            const int pix = i / nc, cc = i - pix * nc;
            const int y = pix / wi, x = pix - y * wi;
            const float v = S.ptr[((size_t)(b * S.H + (y + y0 - S.off_y)) * S.W + (x + x0 - S.off_x)) * S.C + lc0 + cc];
            s += v;
            ss += (double)v * v;
        }
    }
}

__global__ void gn_stats_kernel(nps_conv2d_t a, int G, double* __restrict__ stats) {
    __shared__ double red[16];
    const int b = blockIdx.z, gidx = blockIdx.y;
    const int cpg = a.Cin / G;
    const int g0 = gidx * cpg, g1 = g0 + cpg;
    double s = 0.0, ss = 0.0;
    gn_accum_src(a.src[0], 0, g0, g1, b, a.Hin, a.Win, s, ss);
    if (a.nsrc > 1) gn_accum_src(a.src[1], a.src[0].C, g0, g1, b, a.Hin, a.Win, s, ss);
    if (a.nsrc > 2) gn_accum_src(a.src[2], a.src[0].C + a.src[1].C, g0, g1, b, a.Hin, a.Win, s, ss);
    s = nps::block_sum(s, red);
    ss = nps::block_sum(ss, red);
    if (threadIdx.x == 0) {
        atomicAdd(&stats[(b * G + gidx) * 2], s);
        atomicAdd(&stats[(b * G + gidx) * 2 + 1], ss);
    }
}
}  // namespace

extern "C" int nps_group_norm_stats(const nps_src_t* src, int nsrc, int B, int Hin, int Win, int Cin, int G,
                                    double* stats, int zero_first, void* stream) {
    NPS_CHECK_ARG(src && nsrc >= 1 && nsrc <= NPS_MAX_SRC && stats && B > 0 && G > 0 && Cin % G == 0,
                  "group_norm_stats: bad args");
    nps_conv2d_t a = {};
    a.nsrc = nsrc;
    int csum = 0;
    for (int i = 0; i < nsrc; ++i) {
        a.src[i] = src[i];
        csum += src[i].C;
    }
    NPS_CHECK_ARG(csum == Cin, "group_norm_stats: Cin mismatch");
    a.B = B;
    a.Hin = Hin;
    a.Win = Win;
    a.Cin = Cin;
    hipStream_t s = (hipStream_t)stream;
    if (zero_first) {
        if (hipMemsetAsync(stats, 0, sizeof(double) * 2 * B * G, s) != hipSuccess) {
            nps::set_error("group_norm_stats: memset failed");
            return -2;
        }
    }
    // few blocks per (group, sample): each adds its fp64 partials with 2 atomics to one word, so
    // the block count bounds the same-address atomic serialisation
    const long per = (long)Hin * Win * (Cin / G) / 4;
    int nblk = (int)((per + 256 * 32 - 1) / (256 * 32));
    nblk = nblk < 1 ? 1 : (nblk > 96 ? 96 : nblk);
    gn_stats_kernel<<<dim3(nblk, G, B), 256, 0, s>>>(a, G, stats);
    NPS_CHECK_LAUNCH("group_norm_stats");
    return 0;
}

namespace {
__global__ void stats_sum_kernel(const double* __restrict__ p0, int n0, const double* __restrict__ p1, int n1,
                                 const double* __restrict__ p2, int n2, int B, double* __restrict__ out, int n_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * B) return;
    const int b = i >> 1, k = i & 1;
    double s = 0.0;
    for (int j = 0; j < n0; ++j) s += p0[(b * n0 + j) * 2 + k];
    if (p1)
        for (int j = 0; j < n1; ++j) s += p1[(b * n1 + j) * 2 + k];
    if (p2)
        for (int j = 0; j < n2; ++j) s += p2[(b * n2 + j) * 2 + k];
    out[b * n_out * 2 + k] = s;
}
}  // namespace

extern "C" int nps_stats_sub(void) { return NPS_STATS_SUB; }

extern "C" int nps_stats_sum(const double* p0, int n0, const double* p1, int n1, const double* p2, int n2, int B,
                             double* out, int n_out, void* stream) {
    NPS_CHECK_ARG(p0 && out && B > 0 && n0 > 0 && (!p1 || n1 > 0) && (!p2 || n2 > 0) && n_out > 0,
                  "stats_sum: bad args");
    stats_sum_kernel<<<(2 * B + 255) / 256, 256, 0, (hipStream_t)stream>>>(p0, n0, p1, n1, p2, n2, B, out, n_out);
    NPS_CHECK_LAUNCH("stats_sum");
    return 0;
}

// ------------------------------------------------------------------ frame materialisation
namespace {
// out[B][Hin][Win][Cin] = act(GN(frame)) of the virtual frame (or the plain concat/crop when no
// prologue): one pass, 16-B loads/stores, GELU evaluated once per element instead of once per
// consuming conv tile.
__device__ __forceinline__ f32x4 prologue4(const nps_conv2d_t& a, const float2* tab, int cpg, int c, f32x4 v) {
    if (a.gn_stats != nullptr) {
        if ((cpg & 3) == 0 && c + 4 <= a.Cin && (a.Cin & 3) == 0) {
            const float2 mr = tab[c / cpg];
            const f32x4 ga = *reinterpret_cast<const f32x4*>(a.gn_gamma + c);
            const f32x4 be = *reinterpret_cast<const f32x4*>(a.gn_beta + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (v[e] - mr.x) * mr.y * ga[e] + be[e];
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (c + e < a.Cin) {
                    const float2 mr = tab[(c + e) / cpg];
                    v[e] = (v[e] - mr.x) * mr.y * a.gn_gamma[c + e] + a.gn_beta[c + e];
                }
            }
        }
    }
    if (a.pre_act == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = nps::gelu_erf(v[e]);
    }
    return v;
}

__global__ void frame_pack_kernel(nps_conv2d_t a, float* __restrict__ out) {
    __shared__ float2 tab[16];
    const int b = blockIdx.y;
    if (a.gn_stats != nullptr && threadIdx.x < a.gn_groups) {
        const double cnt = (double)(a.Cin / a.gn_groups) * a.Hin * a.Win;
        const double s1 = a.gn_stats[(b * a.gn_groups + threadIdx.x) * 2];
        const double s2 = a.gn_stats[(b * a.gn_groups + threadIdx.x) * 2 + 1];
        const double mean = s1 / cnt;
        double var = s2 / cnt - mean * mean;
        var = var < 0.0 ? 0.0 : var;
        tab[threadIdx.x] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.gn_eps)));
    }
    __syncthreads();
    const int cpg = a.gn_stats ? a.Cin / a.gn_groups : 1;
    const int stride = gridDim.x * blockDim.x;
    const nps_src_t S0 = a.src[0];
    if (a.nsrc == 1 && S0.off_y == 0 && S0.off_x == 0 && S0.H == a.Hin && S0.W == a.Win && (a.Cin & 3) == 0 &&
        a.out_C <= a.Cin) {
        // one source covering the frame: a flat contiguous sweep
        const int C4 = a.Cin >> 2;
        const int n = a.Hin * a.Win * C4;
        const f32x4* src = reinterpret_cast<const f32x4*>(S0.ptr + (size_t)b * a.Hin * a.Win * a.Cin);
        f32x4* dst = reinterpret_cast<f32x4*>(out + (size_t)b * a.Hin * a.Win * a.Cin);
        float amax = 0.f;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            const int c = (i % C4) * 4;
            const f32x4 r = prologue4(a, tab, cpg, c, src[i]);
            dst[i] = r;
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(r[0]), fabsf(r[1])), fmaxf(fabsf(r[2]), fabsf(r[3]))));
        }
        nps::tag_publish(a.out_tag, amax, nps::wave_salt());
        return;
    }
    // output channel stride oC >= Cin (a.out_C; channels [Cin, oC) are written as zeros)
    const int oC = a.out_C > a.Cin ? a.out_C : a.Cin;
    const int C4 = (oC + 3) / 4;
    const int n = a.Hin * a.Win * C4;
    const nps_src_t S1 = a.src[1], S2 = a.src[2];
    if ((oC & 3) == 0 && (S0.C & 3) == 0 && (a.nsrc < 2 || (S1.C & 3) == 0) && (a.nsrc < 3 || (S2.C & 3) == 0)) {
        // 4-aligned sources (the concatenations of the U-Net blocks): every channel quad lies in one
        // source, so its address is a select, not a branch; U quads per thread are fetched before any is
        // used (the branchy per-quad gather leaves one 16-B load in flight per thread)
        constexpr int U = 4;
        const int lo1 = S0.C, lo2 = S0.C + (a.nsrc > 1 ? S1.C : 0);
        float amax = 0.f;
        for (int i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * U) {
            f32x4 v[U];
            int cq[U], pq[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + u * stride;
                const int ii = i < n ? i : 0;
                const int pix = ii / C4;
                const int c = (ii - pix * C4) * 4;
                const int y = pix / a.Win, x = pix - (pix / a.Win) * a.Win;
                const int si = c < lo1 ? 0 : (c < lo2 ? 1 : 2);
                const float* sp = si == 0 ? S0.ptr : (si == 1 ? S1.ptr : S2.ptr);
                const int sC = si == 0 ? S0.C : (si == 1 ? S1.C : S2.C);
                const int sH = si == 0 ? S0.H : (si == 1 ? S1.H : S2.H);
                const int sW = si == 0 ? S0.W : (si == 1 ? S1.W : S2.W);
                const int yy = y - (si == 0 ? S0.off_y : (si == 1 ? S1.off_y : S2.off_y));
                const int xx = x - (si == 0 ? S0.off_x : (si == 1 ? S1.off_x : S2.off_x));
                const int slo = si == 0 ? 0 : (si == 1 ? lo1 : lo2);
                const bool ok = i < n && c < a.Cin && yy >= 0 && yy < sH && xx >= 0 && xx < sW;
                const float* src = ok ? sp + ((size_t)(b * sH + yy) * sW + xx) * sC + (c - slo) : S0.ptr;
                v[u] = *reinterpret_cast<const f32x4*>(src);
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                v[u] = ok ? v[u] : z;
                cq[u] = c;
                pq[u] = i < n ? pix : -1;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (pq[u] < 0) continue;
                f32x4 r = v[u];
                if (cq[u] < a.Cin) r = prologue4(a, tab, cpg, cq[u], r);  // zero padding is normalised too
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (cq[u] + e >= a.Cin) r[e] = 0.f;
                    amax = fmaxf(amax, fabsf(r[e]));
                }
                *reinterpret_cast<f32x4*>(out + ((size_t)b * a.Hin * a.Win + pq[u]) * oC + cq[u]) = r;
            }
        }
        nps::tag_publish(a.out_tag, amax, nps::wave_salt());
        return;
    }
    float amax = 0.f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int pix = i / C4;
        const int c = (i - pix * C4) * 4;
        const int y = pix / a.Win, x = pix - y * a.Win;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (c < a.Cin) v = prologue4(a, tab, cpg, c, fetch4(a, b, y, x, c));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (c + e >= a.Cin) v[e] = 0.f;
            amax = fmaxf(amax, fabsf(v[e]));
        }
        float* dst = out + ((size_t)(b * a.Hin + y) * a.Win + x) * oC + c;
        if ((oC & 3) == 0) {
            *reinterpret_cast<f32x4*>(dst) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (c + e < oC) dst[e] = v[e];
        }
    }
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}
}  // namespace

extern "C" int nps_frame_pack(const nps_conv2d_t* ap, float* out, void* stream) {
    NPS_CHECK_ARG(ap && out, "frame_pack: null");
    const nps_conv2d_t& a = *ap;
    NPS_CHECK_ARG(a.nsrc >= 1 && a.nsrc <= NPS_MAX_SRC && a.B > 0 && a.Hin > 0 && a.Win > 0 && a.Cin > 0,
                  "frame_pack: bad frame");
    int csum = 0;
    for (int i = 0; i < a.nsrc; ++i) csum += a.src[i].C;
    NPS_CHECK_ARG(csum == a.Cin, "frame_pack: Cin mismatch");
    NPS_CHECK_ARG(!a.gn_stats || (a.gn_groups > 0 && a.gn_groups <= 16 && a.Cin % a.gn_groups == 0),
                  "frame_pack: bad GroupNorm");
    NPS_CHECK_ARG(a.out_C <= a.Cin || a.out_C < a.Cin + 4, "frame_pack: out_C pads at most 3 channels");
    const long n = (long)a.Hin * a.Win * (((a.out_C > a.Cin ? a.out_C : a.Cin) + 3) / 4);
    int nb = (int)((n + 255) / 256);
    nb = nb > 2048 ? 2048 : nb;
    frame_pack_kernel<<<dim3(nb, a.B), 256, 0, (hipStream_t)stream>>>(a, out);
    NPS_CHECK_LAUNCH("frame_pack");
    return 0;
}

// ------------------------------------------------------------------ absmax (input range of split-fp16 convs)
namespace {
__global__ void absmax_kernel(const float* __restrict__ x, long n, float* __restrict__ tag) {
    float m = 0.f;
    const long n4 = ((reinterpret_cast<size_t>(x) & 15) == 0) ? n >> 2 : 0;  // 16-B loads when aligned
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
    nps::tag_publish(tag, m, nps::wave_salt());
}

// plain scalar max|x| into *out (one float; the packed-weight trailer): single-address atomics, used once
// per parameter version
// one partial max|x| per work-group (no atomics, no zero-fill): parts[blockIdx.x]
// (1024 threads, 16-B loads when x is 16-B aligned: at most 63 work-groups must cover a whole weight)
__global__ __launch_bounds__(1024) void absmax_parts_kernel(const float* __restrict__ x, long n,
                                                            float* __restrict__ parts) {
    __shared__ float wm[16];
    float m = 0.f;
    const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x, step = (long)gridDim.x * blockDim.x;
    long tail = 0;
    if ((reinterpret_cast<size_t>(x) & 15) == 0) {
        const long n4 = n >> 2;
        const float4* x4 = reinterpret_cast<const float4*>(x);
        for (long i = t0; i < n4; i += step) {
            const float4 v = x4[i];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
        tail = n4 << 2;
    }
    for (long i = tail + t0; i < n; i += step) m = fmaxf(m, fabsf(x[i]));
    m = nps::wave_max(m);
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x < 64) {
        float v = (int)threadIdx.x < (int)(blockDim.x >> 6) ? wm[threadIdx.x] : 0.f;
        v = nps::wave_max(v);
        if (threadIdx.x == 0) parts[blockIdx.x] = v;
    }
}
}  // namespace

int nps_absmax_parts(const float* x, long n, float* parts, int max_parts, hipStream_t s) {
    long nb = (n + 1024 * 16 - 1) / (1024 * 16);
    nb = nb < 1 ? 1 : (nb > max_parts ? max_parts : nb);
    absmax_parts_kernel<<<(unsigned)nb, 1024, 0, s>>>(x, n, parts);
    NPS_CHECK_LAUNCH("absmax (partials)");
    return (int)nb;
}
namespace {
}  // namespace

extern "C" int nps_absmax(const float* x, long n, float* out, void* stream) {
    NPS_CHECK_ARG(x && out && n > 0, "absmax: bad args");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(out, 0, sizeof(float) * NPS_TAG_FLOATS, s) != hipSuccess) {
        nps::set_error("absmax: memset failed");
        return -2;
    }
    return nps_absmax_into(x, n, out, stream);
}

extern "C" int nps_absmax_into(const float* x, long n, float* out, void* stream) {
    NPS_CHECK_ARG(x && out && n > 0, "absmax: bad args");
    hipStream_t s = (hipStream_t)stream;
    long nb = (n + 256 * 16 - 1) / (256 * 16);
    nb = nb < 1 ? 1 : (nb > 1024 ? 1024 : nb);
    absmax_kernel<<<(unsigned)nb, 256, 0, s>>>(x, n, out);
    NPS_CHECK_LAUNCH("absmax");
    return 0;
}

// ------------------------------------------------------------------ space-to-depth
namespace {
__global__ void space_to_depth_kernel(const float* __restrict__ x, float* __restrict__ out, int H, int W, int C, int pad,
                                      int Hq, int Wq) {
    const int b = blockIdx.y;
    if ((C & 3) == 0) {
        const int C4 = (4 * C) / 4;  // float4 groups of the 4C output channels
        const int n = Hq * Wq * C4;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            const int pix = i / C4, g = i - pix * C4;
            const int yq = pix / Wq, xq = pix - yq * Wq;
            const int cc = g * 4, par = cc / C, c = cc - par * C;
            const int y = 2 * yq + (par >> 1) - pad, xx = 2 * xq + (par & 1) - pad;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (y >= 0 && y < H && xx >= 0 && xx < W)
                v = *reinterpret_cast<const f32x4*>(x + ((size_t)(b * H + y) * W + xx) * C + c);
            *reinterpret_cast<f32x4*>(out + ((size_t)b * Hq * Wq + pix) * 4 * C + cc) = v;
        }
        return;
    }
    const int n = Hq * Wq * 4 * C;  // channel counts that are not a multiple of 4: one float per thread
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int pix = i / (4 * C), cc = i - pix * 4 * C;
        const int yq = pix / Wq, xq = pix - yq * Wq;
        const int par = cc / C, c = cc - par * C;
        const int y = 2 * yq + (par >> 1) - pad, xx = 2 * xq + (par & 1) - pad;
        out[(size_t)b * Hq * Wq * 4 * C + i] =
            (y >= 0 && y < H && xx >= 0 && xx < W) ? x[((size_t)(b * H + y) * W + xx) * C + c] : 0.f;
    }
}
}  // namespace

extern "C" int nps_space_to_depth(const float* x, float* out, int B, int H, int W, int C, int pad, int Hq, int Wq,
                                  void* stream) {
    NPS_CHECK_ARG(x && out && B > 0 && H > 0 && W > 0 && C > 0 && Hq > 0 && Wq > 0, "space_to_depth: bad args");
    const long n = (long)Hq * Wq * C * ((C & 3) ? 4 : 1);
    int nb = (int)((n + 255) / 256);
    nb = nb > 2048 ? 2048 : nb;
    space_to_depth_kernel<<<dim3(nb, B), 256, 0, (hipStream_t)stream>>>(x, out, H, W, C, pad, Hq, Wq);
    NPS_CHECK_LAUNCH("space_to_depth");
    return 0;
}
