// Split-fp16 1x1 convolution with RESIDENT weights for gfx950 (MI355X): the NPS_PREC_X3F16 arithmetic of
// nps_conv2d_fwd (include/nps.h) for the pointwise convs of the reference's grid path — the FNO layer's `w`
// (proc_fno.py:142-146), the U-Net ResidualBlock shortcuts and final 1x1s (proc_unet_modern.py), the encoder and
// decoder 1x1s (enc_grid.py, dec_grid.py:126-130).
//
// conv1x1_wl_kernel (conv2d_x3.hip) re-stages every 32-channel stage's weights through LDS once per 128-pixel
// work-group behind a barrier per stage and keeps one stage of input in flight per wave: at ~3 TB/s its waves
// wait on HBM latency at every stage.  Here a persistent work-group (one per CU, 8 waves) loads its output-channel
// group's whole split-fp16 weight into LDS once — NCB 32-channel blocks x every non-empty 16-channel chunk,
// <= 160 KiB — and then has NO barrier: each wave walks its own contiguous range of 32-pixel blocks, streams its
// pixels' input through a D-deep register ring that runs across block boundaries (D - 1 stages of 32 channels in
// flight per wave, 8 waves per CU), and stores each block from the accumulators with the fused epilogue of
// conv1x1_wl_kernel (bias from LDS, one addend, GELU, GroupNorm moments, range tag).  Waves drift apart, so one
// wave's epilogue stores overlap the other waves' loads and MFMAs.
//   * ng = 1, NCB = 6: Cout <= 192 and Cin <= 208 (13 chunks x 12 KiB).
//   * ng = 2: the output channels split over two work-groups of one XCD (consecutive ranks on XCD blockIdx % 8)
//     that walk the SAME pixel blocks, so the second reads the input from that XCD's L2: NCB = 3 for Cout <= 192,
//     Cin <= 416 (the U-Net's 388-channel shortcut); NCB = 4 for 192 < Cout <= 256, Cin <= 304 (the decoder's 225).
//   * The last stage's second chunk stays out of LDS when it holds no input channel.
//   * Stage, chunk and fragment math is conv1x1_wl_kernel's (the ntaps == 1 packing of pack_weights_x3_kernel), and
//     the epilogue keeps store_tile's float order, so both kernels give bit-identical outputs.
#include "conv2d_common.hpp"

#include <cstdlib>
#include <type_traits>

namespace {

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (N > 0) {
        static_for<N - 1>(f);
        f(std::integral_constant<int, N - 1>{});
    }
}

// 64 zero bytes: the load address of input / addend elements outside the frame, so loads are unconditional
__device__ __attribute__((aligned(64))) float x1r_zero[16];
// store target of quads past Cout or outside the output (never read): offsets up to 256 channels
__device__ __attribute__((aligned(64))) float x1r_sink[512];

// LDS bytes: nres resident chunks x NCB blocks x 2 KiB + the bias table
__host__ __device__ constexpr int x1r_lds_bytes(int ncb, int nres) { return nres * ncb * 2048 + ncb * 32 * 4; }
// resident chunks of Cin channels: 2 per 32-channel stage, the last stage's second chunk dropped when every channel
// it would carry (32 (nst - 1) + 16 h + 8 + [0, 8), h = 0, 1) is >= Cin
__host__ __device__ constexpr int x1r_nres(int Cin) {
    return 2 * ((Cin + 31) / 32) - ((32 * ((Cin + 31) / 32 - 1) + 8 >= Cin) ? 1 : 0);
}

template <int NCB, int D>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void conv1x1_res_kernel(
    const nps_conv2d_t a, int ng, int nres) {
    extern __shared__ __attribute__((aligned(16))) char wres[];  // [nres][NCB][hi | lo][64][16 B], bias[NCB * 32]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    const int xcd = blockIdx.x & 7, rank = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
    const int grp = rank % ng, team = rank / ng, nteam = per_xcd / ng;
    const int co_lo = grp * NCB * 32;
    {  // this group's weight blocks of every resident chunk -> LDS
        const size_t gstride = (size_t)packed_ncb(a.Cout) * 2048;
        const char* wg = reinterpret_cast<const char*>(a.wpack) + (size_t)(co_lo / 32) * 2048;
        const int n16 = nres * NCB * 128;  // 16-B pieces
        for (int i = tid; i < n16; i += 512) {
            const int c = i / (NCB * 128), r = i - c * (NCB * 128);
            *reinterpret_cast<f32x4*>(wres + (size_t)i * 16) =
                *reinterpret_cast<const f32x4*>(wg + (size_t)c * gstride + (size_t)r * 16);
        }
        float* bt = reinterpret_cast<float*>(wres + (size_t)nres * NCB * 2048);
        if (tid < NCB * 32) bt[tid] = (a.bias != nullptr && co_lo + tid < a.Cout) ? a.bias[co_lo + tid] : 0.f;
    }
    __syncthreads();  // the only barrier
    const float* btab = reinterpret_cast<const float*>(wres + (size_t)nres * NCB * 2048) + 4 * h;
    const int npx = a.Hout * a.Wout;
    const int bpi = (npx + 31) / 32;  // 32-pixel blocks per sample
    const int NB = a.B * bpi;
    // Block order: grid-stride — wave wid takes blocks wid, wid + nwv, ... — so the waves in flight stream one
    // contiguous window of the tensor (DRAM locality).  Measured against a contiguous range per wave and against
    // per-sample windows (profiles/r5/experiments/x1_resident_weights_ab.txt): this order was the fastest.
    const int nwv = nteam * 64;
    const int wid = (team * 8 + xcd) * 8 + wave;  // the ng groups of a team share it: the same pixel blocks
    const int nblk = wid < NB ? (NB - 1 - wid) / nwv + 1 : 0;
    const int nst = (a.Cin + 2 * CK - 1) / (2 * CK);
    const bool half_last = (nres & 1) != 0;  // the last stage has one resident chunk
    const int nitem = nblk * nst;
    const float xs = in_scale_of(a);
    const bool scaled = has_in_scale(a);
    const float inv = 1.f / (pow2_scale_for(a.wpack[packed_body(a.Cout, a.Cin, 1)]) * xs);

    // ---- input stream: item i = (block wid + (i / nst) nwv, stage i % nst); the pixel's frame coordinates are
    // computed once per issued block
    int iss_j = wid - nwv, iss_b = 0, iss_fy = 0, iss_fx = 0, iss_st = 0;
    bool iss_first = true;
    bool iss_pin = false;
    auto issue = [&](int i, f32x4 (&r)[4]) __attribute__((always_inline)) {
        const bool live = i < nitem;
        int st = iss_st + 1;
        if (st == nst || iss_first) {  // uniform: the next block (items are issued in order)
            st = 0;
            iss_first = false;
            iss_j += nwv;
            iss_b = iss_j / bpi;
            const int p = (iss_j - iss_b * bpi) * 32 + (lane & 31);
            const int oy = p / a.Wout, ox = p - (p / a.Wout) * a.Wout;
            const int ye = oy - a.pad_y, xe = ox - a.pad_x;
            iss_pin = p < npx && ye >= 0 && ye < a.Hin + 2 * a.circ && xe >= 0 && xe < a.Win + 2 * a.circ;
            iss_fy = a.circ ? nps::wrap_mod(ye - a.circ, a.Hin) : ye;
            iss_fx = a.circ ? nps::wrap_mod(xe - a.circ, a.Win) : xe;
        }
        iss_st = st;
        const int c0 = st * 2 * CK + h * CK;
        int sidx = 0, lo = 0, sb = 0;
#pragma unroll
        for (int si = 0; si < NPS_MAX_SRC; ++si) {
            if (si < a.nsrc) {
                const int hi = lo + a.src[si].C;
                if (c0 >= lo && c0 < hi) {  // (sources lie on 16-channel boundaries: host-checked)
                    sidx = si;
                    sb = lo;
                }
                lo = hi;
            }
        }
        const nps_src_t S0 = a.src[0], S1 = a.src[1], S2 = a.src[2];
        const float* sptr = sidx == 0 ? S0.ptr : (sidx == 1 ? S1.ptr : S2.ptr);
        const int sC = sidx == 0 ? S0.C : (sidx == 1 ? S1.C : S2.C);
        const int sH = sidx == 0 ? S0.H : (sidx == 1 ? S1.H : S2.H);
        const int sW = sidx == 0 ? S0.W : (sidx == 1 ? S1.W : S2.W);
        const int yy = iss_fy - (sidx == 0 ? S0.off_y : (sidx == 1 ? S1.off_y : S2.off_y));
        const int xx = iss_fx - (sidx == 0 ? S0.off_x : (sidx == 1 ? S1.off_x : S2.off_x));
        const bool ok = live && iss_pin && yy >= 0 && yy < sH && xx >= 0 && xx < sW;
        const float* sp = ok ? sptr + ((size_t)(iss_b * sH + yy) * sW + xx) * sC + (c0 - sb) : x1r_zero;
        const int cl = a.Cin - c0;  // channels of this lane's 16 inside Cin
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const f32x4*>((ok && q * 4 < cl) ? sp + q * 4 : x1r_zero);
    };

    f32x16 acc[NCB];
#pragma unroll
    for (int i = 0; i < NCB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    f32x4 raw[D][4];
    static_for<D - 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        issue(j, raw[j]);
    });
    float amax = 0.f;
    double s1 = 0.0, s2 = 0.0;
    int stat_b = -1;  // sample whose moments (s1, s2) hold
    const bool vec4 = !a.out_nchw && (a.out_C & 3) == 0 && (a.Cout & 3) == 0;
    const bool add = a.addend0 != nullptr;
    int out_j = wid;  // block of the next epilogue

    // epilogue of block out_j: conv1x1_wl_kernel's fused epilogue (store_tile's float order) per 32-channel block;
    // every address is one per-lane base + a compile-time offset, out-of-range quads go to the sink
    auto epilogue = [&]() __attribute__((always_inline)) {
        const int j = out_j;
        out_j += nwv;
        const int b = j / bpi;
        const int p = (j - b * bpi) * 32 + (lane & 31);
        const int oy = p / a.Wout, ox = p - (p / a.Wout) * a.Wout;
        const int dy = oy * a.out_os + a.out_off_y, dx = ox * a.out_os + a.out_off_x;
        const bool pout = p < npx && dy >= 0 && dy < a.out_H && dx >= 0 && dx < a.out_W;
        // NHWC: channel c of the pixel at base + c; NCHW (the decoder's planar pre-output, dec_grid.py:126-130):
        // at base + c * plane, so for each channel the wave's 32 pixels are one contiguous run
        const size_t plane = (size_t)a.out_H * a.out_W;
        const size_t base = a.out_nchw ? ((size_t)b * a.out_C + co_lo + 4 * h) * plane + (size_t)(pout ? dy : 0) * a.out_W +
                                             (pout ? dx : 0)
                                       : (((size_t)b * a.out_H + (pout ? dy : 0)) * a.out_W + (pout ? dx : 0)) * a.out_C +
                                             co_lo + 4 * h;
        const int cmax = pout ? a.Cout - co_lo - 4 * h : 0;  // quad offset o (within the group) is valid iff o < cmax
        if (a.out_stats != nullptr && b != stat_b) {         // uniform: one publish per sample change
            if (stat_b >= 0) stats_publish(a, stat_b, s1, s2);
            s1 = s2 = 0.0;
            stat_b = b;
        }
        float* const ob = a.out + base;
        const float* const ab = add ? a.addend0 + base : x1r_zero;
        f32x4 a0[4];
        auto load = [&](int cb) {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int o = cb * 32 + 8 * m;
                if (vec4) {
                    a0[m] = *reinterpret_cast<const f32x4*>((add && o < cmax) ? ab + o : x1r_zero);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) a0[m][e] = (add && o + e < cmax) ? ab[o + e] : 0.f;
                }
            }
        };
        load(0);
        static_for<NCB>([&](auto cbc) {
            constexpr int cb = decltype(cbc)::value;
            float f1 = 0.f, f2 = 0.f;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int o = cb * 32 + 8 * m;
                const f32x4 bi = *reinterpret_cast<const f32x4*>(btab + o);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const bool ok = o + e < cmax;
                    float v = acc[cb][4 * m + e] * inv + bi[e];
                    if (!a.add_after_act) v = v + a0[m][e];
                    if (a.act == 1) v = nps::gelu_erf(v);
                    if (a.add_after_act) v = v + a0[m][e];
                    acc[cb][4 * m + e] = v;
                    amax = ok ? fmaxf(amax, fabsf(v)) : amax;
                    f1 += ok ? v : 0.f;
                    f2 += ok ? v * v : 0.f;
                }
            }
            s1 += (double)f1;
            s2 += (double)f2;
            if constexpr (cb + 1 < NCB) {  // the next block's addend before this block's stores (in-order vmcnt)
                __builtin_amdgcn_sched_barrier(0);
                if (add) load(cb + 1);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int o = cb * 32 + 8 * m;
                const f32x4 r = {acc[cb][4 * m], acc[cb][4 * m + 1], acc[cb][4 * m + 2], acc[cb][4 * m + 3]};
                if (a.out_nchw) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (o + e < cmax) ob[(size_t)(o + e) * plane] = r[e];
                } else if (vec4) {
                    *reinterpret_cast<f32x4*>(o < cmax ? ob + o : x1r_sink + o) = r;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (o + e < cmax) ob[o + e] = r[e];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[cb][r] = 0.f;
        });
    };

    const int npad = (nitem + D - 1) / D * D;
    for (int i0 = 0; i0 < npad; i0 += D) {
        static_for<D>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            constexpr int jn = (j + D - 1) % D;
            const int i = i0 + j;
            issue(i + D - 1, raw[jn]);
            __builtin_amdgcn_sched_barrier(0);
            if (i < nitem) {  // uniform
                const int st = i - (i / nst) * nst;
                const char* wb = wres + (size_t)(2 * st) * NCB * 2048 + lane * 16;
                const int nk = (half_last && st == nst - 1) ? 1 : 2;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    if (k < nk) {
                        f16x4 h0, l0, h1, l1;
                        f32x4 v0 = raw[j][2 * k], v1 = raw[j][2 * k + 1];
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
                            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bh, acc[cb], 0, 0, 0);
                            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bl, acc[cb], 0, 0, 0);
                            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Al, Bh, acc[cb], 0, 0, 0);
                        }
                        // the A fragments two co blocks ahead of their MFMAs (not all 2 NCB hoisted: registers)
                        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                        static_for<NCB>([&](auto cc) {
                            constexpr int cb = decltype(cc)::value;
                            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                            if constexpr (cb + 2 < NCB) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                        });
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if (st == nst - 1) epilogue();
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    if (a.out_stats != nullptr && stat_b >= 0) stats_publish(a, stat_b, s1, s2);
    nps::tag_publish(a.out_tag, amax, nps::wave_salt());
}

template <int NCB, int D>
void launch(const nps_conv2d_t& a, unsigned grid, int ng, int nres, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)conv1x1_res_kernel<NCB, D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    conv1x1_res_kernel<NCB, D><<<grid, 512, x1r_lds_bytes(NCB, nres), s>>>(a, ng, nres);
}

}  // namespace

int nps_conv1x1_res_plan(const nps_conv2d_t& a, int all, int* ncb, int* ng, int* nres) {
    // all = 0: only the planar (NCHW) 1x1s with 192 < Cout <= 256 — the decoder's pre-output, which the LDS-staged
    // kernel (Cout <= 192, NHWC) cannot take and the co-block kernel ran at 1.4 TB/s; all = 1 (dev knob
    // NPS_X1_RES=1): every eligible 1x1
    if (!all && !(a.out_nchw && a.Cout > 192 && a.Cout <= 256)) return 0;
    if (a.KH * a.KW != 1 || a.accumulate || a.addend1 != nullptr || a.gn_stats != nullptr || a.pre_act != 0 ||
        a.spec_z != nullptr)
        return 0;
    if (a.out_nchw && (a.addend0 != nullptr || a.out_stats != nullptr)) return 0;
    if (a.out_stats != nullptr && a.Cout > 192) return 0;  // (moments of the stored values: addend / act included)
    if ((long)a.B * ((a.Hout * a.Wout + 31) / 32) >= (1L << 31)) return 0;
    const int nr = x1r_nres(a.Cin);
    const int lmax = 160 * 1024;
    int c = 0, g = 0;
    if (a.Cout <= 192 && x1r_lds_bytes(6, nr) <= lmax) {
        c = 6, g = 1;
    } else if (a.Cout <= 192 && x1r_lds_bytes(3, nr) <= lmax) {
        c = 3, g = 2;
    } else if (a.Cout > 192 && a.Cout <= 256 && x1r_lds_bytes(4, nr) <= lmax) {
        c = 4, g = 2;
    } else {
        return 0;
    }
    *ncb = c;
    *ng = g;
    *nres = nr;
    return 1;
}

int nps_launch_conv1x1_res(const nps_conv2d_t& a, int all, hipStream_t s) {
    int ncb = 0, ng = 0, nres = 0;
    if (!nps_conv1x1_res_plan(a, all, &ncb, &ng, &nres)) return 0;
    static long gx = 0;
    if (gx == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 16)
            n = 256;
        gx = n & ~15;  // persistent: one work-group per CU, a multiple of 16 (8 XCDs x 2 channel groups)
    }
    if (ncb == 6)
        launch<6, 3>(a, (unsigned)gx, 1, nres, s);
    else if (ncb == 3)
        launch<3, 4>(a, (unsigned)gx, 2, nres, s);
    else
        launch<4, 4>(a, (unsigned)gx, 2, nres, s);
    return 1;
}
