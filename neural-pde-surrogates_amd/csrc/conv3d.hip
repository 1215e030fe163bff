// 3-D U-Net convolutions of the 3-D U-FNO (BASELINE config C5): every Conv3d / ConvTranspose3d of
// UNetModern(num_spatial_dims=3) (proc_unet_modern.py:199-455; the 3-D Upsample is this build's definition,
// include/nps.h) as one implicit-GEMM kernel on NDHWC activations, bf16 storage on v_mfma_f32_32x32x16_bf16
// or fp32 storage on the exact-fp32 v_mfma_f32_32x32x2_f32, with the GroupNorm+GELU prologue, torch.cat /
// crop_Nd as a virtual frame of up to 3 sources, circular / zero frame extension, and the bias / addend /
// GELU / accumulate-at-offset epilogue.
//
// GEMM: out[co][voxel] = sum over (kd, ci, kh, kw) of W[co][ci][kd][kh][kw] * frame[voxel*S + (kd, kh, kw)][ci].
// Work-group = 256 threads (4 waves): 64 output channels x (TH rows x 32 columns) of one output depth slice;
// wave w owns the 64 channels x rows [w*TH/4, +TH/4) (2 x TH/4 32x32 accumulators).  K loop in stages of
// (kd, 16-channel chunk): the stage's input patch ((TH-1)S+K rows x 31S+K columns x 16 channels, the
// prologue applied while staging) and its K*K x 64 x 16 weights go through a double-buffered LDS ring,
// loaded into registers one stage ahead so the global loads overlap the MFMAs of the current stage.
// LDS images are [pixel | channel row][16] with the two 8-channel halves XOR-swizzled by bit 3 of the row,
// so the ds_read_b128 B / A fragment reads of 32 consecutive rows are bank-conflict free.
#include "nps_common.hpp"

namespace {

typedef unsigned short bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ unsigned f2bf(float v) { return (unsigned)__builtin_bit_cast(bf16_t, (__bf16)v); }

// 8 consecutive channels of one voxel, raw storage bits
template <typename T> struct Vec8;
template <> struct Vec8<bf16_t> {
    u32x4 a;
    __device__ __forceinline__ void zero() { a = u32x4{0u, 0u, 0u, 0u}; }
    __device__ __forceinline__ float get(int e) const {
        const unsigned w = a[e >> 1];
        return bf2f((e & 1) ? (w >> 16) : (w & 0xffffu));
    }
    __device__ __forceinline__ void set(int e, float x) {
        const unsigned h = f2bf(x);
        const unsigned w = a[e >> 1];
        a[e >> 1] = (e & 1) ? ((w & 0xffffu) | (h << 16)) : ((w & 0xffff0000u) | h);
    }
    __device__ __forceinline__ void load(const bf16_t* p) { a = *reinterpret_cast<const u32x4*>(p); }
    __device__ __forceinline__ void load_elem(int e, const bf16_t* p) {
        const unsigned h = *p, w = a[e >> 1];
        a[e >> 1] = (e & 1) ? ((w & 0xffffu) | (h << 16)) : ((w & 0xffff0000u) | h);
    }
    __device__ __forceinline__ void store(bf16_t* p) const { *reinterpret_cast<u32x4*>(p) = a; }
    // channels [4h, 4h + 4) from p (8-B aligned: a 4-channel run of a source with C % 4 == 0)
    __device__ __forceinline__ void load_half(int h, const bf16_t* p) {
        const u32x2 w = *reinterpret_cast<const u32x2*>(p);
        a[2 * h] = w[0];
        a[2 * h + 1] = w[1];
    }
};
template <> struct Vec8<float> {
    u32x4 a, b;
    __device__ __forceinline__ void zero() { a = b = u32x4{0u, 0u, 0u, 0u}; }
    __device__ __forceinline__ float get(int e) const { return __uint_as_float(e < 4 ? a[e] : b[e - 4]); }
    __device__ __forceinline__ void set(int e, float x) {
        if (e < 4) a[e] = __float_as_uint(x); else b[e - 4] = __float_as_uint(x);
    }
    __device__ __forceinline__ void load(const float* p) {
        a = reinterpret_cast<const u32x4*>(p)[0];
        b = reinterpret_cast<const u32x4*>(p)[1];
    }
    __device__ __forceinline__ void load_elem(int e, const float* p) { set(e, *p); }
    __device__ __forceinline__ void load_half(int h, const float* p) {
        if (h == 0) a = *reinterpret_cast<const u32x4*>(p); else b = *reinterpret_cast<const u32x4*>(p);
    }
    __device__ __forceinline__ void store(float* p) const {
        reinterpret_cast<u32x4*>(p)[0] = a;
        reinterpret_cast<u32x4*>(p)[1] = b;
    }
};

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <typename T> __device__ __forceinline__ void st1(T* p, float v);
template <> __device__ __forceinline__ void st1<bf16_t>(bf16_t* p, float v) { *p = (bf16_t)f2bf(v); }
template <> __device__ __forceinline__ void st1<float>(float* p, float v) { *p = v; }

// extended-frame index -> core-frame index, -1 in the zero padding
__device__ __forceinline__ int ext_to_core(int f, int n, int circ, int zpad) {
    const int g = f - zpad;
    if (g < 0 || g >= n + 2 * circ) return -1;
    return circ ? nps::wrap_mod(g - circ, n) : g;
}

// channels [c0, c0+8) of core voxel (cd, ch, cw): each source fills the channels it holds where it covers
// the voxel; everything else reads 0
template <typename T>
__device__ __forceinline__ void load_piece(Vec8<T>& r, const nps_conv3d_t& a, int b, int cd, int ch, int cw, int c0) {
    r.zero();
    int lo = 0;
#pragma unroll
    for (int si = 0; si < NPS_MAX_SRC; ++si) {
        if (si < a.nsrc) {
            const nps_src3_t& s = a.src[si];
            if (c0 + 8 > lo && c0 < lo + s.C) {
                const int dd = cd - s.off_d, hh = ch - s.off_h, ww = cw - s.off_w;
                if (dd >= 0 && dd < s.D && hh >= 0 && hh < s.H && ww >= 0 && ww < s.W) {
                    const T* p = reinterpret_cast<const T*>(s.ptr) +
                                 ((((size_t)b * s.D + dd) * s.H + hh) * s.W + ww) * s.C;
                    if (c0 >= lo && c0 + 8 <= lo + s.C && (s.C & 7) == 0 && ((c0 - lo) & 7) == 0) {
                        r.load(p + (c0 - lo));
                    } else if ((s.C & 3) == 0 && ((c0 - lo) & 3) == 0) {
                        // 4-channel runs (C % 4 == 0, e.g. 64 + 4 channels): one 8-B (bf16) / 16-B load per
                        // half inside the source instead of 8 element loads
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int c = c0 + 4 * h;
                            if (c >= lo && c + 4 <= lo + s.C) r.load_half(h, p + (c - lo));
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const int c = c0 + e;
                            if (c >= lo && c < lo + s.C) r.load_elem(e, p + (c - lo));
                        }
                    }
                }
            }
            lo += s.C;
        }
    }
}

template <int K, int S, int TH>
struct Geo {
    static constexpr int TW = 32;
    static constexpr int PR = (TH - 1) * S + K;
    static constexpr int PC = (TW - 1) * S + K;
    static constexpr int NPIX = PR * PC;
    static constexpr int NPP = NPIX * 2;           // 8-channel pieces of a stage's patch
    static constexpr int NWP = K * K * 64 * 2;     // 8-channel pieces of a stage's weights
    static constexpr int PPT = (NPP + 255) / 256;  // per thread
    static constexpr int WPT = (NWP + 255) / 256;
    static constexpr int PATCH = NPIX * 16;        // elements
    static constexpr int WTS = K * K * 64 * 16;
    static constexpr int BUF = PATCH + WTS;
    static constexpr int RW = TH / 4;              // rows (32-voxel blocks) per wave
};

__device__ __forceinline__ int swz(int row) { return (row >> 3) & 1; }
#ifndef NPS_C3D_XCD
// 3-D convs: work-group i (on XCD i % 8) takes tile (i % 8) * (n / 8) + i / 8, so each XCD's L2 sees a contiguous
// run of tiles (whole slices, consecutive depths) instead of every 8th; a bijection, outputs unchanged.  C5 +1.1 %
// with the A/B arms in both orders (profiles/r6/experiments/c5_conv3d_glds_ab.txt Pass 10); 0 in a dev build: off
#define NPS_C3D_XCD 1
#endif
#ifndef NPS_PACK3D_U
#define NPS_PACK3D_U 4  // pieces per thread in flight in the frame packs (dev builds: tools/build_variant.sh)
#endif
// 64 zero bytes: the LDS-DMA source of patch slots outside the frame
__device__ __attribute__((aligned(64))) unsigned int c3d_zero16[16];

// SIMPLE: one source covering the core frame at offset 0, channels a multiple of 16, no prologue (the
// frame_pack3d output): a patch slot's address is fixed per tile (only the depth slice moves per stage), so
// staging is one add + one 16-B load and one ds_write per slot
// GLT (bf16 SIMPLE frames): the stage is copied global -> LDS by LDS-DMA (global_load_lds_dwordx4) instead of
// through registers; the lane-linear LDS image keeps the half-swap swizzle by swapping the SOURCE halves, and
// slots outside the frame read a zero line — no staging registers, no commit pass
// SB (with GLT): ONE stage buffer — load, barrier, compute, barrier — so a work-group needs half the LDS and three
// fit a CU: each exposes its own load latency, the other two keep the MFMA pipe fed
template <typename T, int K, int S, int TH, bool SIMPLE, bool GLT = false, bool SB = false>
__device__ __forceinline__ void conv3d_body(const nps_conv3d_t& a, int nchunk, int ntile) {
    using G = Geo<K, S, TH>;
    constexpr bool GL = GLT && SIMPLE && sizeof(T) == 2;
    static_assert(!SB || GLT, "single stage buffer: LDS-DMA staging only");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* ring = reinterpret_cast<T*>(smem);
    // [nchunk*16] GN affine per channel
    float* gscale = reinterpret_cast<float*>(smem + (SB ? 1 : 2) * G::BUF * sizeof(T));
    float* gshift = gscale + nchunk * 16;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ntw = (a.Wout + 31) / 32, nth = (a.Hout + TH - 1) / TH;
    int t = blockIdx.x;
    if (NPS_C3D_XCD) {  // work-group i runs on XCD i % 8: give each XCD a contiguous run of tiles (L2 locality)
        const int n = (int)gridDim.x, full = n & ~7;
        if (t < full) t = (t & 7) * (full >> 3) + (t >> 3);
    }
    const int tw = t % ntw; t /= ntw;
    const int th = t % nth; t /= nth;
    const int md = t % a.Dout;
    const int b = t / a.Dout;
    const int tile = blockIdx.y, z = blockIdx.z;
    const int h0 = th * TH, w0 = tw * 32;
    const int Dext = a.Dc + 2 * (a.circ + a.zpad), Hext = a.Hc + 2 * (a.circ + a.zpad),
              Wext = a.Wc + 2 * (a.circ + a.zpad);
    (void)Dext;
    const bool pro = !SIMPLE && (a.gn_stats != nullptr || a.pre_act != 0);

    if (pro) {  // x' = x * scale[c] + shift[c] (GroupNorm affine of this sample), then the activation
        for (int c = tid; c < nchunk * 16; c += 256) {
            float sc = 1.f, sh = 0.f;
            if (a.gn_stats != nullptr && c < a.Cin) {
                const int g = c / (a.Cin / a.gn_groups);
                const double n = (double)a.Dc * a.Hc * a.Wc * (a.Cin / a.gn_groups);
                const double mean = a.gn_stats[(b * a.gn_groups + g) * 2] / n;
                const double var = fmax(a.gn_stats[(b * a.gn_groups + g) * 2 + 1] / n - mean * mean, 0.0);
                const float rstd = (float)(1.0 / sqrt(var + (double)a.gn_eps));
                sc = a.gn_gamma[c] * rstd;
                sh = a.gn_beta[c] - (float)mean * sc;
            }
            gscale[c] = sc;
            gshift[c] = sh;
        }
        __syncthreads();
    }

    const T* wbase = reinterpret_cast<const T*>(a.wpack) + (size_t)(z * ntile + tile) * K * nchunk * G::WTS;
    const int nstage = K * nchunk;

    Vec8<T> pr[GL ? 1 : G::PPT], wr[GL ? 1 : G::WPT];
    // SIMPLE: per-slot element offset within a depth slice (-1: zero padding / past the patch)
    int soff[G::PPT];
    const T* sbase = reinterpret_cast<const T*>(a.src[0].ptr) + (size_t)b * a.Dc * a.Hc * a.Wc * a.Cin;
    const size_t slice = (size_t)a.Hc * a.Wc * a.Cin;
    if constexpr (SIMPLE) {
#pragma unroll
        for (int i = 0; i < G::PPT; ++i) {
            const int idx = tid + 256 * i;
            soff[i] = -1;
            if (idx < G::NPP) {
                const int pix = idx >> 1, half = idx & 1;
                const int prr = pix / G::PC, pcc = pix - prr * G::PC;
                const int fh = h0 * S + prr, fw = w0 * S + pcc;
                const int ch = fh < Hext ? ext_to_core(fh, a.Hc, a.circ, a.zpad) : -1;
                const int cw = fw < Wext ? ext_to_core(fw, a.Wc, a.circ, a.zpad) : -1;
                // (GL: the slot's LDS half holds channel half half ^ swz(pix), as commit's swizzled store)
                if (ch >= 0 && cw >= 0) soff[i] = (ch * a.Wc + cw) * a.Cin + (GL ? (half ^ swz(pix)) : half) * 8;
            }
        }
    }
    auto fetch = [&](int st) {
        const int kd = st / nchunk, chunk = st - kd * nchunk;
        const int fd = md * S + kd;
        const int cd = ext_to_core(fd, a.Dc, a.circ, a.zpad);
        if constexpr (SIMPLE) {
            const T* sp = sbase + (size_t)(cd < 0 ? 0 : cd) * slice + chunk * 16;
#pragma unroll
            for (int i = 0; i < G::PPT; ++i) {
                pr[i].zero();
                if (cd >= 0 && soff[i] >= 0) pr[i].load(sp + soff[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < (SIMPLE ? 0 : G::PPT); ++i) {
            const int idx = tid + 256 * i;
            pr[i].zero();
            if (idx < G::NPP) {
                const int pix = idx >> 1, half = idx & 1;
                const int prr = pix / G::PC, pcc = pix - prr * G::PC;
                const int fh = h0 * S + prr, fw = w0 * S + pcc;
                const int ch = fh < Hext ? ext_to_core(fh, a.Hc, a.circ, a.zpad) : -1;
                const int cw = fw < Wext ? ext_to_core(fw, a.Wc, a.circ, a.zpad) : -1;
                if (cd >= 0 && ch >= 0 && cw >= 0) load_piece<T>(pr[i], a, b, cd, ch, cw, chunk * 16 + half * 8);
            }
        }
        const T* wsrc = wbase + (size_t)st * G::WTS;
#pragma unroll
        for (int i = 0; i < G::WPT; ++i) {
            const int idx = tid + 256 * i;
            if (idx < G::NWP) wr[i].load(wsrc + idx * 8);
        }
    };
    auto commit = [&](int st, int buf) {
        const int kd = st / nchunk, chunk = st - kd * nchunk;
        const int cd = ext_to_core(md * S + kd, a.Dc, a.circ, a.zpad);
        T* P = ring + buf * G::BUF;
#pragma unroll
        for (int i = 0; i < G::PPT; ++i) {
            const int idx = tid + 256 * i;
            if (idx < G::NPP) {
                const int pix = idx >> 1, half = idx & 1;
                if (pro) {
                    const int prr = pix / G::PC, pcc = pix - prr * G::PC;
                    const int fh = h0 * S + prr, fw = w0 * S + pcc;
                    const bool core = cd >= 0 && fh < Hext && fw < Wext &&
                                      ext_to_core(fh, a.Hc, a.circ, a.zpad) >= 0 &&
                                      ext_to_core(fw, a.Wc, a.circ, a.zpad) >= 0;
                    if (core) {  // frame values, crop zeros included, are normalised (conv padding is not)
                        const int c0 = chunk * 16 + half * 8;
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            float x = fmaf(pr[i].get(e), gscale[c0 + e], gshift[c0 + e]);
                            if (a.pre_act == 1) x = nps::gelu_fast(x);
                            pr[i].set(e, c0 + e < a.Cin ? x : 0.f);
                        }
                    }
                }
                pr[i].store(P + pix * 16 + ((half ^ swz(pix)) * 8));
            }
        }
        T* Wl = P + G::PATCH;
#pragma unroll
        for (int i = 0; i < G::WPT; ++i) {
            const int idx = tid + 256 * i;
            if (idx < G::NWP) {
                const int half = idx & 1, row = idx >> 1;  // row = tap * 64 + co
                wr[i].store(Wl + row * 16 + ((half ^ swz(row & 63)) * 8));
            }
        }
    };

    // GL: stage st -> ring buffer buf by LDS-DMA; wave w's instruction i fills slots [256 i + 64 w, + 64)
    auto fetch_gl = [&](int st, int buf) {
        if constexpr (GL) {
            const int kd = st / nchunk, chunk = st - kd * nchunk;
            const int cd = ext_to_core(md * S + kd, a.Dc, a.circ, a.zpad);
            const T* sp = sbase + (size_t)(cd < 0 ? 0 : cd) * slice + chunk * 16;
            T* P = ring + buf * G::BUF;
#pragma unroll
            for (int i = 0; i < G::PPT; ++i) {
                const int idx = tid + 256 * i;
                if (256 * i + 64 * wave < G::NPP && idx < G::NPP) {
                    const void* src = (cd >= 0 && soff[i] >= 0) ? (const void*)(sp + soff[i]) : (const void*)c3d_zero16;
                    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(P + (256 * i + 64 * wave) * 8),
                                                     16, 0, 0);
                }
            }
            const T* wsrc = wbase + (size_t)st * G::WTS;
            T* Wl = P + G::PATCH;
#pragma unroll
            for (int i = 0; i < G::WPT; ++i) {
                const int idx = tid + 256 * i;
                if (256 * i + 64 * wave < G::NWP && idx < G::NWP) {
                    const int half = idx & 1, row = idx >> 1;
                    __builtin_amdgcn_global_load_lds((const void*)(wsrc + row * 16 + ((half ^ swz(row & 63)) * 8)),
                                                     (__attribute__((address_space(3))) void*)(Wl + (256 * i + 64 * wave) * 8),
                                                     16, 0, 0);
                }
            }
        }
    };

    f32x16 acc[2][G::RW];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < G::RW; ++r)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[cb][r][q] = 0.f;

    if constexpr (GL) {
        fetch_gl(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        fetch(0);
        commit(0, 0);
    }
    __syncthreads();
    const int col = lane & 31, hl = lane >> 5;
    for (int st = 0; st < nstage; ++st) {
        const int buf = SB ? 0 : (st & 1);
        if constexpr (SB) {
        } else if constexpr (GL) {
            if (st + 1 < nstage) fetch_gl(st + 1, buf ^ 1);
        } else {
            if (st + 1 < nstage) fetch(st + 1);
        }
        const T* P = ring + buf * G::BUF;
        const T* Wl = P + G::PATCH;
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
                const int tap = kh * K + kw;
                if constexpr (sizeof(T) == 2) {
                    bf16x8 A[2], Bv[G::RW];
#pragma unroll
                    for (int cb = 0; cb < 2; ++cb) {
                        const int co = cb * 32 + col;
                        A[cb] = *reinterpret_cast<const bf16x8*>(Wl + (tap * 64 + co) * 16 + ((hl ^ swz(co)) * 8));
                    }
#pragma unroll
                    for (int r = 0; r < G::RW; ++r) {
                        const int pix = ((wave * G::RW + r) * S + kh) * G::PC + col * S + kw;
                        Bv[r] = *reinterpret_cast<const bf16x8*>(P + pix * 16 + ((hl ^ swz(pix)) * 8));
                    }
#pragma unroll
                    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                        for (int r = 0; r < G::RW; ++r)
                            acc[cb][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[cb], Bv[r], acc[cb][r], 0, 0, 0);
                } else {
#pragma unroll
                    for (int ks = 0; ks < 8; ++ks) {
                        const int k = 2 * ks + hl;
                        float A[2], Bv[G::RW];
#pragma unroll
                        for (int cb = 0; cb < 2; ++cb) {
                            const int co = cb * 32 + col;
                            A[cb] = Wl[(tap * 64 + co) * 16 + (((k >> 3) ^ swz(co)) * 8) + (k & 7)];
                        }
#pragma unroll
                        for (int r = 0; r < G::RW; ++r) {
                            const int pix = ((wave * G::RW + r) * S + kh) * G::PC + col * S + kw;
                            Bv[r] = P[pix * 16 + (((k >> 3) ^ swz(pix)) * 8) + (k & 7)];
                        }
#pragma unroll
                        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                            for (int r = 0; r < G::RW; ++r)
                                acc[cb][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[cb], Bv[r], acc[cb][r], 0, 0, 0);
                    }
                }
            }
        }
        if constexpr (SB) {
            if (st + 1 < nstage) {
                __syncthreads();  // every read of the buffer is done
                fetch_gl(st + 1, 0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else if constexpr (GL) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage st + 1 has landed
        } else {
            if (st + 1 < nstage) commit(st + 1, buf ^ 1);
        }
        __syncthreads();
    }

    // epilogue: lane holds voxel column `col`, channels 8j + 4*hl + (0..3) of each 32-channel block
    const int pd = a.transposed ? (z >> 2) : 0, ph = a.transposed ? ((z >> 1) & 1) : 0,
              pw = a.transposed ? (z & 1) : 0;
    const int od = md * a.out_os + a.out_off_d + pd;
    // out_stats: moments of the stored values (fp32 per 4-channel quad, fp64 across) — with accumulate, of the
    // change (stored value minus the value it replaced: s^2 - o^2 = (s - o)(s + o)), so a buffer seeded with out's
    // moments ends with the accumulated tensor's (the 2-D convs' convention, include/nps.h out_stats) — published
    // per wave at the end, so no early return: every lane reaches the wave-collective publish
    const bool st = a.out_stats != nullptr;
    float f1 = 0.f, f2 = 0.f;  // this lane's (at most 2 x RW x 16) stored values: fp32, then fp64 per wave
    auto mom = [&](float x0, float x1, float x2, float x3) {
        f1 += (x0 + x1) + (x2 + x3);
        f2 += (x0 * x0 + x1 * x1) + (x2 * x2 + x3 * x3);
    };
    auto momd = [&](const float (&x)[4], const float (&o)[4]) {  // the change of 4 accumulated values
        f1 += ((x[0] - o[0]) + (x[1] - o[1])) + ((x[2] - o[2]) + (x[3] - o[3]));
        f2 += ((x[0] - o[0]) * (x[0] + o[0]) + (x[1] - o[1]) * (x[1] + o[1])) +
              ((x[2] - o[2]) * (x[2] + o[2]) + (x[3] - o[3]) * (x[3] + o[3]));
    };
    if (od >= 0 && od < a.out_D) {
    T* out = reinterpret_cast<T*>(a.out);
    const T* add = reinterpret_cast<const T*>(a.addend);
    const int w = w0 + col;
    const int ow = w * a.out_os + a.out_off_w + pw;
    const bool vec4 = (a.out_C & 3) == 0 && (a.Cout & 3) == 0;
#pragma unroll
    for (int r = 0; r < G::RW; ++r) {
        const int h = h0 + wave * G::RW + r;
        const int oh = h * a.out_os + a.out_off_h + ph;
        if (h >= a.Hout || w >= a.Wout || oh < 0 || oh >= a.out_H || ow < 0 || ow >= a.out_W) continue;
        const size_t vox = (((size_t)b * a.out_D + od) * a.out_H + oh) * a.out_W + ow;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co0 = tile * 64 + cb * 32 + 8 * j + 4 * hl;
                if (co0 >= a.Cout) continue;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int co = co0 + e;
                    v[e] = acc[cb][r][4 * j + e] + ((a.bias != nullptr && co < a.Cout) ? a.bias[co] : 0.f);
                }
                T* op = out + vox * a.out_C + co0;
                const T* ap = add != nullptr ? add + vox * a.out_C + co0 : nullptr;
                if (vec4 && sizeof(T) == 4) {
                    f32x4 o = {v[0], v[1], v[2], v[3]};
                    if (ap) o += *reinterpret_cast<const f32x4*>(ap);
                    if (a.act == 1)
#pragma unroll
                        for (int e = 0; e < 4; ++e) o[e] = nps::gelu_erf(o[e]);
                    f32x4 old = {0.f, 0.f, 0.f, 0.f};
                    if (a.accumulate) {
                        old = *reinterpret_cast<const f32x4*>(op);
                        o += old;
                    }
                    *reinterpret_cast<f32x4*>(op) = o;
                    if (st) {
                        const float x4[4] = {o[0], o[1], o[2], o[3]}, o4[4] = {old[0], old[1], old[2], old[3]};
                        momd(x4, o4);
                    }
                } else if (vec4) {  // bf16: 4 channels = one 8-B access
                    float o[4] = {v[0], v[1], v[2], v[3]};
                    if (ap) {
                        const u32x2 w = *reinterpret_cast<const u32x2*>(ap);
                        o[0] += bf2f(w[0] & 0xffffu); o[1] += bf2f(w[0] >> 16);
                        o[2] += bf2f(w[1] & 0xffffu); o[3] += bf2f(w[1] >> 16);
                    }
                    if (a.act == 1)
#pragma unroll
                        for (int e = 0; e < 4; ++e) o[e] = nps::gelu_erf(o[e]);
                    float old[4] = {0.f, 0.f, 0.f, 0.f};
                    if (a.accumulate) {
                        const u32x2 w = *reinterpret_cast<const u32x2*>(op);
                        old[0] = bf2f(w[0] & 0xffffu); old[1] = bf2f(w[0] >> 16);
                        old[2] = bf2f(w[1] & 0xffffu); old[3] = bf2f(w[1] >> 16);
#pragma unroll
                        for (int e = 0; e < 4; ++e) o[e] += old[e];
                    }
                    const u32x2 r = {f2bf(o[0]) | (f2bf(o[1]) << 16), f2bf(o[2]) | (f2bf(o[3]) << 16)};
                    *reinterpret_cast<u32x2*>(op) = r;
                    if (st) {  // (as stored)
                        const float x4[4] = {bf2f(r[0] & 0xffffu), bf2f(r[0] >> 16), bf2f(r[1] & 0xffffu),
                                             bf2f(r[1] >> 16)};
                        momd(x4, old);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if (co0 + e >= a.Cout) continue;
                        float o = v[e];
                        if (ap) o += ld1<T>(ap + e);
                        if (a.act == 1) o = nps::gelu_erf(o);
                        const float old = a.accumulate ? ld1<T>(op + e) : 0.f;
                        if (a.accumulate) o += old;
                        st1<T>(op + e, o);
                        if (st) {
                            const float q = ld1<T>(op + e);  // (as stored)
                            f1 += q - old;
                            f2 += (q - old) * (q + old);
                        }
                    }
                }
            }
        }
    }
    }
    if (st) {  // (uniform) one atomic pair per work-group: the 4 waves' sums meet in the (free) ring first
        const double s1 = nps::wave_sum((double)f1);
        const double s2 = nps::wave_sum((double)f2);
        double* red = reinterpret_cast<double*>(smem);
        __syncthreads();  // every wave is past its last ring read
        if (lane == 0) {
            red[2 * wave] = s1;
            red[2 * wave + 1] = s2;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double* q = a.out_stats + ((size_t)b * NPS_STATS_SUB + blockIdx.x % NPS_STATS_SUB) * 2;
            atomicAdd(q, (red[0] + red[2]) + (red[4] + red[6]));
            atomicAdd(q + 1, (red[1] + red[3]) + (red[5] + red[7]));
        }
    }
}

template <typename T, int K, int S, int TH, bool SIMPLE, bool GLT = false, bool SB = false>
__global__ __launch_bounds__(256) void conv3d_kernel(const nps_conv3d_t a, int nchunk, int ntile) {
    conv3d_body<T, K, S, TH, SIMPLE, GLT, SB>(a, nchunk, ntile);
}
// (dev variant: the same body held to two waves per SIMD, for register-heavy tile shapes)
template <typename T, int K, int S, int TH, bool SIMPLE, bool GLT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv3d_kernel_o2(const nps_conv3d_t a,
                                                                                             int nchunk, int ntile) {
    conv3d_body<T, K, S, TH, SIMPLE, GLT>(a, nchunk, ntile);
}
// (register-staged, held to four waves per SIMD: the 1x1x1 over several sources, a streaming kernel)
template <typename T, int K, int S, int TH, bool SIMPLE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void conv3d_kernel_o4r(const nps_conv3d_t a,
                                                                                              int nchunk, int ntile) {
    conv3d_body<T, K, S, TH, SIMPLE>(a, nchunk, ntile);
}
// (one stage buffer held to four waves per SIMD — four work-groups per CU)
template <typename T, int K, int S, int TH, bool SIMPLE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void conv3d_kernel_o4(const nps_conv3d_t a,
                                                                                             int nchunk, int ntile) {
    conv3d_body<T, K, S, TH, SIMPLE, true, true>(a, nchunk, ntile);
}

// wpack[(((((z*ntile + tile)*K + kd)*nchunk + chunk)*K*K + tap)*64 + col)*16 + k]
template <typename T>
__global__ void conv3d_pack_kernel(const float* __restrict__ w, T* __restrict__ wp, int Cout, int Cin, int K,
                                   int transposed, int nchunk, int ntile, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        long r = i;
        const int k = (int)(r % 16); r /= 16;
        const int col = (int)(r % 64); r /= 64;
        const int tap = (int)(r % (K * K)); r /= K * K;
        const int chunk = (int)(r % nchunk); r /= nchunk;
        const int kd = (int)(r % K); r /= K;
        const int tile = (int)(r % ntile);
        const int z = (int)(r / ntile);
        const int co = tile * 64 + col, ci = chunk * 16 + k, kh = tap / K, kw = tap % K;
        float v = 0.f;
        if (co < Cout && ci < Cin) {
            if (transposed) {  // phase (pd, ph, pw): tap t of an axis uses kernel index p + 2(1 - t)
                const int qd = (z >> 2) + 2 * (1 - kd), qh = ((z >> 1) & 1) + 2 * (1 - kh), qw = (z & 1) + 2 * (1 - kw);
                v = w[((((size_t)ci * Cout + co) * 4 + qd) * 4 + qh) * 4 + qw];
            } else {
                v = w[((((size_t)co * Cin + ci) * K + kd) * K + kh) * K + kw];
            }
        }
        if constexpr (sizeof(T) == 2) wp[i] = (T)f2bf(v); else wp[i] = v;
    }
}

// per (b, group) fp64 (sum, sum of squares) of a core frame.  Each source is swept over its own voxels
// (those inside the frame), one work item = 8 consecutive channels of one voxel, so consecutive threads read
// consecutive 16-B (bf16) / 32-B (fp32) pieces; per-thread group sums in registers, one block reduction.
template <typename T>
__global__ __launch_bounds__(256) void gn_stats3d_kernel(const nps_conv3d_t a, int G, double* __restrict__ stats) {
    __shared__ double scratch[4];
    const int b = blockIdx.y;
    const int cpg = a.Cin / G;
    double s[8], q[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) s[g] = q[g] = 0.0;
    int lo = 0;
#pragma unroll
    for (int si = 0; si < NPS_MAX_SRC; ++si) {
        if (si < a.nsrc) {
            const nps_src3_t& src = a.src[si];
            const int nck = (src.C + 7) / 8;
            const int nitem = src.D * src.H * src.W * nck;  // < 2^31 per sample (host-checked)
            const T* base = reinterpret_cast<const T*>(src.ptr) + (size_t)b * src.D * src.H * src.W * src.C;
            const bool vec = (src.C & 7) == 0;
            const bool inside = src.off_d >= 0 && src.off_h >= 0 && src.off_w >= 0 && src.off_d + src.D <= a.Dc &&
                                src.off_h + src.H <= a.Hc && src.off_w + src.W <= a.Wc;
            const long nel = (long)src.D * src.H * src.W * src.C;  // elements per sample
            if (inside && (src.C & 3) == 0 && (cpg & 3) == 0 && (lo & 3) == 0 && (nel & 7) == 0 &&
                nel < (1L << 31)) {
                // the source lies wholly inside the frame: a linear sweep of its elements 8 at a time (16-B loads
                // for bf16 whatever C % 8 is), each 4-element half in one group (C, the channels per group and the
                // source's first channel all % 4 == 0)
                const int nfl = (int)(nel / 8);
                auto acc8 = [&](const Vec8<T>& v, int it) {
                    if (G == 1) {  // one group (GroupNorm(1)): no channel index at all
                        float fs = 0.f, fq = 0.f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const float x = v.get(e);
                            fs += x;
                            fq = fmaf(x, x, fq);
                        }
                        s[0] += fs;
                        q[0] += fq;
                        return;
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int g0 = (lo + (int)((unsigned)(it * 8 + 4 * h) % (unsigned)src.C)) / cpg;
                        float fs = 0.f, fq = 0.f;
#pragma unroll
                        for (int e = 4 * h; e < 4 * h + 4; ++e) {
                            const float x = v.get(e);
                            fs += x;
                            fq = fmaf(x, x, fq);
                        }
#pragma unroll
                        for (int g = 0; g < 8; ++g)
                            if (g == g0) {
                                s[g] += fs;
                                q[g] += fq;
                            }
                    }
                };
                // U pieces per thread in flight (one 16-B load per piece): with one, a wave kept 1 KiB in flight
                // and the sweep ran at ~1.6 TB/s (latency-bound)
                constexpr int U = 4;
                const int stride = gridDim.x * 256;
                int it = blockIdx.x * 256 + threadIdx.x;
                for (; it + (U - 1) * stride < nfl; it += U * stride) {
                    Vec8<T> v[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) v[u].load(base + (size_t)(it + u * stride) * 8);
#pragma unroll
                    for (int u = 0; u < U; ++u) acc8(v[u], it + u * stride);
                }
                for (; it < nfl; it += stride) {
                    Vec8<T> v;
                    v.load(base + (size_t)it * 8);
                    acc8(v, it);
                }
                lo += src.C;
                continue;
            }
            // (cropped / unaligned sources) U pieces per thread in flight, as the fast path; a piece outside the
            // frame loads nothing and adds zeros
            auto fetch = [&](Vec8<T>& v, int it) {
                const int ck = it % nck;
                const int vox = it / nck;
                const int ww = vox % src.W;
                const int r = vox / src.W;
                const int hh = r % src.H, dd = r / src.H;
                const int cd = dd + src.off_d, ch = hh + src.off_h, cw = ww + src.off_w;
                v.zero();
                if (cd < 0 || cd >= a.Dc || ch < 0 || ch >= a.Hc || cw < 0 || cw >= a.Wc) return;
                const T* p = base + (size_t)vox * src.C + ck * 8;
                if (vec) {
                    v.load(p);
                } else if ((src.C & 3) == 0) {  // 4-channel runs (e.g. the 4 conditioning channels)
                    v.load_half(0, p);
                    if (ck * 8 + 8 <= src.C) v.load_half(1, p + 4);
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        if (ck * 8 + e < src.C) v.load_elem(e, p + e);
                }
            };
            constexpr int U = 4;
            const int stride = gridDim.x * 256;
            const int it0 = blockIdx.x * 256 + threadIdx.x;
            for (int itb = it0; itb < nitem; itb += U * stride) {
                Vec8<T> vv[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (itb + u * stride < nitem) fetch(vv[u], itb + u * stride);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int it = itb + u * stride;
                    if (it >= nitem) break;
                    const Vec8<T>& v = vv[u];
                    const int ck = it % nck;
                    const int c0 = lo + ck * 8;
                    if (vec && (cpg & 7) == 0 && (lo & 7) == 0) {  // the 8 channels lie in one group
                        const int g0 = c0 / cpg;
                        float fs = 0.f, fq = 0.f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const float x = v.get(e);
                            fs += x;
                            fq = fmaf(x, x, fq);
                        }
#pragma unroll
                        for (int g = 0; g < 8; ++g)
                            if (g == g0) {
                                s[g] += fs;
                                q[g] += fq;
                            }
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            if (ck * 8 + e >= src.C) continue;
                            const float x = v.get(e);
                            const int ge = (c0 + e) / cpg;
#pragma unroll
                            for (int g = 0; g < 8; ++g)
                                if (g == ge) {
                                    s[g] += x;
                                    q[g] += (double)x * x;
                                }
                        }
                    }
                }
            }
            lo += src.C;
        }
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        if (g < G) {
            const double ts = nps::block_sum(s[g], scratch);
            const double tq = nps::block_sum(q[g], scratch);
            if (threadIdx.x == 0) {
                atomicAdd(stats + (b * G + g) * 2, ts);
                atomicAdd(stats + (b * G + g) * 2 + 1, tq);
            }
        }
    }
}

// out[b][voxel][c] = act(GN(frame))[c] for c < Cin, 0 for Cin <= c < Cpad: the conv3d prologue applied once
// per frame element (the fused prologue would apply it to every element K x ~1.3 times, once per depth tap
// and halo); the conv then reads a single 16-channel-aligned source (conv3d_kernel SIMPLE).  One item = 8
// channels of one voxel (16-B loads / stores for bf16).
template <typename T>
__global__ __launch_bounds__(256) void frame_pack3d_kernel(const nps_conv3d_t a, T* __restrict__ out, int Cpad,
                                                           bool mflat_disabled) {
    __shared__ __attribute__((aligned(16))) float scl[512], sft[512];
    const int b = blockIdx.y;
    const bool gn = a.gn_stats != nullptr;
    for (int c = threadIdx.x; c < Cpad; c += 256) {
        float sc = 1.f, sh = 0.f;
        if (gn && c < a.Cin) {
            const int g = c / (a.Cin / a.gn_groups);
            const double n = (double)a.Dc * a.Hc * a.Wc * (a.Cin / a.gn_groups);
            const double mean = a.gn_stats[(b * a.gn_groups + g) * 2] / n;
            const double var = fmax(a.gn_stats[(b * a.gn_groups + g) * 2 + 1] / n - mean * mean, 0.0);
            const float rstd = (float)(1.0 / sqrt(var + (double)a.gn_eps));
            sc = a.gn_gamma[c] * rstd;
            sh = a.gn_beta[c] - (float)mean * sc;
        }
        scl[c] = sc;
        sft[c] = sh;
    }
    __syncthreads();
    const int npc = Cpad / 8;
    const int nitem = a.Dc * a.Hc * a.Wc * npc;
    T* ob = out + (size_t)b * a.Dc * a.Hc * a.Wc * Cpad;
    // one source covering the frame exactly, C % 4 == 0: its voxel index is the frame's, no decomposition
    const nps_src3_t& s0 = a.src[0];
    const bool flat = a.nsrc == 1 && s0.off_d == 0 && s0.off_h == 0 && s0.off_w == 0 && s0.D == a.Dc &&
                      s0.H == a.Hc && s0.W == a.Wc && (s0.C & 3) == 0;
    const bool mflat_off = mflat_disabled;
    const T* fb = reinterpret_cast<const T*>(s0.ptr) + (size_t)b * a.Dc * a.Hc * a.Wc * s0.C;
    // several sources, each covering the frame exactly (no crop offset), C % 4 == 0: a 4-channel half of a piece
    // lies in one source at the frame's voxel index — no coordinate decode, no per-source bounds checks
    bool mflat = !flat && a.nsrc >= 2 && !mflat_off;
    int mlo[NPS_MAX_SRC + 1];
    const T* mb[NPS_MAX_SRC];
    mlo[0] = 0;
#pragma unroll
    for (int si = 0; si < NPS_MAX_SRC; ++si) {
        const nps_src3_t& q = a.src[si];
        const bool in = si < a.nsrc;
        mflat = mflat && (!in || (q.off_d == 0 && q.off_h == 0 && q.off_w == 0 && q.D == a.Dc && q.H == a.Hc &&
                                  q.W == a.Wc && (q.C & 3) == 0));
        mlo[si + 1] = mlo[si] + (in ? q.C : 0);
        mb[si] = in ? reinterpret_cast<const T*>(q.ptr) + (size_t)b * a.Dc * a.Hc * a.Wc * q.C : nullptr;
    }
    auto fetch = [&](Vec8<T>& v, int it) {
        const int vox = it / npc;
        const int pc = it - vox * npc;
        if (flat) {
            v.zero();
            const T* p = fb + (size_t)vox * s0.C + pc * 8;
            if (pc * 8 + 4 <= s0.C) v.load_half(0, p);
            if (pc * 8 + 8 <= s0.C) v.load_half(1, p + 4);
            return;
        }
        if (mflat) {
            v.zero();
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = pc * 8 + 4 * h;
                if (c >= a.Cin) break;
                const int si = c < mlo[1] ? 0 : (c < mlo[2] ? 1 : 2);
                const int lo = si == 0 ? 0 : (si == 1 ? mlo[1] : mlo[2]);
                const int sC = (si == 0 ? mlo[1] : (si == 1 ? mlo[2] : mlo[3])) - lo;
                const T* p = (si == 0 ? mb[0] : (si == 1 ? mb[1] : mb[2])) + (size_t)vox * sC + (c - lo);
                v.load_half(h, p);
            }
            return;
        }
        const int cw = vox % a.Wc, r = vox / a.Wc;
        const int ch = r % a.Hc, cd = r / a.Hc;
        load_piece<T>(v, a, b, cd, ch, cw, pc * 8);
    };
    auto put = [&](Vec8<T>& v, int it) {
        const int vox = it / npc;
        const int pc = it - vox * npc;
        if (gn || a.pre_act) {
            // the piece's 8 affine pairs as 16-B LDS reads, GELU on packed pairs (gelu_fast2)
            const f32x4 s0 = *reinterpret_cast<const f32x4*>(scl + pc * 8), s1 = *reinterpret_cast<const f32x4*>(scl + pc * 8 + 4);
            const f32x4 h0 = *reinterpret_cast<const f32x4*>(sft + pc * 8), h1 = *reinterpret_cast<const f32x4*>(sft + pc * 8 + 4);
            float y[8];
#pragma unroll
            for (int e = 0; e < 8; ++e)
                y[e] = fmaf(v.get(e), e < 4 ? s0[e] : s1[e - 4], e < 4 ? h0[e] : h1[e - 4]);
            if (a.pre_act == 1) {
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    const nps::f32x2 g = nps::gelu_fast2(nps::f32x2{y[e], y[e + 1]});
                    y[e] = g[0];
                    y[e + 1] = g[1];
                }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) v.set(e, pc * 8 + e < a.Cin ? y[e] : 0.f);
        }
        v.store(ob + (size_t)vox * Cpad + pc * 8);
    };
    // U pieces per thread: all loads issued before the first store (vmcnt retires loads and stores in order)
    constexpr int U = NPS_PACK3D_U;
    const int stride = gridDim.x * 256;
    int it = blockIdx.x * 256 + threadIdx.x;
    for (; it + (U - 1) * stride < nitem; it += U * stride) {
        Vec8<T> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) fetch(v[u], it + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) put(v[u], it + u * stride);
    }
    for (; it < nitem; it += stride) {
        Vec8<T> v;
        fetch(v, it);
        put(v, it);
    }
}

// frame_pack3d for frames whose sources all cover the frame at offset 0 (C % 4 == 0): thread = (voxel lane, piece
// pc) with pc fixed for the thread's life, so the piece's source pointers, channel offsets and GroupNorm affine
// (computed as frame_pack3d_kernel does) stay in registers and a voxel costs one multiply-add per half, the
// loads, the affine + GELU and one coalesced 16-B store — no division per item, no LDS table.  Blocks of
// npc x (256 / npc) threads (npc = Cpad / 8 <= 64).  Bit-identical to frame_pack3d_kernel.
template <typename T>
__global__ __launch_bounds__(256) void frame_pack3d_flat_kernel(const nps_conv3d_t a, T* __restrict__ out, int Cpad) {
    const int npc = Cpad / 8, vpb = 256 / npc;
    const int tid = threadIdx.x;
    if (tid >= npc * vpb) return;  // (no barrier in this kernel)
    const int pc = tid % npc, vl = tid / npc;
    const int b = blockIdx.y;
    const int nvox = a.Dc * a.Hc * a.Wc;
    const bool gn = a.gn_stats != nullptr, tr = gn || a.pre_act != 0;
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = pc * 8 + e;
        sc[e] = 1.f;
        sh[e] = 0.f;
        if (gn && c < a.Cin) {  // (frame_pack3d_kernel's table entry for channel c)
            const int g = c / (a.Cin / a.gn_groups);
            const double n = (double)a.Dc * a.Hc * a.Wc * (a.Cin / a.gn_groups);
            const double mean = a.gn_stats[(b * a.gn_groups + g) * 2] / n;
            const double var = fmax(a.gn_stats[(b * a.gn_groups + g) * 2 + 1] / n - mean * mean, 0.0);
            const float rstd = (float)(1.0 / sqrt(var + (double)a.gn_eps));
            sc[e] = a.gn_gamma[c] * rstd;
            sh[e] = a.gn_beta[c] - (float)mean * sc[e];
        }
    }
    // the piece's two 4-channel halves: this sample's source pointer at the half's first channel (null past Cin)
    // and the source's channels per voxel; a whole 8-aligned piece of one source loads as one 16-B access
    const T* hp[2] = {nullptr, nullptr};
    int hC[2] = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int c = pc * 8 + 4 * h;
        int lo = 0;
#pragma unroll
        for (int si = 0; si < NPS_MAX_SRC; ++si) {
            if (si < a.nsrc) {
                const nps_src3_t& q = a.src[si];
                if (c < a.Cin && c >= lo && c < lo + q.C) {
                    hp[h] = reinterpret_cast<const T*>(q.ptr) + (size_t)b * nvox * q.C + (c - lo);
                    hC[h] = q.C;
                }
                lo += q.C;
            }
        }
    }
    const bool whole = hp[0] != nullptr && hp[1] == hp[0] + 4 && (hC[0] & 7) == 0 &&
                       ((reinterpret_cast<size_t>(hp[0]) & 15) == 0);
    T* ob = out + (size_t)b * nvox * Cpad + pc * 8;
    auto fetch = [&](Vec8<T>& v, int vx) {
        if (whole) {
            v.load(hp[0] + (size_t)vx * hC[0]);
            return;
        }
        v.zero();
        if (hp[0] != nullptr) v.load_half(0, hp[0] + (size_t)vx * hC[0]);
        if (hp[1] != nullptr) v.load_half(1, hp[1] + (size_t)vx * hC[1]);
    };
    auto put = [&](Vec8<T>& v, int vx) {
        if (tr) {
            float y[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = fmaf(v.get(e), sc[e], sh[e]);
            if (a.pre_act == 1) {
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    const nps::f32x2 g = nps::gelu_fast2(nps::f32x2{y[e], y[e + 1]});
                    y[e] = g[0];
                    y[e + 1] = g[1];
                }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) v.set(e, pc * 8 + e < a.Cin ? y[e] : 0.f);
        }
        v.store(ob + (size_t)vx * Cpad);
    };
    constexpr int U = NPS_PACK3D_U;
    const int stride = gridDim.x * vpb;
    int vx = blockIdx.x * vpb + vl;
    for (; vx + (U - 1) * stride < nvox; vx += U * stride) {
        Vec8<T> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) fetch(v[u], vx + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) put(v[u], vx + u * stride);
    }
    for (; vx < nvox; vx += stride) {
        Vec8<T> v;
        fetch(v, vx);
        put(v, vx);
    }
}

// 1x1x1 Conv3d on bf16 storage (K = 1, stride 1, no frame extension): the ResidualBlock shortcut over
// cat(h, crop_Nd(skip), crop_Nd(vb)) and the U-Net's final GroupNorm + GELU + 1x1 (proc_unet_modern.py:84, :265,
// :429).  A pointwise GEMM has no patch to share between output positions, and conv3d_kernel's 16-channel stages
// (one barrier, one dependent global load and 4 MFMAs each) left it latency-bound near 2 TB/s.  Here the packed
// weight of all Cout (NCB 32-channel blocks) and the bias stay in LDS for the whole launch; each wave takes 32
// voxels of its sample at a time, issues the loads of ALL its Cin channels (one 8-channel piece per 16-channel
// K-step and lane, at most NCH K-steps) for the NEXT tile before it runs the K-steps and the epilogue of this one
// (two tiles in flight per wave, no barrier).  Operand rounding, K order, prologue and epilogue are conv3d_kernel's,
// so the results are bit-identical; only the moments' fp32 partial sums group differently.
// (Measured alternative, not kept: the tile staged through LDS with voxel-major coalesced quad loads and 16-B
// stores — 2x slower, its per-quad addressing cost more than the fragment-shaped accesses it replaced.)
// Grid: work-groups per sample x B, one round of resident work-groups.
template <int NCB, int NCH, bool PRO>
__global__ __launch_bounds__(256) void conv3d_1x1_kernel(const nps_conv3d_t a, int nchunk) {
    constexpr int NCO = NCB * 32;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    bf16_t* Wl = reinterpret_cast<bf16_t*>(smem);  // [nchunk][NCO][16], 8-channel halves swizzled by row bit 3
    float* bsh = reinterpret_cast<float*>(smem + (size_t)nchunk * NCO * 32);  // [NCO] bias, zero past Cout
    float* gscale = bsh + NCO;
    float* gshift = gscale + nchunk * 16;
    double* red = reinterpret_cast<double*>(gshift + nchunk * 16);  // [4 waves][2]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.y;
    // packed rows [tile][kd = 0][chunk][tap = 0][64][16]: NCO = 64 x the packing's Cout tiles (host-checked)
    const bf16_t* wg = reinterpret_cast<const bf16_t*>(a.wpack);
    for (int i = tid; i < nchunk * NCO * 2; i += 256) {
        const int half = i & 1, row = i >> 1;  // row = chunk * NCO + co
        const int chunk = row / NCO, co = row - chunk * NCO;
        const u32x4 v = *reinterpret_cast<const u32x4*>(wg + ((size_t)((co >> 6) * nchunk + chunk) * 64 + (co & 63)) * 16 +
                                                        half * 8);
        *reinterpret_cast<u32x4*>(Wl + row * 16 + ((half ^ swz(co)) * 8)) = v;
    }
    if (tid < NCO) bsh[tid] = (a.bias != nullptr && tid < a.Cout) ? a.bias[tid] : 0.f;
    if constexpr (PRO) {  // as conv3d_kernel
        for (int c = tid; c < nchunk * 16; c += 256) {
            float sc = 1.f, sh = 0.f;
            if (a.gn_stats != nullptr && c < a.Cin) {
                const int g = c / (a.Cin / a.gn_groups);
                const double n = (double)a.Dc * a.Hc * a.Wc * (a.Cin / a.gn_groups);
                const double mean = a.gn_stats[(b * a.gn_groups + g) * 2] / n;
                const double var = fmax(a.gn_stats[(b * a.gn_groups + g) * 2 + 1] / n - mean * mean, 0.0);
                const float rstd = (float)(1.0 / sqrt(var + (double)a.gn_eps));
                sc = a.gn_gamma[c] * rstd;
                sh = a.gn_beta[c] - (float)mean * sc;
            }
            gscale[c] = sc;
            gshift[c] = sh;
        }
    }
    __syncthreads();

    const int col = lane & 31, hl = lane >> 5;
    const int nvox = a.Dc * a.Hc * a.Wc;  // = Dout x Hout x Wout (K = 1, no extension)
    const int ntv = (nvox + 31) / 32;
    bf16_t* out = reinterpret_cast<bf16_t*>(a.out);
    const bf16_t* add = reinterpret_cast<const bf16_t*>(a.addend);
    const bool st = a.out_stats != nullptr;
    // sources: first channels lo1 / lo2 of sources 1 / 2 (Cin past the last one), every source C % 4 == 0 and all
    // but the last C % 8 == 0 (host-checked), so a lane's 8-channel piece lies in one source: one 16-B load, or
    // one 8-B half at the last source's end
    const int ns = a.nsrc;
    const int lo1 = ns > 1 ? a.src[0].C : a.Cin, lo2 = ns > 2 ? a.src[0].C + a.src[1].C : a.Cin;
    auto coords = [&](int t, int& cd, int& ch, int& cw) {
        const int v = t * 32 + col;
        cw = v % a.Wc;
        const int r = v / a.Wc;
        ch = r % a.Hc;
        cd = r / a.Hc;
        return v < nvox;
    };
    // the NCH pieces of tile t, all loads in flight at once
    auto fetch = [&](int t, Vec8<bf16_t> (&x)[NCH]) {
        int cd, ch, cw;
        const bool vin = coords(t, cd, ch, cw);
        const bf16_t* sp[NPS_MAX_SRC];  // this voxel's channel 0 in each source, or null where it does not cover
#pragma unroll
        for (int si = 0; si < NPS_MAX_SRC; ++si) {
            const nps_src3_t& s = a.src[si];
            const int dd = cd - s.off_d, hh = ch - s.off_h, ww = cw - s.off_w;
            const bool ok = vin && si < ns && dd >= 0 && dd < s.D && hh >= 0 && hh < s.H && ww >= 0 && ww < s.W;
            sp[si] = ok ? reinterpret_cast<const bf16_t*>(s.ptr) + ((((size_t)b * s.D + dd) * s.H + hh) * s.W + ww) * s.C
                        : nullptr;
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            x[c].zero();
            const int c0 = c * 16 + hl * 8;
            if (c >= nchunk || c0 >= a.Cin) continue;
            const int si = c0 < lo1 ? 0 : (c0 < lo2 ? 1 : 2);
            const int cl = c0 - (si == 0 ? 0 : (si == 1 ? lo1 : lo2));
            const int sC = si == 0 ? lo1 : (si == 1 ? lo2 - lo1 : a.Cin - lo2);
            const bf16_t* p = si == 0 ? sp[0] : (si == 1 ? sp[1] : sp[2]);
            if (p == nullptr) continue;
            if (cl + 8 <= sC) x[c].load(p + cl);
            else x[c].load_half(0, p + cl);
        }
    };
    float f1 = 0.f, f2 = 0.f;  // this lane's stored values (changes, under accumulate): conv3d_kernel's momd
    const int tstride = gridDim.x * 4;
    int t = blockIdx.x * 4 + wave;
    Vec8<bf16_t> x[NCH];
    if (t < ntv) fetch(t, x);
    for (; t < ntv; t += tstride) {
        // next tile's loads first (two tiles in flight per wave)
        Vec8<bf16_t> xn[NCH];
        if (t + tstride < ntv) fetch(t + tstride, xn);
        int cd, ch, cw;
        const bool vin = coords(t, cd, ch, cw);
        f32x16 acc[NCB];
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[cb][q] = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (c >= nchunk) break;
            if constexpr (PRO) {  // frame values, crop zeros included, are normalised (as conv3d_kernel's commit)
                const int c0 = c * 16 + hl * 8;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float y = fmaf(x[c].get(e), gscale[c0 + e], gshift[c0 + e]);
                    if (a.pre_act == 1) y = nps::gelu_fast(y);
                    x[c].set(e, c0 + e < a.Cin ? y : 0.f);
                }
            }
            const bf16x8 B = __builtin_bit_cast(bf16x8, x[c].a);
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                const int co = cb * 32 + col;
                const bf16x8 A = *reinterpret_cast<const bf16x8*>(Wl + (c * NCO + co) * 16 + ((hl ^ swz(co)) * 8));
                acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, acc[cb], 0, 0, 0);
            }
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) x[c] = xn[c];
        // epilogue (conv3d_kernel's bf16 vec4 path): lane holds voxel `col`, channels cb*32 + 8j + 4hl + (0..3)
        const int od = cd * a.out_os + a.out_off_d, oh = ch * a.out_os + a.out_off_h, ow = cw * a.out_os + a.out_off_w;
        if (!vin || od < 0 || od >= a.out_D || oh < 0 || oh >= a.out_H || ow < 0 || ow >= a.out_W) continue;
        const size_t vox = (((size_t)b * a.out_D + od) * a.out_H + oh) * a.out_W + ow;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co0 = cb * 32 + 8 * j + 4 * hl;
                if (co0 >= a.Cout) continue;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(bsh + co0);
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = acc[cb][4 * j + e] + bv[e];
                bf16_t* op = out + vox * a.out_C + co0;
                if (add != nullptr) {
                    const u32x2 w = *reinterpret_cast<const u32x2*>(add + vox * a.out_C + co0);
                    o[0] += bf2f(w[0] & 0xffffu); o[1] += bf2f(w[0] >> 16);
                    o[2] += bf2f(w[1] & 0xffffu); o[3] += bf2f(w[1] >> 16);
                }
                if (a.act == 1)
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = nps::gelu_erf(o[e]);
                float old[4] = {0.f, 0.f, 0.f, 0.f};
                if (a.accumulate) {
                    const u32x2 w = *reinterpret_cast<const u32x2*>(op);
                    old[0] = bf2f(w[0] & 0xffffu); old[1] = bf2f(w[0] >> 16);
                    old[2] = bf2f(w[1] & 0xffffu); old[3] = bf2f(w[1] >> 16);
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] += old[e];
                }
                const u32x2 rr = {f2bf(o[0]) | (f2bf(o[1]) << 16), f2bf(o[2]) | (f2bf(o[3]) << 16)};
                *reinterpret_cast<u32x2*>(op) = rr;
                if (st) {  // (as stored)
                    const float s4[4] = {bf2f(rr[0] & 0xffffu), bf2f(rr[0] >> 16), bf2f(rr[1] & 0xffffu),
                                         bf2f(rr[1] >> 16)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        f1 += s4[e] - old[e];
                        f2 += (s4[e] - old[e]) * (s4[e] + old[e]);
                    }
                }
            }
        }
    }
    if (st) {  // (uniform) one atomic pair per work-group, as conv3d_kernel
        const double s1 = nps::wave_sum((double)f1);
        const double s2 = nps::wave_sum((double)f2);
        if (lane == 0) {
            red[2 * wave] = s1;
            red[2 * wave + 1] = s2;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double* q = a.out_stats + ((size_t)b * NPS_STATS_SUB + blockIdx.x % NPS_STATS_SUB) * 2;
            atomicAdd(q, (red[0] + red[2]) + (red[4] + red[6]));
            atomicAdd(q + 1, (red[1] + red[3]) + (red[5] + red[7]));
        }
    }
}

// dev knob NPS_C3D_1X1=0: 1x1x1 bf16 convs on conv3d_kernel (A/B)
bool c3d_1x1_on() {
    static const int g = [] {
        const char* e = std::getenv("NPS_C3D_1X1");
        return (e != nullptr && e[0] == '0') ? 0 : 1;
    }();
    return g != 0;
}

bool c3d_1x1_eligible(const nps_conv3d_t& a) {
    if (!a.bf16 || a.K != 1 || a.stride != 1 || a.transposed || a.circ != 0 || a.zpad != 0) return false;
    if (a.Cout > 128 || a.Cin > 256 || (a.Cout & 3) != 0 || (a.out_C & 3) != 0) return false;
    for (int i = 0; i < a.nsrc; ++i)
        if ((a.src[i].C & 3) != 0 || (i < a.nsrc - 1 && (a.src[i].C & 7) != 0)) return false;
    // (three-source frames, the up-path cat(h, skip, vb): measured slower than conv3d_kernel — 437 vs 360 us at
    // 132 -> 64 over 16 x 128^2, B = 8, double-buffered; 538 vs 363 single-buffered at 4 waves per SIMD; C5 -2 %,
    // profiles/r6/experiments/c5_1x1x1_three_source_ab.txt; two sources and GN-prologue frames gain)
    if (a.nsrc > 2) return false;
    return c3d_1x1_on();
}

template <int NCB, int NCH, bool PRO>
int launch_1x1(const nps_conv3d_t& a, int nchunk, hipStream_t s) {
    const size_t lds = (size_t)nchunk * NCB * 32 * 32 + NCB * 32 * sizeof(float) + 2 * (size_t)nchunk * 16 * sizeof(float) +
                       8 * sizeof(double);
    NPS_CHECK_ARG(lds <= 160 * 1024, "conv3d (1x1x1): %zu B of LDS", lds);
    const long nvox = (long)a.Dc * a.Hc * a.Wc;
    NPS_CHECK_ARG(nvox < (1L << 31) - 32, "conv3d (1x1x1): volume too large");
    const long ntv = (nvox + 31) / 32;
    // one round of resident work-groups (occupancy x CUs) over the whole grid, split over the samples; at most
    // one tile per wave
    static int ncu = 0;
    static int occ_by_chunks[NCH + 1] = {};  // resident work-groups per CU, per K-step count (the LDS it takes)
    if (ncu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    int& occ = occ_by_chunks[nchunk];
    if (occ == 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv3d_1x1_kernel<NCB, NCH, PRO>, 256, lds) !=
                         hipSuccess || occ <= 0))
        occ = 2;
    const long resident = (long)ncu * occ;
    long per = (resident + a.B - 1) / a.B;
    if (per > (ntv + 3) / 4) per = (ntv + 3) / 4;
    conv3d_1x1_kernel<NCB, NCH, PRO><<<dim3((unsigned)per, (unsigned)a.B), 256, lds, s>>>(a, nchunk);
    NPS_CHECK_LAUNCH("conv3d (1x1x1)");
    return 0;
}

template <bool PRO>
int dispatch_1x1(const nps_conv3d_t& a, int nchunk, hipStream_t s) {
    const bool w4 = a.Cout > 64;
    if (nchunk <= 5) return w4 ? launch_1x1<4, 5, PRO>(a, nchunk, s) : launch_1x1<2, 5, PRO>(a, nchunk, s);
    if (nchunk <= 9) return w4 ? launch_1x1<4, 9, PRO>(a, nchunk, s) : launch_1x1<2, 9, PRO>(a, nchunk, s);
    return w4 ? launch_1x1<4, 16, PRO>(a, nchunk, s) : launch_1x1<2, 16, PRO>(a, nchunk, s);
}

template <typename T, int K, int S, int TH, bool SIMPLE, bool O2 = false, bool GLT = false, bool SB = false,
          bool O4R = false>
int launch(const nps_conv3d_t& a, int nchunk, int ntile, hipStream_t s) {
    auto kern = conv3d_kernel<T, K, S, TH, SIMPLE, GLT, SB>;
    if constexpr (O4R) kern = conv3d_kernel_o4r<T, K, S, TH, SIMPLE>;
    if constexpr (O2 && SB) kern = conv3d_kernel_o4<T, K, S, TH, SIMPLE>;
    if constexpr (O2 && !SB) kern = conv3d_kernel_o2<T, K, S, TH, SIMPLE, GLT>;
    using G = Geo<K, S, TH>;
    const size_t lds = (SB ? 1 : 2) * (size_t)G::BUF * sizeof(T) + 2 * (size_t)nchunk * 16 * sizeof(float);
    NPS_CHECK_ARG(lds <= 160 * 1024, "conv3d: %zu B of LDS (Cin too large for the GroupNorm table)", lds);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)kern,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    const long ntiles = (long)a.B * a.Dout * ((a.Hout + TH - 1) / TH) * ((a.Wout + 31) / 32);
    NPS_CHECK_ARG(ntiles < (1L << 31), "conv3d: grid too large");
    const dim3 grid((unsigned)ntiles, (unsigned)ntile, a.transposed ? 8u : 1u);
    kern<<<grid, 256, lds, s>>>(a, nchunk, ntile);
    NPS_CHECK_LAUNCH("conv3d");
    return 0;
}

bool simple_frame(const nps_conv3d_t& a) {
    const nps_src3_t& s = a.src[0];
    return a.nsrc == 1 && s.off_d == 0 && s.off_h == 0 && s.off_w == 0 && s.D == a.Dc && s.H == a.Hc &&
           s.W == a.Wc && (a.Cin & 15) == 0 && a.gn_stats == nullptr && a.pre_act == 0;
}

template <typename T>
int dispatch(const nps_conv3d_t& a, int nchunk, int ntile, hipStream_t s) {
    const bool sim = simple_frame(a);
    // bf16 fast-path frames: stage copies by LDS-DMA into ONE stage buffer (SB) — three work-groups per CU (3x3x3),
    // four for the register-light 2x2x2 phases (held to 4 waves per SIMD); NPS_C3D_GLDS=0: the register-staged
    // double-buffered kernels.  Dev knob NPS_C3D_TH16 (3x3x3 stride 1, measured no faster, records in
    // profiles/r6/experiments/c5_conv3d_glds_ab.txt): 1 / 2 / 3 / 5 16-row tiles (2: two waves per SIMD, 3: LDS-DMA,
    // 5: both), 4 8-row LDS-DMA with two stage buffers, 7 the one-buffer kernel held to 4 waves per SIMD
    static int th16 = -1, glds = 1;
    if (th16 < 0) {
        const char* e = std::getenv("NPS_C3D_TH16");
        th16 = (e != nullptr && e[0] >= '1' && e[0] <= '7' && e[0] != '6') ? e[0] - '0' : 0;
        const char* g = std::getenv("NPS_C3D_GLDS");
        glds = (g != nullptr && g[0] == '0') ? 0 : 1;
    }
    if constexpr (sizeof(T) == 2)
        if (sim && glds) {
            if (a.K == 3 && a.stride == 1) {
                if (th16 == 1) return launch<T, 3, 1, 16, true>(a, nchunk, ntile, s);
                if (th16 == 2) return launch<T, 3, 1, 16, true, true>(a, nchunk, ntile, s);
                if (th16 == 3) return launch<T, 3, 1, 16, true, false, true>(a, nchunk, ntile, s);
                if (th16 == 4) return launch<T, 3, 1, 8, true, false, true>(a, nchunk, ntile, s);
                if (th16 == 5) return launch<T, 3, 1, 16, true, true, true>(a, nchunk, ntile, s);
                if (th16 == 7) return launch<T, 3, 1, 8, true, true, true, true>(a, nchunk, ntile, s);
                return launch<T, 3, 1, 8, true, false, true, true>(a, nchunk, ntile, s);
            }
            if (a.K == 3 && a.stride == 2) return launch<T, 3, 2, 4, true, false, true, true>(a, nchunk, ntile, s);
            if (a.K == 2 && a.stride == 1) return launch<T, 2, 1, 8, true, true, true, true>(a, nchunk, ntile, s);
        }
    if (a.K == 3 && a.stride == 1)
        return sim ? launch<T, 3, 1, 8, true>(a, nchunk, ntile, s) : launch<T, 3, 1, 8, false>(a, nchunk, ntile, s);
    if (a.K == 3 && a.stride == 2)
        return sim ? launch<T, 3, 2, 4, true>(a, nchunk, ntile, s) : launch<T, 3, 2, 4, false>(a, nchunk, ntile, s);
    if (a.K == 2 && a.stride == 1)
        return sim ? launch<T, 2, 1, 8, true>(a, nchunk, ntile, s) : launch<T, 2, 1, 8, false>(a, nchunk, ntile, s);
    if (a.K == 1 && a.stride == 1) {
        // bf16 multi-source 1x1x1 (the C5 shortcuts over cat(h, skip, vb)): a streaming kernel, held to four waves
        // per SIMD (four work-groups per CU, 128 VGPRs): (64, 64, 4) -> 64 at 16x128^2 471 -> 385 us, bit-identical
        // (profiles/r6/experiments/c5_conv3d_glds_ab.txt); NPS_C3D_K1O4=0: three work-groups
        static int k1 = -1;
        if (k1 < 0) {
            const char* e = std::getenv("NPS_C3D_K1O4");
            k1 = (e != nullptr && e[0] == '0') ? 0 : 1;
        }
        if constexpr (sizeof(T) == 2)
            if (!sim && k1) return launch<T, 1, 1, 8, false, false, false, false, true>(a, nchunk, ntile, s);
        return sim ? launch<T, 1, 1, 8, true>(a, nchunk, ntile, s) : launch<T, 1, 1, 8, false>(a, nchunk, ntile, s);
    }
    NPS_CHECK_ARG(false, "conv3d: K=%d stride=%d not supported (K in {1,2,3}, stride 2 only for K=3)", a.K, a.stride);
}

int check_frame(const nps_conv3d_t& a, const char* who) {
    NPS_CHECK_ARG(a.nsrc >= 1 && a.nsrc <= NPS_MAX_SRC && a.B > 0 && a.Dc > 0 && a.Hc > 0 && a.Wc > 0 && a.Cin > 0,
                  "%s: bad frame", who);
    int cs = 0;
    for (int i = 0; i < a.nsrc; ++i) {
        const nps_src3_t& s = a.src[i];
        NPS_CHECK_ARG(s.ptr != nullptr && s.C > 0 && s.D > 0 && s.H > 0 && s.W > 0, "%s: bad source %d", who, i);
        cs += s.C;
    }
    NPS_CHECK_ARG(cs == a.Cin, "%s: sources hold %d channels, frame Cin %d", who, cs, a.Cin);
    return 0;
}

}  // namespace

extern "C" size_t nps_conv3d_packed_bytes(int Cout, int Cin, int K, int transposed, int bf16) {
    if (Cout <= 0 || Cin <= 0 || K <= 0) return 0;
    const size_t nphase = transposed ? 8 : 1, nchunk = (Cin + 15) / 16, ntile = (Cout + 63) / 64;
    return nphase * ntile * K * nchunk * K * K * 64 * 16 * (bf16 ? 2 : 4);
}

extern "C" int nps_conv3d_pack_weights(const float* w, void* wpack, int Cout, int Cin, int K, int transposed, int bf16,
                                       void* stream) {
    NPS_CHECK_ARG(w && wpack && Cout > 0 && Cin > 0 && (K >= 1 && K <= 3) && (!transposed || K == 2),
                  "conv3d_pack_weights: bad args");
    const int nchunk = (Cin + 15) / 16, ntile = (Cout + 63) / 64;
    const long n = (long)(transposed ? 8 : 1) * ntile * K * nchunk * K * K * 64 * 16;
    const long nb = (n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192;
    hipStream_t s = (hipStream_t)stream;
    if (bf16)
        conv3d_pack_kernel<bf16_t><<<(unsigned)nb, 256, 0, s>>>(w, reinterpret_cast<bf16_t*>(wpack), Cout, Cin, K,
                                                                 transposed, nchunk, ntile, n);
    else
        conv3d_pack_kernel<float><<<(unsigned)nb, 256, 0, s>>>(w, reinterpret_cast<float*>(wpack), Cout, Cin, K,
                                                                transposed, nchunk, ntile, n);
    NPS_CHECK_LAUNCH("conv3d_pack_weights");
    return 0;
}

extern "C" int nps_conv3d_fwd(const nps_conv3d_t* ap, void* stream) {
    NPS_CHECK_ARG(ap != nullptr, "conv3d: null args");
    const nps_conv3d_t& a = *ap;
    if (check_frame(a, "conv3d") < 0) return -1;
    NPS_CHECK_ARG(a.wpack && a.out && a.Cout > 0 && a.out_C >= a.Cout && a.out_os >= 1 && a.out_D > 0 &&
                      a.out_H > 0 && a.out_W > 0 && a.circ >= 0 && a.zpad >= 0,
                  "conv3d: bad output / weight args");
    NPS_CHECK_ARG(!a.transposed || (a.K == 2 && a.stride == 1), "conv3d: transposed = 8 phases of K=2, stride 1");
    NPS_CHECK_ARG(a.circ <= a.Dc && a.circ <= a.Hc && a.circ <= a.Wc, "conv3d: circular extension beyond the frame");
    const int ext = 2 * (a.circ + a.zpad);
    NPS_CHECK_ARG(a.Dout == (a.Dc + ext - a.K) / a.stride + 1 && a.Hout == (a.Hc + ext - a.K) / a.stride + 1 &&
                      a.Wout == (a.Wc + ext - a.K) / a.stride + 1 && a.Dout > 0 && a.Hout > 0 && a.Wout > 0,
                  "conv3d: output extent %dx%dx%d does not match the frame", a.Dout, a.Hout, a.Wout);
    NPS_CHECK_ARG(a.gn_stats == nullptr || (a.gn_gamma && a.gn_beta && a.gn_groups >= 1 && a.gn_groups <= 8 &&
                                            a.Cin % a.gn_groups == 0),
                  "conv3d: bad GroupNorm prologue");
    NPS_CHECK_ARG(a.pre_act == 0 || a.pre_act == 1, "conv3d: pre_act 0 or 1");
    // (out_stats: moments of the values stored, after addend / act — of the change under accumulate; the 8 phases
    // of a transposed conv write disjoint elements)
    const int nchunk = (a.Cin + 15) / 16, ntile = (a.Cout + 63) / 64;
    hipStream_t s = (hipStream_t)stream;
    if (c3d_1x1_eligible(a))
        return (a.gn_stats != nullptr || a.pre_act != 0) ? dispatch_1x1<true>(a, nchunk, s)
                                                         : dispatch_1x1<false>(a, nchunk, s);
    return a.bf16 ? dispatch<bf16_t>(a, nchunk, ntile, s) : dispatch<float>(a, nchunk, ntile, s);
}

extern "C" int nps_frame_pack3d(const nps_conv3d_t* ap, void* out, int Cpad, void* stream) {
    NPS_CHECK_ARG(ap != nullptr && out != nullptr, "frame_pack3d: null args");
    const nps_conv3d_t& a = *ap;
    if (check_frame(a, "frame_pack3d") < 0) return -1;
    NPS_CHECK_ARG(Cpad >= a.Cin && Cpad % 8 == 0 && Cpad <= 512, "frame_pack3d: Cpad %d (>= Cin, %% 8, <= 512)", Cpad);
    NPS_CHECK_ARG(a.gn_stats == nullptr || (a.gn_gamma && a.gn_beta && a.gn_groups >= 1 && a.Cin % a.gn_groups == 0),
                  "frame_pack3d: bad GroupNorm prologue");
    const long nitem = (long)a.Dc * a.Hc * a.Wc * (Cpad / 8);
    NPS_CHECK_ARG(nitem < (1L << 31), "frame_pack3d: frame too large");
    const long nb = (nitem + 2047) / 2048 < 1024 ? (nitem + 2047) / 2048 : 1024;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)(nb > 0 ? nb : 1), (unsigned)a.B);
    static int mflat_off = -1;  // dev knob NPS_PACK3D_MFLAT=0: multi-source frames through the general decode
    static int flat_on = 1;     // NPS_PACK3D_FLAT=0: offset-0 frames on frame_pack3d_kernel instead of the flat kernel
    if (mflat_off < 0) {
        const char* e = std::getenv("NPS_PACK3D_MFLAT");
        mflat_off = (e != nullptr && e[0] == '0') ? 1 : 0;
        const char* f = std::getenv("NPS_PACK3D_FLAT");
        flat_on = (f != nullptr && f[0] == '0') ? 0 : 1;
    }
    bool flat = flat_on && mflat_off == 0;
    for (int i = 0; i < a.nsrc; ++i) {
        const nps_src3_t& q = a.src[i];
        flat = flat && q.off_d == 0 && q.off_h == 0 && q.off_w == 0 && q.D == a.Dc && q.H == a.Hc && q.W == a.Wc &&
               (q.C & 3) == 0;
    }
    if (flat && Cpad / 8 <= 64) {
        const long nvox = (long)a.Dc * a.Hc * a.Wc, vpb = 256 / (Cpad / 8);
        const long nbv = (nvox + vpb * 8 - 1) / (vpb * 8) < 1024 ? (nvox + vpb * 8 - 1) / (vpb * 8) : 1024;
        const dim3 fgrid((unsigned)(nbv > 0 ? nbv : 1), (unsigned)a.B);
        if (a.bf16)
            frame_pack3d_flat_kernel<bf16_t><<<fgrid, 256, 0, s>>>(a, reinterpret_cast<bf16_t*>(out), Cpad);
        else
            frame_pack3d_flat_kernel<float><<<fgrid, 256, 0, s>>>(a, reinterpret_cast<float*>(out), Cpad);
        NPS_CHECK_LAUNCH("frame_pack3d");
        return 0;
    }
    if (a.bf16)
        frame_pack3d_kernel<bf16_t><<<grid, 256, 0, s>>>(a, reinterpret_cast<bf16_t*>(out), Cpad, mflat_off != 0);
    else
        frame_pack3d_kernel<float><<<grid, 256, 0, s>>>(a, reinterpret_cast<float*>(out), Cpad, mflat_off != 0);
    NPS_CHECK_LAUNCH("frame_pack3d");
    return 0;
}

extern "C" int nps_gn_stats3d(const nps_conv3d_t* ap, int G, double* stats, void* stream) {
    NPS_CHECK_ARG(ap != nullptr && stats != nullptr, "gn_stats3d: null args");
    const nps_conv3d_t& a = *ap;
    if (check_frame(a, "gn_stats3d") < 0) return -1;
    NPS_CHECK_ARG(G >= 1 && G <= 8 && a.Cin % G == 0, "gn_stats3d: groups %d must divide Cin %d (<= 8)", G, a.Cin);
    long nitem = 0;
    for (int i = 0; i < a.nsrc; ++i) nitem += (long)a.src[i].D * a.src[i].H * a.src[i].W * ((a.src[i].C + 7) / 8);
    NPS_CHECK_ARG(nitem < (1L << 31), "gn_stats3d: frame too large");
    nitem = nitem > 0 ? nitem : 1;  // items per sample (grid.y = sample)
    const long nb = (nitem + 2047) / 2048 < 512 ? (nitem + 2047) / 2048 : 512;
    hipStream_t s = (hipStream_t)stream;
    if (a.bf16)
        gn_stats3d_kernel<bf16_t><<<dim3((unsigned)nb, (unsigned)a.B), 256, 0, s>>>(a, G, stats);
    else
        gn_stats3d_kernel<float><<<dim3((unsigned)nb, (unsigned)a.B), 256, 0, s>>>(a, G, stats);
    NPS_CHECK_LAUNCH("gn_stats3d");
    return 0;
}
