// bf16-storage kernels of the 3-D FNO path (BASELINE config C5: "3D rFFT spectral conv, bf16"): dtype
// conversion and the pointwise (kernel-1) Conv3d `w` of FNO_Layer (proc_fno.py:104-107, :142-146) as a bf16
// MFMA GEMM with fp32 accumulation.  The spectral passes' bf16 variants live in spectral.hip.
#include "nps_common.hpp"

namespace {

typedef unsigned short bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16_t f2bf(float v) { return __builtin_bit_cast(bf16_t, (__bf16)v); }
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float((unsigned)v << 16); }

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = f2bf(x[i]);
}
__global__ void bf16_to_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = bf2f(x[i]);
}

// w[Cout][Cin] (fp32, kernel 1) -> wp[Cout][KR] bf16 with KR = Cin rounded up to 16, + 8 (LDS rows 16 B off
// a multiple of 32 B: conflict-free ds_read_b128 of the A fragments), zeros past Cin
__global__ void pack_1x1_bf16_kernel(const float* __restrict__ w, bf16_t* __restrict__ wp, int Cout, int Cin, int KR) {
    const long n = (long)Cout * KR;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int co = (int)(i / KR), k = (int)(i - (long)co * KR);
        wp[i] = k < Cin ? f2bf(w[(size_t)co * Cin + k]) : (bf16_t)0;
    }
}

// out[px][co] = act(sum_k w[co][k] x[px][k] + bias[co] (+ addend[px][co])), bf16 in / out, fp32 accumulate, on
// v_mfma_f32_32x32x16_bf16.  Work-group = 128 pixels (4 waves x 32) x all Cout (NCB 32-channel blocks, one
// 32x32 accumulator each); the packed weight sits in LDS, the B fragment (8 channels of one pixel per lane)
// is one 16-B load from the NHWC source.  Sources cover the frame (offset 0); the channel runs of 8 a lane
// loads lie in one source (every source but the last has C % 8 == 0; host-checked), the last source's tail
// is read element-wise and zero-filled.
template <int NCB>
__global__ __launch_bounds__(256) void conv1x1_bf16_kernel(const nps_conv2d_t a, int KR) {
    extern __shared__ __attribute__((aligned(16))) bf16_t wl[];  // [NCB*32][KR]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.y;
    const int npx = a.Hout * a.Wout;
    const int P = blockIdx.x * 128 + wave * 32 + (lane & 31);
    const int h = lane >> 5;
    const bf16_t* wg = reinterpret_cast<const bf16_t*>(a.wpack);
    const int nco = NCB * 32;
    for (int i = tid; i < nco * KR / 8; i += 256) {  // 16-B pieces; rows past Cout are zero
        const int co = (i * 8) / KR;
        const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        reinterpret_cast<u16x8*>(wl)[i] = co < a.Cout ? reinterpret_cast<const u16x8*>(wg)[i] : z;
    }
    __syncthreads();
    f32x16 acc[NCB];
#pragma unroll
    for (int i = 0; i < NCB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const bool pin = P < npx;
    const int nsteps = (a.Cin + 15) / 16;
    for (int s = 0; s < nsteps; ++s) {
        const int c = 16 * s + 8 * h;  // this lane's 8-channel run
        u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        int lo = 0;
#pragma unroll
        for (int si = 0; si < NPS_MAX_SRC; ++si) {
            if (si < a.nsrc) {
                const int sC = a.src[si].C;
                if (pin && c >= lo && c < lo + sC) {
                    const bf16_t* px =
                        reinterpret_cast<const bf16_t*>(a.src[si].ptr) + ((size_t)b * npx + P) * sC + (c - lo);
                    if (c - lo + 8 <= sC) {
                        v = *reinterpret_cast<const u16x8*>(px);
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] = (c - lo + e < sC) ? px[e] : (bf16_t)0;
                    }
                }
                lo += sC;
            }
        }
        const bf16x8 bv = __builtin_bit_cast(bf16x8, v);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
            const bf16x8 av =
                *reinterpret_cast<const bf16x8*>(wl + (size_t)(cb * 32 + (lane & 31)) * KR + 16 * s + 8 * h);
            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[cb], 0, 0, 0);
        }
    }
    if (!pin) return;
    // D: column = pixel P (lane & 31), rows co = cb*32 + 8g + 4h + e (g = reg >> 2, e = reg & 3)
    bf16_t* out = reinterpret_cast<bf16_t*>(a.out) + ((size_t)b * npx + P) * a.out_C;
    const bf16_t* add =
        a.addend0 ? reinterpret_cast<const bf16_t*>(a.addend0) + ((size_t)b * npx + P) * a.out_C : nullptr;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int co0 = cb * 32 + 8 * g + 4 * h;
            if (co0 >= a.Cout) continue;
            u16x4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = acc[cb][4 * g + e];
                if (a.bias) v += a.bias[co0 + e];
                if (add) v += bf2f(add[co0 + e]);
                if (a.act == 1) v = nps::gelu_erf(v);
                r[e] = f2bf(v);
            }
            *reinterpret_cast<u16x4*>(out + co0) = r;
        }
    }
}

}  // namespace

extern "C" int nps_f32_to_bf16(const float* x, long n, void* y, void* stream) {
    NPS_CHECK_ARG(x && y && n > 0, "f32_to_bf16: bad args");
    const long nb = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
    f32_to_bf16_kernel<<<(unsigned)nb, 256, 0, (hipStream_t)stream>>>(x, reinterpret_cast<bf16_t*>(y), n);
    NPS_CHECK_LAUNCH("f32_to_bf16");
    return 0;
}

extern "C" int nps_bf16_to_f32(const void* x, long n, float* y, void* stream) {
    NPS_CHECK_ARG(x && y && n > 0, "bf16_to_f32: bad args");
    const long nb = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
    bf16_to_f32_kernel<<<(unsigned)nb, 256, 0, (hipStream_t)stream>>>(reinterpret_cast<const bf16_t*>(x), y, n);
    NPS_CHECK_LAUNCH("bf16_to_f32");
    return 0;
}

extern "C" int nps_conv1x1_bf16_kr(int Cin) { return (Cin + 15) / 16 * 16 + 8; }

extern "C" int nps_pack_1x1_bf16(const float* w, void* wp, int Cout, int Cin, void* stream) {
    NPS_CHECK_ARG(w && wp && Cout > 0 && Cin > 0, "pack_1x1_bf16: bad args");
    const int KR = nps_conv1x1_bf16_kr(Cin);
    const long n = (long)Cout * KR;
    const long nb = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
    pack_1x1_bf16_kernel<<<(unsigned)nb, 256, 0, (hipStream_t)stream>>>(w, reinterpret_cast<bf16_t*>(wp), Cout, Cin,
                                                                         KR);
    NPS_CHECK_LAUNCH("pack_1x1_bf16");
    return 0;
}

extern "C" int nps_conv1x1_bf16(const nps_conv2d_t* ap, void* stream) {
    NPS_CHECK_ARG(ap != nullptr, "conv1x1_bf16: null args");
    const nps_conv2d_t& a = *ap;
    NPS_CHECK_ARG(a.nsrc >= 1 && a.nsrc <= NPS_MAX_SRC && a.B > 0 && a.Cout > 0 && a.Cout <= 256 && a.wpack && a.out,
                  "conv1x1_bf16: bad args (Cout <= 256)");
    int cs = 0;
    for (int s = 0; s < a.nsrc; ++s) {
        NPS_CHECK_ARG(a.src[s].ptr && a.src[s].H == a.Hout && a.src[s].W == a.Wout && a.src[s].off_y == 0 &&
                          a.src[s].off_x == 0,
                      "conv1x1_bf16: sources must cover the frame");
        NPS_CHECK_ARG(s == a.nsrc - 1 || a.src[s].C % 8 == 0, "conv1x1_bf16: source %d C %% 8 != 0", s);
        cs += a.src[s].C;
    }
    NPS_CHECK_ARG(cs == a.Cin && a.Hin == a.Hout && a.Win == a.Wout && a.out_C == a.Cout && !a.out_nchw &&
                      a.out_os == 1 && !a.accumulate && (a.Cout & 3) == 0,
                  "conv1x1_bf16: unsupported layout");
    const int KR = nps_conv1x1_bf16_kr(a.Cin);
    const int ncb = (a.Cout + 31) / 32;
    const int npx = a.Hout * a.Wout;
    const dim3 grid((unsigned)((npx + 127) / 128), (unsigned)a.B);
    const size_t lds = (size_t)ncb * 32 * KR * 2;
    NPS_CHECK_ARG(lds <= 64 * 1024, "conv1x1_bf16: weights %zu B too large for LDS", lds);
    hipStream_t s = (hipStream_t)stream;
    switch (ncb) {
        case 1: conv1x1_bf16_kernel<1><<<grid, 256, lds, s>>>(a, KR); break;
        case 2: conv1x1_bf16_kernel<2><<<grid, 256, lds, s>>>(a, KR); break;
        case 3: conv1x1_bf16_kernel<3><<<grid, 256, lds, s>>>(a, KR); break;
        case 4: conv1x1_bf16_kernel<4><<<grid, 256, lds, s>>>(a, KR); break;
        case 6: conv1x1_bf16_kernel<6><<<grid, 256, lds, s>>>(a, KR); break;
        case 8: conv1x1_bf16_kernel<8><<<grid, 256, lds, s>>>(a, KR); break;
        default: NPS_CHECK_ARG(false, "conv1x1_bf16: Cout %d not in {32..128, 192, 256}", a.Cout);
    }
    NPS_CHECK_LAUNCH("conv1x1_bf16");
    return 0;
}
