// SpectralConv3d (proc_fno.py:291-376) for gfx950: weight packing and gradient unpacking for the four
// retained corners.  The transform itself is the 2-D pipeline of spectral.hip applied per axis on
// NDHWC activations (see nps_hip.ops.spectral_conv3d):
//   W: nps_spectral_dft_w over (B, D*H, W)            -> X1 [B][D*H][m3][C]
//   H: nps_spectral_dft_h over (B*D, H), m2 := m3     -> X2 [B*D][R2][m3][C]
//   D: nps_spectral_dft_h over (B, D),  m2 := R2*m3   -> X3 [B][R1][R2*m3][C]
//   mix with wpack[R1][R2][m3][Cin][Cout], then the inverse chain, c2r over W with 1/(D*H*W).
// Retained rows per axis: R1 = min(D, 2*m1), R2 = min(H, 2*m2) (rows [:m] and [-m:]).
#include "nps_common.hpp"

namespace {

__device__ __forceinline__ int row_k(int r, int N, int R, int m) { return r < m ? r : N - R + r; }
__device__ __forceinline__ int k_row(int k, int N, int R, int m) { return k < m ? k : k - (N - R); }

// Corner that owns frequency (k1, k2): the reference writes out_ft corners in the order
// w1 [:m1, :m2], w2 [-m1:, :m2], w3 [:m1, -m2:], w4 [-m1:, -m2:] (proc_fno.py:342-350), so where
// corners overlap the later one wins.  Returns 1..4.
__device__ __forceinline__ int owner(int k1, int k2, int D, int H, int m1, int m2) {
    const bool a1 = k1 < m1, b1 = k1 >= D - m1, a2 = k2 < m2, b2 = k2 >= H - m2;
    if (b1 && b2) return 4;
    if (a1 && b2) return 3;
    if (b1 && a2) return 2;
    return 1;
}

// wpack[r1][r2][k3][i][o] (complex64) from weights1..4 [Cin][Cout][m1][m2][m3]
__global__ void spec3_pack_kernel(const float2* __restrict__ w1, const float2* __restrict__ w2,
                                  const float2* __restrict__ w3, const float2* __restrict__ w4, float2* __restrict__ wp,
                                  int Cin, int Cout, int D, int H, int R1, int R2, int m1, int m2, int m3) {
    const size_t n = (size_t)R1 * R2 * m3 * Cin * Cout;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int o = i % Cout;
    size_t t = i / Cout;
    const int ci = t % Cin;
    t /= Cin;
    const int k3 = t % m3;
    t /= m3;
    const int r2 = t % R2;
    const int r1 = (int)(t / R2);
    const int k1 = row_k(r1, D, R1, m1), k2 = row_k(r2, H, R2, m2);
    const int c = owner(k1, k2, D, H, m1, m2);
    const int j1 = (c == 1 || c == 3) ? k1 : k1 - (D - m1);
    const int j2 = (c == 1 || c == 2) ? k2 : k2 - (H - m2);
    const float2* w = c == 1 ? w1 : (c == 2 ? w2 : (c == 3 ? w3 : w4));
    wp[i] = w[((((size_t)ci * Cout + o) * m1 + j1) * m2 + j2) * m3 + k3];
}

// gw_c[i][o][j1][j2][k3] = gwpack at the mode (j1, j2, k3) of corner c maps to, where corner c owns it;
// 0 where a later corner overwrote that position in the reference (its output never saw w_c there).
__global__ void spec3_unpack_grad_kernel(const float2* __restrict__ gwp, float2* __restrict__ gw1,
                                         float2* __restrict__ gw2, float2* __restrict__ gw3, float2* __restrict__ gw4,
                                         int Cin, int Cout, int D, int H, int R1, int R2, int m1, int m2, int m3) {
    const size_t n = (size_t)Cin * Cout * m1 * m2 * m3;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int k3 = idx % m3;
    size_t t = idx / m3;
    const int j2 = t % m2;
    t /= m2;
    const int j1 = t % m1;
    t /= m1;
    const int o = t % Cout;
    const int ci = (int)(t / Cout);
    float2* gw[4] = {gw1, gw2, gw3, gw4};
#pragma unroll
    for (int c = 1; c <= 4; ++c) {
        const int k1 = (c == 1 || c == 3) ? j1 : D - m1 + j1;
        const int k2 = (c == 1 || c == 2) ? j2 : H - m2 + j2;
        float2 g = make_float2(0.f, 0.f);
        if (owner(k1, k2, D, H, m1, m2) == c) {
            const int r1 = k_row(k1, D, R1, m1), r2 = k_row(k2, H, R2, m2);
            g = gwp[((((size_t)r1 * R2 + r2) * m3 + k3) * Cin + ci) * Cout + o];
        }
        gw[c - 1][idx] = g;
    }
}

}  // namespace

extern "C" int nps_spectral3d_pack_weights(const float* w1, const float* w2, const float* w3, const float* w4,
                                           float* wpack, int Cin, int Cout, int D, int H, int m1, int m2, int m3,
                                           void* stream) {
    NPS_CHECK_ARG(w1 && w2 && w3 && w4 && wpack && Cin > 0 && Cout > 0 && m1 > 0 && m1 <= D && m2 > 0 && m2 <= H &&
                      m3 > 0,
                  "spectral3d_pack_weights: bad args");
    const int R1 = D < 2 * m1 ? D : 2 * m1, R2 = H < 2 * m2 ? H : 2 * m2;
    const size_t n = (size_t)R1 * R2 * m3 * Cin * Cout;
    spec3_pack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        reinterpret_cast<const float2*>(w1), reinterpret_cast<const float2*>(w2), reinterpret_cast<const float2*>(w3),
        reinterpret_cast<const float2*>(w4), reinterpret_cast<float2*>(wpack), Cin, Cout, D, H, R1, R2, m1, m2, m3);
    NPS_CHECK_LAUNCH("spectral3d_pack_weights");
    return 0;
}

extern "C" int nps_spectral3d_unpack_grad(const float* gwpack, float* gw1, float* gw2, float* gw3, float* gw4, int Cin,
                                          int Cout, int D, int H, int m1, int m2, int m3, void* stream) {
    NPS_CHECK_ARG(gwpack && gw1 && gw2 && gw3 && gw4 && Cin > 0 && Cout > 0 && m1 > 0 && m1 <= D && m2 > 0 &&
                      m2 <= H && m3 > 0,
                  "spectral3d_unpack_grad: bad args");
    const int R1 = D < 2 * m1 ? D : 2 * m1, R2 = H < 2 * m2 ? H : 2 * m2;
    const size_t n = (size_t)Cin * Cout * m1 * m2 * m3;
    spec3_unpack_grad_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        reinterpret_cast<const float2*>(gwpack), reinterpret_cast<float2*>(gw1), reinterpret_cast<float2*>(gw2),
        reinterpret_cast<float2*>(gw3), reinterpret_cast<float2*>(gw4), Cin, Cout, D, H, R1, R2, m1, m2, m3);
    NPS_CHECK_LAUNCH("spectral3d_unpack_grad");
    return 0;
}
