// Composite C-ABI of the spectral convolutions (include/nps.h "one call per module"): SpectralConv2d and
// SpectralConv3d forward / backward (proc_fno.py:257-288, :334-376) and the 2-D FNO layer act(conv(x) + w(x))
// (proc_fno.py:142-146), each sequencing the stage kernels of spectral.hip / spectral3d.hip on the caller's
// stream inside a caller-provided workspace.  A C caller binding libnps_hip.so needs nothing else: the weights
// are the modules' own nn.Parameters (complex64, reference layout), packed into the workspace per call.
// Host code only; every launch is stream-ordered, nothing synchronises or allocates.
#include "nps_common.hpp"

namespace {

constexpr size_t C64 = 8;  // bytes per complex64

size_t al256(size_t n) { return (n + 255) & ~size_t(255); }

// Carves 256-B aligned regions out of the workspace in a fixed order (the same order the size functions sum).
struct Carve {
    char* base;
    size_t off = 0;
    float* take(size_t bytes) {
        float* p = reinterpret_cast<float*>(base + off);
        off += al256(bytes);
        return p;
    }
};

struct Spec2 {
    size_t wp, x1, x2, y, z;  // bytes of wpack [R][m2][Cin][Cout], X1 [B][H][m2][Cin], X2 [B][R][m2][Cin],
                              // Y [B][R][m2][Cout], Z [B][H][m2][Cout]
};
Spec2 spec2_sizes(int B, int Cin, int Cout, int H, int m1, int m2) {
    const size_t R = (size_t)(H < 2 * m1 ? H : 2 * m1);
    Spec2 s;
    s.wp = R * m2 * Cin * Cout * C64;
    s.x1 = (size_t)B * H * m2 * Cin * C64;
    s.x2 = (size_t)B * R * m2 * Cin * C64;
    s.y = (size_t)B * R * m2 * Cout * C64;
    s.z = (size_t)B * H * m2 * Cout * C64;
    return s;
}
// forward: [wp][X1][X2][Y][Z]; backward adds [gX2][gwp] (X1 -> gX1, Y -> gY, Z -> gZ reuse their regions)
size_t spec2_ws(int B, int Cin, int Cout, int H, int m1, int m2) {
    const Spec2 s = spec2_sizes(B, Cin, Cout, H, m1, m2);
    return al256(s.wp) + al256(s.x1) + al256(s.x2) + al256(s.y) + al256(s.z) + al256(s.x2) + al256(s.wp);
}

bool spec2_args_ok(int B, int Cin, int Cout, int H, int W, int m1, int m2) {
    // proc_fno.py:134-139: modes at most the spatial dims (W // 2 + 1 for the last)
    return B > 0 && Cin > 0 && Cout > 0 && H > 0 && W > 0 && m1 > 0 && m2 > 0 && m1 <= H && m2 <= W / 2 + 1;
}

// Z = the spectral conv up to its W-pass synthesis, for the frame `src` (nsrc sources covering B x H x W x Cin)
int spec2_z(const nps_src_t* src, int nsrc, const float* w1, const float* w2, Carve& c, const Spec2& sz, int B,
            int Cin, int Cout, int H, int W, int m1, int m2, float** Zout, float** X2out, float** wpout, void* s) {
    const int R = H < 2 * m1 ? H : 2 * m1;
    float* wp = c.take(sz.wp);
    float* X1 = c.take(sz.x1);
    float* X2 = c.take(sz.x2);
    float* Y = c.take(sz.y);
    float* Z = c.take(sz.z);
    int rc;
    if ((rc = nps_spectral_pack_weights(w1, w2, wp, Cin, Cout, H, m1, m2, s)) < 0) return rc;
    if ((rc = nps_spectral_dft_w(src, nsrc, B, H, W, Cin, m2, X1, s)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(X1, X2, B, H, m1, m2, Cin, s)) < 0) return rc;
    if ((rc = nps_spectral_mix(X2, wp, Y, B, R, m2, Cin, Cout, s)) < 0) return rc;
    if ((rc = nps_spectral_idft_h(Y, Z, B, H, m1, m2, Cout, s)) < 0) return rc;
    *Zout = Z;
    if (X2out) *X2out = X2;
    if (wpout) *wpout = wp;
    return 0;
}

// the fused-synthesis conditions of nps_conv2d_fwd's spec_z (conv2d.hip), as a predicate
bool fno_fusable(const nps_conv2d_t& a, int m2) {
    return a.precision == NPS_PREC_X3F16 && a.KH == 1 && a.KW == 1 && a.stride == 1 && a.dil == 1 && a.Cout <= 192 &&
           !a.gn_stats && !a.pre_act && !a.accumulate && !a.addend0 && !a.addend1 && !a.out_nchw &&
           (a.out_C & 3) == 0 && (a.Cout & 3) == 0 && m2 > 0 && m2 <= 16 && (a.Wout & 127) == 0 && a.pad_y == 0 &&
           a.pad_x == 0 && a.circ == 0 && a.out_os == 1 && a.out_off_y == 0 && a.out_off_x == 0 &&
           a.out_H == a.Hout && a.out_W == a.Wout && a.nphase <= 1 && !a.s2d;
}

struct Spec3 {
    size_t wp, x1, x2, x3, y, z1, z2;
};
Spec3 spec3_sizes(int B, int Cin, int Cout, int D, int H, int m1, int m2, int m3) {
    const size_t R1 = (size_t)(D < 2 * m1 ? D : 2 * m1), R2 = (size_t)(H < 2 * m2 ? H : 2 * m2);
    Spec3 s;
    s.wp = R1 * R2 * m3 * Cin * Cout * C64;
    s.x1 = (size_t)B * D * H * m3 * Cin * C64;   // X1 [B][D*H][m3][Cin]
    s.x2 = (size_t)B * D * R2 * m3 * Cin * C64;  // X2 [B*D][R2][m3][Cin]
    s.x3 = (size_t)B * R1 * R2 * m3 * Cin * C64; // X3 [B][R1][R2*m3][Cin]
    s.y = (size_t)B * R1 * R2 * m3 * Cout * C64; // Y  [B][R1][R2*m3][Cout]
    s.z1 = (size_t)B * D * R2 * m3 * Cout * C64; // Z1 [B][D][R2*m3][Cout]
    s.z2 = (size_t)B * D * H * m3 * Cout * C64;  // Z2 [B*D][H][m3][Cout]
    return s;
}
// forward: [wp][X1][X2][X3][Y][Z1][Z2]; backward adds [gX3][gwp] (X2 -> gX2, X1 -> gX1, Y -> gY, Z1 -> gZ1,
// Z2 -> gZ2)
size_t spec3_ws(int B, int Cin, int Cout, int D, int H, int m1, int m2, int m3) {
    const Spec3 s = spec3_sizes(B, Cin, Cout, D, H, m1, m2, m3);
    return al256(s.wp) + al256(s.x1) + al256(s.x2) + al256(s.x3) + al256(s.y) + al256(s.z1) + al256(s.z2) +
           al256(s.x3) + al256(s.wp);
}
bool spec3_args_ok(int B, int Cin, int Cout, int D, int H, int W, int m1, int m2, int m3) {
    return B > 0 && Cin > 0 && Cout > 0 && D > 0 && H > 0 && W > 0 && m1 > 0 && m2 > 0 && m3 > 0 && m1 <= D &&
           m2 <= H && m3 <= W / 2 + 1;
}

}  // namespace

extern "C" size_t nps_spectral_conv2d_workspace(int B, int Cin, int Cout, int H, int W, int m1, int m2) {
    if (!spec2_args_ok(B, Cin, Cout, H, W, m1, m2)) return 0;
    return spec2_ws(B, Cin, Cout, H, m1, m2);
}

extern "C" int nps_spectral_conv2d_fwd(const float* x, const float* w1, const float* w2, float* y, void* ws, int B,
                                       int Cin, int Cout, int H, int W, int m1, int m2, int accumulate, int act,
                                       void* stream) {
    NPS_CHECK_ARG(x && w1 && w2 && y && ws, "spectral_conv2d_fwd: NULL pointer");
    NPS_CHECK_ARG(spec2_args_ok(B, Cin, Cout, H, W, m1, m2),
                  "spectral_conv2d_fwd: modes should be at most the spatial dim (// 2 + 1 for the last spatial "
                  "dimension) (H=%d W=%d m1=%d m2=%d)", H, W, m1, m2);
    NPS_CHECK_ARG(act == 0 || act == 1, "spectral_conv2d_fwd: act is 0 (none) or 1 (GELU)");
    const nps_src_t src = {x, Cin, H, W, 0, 0};
    Carve c{static_cast<char*>(ws)};
    const Spec2 sz = spec2_sizes(B, Cin, Cout, H, m1, m2);
    float* Z = nullptr;
    int rc = spec2_z(&src, 1, w1, w2, c, sz, B, Cin, Cout, H, W, m1, m2, &Z, nullptr, nullptr, stream);
    if (rc < 0) return rc;
    return nps_spectral_idft_w(Z, y, B, H, W, m2, Cout, accumulate ? 1 : 0, nullptr, act, nullptr, stream);
}

extern "C" int nps_spectral_conv2d_bwd(const float* x, const float* w1, const float* w2, const float* dy, float* dx,
                                       float* dw1, float* dw2, void* ws, int B, int Cin, int Cout, int H, int W,
                                       int m1, int m2, void* stream) {
    NPS_CHECK_ARG(x && w1 && w2 && dy && ws, "spectral_conv2d_bwd: NULL pointer");
    NPS_CHECK_ARG((dw1 == nullptr) == (dw2 == nullptr), "spectral_conv2d_bwd: dw1 and dw2 are both given or both NULL");
    NPS_CHECK_ARG(spec2_args_ok(B, Cin, Cout, H, W, m1, m2), "spectral_conv2d_bwd: bad shape (H=%d W=%d m1=%d m2=%d)",
                  H, W, m1, m2);
    const int R = H < 2 * m1 ? H : 2 * m1;
    const Spec2 sz = spec2_sizes(B, Cin, Cout, H, m1, m2);
    Carve c{static_cast<char*>(ws)};
    float* wp = c.take(sz.wp);
    float* X1 = c.take(sz.x1);  // later gX1
    float* X2 = c.take(sz.x2);
    float* gY = c.take(sz.y);
    float* gZ = c.take(sz.z);
    float* gX2 = c.take(sz.x2);
    float* gwp = c.take(sz.wp);
    const nps_src_t src = {x, Cin, H, W, 0, 0};
    int rc;
    // the forward's retained spectrum X2 (mix_bwd's conj(X2) for the weight gradient) and the packed weight
    if ((rc = nps_spectral_pack_weights(w1, w2, wp, Cin, Cout, H, m1, m2, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_w(&src, 1, B, H, W, Cin, m2, X1, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(X1, X2, B, H, m1, m2, Cin, stream)) < 0) return rc;
    // adjoint chain: irfft2's adjoint, the H pass, the mixing's two adjoint products
    if ((rc = nps_spectral_idft_w_bwd(dy, gZ, B, H, W, m2, Cout, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(gZ, gY, B, H, m1, m2, Cout, stream)) < 0) return rc;
    if ((rc = nps_spectral_mix_bwd(X2, wp, gY, gX2, gwp, B, R, m2, Cin, Cout, stream)) < 0) return rc;
    if (dx != nullptr) {
        if ((rc = nps_spectral_idft_h(gX2, X1, B, H, m1, m2, Cin, stream)) < 0) return rc;
        if ((rc = nps_spectral_dft_w_bwd(X1, dx, B, H, W, m2, Cin, stream)) < 0) return rc;
    }
    if (dw1 != nullptr)
        if ((rc = nps_spectral_unpack_grad(gwp, dw1, dw2, Cin, Cout, H, m1, m2, stream)) < 0) return rc;
    return 0;
}

extern "C" size_t nps_fno_layer2d_workspace(int B, int Cin, int Cout, int H, int W, int m1, int m2) {
    return nps_spectral_conv2d_workspace(B, Cin, Cout, H, W, m1, m2);
}

extern "C" int nps_fno_layer2d_fwd(const nps_conv2d_t* w, const float* w1, const float* w2, int m1, int m2, void* ws,
                                   void* stream) {
    NPS_CHECK_ARG(w && w1 && w2 && ws, "fno_layer2d_fwd: NULL pointer");
    const nps_conv2d_t& a = *w;
    NPS_CHECK_ARG(a.KH == 1 && a.KW == 1 && a.stride == 1 && a.dil == 1 && a.Hout == a.Hin && a.Wout == a.Win &&
                      a.spec_z == nullptr && !a.accumulate,
                  "fno_layer2d_fwd: w is the layer's 1x1 conv over the whole frame (no accumulate, spec_z unset)");
    NPS_CHECK_ARG(a.act == 0 || a.act == 1, "fno_layer2d_fwd: act is 0 (none) or 1 (GELU)");
    const int B = a.B, Cin = a.Cin, Cout = a.Cout, H = a.Hin, W = a.Win;
    NPS_CHECK_ARG(spec2_args_ok(B, Cin, Cout, H, W, m1, m2), "fno_layer2d_fwd: bad modes (H=%d W=%d m1=%d m2=%d)", H,
                  W, m1, m2);
    Carve c{static_cast<char*>(ws)};
    const Spec2 sz = spec2_sizes(B, Cin, Cout, H, m1, m2);
    float* Z = nullptr;
    int rc = spec2_z(a.src, a.nsrc, w1, w2, c, sz, B, Cin, Cout, H, W, m1, m2, &Z, nullptr, nullptr, stream);
    if (rc < 0) return rc;
    nps_conv2d_t f = a;
    if (fno_fusable(a, m2)) {
        // one output pass: the 1x1's epilogue synthesises the c2r W pass (1 / (H W), irfft2's norm), then act
        f.spec_z = Z;
        f.spec_m2 = m2;
        f.spec_scale = 1.0f / ((float)H * (float)W);
        return nps_conv2d_fwd(&f, stream);
    }
    // w(x) + bias without the activation, then y = act(y + c2r(Z) / (H W)) in the idft_w pass
    NPS_CHECK_ARG(!a.out_nchw && a.out_C == Cout && a.out_H == H && a.out_W == W && a.out_os == 1 && a.out_off_y == 0 &&
                      a.out_off_x == 0 && !a.addend0 && !a.addend1 && a.out_stats == nullptr,
                  "fno_layer2d_fwd: the unfused synthesis needs a dense NHWC [B][H][W][Cout] output, no addend / "
                  "out_stats");
    f.act = 0;
    if ((rc = nps_conv2d_fwd(&f, stream)) < 0) return rc;
    return nps_spectral_idft_w(Z, a.out, B, H, W, m2, Cout, 1, nullptr, a.act, a.out_tag, stream);
}

extern "C" size_t nps_spectral_conv3d_workspace(int B, int Cin, int Cout, int D, int H, int W, int m1, int m2, int m3) {
    if (!spec3_args_ok(B, Cin, Cout, D, H, W, m1, m2, m3)) return 0;
    return spec3_ws(B, Cin, Cout, D, H, m1, m2, m3);
}

extern "C" int nps_spectral_conv3d_fwd(const float* x, const float* w1, const float* w2, const float* w3,
                                       const float* w4, float* y, void* ws, int B, int Cin, int Cout, int D, int H,
                                       int W, int m1, int m2, int m3, int accumulate, int act, void* stream) {
    NPS_CHECK_ARG(x && w1 && w2 && w3 && w4 && y && ws, "spectral_conv3d_fwd: NULL pointer");
    NPS_CHECK_ARG(spec3_args_ok(B, Cin, Cout, D, H, W, m1, m2, m3),
                  "spectral_conv3d_fwd: modes should be at most the spatial dim (// 2 + 1 for the last spatial "
                  "dimension) (D=%d H=%d W=%d m=%d,%d,%d)", D, H, W, m1, m2, m3);
    NPS_CHECK_ARG(act == 0 || act == 1, "spectral_conv3d_fwd: act is 0 (none) or 1 (GELU)");
    const int R1 = D < 2 * m1 ? D : 2 * m1, R2 = H < 2 * m2 ? H : 2 * m2;
    const Spec3 sz = spec3_sizes(B, Cin, Cout, D, H, m1, m2, m3);
    Carve c{static_cast<char*>(ws)};
    float* wp = c.take(sz.wp);
    float* X1 = c.take(sz.x1);
    float* X2 = c.take(sz.x2);
    float* X3 = c.take(sz.x3);
    float* Y = c.take(sz.y);
    float* Z1 = c.take(sz.z1);
    float* Z2 = c.take(sz.z2);
    const nps_src_t src = {x, Cin, D * H, W, 0, 0};  // NDHWC viewed as (B, D*H, W, C)
    int rc;
    if ((rc = nps_spectral3d_pack_weights(w1, w2, w3, w4, wp, Cin, Cout, D, H, m1, m2, m3, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_w(&src, 1, B, D * H, W, Cin, m3, X1, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(X1, X2, B * D, H, m2, m3, Cin, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(X2, X3, B, D, m1, R2 * m3, Cin, stream)) < 0) return rc;
    if ((rc = nps_spectral_mix(X3, wp, Y, B, R1, R2 * m3, Cin, Cout, stream)) < 0) return rc;
    if ((rc = nps_spectral_idft_h(Y, Z1, B, D, m1, R2 * m3, Cout, stream)) < 0) return rc;
    if ((rc = nps_spectral_idft_h(Z1, Z2, B * D, H, m2, m3, Cout, stream)) < 0) return rc;
    return nps_spectral_idft_w(Z2, y, B, D * H, W, m3, Cout, accumulate ? 1 : 0, nullptr, act, nullptr, stream);
}

extern "C" int nps_spectral_conv3d_bwd(const float* x, const float* w1, const float* w2, const float* w3,
                                       const float* w4, const float* dy, float* dx, float* dw1, float* dw2,
                                       float* dw3, float* dw4, void* ws, int B, int Cin, int Cout, int D, int H, int W,
                                       int m1, int m2, int m3, void* stream) {
    NPS_CHECK_ARG(x && w1 && w2 && w3 && w4 && dy && ws, "spectral_conv3d_bwd: NULL pointer");
    const bool gw = dw1 != nullptr;
    NPS_CHECK_ARG((dw2 != nullptr) == gw && (dw3 != nullptr) == gw && (dw4 != nullptr) == gw,
                  "spectral_conv3d_bwd: dw1..dw4 are all given or all NULL");
    NPS_CHECK_ARG(spec3_args_ok(B, Cin, Cout, D, H, W, m1, m2, m3), "spectral_conv3d_bwd: bad shape");
    const int R1 = D < 2 * m1 ? D : 2 * m1, R2 = H < 2 * m2 ? H : 2 * m2;
    const Spec3 sz = spec3_sizes(B, Cin, Cout, D, H, m1, m2, m3);
    Carve c{static_cast<char*>(ws)};
    float* wp = c.take(sz.wp);
    float* X1 = c.take(sz.x1);   // later gX1
    float* X2 = c.take(sz.x2);   // later gX2
    float* X3 = c.take(sz.x3);
    float* gY = c.take(sz.y);
    float* gZ1 = c.take(sz.z1);
    float* gZ2 = c.take(sz.z2);
    float* gX3 = c.take(sz.x3);
    float* gwp = c.take(sz.wp);
    const nps_src_t src = {x, Cin, D * H, W, 0, 0};
    int rc;
    if ((rc = nps_spectral3d_pack_weights(w1, w2, w3, w4, wp, Cin, Cout, D, H, m1, m2, m3, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_w(&src, 1, B, D * H, W, Cin, m3, X1, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(X1, X2, B * D, H, m2, m3, Cin, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(X2, X3, B, D, m1, R2 * m3, Cin, stream)) < 0) return rc;
    if ((rc = nps_spectral_idft_w_bwd(dy, gZ2, B, D * H, W, m3, Cout, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(gZ2, gZ1, B * D, H, m2, m3, Cout, stream)) < 0) return rc;
    if ((rc = nps_spectral_dft_h(gZ1, gY, B, D, m1, R2 * m3, Cout, stream)) < 0) return rc;
    if ((rc = nps_spectral_mix_bwd(X3, wp, gY, gX3, gwp, B, R1, R2 * m3, Cin, Cout, stream)) < 0) return rc;
    if (dx != nullptr) {
        if ((rc = nps_spectral_idft_h(gX3, X2, B, D, m1, R2 * m3, Cin, stream)) < 0) return rc;
        if ((rc = nps_spectral_idft_h(X2, X1, B * D, H, m2, m3, Cin, stream)) < 0) return rc;
        if ((rc = nps_spectral_dft_w_bwd(X1, dx, B, D * H, W, m3, Cin, stream)) < 0) return rc;
    }
    if (gw)
        if ((rc = nps_spectral3d_unpack_grad(gwp, dw1, dw2, dw3, dw4, Cin, Cout, D, H, m1, m2, m3, stream)) < 0)
            return rc;
    return 0;
}
