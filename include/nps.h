/*
 * nps.h — C ABI of libnps_hip.so, the MI355X (gfx950) kernels behind the
 * neural-operator rollout hot path of yoeripoels/neural-pde-surrogates.
 *
 * The reference has no native code: every entry point below replaces the aten
 * calls that one reference Python site makes (cited per function, paths
 * relative to the reference's src/).  The drop-in boundary above this ABI is
 * the reference's own nn.Module / cfg surface, mirrored in
 * neural-pde-surrogates_amd/{models,trainers}.
 *
 * Conventions
 *  - Activations are fp32 NHWC ([B][H][W][C], C fastest) unless a field says
 *    otherwise; spectra are interleaved complex64 (float2).
 *  - All pointers are device pointers owned by the caller (PyTorch's caching
 *    allocator); the library never allocates.  `stream` is a hipStream_t
 *    (torch.cuda.current_stream().cuda_stream); every call is asynchronous
 *    and stream-ordered, never synchronises, and is hipGraph-capturable.
 *  - Return 0 on success, <0 on error (-1 bad argument / unsupported shape,
 *    -2 HIP launch error); nps_last_error() describes the last failure of the
 *    calling thread.
 */
#ifndef NPS_H
#define NPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NPS_MAX_SRC 3

/* One channel-slice of a virtual (concatenated) conv input.
 * Replaces torch.cat along channels (proc_unet_modern.py:191, :351, :418;
 * proc_ufno.py:111; proc_dilatedresnet.py:49 [ref line 165]) and
 * crop_Nd's zero-pad/crop (models/common.py:20-34): the source tensor
 * [B][H][W][C] sits at (off_y, off_x) of the virtual input frame; frame
 * positions it does not cover read as 0 (before any normalisation). */
typedef struct {
    const float* ptr;
    int C, H, W;
    int off_y, off_x;
} nps_src_t;

/* Implicit-GEMM 2-D convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32).
 * Replaces nn.Conv2d / nn.ConvTranspose2d forward as built by
 * models/common.py:37-47, 93-120 (valid / zero / circular padding, stride,
 * dilation; a 4x4/s2 transposed conv is issued as 4 phase convs, see
 * DESIGN.md), with fused prologue GroupNorm+GELU (proc_unet_modern.py:245-247,
 * :194) and fused epilogue bias / addends / GELU / accumulate-at-offset
 * (the residual `crop_Nd(h) + shortcut` of proc_unet_modern.py:250, the
 * U-FNO sum+GELU of proc_ufno.py:118, the DRN residual of
 * proc_dilatedresnet.py:49). */
typedef struct {
    int nsrc;
    nps_src_t src[NPS_MAX_SRC];
    int B, Hin, Win, Cin;           /* virtual input frame; Cin = sum of src[i].C */
    /* prologue: x' = act(GN(x)) on every frame value (incl. crop zeros) */
    const double* gn_stats;         /* [B][G][2] = (sum, sum of squares) over the frame, or NULL */
    const float* gn_gamma;          /* [Cin] */
    const float* gn_beta;           /* [Cin] */
    int gn_groups;
    float gn_eps;
    int pre_act;                    /* 0 none, 1 GELU(erf) */
    /* geometry: input row for output row oy and tap ky is
     *   y_ext = oy*stride + ky*dil - pad_y  in a frame extended circularly by `circ`
     * on each side; y_ext outside [0, Hin+2*circ) reads 0 (after the prologue). */
    int KH, KW, stride, dil, pad_y, pad_x, circ;
    int Hout, Wout;
    const float* wpack;             /* nps_conv2d_pack_weights layout */
    const float* bias;              /* [Cout] or NULL */
    int Cout;
    /* epilogue: dest pixel = (oy*out_os + out_off_y, ox*out_os + out_off_x) */
    float* out;
    int out_C, out_H, out_W, out_os, out_off_y, out_off_x;
    int out_nchw;                   /* 1: out is [B][out_C][out_H][out_W] */
    int accumulate;                 /* out += result */
    const float* addend0;           /* indexed like out, or NULL */
    const float* addend1;
    int act;                        /* 0 none, 1 GELU */
    int add_after_act;              /* 0: act(acc+bias+addends); 1: act(acc+bias)+addends */
    /* tiling, chosen by nps_conv2d_plan() */
    int TH, TW, lattice, waves;
} nps_conv2d_t;

/* Floats of the packed weight buffer for a conv with the given shape
 * (ntaps = KH*KW). */
size_t nps_conv2d_packed_size(int Cout, int Cin, int ntaps);
/* Pack w[Cout][Cin][KH][KW] (nn.Conv2d layout, device pointer) into the
 * MFMA-fragment-native layout.  `transposed_phase` >= 0 packs the
 * stride-2 4x4 transposed-conv weight w[Cin][Cout][4][4]
 * (nn.ConvTranspose2d layout) as the 2x2 conv of output phase
 * (py, px) = (phase>>1, phase&1); KH = KW = 2 then.  transposed_phase == -2 packs a 3x3 stride-2
 * weight w[Cout][Cin/4][3][3] for the space-to-depth 2x2 form (KH = KW = 2, Cin = 4C). */
int nps_conv2d_pack_weights(const float* w, float* wpack, int Cout, int Cin, int KH, int KW,
                            int transposed_phase, void* stream);
/* Stride-2 3x3 convs (U-Net Downsample, proc_unet_modern.py:445-455) run as 2x2 stride-1 convs
 * over a space-to-depth copy: out[B][Hq][Wq][4C], channel (dy*2+dx)*C + c = x[2y+dy-pad][2x+dx-pad][c]
 * (zero outside); pack the weight with transposed_phase = -2 (Cin = 4C).  C % 4 == 0. */
int nps_space_to_depth(const float* x, float* out, int B, int H, int W, int C, int pad, int Hq, int Wq,
                       void* stream);
/* Fill TH/TW/lattice/waves of `a` for its shape; returns the LDS bytes used. */
int nps_conv2d_plan(nps_conv2d_t* a);
int nps_conv2d_fwd(const nps_conv2d_t* a, void* stream);

/* Materialise a virtual frame: out[B][Hin][Win][Cin] = act(GN(frame)) using the prologue fields
 * of `a` (or the plain concat/crop when there is none).  One HBM pass that evaluates the
 * GroupNorm affine + GELU once per element (proc_unet_modern.py:245-247) ahead of a conv that
 * then stages raw bytes only. */
int nps_frame_pack(const nps_conv2d_t* a, float* out, void* stream);

/* GroupNorm statistics over a virtual frame (same source semantics as the conv):
 * stats[B][G][2] += (sum, sumsq) in fp64.  Replaces the moments of
 * nn.GroupNorm (proc_unet_modern.py:235-236, :155).  stats must be zeroed
 * first (the call does it when zero_first != 0). */
int nps_group_norm_stats(const nps_src_t* src, int nsrc, int B, int Hin, int Win, int Cin, int G,
                         double* stats, int zero_first, void* stream);

/* ---- SpectralConv2d forward (proc_fno.py:257-288) ----------------------
 * Truncated DFTs replace rfft2 / irfft2: only the 2*m1 x m2 retained modes
 * are ever formed.  rows R = min(H, 2*m1) distinct retained k1 rows.
 *  X1[B][H][m2][C]    = sum_w x e^{-2pi i k2 w/W}          (nps_spectral_dft_w)
 *  X2[B][R][m2][C]    = sum_h X1 e^{-2pi i k1 h/H}          (nps_spectral_dft_h)
 *  Y [B][R][m2][Co]   = sum_i X2 * Wsel[i][o]               (nps_spectral_mix)
 *  Z [B][H][m2][Co]   = sum_r Y e^{+2pi i k1 h/H}           (nps_spectral_idft_h)
 *  y [B][H][W][Co]    = c2r_W(Z) / (H*W)  (+ epilogue)      (nps_spectral_idft_w)
 * c2r keeps Re of the DC (and Nyquist) bin only, as pocketfft/MKL do. */
int nps_spectral_dft_w(const nps_src_t* src, int nsrc, int B, int H, int W, int C, int m2,
                       float* X1, void* stream);
int nps_spectral_dft_h(const float* X1, float* X2, int B, int H, int m1, int m2, int C, void* stream);
/* wpack: [R][m2][Cin][Cout] complex — nps_spectral_pack_weights from the two
 * nn.Parameters weights1/weights2 [Cin][Cout][m1][m2] (complex64). */
int nps_spectral_pack_weights(const float* w1, const float* w2, float* wpack, int Cin, int Cout, int H,
                              int m1, int m2, void* stream);
int nps_spectral_mix(const float* X2, const float* wpack, float* Y, int B, int R, int m2, int Cin, int Cout,
                     void* stream);
int nps_spectral_idft_h(const float* Y, float* Z, int B, int H, int m1, int m2, int Cout, void* stream);
/* out[B][H][W][Cout] (= or +=) y ; optional addend, act as in nps_conv2d_t */
int nps_spectral_idft_w(const float* Z, float* out, int B, int H, int W, int m2, int Cout, int accumulate,
                        const float* addend, int act, void* stream);

/* ---- grid encoder / decoder / wrapper ---------------------------------
 * Encoder input packing, enc_grid.py:41-50 + enc_proc_dec.py:127-137:
 * xin[B][H][W][Cp] = [u(B,c,tw,H,W) flattened c*tw | pos(B,H,W,2) | cond(B,K) broadcast | sc(B,S,H,W)],
 * zero-padded to Cp channels; vb[B][H][W][K+S] = [cond broadcast | sc]. */
int nps_pack_grid_input(const float* u, const float* pos, const float* cond, const float* sc, float* xin,
                        float* vb, int B, int CT, int H, int W, int K, int S, int Cp, void* stream);
/* TimeConvDense conv1d chain + add_delta + tanh + spatial-cond mask
 * (dec_grid.py:126-146, :8-31; activation_wrapper.py:34-35).
 * pre: [B][num_c*3*tw][H][W] (planar pre_decoder output), u: model input
 * (B,num_c,tw,H,W); out: (B,num_c,tw,H,W).  dtcum[tw] = fp32 cumsum(dt).
 * mask: (B,S,H,W) channel `mask_ch` or NULL. */
int nps_timeconv_decode(const float* pre, const float* u, const float* w1, const float* b1, const float* w2,
                        const float* b2, const float* dtcum, const float* mask, int mask_S, int mask_ch,
                        float* out, int B, int num_c, int tw, int H, int W, int act_tanh, void* stream);
/* sums[p] = sum over plane p (plane_size floats at base + p*plane_stride), fp64 */
int nps_plane_sums(const float* base, long plane_stride, int plane_size, int nplanes, double* sums,
                   void* stream);
/* approx_volume_preserve 'individual_static' rescale + mask (activation_wrapper.py:80-105), in place.
 * new_tot[B*c*tw], prev_tot[B*c] (fp64 sums); mpdcum[tw] = fp32 cumsum(max_pct_dif). */
int nps_volume_rescale(float* u, const double* new_tot, const double* prev_tot, const float* mpdcum,
                       const float* mask, int mask_S, int mask_ch, int B, int num_c, int tw, int H, int W,
                       void* stream);
/* MSE_sum between two equal-size tensors, fp64: *out += sum((a-b)^2)  (nn.MSELoss(reduction='sum')) */
int nps_sq_err_sum(const float* a, const float* b, long n, double* out, void* stream);
/* layout transforms at module boundaries */
int nps_nchw_to_nhwc(const float* in, float* out, int B, int C, int H, int W, void* stream);
int nps_nhwc_to_nchw(const float* in, float* out, int B, int C, int H, int W, void* stream);

const char* nps_last_error(void);
const char* nps_version(void);

#ifdef __cplusplus
}
#endif
#endif /* NPS_H */
