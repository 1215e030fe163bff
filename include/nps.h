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
    /* arithmetic: NPS_PREC_F32 = exact fp32 MFMA (v_mfma_f32_32x32x2_f32); NPS_PREC_X3F16 = 3-pass
     * split fp16 (x = hi + lo, products hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16, fp32
     * accumulate, ~2^-21 relative per product; weights pre-scaled by an exact power of 2) — only where
     * nps_conv2d_x3_eligible() and nps_conv2d_x3_sources_ok(), with the weight packed by
     * nps_conv2d_pack_weights_x3 */
    int precision;
    /* Input range of a NPS_PREC_X3F16 conv.  The input is scaled by an exact power of 2 (max|x| into
     * [2^13, 2^14)) before the fp16 split and the result scaled back, so values of any magnitude keep
     * fp32-class accuracy (|x| >= max|x| * 2^-16 keep 22 bits; smaller ones an absolute error below
     * max|x| * 2^-37).  Each pointer is NULL or a RANGE TAG (NPS_TAG_FLOATS floats: NPS_TAG_SUB
     * sub-slots NPS_TAG_STRIDE floats apart, the tag's value is their max) holding an upper bound of
     * |x| over the source(s) it covers; the conv uses the max of the non-NULL tags, and scale 1 when
     * all three are NULL.  in_scale: set explicitly (nps_absmax of a gradient) or the tag of source 0;
     * in_tag1 / in_tag2: the tags of sources 1 / 2. */
    const float* in_scale;
    const float* in_tag1;
    const float* in_tag2;
    /* Range tag of the output (any precision, NULL = none): the conv raises it (atomic max of the
     * non-negative float bits, one sub-slot per wave) to >= max |value| of every element it writes.
     * Zero it before the first writer (tags are allocated from a zeroed arena, see ops.py). */
    float* out_tag;
    /* GroupNorm(1) moments of the output (NULL = none): [B][NPS_STATS_SUB][2] fp64 (sum, sum of squares;
     * the sample's moments are the sum over the sub-slots, which spread the atomics) to which the
     * conv ADDS, per sample, the moments of the values it stores — an accumulating conv the change of
     * the moments (stored value minus the value it replaced).  So a zeroed buffer after convs that write
     * every element of `out` once (a conv, the 4 phases of a transposed conv), or a buffer seeded with
     * `out`'s moments after an accumulating conv, holds what nps_group_norm_stats(G = 1) would compute
     * from `out`, without that pass.  Split-fp16 convs with NHWC output and Cout, out_C multiples of 4
     * only (1x1: Cout <= 192, bias-only epilogue); nps_conv2d_fwd refuses others. */
    double* out_stats;
    /* The 4 output phases of a k4/s2 ConvTranspose2d in ONE launch (split-fp16 2x2 convs; 0 or 1 = a single
     * conv): phase ph = 2 py + px uses the packed weight at wpack + ph * phase_wstride floats (its own
     * power-of-2 scale in its trailer) and writes at out_off + (py, px) (out_os = 2).  The phases share
     * the input patch: their work-groups are numbered phase-fastest on one XCD, so the patch is fetched
     * from HBM once (replaces 4 launches of the Upsample, common.py:93-120). */
    int nphase;
    long phase_wstride;
    /* Space-to-depth view (split-fp16 2x2 convs, one source, no prologue; 0 = off): the frame (Hin x Win x
     * Cin, Cin = 4 C) is the space-to-depth of src[0] (H x W x C, C % 16 == 0): frame pixel (y, x) channel
     * p C + c reads src[0] pixel (2 y + (p >> 1) - s2d_pad, 2 x + (p & 1) - s2d_pad) channel c, zero outside.
     * The U-Net Downsample's valid 3x3/s2 conv with padding s2d_pad (proc_unet_modern.py:439-455) runs as
     * a 2x2 stride-1 conv over this view (weight from nps_conv2d_pack_weights_x3 with transposed_phase = -2)
     * without materialising the space-to-depth copy. */
    int s2d;
    int s2d_pad;
    /* FNO layer fusion (1x1 split-fp16 convs on the LDS-weight kernel only; NULL = off): the truncated c2r W pass
     * of the spectral conv is added to the conv's result before the bias / act epilogue — out[b][y][x][o] =
     * act(w(x) + bias + spec_scale * sum_k c_k Re(spec_z[b][y][k][o] e^{2 pi i k x / W})), c_k = 2 except DC /
     * Nyquist (Im dropped), as nps_spectral_idft_w with accumulate (proc_fno.py:142-146: conv(x) + w(x)) — so the
     * separate idft_w read-modify-write of the output is gone.  spec_z: [B][Hout][spec_m2][Cout] complex64 (the
     * spectral pipeline's Z), Wout % 128 == 0, spec_m2 <= 16, no addend / accumulate. */
    const float* spec_z;
    int spec_m2;
    float spec_scale;
} nps_conv2d_t;

/* Range tags (nps_conv2d_t.in_scale / in_tag* / out_tag): 64 sub-slots 256 B apart, so the atomics of
 * thousands of work-groups spread over 64 addresses; readers take the max over the sub-slots. */
#define NPS_TAG_SUB 64
#define NPS_TAG_STRIDE 64
#define NPS_TAG_FLOATS (NPS_TAG_SUB * NPS_TAG_STRIDE)
/* sub-slots per sample of a moments buffer (nps_conv2d_t.out_stats) */
#ifndef NPS_STATS_SUB
#define NPS_STATS_SUB 16
#endif
int nps_stats_sub(void); /* NPS_STATS_SUB of this build (the moments buffers' sub-slot count) */

#define NPS_PREC_F32 0
#define NPS_PREC_X3F16 1

/* Floats of the packed weight buffer for a conv with the given shape
 * (ntaps = KH*KW). */
size_t nps_conv2d_packed_size(int Cout, int Cin, int ntaps);
/* Pack w[Cout][Cin][KH][KW] (nn.Conv2d layout, device pointer) into the
 * MFMA-fragment-native layout.  `transposed_phase` >= 0 packs the
 * stride-2 4x4 transposed-conv weight w[Cin][Cout][4][4]
 * (nn.ConvTranspose2d layout) as the 2x2 conv of output phase
 * (py, px) = (phase>>1, phase&1); KH = KW = 2 then.  transposed_phase == -2 packs a 3x3 stride-2
 * weight w[Cout][Cin/4][3][3] for the space-to-depth 2x2 form (KH = KW = 2, Cin = 4C).
 * transposed_phase == -3 packs the input-gradient conv of a stride-1 conv whose weight is
 * w[Cin][Cout][KH][KW] (Cout / Cin: the packed conv's): w transposed and flipped, element (co, ci, ky, kx) =
 * w[ci][co][KH-1-ky][KW-1-kx]. */
int nps_conv2d_pack_weights(const float* w, float* wpack, int Cout, int Cin, int KH, int KW,
                            int transposed_phase, void* stream);
/* Same transforms, packed as [hi | lo] fp16 MFMA fragments of s*w for precision = NPS_PREC_X3F16, with s
 * the power of 2 that maps max|w| into [2^13, 2^14) (max|w| is kept in the buffer's trailer; same buffer
 * size as nps_conv2d_packed_size).  1x1 weights are packed in 32-channel chunk pairs (each MFMA lane half
 * owns a contiguous 16-channel run), so the chunk count of a 1x1 packing is even. */
int nps_conv2d_pack_weights_x3(const float* w, float* wpack, int Cout, int Cin, int KH, int KW,
                               int transposed_phase, void* stream);
/* One weight of a batched split-fp16 packing: the arguments of nps_conv2d_pack_weights_x3. */
typedef struct {
    const float* w;
    float* wpack;
    int Cout, Cin, KH, KW;
    int transposed_phase;
} nps_pack_job_t;
/* n nps_conv2d_pack_weights_x3 calls (same results, bit for bit) in two launches per 48 jobs instead of two per job:
 * after an optimizer step every conv weight of the model is repacked (forward and input-gradient forms, trainers/
 * base.py:493 -> the next forward / backward), ~200 packings per U-FNO training step whose launch cost, not their
 * bytes, dominated.  jobs: a host array (copied into the launches' arguments). */
int nps_conv2d_pack_weights_x3_batch(const nps_pack_job_t* jobs, int n, void* stream);
/* 1 when a conv of this geometry runs on the split-fp16 kernel (stride-1: undilated 1x1 / 2x2 / 3x3, and
 * 5x5 at any dilation — the dilated ResNet's convs, proc_dilatedresnet.py:15-84). */
int nps_conv2d_x3_eligible(int KH, int KW, int stride, int dil);
/* 1 when the split-fp16 kernel applies a frame prologue itself (gn_groups > 0: GroupNorm affine with that
 * many groups; pre_act 1: GELU) — the 3x3 kernel, with Cin / gn_groups a multiple of 4 — so the caller
 * passes gn_* / pre_act to nps_conv2d_fwd instead of running nps_frame_pack first
 * (replaces ResidualBlock's norm -> act -> conv, proc_unet_modern.py:62-99). */
int nps_conv2d_x3_prologue_ok(int KH, int KW, int Cin, int gn_groups, int pre_act);
/* 1 when the split-fp16 kernel can stage this virtual frame directly: every source boundary on a
 * multiple of 16 channels, every source's C a multiple of 4 (otherwise nps_frame_pack it first). */
int nps_conv2d_x3_sources_ok(const nps_src_t* src, int nsrc);
/* Range tag `tag` (NPS_TAG_FLOATS floats) := max |x[i]| (zeroed, then raised) — the input range a
 * split-fp16 conv scales by (nps_conv2d_t.in_scale / in_tag*). */
int nps_absmax(const float* x, long n, float* tag, void* stream);
/* The same without the zeroing: raises `tag` (already zero, e.g. fresh from a zero-filled arena, or a valid lower
 * bound) to >= max |x[i]| — no memset launch. */
int nps_absmax_into(const float* x, long n, float* tag, void* stream);
/* Stride-2 3x3 convs (U-Net Downsample, proc_unet_modern.py:445-455) run as 2x2 stride-1 convs
 * over a space-to-depth copy: out[B][Hq][Wq][4C], channel (dy*2+dx)*C + c = x[2y+dy-pad][2x+dx-pad][c]
 * (zero outside); pack the weight with transposed_phase = -2 (Cin = 4C). */
int nps_space_to_depth(const float* x, float* out, int B, int H, int W, int C, int pad, int Hq, int Wq,
                       void* stream);
/* Fill TH/TW/lattice/waves of `a` for its shape; returns the LDS bytes used. */
int nps_conv2d_plan(nps_conv2d_t* a);
/* Highest byte (exclusive) of the packed split-fp16 weight that the launch of the planned *a reads (host-only
 * arithmetic of the kernel the launcher picks; must be <= 4 * nps_conv2d_packed_size).  Replaces no reference
 * interface: a check of this build's packing (tests/test_cabi.py). */
long nps_conv2d_x3_weight_span(const nps_conv2d_t* a);
int nps_conv2d_fwd(const nps_conv2d_t* a, void* stream);

/* Materialise a virtual frame: out[B][Hin][Win][Cin] = act(GN(frame)) using the prologue fields
 * of `a` (or the plain concat/crop when there is none); with a->out_C in (Cin, Cin + 4) the output
 * rows are out_C channels wide, the extra channels zero (4-channel alignment for the split-fp16 conv).  One HBM pass that evaluates the
 * GroupNorm affine + GELU once per element (proc_unet_modern.py:245-247) ahead of a conv that
 * then stages raw bytes only. */
int nps_frame_pack(const nps_conv2d_t* a, float* out, void* stream);

/* GroupNorm statistics over a virtual frame (same source semantics as the conv):
 * stats[B][G][2] += (sum, sumsq) in fp64.  Replaces the moments of
 * nn.GroupNorm (proc_unet_modern.py:235-236, :155).  stats must be zeroed
 * first (the call does it when zero_first != 0). */
int nps_group_norm_stats(const nps_src_t* src, int nsrc, int B, int Hin, int Win, int Cin, int G,
                         double* stats, int zero_first, void* stream);
/* Test hook: run the split-fp16 conv kernels on a persistent grid of `wgs` work-groups (> 0; 0 = one per
 * CU, the default) so every work-group walks many tiles. */
int nps_x3_set_grid(long wgs);

/* GroupNorm(1) moments of a virtual frame from those of its sources, each covering the frame exactly
 * (nps_conv2d_t.out_stats) — the per-source moments of torch.cat's GroupNorm (proc_unet_modern.py:235-236):
 * part i is [B][n_i][2] (n_i sub-slots; p1, p2 may be NULL), out is [B][n_out][2] and receives
 * out[b][0][k] = sum over parts and sub-slots of p_i[b][s][k] (its other sub-slots are left as they are). */
int nps_stats_sum(const double* p0, int n0, const double* p1, int n1, const double* p2, int n2, int B, double* out,
                  int n_out, void* stream);

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
/* out[B][H][W][Cout] (= or +=) y ; optional addend, act as in nps_conv2d_t; out_tag (or NULL): the
 * output's range tag, raised to cover every value written (nps_conv2d_t.out_tag) */
int nps_spectral_idft_w(const float* Z, float* out, int B, int H, int W, int m2, int Cout, int accumulate,
                        const float* addend, int act, float* out_tag, void* stream);

/* ---- one call per module: SpectralConv2d / SpectralConv3d / FNO_Layer (composites of the stages) ------
 * The stage entry points above and below, sequenced inside the library, so a C caller runs a whole module
 * from this header alone.  x / y / dx: fp32 NHWC ([B][H][W][C]; 3-D: NDHWC, i.e. [B][D*H][W][C]); w1..w4 /
 * dw1..dw4: the modules' complex64 nn.Parameters in the reference layout ([Cin][Cout][m1][m2](+[m3]),
 * interleaved re/im), packed per call into the workspace; ws: caller-owned device memory of at least the
 * *_workspace() bytes (the same size serves forward and backward; 0 = bad shape).  No range tags or carried
 * moments: the plain reference semantics.  Errors: as every entry point (mode bounds as proc_fno.py:134-139). */
size_t nps_spectral_conv2d_workspace(int B, int Cin, int Cout, int H, int W, int m1, int m2);
/* SpectralConv2d.forward (proc_fno.py:257-288): y = irfft2(P(rfft2(x))) with accumulate = 0 (act = 0);
 * y = act(y + irfft2(...)) with accumulate = 1 (act 0 none / 1 GELU: FNO_Layer's sum + activation, :142-146). */
int nps_spectral_conv2d_fwd(const float* x, const float* w1, const float* w2, float* y, void* ws, int B, int Cin,
                            int Cout, int H, int W, int m1, int m2, int accumulate, int act, void* stream);
/* Its backward under torch.fft / complex-einsum autograd: dx = dL/dx (written; NULL = skip),
 * dw1 / dw2 = dL/dweights1, dL/dweights2 (written, PyTorch's conj(x) * g convention; both or neither). */
int nps_spectral_conv2d_bwd(const float* x, const float* w1, const float* w2, const float* dy, float* dx, float* dw1,
                            float* dw2, void* ws, int B, int Cin, int Cout, int H, int W, int m1, int m2,
                            void* stream);
/* FNO_Layer.forward (proc_fno.py:142-146, 2-D, conv_mode 'single'): w->out = act(SpectralConv2d(x) + w(x)).  `w`
 * is the layer's 1x1 conv `w`, filled in and nps_conv2d_plan()ned by the caller (src = the layer's input frame
 * covered by its sources, wpack, bias, out = y, act = the layer's activation, range tags), spec_z unset.  The
 * library picks the synthesis: fused into the 1x1's epilogue (nps_conv2d_t.spec_z: split-fp16, Wout % 128 == 0,
 * m2 <= 16, Cout <= 192, Cout % 4 == 0, no addend / accumulate), else the 1x1 then nps_spectral_idft_w
 * accumulating with the activation.  ws: nps_fno_layer2d_workspace bytes. */
size_t nps_fno_layer2d_workspace(int B, int Cin, int Cout, int H, int W, int m1, int m2);
int nps_fno_layer2d_fwd(const nps_conv2d_t* w, const float* w1, const float* w2, int m1, int m2, void* ws,
                        void* stream);
/* SpectralConv3d (proc_fno.py:291-376): the same pair over (D, H, W) with the four corner weights. */
size_t nps_spectral_conv3d_workspace(int B, int Cin, int Cout, int D, int H, int W, int m1, int m2, int m3);
int nps_spectral_conv3d_fwd(const float* x, const float* w1, const float* w2, const float* w3, const float* w4,
                            float* y, void* ws, int B, int Cin, int Cout, int D, int H, int W, int m1, int m2, int m3,
                            int accumulate, int act, void* stream);
int nps_spectral_conv3d_bwd(const float* x, const float* w1, const float* w2, const float* w3, const float* w4,
                            const float* dy, float* dx, float* dw1, float* dw2, float* dw3, float* dw4, void* ws,
                            int B, int Cin, int Cout, int D, int H, int W, int m1, int m2, int m3, void* stream);

/* ---- bf16 storage (BASELINE config C5: the 3-D rFFT spectral conv in bf16) ----------------------------
 * Activations in HBM as bf16 (16-bit storage of NDHWC tensors viewed as (B, D*H, W, C)), every sum in fp32:
 * the same transforms as the fp32 entry points above.  Replaces the fp32 SpectralConv3d / FNO_Layer chain of
 * proc_fno.py:291-376, :142-146 for a bf16 model (the reference has no bf16 path: CPU FFT rejects bf16,
 * SURVEY.md §0.5); parity is checked against the fp32 HIP path, itself pinned to the oracle. */
int nps_spectral_dft_w_bf16(const nps_src_t* src, int nsrc, int B, int H, int W, int C, int m2, float* X1,
                            void* stream);
/* wpack: the nps_spectral(3d)_pack_weights layout with every complex value as a packed bf16 (re, im) pair
 * (nps_f32_to_bf16 of the fp32 packing) */
int nps_spectral_mix_bf16(const float* X2, const void* wpack, float* Y, int B, int R, int m2, int Cin, int Cout,
                          void* stream);
/* out / addend bf16 [B][H][W][Cout]; out (= or +=) act(c2r(Z)/(H W) + addend) */
int nps_spectral_idft_w_bf16(const float* Z, void* out, int B, int H, int W, int m2, int Cout, int accumulate,
                             const void* addend, int act, void* stream);
/* elementwise conversion (bf16 round-to-nearest-even) */
int nps_f32_to_bf16(const float* x, long n, void* y, void* stream);
int nps_bf16_to_f32(const void* x, long n, float* y, void* stream);
/* pointwise conv (FNO_Layer `w` with kernel 1, proc_fno.py:104-107) in bf16: a->src / a->out / a->addend0 bf16
 * NHWC (sources covering the frame, all but the last with C % 8 == 0), a->wpack from nps_pack_1x1_bf16
 * ([Cout][nps_conv1x1_bf16_kr(Cin)] bf16), a->bias fp32, epilogue act(acc + bias + addend0) on
 * v_mfma_f32_32x32x16_bf16 with fp32 accumulation; Cout in {32, 64, 96, 128, 192, 256}. */
int nps_conv1x1_bf16_kr(int Cin);
int nps_pack_1x1_bf16(const float* w, void* wp, int Cout, int Cin, void* stream);
int nps_conv1x1_bf16(const nps_conv2d_t* a, void* stream);

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

/* ==== backward (training) ================================================
 * The pushforward train_step (trainers/autoregressivepushforwardtrainer.py:43-163) and
 * trainers/base.py:492 `loss.backward()` differentiate every op above.  Input gradients of a
 * conv are forward convs of dy (nps_conv2d_fwd) with flipped / transposed / phase-split weights;
 * the entries below provide the rest. */

/* Weight gradient of a stride-1 (optionally dilated, zero- or circularly-padded) conv on fp32
 * MFMA: g[m][n][ky*KW + kx] += sum_{b,py,px} a[b][py][px][m] * X[b][y][x][n] with
 * (y, x) = (py + ky*dil - pad_y, px + kx*dil - pad_x) in the frame extended circularly by
 * `circ` (outside it reads 0) — the same geometry as nps_conv2d_t.  For a conv, a = dy and
 * X = its input, so g is the nn.Conv2d weight grad [Cout][Cin][KH][KW]; stride-2 and transposed
 * convs are issued in their space-to-depth / phase form.  Replaces aten
 * convolution_backward's weight output for models/common.py:37-47, 93-120. */
typedef struct {
    const float* a;                 /* [B][Ha][Wa][M] (NHWC) */
    int B, Ha, Wa, M;
    const float* x;                 /* [B][Hx][Wx][N] (NHWC) */
    int Hx, Wx, N;
    int KH, KW, dil, pad_y, pad_x, circ;
    float* g;                       /* [M][N][KH*KW], accumulated with += */
    /* [M] or NULL: the split-fp16 entry points (nps_conv2d_wgrad_x3 / _set) also give db[m] = sum_{b,py,px}
     * a[b][py][px][m] — the conv's bias gradient when a = dy — with g's semantics (+= / =), from the values the
     * kernel stages anyway (no nps_channel_sums pass over dy).  Must be NULL for nps_conv2d_wgrad. */
    float* db;
} nps_wgrad_t;
size_t nps_wgrad_lds_bytes(int KH, int KW);
int nps_conv2d_wgrad(const nps_wgrad_t* p, void* stream);
/* The same weight gradient in the split-fp16 arithmetic of NPS_PREC_X3F16 (3 fp16 MFMA products per
 * fp32 product, fp32 accumulation) for undilated 1x1 / 2x2 / 3x3 kernels (KH == KW) over channel
 * counts M, N that are multiples of 4: a and x are scaled by exact powers of two from their range tags
 * a_range / x_range (NPS_TAG_FLOATS floats, e.g. from nps_absmax) before the split.  ws: a device
 * workspace of nps_wgrad_x3_ws_floats(M, N, KH, KW) floats (the split-K partials accumulate there
 * tap-major, then fold into g).  Same geometry and += semantics as nps_conv2d_wgrad. */
size_t nps_wgrad_x3_ws_floats(int M, int N, int KH, int KW);  /* KH*KW*M*N partials + M (the bias row) */
int nps_conv2d_wgrad_x3(const nps_wgrad_t* p, const float* a_range, const float* x_range, float* ws, void* stream);
/* The same, storing G = the weight gradient (g need not be zeroed beforehand) instead of adding to it. */
int nps_conv2d_wgrad_x3_set(const nps_wgrad_t* p, const float* a_range, const float* x_range, float* ws,
                            void* stream);
/* out[c] += sum over `rows` rows of x[row][c] (conv bias gradients; parameter-partial reductions) */
int nps_channel_sums(const float* x, long rows, int C, float* out, void* stream);

/* Backward of nps_frame_pack: torch.cat + crop_Nd + GroupNorm + GELU (proc_unet_modern.py:245-247,
 * :194, common.py:20-34) given gy = dL/d(frame).  dsrc[i] (shape of source i, or NULL) receives the
 * gradient of each source (0 where the source lies outside the frame); dgamma/dbeta [Cin] are written
 * when the prologue has a GroupNorm; work = [B][2][Cin] fp64 scratch. */
int nps_frame_pack_bwd(const nps_conv2d_t* a, const float* gy, float* const* dsrc, float* dgamma, float* dbeta,
                       double* work, void* stream);
/* The same, also raising the range tag dtag[i] (NPS_TAG_FLOATS floats, or NULL; dtag itself may be NULL) to
 * cover |dsrc[i]| — the range of the gradient the next conv backward reads as its dy. */
int nps_frame_pack_bwd_tagged(const nps_conv2d_t* a, const float* gy, float* const* dsrc, float* const* dtag,
                              float* dgamma, float* dbeta, double* work, void* stream);
/* The same with gy_plain (or NULL): the gradient of the plain concatenation of the same sources (the frame without
 * prologue, shaped like gy) from a second consumer — the ResidualBlock's shortcut conv or identity path
 * (proc_unet_modern.py:243-250) — added into dsrc in the same pass instead of by a separate accumulation.
 * Unlike the two above, `work` must hold zeros on entry (e.g. a slice of a zero-filled buffer used once): no
 * memset launch per frame. */
int nps_frame_pack_bwd2(const nps_conv2d_t* a, const float* gy, const float* gy_plain, float* const* dsrc,
                        float* const* dtag, float* dgamma, float* dbeta, double* work, void* stream);

/* element-wise pieces of the differentiated graph */
int nps_gelu(const float* x, float* y, long n, void* stream);                                /* nn.GELU() */
int nps_gelu_bwd(const float* x, const float* gy, float* gx, long n, void* stream);
/* out[b][y+off_y][x+off_x][c] += src[b][y][x][c] (crop_Nd(h) + shortcut, proc_unet_modern.py:250) */
int nps_add_at(float* out, const float* src, int B, int Ho, int Wo, int Hs, int Ws, int C, int off_y, int off_x,
               void* stream);
/* out = base + that placement of src, in one pass (out, base: [B][Ho][Wo][C]; C % 4 == 0, 16-B aligned);
   out_stats: NULL, or [B][NPS_STATS_SUB][2] fp64 to which the launch ADDS out's GroupNorm(1) moments (sum, sum of
   squares per sample), as nps_conv2d_t.out_stats */
int nps_add_at_copy(float* out, const float* base, const float* src, int B, int Ho, int Wo, int Hs, int Ws, int C,
                    int off_y, int off_x, double* out_stats, void* stream);
/* circular_pad_2d (models/common.py:61-90) on NHWC and its adjoint (wrap-sum) */
int nps_circular_pad(const float* x, float* out, int B, int H, int W, int C, int pad, void* stream);
int nps_circular_fold(const float* gp, float* gx, int B, int H, int W, int C, int pad, void* stream);
/* out = (*scale) * (a - b): gradient of sqrt(MSELoss(sum)) (autoregressivepushforwardtrainer.py:158-162) */
int nps_scaled_diff(const float* a, const float* b, const double* scale, float* out, long n, void* stream);

/* SpectralConv2d backward (proc_fno.py:257-288 under torch.fft autograd):
 *  gZ  = (c_k / (H W)) DFT_W(gy)  on the m2 kept bins (c_k = 1 for DC/Nyquist, else 2)  idft_w_bwd
 *  gY  = nps_spectral_dft_h(gZ);   gX2, gwpack = mix_bwd(X2, wpack, gY)
 *  gX1 = nps_spectral_idft_h(gX2); gx[w] = sum_k Re(gX1[k] e^{+2 pi i k w / W})           dft_w_bwd
 *  gweights1/2 = unpack_grad(gwpack)  (PyTorch's complex-gradient convention, conj(x) * g) */
int nps_spectral_idft_w_bwd(const float* gy, float* gZ, int B, int H, int W, int m2, int Cout, void* stream);
int nps_spectral_dft_w_bwd(const float* gX1, float* gx, int B, int H, int W, int m2, int Cin, void* stream);
int nps_spectral_mix_bwd(const float* X2, const float* wpack, const float* gY, float* gX2, float* gwpack, int B,
                         int R, int m2, int Cin, int Cout, void* stream);
int nps_spectral_unpack_grad(const float* gwpack, float* gw1, float* gw2, int Cin, int Cout, int H, int m1, int m2,
                             void* stream);

/* SpectralConv3d (proc_fno.py:291-376: rfftn over (D, H, W) -> 4 retained corners weights1..4 -> irfftn)
 * on NDHWC activations, composed of the 2-D stages above applied per axis:
 *  W: dft_w over (B, D*H, W)                 -> X1 [B][D*H][m3][C]
 *  H: dft_h over (B*D, H), m2 := m3          -> X2 [B*D][R2][m3][C]        R2 = min(H, 2*m2)
 *  D: dft_h over (B, D),   m2 := R2*m3       -> X3 [B][R1][R2*m3][C]       R1 = min(D, 2*m1)
 *  mix(X3, wpack, R := R1, m2 := R2*m3); idft_h (D), idft_h (H), idft_w over (B, D*H, W) (1/(D*H*W)).
 * The backward is the same adjoint chain as the 2-D one, axis by axis.
 * wpack: [R1][R2][m3][Cin][Cout] complex; where corners overlap the later reference write wins
 * (w1 [:m1,:m2] < w2 [-m1:,:m2] < w3 [:m1,-m2:] < w4 [-m1:,-m2:], proc_fno.py:342-350). */
int nps_spectral3d_pack_weights(const float* w1, const float* w2, const float* w3, const float* w4, float* wpack,
                                int Cin, int Cout, int D, int H, int m1, int m2, int m3, void* stream);
/* gweights1..4 [Cin][Cout][m1][m2][m3] from gwpack (0 where a later corner owns the mode) */
int nps_spectral3d_unpack_grad(const float* gwpack, float* gw1, float* gw2, float* gw3, float* gw4, int Cin, int Cout,
                               int D, int H, int m1, int m2, int m3, void* stream);

/* TimeConvDense + add_delta + tanh + mask backward (dec_grid.py:126-146, :8-31): gpre is planar like
 * `pre`; ws[blocks][params] receives per-block partials of [w1 | b1 | w2 | b2] (blocks = B*ceil(H*W/64),
 * params = 2c*c*ka + 2c + c*2c*kb + c), reduced with nps_channel_sums. */
int nps_timeconv_decode_bwd(const float* pre, const float* u, const float* w1, const float* b1, const float* w2,
                            const float* b2, const float* dtcum, const float* mask, int mask_S, int mask_ch,
                            const float* gout, float* gpre, float* ws, int B, int num_c, int tw, int H, int W,
                            int act_tanh, void* stream);
/* 'individual_static' volume rescale backward (activation_wrapper.py:80-105):
 * D[plane] = sum g (1 - m) u_in (nps_plane_dot), then gu_in (nps_volume_rescale_bwd). */
int nps_plane_dot(const float* g, const float* u, const float* mask, int mask_S, int mask_ch, int B, int nct, int H,
                  int W, double* D, void* stream);
int nps_volume_rescale_bwd(const float* g, const double* new_tot, const double* prev_tot, const float* mpdcum,
                           const float* mask, int mask_S, int mask_ch, const double* D, float* gu, int B, int num_c,
                           int tw, int H, int W, void* stream);

/* ---- 3-D U-Net of the 3-D U-FNO (BASELINE config C5: U-FNO 3D over a time-bundled D x H x W volume) ----
 * The reference builds the 3-D U-Net's ResidualBlock / Down / Middle / Downsample from nn.Conv3d and
 * nn.GroupNorm (proc_unet_modern.py:199-455 with num_spatial_dims=3) but has no 3-D Upsample
 * (models/common.py:103-120 raises); this build defines it per axis as the 2-D rule: circular pad 1,
 * then ConvTranspose3d(k=4, s=2, p=0) (DESIGN.md "3-D U-FNO").  Activations are NDHWC; storage and MFMA
 * arithmetic are bf16 (v_mfma_f32_32x32x16_bf16, fp32 accumulate) or exact fp32 (v_mfma_f32_32x32x2_f32). */
typedef struct {
    const void* ptr;            /* [B][D][H][W][C] NDHWC, element type per nps_conv3d_t.bf16 */
    int C, D, H, W;
    int off_d, off_h, off_w;    /* placement in the core frame (crop_Nd: < 0 crops, > 0 zero-pads) */
} nps_src3_t;

typedef struct {
    int nsrc;
    nps_src3_t src[NPS_MAX_SRC];
    int B, Dc, Hc, Wc, Cin;     /* core frame (the virtual concatenation); Cin = sum of src[i].C */
    /* frame extension, per side of every spatial axis: circular by `circ` (circular_pad), then `zpad`
     * zeros; the conv is valid over the extended frame */
    int circ, zpad;
    /* prologue on core-frame values (sources' zeros included): x' = act(GN(x)) */
    const double* gn_stats;     /* [B][G][2] (sum, sum of squares) from nps_gn_stats3d, or NULL */
    const float* gn_gamma;      /* [Cin] */
    const float* gn_beta;
    int gn_groups;
    float gn_eps;
    int pre_act;                /* 0 none, 1 GELU(erf) */
    int K, stride;              /* K^3 taps; K in {1, 2, 3}, stride 1 or 2 (K = 3) */
    int transposed;             /* 1: a k4/s2 ConvTranspose3d as 8 phase convs with K = 2, stride 1 */
    int Dout, Hout, Wout;       /* conv output positions (per phase) */
    const void* wpack;          /* nps_conv3d_pack_weights layout */
    const float* bias;          /* [Cout] or NULL */
    int Cout;
    /* epilogue: destination index per axis = m*out_os + out_off (+ the phase bit when transposed);
     * positions outside [0, out_D) x [0, out_H) x [0, out_W) are skipped (crop) */
    void* out;
    int out_C, out_D, out_H, out_W, out_os, out_off_d, out_off_h, out_off_w;
    int accumulate;             /* out += result (crop_Nd(h) + shortcut, proc_unet_modern.py:250) */
    const void* addend;         /* indexed like out, or NULL (proc_ufno.py:118 h_fno + h_unet) */
    int act;                    /* 0 none, 1 GELU, after bias + addend */
    int bf16;                   /* 1: bf16 storage / bf16 MFMA; 0: fp32 storage / exact fp32 MFMA */
    /* [B][NPS_STATS_SUB][2] fp64 or NULL: the launch ADDS the (sum, sum of squares) of the values it stores
     * (as stored: bf16-rounded for bf16 storage; after addend and act) — with accumulate, of the change (stored
     * minus replaced value), as nps_conv2d_t.out_stats — the GroupNorm(1) moments of its output, carried to the
     * next frame instead of an nps_gn_stats3d pass. */
    double* out_stats;
} nps_conv3d_t;

/* Conv3d weight (Cout, Cin, K, K, K) or, transposed != 0, ConvTranspose3d weight (Cin, Cout, 4, 4, 4) ->
 * the kernel's packing ([phase][64-channel Cout tile][kd][16-channel Cin chunk][kh][kw][64][16], zero
 * padded), fp32 or bf16 elements.  nps_conv3d_packed_bytes gives the buffer size. */
size_t nps_conv3d_packed_bytes(int Cout, int Cin, int K, int transposed, int bf16);
int nps_conv3d_pack_weights(const float* w, void* wpack, int Cout, int Cin, int K, int transposed, int bf16,
                            void* stream);
int nps_conv3d_fwd(const nps_conv3d_t* a, void* stream);
/* act(GN(frame)) of a's core frame (sources, GroupNorm prologue, pre_act) materialised once as
 * out[B][Dc][Hc][Wc][Cpad] (channels >= Cin zero, Cpad % 8 == 0): the conv that follows reads one aligned
 * source without a prologue (the fused prologue recomputes each element for every depth tap and halo). */
int nps_frame_pack3d(const nps_conv3d_t* a, void* out, int Cpad, void* stream);
/* GroupNorm moments of a core frame (a's sources and B, Dc, Hc, Wc, Cin, bf16): ADDS per (b, group) the
 * fp64 (sum, sum of squares) of the frame's values (uncovered positions count as 0) to stats[B][G][2] */
int nps_gn_stats3d(const nps_conv3d_t* a, int G, double* stats, void* stream);

const char* nps_last_error(void);
const char* nps_version(void);

/* ---- on-disk data path: device-resident windowing (common/data_creator.py:48-78, create_data) ----
 * out[b][c][t][hw] = u[b][c][steps[b] + offset + t][hw], t < tw; u (B, C, T, H*W) and out (B, C, tw, H*W)
 * contiguous fp32 device arrays, steps[B] int32 on the device (offset = -tw: model inputs, 0: labels;
 * the caller checks steps[b] + offset >= 0 and steps[b] + offset + tw <= T, as the reference asserts). */
int nps_gather_windows(const float* u, const int* steps, float* out, int B, int C, int T, long HW, int tw, int offset,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NPS_H */
