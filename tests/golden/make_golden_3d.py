"""Generate the 3-D golden fixtures (SpectralConv3d with corner overlaps + grads, FNO-3D processor, and the
3-D U-Net / U-FNO pieces the reference can build: a single-resolution 3-D UNetModern and U-FNO — the
reference has no 3-D Upsample, common.py:103-120 — and the 3-D Downsample on its own).

CONTAINER-ONLY TOOL, same contract as make_golden.py (imports the reference from /root/reference with
the two unused import-time dependencies stubbed; only the written tensors travel):
    python tests/golden/make_golden_3d.py
"""
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF_SRC, OUT_DIR, _install_stubs  # noqa: E402


def main():
    _install_stubs()
    os.chdir(tempfile.mkdtemp())
    sys.path.insert(0, REF_SRC)
    import torch
    torch.set_num_threads(8)
    from models.enc_proc_dec_components.proc_fno import SpectralConv3d, FNO
    from models.enc_proc_dec_components.proc_unet_modern import UNetModern, Downsample
    from models.enc_proc_dec_components.proc_ufno import UFNO

    def save(name, **payload):
        path = os.path.join(OUT_DIR, f"{name}.pt")
        torch.save(payload, path)
        print(f"wrote {name}.pt  ({os.path.getsize(path) / 1024:.1f} KiB)")

    gen = torch.Generator().manual_seed(4321)

    def rnd(*shape, lo=-1.0, hi=1.0):
        return torch.rand(*shape, generator=gen) * (hi - lo) + lo

    # SpectralConv3d with grads: (a) corners overlap along D (2*m1 > D) and H (2*m2 > H), odd W;
    # (b) disjoint corners, Nyquist bin along W kept (m3 == W//2 + 1)
    cases = [
        ("spectral3d_overlap", dict(in_channels=3, out_channels=4, modes=(3, 3, 2)), (2, 3, 5, 4, 7)),
        ("spectral3d_nyq", dict(in_channels=4, out_channels=3, modes=(2, 3, 4)), (1, 4, 6, 8, 6)),
    ]
    for name, kw, xs in cases:
        torch.manual_seed(42)
        m = SpectralConv3d(**kw)
        x = rnd(*xs).requires_grad_(True)
        y = m(x)
        g = rnd(*y.shape)
        y.backward(g)
        save(name, kwargs=dict(kw, modes=list(kw["modes"])), state_dict=m.state_dict(), x=x.detach(), y=y.detach(),
             g=g, dx=x.grad, dw=[getattr(m, f"weights{i}").grad for i in range(1, 5)])

    # FNO-3D processor (proc_fno.py:22-83 with num_spatial_dims=3, concat conditioning, GELU layers)
    torch.manual_seed(42)
    kw = dict(num_spatial_dims=3, n_cond=2, hidden_features=6, fno_modes=(3, 4, 3), hidden_blocks=2,
              cond_mode="concat", fno_kernel_size=1, fno_conv_mode="single", padding_mode="circular")
    m = FNO(pde=None, **kw)
    h = rnd(2, 6, 6, 8, 6).requires_grad_(True)
    vb = rnd(2, 2, 6, 8, 6)
    y = m(h, variables_broadcast=vb)
    g = rnd(*y.shape)
    y.backward(g)
    save("fno3d", kwargs=dict(kw, fno_modes=list(kw["fno_modes"])), state_dict=m.state_dict(), h=h.detach(), vb=vb,
         y=y.detach(), g=g, dh=h.grad)

    # 3-D U-Net, single resolution (no Up/Downsample): ResidualBlocks of Conv3d, GroupNorm, crop_Nd, the
    # concat of h / skip / conditioning, the final GroupNorm(8) + 1x1x1 conv — proc_unet_modern.py:24-250
    with torch.no_grad():
        torch.manual_seed(42)
        kw = dict(num_spatial_dims=3, n_cond=2, hidden_features=8, cond_mode="concat", norm=True, ch_mults=[1],
                  is_attn=[False], mid_attn=False, n_blocks=1, use1x1=True, padding_mode="circular")
        m = UNetModern(pde=None, **kw)
        h, vb = rnd(2, 8, 9, 10, 12), rnd(2, 2, 9, 10, 12, lo=0.0)
        save("unet3d_single", kwargs=kw, state_dict=m.state_dict(), h=h, vb=vb, y=m(h, variables_broadcast=vb))
        # 3-D Downsample (valid 3x3x3 stride-2 conv on h and on the conditioning), proc_unet_modern.py:439-455
        torch.manual_seed(42)
        m = Downsample(8, num_spatial_dims=3, n_cond=2, padding_kwargs=dict(padding_mode="circular"))
        yh, yv = m(h, variables_broadcast=vb)
        save("downsample3d", state_dict=m.state_dict(), h=h, vb=vb, yh=yh, yv=yv)
        # 3-D U-FNO, single-resolution U-Nets (proc_ufno.py:25-118 with num_spatial_dims=3)
        torch.manual_seed(42)
        kw = dict(num_spatial_dims=3, n_cond=2, hidden_features=8, hidden_blocks=2, cond_mode="concat",
                  padding_mode="circular", fno_modes=(3, 4, 3), fno_kernel_size=1, fno_conv_mode="single", norm=True,
                  ch_mults=[1], is_attn=[False], mid_attn=False, n_blocks=1, use1x1=True)
        m = UFNO(pde=None, **kw)
        h, vb = rnd(2, 8, 8, 10, 12), rnd(2, 2, 8, 10, 12, lo=0.0)
        save("ufno3d_single", kwargs=dict(kw, fno_modes=list(kw["fno_modes"])), state_dict=m.state_dict(), h=h,
             vb=vb, y=m(h, variables_broadcast=vb))


if __name__ == "__main__":
    main()
