"""Encode-Process-Decode grid model (reference models/enc_proc_dec.py).

`create_model` resolves component names exactly like the reference
(enc_proc_dec.py:14-38), against this package.  The forward packs
[u | pos | cond | spatial_cond] into one NHWC tensor with one HIP kernel and
then runs encoder -> processors -> decoder as fused HIP launches on NHWC
tensors; only the final (B, c, tw, H, W) output leaves that layout.
"""
from argparse import Namespace
from typing import Union

import torch
from torch import nn

from models.base import ModelInterface
from nps_hip import ops
from nps_hip import autograd as ad
from pdes import PDE
from utils.attr import getattr_nested


def create_model(model: Union[nn.Module, dict, Namespace, str], pde: PDE, base_args: dict, extra_kwargs: dict = None):
    """enc_proc_dec.py:14-38."""
    import models
    if isinstance(model, nn.Module):
        return model
    if isinstance(model, (dict, Namespace, str)):
        if isinstance(model, str):
            model_class = model
            model_kwargs = dict(base_args)
        else:
            if isinstance(model, Namespace):
                model = vars(model)
            model = dict(model)
            model_class = model.pop("object")
            model_kwargs = dict(list(base_args.items()) + list(model.items()))
        if extra_kwargs is not None:
            model_kwargs = dict(list(model_kwargs.items()) + list(extra_kwargs.items()))
        for module in [models.enc_proc_dec_components, models, models.common]:
            if (model_init := getattr_nested(module, model_class)) is not False:
                return model_init(**model_kwargs, pde=pde)
        raise ValueError(f"Cannot find object {model_class} in any of the model modules")
    raise ValueError("Model was not the correct type: Should be nn.Module / dict / argparse.Namespace")


class EncProcDec(ModelInterface):
    """enc_proc_dec.py:41-183."""

    def __init__(self, pde: PDE, encoder, processor, decoder, bc_encoder=None, num_c: int = 1,
                 num_spatial_dims: int = 1, time_window: int = 25, data_structure: str = "grid",
                 processor_residual: bool = False, **base_args):
        super().__init__()
        self.pde = pde
        self.num_c = num_c
        self.num_spatial_dims = num_spatial_dims
        self.time_window = time_window
        self.processor_residual = processor_residual
        self.data_structure = data_structure
        base_args["num_c"] = num_c
        base_args["num_spatial_dims"] = num_spatial_dims
        base_args["time_window"] = time_window
        if bc_encoder is not None:
            self.bc_encoder = create_model(bc_encoder, self.pde, base_args,
                                           extra_kwargs=dict(bc_encoder_in=self.pde.n_cond_dynamic))
            self.n_cond = self.pde.n_cond_static + self.pde.n_cond_spatial + self.bc_encoder.n_out
        else:
            self.bc_encoder = None
            self.n_cond = self.pde.n_cond_static + self.pde.n_cond_spatial
        base_args["n_cond"] = self.n_cond
        self.encoder = create_model(encoder, self.pde, base_args)
        if isinstance(processor, (list, tuple)):
            self.processor = nn.ModuleList([create_model(p, self.pde, base_args) for p in processor])
        else:
            self.processor = nn.ModuleList([create_model(processor, self.pde, base_args)])
        self.decoder = create_model(decoder, self.pde, base_args)

    def __repr__(self):
        return f'{self.encoder}-{self.processor}-{self.decoder}'

    @property
    def model_interface(self):
        mi = [p.model_interface for p in self.processor]
        assert mi.count(mi[0]) == len(mi), "Not all processors have the same model interface!"
        return mi[0]

    @property
    def data_interface(self):
        return set.intersection(*[set(p.data_interface) for p in self.processor])

    def forward_fused(self, x, cond=None, bc=None, pos=None, t_cond=None, spatial_cond=None, final_tanh=False,
                      mask_channel=None):
        """EncProcDec.forward (enc_proc_dec.py:117-183, grid branch) with the optional activation_wrapper
        tanh + spatial-cond mask fused into the decoder kernel."""
        check_none = lambda v: None if (v is None or torch.numel(v) == 0) else v
        cond, bc, pos, t_cond, spatial_cond = map(check_none, (cond, bc, pos, t_cond, spatial_cond))
        if self.data_structure != "grid":
            raise NotImplementedError("graph data_structure is deprecated in the reference and not built")
        if self.num_spatial_dims != 2:
            raise NotImplementedError("EncProcDec: 2-D grids only on the MI355X path")
        if not x.is_cuda:
            raise RuntimeError("nps: the model runs on the MI355X; move inputs to the GPU")
        u = x.contiguous()
        variables = self.embed_conditioning_signal(cond, bc, t_cond)
        sc = spatial_cond.float().contiguous() if spatial_cond is not None else None
        n_in = self.encoder.n_in
        Cp = ((n_in + 3) // 4) * 4
        xin, vb = ops.pack_grid_input(u, pos.float().contiguous(), variables, sc, Cp)
        mask = sc if mask_channel is not None else None
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            # training: the same kernels unfused, each with its HIP backward (nps_hip.autograd)
            h = self.encoder.run_packed_ad(xin)
            for i, p in enumerate(self.processor):
                h_next = p.run_ad(h, vb)
                h = ad.add_at(h_next, h) if (self.processor_residual and i > 0) else h_next
            return self.decoder.run_ad(h, u, final_tanh=final_tanh, mask=mask, mask_ch=mask_channel or 0)
        h = self.encoder.run_packed(xin)
        for i, p in enumerate(self.processor):
            h_next = p.run(h, vb)
            if self.processor_residual and i > 0:
                h_next = h_next + h
            h = h_next
        return self.decoder.run(h, u, final_tanh=final_tanh, mask=mask, mask_ch=mask_channel or 0)

    def forward(self, x, cond=None, bc=None, pos=None, t_cond=None, spatial_cond=None):
        return self.forward_fused(x, cond=cond, bc=bc, pos=pos, t_cond=t_cond, spatial_cond=spatial_cond)
