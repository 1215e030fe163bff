"""ModelInterface (reference models/base.py:1-74)."""
from abc import abstractmethod, ABCMeta
from typing import List

import torch

from common.interfaces import M, D


class ModelInterface(torch.nn.Module, metaclass=ABCMeta):
    @property
    @abstractmethod
    def model_interface(self) -> M:
        raise NotImplementedError("model_interface not set!")

    @property
    @abstractmethod
    def data_interface(self) -> List[D]:
        return []

    def embed_conditioning_signal(self, cond: torch.Tensor = None, boundary_conditions: torch.Tensor = None,
                                  t_cond: torch.Tensor = None, spatial_cond: torch.Tensor = None,
                                  unsqueeze_dims: int = 0):
        """base.py:24-73.  The stack of cond columns is cond itself; bc / t_cond need a bc_encoder,
        which the grid path does not build."""
        if cond is not None and torch.numel(cond) == 0:
            cond = None
        if boundary_conditions is not None and torch.numel(boundary_conditions) == 0:
            boundary_conditions = None
        if t_cond is not None and torch.numel(t_cond) == 0:
            t_cond = None
        if (boundary_conditions is not None or t_cond is not None) and getattr(self, "bc_encoder", None) is not None:
            raise NotImplementedError("bc_encoder conditioning is not on the MI355X path")
        if cond is None:
            return None
        variables = cond.reshape(cond.shape[0], -1).float().contiguous()
        for _ in range(unsqueeze_dims):
            variables = variables.unsqueeze(-1)
        return variables
