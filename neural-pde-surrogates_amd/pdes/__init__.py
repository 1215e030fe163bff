"""PDE metadata (reference pdes/base.py:4-52): only `dt` and the grid reach the hot path."""
import torch


class PDE:
    def __init__(self, tmin, tmax, nt, name, n_cond_static=0, n_cond_dynamic=0, n_cond_spatial=0, **kwargs):
        self.tmin = tmin
        self.tmax = tmax
        self.nt = nt
        self.name = name
        self.n_cond_static = n_cond_static
        self.n_cond_dynamic = n_cond_dynamic
        self.n_cond_spatial = n_cond_spatial
        for k, v in kwargs.items():
            setattr(self, k, v)

    def __repr__(self):
        return self.name


class PDE2D(PDE):
    def __init__(self, tmin, tmax, nt, L1, L2, nx1, nx2, x, name, n_cond_static=0, n_cond_dynamic=0,
                 n_cond_spatial=0, **kwargs):
        super().__init__(tmin, tmax, nt, name, n_cond_static, n_cond_dynamic, n_cond_spatial, **kwargs)
        self.L1, self.L2 = L1, L2
        self.L = [L1, L2]
        self.nx1, self.nx2 = nx1, nx2
        self.dt = self.tmax / (nt - 1)  # pdes/base.py:43
        self.dx1 = self.L1 / (nx1 - 1)
        self.dx2 = self.L2 / (nx2 - 1)
        self.dxs = [self.dx1, self.dx2]
        if x is None:
            xs = [torch.linspace(0, L1, nx1), torch.linspace(0, L2, nx2)]
            x = torch.movedim(torch.stack(torch.meshgrid(*xs, indexing="ij")), 0, -1)
        self.x = x
