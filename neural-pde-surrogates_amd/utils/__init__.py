"""Host utilities of the reference's `utils` package that the hot path and train.py import
(reference utils/__init__.py): attribute lookup, parameter count, seeding, misc helpers."""
import os
import random

import numpy as np
import torch

from .attr import getattr_nested, rgetattr, rsetattr  # noqa: F401
from . import misc  # noqa: F401


def count_parameters(model, provided_as_params=False):
    """Trainable parameter count of a module (or of an iterable of parameters)."""
    params = model if provided_as_params else model.parameters()
    return sum(p.numel() for p in params if p.requires_grad)


def set_seed(seed=1234):
    """Seed Python, numpy and torch (utils/set_seed.py:7-14; configs/parse.py:318 calls it with 42)."""
    random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
