from . import enc_grid  # noqa: F401
from . import dec_grid  # noqa: F401
from .proc_dilatedresnet import DilatedResnet  # noqa: F401
from .proc_fno import FNO  # noqa: F401
from .proc_unet_modern import UNetModern  # noqa: F401
from .proc_ufno import UFNO  # noqa: F401
