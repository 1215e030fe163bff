"""Mirror of the reference `models` package (src/models/__init__.py) backed by gfx950 HIP kernels."""
from common.launch import init_from_env

init_from_env()  # under torchrun: bind LOCAL_RANK's GPU before train.py:32 moves the model to "cuda"

from . import common  # noqa: F401,E402
from .enc_proc_dec import EncProcDec  # noqa: F401
from . import enc_proc_dec_components  # noqa: F401
from .activation_wrapper import activation_wrapper  # noqa: F401
