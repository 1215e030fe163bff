"""Mirror of the reference `models` package (src/models/__init__.py) backed by gfx950 HIP kernels."""
from . import common  # noqa: F401
from .enc_proc_dec import EncProcDec  # noqa: F401
from . import enc_proc_dec_components  # noqa: F401
from .activation_wrapper import activation_wrapper  # noqa: F401
