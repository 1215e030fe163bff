"""CPU oracle for the neural-operator rollout hot path — TEST INFRASTRUCTURE ONLY.

This package is a functional fp32 PyTorch-CPU restatement of the reference
(yoeripoels/neural-pde-surrogates, snapshot 2025-02-24) forward path: the
SpectralConv2d/3d, FNO/U-FNO, modern U-Net and dilated ResNet processors, the
grid encoder/decoder, the `activation_wrapper` post-processing and the
`simulate` rollout loop.  Every function cites the reference file:line it
restates.

It is pinned against golden vectors generated from the reference itself
(`tests/golden/make_golden.py`, fixtures in `tests/golden/*.pt`; checked by
`tests/test_oracle_golden.py`).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import this package.  The product path (`neural-pde-surrogates_amd/`)
never imports it and fails loudly when its HIP library is missing.
"""
from .functional import *  # noqa: F401,F403
from .model import OracleModel, build_oracle_model  # noqa: F401
from .rollout import simulate  # noqa: F401
