"""Training / rollout drivers resolved by name from the cfgs (train.py:70: getattr(trainers, object))."""
from .base import TrainInterface  # noqa: F401
from .autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer  # noqa: F401
