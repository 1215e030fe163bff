"""Training / rollout drivers resolved by name from the cfgs (train.py:70: getattr(trainers, object))."""
from common.launch import init_from_env

init_from_env()  # under torchrun: bind LOCAL_RANK's GPU and open the group before train.py builds anything

from .base import TrainInterface  # noqa: F401,E402
from .autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer  # noqa: F401
