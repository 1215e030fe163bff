"""On-disk dataset path (reference data/): memmap trajectories + conditioning, train/valid/test splits,
and the device-resident batch loader that replaces the per-step host->device copies."""
from common.launch import init_from_env

init_from_env()  # under torchrun (train.py:17 imports data first): see common/launch.py

from data.base import DatasetInterface  # noqa: F401,E402
from data.memmap_dataset import MemMapDataset  # noqa: F401
from data.PDE2D import PDE2DDataset  # noqa: F401
from data.device_loader import DeviceLoader  # noqa: F401
