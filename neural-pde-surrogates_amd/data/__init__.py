"""On-disk dataset path (reference data/): memmap trajectories + conditioning, train/valid/test splits,
and the device-resident batch loader that replaces the per-step host->device copies."""
from data.base import DatasetInterface  # noqa: F401
from data.memmap_dataset import MemMapDataset  # noqa: F401
from data.PDE2D import PDE2DDataset  # noqa: F401
from data.device_loader import DeviceLoader  # noqa: F401
