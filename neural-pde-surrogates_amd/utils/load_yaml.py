"""utils/load_yaml.py: dataset metadata (snapshots.yaml, split.yaml) are plain lists / scalars, read with
the safe loader."""
import yaml


def load_yaml(path):
    with open(path, "r") as f:
        return yaml.load(f, Loader=yaml.SafeLoader)
