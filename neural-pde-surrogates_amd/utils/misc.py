"""Host-side helpers the training driver and train.py use (reference utils/misc.py): a flushing stdout
tee, the experiment directories, float conversion of loss dicts, dict pretty-printing and the
batch-size probe of a collated batch.  Nothing here touches the device."""
import os
from typing import Dict, List, Union

import torch


class Logger:
    """File-like stdout wrapper that flushes every write (train.py:104-105 installs it as sys.stdout);
    with write_log the text is also appended to `filename`."""

    def __init__(self, default_stdout, write_log=True, filename="log.txt"):
        self.terminal = default_stdout
        self.write_log = write_log
        self.log = open(filename, "a") if write_log else None

    def write(self, message):
        for stream in (self.log, self.terminal):
            if stream is not None:
                stream.write(message)
                stream.flush()

    def flush(self):
        for stream in (self.log, self.terminal):
            if stream is not None:
                stream.flush()

    def __getattr__(self, attr):
        return getattr(self.terminal, attr)


def check_directory() -> None:
    """The relative output directories TrainInterface.train expects (experiments/log, models/output)."""
    for d in ("experiments", os.path.join("experiments", "log"), os.path.join("models", "output")):
        if not os.path.exists(d):
            os.mkdir(d)


def to_float(x: Union[float, torch.Tensor]) -> float:
    return x if isinstance(x, float) else x.item()


def to_floatdict(x: Dict[str, Union[float, torch.Tensor]]) -> Dict[str, float]:
    return {k: to_float(v) for k, v in x.items()}


def to_floatlist(x: List[Union[float, torch.Tensor]]) -> List[float]:
    return [to_float(v) for v in x]


def dict_str(x: dict, prefix: str = "", mapping: str = ": ", postfix: str = "", subdir_prefix: str = "  ") -> str:
    """One `prefix key mapping value postfix` line per entry; nested dicts indented by subdir_prefix."""
    lines = []
    for k, v in x.items():
        if isinstance(v, dict):
            inner = dict_str(v, prefix=subdir_prefix + prefix, mapping=mapping, postfix=postfix)
            lines.append(f"{prefix}{k}{mapping}\n{inner}{postfix}")
        else:
            lines.append(f"{prefix}{k}{mapping}{v}{postfix}")
    return "\n".join(lines)


def get_batch_size(batch) -> int:
    """Leading size shared by every tensor / list of a collated batch (the sample count)."""
    sizes = [x.shape[0] if isinstance(x, torch.Tensor) else len(x) for x in batch
             if isinstance(x, (torch.Tensor, list))]
    if not sizes:
        raise ValueError("Could not determine elements_in_batch from batch of data!")
    if any(s != sizes[0] for s in sizes):
        raise AssertionError(f"inconsistent batch sizes {sizes}")
    return sizes[0]


def default(value, d):
    return d if value is None else value
