"""bench.py --gpus N brings up N ranks itself (VERDICT r4 Missing #1 / Next #1).

`python3 bench.py --gpus 2` — the driver's BENCH command form, no torchrun — must start two ranks (one
process per GPU) before any GPU call, for every mode; under a launcher whose WORLD_SIZE differs from --gpus
it must exit non-zero.  --launch-check runs the same bring-up (launcher, process group, rank -> shard of the
global batch) over gloo without touching a GPU, so this runs on the CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=180):
    env = dict(os.environ, NPS_BENCH_REHEARSAL="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("mode_args,gb", [([], 16), (["--mode", "train"], 16), (["--model", "ufno3d"], 8)])
def test_gpus_2_starts_two_ranks(mode_args, gb):
    r = _bench(["--gpus", "2", "--launch-check", *mode_args])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["dist"]["world_size"] == 2 and line["n_gpus"] == 2
    assert line["dist"]["backend"] == "gloo"
    assert line["shards"] == [[0, gb // 2], [gb // 2, gb]]


def test_gpus_1_is_one_process():
    r = _bench(["--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["dist"]["world_size"] == 1 and line["shards"] == [[0, 16]]


def test_world_size_mismatch_exits_nonzero():
    r = _bench(["--gpus", "2", "--launch-check"], env_extra=dict(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=4" in r.stderr


def test_indivisible_batch_exits_nonzero():
    r = _bench(["--gpus", "3", "--launch-check"])
    assert r.returncode != 0
