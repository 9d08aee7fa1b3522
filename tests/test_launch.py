"""bench.py --gpus N without torchrun: mme.launch spawns N ranks and checks the group size.

Runs the launcher on the CPU with gloo (the ranks are tests/launch_target.py, which
does what bench.py's ranks do up to the first collective)."""
import os
import subprocess
import sys

import pytest

from mme import launch

HERE = os.path.dirname(os.path.abspath(__file__))
TARGET = os.path.join(HERE, "launch_target.py")


@pytest.fixture(autouse=True)
def _no_outer_group(monkeypatch):
    for k in launch.ENV_KEYS:
        monkeypatch.delenv(k, raising=False)


@pytest.mark.parametrize("world", [2, 4])
def test_spawn_ranks_builds_the_requested_group(tmp_path, world):
    rc = launch.spawn_ranks(world, [TARGET, str(world), str(tmp_path)], timeout_s=120)
    assert rc == 0
    for r in range(world):
        w, backend, *ids = (tmp_path / f"rank{r}.txt").read_text().split()
        assert int(w) == world and backend == "gloo"
        assert [int(i) for i in ids] == [11 * q for q in range(world)]  # rank q has local rank q


def test_failing_rank_fails_the_job(tmp_path):
    rc = launch.spawn_ranks(3, [TARGET, "3", str(tmp_path), "1"], timeout_s=120)
    assert rc == 7


def test_world_size_mismatch_is_an_error(monkeypatch):
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(launch.LaunchError):
        launch.init_distributed(8, "gloo")


def test_single_rank_needs_no_group():
    assert launch.init_distributed(1, "gloo") == (0, 1, 0)
    assert not launch.under_launcher()


def test_bench_parent_spawns_before_touching_the_gpu(tmp_path):
    """bench.py --gpus 2 in a process with no launcher environment re-runs itself as 2 ranks;
    on this GPU-less box each rank fails at its first device call, so the parent must exit
    non-zero (never a silent single-process n_gpus=1 line)."""
    env = {k: v for k, v in os.environ.items() if k not in launch.ENV_KEYS}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2", "--steps",
                        "1", "--warmup", "0"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout
