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


def test_launcher_world_is_the_default(monkeypatch):
    """torchrun --nproc-per-node N bench.py (no --gpus): the expected size is the launcher's."""
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert launch.init_distributed(None, "gloo") == (0, 1, 0)


def test_same_device_needs_gloo(monkeypatch):
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(launch.LaunchError, match="gloo"):
        launch.init_distributed(2, "nccl", same_device=True)


def test_sigterm_to_the_parent_ends_the_ranks(tmp_path):
    """A job timeout's SIGTERM to the spawning parent must not orphan the ranks."""
    import signal
    import time
    script = tmp_path / "parent.py"
    script.write_text(
        "import sys\n"
        f"sys.path.insert(0, {os.path.join(os.path.dirname(HERE), 'multimodal-embedding_amd')!r})\n"
        "from mme import launch\n"
        "sys.exit(launch.spawn_ranks(2, ['-c', 'import os, time; "
        f"open(r\"{tmp_path}/pid%s\" % os.environ[\"RANK\"], \"w\").write(str(os.getpid())); time.sleep(300)']))\n")
    env = {k: v for k, v in os.environ.items() if k not in launch.ENV_KEYS}
    p = subprocess.Popen([sys.executable, str(script)], env=env)
    t0 = time.time()
    while not all((tmp_path / f"pid{r}").exists() for r in range(2)) and time.time() - t0 < 60:
        time.sleep(0.1)
    pids = [int((tmp_path / f"pid{r}").read_text()) for r in range(2)]
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) == 128 + signal.SIGTERM
    for pid in pids:
        try:
            os.kill(pid, 0)
            # a zombie is reaped by its parent, which has exited; /proc shows its state
            with open(f"/proc/{pid}/status") as f:
                assert "zombie" in f.read()
        except ProcessLookupError:
            pass
