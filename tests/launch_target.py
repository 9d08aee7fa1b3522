"""Rank body for tests/test_launch.py: what bench.py's spawned ranks do, on gloo.

argv: <expected_world> <out_dir> [fail_rank]. Brings the group up through
mme.launch.init_distributed, all-gathers every rank's id and writes it to
<out_dir>/rank<r>.txt; `fail_rank` exits 7 before joining the group."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mme import launch  # noqa: E402


def main():
    expected, out_dir = int(sys.argv[1]), sys.argv[2]
    fail_rank = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    rank, world, local = launch.env_rank_world()
    if rank == fail_rank:
        sys.exit(7)
    try:
        rank, world, local = launch.init_distributed(expected, "gloo")
    except launch.LaunchError as e:
        print(e, file=sys.stderr)
        sys.exit(3)
    ids = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(ids, torch.tensor([rank * 10 + local]))
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write(f"{world} {dist.get_backend()} " + " ".join(str(int(i)) for i in ids))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
