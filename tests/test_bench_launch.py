"""bench.py's self-launch of N ranks (one process per GPU, no
collective on the data path): the torchrun-style environment per rank, a
gloo process group formed by the spawned children, and failure propagation.
CPU only -- the children here are small Python programs, not the GPU bench."""
import os
import sys
import time

import bench

CHILD_GROUP = r"""
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
assert r == int(os.environ["RANK"]) == int(os.environ["LOCAL_RANK"]) and w == int(os.environ["WORLD_SIZE"])
t = torch.tensor([float(r)])
dist.all_reduce(t, op=dist.ReduceOp.MAX)
open(os.path.join(sys.argv[1], f"rank{r}"), "w").write(f"{w} {int(t.item())}")
dist.destroy_process_group()
"""

CHILD_FAIL = r"""
import os, sys, time
if os.environ["RANK"] == "1":
    sys.exit(5)
time.sleep(60)
"""


def test_rank_envs_torchrun_style():
    envs = bench.rank_envs(3, 29555, base={"PATH": "/usr/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["PATH"] == "/usr/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_spawned_ranks_form_one_group(tmp_path):
    rc = bench.spawn_ranks([sys.executable, "-c", CHILD_GROUP, str(tmp_path)], 2, timeout=120)
    assert rc == 0
    assert sorted(os.listdir(tmp_path)) == ["rank0", "rank1"]
    for r in range(2):
        assert (tmp_path / f"rank{r}").read_text() == "2 1"      # world 2, max over ranks 1


def test_failing_rank_stops_the_launch():
    t0 = time.monotonic()
    rc = bench.spawn_ranks([sys.executable, "-c", CHILD_FAIL], 3, timeout=120)
    assert rc == 5
    assert time.monotonic() - t0 < 30          # the sleeping ranks were terminated


def test_world_size_must_match_gpus(monkeypatch):
    """Under torchrun, --gpus must equal WORLD_SIZE (no silent 1-rank run)."""
    import pytest
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()
