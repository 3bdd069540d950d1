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


class _FakeCuda:
    def __init__(self, n):
        self.n, self.current = n, None

    def device_count(self):
        return self.n

    def set_device(self, d):
        self.current = d


class _FakeTorch:
    def __init__(self, n):
        self.cuda = _FakeCuda(n)

    @staticmethod
    def device(s):
        return ("device", s)


class _FakeDist:
    def __init__(self):
        self.calls = []

    def init_process_group(self, backend, **kw):
        self.calls.append((backend, kw))


def _args(gpus, backend):
    import argparse
    return argparse.Namespace(gpus=gpus, dist_backend=backend)


def test_init_rank_nccl_binds_each_rank_to_its_device():
    """The RCCL branch: each rank of 4 gets its own GPU as device_id."""
    for r in range(4):
        env = {"WORLD_SIZE": "4", "RANK": str(r), "LOCAL_RANK": str(r)}
        t, d = _FakeTorch(8), _FakeDist()
        world, rank, local, shared = bench.init_rank(_args(4, "nccl"), env, t, d)
        assert (world, rank, local, shared) == (4, r, r, False)
        assert t.cuda.current == r
        assert d.calls == [("nccl", {"device_id": ("device", f"cuda:{r}")})]
        assert env["MASTER_ADDR"] == "127.0.0.1"


def test_init_rank_nccl_refuses_missing_gpu():
    import pytest
    env = {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.init_rank(_args(2, "nccl"), env, _FakeTorch(1), _FakeDist())


def test_init_rank_gloo_rehearsal_is_marked_shared():
    """Two gloo ranks on one GPU: both use device 0 and the line is a rehearsal."""
    for r in range(2):
        env = {"WORLD_SIZE": "2", "RANK": str(r), "LOCAL_RANK": str(r)}
        t, d = _FakeTorch(1), _FakeDist()
        world, rank, local, shared = bench.init_rank(_args(2, "gloo"), env, t, d)
        assert (world, local, shared) == (2, 0, True)
        assert d.calls == [("gloo", {})]


def test_init_rank_multinode_is_not_a_rehearsal():
    """torchrun over 2 nodes x 8 GPUs: WORLD_SIZE 16 > 8 visible GPUs, but 8
    ranks per node (LOCAL_WORLD_SIZE), one GPU each -- a real measurement."""
    for r in (0, 9, 15):
        env = {"WORLD_SIZE": "16", "RANK": str(r), "LOCAL_RANK": str(r % 8), "LOCAL_WORLD_SIZE": "8"}
        t, d = _FakeTorch(8), _FakeDist()
        world, rank, local, shared = bench.init_rank(_args(16, "nccl"), env, t, d)
        assert (world, rank, local, shared) == (16, r, r % 8, False)


def test_single_rank_forms_no_group():
    env = {}
    t, d = _FakeTorch(1), _FakeDist()
    assert bench.init_rank(_args(1, "nccl"), env, t, d) == (1, 0, 0, False)
    assert d.calls == []


def test_host_threads_reports_affinity():
    threads, affinity, quota = bench.host_threads()
    assert affinity == len(os.sched_getaffinity(0))
    assert 1 <= threads <= affinity
    assert quota is None or threads <= quota


def test_committed_profiles_feed_the_bench_line():
    """The roofline's traffic and utilisation come from committed rocprofv3
    PMC summaries (profiles/): both present for fp32 and bf16, shares in (0, 1]."""
    for prec in ("fp32", "bf16"):
        bpw, src = bench.load_traffic(prec)
        assert bpw and 64_004 * 0.99 < bpw < 64_004 * 1.1, (prec, bpw)
        u = bench.load_utilisation(prec)
        assert u is not None and u["source"].startswith("profiles/")
        assert 0.0 < u["valu_active"] <= 2.0 and 0.0 < u["mfma_busy"] <= 1.0
    assert bench.FLOP_PER_WINDOW == 2_262_440
