"""Multi-GPU partitioning exercised on CPU: the shard ranges, and
a world_size-2 gloo run whose per-rank results reassemble into the unsharded
result clip for clip (no collective on the data path; gather only to check)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from wakeword.shard import shard_range, weak_shard

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 2), (8, 8), (65536, 8), (1048576, 8), (13, 5)])
def test_shard_range_partitions(n, world):
    ranges = [shard_range(n, r, world) for r in range(world)]
    covered = []
    for first, count in ranges:
        covered.extend(range(first, first + count))
    assert covered == list(range(n))                       # disjoint, ordered, complete
    counts = [c for _, c in ranges]
    assert max(counts) - min(counts) <= 1                   # balanced


def test_shard_range_rejects_bad_requests():
    for args in [(10, 2, 2), (10, -1, 2), (10, 0, 0), (-1, 0, 1)]:
        with pytest.raises(ValueError):
            shard_range(*args)


def test_weak_shard_is_disjoint_per_rank():
    assert [weak_shard(4, r) for r in range(3)] == [(0, 4), (4, 4), (8, 4)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_world2_sharded_equals_unsharded(tmp_path, xiaoa_sd):
    import torch
    from oracle import wk_oracle as O
    from oracle.wk_torch_cpu import TorchCpuPath
    n_total = 5
    out = tmp_path / "shards.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "dist_shard_worker.py"), str(out), str(n_total)]
    subprocess.run(cmd, check=True, env=env, timeout=300, capture_output=True)
    res = json.loads(out.read_text())
    assert res["world"] == 2 and res["max_seconds"] > 0
    parts = sorted(res["parts"], key=lambda p: p["rank"])
    assert [(p["first"], p["count"]) for p in parts] == [(0, 3), (3, 2)]
    sharded = np.concatenate([np.asarray(p["logits"], np.float32) for p in parts])
    with torch.no_grad():
        whole = TorchCpuPath(xiaoa_sd)(torch.from_numpy(O.synth_clips(1234, 0, n_total))).reshape(-1).numpy()
    # The torch-CPU path is not bit batch-invariant (BLAS blocking differs with
    # the batch size); the HIP path is, see test_gpu_parity.py
    # test_deterministic_and_batch_invariant.
    np.testing.assert_allclose(sharded, whole, rtol=0, atol=1e-5)
