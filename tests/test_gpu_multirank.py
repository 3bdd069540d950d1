"""SURVEY 8(e) on the device: N ranks, one process each, no collective on the
data path.  Two ranks share the box's one GPU over a gloo group (the rehearsal
mode of bench.py; the driver's 8-GPU node runs one rank per GPU over RCCL),
each scoring its shard through the product path.  The shards reassemble into
the unsharded launch bit for bit (the fused kernel is batch-invariant), and
bench.py's self-launched N-rank line reports the world it ran."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import bench

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_two_ranks_shard_equals_unsharded(tmp_path, precision):
    n_total = 4099   # ragged: 2050 + 2049
    out = tmp_path / "parts.json"
    rc = bench.spawn_ranks([sys.executable, os.path.join(HERE, "dist_gpu_worker.py"), str(out), str(n_total),
                            precision], 2, timeout=240)
    assert rc == 0
    res = json.loads(out.read_text())
    assert res["world"] == 2 and res["max_seconds"] > 0
    parts = sorted(res["parts"], key=lambda p: p["rank"])
    assert [(p["first"], p["count"]) for p in parts] == [(0, 2050), (2050, 2049)]
    sharded = np.concatenate([np.asarray(p["logits"], np.float32) for p in parts])
    whole = np.asarray(res["whole"], np.float32)
    assert np.isfinite(sharded).all()
    np.testing.assert_array_equal(sharded, whole)


@pytest.mark.gpu
def test_bench_self_launch_reports_world(tmp_path):
    """`bench.py --gpus 2` spawns two ranks itself (gloo here: they share the GPU);
    rank 0's line carries n_gpus = 2 and the process-group world it observed,
    and, the ranks sharing one GPU, is marked a rehearsal with no throughput."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "2",
           "--warmup", "1", "--batch", "8192", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["process_group_world_size"] == 2
    assert line["config"]["global_batch"] == 2 * 8192 and line["rehearsal"] is True
    assert line["value"] is None and line["roofline"]["frac"] is None and line["ms_per_step"] > 0
