"""Worker for tests/test_sharding.py (launched by torch.distributed.run, gloo, CPU).

Each rank runs the CPU oracle path over its shard of the global clip range
(wakeword.shard.shard_range), with bench.py's barrier + max-over-ranks timing
pattern, and rank 0 writes all ranks' logits (gathered only for the check) to
the output file."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import wk_oracle as O  # noqa: E402
from oracle.wk_torch_cpu import TorchCpuPath  # noqa: E402
from wakeword.onnx_reader import read_onnx, xiaoa_state_dict  # noqa: E402
from wakeword.shard import shard_range  # noqa: E402


def main():
    out_path, n_total = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.set_num_threads(1)
    inits, _, _ = read_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"))
    path = TorchCpuPath(xiaoa_state_dict(inits))
    first, count = shard_range(n_total, rank, world)
    x = torch.from_numpy(O.synth_clips(1234, first, count))
    dist.barrier()
    t0 = time.perf_counter()
    with torch.no_grad():
        logits = path(x).reshape(-1).numpy().tolist() if count else []
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    parts = [None] * world
    dist.all_gather_object(parts, {"rank": rank, "first": first, "count": count, "logits": logits})
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump({"world": world, "max_seconds": float(t[0]), "parts": parts}, fh)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
