"""Worker for tests/test_gpu_multirank.py: one rank of a gloo world (ranks may
share the GPU, as in bench.py's gloo rehearsal), launched by bench.spawn_ranks.

Each rank scores its shard of the global clip range (wakeword.shard.
shard_range) through the product path (device generator -> wk_forward, fused
HIP kernel), with bench.py's barrier + max-over-ranks timing; the logits are
gathered on the host only for the check, and rank 0 writes them with its own
unsharded run of the whole range to the output file."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "esp32-wake-word_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import wakeword  # noqa: E402
from wakeword.shard import shard_range  # noqa: E402


def main():
    out_path, n_total, precision = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    model = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), precision=precision)
    first, count = shard_range(n_total, rank, world)
    x = wakeword.synth_clips(1234, first, count) if count else None
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    logits = model.detect(x) if count else None
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    model.check_device_errors()
    part = {"rank": rank, "first": first, "count": count,
            "logits": logits.cpu().numpy().tolist() if count else []}
    parts = [None] * world
    dist.all_gather_object(parts, part)
    if rank == 0:
        whole = model.detect(wakeword.synth_clips(1234, 0, n_total)).cpu().numpy().tolist()
        with open(out_path, "w") as fh:
            json.dump({"world": world, "max_seconds": float(t[0]), "parts": parts, "whole": whole}, fh)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
