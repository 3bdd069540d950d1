"""bench.py -- windows/s of the MI355X wake-word hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Started without torchrun (WORLD_SIZE unset) and with --gpus N > 1, the
process launches N ranks itself before touching the GPU: N fresh child
processes of this script with torchrun's environment (RANK = LOCAL_RANK = i,
WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a free MASTER_PORT), one GPU each, and
exits with the first failing child's status.  Every rank checks its handle's
device error word after the timed region (wk_check_device_errors, outside the
timing); a flag on any rank means a role hand-off aborted and the logits are
invalid, and then no bench line is printed (exit status 3).

One step = one pass of the hot path (1 s @ 16 kHz audio -> MFCC (torchaudio
definition + CMVN) -> xiaoa CNN -> logit, fp32) over one batch of B synthetic
clips that are already resident in HBM (B = 65,536 per
GPU).  Multi-GPU = one process per GPU, each rank takes its own contiguous
range of global clip indices (weak scaling, no collective on the data path;
torch.distributed is used only for the barrier and the max-over-ranks time).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "esp32-wake-word_amd"))
sys.path.insert(0, REPO)

# Algorithmic work per window: front-end 960,744 + CNN 1,301,696 flop.
FLOP_FE = 960_744
FLOP_CNN = 1_301_696
FLOP_PER_WINDOW = FLOP_FE + FLOP_CNN
BYTES_PER_WINDOW_F32 = 64_004          # 16000 fp32 samples in + 1 fp32 logit out
PEAK_FP32_TFLOPS = 157.3               # MI355X fp32 vector == fp32 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0              # MI355X dense bf16 MFMA


def roofline_peak(precision: str):
    """(peak TFLOP/s, basis) of the fused kernel for a precision.  fp32 and the
    fp32-grade split-bf16 path are priced at the fp32 peak: every flop of the
    algorithm is fp32 work (bf16x3 reproduces fp32 convolutions, and its three
    bf16 products per fp32 product are not algorithmic work).  The bf16 path runs
    the front-end's 960,744 flop on the fp32 pipes and the CNN's 1,301,696 on
    the bf16 matrix cores; on one SIMD the two do not overlap
    (tools/debug/mfma_rate.hip), so its ceiling is the two times in series:
    2,262,440 / (960,744 / 157.3 T + 1,301,696 / 2.5 P) = 341 TFLOP/s."""
    if precision == "bf16":
        t = FLOP_FE / (PEAK_FP32_TFLOPS * 1e12) + FLOP_CNN / (PEAK_BF16_TFLOPS * 1e12)
        return FLOP_PER_WINDOW / t / 1e12, "front-end on the fp32 pipes + CNN on bf16 MFMA, in series"
    return PEAK_FP32_TFLOPS, "fp32 VALU / fp32 MFMA (equal peaks on MI355X)"


# --precision -> (dtype, workload) of the bench line
PRECISIONS = {
    "fp32": ("f32", "config2: fused MFCC(torchaudio+CMVN)+xiaoa CNN fp32, B clips per GPU"),
    "bf16": ("bf16 convolutions, f32 front-end/classifier",
             "config4: fused MFCC(torchaudio+CMVN) fp32 + xiaoa CNN bf16, B clips per GPU"),
    "bf16x3": ("f32-grade convolutions as split bf16 (hi*hi + hi*lo + lo*hi, f32 accumulate), f32 front-end/classifier",
               "config2: fused MFCC(torchaudio+CMVN)+xiaoa CNN at the fp32 logit tolerance, B clips per GPU"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="clips per GPU per step")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--audio", default="f32", choices=["f32", "i16"],
                    help="sample type of the resident clips: f32 (the metric's workload, 64,000 B/window) or "
                         "i16 PCM (32,000 B/window, scaled by 1/32768 on load)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for the start/stop barriers and the max-over-ranks time (nccl = "
                         "RCCL over xGMI; gloo lets several ranks share one GPU for a rehearsal of the N>1 path)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the config 4 / 5 / 3 measurements added to the line after the headline (N=1 only)")
    ap.add_argument("--precision", default="fp32", choices=list(PRECISIONS),
                    help="CNN convolutions: fp32 MFMA (config 2, default), bf16 (config 4), or bf16x3 "
                         "(config 2 at fp32-grade accuracy on split-bf16 MFMA); front-end fp32 always")
    return ap.parse_args()


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_envs(n: int, port: int, base=None):
    """torchrun's per-rank environment for n local ranks (one GPU each)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "ROLE_RANK": str(r), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                  "TORCHELASTIC_RUN_ID": "bench"})
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL (the host driver's only mode)
        envs.append(e)
    return envs


def spawn_ranks(argv, n: int, timeout: float = None) -> int:
    """Run `argv` as n ranks (child processes, torchrun-style env) and wait.
    Returns 0 if all ranks succeed, else the first failing rank's status (the
    others are terminated).  Called before any GPU call in this process."""
    procs = [subprocess.Popen(argv, env=e) for e in rank_envs(n, free_port())]
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0 and rc == 0:
                    rc = r if r > 0 else 128 - r
                    for q in pending:
                        q.terminate()
            if deadline is not None and time.monotonic() > deadline and pending:
                rc = rc or 124
                for q in pending:
                    q.kill()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def host_threads():
    """CPU threads this process may run on: the affinity mask, capped by the
    cgroup CPU quota when one is set (a GPU box shows the whole machine's CPUs
    in its affinity mask but grants each GPU a share of them)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


CPU_BATCHES = (256, 4096)   # BASELINE.md section 3 / SURVEY 8(d): batch 256 and 4096


def cpu_baseline(seconds: float, batches=CPU_BATCHES):
    """The ml_models CPU path (torch fp32 restatement, oracle/wk_torch_cpu.py) on
    the host cores, timed on a bounded sample of the same synthetic workload:
    about seconds / len(batches) per batch size, all host threads
    (torch.set_num_threads), outside any GPU timing.  `value` is the best of
    the batch sizes; every batch size's rate is listed."""
    import torch
    from oracle import wk_oracle as O
    from oracle.wk_torch_cpu import TorchCpuPath
    from wakeword.onnx_reader import read_onnx, xiaoa_state_dict
    threads, affinity, quota = host_threads()
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        inits, _, _ = read_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"))
        path = TorchCpuPath(xiaoa_state_dict(inits))
        per = {}
        parts = []
        for batch in batches:
            x = torch.from_numpy(O.synth_clips(1234, 0, batch))
            path(x)  # warm-up
            n, t0 = 0, time.perf_counter()
            while True:
                path(x)
                n += batch
                el = time.perf_counter() - t0
                if el >= seconds / len(batches) and n >= 2 * batch:
                    break
            per[str(batch)] = round(n / el, 1)
            parts.append(f"batch {batch}: {n} windows in {el:.1f} s")
    finally:
        torch.set_num_threads(old)
    best = max(per, key=per.get)
    return {"value": per[best], "unit": "windows/s", "cores": threads, "batch": int(best),
            "by_batch": per, "host_cpus": affinity, "cgroup_cpu_quota": quota,
            "kind": "port",
            "sample": "; ".join(parts) + " (synthetic clips, seed 1234); torch-CPU fp32 restatement of the "
                      "torchaudio MFCC+CMVN front-end + LightweightKWS on the xiaoa.onnx weights "
                      f"(oracle/wk_torch_cpu.py), torch.set_num_threads({threads})"}


CONFIG4_CLIPS = 131_072   # 1,048,576 clips over 8 GPUs = 131,072 per rank
HBM_ROOF_F32_WPS = PEAK_HBM_GBS * 1e9 / BYTES_PER_WINDOW_F32   # 125.0 M windows/s with fp32 audio


def extra_config4(torch, wakeword, _lib, local, seed, steps=10, warmup=2):
    """Config 4 on this GPU: one rank's share (131,072 clips) through the fused
    kernel with bf16 convolutions, fp32 audio resident in HBM.  Its governing
    roof is HBM (125 M windows/s with fp32 input); the blended
    compute ceiling of roofline_peak("bf16") is listed beside it."""
    B = CONFIG4_CLIPS
    model = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), device=local, precision="bf16")
    clips = wakeword.synth_clips(seed, 0, B, 16000, device=local)
    logits = torch.empty((B,), dtype=torch.float32, device=f"cuda:{local}")
    L = _lib.lib()
    stream = torch.cuda.current_stream(local)
    sptr = C.c_void_p(stream.cuda_stream)

    def step():
        _lib.check(L.wk_forward(model._h.h, C.c_void_p(clips.data_ptr()), _lib.WK_DTYPE_F32, B, 16000, 16000,
                                C.c_void_p(logits.data_ptr()), None, sptr), "wk_forward")
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    flags = C.c_uint32(0)
    _lib.check(L.wk_check_device_errors(model._h.h, C.byref(flags)), "wk_check_device_errors")
    ok = flags.value == 0 and bool(torch.isfinite(logits).all())
    value = B * steps / el
    gbs = BYTES_PER_WINDOW_F32 * B / (launch_ms * 1e-3) / 1e9
    peak_c, basis_c = roofline_peak("bf16")
    achieved_c = FLOP_PER_WINDOW * B / (launch_ms * 1e-3) / 1e12
    del clips
    return {"workload": "config4: fused MFCC(torchaudio+CMVN) fp32 + xiaoa CNN bf16, one rank's share of "
                        "1,048,576 clips (131,072), fp32 audio resident in HBM",
            "value": round(value, 1), "unit": "windows/s per GPU", "batch_per_gpu": B, "steps": steps,
            "warmup": warmup, "ms_per_step": round(el / steps * 1e3, 4), "dtype": PRECISIONS["bf16"][0],
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4), "launch_ms": round(launch_ms, 4),
                         "windows_per_s_roof": round(HBM_ROOF_F32_WPS, 1)},
            "compute_ceiling": {"achieved": round(achieved_c, 3), "peak": round(peak_c, 1), "unit": "TFLOP/s",
                                "frac": round(achieved_c / peak_c, 4), "basis": basis_c},
            "logits_finite_and_no_device_error": ok}


def extra_config5(local):
    """Config 5 (bench_ctc.run_ctc): CTC head, B = 4096 utterances of 3 s, V = 4000, fp16."""
    import bench_ctc
    line = bench_ctc.run_ctc(batch=4096, vocab=4000, seconds=3, steps=5, warmup=1, precision="fp16", device=local)
    k = line["kernels"]
    return {"workload": line["config"]["workload"] + f", B = 4096, V = 4000, T = {line['config']['T']}, fp16",
            "value": line["value"], "unit": line["unit"], "ms_per_step": line["ms_per_step"],
            "steps": line["steps"], "warmup": line["warmup"], "dtype": line["dtype"],
            "call": line["config"]["call"], "roofline": line["roofline"],
            "output_kernel": {x: k["output"][x] for x in ("ms", "achieved", "peak", "unit", "frac")}
            if "output" in k else None,
            "stages": {s: {"ms": v["ms"], "frac": v["frac"], "bound": v["bound"]} for s, v in k.items()},
            "data": line["data"]}


def extra_config3(wakeword, local):
    """Config 3 (bench_stream.run_stream): 60 s stream pushed hop by hop (30 ms), p50 push -> logit on
    the host; throughput of a 1 h resident backlog."""
    import bench_stream
    line = bench_stream.run_stream(60, 480, 3600, device=local)
    line.pop("metric", None)
    line["workload"] = "config3: streaming 1 s windows at 30 ms hop, fp32, batch 1 per push"
    return line


def load_traffic(precision="fp32"):
    """HBM bytes per window from the committed rocprofv3 PMC summary of this precision, if any."""
    p = os.path.join(REPO, "profiles", "hbm_traffic.json" if precision == "fp32" else f"hbm_traffic_{precision}.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        return d.get("bytes_per_window"), d.get("source")
    except (OSError, ValueError):
        return None, None


def load_utilisation(precision="fp32"):
    """Datapath shares of the fused kernel from the committed rocprofv3 --pmc
    summary that hbm_traffic*.json names (VALU and MFMA
    utilisation beside the HBM figure).  Kernel cycles = GRBM_GUI_ACTIVE / 8
    XCDs; valu_active = SQ_ACTIVE_INST_VALU x 4 / (1,024 SIMDs x cycles),
    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1,024 x cycles).  None if absent."""
    tf = "hbm_traffic.json" if precision == "fp32" else f"hbm_traffic_{precision}.json"
    cm = {"fp32": 0, "bf16": 1, "bf16x3": 2}[precision]
    try:
        with open(os.path.join(REPO, "profiles", tf)) as fh:
            src = json.load(fh)["source"].split()[0]
        with open(os.path.join(REPO, src)) as fh:
            d = json.load(fh)
        k = next(v for n, v in d.items() if n.startswith(f"wk_fused_kernel<float, {cm}, false>"))
        cyc = k["GRBM_GUI_ACTIVE"] / 8.0
        return {"valu_active": round(k["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cyc), 3),
                "mfma_busy": round(k["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 3),
                "eff_clock_ghz": round(k["eff_clock_ghz"], 3) if k.get("eff_clock_ghz") else None,
                "source": src}
    except (OSError, ValueError, KeyError, StopIteration):
        return None


def init_rank(args, env, torch, dist):
    """This rank's (world, rank, local device, shared) from torchrun's
    environment, with the process group formed: nccl (RCCL) with the rank's
    own device as `device_id`, or gloo.  shared = more ranks on THIS node
    (LOCAL_WORLD_SIZE, torchrun's per-node count; WORLD_SIZE when unset) than
    visible GPUs (a gloo rehearsal of the N>1 path on one GPU): the line then
    carries no throughput.  A multi-node job with one rank per GPU on every
    node is not a rehearsal."""
    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", "0"))
    local_world = int(env.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPU(s) visible")
    shared = local_world > ndev
    local = local % ndev   # (gloo rehearsal: ranks may share a GPU)
    torch.cuda.set_device(local)
    if world > 1:
        env.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    return world, rank, local, shared


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # self-launch: N ranks before this process makes any GPU call
        sys.exit(spawn_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
    import torch
    import torch.distributed as dist
    import wakeword
    from wakeword import _lib
    from wakeword.shard import weak_shard

    world, rank, local, shared = init_rank(args, os.environ, torch, dist)

    def barrier():
        if world > 1:
            dist.barrier()

    pg_world = dist.get_world_size() if world > 1 else 1

    B = args.batch
    model = wakeword.load_onnx(os.path.join(REPO, "tests", "golden", "xiaoa.onnx"), device=local,
                               precision=args.precision)
    first, count = weak_shard(B, rank)                     # per-rank clip split, no collective
    clips = wakeword.synth_clips(args.seed, first, count, 16000, device=local)   # resident in HBM
    adt = _lib.WK_DTYPE_F32
    if args.audio == "i16":
        clips = (clips * 32768.0).round().clamp(-32768, 32767).to(torch.int16)
        adt = _lib.WK_DTYPE_I16
    logits = torch.empty((B,), dtype=torch.float32, device=f"cuda:{local}")
    L = _lib.lib()
    h = model._h.h
    stream = torch.cuda.current_stream(local)
    sptr = C.c_void_p(stream.cuda_stream)
    aptr, lptr = C.c_void_p(clips.data_ptr()), C.c_void_p(logits.data_ptr())

    def step():
        st = L.wk_forward(h, aptr, adt, B, 16000, 16000, lptr, None, sptr)
        if st != 0:
            _lib.check(st, "wk_forward")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    # outside the timed region: this rank's device error word (role hand-off
    # aborts) and the logits' finiteness, reduced with the times
    flags = C.c_uint32(0)
    st_err = L.wk_check_device_errors(h, C.byref(flags))
    bad = float(st_err != 0 or flags.value != 0 or not bool(torch.isfinite(logits).all()))
    t = torch.tensor([elapsed, launch_ms, bad], dtype=torch.float64,
                     device=f"cuda:{local}" if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)   # the slowest rank's time, any rank's error
    elapsed, launch_ms, bad = float(t[0]), float(t[1]), float(t[2])
    if bad:
        if rank == 0:
            print(f"bench: a rank reported a device error or non-finite logits (this rank: status {st_err}, "
                  f"flags {flags.value:#x}); no measurement printed", file=sys.stderr)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(3)

    if rank == 0:
        total = world * B * args.steps
        value = total / elapsed
        achieved = FLOP_PER_WINDOW * B / (launch_ms * 1e-3) / 1e12
        peak, peak_basis = roofline_peak(args.precision)
        traffic_bpw, traffic_src = load_traffic(args.precision)
        out = {
            "metric": "audio windows/sec (1s@16kHz, 40-MFCC) through xiaoa CNN at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": PRECISIONS[args.precision][0],
            "data": "synthetic: device counter-hash generator, clamp(0.1*N(0,1))+440 Hz sine on odd clips "
                    "(SURVEY 8(d) config 2); xiaoa.onnx weights",
            "config": {"workload": PRECISIONS[args.precision][1],
                       "audio": "fp32 samples" if args.audio == "f32" else "int16 PCM samples",
                       "batch_per_gpu": B, "global_batch": world * B, "seq_len": 16000,
                       "parallelism": f"dp{world} (per-rank clip split, no collectives)",
                       "process_group_world_size": pg_world,
                       **({"dist_backend": args.dist_backend} if world > 1 else {})},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 3), "peak": round(peak, 1),
                         "peak_basis": peak_basis,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                         "traffic": (traffic_bpw * B if traffic_bpw else None),
                         "launch_ms": round(launch_ms, 4),
                         "flop_per_window": FLOP_PER_WINDOW,
                         "hbm_gbs_algorithmic": round((BYTES_PER_WINDOW_F32 if args.audio == "f32" else 32_004) * B
                                                      / (launch_ms * 1e-3) / 1e9, 1)},
            "logits_finite": True,
            "device_errors": 0,
        }
        if shared:
            # ranks time-share one GPU: the launch path ran, but nothing here is
            # an N-GPU throughput or a kernel rate
            out["value"] = None
            out["rehearsal"] = True
            out["note"] = (f"{world} ranks shared {torch.cuda.device_count()} GPU(s) over {args.dist_backend}: "
                           "rehearsal of the N>1 launch, barrier and max-over-ranks path; no throughput")
            for k in ("achieved", "frac", "launch_ms", "hbm_gbs_algorithmic"):
                out["roofline"][k] = None
        if traffic_src:
            out["roofline"]["traffic_source"] = traffic_src
        util = load_utilisation(args.precision)
        if util:
            out["roofline"]["utilisation"] = util
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        if world == 1 and not shared and not args.no_extras:
            # SURVEY 8(d) configs 4, 5, 3, measured after the headline's timed
            # region and its CPU leg (the headline above is unchanged by them)
            # (a Python-level failure in one of them is recorded in its key; the
            # headline line is printed regardless)
            del clips
            for key, fn in (("config4", lambda: extra_config4(torch, wakeword, _lib, local, args.seed)),
                            ("config5", lambda: extra_config5(local)),
                            ("config3", lambda: extra_config3(wakeword, local))):
                torch.cuda.empty_cache()
                try:
                    out[key] = fn()
                except Exception as e:   # noqa: BLE001 -- reported, not hidden
                    out[key] = {"error": f"{type(e).__name__}: {e}"}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
