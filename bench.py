"""Benchmark: RGBD keypoint inference throughput (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64] [--precision fp16]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Without a launcher (no WORLD_SIZE in the environment) and N > 1, this process starts the N
ranks itself -- torchrun as a child process, before anything here touches the GPU (the
reference's own multi-process launch is mp.spawn, perseus/detector/train.py:371-375) -- and
exits with its status.  Every rank checks that the process group has N ranks.

One step = one KeypointCNN forward (perseus/detector/models.py:34-40) over a batch of 64
synthetic 256x256 RGBD frames already resident in HBM (BASELINE.json configs[1]).  At
N > 1 each rank runs its own frame shard (weak scaling, weights replicated) and the
keypoints of the whole run are all-gathered once over RCCL at the end of the timed
region (configs[2]).  Rank 0 prints one JSON line; see DESIGN.md "measurement".
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_FP16_DENSE_PEAK = 2.5e15  # MI355X_MICROARCH.md: ~2.5 PF dense fp16/bf16
MFMA_FP32_PEAK = 157.3e12      # f32-input MFMA peak (= vector f32 rate)
HBM_PEAK = 8.0e12
REPS = 20  # back-to-back launches per timed launch in the per-kernel pass
# parity_mode leg: the peak its roofline fraction is taken against, and what it executes
PARITY_PEAK = {"fp32": (MFMA_FP32_PEAK, 1, "v_mfma_f32_16x16x4_f32 (exact f32 products), f32 NHWC"),
               "fp16x3": (MFMA_FP16_DENSE_PEAK, 3, "3 v_mfma_f32_16x16x32_f16 products per MAC (x_hi w_hi + x_lo w_hi + "
                                                   "x_hi w_lo) on hi/lo fp16 planes, f32 accumulate")}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--precision", default="fp16", choices=["fp16", "fp32"])
    p.add_argument("--parity-precision", default="fp16x3", choices=["fp16x3", "fp32"],
                   help="mode of the parity_mode leg (the fast mode that meets the 1e-3 px bar); the exact-f32 "
                        "mode is always measured beside it as fp32_mode")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-passes", type=int, default=3)
    p.add_argument("--no-factors", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--no-trajset", action="store_true")
    p.add_argument("--traj", type=int, default=1000, help="configs[2]: trajectories in the set")
    p.add_argument("--traj-len", type=int, default=24, help="configs[2]: frames per trajectory")
    p.add_argument("--no-streaming", action="store_true")
    p.add_argument("--stream-ticks", type=int, default=300, help="configs[4]: paced ticks per streaming mode")
    p.add_argument("--stream-window", type=int, default=24, help="configs[4]: pose-stage window (frames per camera)")
    p.add_argument("--launcher-check", action="store_true",
                   help="CPU-only rehearsal of the N-rank launch: every rank joins a gloo group, checks its size "
                        "and rank 0 prints the ranks that joined (no GPU work)")
    return p.parse_args()


def launch_ranks(args) -> int:
    """`bench.py --gpus N` with no launcher around it: run the same command line as N ranks
    under torchrun (a child process; this parent never initialises HIP, so no GPU state is
    inherited or exec'd over) and return its exit status."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:  # a free rendezvous port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def launcher_check(args, world, rank):
    """--launcher-check: the rank processes join a gloo group of --gpus ranks (CPU only)."""
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    n = dist.get_world_size()
    if n != args.gpus:
        raise SystemExit(f"rank {rank}: process group has {n} ranks, --gpus {args.gpus}")
    t = torch.tensor([1 << rank], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launcher_check": True, "n_gpus": n, "world_env": world, "ranks_mask": int(t.item())}))
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from perseus_amd import shard, synth
    from perseus_amd.detector import KeypointCNN

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))  # before any GPU call in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}: run `bench.py --gpus N` alone or under a "
                         f"launcher of N ranks")
    if args.launcher_check:
        return launcher_check(args, world, rank)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"rank {rank}: RCCL group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    B = args.batch
    state = synth.synthetic_state_dict(args.seed)
    model = KeypointCNN(num_channels=4, precision=args.precision)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    model.eval()
    variants = {"headline": bench_variants(model)}
    # this rank's frame shard, resident in HBM before timing
    x_host = synth.synthetic_frames(args.seed, B, first=rank * B)
    x = torch.from_numpy(x_host).to(dev)
    model.reserve(B, dev)
    kp = torch.empty((args.steps, B, 16), dtype=torch.float32, device=dev)
    # CPU-side reference for the accuracy legs, computed before any GPU work so that the
    # GPU legs below run back to back
    yref = px_reference(state, x_host) if rank == 0 else None

    # ---- measurement legs (untimed for `value`).  They run BEFORE the timed loop: the
    # GPU comes out of them at its sustained clock, so the K-step window measures the
    # steady state even when K is small (the first ~8 ms of load after an
    # idle period run ~15 % slower while the clocks ramp; with only W warm-up forwards in
    # front, a 20-step window would average that ramp in).
    with torch.no_grad():
        px = px_error(model, x, yref) if rank == 0 else None
        # configs[4] first: its 30 Hz pacing leaves the GPU mostly idle, the legs after it
        # bring the clocks back up before the timed loop
        stream = None if (args.no_streaming or rank != 0) else streaming_leg(model, dev, args.stream_ticks,
                                                                             window=args.stream_window)
        # per-launch device time on the forward's stream: each launch of the forward issued
        # REPS times back to back between two HIP events (pa_detector_time_launch), median
        # over passes; no per-launch event gaps, so it agrees with rocprofv3 kernel-trace.
        n_launch = len(model.profile(x)[0])
        per_launch = []
        for idx in range(n_launch):
            v = [model.time_launch(x, idx, REPS) for _ in range(args.profile_passes)]
            per_launch.append((idx, v[0][0], statistics.median(ms for _, ms in v)))
        fac = factor_leg(dev, args.seed, rank) if not args.no_factors else None
        par = None if args.no_parity else parity_leg(state, x, yref, args.parity_precision, B, dev, rank, variants)
        par32 = None if (args.no_parity or args.parity_precision == "fp32") else \
            parity_leg(state, x, yref, "fp32", B, dev, rank, variants)
        tset = None if args.no_trajset else trajset_leg(model, x, args, dev, world, rank)

        # ---- the timed region: W warm-up forwards, then exactly K forwards
        for _ in range(args.warmup):
            model(x)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.steps):
            model(x, out=kp[i])  # keypoints straight into the step's slot
        if world > 1:  # ONE RCCL all-gather of every rank's keypoints (configs[2])
            shard.gather_keypoints(kp.view(-1, kp.shape[-1]), counts=[args.steps * B] * world)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames = world * B * args.steps
    value = frames / elapsed
    flops_frame = model.flops_per_frame()

    line = None
    if rank == 0:
        roof = roofline(per_launch, B, args.precision)
        per_kernel = per_kernel_rooflines(per_launch, B, args.precision)
        # rank 0 at every world size, after the timed region (the other ranks wait at the
        # closing barrier): the driver's N = 1..8 lines each carry the CPU baseline
        cpu = None if args.no_cpu_baseline else cpu_baseline(state, x_host)
        per_gpu = value / world
        line = {
            "metric": "RGBD frames/sec/GPU (256x256, batch 64); keypoint px-L2 vs CPU ref",
            "value": round(value, 1),
            "unit": "frames/s",
            "n_gpus": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (seeded RGBD frames + seeded ResNet-18 weights; no dataset/checkpoint offline)",
            "config": {"workload": "keypointcnn_rgbd256_b64_forward", "per_gpu_batch": B, "global_batch": B * world,
                       "H": 256, "W": 256, "channels": 4, "precision": args.precision,
                       "inputs": "device-resident f32 NCHW", "parallelism": f"dp{world}"},
            "frames_per_s_per_gpu": round(per_gpu, 1),
            "e2e_mfma_roofline_frac": round(per_gpu * flops_frame /
                                            (MFMA_FP16_DENSE_PEAK if args.precision == "fp16" else MFMA_FP32_PEAK), 4),
            "roofline": roof,
            "px_l2": px,
            "parity_mode": par,
            "fp32_mode": par32,
            "trajectory_set": tset,
            "streaming": stream,
            "cpu_baseline": cpu,
            "kernels_ms": {f"{i:02d}_{n}": round(ms, 4) for i, n, ms in per_launch},
            "per_kernel_roofline": per_kernel,
            "factors": fac,
            # kernel variants set on the models of this line ({} everywhere = the shipped kernels), and
            # whether the library was a measurement build with the timing-only (wrong-result) variants
            "variants": variants,
            "timing_variants_built": bool(_lib_timing_variants()),
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return line


def bench_variants(m, env="PERSEUS_AMD_BENCH_VARIANTS"):
    """A/B of kernel variants (tools/gpu_check.sh benchab / benchabx3): L:V[,L:V] from
    PERSEUS_AMD_BENCH_VARIANTS on the headline model, from PERSEUS_AMD_BENCH_VARIANTS_PARITY on the
    parity-mode models; unset in every recorded line.  Returns the map applied ({} = shipped
    kernels), which the output line carries under "variants"."""
    v = {}
    if os.environ.get(env):
        v = dict(tuple(int(t) for t in lv.split(":")) for lv in os.environ[env].split(","))
        m.set_variants(v)
    return {str(k): val for k, val in v.items()}


def _lib_timing_variants() -> int:
    from perseus_amd import _lib

    return _lib.lib().pa_debug_timing_variants_built()


def parity_leg(state, x, yref, precision, B, dev, rank, variants=None, warm=3, reps=20):
    """The parity-grade mode at the headline batch: frames/s over `reps` back-to-back
    forwards between HIP events on the forward's stream, its end-to-end MFMA-roofline
    fraction, and its px-L2 against the CPU f32 reference (rank 0)."""
    import numpy as np
    import torch

    from perseus_amd.detector import KeypointCNN

    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    m.eval()
    applied = bench_variants(m, "PERSEUS_AMD_BENCH_VARIANTS_PARITY")
    if variants is not None:
        variants[precision] = applied
    m.reserve(B, dev)
    out = torch.empty((B, 16), dtype=torch.float32, device=dev)
    for _ in range(warm):
        m(x, out=out)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        m(x, out=out)
    e1.record(s)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    fps = B / (ms * 1e-3)
    fl = m.flops_per_frame()
    peak, prods, note = PARITY_PEAK[precision]
    res = {"precision": precision, "batch": B, "frames_per_s": round(fps, 1), "ms_per_step": round(ms, 4),
           "roofline": {"bound": "mfma", "achieved": round(fps * fl / 1e12, 2), "peak": peak / 1e12,
                        "unit": "TFLOP/s", "frac": round(fps * fl / peak, 4),
                        "mfma_issue_frac": round(prods * fps * fl / peak, 4), "note": note},
           "timing": f"{reps} back-to-back forwards between HIP events after {warm} warm-ups"}
    if rank == 0:
        res["px_l2"] = px_error(m, x, yref)
    m._release()
    return res


def trajset_leg(model, x, args, dev, world, rank, reps=3):
    """configs[2]: the 24-frame x 1k-trajectory set, sharded by whole trajectories
    (shard.trajectory_range, so no dynamics / const-vel pair crosses ranks).  Per rank:
    forward over its frames (device-resident, one call; the library runs it in chunks),
    pa_trajectory_linearize over its trajectories (the keypoints never leave HBM), then
    ONE all-gather of every rank's keypoints (RCCL).  Strong scaling: the set is fixed,
    frames/s = set size / max-over-ranks time of the whole sequence (median of `reps`)."""
    import torch
    import torch.distributed as dist

    from perseus_amd import pipeline, shard, synth

    T, L = args.traj, args.traj_len
    f0, f1 = shard.trajectory_range(T, L, world, rank)
    n = f1 - f0
    counts = shard.shard_counts(T * L, world, traj_len=L)  # static: the gather is one collective
    t_local = n // L
    # distinct frames in HBM (the bench batch tiled: content does not change the work)
    reps_x = (n + x.shape[0] - 1) // x.shape[0]
    xs = x.repeat(reps_x, 1, 1, 1)[:n].contiguous()
    ys = torch.empty((n, 16), dtype=torch.float32, device=dev)
    tr = synth.synthetic_trajectories(args.seed + 11 + rank, t_local, L)
    a, out = pipeline.prepare_trajectories(ys, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"],
                                           T=t_local, L=L, dt=1 / 12, proj_sigmas=[1.0, 1.0],
                                           dyn_sigmas=[0.1] * 6, cv_sigmas=[0.1] * 3)
    model.reserve(min(n, 1024), dev)

    def run():
        model(xs, out=ys)
        pipeline.launch(a, dev)
        return shard.gather_keypoints(ys, counts=counts)

    g = run()  # warm-up (and the gathered shape check)
    times = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        times.append(el)
    el = statistics.median(times)
    del xs
    return {"workload": f"configs[2]: {T} trajectories x {L} frames, trajectory-sharded", "frames": T * L,
            "frames_per_rank": n, "trajectories_per_rank": t_local, "ms": round(el * 1e3, 3),
            "frames_per_s": round(T * L / el, 1), "scaling": "strong", "gathered_rows": int(g.shape[0]),
            "steps": "forward (chunked) + pa_trajectory_linearize + one all_gather of keypoints",
            "timing": f"wall clock, barrier + synchronize, max over ranks, median of {reps}"}


def streaming_leg(model, dev, ticks=300, hz=30.0, cams=3, window=24,
                  modes=("pose", "pose_parity", "pose_ahead", "pose_parity_ahead", "pixels"), zero_copy=None,
                  zero_copy_out=True):
    """configs[4]: 3 x 720p RGBD cameras paced at `hz`, one StreamingPipeline tick per
    camera period (pinned host staging of the centre crops, one hipGraph replay: H2D,
    fused-preprocess forward at B = cams, denormalize, D2H pixels; mode "pose" adds the
    pose stage over a `window`-frame fixed-lag window per camera: advance, linearize the
    reference's factors, one GN step, retract, D2H poses; "pose_parity" is the same tick
    with the detector in fp16x3, the mode that meets north_star's 1e-3 px, in its latency
    mode; "_ahead": the same ticks with the next tick's pre half run right after the results,
    in the gap before the next frames, StreamingPipeline(pre_ahead=True)).  Latency = host
    time from the start of staging to results on the host, p50 / p99 / max over `ticks` paced
    ticks (mode "pixels": ticks // 3); device_ms = one tick's device work between HIP events
    on the pipeline's stream (20 back to back; "_ahead": including the next tick's pre half),
    latency_path_ms ("_ahead") = from a tick's start to its results (median of 20 ticks)."""
    import numpy as np
    import torch

    from perseus_amd.detector import KeypointCNN
    from perseus_amd.streaming import StreamingPipeline

    parity = None
    if any(m.startswith("pose_parity") for m in modes):  # the same weights in the parity-grade precision
        parity = KeypointCNN(num_channels=4, precision="fp16x3")
        parity.load_state_dict(model.state_dict())

    rng = np.random.default_rng(0)
    n_src = 8  # rotate through a few distinct synthetic camera ticks
    rgbs = rng.integers(0, 256, (n_src, cams, 720, 1280, 3), dtype=np.uint8)
    deps = rng.uniform(0.12, 0.48, (n_src, cams, 720, 1280)).astype(np.float32)
    res = {"workload": f"configs[4]: {cams} x 720p RGBD @ {hz:g} Hz, centre crop 256, B = {cams} per tick",
           "unit": "ms", "timing": "host time from staging start to results on the host, paced ticks"}
    for mode in modes:
        kw = dict(pose_window=window, proj_sigma=40.0) if mode.startswith("pose") else {}
        ahead = mode.endswith("_ahead")
        pipe = StreamingPipeline(parity if mode.startswith("pose_parity") else model, n_cams=cams, graph=True,
                                 host_crop=True, device=dev, zero_copy=zero_copy, pre_ahead=ahead,
                                 zero_copy_out=zero_copy_out, **kw)
        for i in range(10):
            pipe(rgbs[i % n_src], deps[i % n_src])
        n = ticks if mode.startswith("pose") else max(ticks // 3, 30)
        lat = []
        period = 1.0 / hz
        t_next = time.perf_counter()
        for i in range(n):
            while time.perf_counter() < t_next:
                pass
            t0 = time.perf_counter()
            pipe(rgbs[i % n_src], deps[i % n_src])
            lat.append(time.perf_counter() - t0)
            t_next += period
        lat = np.array(lat) * 1e3
        s = pipe.stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            for _ in range(20):
                pipe.replay()
            e1.record(s)
        s.synchronize()
        r = {"ticks": n, "p50_ms": round(float(np.percentile(lat, 50)), 4),
             "p99_ms": round(float(np.percentile(lat, 99)), 4), "max_ms": round(float(lat.max()), 4),
             "device_ms_per_tick": round(e0.elapsed_time(e1) / 20, 4)}
        if ahead:
            path = []
            for _ in range(20):
                with torch.cuda.stream(s):
                    e0.record(s)
                    pipe.replay()
                s.synchronize()
                path.append(e0.elapsed_time(pipe._done))
            r["latency_path_ms"] = round(float(np.median(path)), 4)
        if mode.startswith("pose"):
            r["window_frames"] = window
            r["precision"] = pipe.model.precision
            r["stage"] = ("forward_rgbd_px (latency mode) + " +
                          ("pa_window_pose_tick_pre (next tick's, after the results) + _post" if pipe.pre_ahead else
                           "pa_window_pose_tick_pre (beside the forward) + _post" if pipe.split_pose else
                           "pa_window_pose_tick (advance + linearize, GN step + retract: two launches)"
                           if getattr(pipe, "fused_pose", False) else
                           "pa_window_advance_n + pa_trajectory_linearize + pa_trajectory_gn_step (delta + info) + "
                           "pa_window_retract_newest"))
            r["solved_last_tick"] = int((pipe.info_h.numpy() == 0).sum())
        res[mode] = r
        pipe.close()
    return res


def conv_flops(B, fused_stem=True, fused_ds=True, fused_head=True):
    """Algorithmic FLOPs per launch, in forward order (matches pa_detector_profile)."""
    stem = 2.0 * B * 128 * 128 * 64 * 49 * 4  # true K = 196
    fl = [stem] if fused_stem else [stem, 0.0]  # fp16 fuses conv7x7 + maxpool
    hw, cin = 64, 64
    for li, cout in enumerate((64, 128, 256, 512)):
        for bi in range(2):
            s = 2 if (li > 0 and bi == 0) else 1
            ho = hw // s
            c_in = cin if bi == 0 else cout
            c1 = 2.0 * B * ho * ho * cout * 9 * c_in
            if bi == 0 and li > 0:
                ds = 2.0 * B * ho * ho * cout * c_in
                fl += [c1 + ds] if fused_ds else [c1, ds]  # conv1 s2 (+ fused 1x1 s2 downsample)
            else:
                fl.append(c1)
            fl.append(2.0 * B * ho * ho * cout * 9 * cout)          # conv2
            hw = ho
        cin = cout
    if fused_head:  # avgpool + fc in layer4's last conv epilogue
        fl[-1] += 2.0 * B * 512 * 16
    else:
        fl.append(2.0 * B * 512 * 16)
    return fl


def roofline(per_launch, B, precision):
    fl = None
    fused_head = per_launch[-1][1] != "avgpool_fc"
    for fs in (True, False):
        for fd in (True, False):
            c = conv_flops(B, fused_stem=fs, fused_ds=fd, fused_head=fused_head)
            if len(c) == len(per_launch):
                fl = c
                break
        if fl:
            break
    if fl is None:
        return None
    groups = {}
    for (idx, name, ms), f in zip(per_launch, fl):
        g = groups.setdefault(name, [0.0, 0.0, 0, []])
        g[0] += ms
        g[1] += f
        g[2] += 1
        g[3].append(idx)
    name, (ms, f, n, idxs) = max(groups.items(), key=lambda kv: kv[1][0])
    peak = MFMA_FP16_DENSE_PEAK if precision == "fp16" else MFMA_FP32_PEAK
    traffic = pmc_traffic(precision, B, idxs, [nm for _, nm, _ in per_launch])
    if f == 0:  # bandwidth kernel dominant (maxpool)
        return {"kernel": name, "bound": "hbm", "achieved": None, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": None, "traffic": traffic, "launches": n, "avg_ms": ms / n}
    achieved = f / (ms * 1e-3)
    return {"kernel": name, "bound": "mfma", "achieved": round(achieved / 1e12, 2), "peak": peak / 1e12,
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic, "launches": n,
            "avg_ms": round(ms / n, 5), "flops_per_launch": f / n}


def per_kernel_rooflines(per_launch, B, precision):
    """north_star's per-kernel figures: the conv stem's achieved HBM GB/s (algorithmic
    bytes: the f32 NCHW input it reads, the pooled fp16 NHWC map it writes, its packed
    fp16 weights) against the 8 TB/s peak, with the PMC bytes of that launch when the
    committed record matches these kernels; and every 3x3 conv launch's MFMA utilisation
    (algorithmic FLOPs / launch time) against the dense fp16 peak."""
    if precision != "fp16" or not per_launch or per_launch[0][1] != "stem_conv7x7_pool":
        return None
    fl = conv_flops(B, fused_stem=True, fused_ds=True, fused_head=per_launch[-1][1] != "avgpool_fc")
    if len(fl) != len(per_launch):
        return None
    names = [nm for _, nm, _ in per_launch]
    stem_ms = per_launch[0][2]
    stem_bytes = B * 4 * 256 * 256 * 4 + B * 64 * 64 * 64 * 2 + 64 * 7 * 32 * 2
    stem = {"kernel": per_launch[0][1], "bound": "hbm", "us": round(stem_ms * 1e3, 2), "alg_bytes": stem_bytes,
            "achieved_gbps": round(stem_bytes / (stem_ms * 1e-3) / 1e9, 1),
            "frac": round(stem_bytes / (stem_ms * 1e-3) / HBM_PEAK, 4), "peak_gbps": HBM_PEAK / 1e9,
            "pmc_bytes": pmc_traffic(precision, B, [per_launch[0][0]], names),
            "mfma_frac": round(fl[0] / (stem_ms * 1e-3) / MFMA_FP16_DENSE_PEAK, 4)}
    convs = {f"{i:02d}_{nm}": round(f / (ms * 1e-3) / MFMA_FP16_DENSE_PEAK, 4)
             for (i, nm, ms), f in zip(per_launch, fl) if nm.startswith("conv3x3")}
    return {"stem": stem, "conv3x3_mfma_frac": convs, "mfma_peak_tflops": MFMA_FP16_DENSE_PEAK / 1e12,
            "timing": "per-launch HIP events (pa_detector_time_launch), as kernels_ms",
            "mfma_busy_counter": pmc_mfma(precision, B, names)}


def factor_leg(dev, seed, rank, T=1000, L=24, reps=20):
    """Config 3 side measurement: pa_trajectory_linearize over 1000 trajectories x 24
    frames (8 projection factors per frame, a dynamics + const-vel factor per frame
    pair, whitened, Jacobians on), `reps` launches back to back between HIP events on
    the launch stream.  Algorithmic bytes: every input read once, every output written
    once (DESIGN.md "factor kernels")."""
    import torch

    from perseus_amd import pipeline, synth

    tr = synth.synthetic_trajectories(seed + 1 + rank, T, L)
    y = torch.as_tensor(tr["y"], device=dev)
    a, out = pipeline.prepare_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"], T=T,
                                           L=L, dt=1 / 12, proj_sigmas=[1.0, 1.0], dyn_sigmas=[0.1] * 6,
                                           cv_sigmas=[0.1] * 3)
    for _ in range(3):
        pipeline.launch(a, dev)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        pipeline.launch(a, dev)
    e1.record(s)
    torch.cuda.synchronize(dev)
    t = e0.elapsed_time(e1) / reps * 1e-3
    F, n, m = T * L, T * L * 8, T * (L - 1)
    bytes_in = F * (16 * 4 + 12 * 8 + 3 * 8 + 3 * 8)
    bytes_out = n * (2 + 12 + 1) * 8 + n * 4 + m * (6 + 36 + 18 + 18 + 36 + 1) * 8 + m * (3 + 9 + 9 + 1) * 8
    # the consumer: one damped GN step per trajectory from these factors
    # (pa_trajectory_gn_step: block assembly + the two-ended block-tridiagonal solve), its
    # outputs and workspace allocated once (GNPlan), so the events time the launches only
    plan = pipeline.GNPlan(out, T=T, L=L, lam=1e-3)
    for _ in range(2):
        plan.launch()
    e0.record(s)
    for _ in range(reps):
        plan.launch()
    e1.record(s)
    torch.cuda.synchronize(dev)
    t_gn = e0.elapsed_time(e1) / reps * 1e-3
    solved = int((plan.out["info"] == 0).sum())
    # the streaming pose stage's size (3 cameras x 24 frames): the cyclic-reduction form
    tr3 = synth.synthetic_trajectories(seed + 2 + rank, 3, L)
    a3, out3 = pipeline.prepare_trajectories(torch.as_tensor(tr3["y"], device=dev), tr3["poses"], tr3["vels"],
                                            tr3["angvels"], tr3["corners"], tr3["K"], T=3, L=L, dt=1 / 12,
                                            proj_sigmas=[1.0, 1.0], dyn_sigmas=[0.1] * 6, cv_sigmas=[0.1] * 3)
    pipeline.launch(a3, dev)
    plan3 = pipeline.GNPlan(out3, T=3, L=L, lam=1e-3)
    for _ in range(2):
        plan3.launch()
    e0.record(s)
    for _ in range(reps):
        plan3.launch()
    e1.record(s)
    torch.cuda.synchronize(dev)
    t_gn3 = e0.elapsed_time(e1) / reps * 1e-3
    return {"workload": f"trajectory_linearize_{T}x{L}", "frames": F, "factors": n + 2 * m,
            "us_per_launch": round(t * 1e6, 2), "frames_per_s": round(F / t, 1), "factors_per_s": round((n + 2 * m) / t),
            "alg_bytes": bytes_in + bytes_out, "hbm_gbps": round((bytes_in + bytes_out) / t / 1e9, 1),
            "hbm_frac": round((bytes_in + bytes_out) / t / HBM_PEAK, 4), "dtype": "f64",
            "gn_step": {"us_per_step": round(t_gn * 1e6, 2), "trajectories": T, "solved": solved,
                        "trajectories_per_s": round(T / t_gn, 1), "us_per_step_3x24": round(t_gn3 * 1e6, 2),
                        "solved_3x24": int((plan3.out["info"] == 0).sum())}}


def csrc_digest() -> str:
    """SHA-256 (16 hex) over the library's kernel sources and headers with their comments
    removed and whitespace runs collapsed: the PMC record is only valid for the exact kernels
    it was taken on, and a comment-only edit does not change a kernel."""
    import glob
    import hashlib

    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "perseus_amd", "csrc", "*"))):
        with open(f, "rb") as fh:
            code = strip_comments(fh.read())
        h.update(os.path.basename(f).encode() + b"\0" + code)
    return h.hexdigest()[:16]


def strip_comments(src: bytes) -> bytes:
    """C/C++ source without its comments (string and character literals kept intact, so a
    "//" inside one is code), horizontal whitespace runs collapsed per line and blank lines
    dropped; line breaks stay (they end preprocessor directives)."""
    import re

    tok = re.compile(rb'"(?:\\.|[^"\\\n])*"|\'(?:\\.|[^\'\\\n])*\'|//[^\n]*|/\*.*?\*/', re.S)

    def repl(m):  # a comment is one space (C's translation phase 3); a literal is itself
        t = m.group(0)
        return b" " if t.startswith((b"//", b"/*")) else t

    out = []
    for line in tok.sub(repl, src).split(b"\n"):
        line = b" ".join(line.split())
        if line:
            out.append(line)
    return b"\n".join(out)


def pmc_traffic(precision, B, idxs, names):
    """Mean HBM bytes per launch of launch indices `idxs`, from the committed PMC
    summary (profiles/pmc_traffic.json, tools/rocprof_summary.py: FETCH_SIZE x2 +
    WRITE_SIZE, separate rocprofv3 --pmc passes), if it was taken on the same kernel
    sources (csrc digest), launch sequence and batch; else None."""
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(tf) as fh:
            rec = json.load(fh).get(precision)
    except (OSError, ValueError):
        return None
    if not rec or rec.get("batch") != B or rec.get("names") != names or rec.get("csrc") != csrc_digest():
        return None
    v = [rec["bytes_per_launch"][i] for i in idxs]
    return round(sum(v) / len(v))


def pmc_mfma(precision, B, names):
    """rocprofv3-counter MFMA utilisation of every 3x3 conv launch (tools/mfma_counters.py:
    SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x the launch's cycles, and over the nominal
    2.4 GHz cycles of its duration) from the committed record profiles/pmc_mfma.json, if it
    was taken on the same kernel sources (csrc digest), launch sequence and batch; else None."""
    tf = os.path.join(ROOT, "profiles", "pmc_mfma.json")
    try:
        with open(tf) as fh:
            rec = json.load(fh).get(precision)
    except (OSError, ValueError):
        return None
    if not rec or rec.get("batch") != B or rec.get("names") != names or rec.get("csrc") != csrc_digest():
        return None
    pl = rec["per_launch"]
    return {"busy_frac_of_cycles": {f"{i:02d}_{r['launch']}": r["busy_frac_of_cycles"]
                                    for i, r in enumerate(pl) if r["launch"].startswith("conv3x3")},
            "busy_frac_of_nominal": {f"{i:02d}_{r['launch']}": r["busy_frac_of_nominal"]
                                     for i, r in enumerate(pl) if r["launch"].startswith("conv3x3")},
            "clock_ghz": {f"{i:02d}_{r['launch']}": r["clock_ghz"]
                          for i, r in enumerate(pl) if r["launch"].startswith("conv3x3")},
            "source": rec.get("source"),
            "counters": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), and / (1024 x duration x "
                        "2.4 GHz) (the latter comparable with conv3x3_mfma_frac)"}


def px_reference(state, x_host, nframes=64):
    """CPU f32 reference outputs (oracle/resnet_ref.py, the reference's own CPU path
    restated) of the first min(B, `nframes`) bench frames (max / mean over 64
    frames x 8 keypoints; ~1 s of CPU at 16 threads; capped so that a --batch 1024 run does
    not hold a 4 GB f32 stem map on the host)."""
    import torch

    from oracle import resnet_ref as R

    return R.run(state, x_host[:nframes], torch.float32)


def px_error(model, x, yref):
    """Per-keypoint px-L2 of `model` on the first frames of `x` against `yref`, plus the
    integer pixels streaming.py:142-144 draws (int() of the kornia-denormalized px):
    mismatches overall and among coordinates > 1e-3 px from an integer boundary."""
    import numpy as np

    from oracle import resnet_ref as R

    n = yref.shape[0]
    y = model(x[:n]).cpu().numpy()
    d = (np.abs(y - yref) * 127.5).reshape(n, -1, 2)
    l2 = np.sqrt((d ** 2).sum(-1))
    pg, pr = R.denormalize_f32(y), R.denormalize_f32(yref)
    ig, ir = pg.astype(np.int64), pr.astype(np.int64)
    frac = np.abs(pr - np.round(pr))
    safe = frac > 1e-3
    return {"max": float(l2.max()), "mean": float(l2.mean()), "frames": int(n),
            "int_px_mismatch": int((ig != ir).sum()), "int_px_mismatch_safe": int(((ig != ir) & safe).sum()),
            "int_px_coords": int(ig.size), "int_px_safe_coords": int(safe.sum()),
            "vs": "reference-equivalent torch CPU f32 forward (oracle/resnet_ref.py)"}


def cpu_baseline(state, x_host, warm=2, iters=5):
    """torch-CPU f32 forward (the oracle restatement of the reference's CPU path) on the
    box's host cores, at two thread counts: SURVEY 8(d)'s len(os.sched_getaffinity(0))
    and torch's intra-op pool as the box sets it (OMP_NUM_THREADS = the box's CPU share;
    on a shared GPU box the affinity mask lists the whole machine, so the two differ).
    The faster of the two is `value`, with `cores` = the threads it used; both samples
    are reported."""
    import numpy as np
    import torch

    from oracle import resnet_ref as R

    pool = torch.get_num_threads()
    affinity = len(os.sched_getaffinity(0))
    sd = R.to_torch(state, torch.float32)
    x = torch.from_numpy(np.ascontiguousarray(x_host))
    samples, notes = {}, {}
    try:
        for threads in dict.fromkeys((affinity, pool)):
            torch.set_num_threads(threads)
            times = []
            with torch.no_grad():
                for i in range(warm + iters):
                    t0 = time.perf_counter()
                    R.forward(sd, x)
                    dt = time.perf_counter() - t0
                    if i >= warm:
                        times.append(dt)
                    if dt > 3.0 and threads != pool:
                        # oversubscribed (the mask lists the whole machine, the box grants a
                        # share): one forward is the sample, so the bench stays within minutes
                        times = [dt]
                        notes[str(threads)] = f"one forward ({dt:.1f} s): oversubscribed, sample cut"
                        break
            samples[threads] = x.shape[0] / statistics.median(times)
    finally:
        torch.set_num_threads(pool)
    best = max(samples, key=samples.get)
    return {"value": round(samples[best], 2), "unit": "frames/s", "cores": best, "kind": "port",
            "affinity_cores": affinity, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "by_threads": {str(t): round(v, 2) for t, v in samples.items()}, "notes": notes or None,
            "sample": f"{iters} timed (+{warm} warm-up) torch-CPU f32 forwards of the same batch of {x.shape[0]} "
                      f"frames, median, at {len(samples)} thread count(s): the {affinity}-CPU affinity mask "
                      f"(SURVEY 8(d)) and torch's {pool}-thread pool; value = the faster"}


if __name__ == "__main__":
    main()
