"""Headline benchmark: training images/sec of the plastic U-Net (BASELINE.json metric), MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher (no WORLD_SIZE in the environment), --gpus N > 1 makes this process spawn N
rank processes itself (launch_workers: torchrun's env, MASTER_ADDR 127.0.0.1, a free port) and
exit with their status.  Every rank checks after init_process_group("nccl") that the world has
exactly N ranks and that N GPUs are visible, and exits non-zero otherwise.

Workload = config C2 (BASELINE.json configs[1]): UNetp depth 5 / base 64 (14.81 M params), Oja
rule, 1x128x128 synthetic tiles, batch 32 per GPU, fp32.  --config c4 / c5 measure the other
single-GPU configurations (CoordConv U-Net 256x256 bs 32; UNetpRes neurons 8 512x512 bs 16 per GPU
with Dropout2d active) - parity/coverage lines, not the headline.  A step = forward + BCE + backward
(+ RCCL gradient all-reduce when N > 1) + Adam + StepLR over one resident batch, with the per-slot
plastic traces carried step to step.  Timed region: barrier + synchronize on both sides, max over
ranks; value = images of all ranks / time (weak scaling: 32 images per GPU).

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
  roofline      the dominant kernel's algorithmic TFLOP/s vs the fp32 MFMA peak, from HIP events
                bracketing each launch on its own stream during a separate instrumented pass
  kernels       per-kernel-instantiation time/FLOP breakdown of one step
  oja_update    the Oja trace update's algorithmic GB/s (bs x 128^2, cache-resident) and an
                HBM-sized sweep (8192 traces, 1 GiB per pass)
  allreduce     the gradient exchange (N > 1): bucket count and sizes, buckets issued during the
                backward, exposed all-reduce ms per step (HIP events, untimed pass)
  cpu_baseline  the CPU oracle (oracle/ref_cpu.py, fixture-pinned restatement of the reference)
                on the host cores, N=1 only: the reference's own mode (bs=1, Adam per sample) as
                `value`, and the batched mode (bs B, per-slot traces) as `batched`
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (c2/c4: 32, c5: 16)")
    ap.add_argument("--img", type=int, default=None, help="image side (c2: 128, c4: 256, c5: 512)")
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--base", type=int, default=64)
    ap.add_argument("--rule", default="oja")
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--steplr", type=float, default=1e5)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample length (per mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-profile", action="store_true")
    ap.add_argument("--no-oja", action="store_true", help="skip the Oja-update HBM benchmark")
    ap.add_argument("--graph", choices=["on", "off"], default="off",
                    help="on: fwd + BCE + bwd captured once as a HIP graph and replayed (one rank only). "
                         "Off by default: measured no faster on C2 / C4 and slower on C3, whose replay loses "
                         "the weight-gradient side stream's overlap (profiles/r05_experiments/graph_step_ab.txt)")
    a = ap.parse_args()
    dflt = {"c2": (32, 128), "c3": (32, 128), "c4": (32, 256), "c5": (16, 512)}[a.config]
    a.batch = a.batch or dflt[0]
    a.img = a.img or dflt[1]
    return a


CONFIGS = {
    "c2": "C2: UNetp depth %(depth)d base_ch %(base)d, %(rule)s rule, 1x%(img)dx%(img)d, fwd+BCE+bwd+Adam",
    "c3": "C3: UNetp depth %(depth)d base_ch %(base)d bf16 (fp32 accumulation / params / Adam / head), %(rule)s "
          "rule, 1x%(img)dx%(img)d, fwd+BCE+bwd+Adam",
    "c4": "C4: CoordConv-UNet (coord_conv_script.py topology, with_r) base 8 depth 5 + plastic head, %(rule)s rule, "
          "1x%(img)dx%(img)d, fwd+BCE+bwd+Adam",
    "c5": "C5: UNetpRes neurons 8, Dropout2d 0.5 (train mode), %(rule)s rule, 1x%(img)dx%(img)d, fwd+BCE+bwd+Adam",
}


def build_model(args, device, ref=False):
    """The configuration's model: the MI355X product class, or (ref=True) the CPU oracle's."""
    if ref:
        import oracle
        if args.config == "c4":
            return oracle.RefCoordConvUNetp(1, 1, rule=args.rule, nbf=args.img, base_ch=8, with_r=True, depth=5)
        if args.config == "c5":
            return oracle.RefUNetpRes(1, 1, neurons=8, rule=args.rule, nbf=args.img)
        return oracle.RefUNetp(1, 1, rule=args.rule, nbf=args.img, depth=args.depth, base_ch=args.base)
    if args.config == "c4":
        from unet import CoordConvUNetp
        return CoordConvUNetp(1, 1, device, rule=args.rule, nbf=args.img, base_ch=8, with_r=True, depth=5)
    if args.config == "c5":
        from unet import UNetpRes
        return UNetpRes(1, 1, device, neurons=8, rule=args.rule, nbf=args.img)
    from unet import UNetp
    return UNetp(1, 1, device, rule=args.rule, nbf=args.img, depth=args.depth, base_ch=args.base,
                 precision="bf16" if args.config == "c3" else "fp32")


def fp32_mfma_peak_tflops(kernels):
    cu, clk_khz, _ = kernels.device_info(torch.cuda.current_device())
    # v_mfma_f32_32x32x2_f32: 64 FLOP/clk/SIMD x 4 SIMDs per CU (MI355X_MICROARCH.md)
    clk_ghz = clk_khz / 1e6 if clk_khz > 0 else 2.4
    return 256.0 * cu * clk_ghz / 1e3, cu, clk_ghz


def cpu_baseline(args, batch):
    """The oracle on the host cores (SURVEY 8(d) CPU baseline), two timings of one bounded sample
    each (args.cpu_seconds of training, after one untimed warm-up step):
      (i)  the reference's own mode: bs=1, Adam + StepLR per sample, the trace carried sample to
           sample (train.py:91-112) - `value`, the faithful baseline;
      (ii) batched: the bench's per-GPU batch B with per-slot traces [B,N,N] carried step to step
           (the batched semantics of SURVEY 8(a)), one Adam step per batch - `batched`."""
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)

    def run(bs, max_steps):
        torch.manual_seed(0)
        net = build_model(args, None, ref=True)
        net.train()
        opt = oracle.ref_adam(net.parameters(), args.lr)
        sch = oracle.ref_steplr(opt, int(args.steplr))
        g = torch.Generator().manual_seed(4321)
        xs = torch.rand(2, bs, 1, args.img, args.img, generator=g)
        ts = (torch.rand(2, bs, args.img, args.img, generator=g) > 0.5).float()
        hebb = net.initialZeroHebb(bs) if bs > 1 else net.initialZeroHebb()
        x0 = xs[0] if bs > 1 else xs[0, 0:1]
        oracle.ref_train_step(net, opt, sch, x0, ts[0] if bs > 1 else ts[0, 0], hebb)     # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            k = n % 2
            x, t = (xs[k], ts[k]) if bs > 1 else (xs[k, 0:1], ts[k, 0])
            _, _, hebb = oracle.ref_train_step(net, opt, sch, x, t, hebb)
            n += 1
            el = time.perf_counter() - t0
            if (el >= args.cpu_seconds and n >= 2) or n >= max_steps:
                break
        return n, el, type(net).__name__

    n1, el1, name = run(1, 200)
    nb, elb, _ = run(batch, 50)
    return {"value": n1 / el1, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": "oracle/ref_cpu.py %s %dx%d, reference mode (bs=1, fwd+BCE+bwd+Adam per sample, "
                      "train.py:91-112): %d samples in %.1f s on %d threads" % (name, args.img, args.img, n1, el1, threads),
            "batched": {"value": nb * batch / elb, "unit": "images/s", "cores": threads, "kind": "port",
                        "sample": "oracle/ref_cpu.py %s %dx%d, batched mode (bs=%d with per-slot traces "
                                  "[%d,%d,%d] carried step to step, one Adam step per batch): %d steps = %d "
                                  "images in %.1f s on %d threads"
                                  % (name, args.img, args.img, batch, batch, args.img, args.img, nb, nb * batch,
                                     elb, threads)}}


def _launch_time_us(fn, reps):
    """Average device time of one fn() launch: `reps` launches captured in a HIP graph and replayed
    (no Python/ctypes launch overhead between them); eager back-to-back launches if capture fails."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (5 * reps), "hip_graph"
    except Exception:
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps, "eager"


def oja_update_bench(K, B, N, device, feat_channels=64):
    """Algorithmic GB/s of the Oja trace update: 8*B*N^2 + 8*B*N bytes (read H, write H', rows),
    the stand-alone kernel at the bench batch (cache-resident) and over an HBM-sized sweep; plus
    the fused head forward (outconv + GEMM + sigmoid + Oja update in one launch)."""
    res = {}
    eta = torch.full((1,), 0.01, device=device)
    sweep = max(1, (1 << 30) // (4 * N * N))            # 1 GiB of traces (16384 at N=128)
    for label, bb, reps in (("bs%d" % B, B, 100), ("hbm_sweep_%d" % sweep, sweep, 10)):
        H = torch.randn(bb, N, N, device=device)
        X = torch.randn(bb, N, N, device=device)
        Y = torch.rand(bb, N, N, device=device)
        out = torch.empty_like(H)
        us, how = _launch_time_us(lambda: K.trace_update(H, X, Y, eta, 1, out=out), reps)
        nbytes = 8.0 * bb * N * N + 8.0 * bb * N
        res[label] = {"us_per_launch": round(us, 3), "bytes": nbytes, "GB_s": round(nbytes / us / 1e3, 1),
                      "timing": how}
        del H, X, Y, out
    H = 0.1 * torch.randn(B, N, N, device=device)
    w = 0.01 * torch.randn(N, N, device=device)
    a = 0.01 * torch.rand(N, N, device=device)
    # the fused head of the training step: outconv (feat [B,N,N,C]) + Weff GEMM + sigmoid + Oja
    # update in one launch; algorithmic bytes = feat read + X, Y, H' written + H read + w, alpha
    C = feat_channels
    feat = torch.rand(B, N, N, C, device=device)
    wo = 0.1 * torch.randn(C, device=device)
    bo = torch.zeros(1, device=device)
    us, how = _launch_time_us(lambda: K.plastic_head_fwd(feat, wo, bo, H, w, a, eta, 1, True), 50)
    nbytes = 4.0 * B * N * N * C + 16.0 * B * N * N + 8.0 * N * N
    res["fused_head_bs%d" % B] = {"kernel": "pu_plastic_head_fwd (outconv %d->1 + head + Oja)" % C,
                                 "us_per_launch": round(us, 3), "bytes": nbytes,
                                 "GB_s": round(nbytes / us / 1e3, 1), "hbm_frac": round(nbytes / us / 1e3 / 8000.0, 3),
                                 "TFLOP_s": round((2.0 * B * N ** 3 + 2.0 * B * N * N * C) / us / 1e6, 2),
                                 "timing": how}
    return res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_workers(n, argv, cmd=None, poll_s=0.2):
    """`python bench.py --gpus N` without a launcher: start N worker processes (one per GPU) with
    torchrun's environment (WORLD_SIZE, RANK, LOCAL_RANK, MASTER_ADDR=127.0.0.1, MASTER_PORT) and
    wait for them.  Runs before anything touches the GPU (the parent never initialises HIP; the
    workers are fresh processes, not an exec).  If a worker fails the others are terminated (by
    their own PIDs).  Returns rank 0's exit code, or the first non-zero one."""
    import subprocess
    port = _free_port()
    cmd = cmd or [sys.executable, os.path.abspath(__file__)]
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"WORLD_SIZE": str(n), "RANK": str(r), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "PU_BENCH_WORKER": "1"})
        procs.append(subprocess.Popen(cmd + list(argv), env=env))
    rcs = [None] * n
    failed = None
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0) and failed is None:
                    failed = r
                    print("bench: rank %d exited with %d; stopping the other ranks" % (r, rcs[r]), file=sys.stderr)
                    for q in procs:
                        if q.poll() is None:
                            q.terminate()
        time.sleep(poll_s)
    return rcs[failed] if failed is not None else rcs[0]


def check_world(expected, world, devices=None):
    """Exit non-zero when the process group does not have the --gpus ranks asked for, or when
    fewer GPUs are visible than ranks (each rank needs its own device)."""
    if world != expected:
        print("bench: --gpus %d but the process group has %d ranks" % (expected, world), file=sys.stderr)
        sys.exit(3)
    if devices is not None and devices < expected:
        print("bench: --gpus %d but only %d GPU(s) visible" % (expected, devices), file=sys.stderr)
        sys.exit(3)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # torch.cuda.device_count() does not initialise the GPU on this image: safe before spawning
        check_world(args.gpus, args.gpus, torch.cuda.device_count())
        sys.exit(launch_workers(args.gpus, sys.argv[1:]))
    from punet import dp
    world, rank, local = dp.init_from_env("nccl")
    if dist.is_initialized():
        world = dist.get_world_size()
    check_world(args.gpus, world, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)

    from punet import kernels as K
    from punet import _lib
    from punet.engine import Trainer
    build_id = _lib.build_id()

    torch.manual_seed(0)
    net = build_model(args, device)
    net.train()
    dp.broadcast_params(net)
    trainer = Trainer(net, lr=args.lr, steplr=args.steplr, graph=(world == 1 and args.graph == "on"))

    B, S = args.batch, args.img
    g = torch.Generator().manual_seed(1234 + rank)
    NB = 4  # distinct synthetic batches resident in HBM, cycled
    xs = [torch.rand(B, 1, S, S, generator=g).to(device) for _ in range(NB)]
    ts = [(torch.rand(B, S, S, generator=g) > 0.5).float().to(device) for _ in range(NB)]
    hebb = net.initialZeroHebb(B)

    def barrier():
        if world > 1:
            dist.barrier()

    loss = None
    for i in range(args.warmup):
        loss, hebb = trainer.step(xs[i % NB], ts[i % NB], hebb)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss, hebb = trainer.step(xs[i % NB], ts[i % NB], hebb)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per_rank = [elapsed]
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        ts_all = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(ts_all, t)
        per_rank = [x.item() for x in ts_all]
        elapsed = max(per_rank)
    final_loss = loss.item() if loss is not None else float("nan")

    # ---------------- all-reduce accounting (untimed pass): buckets issued, issued during the
    # backward (overlapped), bucket sizes, and the exposed all-reduce time per step - the compute
    # stream's wait between the last backward kernel and Adam (HIP events, punet/engine.py)
    allreduce = {"active": False, "world": world,
                 "note": "single rank: no gradient exchange (the reducer is off at world 1)"}
    if trainer.reducer is not None:
        trainer.measure_allreduce = True
        trainer.allreduce_log = []
        for i in range(max(2, min(5, args.steps))):
            loss, hebb = trainer.step(xs[i % NB], ts[i % NB], hebb)
        torch.cuda.synchronize()
        trainer.measure_allreduce = False
        allreduce = {"active": True, "world": world, "backend": dist.get_backend(),
                     "op": "all_reduce AVG, async, issued from the backward as each bucket completes"}
        allreduce.update(trainer.allreduce_info())
        allreduce.update(trainer.allreduce_stats())
        if world > 1:      # the slowest rank's exposure
            t = torch.tensor([allreduce["exposed_ms_per_step"]], device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            allreduce["exposed_ms_per_step_max_rank"] = round(t.item(), 4)

    # ---------------- instrumented pass: per-launch HIP events on the launching stream
    kern = None
    roof = None
    if not args.no_kernel_profile:
        nprof = max(1, min(3, args.steps))
        # one stream for this pass: with the bf16 trunk's weight-gradient side stream (timed region
        # above) a launch's events would also time the kernels running beside it
        from punet import trunk as _trunk
        side = _trunk._SIDE
        _trunk.set_side_stream(False)
        graph, trainer.graph = trainer.graph, False      # eager steps: the profiler wraps each launch
        try:
            with K.KernelProfiler() as prof:
                for i in range(nprof):
                    loss, hebb = trainer.step(xs[i % NB], ts[i % NB], hebb)
        finally:
            _trunk.set_side_stream(side)
            trainer.graph = graph
        summ = prof.summary()
        kern = {}
        for tag, d in sorted(summ.items(), key=lambda kv: -kv[1]["ms"]):
            e = {"launches_per_step": d["launches"] / nprof, "ms_per_step": round(d["ms"] / nprof, 4)}
            if d["flops"]:
                e["TFLOP_s"] = round(d["flops"] / (d["ms"] * 1e-3) / 1e12, 2)
            if d["bytes"]:
                e["GB_s"] = round(d["bytes"] / (d["ms"] * 1e-3) / 1e9, 1)
            kern[tag] = e
        f32peak, cu, clk = fp32_mfma_peak_tflops(K)
        mfma = {t: d for t, d in summ.items() if d["flops"] and (t.startswith("igemm") or t.startswith("wgrad"))}
        dom = max(mfma.items(), key=lambda kv: kv[1]["ms"])
        dtag, dd = dom
        hbm_bound = ("direct" in dtag or "x6s" in dtag) and dd["bytes"] > 0   # small-channel convs (C4/C5 levels)
        if args.config == "c3":     # v_mfma_f32_32x32x16_bf16: 4096 FLOP/clk/CU dense
            peak = f32peak * 16.0
            basis = "bf16 MFMA 4096 FLOP/clk/CU x %d CU x %.2f GHz (dense)" % (cu, clk)
        elif "x6" in dtag or "wino" in dtag:   # fp32 products as 6 bf16 MFMA products: 4096/6 fp32-FLOP/clk/CU
            peak = f32peak * 16.0 / 6.0
            basis = ("fp32 as 6 bf16 products: bf16 MFMA 4096 FLOP/clk/CU / 6 x %d CU x %.2f GHz "
                     "(fp32-equivalent; native fp32 MFMA peak %.1f TF)" % (cu, clk, f32peak))
        else:
            peak = f32peak
            basis = "fp32 MFMA 256 FLOP/clk/CU x %d CU x %.2f GHz" % (cu, clk)
        # Winograd F(2x2,3x3) layers ("wino" tags) execute 16 products per 4 outputs instead of 36:
        # their MFMA work is 4/9 of the direct-conv FLOPs the profiler records.  `achieved` / `frac`
        # are the executed MFMA rate; the direct-convolution-equivalent rate is reported beside it.
        def executed(tag, flops):
            return flops * (4.0 / 9.0 if "wino" in tag else 1.0)
        ach_eq = dd["flops"] / (dd["ms"] * 1e-3) / 1e12
        ach = executed(dtag, ach_eq)
        tot_eq = sum(d["flops"] for d in mfma.values())
        tot_f = sum(executed(t, d["flops"]) for t, d in mfma.items())
        tot_ms = sum(d["ms"] for d in mfma.values())
        roof = {"kernel": dtag, "bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1),
                "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": None,
                "direct_equivalent_tflop_s": round(ach_eq, 2), "direct_equivalent_frac": round(ach_eq / peak, 4),
                "launches_per_step": dd["launches"] / nprof,
                "avg_launch_us": round(dd["ms"] * 1e3 / dd["launches"], 2),
                "algorithmic_flop_per_launch": dd["flops"] / dd["launches"],
                "executed_mfma_flop_per_launch": executed(dtag, dd["flops"]) / dd["launches"],
                "all_conv_mfma": {"achieved": round(tot_f / (tot_ms * 1e-3) / 1e12, 2),
                                  "frac": round(tot_f / (tot_ms * 1e-3) / 1e12 / peak, 4),
                                  "direct_equivalent_tflop_s": round(tot_eq / (tot_ms * 1e-3) / 1e12, 2),
                                  "flop_per_step": tot_eq / nprof, "executed_flop_per_step": tot_f / nprof,
                                  "ms_per_step": round(tot_ms / nprof, 3)},
                "peak_basis": basis}
        if hbm_bound:   # HBM roofline: algorithmic bytes per launch / launch time vs 8 TB/s
            gbs = dd["bytes"] / (dd["ms"] * 1e-3) / 1e9
            roof.update({"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                         "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_launch": dd["bytes"] / dd["launches"],
                         "mfma_tflop_s": round(ach, 2),
                         "peak_basis": "HBM3E 8 TB/s (MI355X_MICROARCH.md); direct small-channel conv, "
                                       "algorithmic bytes = inputs + outputs + masks"})
        # HBM bytes per launch from the PMC passes (tools/pmc_traffic.py), only when they were
        # taken on this very build (same pu_build_id); otherwise null
        prof_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        roof["traffic_source"] = None
        if os.path.exists(prof_path):
            pmc = json.load(open(prof_path))
            tr = pmc.get("kernels", {}).get(dtag) if pmc.get("build_id") == build_id else None
            if tr:
                roof["traffic"] = tr.get("hbm_bytes_per_launch")
                roof["traffic_source"] = "profiles/pmc_traffic.json (build %s, 2*FETCH_SIZE + WRITE_SIZE)" % build_id
                if tr.get("mfma_busy_frac") is not None:
                    roof["pmc_mfma_busy_frac"] = tr["mfma_busy_frac"]

    oja = None
    if rank == 0 and not args.no_oja:
        oja = oja_update_bench(K, B, S, device, feat_channels=net.outc.conv.weight.shape[1])

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, B)

    if rank == 0:
        value = world * B * args.steps / elapsed
        line = {
            "metric": "training images/sec (%dx%d, bs=%d per GPU)" % (S, S, B),
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "world_size_seen": world,
            "per_rank_ms_per_step": [round(e * 1e3 / args.steps, 3) for e in per_rank],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.config == "c3" else "f32",
            "data": "synthetic: x~U[0,1) [B,1,%d,%d], targets (U>0.5); random init (seed 0)" % (S, S),
            "config": {"workload": CONFIGS[args.config] % vars(args),
                       "global_batch": world * B, "per_gpu_batch": B, "img": S,
                       "parallelism": "dp%d" % world if world > 1 else "single",
                       "step_launch": "hip_graph (fwd + BCE + bwd replayed, Adam eager)" if trainer.graph
                       else "eager",
                       "fp32_gemm": None if args.config == "c3" else
                       {"split6": "fp32 operands split exactly into 3 bf16 terms, 6 bf16 MFMA products per fp32 "
                                  "product, fp32 accumulation (error of an fp32 product)",
                        "native": "v_mfma_f32_32x32x2_f32"}[K.fp32_math()]},
            "build_id": build_id,
            "final_loss": final_loss,
            "roofline": roof,
            "oja_update": oja,
            "allreduce": allreduce,
            "cpu_baseline": cpu,
            "kernels": kern,
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
