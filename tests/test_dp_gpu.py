"""Data-parallel training step on the GPU: two ranks share cuda:0 over gloo (a one-GPU box cannot
run a two-rank RCCL group), running punet.engine.Trainer with the overlapped bucketed gradient
all-reduce (punet.dp.BucketReducer) that the multi-GPU bench uses over RCCL.  The result must match
one process training on the whole global batch: the same loss and the same averaged gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, PKG

pytestmark = pytest.mark.gpu

B, N, STEPS = 4, 32, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data():
    g = torch.Generator().manual_seed(11)
    xs = [torch.rand(B, 1, N, N, generator=g) for _ in range(STEPS)]
    ts = [(torch.rand(B, N, N, generator=g) > 0.5).float() for _ in range(STEPS)]
    return xs, ts


def _run(net_ctor, lo, hi, dev, bucket_mb):
    from punet.engine import Trainer
    from punet import dp
    torch.manual_seed(0)
    net = net_ctor(dev)
    dp.broadcast_params(net)
    tr = Trainer(net, lr=1e-3, steplr=1e5, bucket_mb=bucket_mb)
    xs, ts = _data()
    hebb = net.initialZeroHebb(hi - lo)
    out = {"loss": [], "grads": [], "overlapped": [], "owns": []}
    for s in range(STEPS):
        loss, hebb = tr.step(xs[s][lo:hi].to(dev), ts[s][lo:hi].to(dev), hebb)
        out["owns"].append(tr.gradbuf.owns_grads())     # every grad landed in the flat buffer
        if dist.is_initialized():
            dist.all_reduce(loss, op=dist.ReduceOp.SUM)
            loss /= dist.get_world_size()
        out["loss"].append(loss.item())
        out["grads"].append({n: p.grad.detach().cpu().clone() for n, p in net.named_parameters()
                             if p.grad is not None})
        out["overlapped"].append(tr.overlapped_buckets)
    out["hebb"] = hebb.cpu()
    return out


def _ctor(dev):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from unet import UNetp
    return UNetp(1, 1, dev, rule="oja", nbf=N, depth=4, base_ch=16)


def _worker(rank, world, port, out_dir):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    lo, hi = rank * B // world, (rank + 1) * B // world
    out = _run(_ctor, lo, hi, dev, bucket_mb=0.05)
    torch.save(out, os.path.join(out_dir, "r%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_dp_matches_single_process(tmp_path, gpu_device):
    world = 2
    ref = _run(_ctor, 0, B, gpu_device, bucket_mb=16)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(os.path.join(tmp_path, "r%d.pt" % r), weights_only=True) for r in range(world)]
    assert all(ref["owns"])
    for r in res:
        assert all(r["owns"]), r["owns"]       # the fused head's outconv grads do not divert the trunk's
        assert all(o >= 2 for o in r["overlapped"]), r["overlapped"]    # buckets went out during backward
        for s in range(STEPS):
            assert abs(r["loss"][s] - ref["loss"][s]) < 1e-5 * abs(ref["loss"][s])
    # step 0: both runs start from the same parameters, so the averaged gradients must agree
    for n, g in ref["grads"][0].items():
        sc = max(g.abs().max().item(), 1e-30)
        for r in res:
            torch.testing.assert_close(r["grads"][0][n], g, rtol=1e-4, atol=1e-5 * sc)
    # per-rank traces are the slots of the single-process run (never synchronised)
    torch.testing.assert_close(torch.cat([r["hebb"] for r in res]), ref["hebb"], rtol=1e-4, atol=1e-6)


def _worker_nccl(rank, world, port, out_dir, side=False):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from punet import trunk
    trunk.set_side_stream(side)       # weight gradients (and bucket issue) on the trunk's side stream
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    from punet.engine import Trainer
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    net = _ctor(dev)
    tr = Trainer(net, lr=1e-3, steplr=1e5, bucket_mb=0.05, force_reduce=True)
    assert tr.reducer is not None
    xs, ts = _data()
    hebb = net.initialZeroHebb(B)
    out = {"loss": [], "grads": [], "overlapped": [], "owns": []}
    tr.measure_allreduce = True       # bench.py's `allreduce` block (events only, no effect on results)
    for s in range(STEPS):
        loss, hebb = tr.step(xs[s].to(dev), ts[s].to(dev), hebb)
        out["owns"].append(tr.gradbuf.owns_grads())
        out["loss"].append(loss.item())
        out["grads"].append({n: p.grad.detach().cpu().clone() for n, p in net.named_parameters()
                             if p.grad is not None})
        out["overlapped"].append(tr.overlapped_buckets)
    out["params"] = {n: p.detach().cpu().clone() for n, p in net.named_parameters()}
    torch.cuda.synchronize()
    out["ar_info"], out["ar_stats"] = tr.allreduce_info(), tr.allreduce_stats()
    torch.save(out, os.path.join(out_dir, "nccl.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("side", [False, True])
def test_rccl_async_bucket_path_world1(tmp_path, gpu_device, side):
    """The production RCCL path of BucketReducer (ReduceOp.AVG, async_op all-reduces issued from
    the autograd thread on RCCL's stream, finish() ordering the compute stream by work.wait()) in
    a world of one rank: AVG over one rank is the identity, so two steps must reproduce the
    no-reducer run bit for bit - a missing stream dependency would let Adam read gradients the
    collective is still writing.  side=True: the weight gradients run on the trunk's side stream
    (PU_WSTREAM) and the buckets are issued from it; the reference run keeps one stream."""
    from punet.engine import Trainer
    torch.manual_seed(0)
    net = _ctor(gpu_device)
    tr = Trainer(net, lr=1e-3, steplr=1e5)
    xs, ts = _data()
    hebb = net.initialZeroHebb(B)
    ref_loss, ref_grads = [], []
    for s in range(STEPS):
        loss, hebb = tr.step(xs[s].to(gpu_device), ts[s].to(gpu_device), hebb)
        ref_loss.append(loss.item())
        ref_grads.append({n: p.grad.detach().cpu().clone() for n, p in net.named_parameters() if p.grad is not None})
    ref_params = {n: p.detach().cpu().clone() for n, p in net.named_parameters()}
    mp.spawn(_worker_nccl, args=(1, _free_port(), str(tmp_path), side), nprocs=1, join=True)
    r = torch.load(os.path.join(tmp_path, "nccl.pt"), weights_only=True)
    assert all(r["owns"]), r["owns"]
    assert all(o >= 2 for o in r["overlapped"]), r["overlapped"]
    # the bench's `allreduce` block: layout, per-step counts and a non-negative exposed time
    info, st = r["ar_info"], r["ar_stats"]
    assert info["buckets"] >= 2 and len(info["bucket_mb"]) == info["buckets"]
    assert abs(sum(info["bucket_mb"]) - info["grad_mb"]) < 1e-3 * (info["buckets"] + 1)
    assert st["steps"] == STEPS and st["buckets_issued"] == info["buckets"]
    assert 2 <= st["buckets_overlapped"] <= st["buckets_issued"]
    assert 0.0 <= st["exposed_ms_per_step"] < 1e3
    assert r["loss"] == ref_loss
    for s in range(STEPS):
        for n, g in ref_grads[s].items():
            assert torch.equal(r["grads"][s][n], g), (s, n)
    for n, p in ref_params.items():
        assert torch.equal(r["params"][n], p), n


# ------------------------------------------------------------------ the two DP configs (C5, C3)
# C5 = UNetpRes with Dropout2d (unet_p_res.py:62,69) over 4 ranks; C3 = the bf16 trunk with the
# weight gradients (and the bucket issue) on the side stream.  Both at world 2 over gloo on one GPU.
#
# Exact check: every rank's averaged gradient must equal, bit for bit, (g_0 + g_1) / 2 of two
# single-process runs on the ranks' shards (same batch per launch -> same kernels and plans; a
# two-operand sum is order-free).  Loose check: the single process on the global batch.
DP_B, DP_N = 4, 32


def _global_mask(step, name, C, p):
    g = torch.Generator().manual_seed(1000 * step + sum(map(ord, name)))
    return torch.empty(DP_B, C).bernoulli_(1.0 - p, generator=g).div_(1.0 - p)


def _dp_net(kind, dev):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from unet import UNetp, UNetpRes
    if kind == "res":
        return UNetpRes(1, 1, dev, neurons=8, rule="oja", nbf=DP_N)
    return UNetp(1, 1, dev, rule="oja", nbf=DP_N, depth=4, base_ch=64, precision="bf16")


def _dp_data():
    g = torch.Generator().manual_seed(23)
    xs = [torch.rand(DP_B, 1, DP_N, DP_N, generator=g) for _ in range(STEPS)]
    ts = [(torch.rand(DP_B, DP_N, DP_N, generator=g) > 0.5).float() for _ in range(STEPS)]
    return xs, ts


def _dp_run(kind, lo, hi, dev, inject, record=False, bucket_mb=0.05):
    """STEPS Trainer steps on slots [lo, hi) of the global batch.  inject: Dropout2d masks are the
    rows [lo, hi) of _global_mask (the single-process masks); record: keep the masks drawn."""
    from punet.engine import Trainer
    from punet import dp
    torch.manual_seed(0)
    net = _dp_net(kind, dev)
    net.train()
    dp.broadcast_params(net)
    tr = Trainer(net, lr=1e-3, steplr=1e5, bucket_mb=bucket_mb)
    trunk = net._trunk_plan()
    state = {"step": 0}
    drawn = []
    if kind == "res":
        if inject:
            trunk.mask_fn = lambda name, B, C, p: _global_mask(state["step"], name, C, p)[lo:hi].contiguous().to(dev)
        elif record:
            orig = trunk._mask

            def rec(name, B, C, p, device):
                m = orig(name, B, C, p, device)
                drawn.append(m.detach().cpu().clone())
                return m
            trunk._mask = rec
    xs, ts = _dp_data()
    hebb = net.initialZeroHebb(hi - lo)
    out = {"loss": [], "grads": [], "overlapped": [], "owns": []}
    for s in range(STEPS):
        state["step"] = s
        loss, hebb = tr.step(xs[s][lo:hi].to(dev), ts[s][lo:hi].to(dev), hebb)
        out["owns"].append(tr.gradbuf.owns_grads())
        out["loss"].append(loss.item())
        out["grads"].append({n: p.grad.detach().cpu().clone() for n, p in net.named_parameters()
                             if p.grad is not None})
        out["overlapped"].append(tr.overlapped_buckets)
    out["hebb"] = hebb.cpu()
    out["masks"] = drawn
    out["side"] = getattr(trunk, "_ws", None) is not None
    return out


def _dp_worker(rank, world, port, out_dir, kind, inject, record):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from punet import trunk as _trunk
    _trunk.set_side_stream(True if kind == "bf16" else False)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    lo, hi = rank * DP_B // world, (rank + 1) * DP_B // world
    out = _dp_run(kind, lo, hi, dev, inject, record)
    torch.save(out, os.path.join(out_dir, "%s%d.pt" % (kind, rank)))
    dist.barrier()
    dist.destroy_process_group()


def _shard_refs(kind, dev, inject):
    from punet import trunk as _trunk
    _trunk.set_side_stream(True if kind == "bf16" else False)
    try:
        return [_dp_run(kind, r * DP_B // 2, (r + 1) * DP_B // 2, dev, inject) for r in range(2)], \
            _dp_run(kind, 0, DP_B, dev, inject)
    finally:
        _trunk.set_side_stream("bf16")


def _check_dp(res, shards, glob, loss_tol, grad_tol):
    for r in res:
        assert all(r["owns"]), r["owns"]
        assert all(o >= 2 for o in r["overlapped"]), r["overlapped"]
    # step 0: both ranks hold exactly the mean of the two shard runs' gradients
    for n, g0 in shards[0]["grads"][0].items():
        want = (g0 + shards[1]["grads"][0][n]) / 2
        for r in res:
            assert torch.equal(r["grads"][0][n], want), n
    for r, sh in zip(res, shards):
        assert r["loss"][0] == sh["loss"][0]
    # against the single process on the global batch (other launch shapes: rounding only)
    for s in range(STEPS):
        mean_loss = sum(r["loss"][s] for r in res) / len(res)
        assert abs(mean_loss - glob["loss"][s]) < loss_tol * abs(glob["loss"][s]), (s, mean_loss, glob["loss"][s])
    num = sum(((res[0]["grads"][0][n] - g) ** 2).sum().item() for n, g in glob["grads"][0].items())
    den = sum((g ** 2).sum().item() for g in glob["grads"][0].values())
    assert (num / den) ** 0.5 < grad_tol, (num / den) ** 0.5
    torch.testing.assert_close(torch.cat([r["hebb"] for r in res]), glob["hebb"], rtol=1e-3, atol=1e-5)


def test_dp_unetpres_dropout_masks_per_rank(tmp_path, gpu_device):
    """C5's DP defect: with the same torch.manual_seed on every rank the
    Dropout2d masks must still differ between ranks (punet.dp.rank_generator via the Trainer)."""
    mp.spawn(_dp_worker, args=(2, _free_port(), str(tmp_path), "res", False, True), nprocs=2, join=True)
    res = [torch.load(os.path.join(tmp_path, "res%d.pt" % r), weights_only=True) for r in range(2)]
    m0, m1 = res[0]["masks"], res[1]["masks"]
    assert len(m0) == len(m1) == 8 * STEPS          # 4 pools + 4 up blocks per forward
    assert all(a.shape == b.shape for a, b in zip(m0, m1))
    diff = sum((a != b).sum().item() for a, b in zip(m0, m1))
    total = sum(a.numel() for a in m0)
    assert diff > 0.2 * total, (diff, total)        # independent draws differ on ~40-50 %
    for r in res:
        assert all(r["owns"]) and all(o >= 2 for o in r["overlapped"])


def test_dp_unetpres_injected_masks_match_single_process(tmp_path, gpu_device):
    """UNetpRes train mode (Dropout2d active) over 2 ranks with each rank's masks = its rows of
    the single process's masks: the averaged gradients are the global batch's."""
    mp.spawn(_dp_worker, args=(2, _free_port(), str(tmp_path), "res", True, False), nprocs=2, join=True)
    res = [torch.load(os.path.join(tmp_path, "res%d.pt" % r), weights_only=True) for r in range(2)]
    shards, glob = _shard_refs("res", gpu_device, True)
    _check_dp(res, shards, glob, loss_tol=1e-5, grad_tol=1e-4)


def test_dp_bf16_side_stream_buckets_match_single_process(tmp_path, gpu_device):
    """The bf16 trunk (C3) with the weight gradients and the bucket all-reduces on the side
    stream (PU_WSTREAM) over 2 ranks."""
    mp.spawn(_dp_worker, args=(2, _free_port(), str(tmp_path), "bf16", False, False), nprocs=2, join=True)
    res = [torch.load(os.path.join(tmp_path, "bf16%d.pt" % r), weights_only=True) for r in range(2)]
    assert all(r["side"] for r in res)
    shards, glob = _shard_refs("bf16", gpu_device, False)
    # bf16 activations: the global-batch run may round a few activations the other way
    _check_dp(res, shards, glob, loss_tol=1e-3, grad_tol=2e-2)
