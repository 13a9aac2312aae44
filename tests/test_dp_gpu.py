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
