"""Data-parallel logic on CPU with the gloo backend, world size 2 (the multi-GPU path uses the same
code over RCCL).  The model is the CPU oracle; what is tested is punet.dp: parameter broadcast,
gradient averaging (flat-buffer and coalescing paths) and per-rank traces."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, use_gradbuf):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import oracle
    from punet import dp
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    torch.manual_seed(100 + rank)              # different init on purpose: broadcast must fix it
    net = oracle.RefUNetp(1, 1, rule="oja", nbf=32, depth=3, base_ch=8)
    dp.broadcast_params(net)
    g = torch.Generator().manual_seed(7)        # the same global batch on every rank
    B = 4
    x = torch.rand(B, 1, 32, 32, generator=g)
    t = (torch.rand(B, 32, 32, generator=g) > 0.5).float()
    H = 0.1 * torch.randn(B, 32, 32, generator=g)
    lo, hi = rank * B // world, (rank + 1) * B // world      # contiguous shard
    params = [p for n, p in net.named_parameters() if n != "eta"]
    gradbuf = dp.GradBuffer(params, "cpu") if use_gradbuf else None
    y, hn = net(x[lo:hi], H[lo:hi])
    oracle.bce_loss(y, t[lo:hi]).backward()
    if gradbuf is not None:
        for p, v in zip(params, gradbuf.views):
            v.copy_(p.grad)
            p.grad = v
    dp.allreduce_grads(list(net.parameters()), gradbuf)
    torch.save({"grads": {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None},
                "params": {n: p.detach().clone() for n, p in net.named_parameters()},
                "hebb": hn.detach().clone(), "lo": lo, "hi": hi},
               os.path.join(out_dir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("use_gradbuf", [False, True])
def test_dp_two_ranks_match_single_process(tmp_path, use_gradbuf):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), use_gradbuf), nprocs=world, join=True)
    import oracle
    res = [torch.load(os.path.join(tmp_path, "rank%d.pt" % r), weights_only=True) for r in range(world)]
    # rank 0's init after broadcast == the reference single-process model
    torch.manual_seed(100)
    ref = oracle.RefUNetp(1, 1, rule="oja", nbf=32, depth=3, base_ch=8)
    for n, p in ref.named_parameters():
        for r in res:
            assert torch.equal(r["params"][n], p.detach())
    g = torch.Generator().manual_seed(7)
    x = torch.rand(4, 1, 32, 32, generator=g)
    t = (torch.rand(4, 32, 32, generator=g) > 0.5).float()
    H = 0.1 * torch.randn(4, 32, 32, generator=g)
    y, hn = ref(x, H)
    oracle.bce_loss(y, t).backward()
    for n, p in ref.named_parameters():
        if p.grad is None:
            assert all(n not in r["grads"] for r in res)      # eta: no gradient, not reduced (S3)
            continue
        for r in res:
            torch.testing.assert_close(r["grads"][n], p.grad, rtol=1e-5, atol=1e-9)
    for r in res:                                          # traces are per rank, never synchronised
        torch.testing.assert_close(r["hebb"], hn[r["lo"]:r["hi"]].detach(), rtol=1e-6, atol=1e-8)


def _reducer_worker(rank, world, port, out_dir):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from punet import dp
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    shapes = [(300,), (17, 9), (1000,), (5,), (64, 3, 3), (2,), (4000,)]
    params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
    gb = dp.GradBuffer(params, "cpu")
    red = dp.BucketReducer(gb, bucket_mb=1000 * 4 / (1 << 20))     # ~1000 floats per bucket
    assert len(red.buckets) >= 3
    for step in range(2):
        for i, v in enumerate(gb.views):
            v.copy_(torch.arange(v.numel(), dtype=torch.float32).view_as(v) * (rank + 1) + 100 * i + step)
        red.begin()
        # completion order as a backward would report it, one parameter never reported
        for i in (6, 5, 4, 3, 1, 0):     # param 2 (a bucket of its own) never reports
            gb.ready(params[i])
        early = red.finish()
        assert early >= 1                    # at least one bucket went out during "backward"
        assert gb.reducer is None
        torch.save([v.clone() for v in gb.views], os.path.join(out_dir, "red%d_%d.pt" % (rank, step)))
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_reducer_two_ranks(tmp_path):
    """Overlapped bucketed averaging (punet.dp.BucketReducer): every bucket is averaged exactly
    once, including buckets whose parameters never reported ready, and the reducer disarms."""
    world = 2
    mp.spawn(_reducer_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    shapes = [(300,), (17, 9), (1000,), (5,), (64, 3, 3), (2,), (4000,)]
    for step in range(2):
        got = [torch.load(os.path.join(tmp_path, "red%d_%d.pt" % (r, step)), weights_only=True) for r in range(world)]
        for i, s in enumerate(shapes):
            n = int(torch.tensor(s).prod())
            base = torch.arange(n, dtype=torch.float32).view(s)
            want = sum(base * (r + 1) + 100 * i + step for r in range(world)) / world
            for r in range(world):
                torch.testing.assert_close(got[r][i], want)


def _gen_worker(rank, world, port, out_dir):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from punet import dp
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    torch.manual_seed(5)                     # every rank seeds identically (bench.py / train.py)
    g = dp.rank_generator("cpu")
    m = torch.empty(16, 64).bernoulli_(0.5, generator=g)
    g2 = dp.rank_generator("cpu")            # same rank, same seed: the same stream
    m2 = torch.empty(16, 64).bernoulli_(0.5, generator=g2)
    torch.save({"m": m, "m2": m2}, os.path.join(out_dir, "gen%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_generator_decorrelates_dropout_masks(tmp_path):
    """Dropout2d masks under DP: with the same torch.manual_seed on every rank
    the per-rank generators draw different masks, reproducibly."""
    world = 2
    mp.spawn(_gen_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [torch.load(os.path.join(tmp_path, "gen%d.pt" % r), weights_only=True) for r in range(world)]
    for r in got:
        assert torch.equal(r["m"], r["m2"])
    assert not torch.equal(got[0]["m"], got[1]["m"])
    # independent draws: about half of the mask entries differ between the ranks
    frac = (got[0]["m"] != got[1]["m"]).float().mean().item()
    assert 0.35 < frac < 0.65, frac
