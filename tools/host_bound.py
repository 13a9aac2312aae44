"""Host-side enqueue time of a training step (timing only): how long the Python host takes to
issue K steps (no synchronisation inside the loop) against the GPU time of the same K steps.  If the
two are close, the step is host-bound and the GPU idles between launches.

    python tools/host_bound.py [--config c3] [--steps 20]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    steps = 20
    argv = [a for a in sys.argv[1:]]
    if "--steps" in argv:
        steps = int(argv[argv.index("--steps") + 1])
    sys.argv = [sys.argv[0]] + argv
    args = bench.parse()
    device = torch.device("cuda", 0)
    from punet.engine import Trainer
    torch.manual_seed(0)
    net = bench.build_model(args, device)
    net.train()
    trainer = Trainer(net, lr=args.lr, steplr=args.steplr)
    B, S = args.batch, args.img
    g = torch.Generator().manual_seed(1234)
    xs = [torch.rand(B, 1, S, S, generator=g).to(device) for _ in range(4)]
    ts = [(torch.rand(B, S, S, generator=g) > 0.5).float().to(device) for _ in range(4)]
    hebb = net.initialZeroHebb(B)
    for i in range(5):
        loss, hebb = trainer.step(xs[i % 4], ts[i % 4], hebb)
    torch.cuda.synchronize()
    for rep in range(3):
        per = []
        t0 = time.perf_counter()
        for i in range(steps):
            a = time.perf_counter()
            loss, hebb = trainer.step(xs[i % 4], ts[i % 4], hebb)
            per.append((time.perf_counter() - a) * 1e3)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        per.sort()
        print("config %s: %d steps  host enqueue %.3f ms/step (median step %.3f, max %.3f)  wall %.3f ms/step"
              % (args.config, steps, t_host / steps * 1e3, per[len(per) // 2], per[-1], t_all / steps * 1e3))


if __name__ == "__main__":
    main()
