"""Host-side profile of training steps (cProfile over the Python issue path; timing only).

    python tools/host_profile.py [--config c3] [--steps 10] [--top 45]"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    steps, top = 10, 45
    if "--steps" in argv:
        i = argv.index("--steps")
        steps = int(argv[i + 1])
        del argv[i:i + 2]
    if "--top" in argv:
        i = argv.index("--top")
        top = int(argv[i + 1])
        del argv[i:i + 2]
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
    # the autograd engine runs the backward on its own thread: profile the trunk's backward there
    from punet import trunk as T
    bpr = cProfile.Profile()
    orig = T.UNetpTrunk.backward

    def prof_backward(self, *a, **k):
        bpr.enable()
        try:
            return orig(self, *a, **k)
        finally:
            bpr.disable()
    T.UNetpTrunk.backward = prof_backward
    pr = cProfile.Profile()
    pr.enable()
    for i in range(steps):
        loss, hebb = trainer.step(xs[i % 4], ts[i % 4], hebb)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(top)
    st.sort_stats("cumulative").print_stats(25)
    print("==== trunk backward (autograd thread)")
    bs = pstats.Stats(bpr)
    bs.sort_stats("tottime").print_stats(top)


if __name__ == "__main__":
    main()
