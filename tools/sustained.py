"""Sustained C2 training run: does the bench's 20-step rate hold over a long run?

    python tools/sustained.py [--steps 600] [--chunk 50] [--out profiles/r05_sustained_c2.json]

The bench's workload (UNetp depth 5 / base 64, Oja, 128^2, bs 32, fp32, traces carried, Adam +
StepLR per step), timed in chunks of --chunk steps with HIP events; between chunks the GPU's
current shader clock and power are sampled with rocm-smi (sysfs; a host-side reading, which the
microarchitecture guide notes can read up to ~10 % above the in-kernel clock)."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def smi():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--json"], capture_output=True, text=True,
                           timeout=20)
        d = json.loads(r.stdout)
        card = d[sorted(d)[0]]
        out = {}
        for k, v in card.items():
            kl = k.lower()
            if "sclk" in kl and "speed" in kl:
                out["sclk"] = v
            elif "power" in kl:
                out["power"] = v
        return out
    except Exception as e:          # noqa: BLE001 - a missing tool must not stop the run
        return {"error": str(e)[:80]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--chunk", type=int, default=50)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_sustained_c2.json"))
    a = ap.parse_args()
    from punet.engine import Trainer
    from punet import _lib
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    from unet import UNetp
    net = UNetp(1, 1, dev, rule="oja", nbf=128, depth=5, base_ch=64)
    net.train()
    tr = Trainer(net, lr=3e-4, steplr=1e5)
    B, S, NB = 32, 128, 4
    g = torch.Generator().manual_seed(1234)
    xs = [torch.rand(B, 1, S, S, generator=g).to(dev) for _ in range(NB)]
    ts = [(torch.rand(B, S, S, generator=g) > 0.5).float().to(dev) for _ in range(NB)]
    hebb = net.initialZeroHebb(B)
    for i in range(10):
        loss, hebb = tr.step(xs[i % NB], ts[i % NB], hebb)
    torch.cuda.synchronize()
    chunks = []
    t_start = time.perf_counter()
    step = 0
    while step < a.steps:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.chunk):
            loss, hebb = tr.step(xs[step % NB], ts[step % NB], hebb)
            step += 1
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        c = {"steps": step, "ms_per_step": round(ms / a.chunk, 3), "img_s": round(B * a.chunk / (ms / 1e3), 1),
             "loss": round(loss.item(), 5), "t_s": round(time.perf_counter() - t_start, 2)}
        c.update(smi())
        chunks.append(c)
        print(json.dumps(c), flush=True)
    rates = [c["img_s"] for c in chunks]
    out = {"workload": "C2 UNetp d5 c64 oja 128^2 bs 32 fp32, fwd+BCE+bwd+Adam, traces carried",
           "build_id": _lib.build_id(), "steps": step, "chunk": a.chunk,
           "img_s_first_chunk": rates[0], "img_s_last_chunk": rates[-1],
           "img_s_mean": round(sum(rates) / len(rates), 1), "img_s_min": min(rates), "img_s_max": max(rates),
           "chunks": chunks}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("sustained:", {k: v for k, v in out.items() if k != "chunks"})


if __name__ == "__main__":
    main()
