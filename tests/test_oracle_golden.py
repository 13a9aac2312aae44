"""Pin the CPU oracle (oracle/ref_cpu.py) to the reference's own outputs (tests/golden/*.npz).

The fixtures were produced by tests/golden/gen_golden.py importing yaricom/Plastic-UNet's
``src/unet`` (and ``src/train.py`` with stubs) in the build container.
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import golden

torch.set_num_threads(4)


def _t(a):
    return torch.from_numpy(np.asarray(a))


def close(a, b, rtol=1e-5, atol=1e-6):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), rtol=rtol, atol=atol)


@pytest.mark.parametrize("rule", ["hebb", "oja"])
@pytest.mark.parametrize("N", [32, 128])
def test_head_fixture(rule, N):
    g = golden("head_%s_N%d.npz" % (rule, N))
    w = _t(g["w"]).requires_grad_(True)
    al = _t(g["alpha"]).requires_grad_(True)
    X = _t(g["X"])[None].clone().requires_grad_(True)
    Y, Hn = oracle.plastic_head(X, _t(g["H"])[None], w, al, _t(g["eta"]), rule)
    loss = oracle.bce_loss(Y, _t(g["t"]))
    loss.backward()
    close(Y[0], g["Y"])
    close(Hn[0], g["Hn"])
    close(loss, g["loss"])
    close(X.grad[0], g["dX"], atol=1e-8)
    close(w.grad, g["dw"], atol=1e-8)
    close(al.grad, g["dalpha"], atol=1e-8)


@pytest.mark.parametrize("rule", ["hebb", "oja"])
def test_trace_sequence_fixture(rule):
    g = golden("trace_seq_%s.npz" % rule)
    H = torch.zeros(1, 32, 32)
    for k in range(16):
        Y, H = oracle.plastic_head(_t(g["X"][k])[None], H, _t(g["w"]), _t(g["alpha"]), _t(g["eta"]), rule)
        close(Y[0], g["Y"][k])
        close(H[0], g["H"][k])


def _load(net, g, prefix="p."):
    sd = {k[len(prefix):]: _t(v) for k, v in g.items() if k.startswith(prefix)}
    net.load_state_dict(sd)


def test_unetp_c8_init_matches_reference_rng():
    g = golden("unetp_c8_init.npz")
    torch.manual_seed(0)
    net = oracle.RefUNetp(1, 1, rule="oja", nbf=64)
    sd = net.state_dict()
    assert sorted(sd.keys()) == sorted(k[2:] for k in g)
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), g["p." + k])
    assert sum(p.numel() for p in oracle.RefUNetp(1, 1, nbf=128).parameters()) == 264314


def test_unetp_c8_fwd_bwd():
    gi, g = golden("unetp_c8_init.npz"), golden("unetp_c8_step.npz")
    net = oracle.RefUNetp(1, 1, rule="oja", nbf=64)
    _load(net, gi)
    y, hn = net(_t(g["x"]), _t(g["hebb"]))
    loss = oracle.bce_loss(y, _t(g["t"]))
    loss.backward()
    close(y, g["Y"])
    close(hn, g["Hn"])
    close(loss, g["loss"])
    for k, p in net.named_parameters():
        if p.grad is None:
            assert "g." + k not in g and k == "eta"      # S3: eta never gets a gradient
            continue
        close(p.grad, g["g." + k], rtol=1e-4, atol=1e-7)


def test_unetp_c8_adam_steplr():
    gi, g = golden("unetp_c8_init.npz"), golden("unetp_c8_adam.npz")
    net = oracle.RefUNetp(1, 1, rule="oja", nbf=64)
    _load(net, gi)
    opt = oracle.ref_adam(net.parameters(), 1e-3)
    sch = oracle.ref_steplr(opt, 2)
    hebb = net.initialZeroHebb()
    losses = []
    for k in range(3):
        loss, _, hebb = oracle.ref_train_step(net, opt, sch, _t(g["xs"][k]), _t(g["ts"][k]), hebb)
        losses.append(loss.item())
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-6)
    close(hebb, g["hebb"], rtol=1e-4, atol=1e-6)
    for k, v in net.state_dict().items():
        close(v, g["p." + k], rtol=1e-4, atol=1e-6)


def test_generalised_depth4_base16_two_slots():
    gi, g = golden("unetp_d4c16_bs2_init.npz"), golden("unetp_d4c16_bs2_out.npz")
    net = oracle.RefUNetp(1, 1, rule="hebb", nbf=128, depth=4, base_ch=16)
    _load(net, gi)
    y, hn = net(_t(g["x"]), _t(g["H"]))
    loss = oracle.bce_loss(y, _t(g["t"]))
    loss.backward()
    close(y, g["Y"][:, 0] if g["Y"].ndim == 4 else g["Y"])
    close(hn, g["Hn"])
    close(loss, g["loss"])
    for k, p in net.named_parameters():
        if k == "eta":
            continue
        close(p.grad, g["g." + k], rtol=1e-4, atol=1e-7)


def test_c64_widths_checksums():
    g = golden("unetp_c64_sum.npz")
    net = oracle.det_init_(oracle.RefUNetp(1, 1, rule="oja", nbf=32, depth=5, base_ch=64), 31)
    for k, p in net.named_parameters():
        if k in ("w", "alpha", "eta"):
            continue
        np.testing.assert_allclose(p.detach().double().sum().item(), g["psum." + k][0], rtol=1e-6)
    y, hn = net(_t(g["x"]), _t(g["H"]))
    loss = oracle.bce_loss(y, _t(g["t"]))
    loss.backward()
    close(y, g["Y"])
    close(hn, g["Hn"])
    close(loss, g["loss"])
    for k, p in net.named_parameters():
        if k == "eta":
            continue
        gg = p.grad.double()
        got = np.array([gg.sum().item(), gg.abs().sum().item(), gg.norm().item()])
        np.testing.assert_allclose(got[1:], g["gsum." + k][1:], rtol=1e-4)
        np.testing.assert_allclose(got[0], g["gsum." + k][0], rtol=1e-3, atol=1e-6 * got[1])
        if "ghead." + k in g:
            close(p.grad.reshape(-1)[:16], g["ghead." + k], rtol=1e-3, atol=1e-7)


def test_unetpres_eval_fwd_bwd():
    g, gg = golden("unetpres_n4.npz"), golden("unetpres_n4_grad.npz")
    torch.manual_seed(5)
    net = oracle.RefUNetpRes(1, 1, neurons=4, rule="oja", nbf=101)
    for k, v in net.state_dict().items():       # same RNG consumption order as the reference
        np.testing.assert_array_equal(v.numpy(), g["p." + k])
    net.eval()
    y, hn = net(_t(g["x"]), _t(g["H"]))
    loss = oracle.bce_loss(y, _t(g["t"]))
    loss.backward()
    close(y, g["Y"])
    close(hn, g["Hn"])
    close(loss, g["loss"])
    for k, p in net.named_parameters():
        if k == "eta":
            continue
        close(p.grad, gg["g." + k], rtol=1e-4, atol=1e-7)


def test_residual_block_and_res_up_crop():
    g = golden("res_blocks.npz")
    rb = oracle.ref_cpu._ResidualBlock(6)
    rb.load_state_dict({k[3:]: _t(v) for k, v in g.items() if k.startswith("rb.")})
    close(rb(_t(g["rb_x"])), g["rb_y"])
    up = oracle.ref_cpu._ResUp(8, 4, 0.0)
    up.load_state_dict({k[3:]: _t(v) for k, v in g.items() if k.startswith("up.")})
    up.eval()
    close(up(_t(g["up_x1"]), _t(g["up_x2"])), g["up_y"])


def test_bce_clamp_edges():
    g = golden("bce_edge.npz")
    y = _t(g["y"]).requires_grad_(True)
    loss = oracle.bce_loss(y, _t(g["t"]))
    loss.backward()
    close(loss, g["loss"])
    close(y.grad, g["dy"])
    z = _t(g["z"]).requires_grad_(True)
    yz = torch.sigmoid(z)
    lz = oracle.bce_loss(yz, _t(g["tz"]))
    lz.backward()
    close(yz, g["yz"])
    close(lz, g["lz"])
    close(z.grad, g["dz"])
    assert g["dz"][3] == 0.0 and g["dz"][4] == 0.0        # S9: saturated sigmoid, zero gradient


def test_train_loop_capture():
    g = golden("train_capture.npz")
    net = oracle.RefUNetp(1, 1, rule="oja", nbf=32)
    _load(net, g, "init.")
    out = oracle.ref_train_loop(net, g["X_train"], g["y_train"], g["X_val"], g["y_val"],
                                epochs=2, lr=3e-4, steplr=4)
    np.testing.assert_allclose(out[0], g["all_losses"], rtol=1e-5)
    np.testing.assert_allclose(out[1], g["val_train_losses"], rtol=1e-5)
    np.testing.assert_allclose(out[2], g["val_test_losses"], rtol=1e-5)
    np.testing.assert_allclose(out[3], g["val_accuracies"], rtol=1e-6)
    for k, v in net.state_dict().items():
        close(v, g["final." + k], rtol=1e-4, atol=1e-6)


def test_metrics_fixture():
    g = golden("metrics.npz")
    assert abs(oracle.fast_iou_metric(g["yt"], g["yp"]) - float(g["iou"])) < 1e-12
    for m, r in zip(g["masks"], g["rles"]):
        assert oracle.rle_encode_mask(np.round(m)) == str(r)


def test_add_coords_closed_form():
    x = torch.zeros(2, 1, 5, 5)
    out = oracle.add_coords(x, with_r=True)
    assert out.shape == (2, 4, 5, 5)
    assert torch.allclose(out[0, 1, 3], torch.tensor([-1.0, -0.5, 0.0, 0.5, 1.0]))
    assert torch.allclose(out[0, 2, :, 2], torch.tensor([-1.0, -0.5, 0.0, 0.5, 1.0]))
    assert torch.allclose(out[1, 3, 0, 0], torch.tensor(np.sqrt(2 * 1.5 ** 2), dtype=torch.float32))


@pytest.mark.parametrize("tag,bn,bil", [("bn", True, False), ("bilinear", False, True), ("bn_bilinear", True, True),
                                        ("bn_bilinear_m", True, True)])
def test_unetp_variants_fixture(tag, bn, bil):
    """UNetp(batch_norm / bilinear_upsample): init RNG order, train-mode fwd/bwd, the running
    statistics after two forwards, and the eval-mode forward (reference, unet_p.py:186-193, :235-236).
    bn_bilinear_m: the margin-certified 32x32 fixture (seed 500 + s for the init, see gen_golden.py)."""
    g = golden("unetp_%s.npz" % tag)
    nbf = 32 if tag.endswith("_m") else 64
    torch.manual_seed(500 + int(g["seed"]) if tag.endswith("_m") else 5)
    net = oracle.RefUNetp(1, 1, rule="oja", nbf=nbf, batch_norm=bn, bilinear_upsample=bil)
    for k, v in net.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), g["p." + k])
    net.train()
    xs = _t(g["xs"])
    y, hn = net(xs[0], _t(g["hebb"]))
    loss = oracle.bce_loss(y, _t(g["t"]))
    loss.backward()
    close(y, g["Y"])
    close(hn, g["Hn"])
    close(loss, g["loss"])
    for k, p in net.named_parameters():
        if p.grad is None:
            assert k == "eta"
            continue
        close(p.grad, g["g." + k], rtol=1e-4, atol=1e-7)
    sd = net.state_dict()
    for k in sd:
        if "s1." + k in g:
            close(sd[k], g["s1." + k])
    with torch.no_grad():
        y2, _ = net(xs[1], _t(g["hebb"]))
    close(y2, g["Y2"])
    sd = net.state_dict()
    nbuf = 0
    for k in sd:
        if "s2." + k in g:
            close(sd[k], g["s2." + k])
            nbuf += 1
    assert nbuf == (3 * 18 if bn else 0)      # 18 BatchNorm2d layers x (mean, var, count)
    net.eval()
    with torch.no_grad():
        ye, he = net(xs[2], torch.zeros(nbf, nbf))
    close(ye, g["Ye"])
    close(he, g["He"])


def test_unetp_bn_batched_slots_equal_sequential():
    """Two slots in one training-mode forward == two sequential bs=1 forwards (per-slot
    statistics; running statistics updated in slot order)."""
    g = golden("unetp_bn.npz")
    a = oracle.RefUNetp(1, 1, rule="oja", nbf=64, batch_norm=True)
    _load(a, g)
    b = oracle.RefUNetp(1, 1, rule="oja", nbf=64, batch_norm=True)
    _load(b, g)
    xs = _t(g["xs"])[:2, 0]
    H = torch.stack([_t(g["hebb"])] * 2)
    with torch.no_grad():
        yb, _ = a(xs, H)
        y0, _ = b(xs[0:1], H[0])
        y1, _ = b(xs[1:2], H[1])
    close(yb[0], y0, rtol=0, atol=0)
    close(yb[1], y1, rtol=0, atol=0)
    for k, v in a.state_dict().items():
        close(v, b.state_dict()[k], rtol=0, atol=0)
    for k in a.state_dict():
        if "s2." + k in g:
            close(a.state_dict()[k], g["s2." + k])


def test_unetpres_bn_fixture():
    """UNetpRes(batch_norm=True): residual blocks with BatchNorm (unet_p_res.py:149-153, :171-176),
    training-mode fwd/bwd, running statistics after two forwards, eval-mode forward."""
    g = golden("unetpres_bn.npz")
    torch.manual_seed(6)
    net = oracle.RefUNetpRes(1, 1, neurons=4, dropout_ratio=0.0, rule="oja", nbf=64, batch_norm=True)
    for k, v in net.state_dict().items():          # RNG-order-identical init (fp64 sums stored)
        assert abs(v.double().sum().item() - float(g["sum." + k])) <= 1e-9 * max(1.0, abs(float(g["sum." + k])))
    net.train()
    xs = _t(g["xs"])
    y, hn = net(xs[0], _t(g["hebb"]))
    loss = oracle.bce_loss(y, _t(g["t"]))
    loss.backward()
    close(y, g["Y"])
    close(hn, g["Hn"])
    close(loss, g["loss"])
    for k, p in net.named_parameters():
        if p.grad is None:
            assert k == "eta"
            continue
        close(p.grad, g["g." + k], rtol=1e-4, atol=1e-7)
    for k, v in net.state_dict().items():
        if "s1." + k in g:
            close(v, g["s1." + k])
    with torch.no_grad():
        y2, _ = net(xs[1], _t(g["hebb"]))
    close(y2, g["Y2"])
    nbuf = 0
    for k, v in net.state_dict().items():
        if "s2." + k in g:
            close(v, g["s2." + k])
            nbuf += 1
    assert nbuf == 3 * 10                           # 5 stacks x 2 residual blocks x 1 BatchNorm2d
    net.eval()
    with torch.no_grad():
        ye, he = net(xs[2], torch.zeros(64, 64))
    close(ye, g["Ye"])
    close(he, g["He"])
