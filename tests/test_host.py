"""Host-side logic on CPU: the build's IoU metric / RLE match the reference fixtures, batching of
the training loop, CLI parsing."""
import os
import numpy as np

from conftest import golden


def test_iou_and_rle_match_reference_fixtures():
    from utils import fast_iou_metric, encode
    g = golden("metrics.npz")
    assert abs(fast_iou_metric(g["yt"], g["yp"]) - float(g["iou"])) < 1e-12
    for m, r in zip(g["masks"], g["rles"]):
        assert encode(np.round(m)) == str(r)


def test_train_cli_keeps_reference_flags():
    import train
    a = train.parse_args(["--epochs", "5", "--save_every", "50", "--validate_every", "1", "--learning-rate", "3e-4",
                          "--step-lr", "1e5", "--max-train-time", "-1", "--rollout_every", "100", "--prule", "hebb",
                          "--data", "./data1", "--out", "./out", "--debug"])      # train_model.sh:14-18
    assert (a.epochs, a.save_every, a.validate_every, a.lr, a.steplr, a.prule) == (5, 50, 1, 3e-4, 1e5, "hebb")
    assert a.batch_size == 1 and a.model_type == "unetpres"


def test_batches_shard_contiguously():
    import train
    assert list(train._batches(10, 2, 1, 0)) == [(0, 2), (2, 4), (4, 6), (6, 8), (8, 10)]
    assert list(train._batches(10, 2, 2, 1)) == [(2, 4), (6, 8)]          # rank 1 of 2, drop ragged tail
    assert list(train._batches(3, 1, 1, 0)) == [(0, 1), (1, 2), (2, 3)]     # the reference's bs=1 loop


def _fake_tgs(root, n=30, size=101, seed=0):
    """A TGS-layout directory: train.csv / depths.csv, RGB 8-bit images, 16-bit masks."""
    import os
    from PIL import Image
    rng = np.random.RandomState(seed)
    os.makedirs(os.path.join(root, "train", "images"))
    os.makedirs(os.path.join(root, "train", "masks"))
    ids = ["id%03d" % i for i in range(n)]
    with open(os.path.join(root, "train.csv"), "w") as f:
        f.write("id,rle_mask\n" + "".join("%s,\n" % i for i in ids))
    with open(os.path.join(root, "depths.csv"), "w") as f:
        f.write("id,z\n" + "".join("%s,%d\n" % (i, rng.randint(50, 900)) for i in ids + ["test0"]))
    for k, i in enumerate(ids):
        g = rng.randint(0, 256, (size, size)).astype(np.uint8)
        Image.fromarray(np.stack([g, g, g], -1)).save(os.path.join(root, "train", "images", i + ".png"))
        cov = (0.0, 0.45, 1.0)[k % 3]              # three coverage classes, 10 images each (stratified split)
        m = (rng.rand(size, size) < cov).astype(np.uint16) * 65535
        Image.fromarray(m).save(os.path.join(root, "train", "masks", i + ".png"))
    return ids


def test_tgs_loader_layout_split_and_resize(tmp_path):
    """utils.load_train_dataset (data_set.py:18-70 restated): shapes, [0,1] grey images, binary
    masks, the stratified random_state=42 split, and the skimage-resize restatement."""
    from utils import load_train_dataset, data_set
    root = str(tmp_path / "tgs")
    _fake_tgs(root)
    xt, xv, yt, yv = load_train_dataset(root, 128, 128, 1, val_ratio=0.2)
    assert xt.shape == (24, 1, 128, 128) and xv.shape == (6, 1, 128, 128)
    assert yt.shape == (24, 1, 128, 128) and yv.shape == (6, 1, 128, 128)
    assert 0.0 <= xt.min() and xt.max() <= 1.0
    # same size -> no resize: a 101x101 load returns the grey image exactly
    x101, _, y101, _ = load_train_dataset(root, 101, 101, 1, val_ratio=0.2)
    assert set(np.unique(y101)) <= {0.0, 1.0}
    from PIL import Image
    import os
    g = np.asarray(Image.open(os.path.join(root, "train", "images", "id000.png")).convert("RGB"), np.float64) / 255
    grey = g[..., 0] * 0.2125 + g[..., 1] * 0.7154 + g[..., 2] * 0.0721
    assert any(np.allclose(x[0], grey) for x in x101)
    # resize restatement: interior pixels are bilinear samples at (r + .5) * s - .5, edges fade to 0
    img = np.arange(12, dtype=np.float64).reshape(3, 4)
    r = data_set.resize_bilinear_constant(img, (6, 8))
    assert r.shape == (6, 8)
    # output (2, 3) samples (y, x) = (0.75, 1.25): rows 0/1 weighted .25/.75, columns 1/2 .75/.25
    assert abs(r[2, 3] - (0.25 * (0.75 * img[0, 1] + 0.25 * img[0, 2]) + 0.75 * (0.75 * img[1, 1] + 0.25 * img[1, 2]))) < 1e-12
    assert abs(r[0, 0] - 0.75 * 0.75 * img[0, 0]) < 1e-12          # (-0.25, -0.25): 3 of 4 neighbours are cval 0
    assert data_set.cov_to_class(0.0) == 0 and data_set.cov_to_class(0.35) == 4 and data_set.cov_to_class(1.0) == 10


def test_iou_metric_batch_matches_reference_fixture():
    """utils.iou_metric_batch vs the reference's iou_metric_batch over the 31 logit-space
    thresholds of eval.score_model_best_iou (tests/golden/iou_batch.npz), incl. empty masks."""
    from utils import iou_metric_batch
    g = golden("iou_batch.npz")
    got = np.array([iou_metric_batch(g["y_valid"], g["preds"] > th) for th in g["thresholds"]])
    assert got.dtype == np.float32
    np.testing.assert_array_equal(got, g["ious"])


def test_batch_prefetcher_order_shards_and_slot_rotation():
    """punet.loader.BatchPrefetcher on the CPU device (the ordering logic of the GPU pipeline):
    every yielded batch equals the host slice, ragged last batch included, for depths 2 and 3,
    float64 / memmapped inputs converted to float32."""
    import tempfile
    import torch
    from punet.loader import BatchPrefetcher
    from train import _batches
    g = np.random.RandomState(3)
    X = g.rand(23, 1, 8, 8)                                   # float64 host data
    Y = (g.rand(23, 1, 8, 8) > 0.5).astype(np.float32)
    with tempfile.TemporaryDirectory() as d:
        mm = np.lib.format.open_memmap(d + "/x.npy", mode="w+", dtype=np.float64, shape=X.shape)
        mm[:] = X
        for depth in (2, 3):
            for bs, world, rank in [(4, 1, 0), (3, 2, 1), (5, 1, 0)]:
                ranges = list(_batches(len(X), bs, world, rank))
                pf = BatchPrefetcher(mm, Y, ranges, "cpu", depth=depth)
                seen = []
                for (lo, hi), (x, y) in zip(ranges, pf):
                    assert x.dtype == torch.float32 and x.shape[0] == hi - lo
                    assert torch.equal(x, torch.from_numpy(X[lo:hi].astype(np.float32)))
                    assert torch.equal(y, torch.from_numpy(Y[lo:hi]))
                    seen.append((lo, hi))
                assert seen == ranges
    assert list(BatchPrefetcher(X, Y, [], "cpu")) == []


def test_pmc_kernel_tags_match_bench_tags():
    """tools/pmc_traffic.py keys the PMC bytes by the same kernel tags bench.py's KernelProfiler
    uses (kernels.py), so roofline.traffic finds the dominant kernel's entry."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("pmc_traffic", os.path.join(root, "tools", "pmc_traffic.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.tag_of("void pu::wgrad_halo_x6_kernel<2>(pu::WgradParams)") == "wgrad<128x576,halo,x6>"
    assert m.tag_of("void pu::wgrad_halo_x6_kernel<1>(pu::WgradParams)") == "wgrad<64x576,halo,x6>"
    assert m.tag_of("void pu::igemm_x6_lean_kernel<256, 64, 8, 1, 8, 2>(pu::IgemmParams)") == "igemm<256x64,x6>"
    assert m.tag_of("void pu::wgrad_dma_kernel<128, 256, 2, 2, 3, true, 4, true>(pu::WgradParams)") == \
        "wgrad<128x256,vec4,x6>"
    assert m.tag_of("pu::adam_kernel(pu::AdamBatch, float, float, float, float, float, float, float)") == "adam"


def test_tgs_split_matches_reference_load_train_dataset(tmp_path):
    """The build's load_train_dataset (utils/data_set.py) against the reference's own
    (src/utils/data_set.py:18-63, run by tests/golden/gen_golden.py gen_tgs_split on the same
    synthetic directory): identical train/valid arrays in identical order, without and with the
    24 -> 32 resize.  Pins the CSV join, masks / 65535, coverage classes and the stratified
    random_state=42 split; the resize itself is the build's on both sides (skimage absent)."""
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from tgs_fixture import write_tgs_dir
    from utils.data_set import load_train_dataset
    ref = golden("tgs_split.npz")
    write_tgs_dir(str(tmp_path), ref)
    for tag, S in (("s24", 24), ("s32", 32)):
        got = load_train_dataset(str(tmp_path), S, S, 1, val_ratio=0.2)
        for name, arr in zip(("x_train", "x_valid", "y_train", "y_valid"), got):
            exp = ref[tag + "_" + name]
            assert arr.shape == exp.shape and arr.dtype == exp.dtype, (tag, name, arr.shape, exp.shape)
            assert np.array_equal(arr, exp), (tag, name)
    assert ref["s24_x_valid"].shape[0] == 8            # 20 % of 40, 5 coverage classes x 8
