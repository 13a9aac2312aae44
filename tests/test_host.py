"""Host-side logic on CPU: the build's IoU metric / RLE match the reference fixtures, batching of
the training loop, CLI parsing."""
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
