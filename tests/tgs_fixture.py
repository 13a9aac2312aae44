"""Synthetic TGS directory for the split fixture (tests/golden/gen_golden.py gen_tgs_split) and
its CPU test (tests/test_host.py): the same arrays, laid out as train.csv / depths.csv / PNGs."""
import os

import numpy as np


def tgs_synthetic_inputs():
    """A small TGS-shaped data set (train.csv ids, depths.csv, 8-bit RGB images, 16-bit masks)
    whose salt coverage spans five classes with 8 images each (the stratified split needs >= 2 per
    class).  Returned as arrays; tests/test_host.py writes the same files from the fixture."""
    g = np.random.RandomState(33)
    n, S = 40, 24
    ids = np.array(["%010x" % v for v in g.randint(0, 2 ** 40, size=n)])
    test_ids = np.array(["%010x" % v for v in g.randint(0, 2 ** 40, size=6)])
    depths = g.randint(50, 950, size=n + 6).astype(np.int64)
    grey = g.randint(0, 256, size=(n, S, S)).astype(np.uint8)
    images = np.repeat(grey[..., None], 3, axis=-1)
    masks = np.zeros((n, S, S), dtype=np.uint16)
    fracs = [0.0, 0.08, 0.27, 0.45, 0.97]
    for i in range(n):
        k = int(round(fracs[i % 5] * S * S))
        flat = masks[i].reshape(-1)
        flat[g.permutation(S * S)[:k]] = 65535
    return dict(ids=ids, test_ids=test_ids, depths=depths, images=images, masks=masks)


def write_tgs_dir(d, arrs):
    """Lay out arrs (tgs_synthetic_inputs) as the TGS directory load_train_dataset reads."""
    from PIL import Image
    os.makedirs(os.path.join(d, "train", "images"), exist_ok=True)
    os.makedirs(os.path.join(d, "train", "masks"), exist_ok=True)
    ids, test_ids = [str(s) for s in arrs["ids"]], [str(s) for s in arrs["test_ids"]]
    with open(os.path.join(d, "train.csv"), "w") as f:
        f.write("id,rle_mask\n" + "".join("%s,1 1\n" % i for i in ids))
    with open(os.path.join(d, "depths.csv"), "w") as f:
        # depths.csv lists train and test ids in one table (test ids interleaved)
        rows = list(zip(ids + test_ids, arrs["depths"]))
        order = np.random.RandomState(5).permutation(len(rows))
        f.write("id,z\n" + "".join("%s,%d\n" % rows[k] for k in order))
    for i, idx in enumerate(ids):
        Image.fromarray(arrs["images"][i], mode="RGB").save(os.path.join(d, "train", "images", idx + ".png"))
        Image.fromarray(arrs["masks"][i]).save(os.path.join(d, "train", "masks", idx + ".png"))
