"""Mask inference - drop-in for yaricom/Plastic-UNet src/infer.py (inference :28-48, predict :50-108).

Forward-only with a zero trace per image (S5); the HIP forward runs in chunks of ``batch`` images.
predict() thresholds the probabilities, RLE-encodes (column-major, utils/rle_encode.py) and writes
the submission CSV with the reference's columns (id, rle_mask).
"""
import csv
import os
from optparse import OptionParser

import numpy as np
import torch

from utils import encode


def inference(net, img_data, device):
    """One image [C,H,W] -> probability mask [H,W] (numpy), as infer.py:28-48."""
    return predict_masks(net, np.asarray(img_data)[None], device)[0]


def predict_masks(net, X, device, batch=32):
    net.eval()
    out = []
    with torch.no_grad():
        for s in range(0, len(X), batch):
            xb = torch.from_numpy(np.asarray(X[s:s + batch], dtype=np.float32)).to(device)
            y, _ = net(xb, net.initialZeroHebb(xb.shape[0]))
            out.append(y.cpu().numpy())
    return np.concatenate(out, 0)


def predict(net, ids, X_test, params):
    """Threshold + RLE + CSV (infer.py:50-108).  ids: image ids, X_test: [N,C,H,W]."""
    masks = predict_masks(net, X_test, params["device"])
    thr = params["mask_threshold"]
    rows = [(fn, encode(np.round(m > thr))) for fn, m in zip(ids, masks)]
    path = os.path.join(params["out_dir"], params.get("subm_file", "submission.csv"))
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["id", "rle_mask"])
        w.writerows(rows)
    print("Results encoded to:", path)
    return rows


def get_args():
    parser = OptionParser()
    parser.add_option('--model', '-m', default='MODEL.pth')
    parser.add_option('-i', '--data', dest='data_dir', type='string', help='test set .npz (ids, x_test)')
    parser.add_option('--out', '-o', dest='out_dir', default='./out')
    parser.add_option('-g', '--gpu', action='store_true', dest='gpu', default=True)
    parser.add_option('--mask-threshold', '-t', dest='mask_threshold', type=float, default=0.5)
    parser.add_option('--model-type', dest='model_type', default='unetpres')
    parser.add_option('--nbf', dest='nbf', type='int', default=101)
    (options, args) = parser.parse_args()
    return options


if __name__ == "__main__":
    args = get_args()
    os.makedirs(args.out_dir, exist_ok=True)
    device = torch.device('cuda')
    from unet import UNetp, UNetpRes
    cls = UNetpRes if args.model_type == 'unetpres' else UNetp
    net = cls(n_channels=1, n_classes=1, device=device, nbf=args.nbf)
    net.load_state_dict(torch.load(args.model, weights_only=True))
    d = np.load(args.data_dir)
    predict(net, [str(i) for i in d["ids"]], d["x_test"],
            {"device": device, "mask_threshold": args.mask_threshold, "out_dir": args.out_dir})
