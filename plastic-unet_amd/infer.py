"""Mask inference - drop-in for yaricom/Plastic-UNet src/infer.py: inference (:28-48), predict
(:50-108), start_inference (:110-179) and the CLI (:181-263).

Forward-only with a zero trace per image (S5); the HIP forward runs in chunks of ``batch`` images
(each slot with its own zero trace: the per-image math of the reference).  predict() thresholds
the probabilities, RLE-encodes (column-major, utils/rle_encode.py) and writes the submission CSV
with the reference's columns (id, rle_mask).  start_inference() builds the reference's model
(UNetpRes at the image width), loads the state dict with the weights-only loader, picks the mask
threshold with eval.score_model_best_iou (whose reference version raises at S12 - see there) and
predicts.
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
    """Probability masks [N,H,W] of images X [N,C,H,W], zero trace per image."""
    net.eval()
    out = []
    with torch.no_grad():
        for s in range(0, len(X), batch):
            xb = torch.from_numpy(np.asarray(X[s:s + batch], dtype=np.float32)).to(device)
            y, _ = net(xb, net.initialZeroHebb(xb.shape[0]))
            out.append(y.cpu().numpy())
    return np.concatenate(out, 0)


def _write_mask_png(path, mask):
    from PIL import Image
    tmp = (np.squeeze(mask).astype(np.uint8) * 255)
    Image.fromarray(np.dstack((tmp, tmp, tmp))).save(path)


def predict(net, test_df, params, visualize=False, save_masks=False):
    """Threshold + RLE + CSV (infer.py:50-108).  test_df: the reference's test frame (index = image
    ids, column ``images``), or a pair (ids, X_test [N,C,H,W]).  params: out_dir, mask_threshold,
    img_chan/img_height/img_width (to shape the images), subm_file, device (default: the net's).
    ``visualize`` (matplotlib windows in the reference) is not supported on this host-less path."""
    if isinstance(test_df, tuple):
        ids, X_test = test_df
        ids = list(ids)
    else:
        ids = list(test_df.index)
        X_test = np.array(test_df.images.tolist()).reshape(-1, params["img_chan"], params["img_height"],
                                                             params["img_width"])
    print("Start prediction with the number of test image samples:", len(ids))
    device = params.get("device") or next(net.parameters()).device
    masks = predict_masks(net, X_test, device)
    thr = params["mask_threshold"]
    if save_masks:
        os.makedirs(os.path.join(params["out_dir"], "masks"), exist_ok=True)
        for fn, m in zip(ids, masks):
            _write_mask_png(os.path.join(params["out_dir"], "masks", "%s.png" % fn), m > thr)
    rows = [(fn, encode(np.round(m > thr))) for fn, m in zip(ids, masks)]
    path = os.path.join(params["out_dir"], params.get("subm_file", "submission.csv"))
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["id", "rle_mask"])
        w.writerows(rows)
    print("Results encoded to:", path)
    return rows


def start_inference(model, test_df, X_valid, y_valid, out_dir, img_width, img_height, img_chan,
                    subm_file="submission.csv", gpu=True, visualize=False, save_masks=False, debug=False,
                    mask_threshold=None, model_type="unetpres"):
    """infer.py:110-179: the reference builds UNetpRes(n_channels=img_chan, n_classes=1,
    nbf=img_width), loads ``model`` (a state_dict path), scores the best threshold on the
    validation set and predicts.  ``mask_threshold`` skips the threshold search; ``model_type``
    'unetp' loads a UNetp instead.  The product path is the GPU one (``gpu`` is accepted for the
    signature; there is no CPU fallback)."""
    from unet import UNetp, UNetpRes
    import eval as ev
    device = torch.device("cuda")
    cls = UNetpRes if model_type == "unetpres" else UNetp
    net = cls(n_channels=img_chan, n_classes=1, nbf=img_width, device=device)
    print("Loading model %s" % (model,))
    sd = model if isinstance(model, dict) else torch.load(model, map_location="cpu", weights_only=True)
    net.load_state_dict(sd)
    net.to(device)
    if mask_threshold is None:
        print("Score model for best IoU")
        mask_threshold, iou_best = ev.score_model_best_iou(net, X_valid, y_valid, device, debug=debug)
        print("Best threshold: %f, best IoU: %f" % (mask_threshold, iou_best))
    os.makedirs(out_dir, exist_ok=True)
    params = {"out_dir": out_dir, "device": device, "img_width": img_width, "img_height": img_height,
              "img_chan": img_chan, "mask_threshold": mask_threshold, "subm_file": subm_file, "debug": debug}
    return predict(net, test_df, params, visualize=visualize, save_masks=save_masks)


def get_args():
    parser = OptionParser()
    parser.add_option('--model', '-m', default='MODEL.pth',
                      help="Specify the file in which is stored the model (default : 'MODEL.pth')")
    parser.add_option('-i', '--data', dest='data_dir', type='string', help='the directory with input test data')
    parser.add_option('--out', '-o', dest='out_dir', default='./out', help='directory for ouput images')
    parser.add_option('-g', '--gpu', action='store_true', dest='gpu', default=True, help='use the GPU (always)')
    parser.add_option('--visualize', '-v', action='store_true', default=False)
    parser.add_option('--save', '-s', action='store_true', default=False, help="To save the output masks")
    parser.add_option('--mask-threshold', '-t', dest='mask_threshold', type=float,
                      help="Minimum probability value to consider a mask pixel white")
    parser.add_option('--partial', '-p', action='store_true', default=False)
    parser.add_option('--partial-size', '-d', dest='partial_size', default=100, type='int')
    parser.add_option('--model-type', dest='model_type', default='unetpres', help='unetpres | unetp')
    (options, args) = parser.parse_args()
    return options


if __name__ == "__main__":
    args = get_args()
    os.makedirs(args.out_dir, exist_ok=True)
    if args.data_dir is None:
        raise ValueError("The input data directory or dataset file not specified")
    from utils import load_test_dataset, load_train_dataset
    w = h = 101
    c = 1
    test_df = load_test_dataset(args.data_dir, w, h, c, partial=args.partial, part_size=args.partial_size)
    x_train, x_valid, y_train, y_valid = load_train_dataset(args.data_dir, w, h, c)
    if args.partial:
        x_valid = x_valid[:args.partial_size]
        y_valid = y_valid[:args.partial_size]
    start_inference(model=args.model, test_df=test_df, X_valid=x_valid, y_valid=y_valid, out_dir=args.out_dir,
                    gpu=args.gpu, img_width=w, img_height=h, img_chan=c, visualize=args.visualize,
                    save_masks=args.save, debug=True, mask_threshold=args.mask_threshold,
                    model_type=args.model_type)
