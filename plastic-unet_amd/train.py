"""Model training - drop-in for yaricom/Plastic-UNet src/train.py on MI355X.

Same entry points (train(), start_train(), the optparse CLI flags of train.py:316-358) and the same
per-epoch structure (train.py:78-211): zero the plastic trace each epoch (:88), run the hot loop
(forward -> BCELoss -> backward -> Adam -> StepLR, :91-112), validate with a zero trace (:131-147),
save checkpoints (:153-203).  Differences, all opt-in:
  --batch-size B   B slots per step with per-slot traces (B=1 is the reference's loop exactly)
  --hebb-mode sequential   one trace threaded through the B samples of each step in order
  --batch-norm / --bilinear  the reference constructor flags batch_norm / bilinear_upsample
  --model-type     unetpres (reference default) | unetp, with --depth/--base-ch for UNetp
  --synthetic N / --dataset FILE.npz   input data besides --data DIR (the TGS PNG layout, utils/data_set.py)
  --resident       keep the whole training set in HBM; default: batches stream host -> HBM through
                   pinned, double-buffered asynchronous copies (punet/loader.py) under the previous step
Data-parallel training: launch with torch.distributed.run; each rank trains its contiguous shard
of every global batch and gradients are averaged over RCCL.
Checkpoints: ``{out}/train[_{epoch}]_net.pth`` (state_dict, reference keys), the training parameters
pickled to ``_parameters.dat`` (:199-200), and the HDF5 payload of :178-196 under the same keys in
``{out}/train[_{epoch}]_data.npz`` (h5py is not installed).
"""
import os
import pickle
import sys
import time
from datetime import datetime
from optparse import OptionParser

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from unet import UNetp, UNetpRes  # noqa: E402
from punet import dp  # noqa: E402
from punet.engine import Trainer  # noqa: E402
from punet.loader import BatchPrefetcher  # noqa: E402
from eval import eval_net  # noqa: E402


def _batches(n, bs, world, rank):
    """Global batches of bs*world samples; this rank's contiguous shard of each."""
    g = bs * world
    for s in range(0, n - n % g if n >= g else n, g):
        lo = s + rank * bs
        yield lo, min(lo + bs, n)


def train(net, X_train, X_val, y_train, y_val, params):
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    verbose = rank == 0
    if verbose:
        print("Train samples shape:", X_train.shape)
        print("Train labels shape:", y_train.shape)
        print("Validation samples shape:", X_val.shape)
        print("Validation labels shape:", y_val.shape)
        print(params)
    bs = int(params.get("batch_size", 1))
    device = params["device"]
    all_losses, val_train_losses, val_test_losses, val_accuracies = [], [], [], []
    samples_count = len(X_train)
    loss_between_saves, last_save_epoch = 0.0, 0
    trainer = Trainer(net, lr=params["lr"], steplr=params["steplr"], gamma=params["gamma"])
    ranges = list(_batches(samples_count, bs, world, rank))
    if params.get("prefetch", True):
        # stream batches host -> HBM (pinned, double-buffered, overlapping the previous step)
        batches = BatchPrefetcher(X_train, y_train, ranges, device)
    else:
        # the whole training set resident in HBM (copied once)
        X_dev = torch.from_numpy(np.asarray(X_train, dtype=np.float32)).to(device)
        Y_dev = torch.from_numpy(np.asarray(y_train, dtype=np.float32)).to(device)
        batches = [(X_dev[lo:hi], Y_dev[lo:hi]) for lo, hi in ranges]
    if params["stop_time"] > 0 and verbose:
        print("Training started at: [%s] and set to stop at: [%s]" % (
            datetime.fromtimestamp(time.time()).strftime("%B %d, %Y %H:%M:%S"),
            datetime.fromtimestamp(params["stop_time"]).strftime("%B %d, %Y %H:%M:%S")))
    for epoch in range(params["epochs"]):
        net.train()
        epoch_start_time = time.time()
        seq = getattr(net, "hebb_mode", "slots") == "sequential"
        # trace reset per epoch (train.py:88): per-slot traces, or one trace threaded through
        hebb = net.initialZeroHebb() if seq else net.initialZeroHebb(bs)
        losses_dev = []
        for (lo, hi), (x, yb) in zip(ranges, batches):
            t = yb.reshape(hi - lo, -1)
            if seq:
                loss, hebb = trainer.step(x, t, hebb)
            else:
                h = hebb[: hi - lo]
                loss, h = trainer.step(x, t, h)
                if hi - lo == bs:
                    hebb = h
            losses_dev.append(loss)
        # one host sync per epoch instead of loss.item() per sample (train.py:106)
        epoch_losses = torch.stack(losses_dev).cpu().tolist() if losses_dev else []
        all_losses.extend(epoch_losses)
        epoch_loss = np.mean(all_losses[-max(1, len(epoch_losses))]) if all_losses else float("nan")  # S16
        loss_between_saves += epoch_loss
        epoch_time = time.time() - epoch_start_time
        next_epoch_finish_time = epoch_time + time.time()
        terminate = (params["stop_time"] > 0 and next_epoch_finish_time >= params["stop_time"]) or \
            (epoch + 1) == params["epochs"]
        if params["debug"] and verbose:
            print("Epoch finished! Loss: %f, time spent: %d, terminate due to time limits: %s"
                  % (epoch_loss, epoch_time, terminate))
        if (epoch + 1) % params["val_every"] == 0 or terminate:
            val_acc, val_loss = eval_net(net, X_val, y_val, device)
            val_train_losses.append(epoch_loss)
            val_test_losses.append(val_loss)
            val_accuracies.append(val_acc)
            if params["debug"] and verbose:
                print("Validation accuracy: %f, loss: %f" % (val_acc, val_loss))
                print("Eta:", net.eta.data.cpu().numpy())
        if ((epoch + 1) % params["save_every"] == 0 or terminate) and verbose:
            last_save_epoch = epoch
            loss_between_saves = 0.0
            prefix = params["out_dir"] + "/train"
            if (epoch + 1) % params["rollout"] == 0 and not terminate:
                prefix = prefix + "_" + str(epoch + 1)
            np.savez_compressed(prefix + "_data.npz", **{
                "net/w": net.w.data.cpu().numpy(), "net/alpha": net.alpha.data.cpu().numpy(),
                "net/eta": net.eta.data.cpu().numpy(), "train/all_losses": np.asarray(all_losses),
                "validation/train_losses": np.asarray(val_train_losses),
                "validation/test_losses": np.asarray(val_test_losses),
                "validation/accuracies": np.asarray(val_accuracies)})
            with open(prefix + "_parameters.dat", "wb") as fo:      # train.py:199-200
                pickle.dump({k: (str(v) if isinstance(v, torch.device) else v) for k, v in params.items()}, fo)
            torch.save(net.state_dict(), prefix + "_net.pth")
        if terminate:
            if verbose:
                print("Training terminated due to the time limits!")
                print("Current epoch %d, train loss: %s" % (epoch, epoch_loss))
            break
    return all_losses, val_train_losses, val_test_losses, val_accuracies


def start_train(x_train, x_valid, y_train, y_valid, out_dir, model, img_width, img_height, img_chan,
                max_train_time=-1, load=False, gpu=True, epochs=5, lr=3e-5, val_ratio=0.05, val_every=50,
                save_every=100, gamma=0.666, steplr=1e6, rollout=50000, prule="hebb", debug=False,
                model_type="unetpres", depth=5, base_ch=8, neurons=16, batch_size=1, hebb_mode="slots",
                batch_norm=False, bilinear_upsample=False, prefetch=True):
    world, rank, local = dp.init_from_env()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    stop_time = time.time() + max_train_time if max_train_time > 0 else -1
    params = {"out_dir": out_dir, "device": device, "epochs": epochs, "stop_time": stop_time, "lr": lr,
              "val_ratio": val_ratio, "val_every": val_every, "save_every": save_every, "rollout": rollout,
              "gamma": gamma, "steplr": steplr, "prule": prule, "im_width": img_width, "im_height": img_height,
              "im_chan": img_chan, "debug": debug, "batch_size": batch_size, "prefetch": prefetch}
    if model_type == "unetp":
        net = UNetp(n_channels=img_chan, n_classes=1, nbf=img_width, batch_norm=batch_norm,
                    bilinear_upsample=bilinear_upsample, device=device, rule=prule, depth=depth, base_ch=base_ch,
                    hebb_mode=hebb_mode)
    else:
        net = UNetpRes(n_channels=img_chan, n_classes=1, nbf=img_width, batch_norm=batch_norm,
                       bilinear_upsample=bilinear_upsample, device=device, rule=prule, neurons=neurons,
                       hebb_mode=hebb_mode)
    if load:
        net.load_state_dict(torch.load(model, weights_only=True))
        net.to(device)
        print("Model loaded from %s" % model)
    dp.broadcast_params(net)
    try:
        train(net, x_train, x_valid, y_train, y_valid, params)
    except KeyboardInterrupt:
        torch.save(net.state_dict(), out_dir + "/INTERRUPTED.pth")
        print("Saved interrupt")
        sys.exit(0)
    return net


def parse_args(argv=None):
    parser = OptionParser()
    parser.add_option('-e', '--epochs', dest='epochs', default=5, type='int', help='number of epochs')
    parser.add_option('-l', '--learning-rate', dest='lr', default=3e-5, type='float', help='learning rate')
    parser.add_option('-s', '--step-lr', dest='steplr', default=1e6, type='float', help='the learning rate annealing step')
    parser.add_option('-g', '--gpu', action='store_true', dest='gpu', default=False, help='use cuda (always on)')
    parser.add_option('--prule', '-p', default='hebb', help="the plastic rule to use when training")
    parser.add_option('-c', '--load', dest='load', default=False, help='load file model')
    parser.add_option('--model', '-m', default='MODEL.pth', help="the file in which the model is stored")
    parser.add_option('--max-train-time', dest='max_train_time', default=-1, type='int')
    parser.add_option('--save_every', dest='save_every', default=100, type='int')
    parser.add_option('--validate_every', dest='validate_every', default=50, type='int')
    parser.add_option('--rollout_every', dest='rollout_every', default=50000, type='int')
    parser.add_option('-d', '--data', dest='data_dir', type='string', help='the directory with input data')
    parser.add_option('-i', '--dataset', dest='dataset_file', type='string', help='dataset .npz')
    parser.add_option('-o', '--out', dest='out_dir', type='string', help='results directory')
    parser.add_option('-v', '--debug', action='store_true', dest='debug', default=False)
    # extensions
    parser.add_option('--model-type', dest='model_type', default='unetpres')
    parser.add_option('--depth', dest='depth', type='int', default=5)
    parser.add_option('--base-ch', dest='base_ch', type='int', default=8)
    parser.add_option('--neurons', dest='neurons', type='int', default=16)
    parser.add_option('--img-size', dest='img_size', type='int', default=101)
    parser.add_option('--batch-size', dest='batch_size', type='int', default=1)
    parser.add_option('--synthetic', dest='synthetic', type='int', default=0, help='N synthetic samples')
    parser.add_option('--val-ratio', dest='val_ratio', type='float', default=0.2,
                      help='validation share of the TGS split (data_set.py: test_size)')
    parser.add_option('--hebb-mode', dest='hebb_mode', default='slots',
                      help="slots: one trace per batch slot; sequential: one trace threaded through the batch")
    parser.add_option('--batch-norm', dest='batch_norm', action='store_true', default=False)
    parser.add_option('--bilinear', dest='bilinear', action='store_true', default=False)
    parser.add_option('--seed', dest='seed', type='int', default=0)
    parser.add_option('--resident', dest='resident', action='store_true', default=False,
                      help='copy the whole training set to HBM once instead of streaming batches')
    (options, args) = parser.parse_args(argv)
    return options


def load_data(args):
    S = args.img_size
    if args.synthetic:
        g = np.random.RandomState(args.seed)
        n = args.synthetic
        x = g.rand(n, 1, S, S).astype(np.float32)
        y = (g.rand(n, 1, S, S) > 0.5).astype(np.float32)
        nv = max(1, n // 5)
        return x[nv:], x[:nv], y[nv:], y[:nv]
    if args.dataset_file:
        d = np.load(args.dataset_file)
        return d["x_train"], d["x_valid"], d["y_train"], d["y_valid"]
    if args.data_dir:           # the TGS layout (train.csv, depths.csv, train/{images,masks}/*.png)
        from utils import load_train_dataset
        return load_train_dataset(args.data_dir, S, S, 1, val_ratio=args.val_ratio, debug=args.debug)
    raise ValueError("The input data directory or dataset file not specified")


if __name__ == '__main__':
    args = parse_args()
    if not os.path.isdir(args.out_dir):
        os.makedirs(args.out_dir, exist_ok=True)
    torch.manual_seed(args.seed)
    x_train, x_valid, y_train, y_valid = load_data(args)
    start_train(x_train, x_valid, y_train, y_valid, out_dir=args.out_dir, model=args.model, load=args.load,
                gpu=True, epochs=args.epochs, lr=args.lr, steplr=args.steplr, max_train_time=args.max_train_time,
                save_every=args.save_every, val_every=args.validate_every, rollout=args.rollout_every,
                prule=args.prule, img_width=args.img_size, img_height=args.img_size, img_chan=1,
                debug=args.debug, model_type=args.model_type, depth=args.depth, base_ch=args.base_ch,
                neurons=args.neurons, batch_size=args.batch_size, hebb_mode=args.hebb_mode,
                batch_norm=args.batch_norm, bilinear_upsample=args.bilinear, prefetch=not args.resident)
