"""IoU-threshold metrics of the reference (src/utils/iou_metric.py:6-24, :26-87).

``fast_iou_metric(y_true, y_pred)`` thresholds the prediction at 0.5 and, per leading-axis item,
scores the fraction of IoU thresholds 0.5:0.05:0.95 the item's IoU exceeds.  eval.py:100 passes
flattened vectors, so each *pixel* is an item there; that behaviour is kept (it is what the
reference's validation "accuracy" measures).
"""
import numpy as np

_THRESHOLDS = np.arange(0.5, 1, 0.05)


def get_iou_vector(A, B):
    A = np.asarray(A)
    B = np.asarray(B)
    t = A.reshape(A.shape[0], -1) > 0
    p = B.reshape(B.shape[0], -1) > 0
    inter = np.logical_and(t, p).sum(axis=1)
    union = np.logical_or(t, p).sum(axis=1)
    iou = (inter + 1e-10) / (union + 1e-10)
    return float(np.mean((iou[:, None] > _THRESHOLDS[None, :]).mean(axis=1)))


def fast_iou_metric(y_true_in, y_pred_in):
    return get_iou_vector(y_true_in, np.asarray(y_pred_in) > 0.5)


def _foreground(v):
    """what np.histogram(bins=[0, 0.5, 1]) counts in its upper bin: 0.5 <= v <= 1"""
    v = np.asarray(v, dtype=np.float64)
    return (v >= 0.5) & (v <= 1.0)


def iou_metric_batch(y_true_in, y_pred_in):
    """Mean over the leading axis of the reference's single-object competition score
    (iou_metric, iou_metric.py:26-79): with one true and one predicted object, the precision at an
    IoU threshold is 1 when IoU > threshold else 0 (an empty intersection or union counts as
    1e-9, so two empty masks score 1).  Returned as float32 like iou_metric.py:81-87."""
    yt = np.asarray(y_true_in)
    yp = np.asarray(y_pred_in)
    n = yt.shape[0]
    t = _foreground(yt.reshape(n, -1))
    p = _foreground(yp.reshape(n, -1))
    inter = np.logical_and(t, p).sum(axis=1).astype(np.float64)
    union = (t.sum(axis=1) + p.sum(axis=1)).astype(np.float64) - inter
    inter[inter == 0] = 1e-9
    union[union == 0] = 1e-9
    iou = inter / union
    prec = (iou[:, None] > _THRESHOLDS[None, :]).astype(np.float64).mean(axis=1)
    return np.array(np.mean(prec), dtype=np.float32)
