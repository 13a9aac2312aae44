"""IoU-threshold metric of the reference (src/utils/iou_metric.py:6-24).

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
