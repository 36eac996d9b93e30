"""Detection metrics of the reference's training / evaluation scripts, restated in numpy.

The scripts compute ROC-AUC, partial AUC, average precision and the equal error rate with
scikit-learn on the host (train_visual.py:476-487, test_visual.py:515-565,
train_au_face.py:462-506).  These functions give the same numbers without the sklearn
dependency; the ROC / PR primitives follow scikit-learn's published algorithm (the
reference pins no version; goldens were taken with scikit-learn 1.7.2):

* ``roc_curve``: scores sorted descending (stable), one point per distinct score, the
  collinear points dropped (``drop_intermediate``), a leading (0, 0) point at threshold +inf;
* ``auc``: trapezoidal area (x monotone, either direction);
* ``average_precision_score``: sum over recall steps of precision, -sum(diff(recall) *
  precision[:-1]) on the curve ordered by decreasing threshold.

tests/test_metrics.py pins every function against the reference's own functions run on
seeded score sets (tests/golden/heads.npz).
"""
import numpy as np


def _binary_clf_curve(y_true, y_score):
    y_true = np.asarray(y_true).ravel() == 1
    y_score = np.asarray(y_score, dtype=np.float64).ravel()
    desc = np.argsort(y_score, kind="mergesort")[::-1]
    y_score, y_true = y_score[desc], y_true[desc]
    distinct = np.where(np.diff(y_score))[0]
    idx = np.r_[distinct, y_true.size - 1]
    tps = np.cumsum(y_true, dtype=np.float64)[idx]
    fps = 1 + idx - tps
    return fps, tps, y_score[idx]


def roc_curve(y_true, y_score, drop_intermediate=True):
    fps, tps, thr = _binary_clf_curve(y_true, y_score)
    if drop_intermediate and len(fps) > 2:
        keep = np.where(np.r_[True, np.logical_or(np.diff(fps, 2), np.diff(tps, 2)), True])[0]
        fps, tps, thr = fps[keep], tps[keep], thr[keep]
    tps, fps, thr = np.r_[0, tps], np.r_[0, fps], np.r_[np.inf, thr]
    with np.errstate(invalid="ignore", divide="ignore"):
        fpr = fps / fps[-1] if fps[-1] > 0 else np.full(fps.shape, np.nan)
        tpr = tps / tps[-1] if tps[-1] > 0 else np.full(tps.shape, np.nan)
    return fpr, tpr, thr


def auc(x, y):
    x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
    if x.shape[0] < 2:
        raise ValueError("auc needs at least 2 points")
    direction = 1
    dx = np.diff(x)
    if np.any(dx < 0):
        if np.all(dx <= 0):
            direction = -1
        else:
            raise ValueError("x is neither increasing nor decreasing")
    return float(direction * np.trapezoid(y, x))


def roc_auc_score(y_true, y_score):
    if len(np.unique(y_true)) != 2:
        raise ValueError("only one class present in y_true: ROC AUC is not defined")
    fpr, tpr, _ = roc_curve(y_true, y_score)
    return auc(fpr, tpr)


def average_precision_score(y_true, y_score):
    fps, tps, _ = _binary_clf_curve(y_true, y_score)
    ps = tps + fps
    precision = np.divide(tps, ps, out=np.zeros_like(tps), where=ps != 0)
    recall = tps / tps[-1] if tps[-1] > 0 else np.ones_like(tps)
    precision, recall = np.r_[precision[::-1], 1], np.r_[recall[::-1], 0]
    return float(-np.sum(np.diff(recall) * precision[:-1]))


# ---------------------------------------------------------------- the scripts' functions
def train_visual_metrics(labels, probs):
    """compute_metrics, train_visual.py:476-487 -> (AUC, pAUC@FPR<=0.1, AP, EER, EER threshold)."""
    labels, probs = np.asarray(labels), np.asarray(probs)
    if len(np.unique(labels)) <= 1:
        return 0.0, 0.0, 0.0, 1.0, 0.5
    auc_score = roc_auc_score(labels, probs)
    ap_score = average_precision_score(labels, probs)
    fpr, tpr, thresholds = roc_curve(labels, probs)
    pauc_score = auc(fpr[fpr <= 0.1], tpr[fpr <= 0.1]) / 0.1 if np.sum(fpr <= 0.1) >= 2 else 0.0
    fnr = 1 - tpr
    eer_idx = np.nanargmin(np.abs(fpr - fnr))
    eer = (fpr[eer_idx] + fnr[eer_idx]) / 2
    return auc_score, pauc_score, ap_score, eer, thresholds[eer_idx]


def test_visual_metrics(labels, probs, alpha=0.1):
    """compute_metrics, test_visual.py:515-565: AUC, AP, pAUC on [0, alpha] interpolated and
    normalised (0 = random), EER by linear interpolation at the FPR = FNR crossing, and the
    accuracy / threshold at Youden's J."""
    labels = np.asarray(labels).astype(int)
    probs = np.asarray(probs, dtype=float)
    if len(np.unique(labels)) < 2:
        return {"AUC": 0.0, "pAUC": 0.0, "AP": 0.0, "EER": 1.0}
    auc_score = roc_auc_score(labels, probs)
    ap_score = average_precision_score(labels, probs)
    fpr, tpr, thresholds = roc_curve(labels, probs)
    grid = np.linspace(0.0, alpha, 2001)
    pauc_raw = auc(grid, np.interp(grid, fpr, tpr))
    pauc_norm = (pauc_raw - (alpha ** 2) / 2) / (alpha - (alpha ** 2) / 2)
    fnr = 1 - tpr
    diff = fpr - fnr
    idx = np.where(np.diff(np.sign(diff)) != 0)[0]
    if len(idx) == 0:
        j = np.argmin(np.abs(diff))
        eer = (fpr[j] + fnr[j]) / 2.0
    else:
        j = idx[0]
        x1, y1, x2, y2 = fpr[j], fnr[j], fpr[j + 1], fnr[j + 1]
        w = np.clip((y1 - x1) / ((x2 - x1) - (y2 - y1) + 1e-12), 0.0, 1.0)
        eer = x1 + w * (x2 - x1)
    j_ix = np.argmax(tpr - fpr)
    thr_j = thresholds[j_ix]
    acc_j = ((probs >= thr_j).astype(int) == labels).mean()
    return {"AUC": float(auc_score), "AP": float(ap_score), "pAUC": float(pauc_norm), "EER": float(eer),
            "ACC@J": float(acc_j), "THR@J": float(thr_j)}


def compute_eer_auc(labels, scores):
    """train_au_face.py:462-472 -> (AUC, pAUC@FPR<=0.1, EER, (fpr, tpr)); full ROC (no points dropped)."""
    y = np.asarray(labels).astype(int).ravel()
    s = np.asarray(scores).astype(float).ravel()
    fpr, tpr, _ = roc_curve(y, s, drop_intermediate=False)
    fnr = 1 - tpr
    auc_score = auc(fpr, tpr) if len(fpr) else float("nan")
    mask = fpr <= 0.1
    pauc = auc(fpr[mask], tpr[mask]) / 0.1 if np.sum(mask) >= 2 else float("nan")
    idx = int(np.nanargmin(np.abs(fpr - fnr))) if len(fpr) else 0
    eer = float((fpr[idx] + fnr[idx]) / 2.0) if len(fpr) else float("nan")
    return auc_score, pauc, eer, (fpr, tpr)


def pick_threshold(labels, scores, mode="youden", fpr_target=0.01):
    """train_au_face.py:475-489 -> (threshold, fpr, tpr) at Youden's J or at FPR <= fpr_target."""
    y = np.asarray(labels).astype(int).ravel()
    s = np.asarray(scores).astype(float).ravel()
    fpr, tpr, thr = roc_curve(y, s, drop_intermediate=False)
    if len(fpr) == 0:
        return 0.5, 0.0, 0.0
    if mode == "youden":
        j = int(np.argmax(tpr - fpr))
        return float(thr[j]), float(fpr[j]), float(tpr[j])
    ok = np.where(fpr <= float(fpr_target))[0]
    if len(ok) == 0:
        return float(thr[0]), float(fpr[0]), float(tpr[0])
    i = int(ok[-1])
    return float(thr[i]), float(fpr[i]), float(tpr[i])


def compute_acc_ap_and_counts(labels, scores, thr):
    """train_au_face.py:492-506 -> (acc, AP, correct real, total real, correct fake, total fake)."""
    y = np.asarray(labels).astype(int).ravel()
    s = np.asarray(scores).astype(float).ravel()
    preds = (s >= float(thr)).astype(int)
    acc = float((preds == y).mean())
    ap = float(average_precision_score(y, s)) if y.min() != y.max() else float("nan")
    return (acc, ap, int(((preds == 0) & (y == 0)).sum()), int((y == 0).sum()), int(((preds == 1) & (y == 1)).sum()),
            int((y == 1).sum()))
