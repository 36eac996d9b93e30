"""CPU: xcp.metrics against the reference's own metric functions (train_visual.py:476-487,
test_visual.py:515-565, train_au_face.py:462-506), run on seeded score sets when the goldens
were captured (tools/capture_goldens.py g_heads -> tests/golden/heads.npz); and the
checkpoint unwrapping of test_au_face.py:107-125."""
import numpy as np
import pytest

from xcp import metrics as M


def cases(g):
    i = 0
    while f"m{i}/labels" in g:
        yield i, g[f"m{i}/labels"], g[f"m{i}/scores"]
        i += 1


def test_train_visual_metrics(golden):
    g = golden("heads.npz")
    for i, y, s in cases(g):
        np.testing.assert_allclose(np.array(M.train_visual_metrics(y, s), dtype=np.float64), g[f"m{i}/train_visual"],
                                   rtol=1e-12, atol=1e-12, err_msg=str(i))


def test_test_visual_metrics(golden):
    g = golden("heads.npz")
    for i, y, s in cases(g):
        r = M.test_visual_metrics(y, s)
        keys = [str(k) for k in g[f"m{i}/test_visual_keys"]]
        assert sorted(r) == keys, i
        np.testing.assert_allclose([r[k] for k in keys], g[f"m{i}/test_visual"], rtol=1e-12, atol=1e-12, err_msg=str(i))


def test_au_face_metrics(golden):
    g = golden("heads.npz")
    n = 0
    for i, y, s in cases(g):
        if f"m{i}/eer_auc" not in g:
            continue
        n += 1
        a, p, e, _ = M.compute_eer_auc(y, s)
        np.testing.assert_allclose([a, p, e], g[f"m{i}/eer_auc"], rtol=1e-12, atol=1e-12, equal_nan=True)
        for mode in ("youden", "fpr"):
            thr = M.pick_threshold(y, s, mode=mode, fpr_target=0.05)
            np.testing.assert_allclose(thr, g[f"m{i}/thr_{mode}"], rtol=1e-12)
            np.testing.assert_allclose(M.compute_acc_ap_and_counts(y, s, thr[0]), g[f"m{i}/acc_{mode}"], rtol=1e-12)
    assert n >= 4


def test_primitives_edge_cases():
    assert M.auc([0, 0.5, 1], [0, 0.5, 1]) == pytest.approx(0.5)
    assert M.auc([1, 0.5, 0], [1, 0.5, 0]) == pytest.approx(0.5)   # decreasing x
    with pytest.raises(ValueError):
        M.roc_auc_score([1, 1, 1], [0.1, 0.2, 0.3])
    assert M.roc_auc_score([0, 1], [0.2, 0.9]) == 1.0
    assert M.average_precision_score([0, 1, 1], [0.9, 0.8, 0.7]) == pytest.approx((1 / 2 + 2 / 3) / 2)
