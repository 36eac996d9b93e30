"""The product modules reproduce the reference init bit-for-bit (Xception.py:154-160,
nn.LSTM / nn.Linear defaults) and the reference state_dict layout (288 keys for
XceptionLSTMV).  CPU only: construction, no compute."""
import numpy as np
import torch

from Models.Xception import xception
from Models.XceptionLSTMA import XceptionLSTMA
from Models.XceptionLSTMV import XceptionLSTMV


def _check(prefix, module, g):
    sd = module.state_dict()
    keys = [k[len(prefix) + 1:-len("/shape")] for k in g if k.startswith(prefix + "/") and k.endswith("/shape")]
    assert sorted(keys) == sorted(sd.keys())
    for k, t in sd.items():
        assert tuple(g[f"{prefix}/{k}/shape"]) == tuple(t.shape), k
        if t.dtype == torch.float32:
            a = t.double().reshape(-1)
            assert np.array_equal(a[:16].numpy(), g[f"{prefix}/{k}/head"]), k
            assert a.sum().item() == g[f"{prefix}/{k}/sum"], k
            assert (a * a).sum().item() == g[f"{prefix}/{k}/sumsq"], k
        else:
            assert np.array_equal(t.reshape(-1).numpy().astype(np.int64), g[f"{prefix}/{k}/int"]), k


def test_xceptionlstmv_init_matches_reference(golden):
    g = golden("init.npz")
    torch.manual_seed(0)
    m = XceptionLSTMV(128, pretrained=False)
    assert list(m.state_dict().keys()) == list(g["V128/keys"])
    assert len(m.state_dict()) == 288
    _check("V128", m, g)
    assert not any(p.requires_grad for p in m.feature_extractor.parameters())


def test_xceptionlstma_init_matches_reference(golden):
    torch.manual_seed(0)
    _check("A512", XceptionLSTMA(512, pretrained=False), golden("init.npz"))


def test_xception_num_classes1_init(golden):
    torch.manual_seed(0)
    _check("X1", xception(num_classes=1), golden("init.npz"))


def test_pretrained_never_fetches(monkeypatch, tmp_path):
    monkeypatch.setenv("XCP_XCEPTION_WEIGHTS", str(tmp_path / "missing.pth"))
    monkeypatch.setattr(torch.hub, "get_dir", lambda: str(tmp_path))
    import pytest
    with pytest.raises(RuntimeError, match="never downloads"):
        xception(pretrained=True)


def test_pretrained_local_roundtrip(tmp_path):
    torch.manual_seed(1)
    src = xception()
    p = tmp_path / "w.pth"
    torch.save(src.state_dict(), p)
    dst = xception(pretrained=str(p))
    for (k, a), (_, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert torch.equal(a, b), k
