"""CPU: the oracle's ArcFace / CB-focal restatements and the product heads' constructors
against the reference's own classes (tests/golden/heads.npz, arcface_step.npz)."""
import numpy as np
import torch
import torch.nn as nn

from oracle import xception_oracle as O


def test_oracle_arcface_and_cbfocal(golden):
    g = golden("heads.npz")
    for tag, m_ in (("v", 0.5), ("a", 0.30)):
        w = torch.tensor(g[f"{tag}/weight"]).requires_grad_(True)
        f = torch.tensor(g[f"{tag}/features"]).requires_grad_(True)
        lab = torch.tensor(g[f"{tag}/labels"]).long()
        np.testing.assert_allclose(O.arcface_logits(f, w, None, 30.0, m_).detach().numpy(), g[f"{tag}/logits_nolabel"],
                                   rtol=1e-6, atol=1e-6)
        logits = O.arcface_logits(f, w, lab, 30.0, m_)
        np.testing.assert_allclose(logits.detach().numpy(), g[f"{tag}/logits"], rtol=1e-6, atol=1e-6)
        if tag == "v":
            loss = nn.CrossEntropyLoss()(logits, lab)
        else:
            cw = O.cb_class_weights([300, 1700])
            np.testing.assert_allclose(cw.numpy(), g["a/class_weights"], rtol=1e-7)
            loss = O.cb_focal_loss(logits, lab, cw, 2.0)
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"{tag}/loss"], rtol=1e-6)
        np.testing.assert_allclose(f.grad.numpy(), g[f"{tag}/dfeatures"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(w.grad.numpy(), g[f"{tag}/dweight"], rtol=1e-5, atol=1e-7)


def test_product_heads_init_and_buffers(golden):
    """xcp.heads.ArcFaceHead draws the same init as the reference's (randn, then xavier_uniform_);
    CBFocalLoss builds the same class_weights buffer."""
    from xcp.heads import ArcFaceHead, CBFocalLoss
    torch.manual_seed(1)
    h = ArcFaceHead(128, 2, s=30.0, m=0.5)
    assert list(h.state_dict()) == ["weight"]
    np.testing.assert_array_equal(h.weight.detach().numpy(), golden("arcface_step.npz")["head_init"])
    cb = CBFocalLoss([300, 1700], beta=0.9999, gamma=2.0)
    np.testing.assert_array_equal(cb.class_weights.numpy(), golden("heads.npz")["a/class_weights"])


def test_unwrap_state_dict_vs_reference(golden):
    """xcp.checkpoint.unwrap_state_dict against the reference's _unwrap_state_dict
    (test_au_face.py:107-125) on the containers it handles (EMA / DataParallel)."""
    from xcp.checkpoint import unwrap_state_dict
    g = golden("heads.npz")
    raw = {"model": {"module.conv.weight": torch.ones(2), "module.fc.bias": torch.zeros(3)}, "best_auc": 0.9,
           "n_averaged": torch.tensor(4)}
    assert sorted(unwrap_state_dict(raw)) == [str(k) for k in g["unwrap/keys"]]
    raw2 = {"ema_state_dict": {"n_averaged": torch.tensor(3), "module.block.w": torch.ones(1)}}
    assert sorted(unwrap_state_dict(raw2)) == [str(k) for k in g["unwrap2/keys"]]
    # keys without the prefix are kept whole (the reference truncates them: documented deviation)
    assert sorted(unwrap_state_dict({"model": {"a.weight": torch.ones(1)}})) == ["a.weight"]


def test_checkpoint_round_trip(tmp_path):
    """state_dict round trip through the reference's container ({"model": ...}, DataParallel
    "module." prefix), strict load, and the resume state (optimizer / scaler / epoch)."""
    from Models.XceptionLSTMV import XceptionLSTMV
    from xcp.checkpoint import load_state_dict_flexible, load_training_state, save_training_state
    torch.manual_seed(0)
    a = XceptionLSTMV(128, pretrained=False)
    torch.manual_seed(1)
    b = XceptionLSTMV(128, pretrained=False)
    torch.save({"model": {"module." + k: v for k, v in a.state_dict().items()}}, tmp_path / "dp.pth")
    assert load_state_dict_flexible(b, str(tmp_path / "dp.pth"), verbose=False) == ([], [])
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)
    opt = torch.optim.Adam(a.parameters(), lr=1e-4)
    save_training_state(tmp_path / "ck.pth", a, optimizer=opt, epoch=7)
    c = XceptionLSTMV(128, pretrained=False)
    ck = load_training_state(tmp_path / "ck.pth", c, optimizer=torch.optim.Adam(c.parameters(), lr=1e-4))
    assert ck["epoch"] == 7 and torch.equal(c.lstm.weight_ih_l0, a.lstm.weight_ih_l0)
