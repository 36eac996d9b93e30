"""(Record tool: needs the round-5 commit 57007cf, whose folded finalizes were measured and reverted --
profiles/r05_fold_ab.txt, r05_fold_step_ab.txt.)
Folded BN finalizes (XCP_BN_FOLD) against the partial-row path on one model step: the same
xception(num_classes=1) fp32 / bf16 forward + backward run with engine.BN_FOLD on and off in one
process; prints, per tensor class, how many elements differ and the largest relative difference.
  python tools/fold_ab.py [B] [S]      (GPU box)"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-deepfake-detection_amd"))


def run(fold, prec, B, S):
    import xcp
    from xcp import engine
    from Models.Xception import xception
    engine.BN_FOLD = fold
    torch.manual_seed(0)
    m = xception(num_classes=1).cuda().train()
    g = torch.Generator().manual_seed(7)
    x = torch.rand((B, 3, S, S), generator=g).cuda()
    y = (torch.arange(B, device="cuda") % 3 == 0).float().view(B, 1)
    with xcp.precision(prec):
        out = m(x)
        nn.BCEWithLogitsLoss()(out, y).backward()
    torch.cuda.synchronize()
    r = {"out": out.detach().clone()}
    for n, p in m.named_parameters():
        r["grad/" + n] = p.grad.detach().clone()
    for n, b in m.named_buffers():
        if b.is_floating_point():
            r["buf/" + n] = b.detach().clone()
    return r


def compare(a, b, tag):
    rows = []
    for k in a:
        nd = int((a[k] != b[k]).sum())
        d = (a[k].double() - b[k].double()).abs()
        rows.append((float(d.max() / b[k].double().abs().max().clamp_min(1e-30)), nd, k))
    first = [r for r in rows if r[2].startswith("buf/") and r[1]]
    print(f"  {tag}: {sum(r[1] for r in rows)} differing elements; buffers in module order, first differing:",
          [(k, n, f"{x:.2e}") for x, n, k in first[:6]])
    rows.sort(reverse=True)
    for rel, nd, k in rows[:6]:
        print(f"     {rel:.3e}  ({nd} elements)  {k}")


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 299
    for prec in ("fp32",):
        a, b, b2 = run(True, prec, B, S), run(False, prec, B, S), run(False, prec, B, S)
        print(f"[{prec}] B={B} S={S} XCP_FIN_MAX_ROWS={os.environ.get('XCP_FIN_MAX_ROWS', '2048')}")
        compare(b, b2, "partial rows vs partial rows (determinism)")
        compare(a, b, "fold vs partial rows")
    return
    for prec in ("fp32", "bf16"):
        a, b = run(True, prec, B, S), run(False, prec, B, S)
        worst, ndiff, ntot = [], 0, 0
        for k in a:
            d = (a[k].double() - b[k].double()).abs()
            nd = int((a[k] != b[k]).sum())
            ndiff += nd
            ntot += a[k].numel()
            rel = float(d.max() / b[k].double().abs().max().clamp_min(1e-30))
            worst.append((rel, nd, k))
        worst.sort(reverse=True)
        print(f"[{prec}] B={B} S={S}: {ndiff} of {ntot} elements differ; largest relative differences:")
        for rel, nd, k in worst[:12]:
            print(f"   {rel:.3e}  ({nd} elements)  {k}")


if __name__ == "__main__":
    main()
