"""In-step ablation (timing diagnostic only, results are garbage): the headline train step
(XceptionLSTMV, 16 clips x 16 x 299^2, unfrozen, bf16) with chosen C-ABI launches dropped, to
price what each kernel class costs the STEP (its marginal cost, contention included) rather
than what it costs alone.  Not part of the product path: the skip is a monkeypatch of
xcp._lib.call applied in this process only; GEMMs of fewer than 4096 rows (the LSTM input
projection) are never dropped, and the loss is fed sanitised probabilities (torch's BCE asserts
0 <= p <= 1 on the device, and a dropped launch leaves garbage behind it).

  python tools/step_ablation.py [--steps 8] [--rounds 2] set1 set2 ...

A set is a '+'-joined list of entries `name[:filter]` (name without the `xcp_` prefix):
  gemm_tn             every weight-gradient GEMM launch
  gemm_nt:fwd         pointwise GEMMs with the BN-statistics epilogue (forward)
  gemm_nt:dgrad       pointwise GEMMs without it (input gradients)
  gemm_nt:728         only the 736-pitch middle-flow shapes (combine: gemm_nt:728fwd, gemm_nt:728dgrad)
  dw_bwd, dw_fwd, bn_bwd_apply, colreduce_multi, bn_bwd_reduce, ...
Each round times the unablated step and every set once (interleaved), then prints ms/step.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]


def matcher(spec):
    name, _, flt = spec.partition(":")
    name = "xcp_" + name

    def m(n, args):
        if n != name:
            return False
        if n == "xcp_gemm_nt" and flt:
            stats = args[10]
            M, N, K = args[7], args[8], args[9]
            if M < 4096:   # the LSTM input projection and other head-size GEMMs are never dropped
                return False
            if "728" in flt and not (N == 736 and K == 736):
                return False
            if flt.endswith("fwd") and not stats:
                return False
            if flt.endswith("dgrad") and stats:
                return False
        return True
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("sets", nargs="*")
    a = ap.parse_args()
    import torch
    import bench
    import xcp
    from xcp import _lib
    xcp.set_compute_dtype("bf16")
    xcp.load_library()
    dev = torch.device("cuda:0")
    sys.argv = [sys.argv[0], "--cpu-baseline", "off"]
    args = bench.parse()
    args.mode = "unfrozen"
    run = bench.Run(args, "unfrozen", dev, 0, 1)
    # dropped launches leave garbage (possibly NaN / inf) in their outputs; torch's BCE asserts
    # 0 <= p <= 1 on the device (an assert is a GPU trap), so the loss sees sanitised probabilities
    bce = torch.nn.functional.binary_cross_entropy
    run.crit = lambda out, y: bce(torch.nan_to_num(out.float(), nan=0.5, posinf=1.0, neginf=0.0).clamp(0.0, 1.0), y)
    real = _lib.call
    active = []
    skipped = {"n": 0}

    def call(name, *cargs):
        if name not in _lib.SIZE_QUERIES and any(m(name, cargs) for m in active):
            skipped["n"] += 1
            return 0
        return real(name, *cargs)

    _lib.call = call
    sets = ["(none)"] + a.sets
    res = {s: [] for s in sets}
    for r in range(a.rounds):
        for s in sets:
            active[:] = [] if s == "(none)" else [matcher(x) for x in s.split("+")]
            skipped["n"] = 0
            for _ in range(a.warmup):
                run.step()
            torch.cuda.synchronize()
            n0 = skipped["n"]
            t0 = time.perf_counter()
            for _ in range(a.steps):
                run.step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            res[s].append(ms)
            print(f"round {r} {s:40s} {ms:8.2f} ms/step  ({(skipped['n'] - n0) // a.steps} launches skipped per step)",
                  flush=True)
    base = min(res["(none)"])
    print("\nbest of rounds (ms/step, saving vs the full step):")
    for s in sets:
        b = min(res[s])
        print(f"{s:40s} {b:8.2f}  {base - b:+7.2f}")


if __name__ == "__main__":
    main()
