"""(Record tool: needs the round-5 PRE2 build of gemm.hip, measured and reverted -- profiles/r05_nt_pre2_ab.txt.)
Interleaved A/B of the persistent NT GEMM with and without PRE2 (two K-tiles of the next tile issued
before the epilogue so the stores drain under two K-tiles instead of one), bf16, with / without the
BN-statistics epilogue, at the middle-flow shape and two K depths; checks PRE2 is bitwise equal.

usage (GPU box): python tools/nt_pre2_ab.py [rounds]
"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
from xcp import ops  # noqa: E402
from gemm_ab import timeit  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    ops._lib.load()
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K, ld) in [(256 * 361, 728, 728, 736), (256 * 256, 1024, 768, 768), (256 * 256, 1024, 3072, 3072)]:
        A = torch.randn(M, ld, device=dev, generator=g).bfloat16()
        B = (torch.randn(N, ld, device=dev, generator=g) / K ** 0.5).bfloat16()
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        st = torch.empty(ops.nt_stat_rows(M) * 2 * N, device=dev)
        fl = 2.0 * M * N * K
        outs = {}
        for pre in ("0", "1"):
            os.environ["XCP_NT_PRE2"] = pre
            for t in (0, 3):
                C.zero_(); st.zero_()
                ops.gemm_nt(A, B, C, M, N, K, stats=st, tile=t, lda=ld, ldb=ld)
                torch.cuda.synchronize()
                outs[(pre, t)] = (C.clone(), st.clone())
        for t in (0, 3):
            ok = torch.equal(outs[("0", t)][0], outs[("1", t)][0]) and torch.equal(outs[("0", t)][1], outs[("1", t)][1])
            print(f"M={M} N={N} K={K} tile{t}: PRE2 bitwise equal: {ok}", flush=True)
            assert ok
        del outs
        variants = {f"tile{t}{'+stats' if s else ''} pre2={p}": (t, s, p) for t in (0, 3) for s in (True, False)
                    for p in ("0", "1")}
        res = {k: [] for k in variants}
        for _ in range(rounds):
            for k, (t, s, p) in variants.items():
                os.environ["XCP_NT_PRE2"] = p
                res[k].append(timeit(lambda: ops.gemm_nt(A, B, C, M, N, K, stats=st if s else None, tile=t,
                                                         lda=ld, ldb=ld)))
        for k, v in res.items():
            med = statistics.median(v)
            print(f"M={M} N={N} K={K} {k:22s} median {med:7.1f} us  min {min(v):7.1f}  "
                  f"{fl / med / 1e6:7.1f} TF/s  frac {fl / med / 1e6 / 2500:.3f}", flush=True)
        del A, B, C, st


if __name__ == "__main__":
    main()
