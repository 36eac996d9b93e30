"""A/B of the depthwise backward against the committed version (git HEAD's csrc/dwconv.hip, built
into probe/libdw_base.so, a path the GPU upload carries -- delete it afterwards): both libraries'
xcp_dw_bwd on identical inputs at the step's shapes (with and without a strided-skip gradient),
interleaved rounds, median launch time; the new library also with XCP_DW_BWD_SKIP4=0; outputs compared
against the base (max |diff| of dX, dW partials, BN sums).

  python tools/dw_ab.py build [rev]   # here (rev: git revision of the baseline, default HEAD)
  python tools/dw_ab.py run           # GPU box
"""
import ctypes
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc")
OUT = os.path.join(REPO, "probe")
BASE = os.path.join(OUT, "libdw_base.so")


def build(rev="HEAD"):
    os.makedirs(OUT, exist_ok=True)
    srcs = []
    for f in ("dwconv.hip", "dwframe.hip"):
        txt = subprocess.run(["git", "-C", REPO, "show", f"{rev}:multimodal-deepfake-detection_amd/xcp/csrc/{f}"],
                             capture_output=True, text=True, check=True).stdout
        txt = txt.replace('#include "common.h"', f'#include "{os.path.join(CSRC, "common.h")}"')
        p = os.path.join(OUT, "base_" + f)
        open(p, "w").write(txt)
        srcs.append(p)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950", *srcs,
                        "-o", BASE], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    print("built", BASE, "from", rev)


def run():
    import torch
    sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
    from xcp import _lib, ops
    ops._lib.load()
    new = _lib._lib if hasattr(_lib, "_lib") else None
    libs = {"base": ctypes.CDLL(BASE), "new": ctypes.CDLL(os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp",
                                                                          "libxcp.so"))}
    sig = _lib.SIGNATURES["xcp_dw_bwd"]
    for l in libs.values():
        l.xcp_dw_bwd.argtypes = sig
        l.xcp_dw_bwd.restype = ctypes.c_int
        l.xcp_dw_bwd_chunks.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    variants = {"base": (libs["base"], None), "new": (libs["new"], None), "skip4off": (libs["new"], "S0")}
    # (N, H, W, C, act, residual, strided-skip gradient): the skip shapes are the first units of blocks 2, 3, 12
    shapes = [(256, 19, 19, 736, 2, False, False), (256, 19, 19, 736, 1, True, False), (256, 37, 37, 736, 2, False, False),
              (256, 74, 74, 256, 2, False, False), (256, 147, 147, 128, 2, False, False), (256, 10, 10, 1536, 2, False, False),
              (256, 74, 74, 128, 1, False, True), (256, 37, 37, 256, 1, False, True), (256, 19, 19, 736, 1, False, True)]
    for N, H, W, C, act, res, skip in shapes:
        M = N * H * W
        dY = torch.randn(M * C, device=dev, generator=g).bfloat16()
        X = torch.randn(M * C, device=dev, generator=g).bfloat16()
        dR = torch.randn(M * C, device=dev, generator=g).bfloat16() if res else None
        sO = (H - 1) // 2 + 1
        dS = torch.randn(N * sO * sO * C, device=dev, generator=g).bfloat16() if skip else None
        Wt = torch.randn(9 * C, device=dev, generator=g)
        sc = torch.rand(C, device=dev, generator=g) + 0.5
        sh = torch.randn(C, device=dev, generator=g)
        mu, isd = torch.randn(C, device=dev, generator=g), torch.rand(C, device=dev, generator=g) + 0.5
        P = libs["new"].xcp_dw_bwd_chunks(N, H, W, C)
        outs = {}
        for k in variants:
            outs[k] = (torch.empty(M * C, device=dev, dtype=torch.bfloat16), torch.empty(P * C * 9, device=dev),
                       torch.empty(P * 2 * C, device=dev) if act == 2 else None)
        p = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)   # noqa: E731

        def call(k):
            dX, dWp, bnp = outs[k]
            lib, env = variants[k]
            os.environ.pop("XCP_DW_BWD_ASM", None)
            os.environ.pop("XCP_DW_BWD_SKIP4", None)
            if env == "S0":
                os.environ["XCP_DW_BWD_SKIP4"] = "0"
            elif env is not None:
                os.environ["XCP_DW_BWD_ASM"] = env
            rc = lib.xcp_dw_bwd(1, act, p(dY), p(X), p(Wt), p(sc), p(sh), p(dR), p(dS), sO if skip else 0,
                                sO if skip else 0, 2 if skip else 1, 0, p(dX), p(dWp),
                                    p(bnp), p(mu) if act == 2 else None, p(isd) if act == 2 else None, N, H, W, C, st)
            assert rc == 0, rc

        times = {k: [] for k in variants}
        for _ in range(5):
            for k in variants:
                for _w in range(2):
                    call(k)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _i in range(10):
                    call(k)
                e.record()
                torch.cuda.synchronize()
                times[k].append(s.elapsed_time(e) / 10 * 1e3)
        byts = 2 * M * C * (3 + (1 if res else 0)) + (2 * N * sO * sO * C if skip else 0)
        d = [(outs["base"][i].float() - outs[k][i].float()).abs().max().item() for k in variants if k != "base"
             for i in range(3) if outs["base"][i] is not None]
        line = "  ".join(f"{k} {statistics.median(v):7.1f} us ({byts / statistics.median(v) / 1e3:6.0f} GB/s)" for k, v in times.items())
        print(f"{N}x{H}x{W}x{C} act={act} res={int(res)} skip={int(skip)}: {line}   max|diff| {['%.2e' % x for x in d]}",
              flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2] if len(sys.argv) > 2 else "HEAD")
    else:
        run()
