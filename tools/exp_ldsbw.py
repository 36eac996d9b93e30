"""Runs tools/exp_ldsbw.hip (see there): `build` here, `run` on the GPU box."""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "exp", "libldsbw.so")

if sys.argv[1] == "build":
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    os.path.join(HERE, "exp_ldsbw.hip"), "-o", SO], check=True)
    print("built", SO)
else:
    import torch
    lib = ctypes.CDLL(SO)
    lib.exp_fill.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_long,
                             ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    buf = torch.randint(0, 255, (2 << 30,), dtype=torch.uint8, device=dev)
    out = torch.zeros(4, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    grid, wgb = 256, 8 << 20
    lib.exp_gather.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_long,
                               ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    # GEMM-like gathers: rows of ld bytes, 11 128-B K-chunks each (1408 B of every row)
    for ld in (1536, 1456):
        for wname, wrap_rows in (("hbm", (2 << 30) // 1536 - 8), ("l2", 1024)):
            rows = 4096
            f = lambda: lib.exp_gather(buf.data_ptr(), ld, rows, 11, wrap_rows, out.data_ptr(), grid, st)
            for _ in range(2):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                f()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 5
            byts = grid * rows * 11 * 128
            print(f"gather ld={ld} {wname:4s} {byts / ms / 1e6:8.1f} GB/s  {byts / ms / 1e6 / grid:6.1f} GB/s/CU", flush=True)
    for wrap_name, wrap in (("hbm", 2 << 30), ("l2", 2 << 20)):
        for dma in (1,):
            for depth in (2, 8):
                f = lambda: lib.exp_fill(depth, dma, buf.data_ptr(), wgb, wrap, out.data_ptr(), grid, st)
                for _ in range(2):
                    f()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    f()
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / 5
                gbs = grid * wgb / ms / 1e6
                print(f"{wrap_name:4s} {('reg', 'dma', 'mix')[dma]} depth={depth:2d} in-flight/CU={depth * 8:4d} KB  "
                      f"{gbs:8.1f} GB/s  {gbs / grid:6.1f} GB/s/CU", flush=True)
