"""Per-phase in-kernel cycle stamps of the persistent NT kernel (tile 3) at the middle-flow
shape: a patched copy of csrc/gemm.hip (tools/exp/) where waves 0 and 4 (the two staggered wave
groups) of workgroups 0-7 record the shader clock (s_memtime via clock64) in every phase of
K-tiles 2-5 of their first tile -- on entry to the phase's MFMA section (ds_reads, LDS-DMA
issue and the counted vmcnt wait done), after its first barrier, after the lgkmcnt wait, after
the MFMA issue, after the second barrier -- into a buffer of their own.

  python tools/gemm_phase.py build / run
"""
import ctypes
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc")
OUT = os.path.join(HERE, "exp")
SO = os.path.join(OUT, "libgemm_phase.so")
NPH, P0 = 16, 8   # phases recorded, first phase index
NS = 7            # stamps per phase
NWG = 8


def patched():
    s = open(os.path.join(SRC, "gemm.hip")).read()
    s = s.replace('#include "common.h"\n', '#include "' + os.path.join(SRC, "common.h") + '"\n'
                  "__device__ long long* g_ph;\n", 1)
    old = """  auto sync_mfma = [&](int ih, const bf16x8 (&b)[2][2], int jh) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma_q(ih, b, jh);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };

  int t = slot;"""
    new = """  int ph_ = 0;
  const bool rec_ = blockIdx.x < %d && (threadIdx.x == 0 || threadIdx.x == 256);
  long long* ph_buf = g_ph + ((long)blockIdx.x * 2 + (threadIdx.x >> 8)) * %d * NS_;
  auto stamp_ = [&](int k) {
    const long long c = clock64();
    if (rec_ && ph_ >= %d && ph_ < %d) ph_buf[(ph_ - %d) * NS_ + k] = c;
  };
  auto sync_mfma = [&](int ih, const bf16x8 (&b)[2][2], int jh) {
    stamp_(0);
    __builtin_amdgcn_s_barrier();
    stamp_(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp_(2);
    __builtin_amdgcn_s_setprio(1);
    mfma_q(ih, b, jh);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    stamp_(3);
    __builtin_amdgcn_s_barrier();
    stamp_(4);
    ++ph_;
  };

  int t = slot;""" % (NWG, NPH, P0, P0 + NPH, P0)
    assert old in s
    s = s.replace(old, new, 1)
    s = s.replace("__device__ long long* g_ph;\n", "__device__ long long* g_ph;\n#define NS_ %d\n" % NS, 1)
    k0 = s.index("auto ktile = [&](int kt, auto first) {")
    body = s[k0:]
    for h in range(3):
        a = "      if (nxt) issue(%d, kt + 1);\n" % h
        assert a in body, a
        body = body.replace(a, "      stamp_(5);\n" + a + "      stamp_(6);\n", 1)
    a = "      if (nxt) {\n        issue(3, kt + 1);\n"
    assert a in body
    body = body.replace(a, "      stamp_(5);\n" + a + "        stamp_(6);\n", 1)
    s = s[:k0] + body
    s += ('\nextern "C" int xcp_set_ph(long long* p) {\n'
          '  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ph), &p, sizeof(p));\n}\n')
    return s


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, "gemm_phase.hip")
    open(src, "w").write(patched())
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                        "-munsafe-fp-atomics", src, "-o", SO], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    print("built", SO)


def run():
    import torch
    sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
    from xcp import _lib
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(SO)
    lib.xcp_gemm_nt.argtypes = _lib.SIGNATURES["xcp_gemm_nt"]
    lib.xcp_gemm_nt.restype = ctypes.c_int
    lib.xcp_set_ph.argtypes = [ctypes.c_void_p]
    M, C = 256 * 361, 736
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(M, C, device=dev, generator=g).bfloat16()
    B = (torch.randn(C, C, device=dev, generator=g) / 27).bfloat16()
    Y = torch.empty_like(A)
    st = torch.empty(((M + 127) // 128) * 2 * C, device=dev)
    buf = torch.zeros(NWG * 2 * NPH * NS, device=dev, dtype=torch.int64)
    lib.xcp_set_ph(ctypes.c_void_p(buf.data_ptr()))
    s = torch.cuda.current_stream().cuda_stream
    z = (0, 0, 0, 0, 0, 1, 0)
    for _ in range(20):
        lib.xcp_gemm_nt(1, A.data_ptr(), C, B.data_ptr(), C, Y.data_ptr(), C, M, C, C, st.data_ptr(), *z, 3, s)
    torch.cuda.synchronize()
    buf.zero_()
    lib.xcp_gemm_nt(1, A.data_ptr(), C, B.data_ptr(), C, Y.data_ptr(), C, M, C, C, st.data_ptr(), *z, 3, s)
    torch.cuda.synchronize()
    v = buf.view(NWG, 2, NPH, NS).cpu().long()
    names = ["pre->bar1", "bar1->lgkm", "lgkm->mfma issued", "mfma->bar2", "bar2->next pre"]
    for grp in (0, 1):
        segs = {k: [] for k in names}
        for w in range(NWG):
            for p in range(NPH):
                st_ = v[w, grp, p]
                segs[names[0]].append(int(st_[1] - st_[0]))
                segs[names[1]].append(int(st_[2] - st_[1]))
                segs[names[2]].append(int(st_[3] - st_[2]))
                segs[names[3]].append(int(st_[4] - st_[3]))
                if p + 1 < NPH:
                    segs[names[4]].append(int(v[w, grp, p + 1][0] - st_[4]))
        tot = int(v[:, grp, -1, 4].double().mean() - v[:, grp, 0, 0].double().mean())
        print(f"wave group {grp}: {NPH} phases ({NPH // 4} K-tiles) in {tot} cycles = {tot / (NPH // 4):.0f} per K-tile")
        for k in names:
            x = segs[k]
            print(f"   {k:20s} median {statistics.median(x):7.0f}  mean {sum(x) / len(x):7.0f}  max {max(x):7d}")
        # per phase position within the K-tile (Q0..Q3)
        for q in range(4):
            rd = [int(v[w, grp, p][5] - v[w, grp, p - 1][4]) for w in range(NWG) for p in range(max(q, 1), NPH, 4)]
            iss = [int(v[w, grp, p][6] - v[w, grp, p][5]) for w in range(NWG) for p in range(q, NPH, 4)]
            wt = [int(v[w, grp, p][0] - v[w, grp, p][6]) for w in range(NWG) for p in range(q, NPH, 4)]
            print(f"   Q{q}: ds_reads {statistics.median(rd):5.0f}  DMA issue {statistics.median(iss):5.0f}  "
                  f"vmcnt wait {statistics.median(wt):5.0f}")
            pre = [int(v[w, grp, p + 1][0] - v[w, grp, p][4]) for w in range(NWG) for p in range(q, NPH - 1, 4)]
            b1 = [int(v[w, grp, p][1] - v[w, grp, p][0]) for w in range(NWG) for p in range(q, NPH, 4)]
            print(f"   Q{q}: pre(bar1 wait) median {statistics.median(b1):6.0f}   after-bar2 work (next phase's "
                  f"reads/issue/wait) median {statistics.median(pre) if pre else 0:6.0f}")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
