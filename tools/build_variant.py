"""Link an A/B variant of libxcp.so: the current objects (xcp/build/*.o, from
``python -m xcp.build``) with one csrc file replaced by another source.

usage: python tools/build_variant.py <out_dir> <csrc file name> <replacement .hip>
       (e.g. tools/exp/old gemm.hip /tmp/gemm_old.hip) -> <out_dir>/libxcp.so
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multimodal-deepfake-detection_amd"))

from xcp import build as xb  # noqa: E402


def main():
    out_dir, name, repl = sys.argv[1:4]
    xb.build()
    objdir = os.path.join(xb.HERE, "build")
    os.makedirs(out_dir, exist_ok=True)
    vobj = os.path.join(out_dir, name.replace(".hip", ".o"))
    subprocess.run([xb._hipcc(), *xb.FLAGS, "-I", xb.CSRC, "-c", repl, "-o", vobj], check=True)
    objs = [vobj if os.path.basename(s) == name else os.path.join(objdir, os.path.basename(s).replace(".hip", ".o"))
            for s in xb.sources()]
    out = os.path.join(out_dir, "libxcp.so")
    subprocess.run([xb._hipcc(), "-shared", f"--offload-arch={xb.ARCH}", "-fPIC", *objs, "-o", out], check=True)
    print(out)


if __name__ == "__main__":
    main()
