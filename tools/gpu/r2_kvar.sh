# GPU: targeted kernel tests, then kbench on the current library and on each variant library
# (tools/exp/<v>/libxcp.so), then the current one again, all in one run.
# usage: bash tools/gpu/r2_kvar.sh "<kbench names>" "<pytest -k expr or empty>" <variant>...
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
names="$1"; kexpr="$2"; shift 2
if [ -n "$kexpr" ]; then
  timeout -k 10 170 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "$kexpr" > gpurun_out/kv_tests.log 2>&1 || exit $?
fi
LIB=multimodal-deepfake-detection_amd/xcp/libxcp.so
cp $LIB /tmp/libxcp_cur.so
timeout -k 10 170 python -u tools/kbench.py $names > gpurun_out/kv_cur1.log 2>&1 || exit $?
for v in "$@"; do
  cp tools/exp/$v/libxcp.so $LIB
  timeout -k 10 170 python -u tools/kbench.py $names > gpurun_out/kv_$v.log 2>&1 || { cp /tmp/libxcp_cur.so $LIB; exit 1; }
done
cp /tmp/libxcp_cur.so $LIB
timeout -k 10 170 python -u tools/kbench.py $names > gpurun_out/kv_cur2.log 2>&1
