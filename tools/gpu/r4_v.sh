# Round 4 (v): what bounds the 256x256 NT kernel's main loop: probe variants of gemm_nt256p_kernel
# (timing only, outputs wrong) -- no LDS-DMA fill after K-tile 0, no fragment reads after K-tile 0,
# no MFMAs -- against HEAD at the step shape and at whole rounds (tools/kbench.py ntprobe)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARS:-base nofill noread nomfma}; do
  if [ $v = base ]; then E="XCP_NONE=1"; else E="XCP_LIB_PATH=$PWD/tools/exp/nt_$v/libxcp.so"; fi
  echo "== $v" >> gpurun_out/v_probe.log
  env $E timeout -k 10 120 python -u tools/kbench.py ntprobe >> gpurun_out/v_probe.log 2>&1 || exit $?
done
