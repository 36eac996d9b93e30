# Round 6 (f): what the persistent NT kernel's per-round fixed cost is: the middle-flow op and 4 whole rounds at
# K = 768 / 3072 (tools/kbench.py ntprobe) with the epilogue's stores as built (base), issued to an out-of-range
# offset (no HBM writes: probe/oobstore) and removed (probe/nostore); timing only, the probes' outputs are wrong
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  timeout -k 10 200 python -u tools/kbench.py ntprobe > gpurun_out/f_base_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/oobstore/libxcp.so timeout -k 10 200 python -u tools/kbench.py ntprobe > gpurun_out/f_oob_$r.log 2>&1 || exit $?
  XCP_LIB_PATH=probe/nostore/libxcp.so timeout -k 10 200 python -u tools/kbench.py ntprobe > gpurun_out/f_nost_$r.log 2>&1 || exit $?
done
