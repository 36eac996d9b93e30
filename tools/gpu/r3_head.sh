# Round 3 HEAD record: full GPU suite, smoke, default bench, BN finalize kbench, then the HEAD profiles
# (rocprofv3 kernel trace + stats; FETCH_SIZE / WRITE_SIZE / GRBM_GUI_ACTIVE / SQ passes, one counter
# set per run) of the unfrozen headline step.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -p no:cacheprovider > gpurun_out/h_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/h_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 170 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/h_b.json 2> gpurun_out/h_b.err || exit $?
timeout -k 10 120 python -u tools/kbench.py fin > gpurun_out/h_fin.log 2>&1 || exit $?
bash tools/gpu/r3_profile.sh > gpurun_out/h_prof.log 2>&1
