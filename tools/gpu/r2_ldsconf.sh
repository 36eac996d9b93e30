# GPU: LDS bank-conflict census -- one PMC pass (SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE, SQ_INSTS_LDS)
# over a short headline bench and the XceptionLSTMA line.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv \
  -d gpurun_out/ldsc_lstmv -o p -- python3 -u bench.py --steps 2 --warmup 1 --cpu-baseline off --measured-peaks off \
  > gpurun_out/ldsc_lstmv.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv \
  -d gpurun_out/ldsc_lstma -o p -- python3 -u bench.py --model lstma --steps 2 --warmup 1 --cpu-baseline off \
  --measured-peaks off > gpurun_out/ldsc_lstma.log 2>&1
