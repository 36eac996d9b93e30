set -o pipefail
mkdir -p gpurun_out
for m in 92416 23104 5776; do
  echo "== M=$m" >> gpurun_out/r3_stampsM.log
  STAMP_M=$m timeout -k 10 120 python -u tools/gemm_stamps.py run >> gpurun_out/r3_stampsM.log 2>&1 || exit $?
done
