# GPU: targeted tests, kbench A/B and bench A/B of the current library vs tools/exp/old in one run.
# usage: bash tools/gpu/r2_abk.sh "<kbench names>" "<pytest -k expr>"
set -o pipefail
bash tools/gpu/r2_kvar.sh "$1" "$2" old || exit $?
bash tools/gpu/r2_ab.sh ""
