set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/diag_phases.py ${1:-1024} ${2:-0,2,3,4,1} > gpurun_out/diag.log 2>&1; rc=$?; cat gpurun_out/diag.log; exit $rc
