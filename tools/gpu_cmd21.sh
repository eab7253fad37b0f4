cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
export HH_FLAGS=4
SRC=E.coli ROUNDS=2 bash tools/gpu_ab.sh "-" "- HH_FSM_K=7" > gpurun_out/ab21.txt 2>&1; cat gpurun_out/ab21.txt
unset HH_FLAGS
ROUNDS=1 bash tools/gpu_ab.sh "-" > gpurun_out/ab21k.txt 2>&1; cat gpurun_out/ab21k.txt
