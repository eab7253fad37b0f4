DIAG="paper1 kjv.txt world192.txt" bash tools/gpu_r3_check.sh && bash tools/profile.sh ${PTAG:-r03b} > gpurun_out/profile.log 2>&1; tail -3 gpurun_out/profile.log
