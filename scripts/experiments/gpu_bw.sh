cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 ./scripts/bwprobe 32 > gpurun_out/bwprobe.txt 2>&1; echo rc=$?; cat gpurun_out/bwprobe.txt
