cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python scripts/debug_td.py > gpurun_out/debug_td.txt 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/debug_td.txt
