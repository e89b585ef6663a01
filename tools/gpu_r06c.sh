cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06c
timeout -k 10 60 python -u tools/capture_status_probe.py > gpurun_out/r06c/cap.log 2>&1; echo "cap rc=$?"; cat gpurun_out/r06c/cap.log
timeout -k 10 120 python -u tools/ddp_e4_probe.py 4 512 1 0 > gpurun_out/r06c/own_serial.log 2>&1; echo "own_serial rc=$?"
grep "^\[" gpurun_out/r06c/own_serial.log | tail -4
