set -u
timeout -k 10 600 python -u -m pytest tests/test_raster_gpu.py tests/test_fullsize_parity.py tests/test_training_parity.py -k "depth_cut or config_d or config_e" -x -q --timeout 200 --timeout-method thread > gpurun_out/cutt.log 2>&1; rc=$?; tail -3 gpurun_out/cutt.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_cut.sh big2 "dl3dv recon12:0 recon12:1" main base
