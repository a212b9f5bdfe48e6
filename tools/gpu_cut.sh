set -u
# depth-cut GPU tests, then a same-box A/B of the cut legs: bash tools/gpu_cut.sh TAG NAME...
tag=${1:?tag}; shift
timeout -k 10 600 python -u -m pytest tests/test_raster_gpu.py tests/test_fullsize_parity.py tests/test_training_parity.py -k "depth_cut or config_d or config_e or deferred" -x -v --timeout 200 --timeout-method thread > gpurun_out/cutt.log 2>&1; rc=$?; tail -15 gpurun_out/cutt.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_cut.sh $tag "dl3dv recon12:0 recon12:1" "$@"
