set -u
mkdir -p gpurun_out/final
timeout -k 10 420 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread > gpurun_out/final/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/final/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > gpurun_out/final/bench.log 2>&1; rc=$?; tail -c 600 gpurun_out/final/bench.log; exit $rc
