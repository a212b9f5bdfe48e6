set -u
mkdir -p gpurun_out/bench_r03g
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_r03g/bench.log 2>&1; rc=$?
tail -c 3000 gpurun_out/bench_r03g/bench.log; exit $rc
