#!/bin/bash
# PMC passes (HBM fetch / write bytes, wave stats) on the 6-view 448x768 leg, eager launches.
set -e
export TMPDIR=/tmp
out=gpurun_out/prof_d_pmc
mkdir -p $out
cmd="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --eager --extra dl3dv --extra-steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- $cmd > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- $cmd > $out/write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $out/sq -o run -- $cmd > $out/sq.log 2>&1
python3 tools/pmc_summary.py $out/fetch $out/write $out/sq > $out/pmc_summary.json
echo done
