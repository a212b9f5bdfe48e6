set -u
export TMPDIR=/tmp
out=gpurun_out/cut2; mkdir -p $out
timeout -k 10 200 python3 tools/cut_case.py dl3dv --reps 1 > $out/d.json 2>$out/d.err && cat $out/d.json || exit 1
for c in 0 1 2 3; do
timeout -k 10 200 python3 tools/cut_case.py recon12 --reps 1 --chunk $c > $out/e$c.json 2>$out/e$c.err && cat $out/e$c.json || exit 1
done
