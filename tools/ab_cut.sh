#!/bin/bash
# Same-box A/B of library variants on the depth-cut render legs (tools/cut_case.py under
# rocprofv3 kernel-trace): per-kernel average durations.
# usage: bash tools/ab_cut.sh TAG "KIND[:CHUNK] ..." NAME...   (NAME = main, main:VAR=VALUE or lib/variants/libdsplat_NAME.so)
set -u
TAG=${1:?tag}; CASES=${2:?cases}; shift 2
export TMPDIR=/tmp
out=gpurun_out/abcut_$TAG; mkdir -p $out; : > $out/summary.txt
for round in 1 2; do
  for n in "$@"; do
    # NAME: main, main:VAR=VALUE (the main library under one environment setting) or a variant
    lib=""; envset=""
    case "$n" in
      main) ;;
      main:*) envset=${n#main:} ;;
      *) lib=my_depthsplat_amd/lib/variants/libdsplat_$n.so ;;
    esac
    for c in $CASES; do
      kind=${c%%:*}; chunk=0; [ "$kind" != "$c" ] && chunk=${c##*:}
      d=$out/$(echo ${n} | tr ':=' '__')_${kind}${chunk}_r$round
      env DSPLAT_LIB=$lib $envset timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
        python3 tools/cut_case.py $kind --reps 6 --chunk $chunk > $d.log 2>&1 || { echo "$n $c failed"; tail -5 $d.log; exit 1; }
      f=$(find $d -name '*kernel_stats.csv' | head -1)
      python3 - "$n $c r$round" "$f" >> $out/summary.txt <<'PY'
import csv, sys
rows = {r["Name"]: r for r in csv.DictReader(open(sys.argv[2]))}
parts = []
for k in ("k_preprocess_cut", "k_scatter_cut", "k_project_survivors", "k_sort_lds", "k_sort_render", "k_render_fwd", "k_sort_groups", "k_msd_split"):
    for name, r in rows.items():
        if k in name:
            parts.append(f"{k}={float(r['TotalDurationNs']) / 1e3 / 6:.1f}us/call x{int(r['Calls']) // 6}")
print(sys.argv[1], " ".join(parts))
PY
      rm -rf $d  # traces: only the summary line comes back
    done
  done
done
cat $out/summary.txt
