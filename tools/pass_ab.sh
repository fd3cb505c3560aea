#!/bin/bash
# A/B of the obs-statistics data pass: rocprofv3 kernel stats of tools/stats_prof.py with the default
# library and with $ALT (SPPRL_LIB), per (rows, ob) case.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for a in ${CASES:-"10000000 17" "1000000 11" "1000000 111"}; do
  for L in default ${ALT}; do
    tag=$(echo "$L $a" | tr ' /' '__')
    if [ $L = default ]; then E=""; else E="SPPRL_LIB=$R/$L"; fi
    env $E timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pab/$tag -o run --output-format csv -- \
      python3 $R/tools/stats_prof.py $a 20 > $R/gpurun_out/pab_$tag.log 2>&1 || exit 1
    python3 - $R/gpurun_out/pab/$tag/run_kernel_stats.csv "$L $a" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], " | ".join("%s %.1fus" % (r["Name"].split("(")[0].replace("spp::", "")[:18], float(r["AverageNs"]) / 1e3)
                             for r in rows if "k_st" in r["Name"]))
PY
  done
done
