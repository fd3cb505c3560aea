"""Per-dispatch durations of chosen kernels from a rocprofv3 kernel-trace CSV.
Usage: python tools/trace_kernels.py gpurun_out/prof_X/run_kernel_trace.csv k_dw k_sac_critic_phase"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for pat in sys.argv[2:]:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if pat in r["Kernel_Name"]]
    print("%s: %d dispatches; last 12 (ms): %s" % (pat, len(d), " ".join("%.3f" % x for x in d[-12:])))
