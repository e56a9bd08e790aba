"""Per-round LR search kernel durations of the last bench step in a rocprofv3 kernel trace."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tr = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
idx = [i for i, r in enumerate(tr) if "sgr_flt" in r["Kernel_Name"]][-1]
seq = tr[idx:]
for name in ("sgr_flt", "wiener_stats", "wiener_solve", "proj_err", "sgr_advance", "wiener_trial", "wiener_advance", "sgr_sse"):
    ds = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in seq if name in r["Kernel_Name"]]
    print("%-15s n=%-3d sum=%-6d %s" % (name, len(ds), sum(ds), ds[:24]))
end = [r for r in seq if "sgr_sse" in r["Kernel_Name"]]
print("sgr_flt start -> sgr_sse end: %.1f us" % ((int(end[0]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1000))
