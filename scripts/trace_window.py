"""Average duration of the last K dispatches of a kernel in a rocprofv3
kernel trace (the timed region of bench.py is the last K step-kernel
launches of the run): python scripts/trace_window.py TRACE.csv NEEDLE K"""
import csv, sys

path, needle, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = [r for r in csv.DictReader(open(path)) if needle in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
w = d[-k:]
print(f"{needle}: {len(d)} dispatches; all {sum(d) / len(d) / 1e3:.3f} us; "
      f"last {len(w)} (the timed region) {sum(w) / len(w) / 1e3:.3f} us")
