"""Device busy fraction and inter-kernel gaps over the last N exact batches of
a rocprofv3 kernel trace (`python3 tools/trace_gaps.py run_kernel_trace.csv 20`)."""
import csv
import statistics
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "h16_kernel<8, true, false>" in r["Kernel_Name"]]
seq = rows[idx[-n - 1] + 1: idx[-1] + 8]
gaps, busy, prev = [], 0, None
t0 = int(seq[0]["Start_Timestamp"])
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev is not None:
        gaps.append(s - prev)
    prev = max(prev or 0, e)
    busy += e - s
span = prev - t0
print(f"span {span / 1e6:.3f} ms, kernels {busy / 1e6:.3f} ms, idle {1 - busy / span:.3%}, "
      f"median gap {statistics.median(gaps) / 1e3:.1f} us, max gap {max(gaps) / 1e3:.1f} us")
