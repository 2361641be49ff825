"""Print the kernel timeline of the last bench step from a rocprofv3 kernel trace (csv)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "chunk_kernel" in r["Kernel_Name"]]
s = idx[-2] - int(sys.argv[2] if len(sys.argv) > 2 else 12)
prev = None
t0 = int(rows[idx[-2]]["Start_Timestamp"])
for r in rows[s:]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - prev) / 1e3 if prev else 0
    prev = en
    if (st - t0) / 1e3 > 6000:
        break
    print(f"{(st - t0) / 1e3:9.1f} gap {gap:7.1f} dur {(en - st) / 1e3:8.1f}  {r['Kernel_Name'][:70]}")
