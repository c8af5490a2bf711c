"""Prints the kernel timeline of the last N dispatches of a rocprofv3 --kernel-trace CSV:
start offset (us, relative to the first shown), duration (us), queue, kernel name.
    python tools/trace_timeline.py <run_kernel_trace.csv> [N]"""
import csv
import sys


def main():
    path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
