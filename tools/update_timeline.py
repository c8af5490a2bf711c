"""Timeline of the update phase of the last profiled iteration (rocprofv3 --kernel-trace CSV of
tools/profile.sh): every dispatch from the last rollout's final sampler launch to the next
rollout's first, with start offsets (us), durations and queues; then the per-kernel gaps summary.
    python tools/update_timeline.py <run_kernel_trace.csv> [max_rows]"""
import csv
import sys


def main():
    path = sys.argv[1]
    nmax = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    samp = [i for i, r in enumerate(rows) if "sample_split" in r["Kernel_Name"] or "sample_kernel" in r["Kernel_Name"]]
    gaps = [(a, b) for a, b in zip(samp, samp[1:]) if b - a > 1]
    a, b = gaps[-1]
    sel = rows[a:b + 1]
    t0 = int(sel[0]["Start_Timestamp"])
    for r in sel[:nmax]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r.get('Queue_Id', '?'):>3} {r['Kernel_Name'][:70]}")
    print(f"update phase: {(int(sel[-1]['Start_Timestamp']) - int(sel[0]['End_Timestamp'])) / 1e3:.1f} us, "
          f"{len(sel) - 2} dispatches")


if __name__ == "__main__":
    main()
