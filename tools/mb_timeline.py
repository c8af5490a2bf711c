"""Dispatch timeline around the PPO minibatches of a rocprofv3 --kernel-trace CSV: start / end
offsets and duration (us), queue, kernel, for the dispatches from the k-th TRAIN actor row-tile
launch on (default: the middle one of the trace), n dispatches.
    python tools/mb_timeline.py <run_kernel_trace.csv> [n_dispatches] [k]"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    tr = [i for i, r in enumerate(rows) if "actor_rowtile" in r["Kernel_Name"] and "true" in r["Kernel_Name"]]
    if not tr:
        sys.exit("no TRAIN actor row-tile dispatch in the trace")
    k = int(sys.argv[3]) if len(sys.argv) > 3 else len(tr) // 2
    start = tr[k] - 2
    sel = rows[start:start + n]
    t0 = int(sel[0]["Start_Timestamp"])
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']:>2} {r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
