"""Dispatch timeline of the last minibatches of a rocprofv3 --kernel-trace CSV of tools/bench_update.py
(the dispatches before its old-log-prob timing launches): start / end offsets and duration (us), queue.
    python tools/mb_timeline.py <run_kernel_trace.csv> [n_dispatches]"""
import csv
import sys


def main():
    path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 32
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    lp = [i for i, r in enumerate(rows) if "actor_rowtile" in r["Kernel_Name"] and "false" in r["Kernel_Name"]]
    end = lp[-4] if len(lp) >= 4 else len(rows)
    sel = rows[max(0, end - n):end]
    t0 = int(sel[0]["Start_Timestamp"])
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']:>2} {r['Kernel_Name'][:64]}")


if __name__ == "__main__":
    main()
