"""Derives the sampler's HBM bytes per launch (bench.py's roofline.traffic) from the two PMC passes
of tools/profile_sampler.sh <tag> (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs).
Writes profiles/<tag>_pmc_sampler.json (per-kernel averages) and profiles/traffic.json.
FETCH_SIZE is doubled: on gfx950 it reports half of a 16-B/lane streaming read
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for those widths. Run here, not on the box:
    python tools/traffic_from_pmc.py <tag> [--envs 64]"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    acc = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            n, s = acc.get(k, (0, 0.0))
            acc[k] = (n + 1, s + float(r["Counter_Value"]))
    return {k: (n, s / n) for k, (n, s) in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic.json"))
    args = ap.parse_args()
    base = os.path.join(ROOT, "gpurun_out", f"sprof_{args.tag}")
    fetch = per_kernel(os.path.join(base, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(base, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    summary = {k: {"dispatches": fetch[k][0], "FETCH_SIZE_kB_avg": fetch[k][1],
                   "WRITE_SIZE_kB_avg": write.get(k, (0, 0.0))[1]} for k in fetch}
    with open(os.path.join(ROOT, "profiles", f"{args.tag}_pmc_sampler.json"), "w") as f:
        json.dump(summary, f, indent=1)
    name = max((k for k in fetch if "sample" in k and "kernel" in k), key=lambda k: fetch[k][0])
    fb = 2 * fetch[name][1] * 1024
    wb = write[name][1] * 1024
    out = {"kernel": name, "precision": args.precision, "envs": args.envs, "fetch_bytes_per_launch": fb,
           "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb,
           "method": ("tools/profile_sampler.sh: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate "
                      f"passes over tools/bench_sampler.py ({args.precision}); kB*1024; FETCH_SIZE doubled per "
                      "MI355X_MICROARCH.md (gfx950 counts 16-B/lane streaming reads at half); fabric-side "
                      "counters include Infinity-Cache hits"),
           "source": f"profiles/{args.tag}_pmc_sampler.json"}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
