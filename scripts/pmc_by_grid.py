#!/usr/bin/env python3
"""Per-(kernel, grid size) means of rocprofv3 --pmc counters.

    python scripts/pmc_by_grid.py gpurun_out/r4map/pmc [more dirs] [--filter gemm]

Prints one line per (kernel, grid): dispatches, median duration (us) and the
mean of every counter; kernels are shortened to their name before the
argument list (template arguments kept), so schedules stay distinguishable.
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(name: str) -> str:
    depth, out = 0, []
    for ch in name:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:90]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for d in a.dirs:
        print(f"== {d}")
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        dur = collections.defaultdict(dict)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
                if a.filter and a.filter not in k[0]:
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k in sorted(vals, key=lambda k: (k[1], k[0])):
            cs = " ".join(f"{c}={statistics.mean(v):.4g}" for c, v in sorted(vals[k].items()))
            ds = list(dur[k].values())
            print(f"  grid {k[1]:>8} n={len(ds):3d} {statistics.median(ds):9.1f}us {k[0]}  {cs}")


if __name__ == "__main__":
    main()
