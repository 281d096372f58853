#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (mean per
dispatch) and derive utilisation ratios.

    python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 [--filter gemm]
"""
import argparse
import collections
import csv
import glob
import os


def load(dirs, filt):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                if filt and filt not in k:
                    continue
                key = (k, row.get("Dispatch_Id"))
                per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                if filt and filt not in k:
                    continue
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return per, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    per, dur = load(a.dirs, a.filter)
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k[:110]}")
        if dur.get(k):
            ds = sorted(dur[k])
            print(f"   dispatch time median {ds[len(ds)//2]*1e6:.1f} us over {len(ds)} dispatches")
        for c in sorted(m):
            print(f"   {c:32s} {m[c]:.4g}")
        w = m.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':32s} {m[c] / w:.3f}")
        g = m.get("GRBM_GUI_ACTIVE")
        if g and dur.get(k):
            ds = sorted(dur[k])
            print(f"   effective clock (GUI_ACTIVE/8/t)  {g / 8 / ds[len(ds)//2] / 1e9:.3f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            # MFMA_BUSY summed over all SIMDs (1024); GUI_ACTIVE summed over 8 XCDs
            util = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
            print(f"   MFMA busy fraction (per SIMD)     {util:.3f}")
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            print(f"   LDS bank-conflict cycles / active {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            if t:
                print(f"   L2 hit rate                       {m['TCC_HIT_sum'] / t:.3f}")


if __name__ == "__main__":
    main()
