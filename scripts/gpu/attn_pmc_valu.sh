#!/bin/bash
# One counter pass over attn_run.py: VALU / MFMA co-execution and activity
# split (--kernel-trace only; 8 SQ + 1 GRBM counters).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/attn_pmc_valu
mkdir -p $OUT
P="SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/pmc -o run -- python3 scripts/gpu/attn_run.py > $OUT/pass.log 2>&1
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/attn_pmc_valu/pmc/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, m in agg.items():
    if "attn" not in k:
        continue
    mean = {c: sum(v) / len(v) for c, v in m.items()}
    print("==", k)
    for c in sorted(mean):
        print(f"   {c:32s} {mean[c]:.4g}")
    g = mean.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
    if g:
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_VALU_MFMA_COEXEC_CYCLES"):
            if c in mean:
                print(f"   {c.lower()}_per_simd_cycle   {mean[c] / g:.3f}")
    w = mean.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA", "SQ_ACTIVE_INST_LDS"):
            if c in mean:
                print(f"   {c.lower()}_frac_of_wave_cycles   {mean[c] / w:.3f}")
PY
