"""scripts/kernel_breakdown.py: steady-state window from the roctx range
(init and warm-up kernels no longer count per step)."""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import kernel_breakdown as kb  # noqa: E402


def _csv(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_trace_window_excludes_init_and_matches_wall(tmp_path, capsys):
    tr, mk = str(tmp_path / "kernel_trace.csv"), str(tmp_path / "marker_api_trace.csv")
    ms = 1_000_000
    rows = [["bfloat16tofloat32_copy_kernel", 0, 83 * ms]]          # one-time init, outside
    t = 100 * ms
    for step in range(2):                                            # two 10 ms steps, back to back
        for name, d in (("Custom_Cijk_foo", 4), ("mxk_gemm_bf16_tn_w4i", 3), ("mxk_attn_bwd", 2),
                        ("mxk_adamw_bf16_kernel", 1)):
            rows.append([name, t, t + d * ms])
            t += d * ms
    _csv(tr, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], rows)
    _csv(mk, ["Function", "Start_Timestamp", "End_Timestamp"],
         [["step.forward", 100 * ms, 104 * ms], ["bench.timed", 100 * ms, 120 * ms]])
    kb.main(["--trace", tr, "--markers", mk, "--steps", "2"])
    out = capsys.readouterr().out
    lines = {l.split()[0]: l.split() for l in out.splitlines() if l and not l.startswith(" ")}
    assert float(lines["total"][1]) == 10.0                          # per step, init excluded
    assert float(lines["range"][2]) == 10.0 and "kernel sum / wall = 1.000" in out
    assert float(lines["gemm.hipblaslt"][1]) == 4.0 and "copy/fill" not in lines
