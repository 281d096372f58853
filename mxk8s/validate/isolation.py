"""Pass criterion of BASELINE config 2: the smoke pod's RESULT lines.

The reference's GPU check is "the pod that requests ``nvidia.com/gpu: 1``
prints its GPU" (/root/reference/README.md:293-296, 303-318, 332-335);
BASELINE.md:37 tightens it to "the pod sees exactly 1 gfx950 agent and the
vectoradd result is exact".  ``check_results`` applies that to every RESULT
line of the pod's log:

* every line must carry ``"pass": true`` (not only the last one);
* there must be a vectoradd line;
* its ``visible_gpus`` must equal the pod's ``amd.com/gpu`` limit;
* its ``arch`` must be ``gfx950`` (the ``gcnArchName`` feature suffix
  ``:sramecc+:xnack-`` is ignored);
* when the device plugin told the pod which render nodes / BDFs it
  allocated (``expected_render_nodes`` / ``expected_bdfs``), the ones the
  pod sees must be exactly those.

The binary (``native/tools/vector_add_main.hip``) makes the same checks
itself; this module re-checks the printed facts so that an older payload
image, or one run without the Allocate environment, cannot pass by omission.

``python -m mxk8s.validate.isolation --gpus 1 --arch gfx950 < log`` exits 1
and prints the problems when the log fails.
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Iterable


def parse_results(lines: Iterable[str]) -> list[dict]:
    out = []
    for line in lines:
        line = line.strip()
        if line.startswith("RESULT "):
            line = line[7:]
        if not line.startswith("{"):
            continue
        try:
            out.append(json.loads(line))
        except ValueError:
            out.append({"pass": False, "error": f"unparseable RESULT line: {line[:120]}"})
    return out


def _arch(a: str) -> str:
    return (a or "").split(":", 1)[0]


def check_results(results: list[dict], gpus: int = 1, arch: str = "gfx950") -> list[str]:
    """Problems with a smoke pod's RESULT lines (empty list: config 2 passes)."""
    problems = []
    if not results:
        return ["no RESULT line in the pod log"]
    for r in results:
        if r.get("pass") is not True:
            problems.append(f"{r.get('test', '?')}: pass={r.get('pass')!r}"
                            + (f" ({r['error']})" if r.get("error") else ""))
    va = [r for r in results if r.get("test") == "vectoradd"]
    if not va:
        problems.append("no vectoradd RESULT line")
    for r in va:
        if r.get("visible_gpus") != gpus:
            problems.append(f"vectoradd: the pod sees {r.get('visible_gpus')} GPU(s), "
                            f"its amd.com/gpu limit is {gpus}")
        if arch and _arch(r.get("arch", "")) != arch:
            problems.append(f"vectoradd: arch {r.get('arch')!r}, expected {arch}")
        want = r.get("expected_render_nodes") or []
        if want and sorted(r.get("render_nodes") or []) != sorted(want):
            problems.append(f"vectoradd: render nodes {r.get('render_nodes')} != allocated {want}")
        want = r.get("expected_bdfs") or []
        if want and sorted(r.get("bdfs") or []) != sorted(want):
            problems.append(f"vectoradd: PCI devices {r.get('bdfs')} != allocated {want}")
    return problems


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=1, help="the pod's amd.com/gpu limit")
    ap.add_argument("--arch", default="gfx950")
    a = ap.parse_args(argv)
    problems = check_results(parse_results(sys.stdin), a.gpus, a.arch)
    for p in problems:
        print("FAIL " + p, file=sys.stderr)
    return 1 if problems else 0


if __name__ == "__main__":
    sys.exit(main())
