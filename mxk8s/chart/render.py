"""Offline ``helm template`` for ``charts/amd-gpu-stack``.

    python -m mxk8s.chart.render [--set driver.enabled=false] [-f values.yaml]
        [--namespace amd-gpu] [--release amd-gpu-stack] > deploy/amd-gpu-stack.yaml

Mirrors ``helm install gpu-operator nvidia/gpu-operator -n gpu-operator
--create-namespace --set driver.enabled=false`` (/root/reference/README.md:269-271):
same flag, same meaning (the host driver is pre-installed), rendered without a
cluster, helm or network.
"""
from __future__ import annotations

import argparse
import copy
import os
import sys
from typing import Any, Optional

import yaml

from .gotpl import Engine, _Scope

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHART_DIR = os.path.join(REPO, "charts", "amd-gpu-stack")


def _parse_scalar(v: str) -> Any:
    if v in ("true", "false"):
        return v == "true"
    if v in ("null", "~"):
        return None
    try:
        return int(v)
    except ValueError:
        pass
    try:
        return float(v)
    except ValueError:
        return v


def _split_top(expr: str) -> list[str]:
    """Split on commas outside ``{...}`` (Helm list syntax ``k={a,b}``)."""
    out, depth, cur = [], 0, ""
    for ch in expr:
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
            continue
        depth += ch == "{"
        depth -= ch == "}"
        cur += ch
    out.append(cur)
    return out


def apply_set(values: dict, expr: str) -> None:
    """Helm ``--set a.b.c=v`` (comma-separated assignments, ``{x,y}`` lists)."""
    for item in _split_top(expr):
        if not item:
            continue
        key, _, val = item.partition("=")
        parts = key.split(".")
        d = values
        for p in parts[:-1]:
            if not isinstance(d.get(p), dict):
                d[p] = {}
            d = d[p]
        if val.startswith("{") and val.endswith("}"):
            d[parts[-1]] = [_parse_scalar(x) for x in val[1:-1].split(",") if x]
        else:
            d[parts[-1]] = _parse_scalar(val)


def deep_merge(base: dict, over: dict) -> dict:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def load_values(chart_dir: str = CHART_DIR, files=(), sets=()) -> dict:
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        values = yaml.safe_load(f) or {}
    for fn in files:
        with open(fn) as f:
            values = deep_merge(values, yaml.safe_load(f) or {})
    for s in sets:
        apply_set(values, s)
    return values


def render(values: Optional[dict] = None, namespace: str = "amd-gpu",
           release: str = "amd-gpu-stack", chart_dir: str = CHART_DIR,
           include_notes: bool = False) -> dict[str, str]:
    """Render every template; returns {template path: rendered text}."""
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    if values is None:
        values = load_values(chart_dir)
    tdir = os.path.join(chart_dir, "templates")
    eng = Engine()
    names = sorted(os.listdir(tdir))
    for n in names:
        if n.startswith("_"):
            with open(os.path.join(tdir, n)) as f:
                eng.add(f.read())
    root = {"Values": values,
            "Release": {"Name": release, "Namespace": namespace, "Service": "Helm",
                        "IsInstall": True},
            "Chart": {"Name": chart["name"], "Version": chart["version"],
                      "AppVersion": chart.get("appVersion", "")},
            "Capabilities": {"KubeVersion": {"Version": "v1.34.0"}}}
    out = {}
    for n in names:
        if n.startswith("_") or (n == "NOTES.txt" and not include_notes):
            continue
        with open(os.path.join(tdir, n)) as f:
            nodes = eng.add(f.read())
        out[f"templates/{n}"] = eng.render_nodes(nodes, _Scope(root, root))
    return out


def manifests(rendered: dict[str, str]) -> list[dict]:
    docs = []
    for name in sorted(rendered):
        if name.endswith("NOTES.txt"):
            continue
        for d in yaml.safe_load_all(rendered[name]):
            if d:
                docs.append(d)
    return docs


def to_stream(rendered: dict[str, str]) -> str:
    parts = []
    for name in sorted(rendered):
        if name.endswith("NOTES.txt"):
            continue
        body = rendered[name].strip("\n")
        for doc in [x for x in body.split("\n---") if x.strip()]:
            doc = doc.strip("\n")
            if not doc.strip() or all(l.strip().startswith("#") or not l.strip()
                                      for l in doc.splitlines()):
                continue
            parts.append(f"---\n# Source: amd-gpu-stack/{name}\n{doc}\n")
    return "".join(parts)


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--set", action="append", default=[])
    p.add_argument("-f", "--values", action="append", default=[])
    p.add_argument("-n", "--namespace", default="amd-gpu")
    p.add_argument("--release", default="amd-gpu-stack")
    p.add_argument("--chart", default=CHART_DIR)
    p.add_argument("-o", "--output", default="-")
    a = p.parse_args(argv)
    values = load_values(a.chart, a.values, a.set)
    text = to_stream(render(values, a.namespace, a.release, a.chart))
    if a.output == "-":
        sys.stdout.write(text)
    else:
        with open(a.output, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
