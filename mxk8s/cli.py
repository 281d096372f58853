"""``mxk8s`` command line.

  mxk8s bootstrap [--config mxk8s.toml] [--phase P ...] [--all] [--dry-run] [--root DIR] [--upgrade]
  mxk8s doctor {gpu,node,pod NAME [-n NS]} [--root DIR]
  mxk8s render [--set k=v] [-f values.yaml] [-n NS] [-o FILE]     (offline helm template)
  mxk8s cdi [--root DIR] [--output FILE]                           (ROCm CDI spec)
  mxk8s enum [--root DIR] [--links]                                (GPU inventory JSON)
  mxk8s deploy-files                                               (regenerate deploy/)
  mxk8s validate ...    mxk8s deviceplugin ...    mxk8s labeller ...    mxk8s exporter ...
  mxk8s version
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys


def _bootstrap(a) -> int:
    from . import config
    from .bootstrap import phases
    try:
        cfg = config.load_bootstrap(a.config, overrides={
            "root": a.root, "dry_run": a.dry_run or None, "upgrade": a.upgrade or None,
            "node_name": a.node_name, "advertise_address": a.advertise_address,
            "pod_cidr": a.pod_cidr, "kubernetes_version": a.kubernetes_version})
    except (ValueError, OSError) as e:
        print(f"bootstrap config: {e}", file=sys.stderr)
        return 2
    ctx = phases.Context(root=cfg["root"], dry_run=cfg["dry_run"], upgrade=cfg["upgrade"],
                         node_name=cfg["node_name"], advertise_address=cfg["advertise_address"],
                         pod_cidr=cfg["pod_cidr"], kubernetes_version=cfg["kubernetes_version"])
    only = a.phase or None
    try:
        ran = phases.run(ctx, only=only, resume=not a.no_resume, until=a.until)
    except phases.PhaseError as e:
        print(f"bootstrap stopped: {e}", file=sys.stderr)
        return 2
    if a.dry_run:
        for c in ctx.commands():
            print(c)
    print(json.dumps({"ran": ran, "completed": phases.completed(ctx)}), file=sys.stderr)
    return 0


def _doctor(a) -> int:
    from . import doctor
    h = doctor.Host(a.root)
    if a.what == "gpu":
        checks = doctor.check_gpu(h)
    elif a.what == "node":
        checks = doctor.check_node(h)
    else:
        if not a.name:
            print("doctor pod needs a pod name", file=sys.stderr)
            return 2
        checks = doctor.check_pod(h, a.name, a.namespace)
    return doctor.run(checks)


def _render(a) -> int:
    from .chart import render
    from .chart.gotpl import FailError
    from . import config
    try:
        values = render.load_values(a.chart, a.values, a.set)
        errs = config.validate_values(values)
        if errs:
            print("Error: values don't meet the specifications of the schema(s):\n- "
                  + "\n- ".join(errs), file=sys.stderr)
            return 1
        text = render.to_stream(render.render(values, a.namespace, a.release, a.chart))
    except FailError as e:
        print(f"Error: execution error: {e}", file=sys.stderr)
        return 1
    if a.output == "-":
        sys.stdout.write(text)
    else:
        with open(a.output, "w") as f:
            f.write(text)
    return 0


def _cdi(a) -> int:
    from .native import node
    spec = json.dumps(node.cdi_spec(a.root, a.kind), indent=2) + "\n"
    if a.output:
        import os
        tmp = a.output + ".tmp"
        with open(tmp, "w") as f:
            f.write(spec)
        os.replace(tmp, a.output)
    else:
        sys.stdout.write(spec)
    return 0


def _enum(a) -> int:
    from .native import node
    out = {"gpus": [g.to_dict() for g in node.enumerate_gpus(a.root)]}
    if a.links:
        out["links"] = [dataclasses.asdict(l) for l in node.links(a.root)]
    print(json.dumps(out, indent=2))
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    passthrough = {"validate": "mxk8s.validate.__main__", "deviceplugin": "mxk8s.deviceplugin.__main__",
                   "labeller": "mxk8s.labeller.__main__", "exporter": "mxk8s.exporter.__main__"}
    if argv and argv[0] in passthrough:
        import importlib
        return importlib.import_module(passthrough[argv[0]]).main(argv[1:])

    p = argparse.ArgumentParser(prog="mxk8s", description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("bootstrap", help="idempotent host bring-up")
    b.add_argument("--phase", action="append", help="run only these phases")
    b.add_argument("--all", action="store_true", help="run every phase (default)")
    b.add_argument("--until", default=None, help="stop after this phase")
    b.add_argument("--config", default=os.environ.get("MXK8S_CONFIG"),
                   help="mxk8s.toml with a [bootstrap] table (see mxk8s.config)")
    b.add_argument("--dry-run", action="store_true")
    b.add_argument("--root", default=None)
    b.add_argument("--upgrade", action="store_true")
    b.add_argument("--no-resume", action="store_true")
    b.add_argument("--node-name", default=None)
    b.add_argument("--advertise-address", default=None)
    b.add_argument("--pod-cidr", default=None)
    b.add_argument("--kubernetes-version", default=None)
    d = sub.add_parser("doctor", help="troubleshooting decision trees")
    d.add_argument("what", choices=["gpu", "node", "pod"])
    d.add_argument("name", nargs="?")
    d.add_argument("-n", "--namespace", default="default")
    d.add_argument("--root", default="/")
    r = sub.add_parser("render", help="offline helm template of charts/amd-gpu-stack")
    r.add_argument("--set", action="append", default=[])
    r.add_argument("-f", "--values", action="append", default=[])
    r.add_argument("-n", "--namespace", default="amd-gpu")
    r.add_argument("--release", default="amd-gpu-stack")
    from .chart.render import CHART_DIR
    r.add_argument("--chart", default=CHART_DIR)
    r.add_argument("-o", "--output", default="-")
    c = sub.add_parser("cdi", help="print/write the ROCm CDI spec")
    c.add_argument("--root", default="")
    c.add_argument("--kind", default="amd.com/gpu")
    c.add_argument("--output", default=None)
    e = sub.add_parser("enum", help="GPU inventory (libmxnode)")
    e.add_argument("--root", default="")
    e.add_argument("--links", action="store_true")
    sub.add_parser("deploy-files", help="regenerate deploy/ manifests")
    sub.add_parser("version")
    for name in passthrough:
        sub.add_parser(name, help=f"see `mxk8s {name} --help`")
    a = p.parse_args(argv)
    if a.cmd == "bootstrap":
        return _bootstrap(a)
    if a.cmd == "doctor":
        return _doctor(a)
    if a.cmd == "render":
        return _render(a)
    if a.cmd == "cdi":
        return _cdi(a)
    if a.cmd == "enum":
        return _enum(a)
    if a.cmd == "deploy-files":
        from .bootstrap.manifests import write_deploy
        for f in write_deploy():
            print(f)
        return 0
    if a.cmd == "version":
        from . import __version__
        from .native import node
        print(f"mxk8s {__version__} ({node.version()})")
        return 0
    return 2


if __name__ == "__main__":
    sys.exit(main())
