"""Configuration schema: one source of truth for the Helm chart values and the
bootstrap settings (SURVEY.md §5 "Config / flag system").

The reference configures its stack through scattered shell edits (fstab,
modules-load.d, sysctl.d, containerd's config.toml, a kubeadm flag and one
``--set driver.enabled=false``; /root/reference/README.md:29-271).  Here:

* ``VALUES`` describes every key of ``charts/amd-gpu-stack/values.yaml``
  (type, range, help).  It renders the chart's ``values.schema.json`` —
  which ``helm install``/``helm template`` enforce natively — and
  :func:`validate_values` applies the same rules in ``mxk8s render``.  A test
  keeps values.yaml, the schema and this module in agreement.
* ``BOOTSTRAP`` describes the host bring-up settings.  They come from
  defaults < an ``mxk8s.toml`` file (``[bootstrap]`` table) < ``MXK8S_*``
  environment variables < command-line flags (:func:`load_bootstrap`).

    python -m mxk8s.config schema      # print values.schema.json
    python -m mxk8s.config write       # rewrite the chart's values.schema.json
    python -m mxk8s.config bootstrap [--config mxk8s.toml]   # effective settings
"""
from __future__ import annotations

import dataclasses
import json
import os
import re
import sys
from typing import Any, Callable, Optional

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHART_DIR = os.path.join(REPO, "charts", "amd-gpu-stack")


@dataclasses.dataclass
class F:
    """A leaf: JSON type, optional checks and help text."""
    type: str                              # string|integer|boolean|array|object
    help: str = ""
    minimum: Optional[int] = None
    maximum: Optional[int] = None
    enum: Optional[list] = None
    pattern: Optional[str] = None
    items: Optional[dict] = None           # JSON schema of array items
    const: Any = dataclasses.field(default=None)
    has_const: bool = False


_QTY = r"^[0-9]+(\.[0-9]+)?(m|Ki|Mi|Gi|Ti|k|M|G|T)?$"
_RES = {"type": "object", "additionalProperties": {"anyOf": [
    {"type": "string", "pattern": _QTY}, {"type": "integer", "minimum": 0}]}}
RESOURCES = {"requests": F("object", "resource requests", items=_RES),
             "limits": F("object", "resource limits", items=_RES)}
TOLERATION = {"type": "object", "properties": {
    "key": {"type": "string"}, "operator": {"enum": ["Exists", "Equal"]},
    "value": {"type": "string"},
    "effect": {"enum": ["NoSchedule", "PreferNoSchedule", "NoExecute", ""]}},
    "additionalProperties": False}
VALIDATOR_TESTS = ["rocminfo", "vectoradd", "gemm", "rccl", "ddp"]
COLLECTIVES = ["allreduce", "reducescatter", "allgather", "alltoall"]

VALUES: dict = {
    "driver": {"enabled": F("boolean", "containerised driver: unsupported (host-managed amdgpu)",
                            const=False, has_const=True)},
    "image": {"repository": F("string", "validator / plugin image"),
              "tag": F("string", "image tag"),
              "pullPolicy": F("string", "", enum=["Always", "IfNotPresent", "Never"])},
    "imagePullSecrets": F("array", "", items={"type": "object"}),
    "tolerations": F("array", "tolerations of every workload", items=TOLERATION),
    "nodeSelector": F("object", "node selector of every workload",
                      items={"type": "object", "additionalProperties": {"type": "string"}}),
    "resourceName": F("string", "extended resource advertised by the device plugin",
                      pattern=r"^[a-z0-9.-]+/[a-z0-9.-]+$"),
    "logFormat": F("string", "node daemon log format", enum=["json", "text"]),
    "stateDir": F("string", "host dir for the ECC baseline and health.json", pattern=r"^/"),
    "cdi": {"hostDir": F("string", "CDI spec directory on the host", pattern=r"^/"),
            "specFile": F("string", "spec file name", pattern=r"^[A-Za-z0-9._-]+\.(json|yaml)$"),
            "generate": F("boolean", "regenerate the spec from the plugin's init container")},
    "devicePlugin": {"enabled": F("boolean"), "cdiDevices": F("boolean"), "deviceSpecs": F("boolean"),
                     "healthInterval": F("integer", "seconds", minimum=1, maximum=3600),
                     "eventQuarantineSeconds": F("integer", "", minimum=0, maximum=86400),
                     "eccQuarantineSeconds": F("integer", "0 = out until reboot", minimum=0,
                                               maximum=86400 * 30),
                     "reconcileSeconds": F("integer", "GPU-set / CDI-spec resync, 0 = off",
                                           minimum=0, maximum=86400),
                     "partitionNaming": F("string", "compute-partition resource naming",
                                          enum=["single", "mixed"]),
                     "sharing": {"timeSlicing": {
                         "replicas": F("integer", "advertise each GPU this many times",
                                       minimum=1, maximum=64),
                         "renameByDefault": F("boolean", "advertise <resourceName>.shared"),
                         "failRequestsGreaterThanOne": F("boolean",
                                                         "refuse requests for >1 replica")}},
                     "privileged": F("boolean"), "priorityClassName": F("string"),
                     "resources": RESOURCES},
    "operator": {"enabled": F("boolean", "GPUStackPolicy operator instead of helm-managed operands"),
                 "interval": F("integer", "seconds", minimum=5, maximum=86400),
                 "resources": RESOURCES},
    "partitionManager": {"enabled": F("boolean"),
                         "interval": F("integer", "seconds", minimum=5, maximum=86400),
                         "settleTimeout": F("integer", "seconds", minimum=10, maximum=3600),
                         "drainTimeout": F("integer", "seconds the device plugin gets to "
                                                      "withdraw every device", minimum=1,
                                           maximum=3600),
                         "profiles": F("object", "profile name -> {compute, memory}",
                                       items={"type": "object", "additionalProperties": {
                                           "type": "object", "required": ["compute", "memory"],
                                           "properties": {
                                               "compute": {"enum": ["SPX", "DPX", "QPX", "CPX"]},
                                               "memory": {"enum": ["NPS1", "NPS2", "NPS4"]}}}}),
                         "resources": RESOURCES},
    "nodeValidator": {"enabled": F("boolean", "per-node validation chain gating the plugin / exporter"),
                      "steps": F("array", "validation steps, in order",
                                 items={"enum": ["driver", "cdi", "vectoradd", "plugin"]}),
                      "interval": F("integer", "re-validation check period (s)", minimum=5,
                                    maximum=86400),
                      "stepTimeout": F("integer", "seconds a step may retry", minimum=10,
                                       maximum=86400),
                      "resources": RESOURCES},
    "labeller": {"enabled": F("boolean"), "nfdFeatureFile": F("boolean"),
                 "interval": F("integer", "seconds", minimum=10, maximum=86400),
                 "resources": RESOURCES},
    "exporter": {"enabled": F("boolean"), "port": F("integer", "", minimum=1, maximum=65535),
                 "interval": F("integer", "seconds", minimum=1, maximum=3600),
                 "privileged": F("boolean"), "podResources": F("boolean"),
                 "service": {"type": F("string", "", enum=["ClusterIP", "NodePort", "LoadBalancer"])},
                 "serviceMonitor": {
                     "enabled": F("boolean", "create a Prometheus-operator ServiceMonitor "
                                             "(dcgm-exporter serviceMonitor counterpart)"),
                     "interval": F("string", "scrape interval", pattern=r"^[0-9]+(ms|s|m)$"),
                     "honorLabels": F("boolean", "keep the exporter's gpu / pod labels on clashes"),
                     "additionalLabels": F("object", "extra labels (e.g. the Prometheus selector)",
                                           items={"type": "object",
                                                  "additionalProperties": {"type": "string"}})},
                 "resources": RESOURCES},
    "rccl": {"profile": F("string", "RCCL environment preset (mxk8s/parallel/rccl_env.py)",
                          enum=["none", "xgmi-node"]),
             "env": F("object", "extra NCCL_* / RCCL_* / TORCH_NCCL_* variables",
                      items={"type": "object", "additionalProperties": {"type": "string"},
                             "propertyNames": {"pattern": "^(NCCL_|RCCL_|TORCH_NCCL_|HSA_NO_SCRATCH_RECLAIM|HSA_FORCE_FINE_GRAIN)"}})},
    "validator": {"enabled": F("boolean"),
                  "gpus": F("integer", "amd.com/gpu requested by the validator pod", minimum=1,
                            maximum=8),
                  "tests": F("array", "", items={"enum": VALIDATOR_TESTS}),
                  "gemm": {"sizes": F("array", "", items={"type": "integer", "minimum": 256,
                                                          "maximum": 65536})},
                  "rccl": {"minBytes": F("integer", "", minimum=1),
                           "maxBytes": F("integer", "", minimum=1, maximum=1 << 36),
                           "ops": F("array", "", items={"enum": COLLECTIVES})},
                  "profile": F("boolean"), "debug": F("boolean"),
                  "ddp": {"enabled": F("boolean"),
                          "seqLen": F("integer", "", minimum=128, maximum=131072),
                          "steps": F("integer", "", minimum=1, maximum=100000)},
                  "backoffLimit": F("integer", "", minimum=0, maximum=100),
                  "activeDeadlineSeconds": F("integer", "", minimum=60),
                  "shmSizeLimit": F("string", "", pattern=_QTY),
                  "resources": RESOURCES},
}


def _leaf_schema(f: F) -> dict:
    s: dict = {"type": f.type}
    if f.help:
        s["description"] = f.help
    for k in ("minimum", "maximum", "enum", "pattern"):
        if getattr(f, k) is not None:
            s[k] = getattr(f, k)
    if f.has_const:
        s["const"] = f.const
    if f.items is not None:
        if f.type == "array":
            s["items"] = f.items
        else:
            s.update({k: v for k, v in f.items.items() if k != "type"})
    return s


def json_schema(spec: dict = VALUES) -> dict:
    props = {}
    for k, v in spec.items():
        props[k] = _leaf_schema(v) if isinstance(v, F) else json_schema(v)
    return {"type": "object", "properties": props, "additionalProperties": False}


def values_schema_document() -> dict:
    doc = {"$schema": "https://json-schema.org/draft-07/schema#",
           "title": "amd-gpu-stack values"}
    doc.update(json_schema())
    return doc


# ---- validation (the subset of JSON schema the document above uses) -------
def _check(schema: dict, v: Any, path: str, errs: list) -> None:
    if "anyOf" in schema:
        sub = []
        for alt in schema["anyOf"]:
            e: list = []
            _check(alt, v, path, e)
            if not e:
                return
            sub += e
        errs.append(f"{path}: {v!r} matches no allowed form")
        return
    t = schema.get("type")
    ok = {"string": isinstance(v, str), "boolean": isinstance(v, bool),
          "integer": isinstance(v, int) and not isinstance(v, bool),
          "array": isinstance(v, list), "object": isinstance(v, dict), None: True}[t]
    if not ok:
        errs.append(f"{path}: expected {t}, got {type(v).__name__} ({v!r})")
        return
    if "const" in schema and v != schema["const"]:
        errs.append(f"{path}: must be {schema['const']!r}"
                    + (" - a containerised driver is not supported (the amdgpu driver is "
                       "host-managed; see `mxk8s bootstrap --phase driver-check`)"
                       if path == "driver.enabled" else ""))
    if "enum" in schema and v not in schema["enum"]:
        errs.append(f"{path}: {v!r} not one of {schema['enum']}")
    if "minimum" in schema and isinstance(v, int) and v < schema["minimum"]:
        errs.append(f"{path}: {v} < minimum {schema['minimum']}")
    if "maximum" in schema and isinstance(v, int) and v > schema["maximum"]:
        errs.append(f"{path}: {v} > maximum {schema['maximum']}")
    if "pattern" in schema and isinstance(v, str) and not re.search(schema["pattern"], v):
        errs.append(f"{path}: {v!r} does not match {schema['pattern']}")
    if t == "array" and "items" in schema:
        for i, x in enumerate(v):
            _check(schema["items"], x, f"{path}[{i}]", errs)
    if t == "object":
        props = schema.get("properties", {})
        extra = schema.get("additionalProperties", True)
        names = schema.get("propertyNames", {}).get("pattern")
        for k, x in v.items():
            p = f"{path}.{k}" if path else k
            if names and not re.search(names, k):
                errs.append(f"{p}: key does not match {names}")
            if k in props:
                _check(props[k], x, p, errs)
            elif extra is False:
                errs.append(f"{p}: unknown key")
            elif isinstance(extra, dict):
                _check(extra, x, p, errs)


def validate_values(values: dict) -> list[str]:
    """Errors of a merged values tree against the chart schema ([] = valid)."""
    errs: list = []
    _check(json_schema(), values, "", errs)
    v = values.get("validator", {})
    r = v.get("rccl", {})
    if isinstance(r.get("minBytes"), int) and isinstance(r.get("maxBytes"), int) \
            and r["minBytes"] > r["maxBytes"]:
        errs.append("validator.rccl: minBytes > maxBytes")
    return errs


# ---- bootstrap settings ------------------------------------------------------
@dataclasses.dataclass
class B:
    type: type
    default: Any
    help: str
    check: Optional[Callable[[Any], bool]] = None


def _cidr(s: str) -> bool:
    m = re.match(r"^(\d+)\.(\d+)\.(\d+)\.(\d+)/(\d+)$", s)
    return bool(m) and all(int(x) < 256 for x in m.groups()[:4]) and 8 <= int(m.group(5)) <= 30


BOOTSTRAP: dict = {
    "root": B(str, "/", "filesystem root the phases write under (tests / dry runs)"),
    "node_name": B(str, "", "kubeadm nodeRegistration.name (default: hostname)"),
    "advertise_address": B(str, "", "API server advertise address (default: auto)"),
    "pod_cidr": B(str, "10.244.0.0/16", "pod network CIDR (Flannel's default)", _cidr),
    "kubernetes_version": B(str, "v1.34.1", "kubeadm kubernetesVersion",
                            lambda s: bool(re.match(r"^v1\.\d+\.\d+$", s))),
    "upgrade": B(bool, False, "apt-get upgrade in the prep phase"),
    "dry_run": B(bool, False, "print commands, write files under root only"),
}


def _coerce(name: str, spec: B, raw: Any) -> Any:
    if spec.type is bool and isinstance(raw, str):
        low = raw.strip().lower()
        if low in ("1", "true", "yes", "on"):
            return True
        if low in ("0", "false", "no", "off", ""):
            return False
        raise ValueError(f"{name}: not a boolean: {raw!r}")
    if not isinstance(raw, spec.type):
        raise ValueError(f"{name}: expected {spec.type.__name__}, got {raw!r}")
    return raw


def load_bootstrap(path: Optional[str] = None, env: Optional[dict] = None,
                   overrides: Optional[dict] = None) -> dict:
    """Effective bootstrap settings: defaults < TOML file < MXK8S_* env < overrides."""
    env = os.environ if env is None else env
    cfg = {k: s.default for k, s in BOOTSTRAP.items()}
    if path:
        try:
            import tomllib as toml   # py >= 3.11
        except ImportError:          # pragma: no cover - py3.10 image
            import tomli as toml
        with open(path, "rb") as f:
            data = toml.load(f)
        table = data.get("bootstrap", data)
        for k, raw in table.items():
            if k not in BOOTSTRAP:
                raise ValueError(f"{path}: unknown bootstrap setting {k!r}")
            cfg[k] = _coerce(k, BOOTSTRAP[k], raw)
    for k, spec in BOOTSTRAP.items():
        e = env.get("MXK8S_" + k.upper())
        if e is not None:
            cfg[k] = _coerce("MXK8S_" + k.upper(), spec, e)
    for k, v in (overrides or {}).items():
        if v is not None and k in BOOTSTRAP:
            cfg[k] = _coerce(k, BOOTSTRAP[k], v)
    for k, spec in BOOTSTRAP.items():
        if spec.check and cfg[k] and not spec.check(cfg[k]):
            raise ValueError(f"bootstrap setting {k}={cfg[k]!r} is invalid ({spec.help})")
    return cfg


def main(argv=None) -> int:
    import argparse
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)
    sub.add_parser("schema")
    sub.add_parser("write")
    b = sub.add_parser("bootstrap")
    b.add_argument("--config", default=None)
    a = p.parse_args(argv)
    if a.cmd == "schema":
        print(json.dumps(values_schema_document(), indent=2))
    elif a.cmd == "write":
        out = os.path.join(CHART_DIR, "values.schema.json")
        with open(out, "w") as f:
            f.write(json.dumps(values_schema_document(), indent=2) + "\n")
        print(out)
    else:
        print(json.dumps(load_bootstrap(a.config), indent=2))
    return 0


if __name__ == "__main__":
    sys.exit(main())
