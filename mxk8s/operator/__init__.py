"""GPU stack operator — the ClusterPolicy controller of the GPU Operator the
reference installs (/root/reference/README.md:264-272),
re-built as a small level-triggered reconciler over the same chart.

A cluster-scoped ``GPUStackPolicy`` (``mxk8s.io/v1alpha1``) holds the chart
values as its ``spec`` (what ``ClusterPolicy`` is to the NVIDIA chart).  Every
``interval`` the controller:

  1. reads the policy (the oldest by name when there are several; the others
     are marked ``ignored``) and merges its spec over the chart defaults;
  2. validates it against the one values schema (``mxk8s/config.py``) and
     renders the operands with the chart's own templates (``mxk8s/chart``) —
     device plugin, labeller, exporter, partition manager, validator, RBAC;
  3. applies each object: created when missing, replaced when the live object
     drifted from the rendered one (rendered fields not a subset of the live
     object — an edited argument, a deleted volume, ...), a Job is re-created
     (its template is immutable);
  4. deletes objects it created earlier that the current spec no longer
     renders (``exporter.enabled: false`` removes the exporter), found by the
     ``app.kubernetes.io/managed-by=mxk8s-operator`` + policy labels;
  5. writes ``status``: state ``ready`` (every DaemonSet has its pods ready, the
     validator Job succeeded), ``notReady`` or ``error`` (invalid spec / render
     failure — nothing is applied then), per-operand readiness, the observed
     generation.

Where the NVIDIA operator gates operands per node with ``nvidia.com/gpu.deploy.*``
labels, this single-node stack uses the chart's node selector and tolerations.
"""
from __future__ import annotations

import copy
import dataclasses
import logging
from typing import Optional

from ..chart import render as chart_render
from ..chart.gotpl import FailError
from ..config import validate_values
from ..utils.kube import KubeClient, KubeError, collection_path, object_path

log = logging.getLogger("mxk8s.operator")

GROUP_VERSION = "mxk8s.io/v1alpha1"
KIND = "GPUStackPolicy"
POLICIES = collection_path(GROUP_VERSION, KIND)
MANAGED_BY = "app.kubernetes.io/managed-by"
MANAGER = "mxk8s-operator"
POLICY_LABEL = "mxk8s.io/policy"
# kinds the chart renders as operands (garbage collection scans these)
OPERAND_KINDS = [("apps/v1", "DaemonSet"), ("v1", "Service"), ("v1", "ConfigMap"),
                 ("batch/v1", "Job"), ("v1", "ServiceAccount"),
                 ("rbac.authorization.k8s.io/v1", "ClusterRole"),
                 ("rbac.authorization.k8s.io/v1", "ClusterRoleBinding"),
                 ("monitoring.coreos.com/v1", "ServiceMonitor")]   # 404 without the CRD: skipped


def is_subset(want, have) -> bool:
    """Every field of ``want`` is present with the same value in ``have``
    (server-side defaults and status on ``have`` are ignored)."""
    if isinstance(want, dict):
        return isinstance(have, dict) and all(k in have and is_subset(v, have[k])
                                              for k, v in want.items())
    if isinstance(want, list):
        return isinstance(have, list) and len(want) == len(have) and \
            all(is_subset(a, b) for a, b in zip(want, have))
    if isinstance(want, (int, float)) and isinstance(have, str) or \
            isinstance(have, (int, float)) and isinstance(want, str):
        return str(want) == str(have)
    return want == have


@dataclasses.dataclass
class ReconcileResult:
    state: str
    message: str = ""
    created: list = dataclasses.field(default_factory=list)
    updated: list = dataclasses.field(default_factory=list)
    deleted: list = dataclasses.field(default_factory=list)
    operands: list = dataclasses.field(default_factory=list)


class Controller:
    def __init__(self, client: KubeClient, namespace: str = "amd-gpu",
                 release: str = "amd-gpu-stack", chart_dir: str = chart_render.CHART_DIR):
        self.client = client
        self.namespace = namespace
        self.release = release
        self.chart_dir = chart_dir

    # ---------------------------------------------------------- rendering
    def desired(self, spec: dict) -> list[dict]:
        values = chart_render.deep_merge(chart_render.load_values(self.chart_dir), spec or {})
        values.setdefault("operator", {})["enabled"] = False   # render the operands themselves
        errs = validate_values(values)
        if errs:
            raise ValueError("; ".join(errs[:5]))
        docs = chart_render.manifests(chart_render.render(values, self.namespace, self.release,
                                                          self.chart_dir))
        return docs

    def _label(self, obj: dict, policy: str) -> dict:
        o = copy.deepcopy(obj)
        md = o.setdefault("metadata", {})
        if o["kind"] not in ("ClusterRole", "ClusterRoleBinding", "CustomResourceDefinition"):
            md.setdefault("namespace", self.namespace)
        md.setdefault("labels", {}).update({MANAGED_BY: MANAGER, POLICY_LABEL: policy})
        return o

    # ------------------------------------------------------------- apply
    def apply(self, obj: dict, res: ReconcileResult) -> dict:
        path = object_path(obj, self.namespace)
        name = f"{obj['kind']}/{obj['metadata']['name']}"
        try:
            live = self.client.get(path)
        except KubeError as e:
            if e.status != 404:
                raise
            coll = path.rsplit("/", 1)[0]
            res.created.append(name)
            log.info("creating %s", name, extra={"event": "operand_created", "component": name})
            return self.client.create(coll, obj)
        if is_subset(obj, live):
            return live
        if obj["kind"] == "Job":    # pod template is immutable: re-create
            self.client.delete(path)
            res.updated.append(name)
            return self.client.create(path.rsplit("/", 1)[0], obj)
        new = copy.deepcopy(obj)
        new["metadata"]["resourceVersion"] = live.get("metadata", {}).get("resourceVersion", "")
        res.updated.append(name)
        log.warning("%s drifted from the policy; replacing", name,
                    extra={"event": "operand_drift", "component": name})
        return self.client.replace(path, new)

    def garbage_collect(self, policy: str, keep: set, res: ReconcileResult) -> None:
        sel = f"{MANAGED_BY}={MANAGER},{POLICY_LABEL}={policy}"
        for api, kind in OPERAND_KINDS:
            ns = None if kind in ("ClusterRole", "ClusterRoleBinding") else self.namespace
            try:
                items = self.client.list(collection_path(api, kind, ns), sel)
            except KubeError as e:
                if e.status == 404:
                    continue
                raise
            for it in items:
                it.setdefault("apiVersion", api)
                it.setdefault("kind", kind)
                path = object_path(it, self.namespace)
                if path not in keep:
                    self.client.delete(path)
                    res.deleted.append(f"{kind}/{it['metadata']['name']}")
                    log.info("deleting %s/%s (no longer in the policy)", kind,
                             it["metadata"]["name"], extra={"event": "operand_deleted"})

    @staticmethod
    def readiness(obj: dict) -> Optional[bool]:
        st = obj.get("status", {}) or {}
        if obj["kind"] == "DaemonSet":
            want = st.get("desiredNumberScheduled")
            return want is not None and want > 0 and st.get("numberReady", 0) >= want
        if obj["kind"] == "Job":
            return st.get("succeeded", 0) >= 1
        return None

    # --------------------------------------------------------- reconcile
    def reconcile_once(self) -> ReconcileResult:
        pols = sorted(self.client.list(POLICIES), key=lambda p: p["metadata"]["name"])
        if not pols:
            return ReconcileResult("none", "no GPUStackPolicy")
        pol, others = pols[0], pols[1:]
        for o in others:
            self.client.patch_status(f"{POLICIES}/{o['metadata']['name']}",
                                     {"state": "ignored",
                                      "message": f"only {pol['metadata']['name']} is reconciled"})
        name = pol["metadata"]["name"]
        res = ReconcileResult("ready")
        try:
            docs = self.desired(pol.get("spec", {}))
        except (ValueError, FailError) as e:
            res.state, res.message = "error", f"invalid policy: {e}"
            log.error("policy %s: %s", name, res.message, extra={"event": "policy_invalid"})
            self._status(pol, res)
            return res
        keep = set()
        not_ready = []
        for d in docs:
            obj = self._label(d, name)
            live = self.apply(obj, res)
            keep.add(object_path(obj, self.namespace))
            r = self.readiness(live)
            if r is not None:
                res.operands.append({"kind": obj["kind"], "name": obj["metadata"]["name"],
                                     "ready": r})
                if not r:
                    not_ready.append(obj["metadata"]["name"])
        self.garbage_collect(name, keep, res)
        if not_ready:
            res.state = "notReady"
            res.message = "waiting for " + ", ".join(not_ready)
        else:
            res.message = f"{len(keep)} operand objects in sync"
        self._status(pol, res)
        return res

    def _status(self, pol: dict, res: ReconcileResult) -> None:
        self.client.patch_status(f"{POLICIES}/{pol['metadata']['name']}", {
            "state": res.state, "message": res.message, "operands": res.operands,
            "observedGeneration": pol["metadata"].get("generation", 1)})


def crd() -> dict:
    """The GPUStackPolicy CustomResourceDefinition (spec = chart values, kept
    schema-less here and validated by the controller against values.schema.json
    so one schema serves helm and the operator)."""
    return {
        "apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
        "metadata": {"name": "gpustackpolicies.mxk8s.io"},
        "spec": {"group": "mxk8s.io", "scope": "Cluster",
                 "names": {"kind": KIND, "plural": "gpustackpolicies", "singular": "gpustackpolicy",
                           "shortNames": ["gsp"]},
                 "versions": [{"name": "v1alpha1", "served": True, "storage": True,
                               "subresources": {"status": {}},
                               "additionalPrinterColumns": [
                                   {"name": "State", "type": "string", "jsonPath": ".status.state"},
                                   {"name": "Message", "type": "string",
                                    "jsonPath": ".status.message"}],
                               "schema": {"openAPIV3Schema": {
                                   "type": "object",
                                   "properties": {
                                       "spec": {"type": "object",
                                                "x-kubernetes-preserve-unknown-fields": True},
                                       "status": {"type": "object",
                                                  "x-kubernetes-preserve-unknown-fields": True}}}}}]}}
