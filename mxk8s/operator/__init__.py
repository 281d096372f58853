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
import hashlib
import json
import dataclasses
import logging
import re
import threading
import time
from fractions import Fraction
from typing import Optional, Sequence

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


_SUFFIX = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": 1,
           "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18,
           "Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_QTY = re.compile(r"^([+-]?(?:\d+\.?\d*|\.\d+))(?:[eE]([+-]?\d+))?(Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE])?$")


def parse_quantity(v) -> Optional[Fraction]:
    """A Kubernetes resource.Quantity (``500m``, ``0.5``, ``1Gi``, ``1e3``) as an
    exact number; None when ``v`` is not one.  The API server stores
    quantities in canonical form (``0.5`` -> ``500m``, ``1024Mi`` -> ``1Gi``),
    so rendered and live values are compared by value, not by spelling."""
    if isinstance(v, bool):
        return None
    if isinstance(v, (int, float)):
        return Fraction(v)
    if not isinstance(v, str):
        return None
    m = _QTY.match(v.strip())
    if not m:
        return None
    num = Fraction(m.group(1)) * (Fraction(10) ** int(m.group(2)) if m.group(2) else 1)
    return num * _SUFFIX[m.group(3) or ""]


def _named(items) -> bool:
    return bool(items) and all(isinstance(x, dict) and "name" in x for x in items)


# Named list items the API server or an admission webhook may add to a live
# object without the chart asking for them; every other extra item is drift.
# A cluster with its own mutating webhooks lists their names with
# Controller(injected=...) / the operator's --injected-name flag.
INJECTED_NAME_PREFIXES = ("kube-api-access",)
# lists whose order is semantic: init containers run in order (the node
# validator's driver -> cdi -> vectoradd -> plugin chain depends on it)
ORDERED_NAMED_LISTS = ("initContainers", "containers")


def is_subset(want, have, key: str = "", injected: tuple = INJECTED_NAME_PREFIXES) -> bool:
    """``have`` (live) is in sync with ``want`` (rendered): every field of
    ``want`` is present with the same value, server-side defaults and status
    on ``have`` are ignored, and quantities compare by value.  Lists of named
    items (containers, env, volumes, volumeMounts, ports) are matched by
    name, so that server-defaulted fields inside an item are tolerated; but
    the set of names must be the same — an item the chart dropped, or one it
    added, is drift — except names an admission controller injects
    (``INJECTED_NAME_PREFIXES``).  ``initContainers`` / ``containers`` must
    also keep their order.  Other lists (args, command, tolerations) keep
    their order and length."""
    if isinstance(want, dict):
        return isinstance(have, dict) and all(k in have and is_subset(v, have[k], k, injected)
                                              for k, v in want.items())
    if isinstance(want, list):
        if not isinstance(have, list):
            return False
        if _named(want):
            live = [x for x in have if not (isinstance(x, dict) and isinstance(x.get("name"), str)
                                            and x["name"].startswith(injected))]
            if not _named(live) and live:
                return False
            want_names = [w["name"] for w in want]
            live_names = [x["name"] for x in live]
            if key in ORDERED_NAMED_LISTS:
                if want_names != live_names:
                    return False
            elif sorted(want_names) != sorted(live_names):
                return False
            by_name = {x["name"]: x for x in live}
            return all(is_subset(w, by_name[w["name"]], "", injected) for w in want)
        return len(want) == len(have) and all(is_subset(a, b, "", injected)
                                              for a, b in zip(want, have))
    if want == have:
        return True
    if isinstance(want, bool) or isinstance(have, bool):
        return False
    if isinstance(want, (int, float, str)) and isinstance(have, (int, float, str)):
        if str(want) == str(have):
            return True
        qw, qh = parse_quantity(want), parse_quantity(have)
        return qw is not None and qw == qh
    return False


def drift_names(want, have, injected: tuple = INJECTED_NAME_PREFIXES, path: str = "") -> list:
    """Named list items that differ between ``want`` and ``have``, as
    ``"<path>: +name"`` (only live) / ``"<path>: -name"`` (only rendered):
    what an admin adds to ``--injected-name`` when a mutating admission
    policy, not the chart, put the ``+`` items there."""
    out = []
    if isinstance(want, dict) and isinstance(have, dict):
        for k, v in want.items():
            if k in have:
                out += drift_names(v, have[k], injected, f"{path}.{k}" if path else k)
    elif isinstance(want, list) and isinstance(have, list) and _named(want):
        live = [x for x in have if isinstance(x, dict) and isinstance(x.get("name"), str)
                and not x["name"].startswith(injected)]
        wn = {w["name"] for w in want}
        ln = {x["name"] for x in live}
        out += [f"{path}: +{n}" for n in sorted(ln - wn)]
        out += [f"{path}: -{n}" for n in sorted(wn - ln)]
        by_name = {x["name"]: x for x in live}
        for w in want:
            if w["name"] in by_name:
                out += drift_names(w, by_name[w["name"]], injected, f"{path}[{w['name']}]")
    return out


@dataclasses.dataclass
class ReconcileResult:
    state: str
    message: str = ""
    created: list = dataclasses.field(default_factory=list)
    updated: list = dataclasses.field(default_factory=list)
    deleted: list = dataclasses.field(default_factory=list)
    operands: list = dataclasses.field(default_factory=list)
    pending: list = dataclasses.field(default_factory=list)   # retried next pass
    backoff: list = dataclasses.field(default_factory=list)   # replace held by the backoff


class Controller:
    def __init__(self, client: KubeClient, namespace: str = "amd-gpu",
                 release: str = "amd-gpu-stack", chart_dir: str = chart_render.CHART_DIR,
                 delete_wait_s: float = 5.0, injected: Sequence[str] = (),
                 replace_backoff_s: float = 1.0, replace_backoff_max_s: float = 300.0,
                 clock=time.monotonic):
        self.client = client
        self.clock = clock            # replace backoff time source (tests inject one)
        # consecutive replaces of one object back off exponentially: a
        # mutating admission policy that re-adds an item after every replace
        # would otherwise make each reconcile replace it again, and the
        # MODIFIED event wake the loop again (a hot loop)
        self.replace_backoff_s = replace_backoff_s
        self.replace_backoff_max_s = replace_backoff_max_s
        # path -> [consecutive replaces, next allowed, names logged, desired hash];
        # a new desired object (a policy edit) starts a fresh backoff
        self._replaces: dict = {}
        self.injected = tuple(INJECTED_NAME_PREFIXES) + tuple(injected)
        self.namespace = namespace
        self.release = release
        self.chart_dir = chart_dir
        self.delete_wait_s = delete_wait_s
        self.wakeups: list[str] = []      # what ended each wait_for_change (tests, logs)

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

    def _label(self, obj: dict, policy: dict) -> dict:
        """Operand as applied: managed-by + policy labels (garbage collection
        by this controller) and an ownerReference to the policy, so that the
        cluster's garbage collector removes every operand when the policy is
        deleted (ClusterPolicy semantics; the policy is cluster-scoped, so it
        may own namespaced and cluster-scoped objects alike)."""
        o = copy.deepcopy(obj)
        md = o.setdefault("metadata", {})
        if o["kind"] not in ("ClusterRole", "ClusterRoleBinding", "CustomResourceDefinition"):
            md.setdefault("namespace", self.namespace)
        pmd = policy["metadata"]
        md.setdefault("labels", {}).update({MANAGED_BY: MANAGER, POLICY_LABEL: pmd["name"]})
        if pmd.get("uid"):
            md["ownerReferences"] = [{"apiVersion": GROUP_VERSION, "kind": KIND, "name": pmd["name"],
                                      "uid": pmd["uid"], "controller": True,
                                      "blockOwnerDeletion": True}]
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
        if is_subset(obj, live, injected=self.injected):
            self._replaces.pop(path, None)
            return live
        if obj["kind"] == "Job":    # pod template is immutable: re-create
            return self._recreate_job(path, name, obj, live, res)
        want = hashlib.sha256(json.dumps(obj, sort_keys=True, default=str).encode()).hexdigest()
        st = self._replaces.get(path)
        if st is None or st[3] != want:
            st = self._replaces[path] = [0, 0.0, None, want]
        now = self.clock()
        if now < st[1]:
            res.backoff.append(name)      # backing off: retried when the backoff ends
            return live
        names = drift_names(obj, live, self.injected)
        if names and names != st[2]:
            log.warning("%s drift in named items %s; if an admission controller adds them, "
                        "pass --injected-name", name, ", ".join(names),
                        extra={"event": "operand_drift_names", "component": name})
            st[2] = names
        st[0] += 1
        st[1] = now + min(self.replace_backoff_max_s, self.replace_backoff_s * 2 ** (st[0] - 1))
        new = copy.deepcopy(obj)
        new["metadata"]["resourceVersion"] = live.get("metadata", {}).get("resourceVersion", "")
        res.updated.append(name)
        log.warning("%s drifted from the policy; replacing", name,
                    extra={"event": "operand_drift", "component": name})
        return self.client.replace(path, new)

    def _recreate_job(self, path: str, name: str, obj: dict, live: dict,
                      res: ReconcileResult) -> dict:
        """Delete with Background propagation (the server's default for Jobs
        is Orphan: the old validator pod, holding GPUs, would keep running and
        the Job would linger behind the orphan finalizer), wait briefly for it
        to be gone, then create.  Still there, or a 409 on the create: the
        re-creation is pending and retried on the next pass, never raised."""
        if "deletionTimestamp" not in live.get("metadata", {}):
            self.client.delete(path, propagation="Background")
            log.warning("%s drifted from the policy; re-creating", name,
                        extra={"event": "operand_drift", "component": name})
        end = time.monotonic() + self.delete_wait_s
        while True:
            try:
                cur = self.client.get(path)
            except KubeError as e:
                if e.status != 404:
                    raise
                break
            if time.monotonic() >= end:
                res.pending.append(name)
                return cur
            time.sleep(0.05)
        try:
            new = self.client.create(path.rsplit("/", 1)[0], obj)
        except KubeError as e:
            if e.status != 409:
                raise
            res.pending.append(name)
            return live
        res.updated.append(name)
        return new

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
        prev = {(o.get("kind"), o.get("name")): o
                for o in (pol.get("status") or {}).get("operands", []) or []}
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        for d in docs:
            obj = self._label(d, pol)
            live = self.apply(obj, res)
            keep.add(object_path(obj, self.namespace))
            r = self.readiness(live)
            if r is not None:
                key = (obj["kind"], obj["metadata"]["name"])
                old = prev.get(key)
                ltt = old.get("lastTransitionTime") if old and old.get("ready") == r else now
                res.operands.append({"kind": key[0], "name": key[1], "ready": r,
                                     "lastTransitionTime": ltt or now})
                if not r:
                    not_ready.append(obj["metadata"]["name"])
        self.garbage_collect(name, keep, res)
        if not_ready or res.pending or res.backoff:
            res.state = "notReady"
            res.message = "waiting for " + ", ".join(
                not_ready + [f"{p} (re-creating)" for p in res.pending]
                + [f"{p} (drifted; replace backing off)" for p in res.backoff])
        else:
            res.message = f"{len(keep)} operand objects in sync"
        self._status(pol, res)
        return res

    def _status(self, pol: dict, res: ReconcileResult) -> None:
        st = {"state": res.state, "message": res.message, "operands": res.operands,
              "observedGeneration": pol["metadata"].get("generation", 1)}
        old = pol.get("status") or {}
        if all(old.get(k) == v for k, v in st.items()):
            return                         # no status write (and no watch event) when in sync
        self.client.patch_status(f"{POLICIES}/{pol['metadata']['name']}", st)

    # ----------------------------------------------------------- watching
    def _watched(self) -> list[tuple[str, Optional[str]]]:
        sel = f"{MANAGED_BY}={MANAGER}"
        return [(POLICIES, None),
                (collection_path("apps/v1", "DaemonSet", self.namespace), sel),
                (collection_path("batch/v1", "Job", self.namespace), sel)]

    def wait_for_change(self, timeout: float, stop=None) -> str:
        """Block until a policy or a managed DaemonSet / Job changes (a watch
        per collection, resumed at the collection's resourceVersion), or
        ``timeout`` (the resync: drift on kinds not watched).  Returns what
        woke it ("watch:<collection>" / "resync" / "stop")."""
        woke = threading.Event()
        why: list[str] = []
        cancels: list = []
        lock = threading.Lock()
        done = threading.Event()        # set when this call returns: late opens cancel themselves

        def opened(cancel):
            with lock:
                cancels.append(cancel)
                late = done.is_set()
            if late:
                cancel()

        def watch_one(path, sel, rv):
            try:
                for ev in self.client.watch(path, rv, timeout, sel, on_open=opened):
                    if ev.get("type") in ("ADDED", "MODIFIED", "DELETED"):
                        why.append("watch:" + path.rsplit("/", 1)[1])
                        woke.set()
                        return
                    if ev.get("type") == "ERROR":   # e.g. 410 Gone: resync now
                        why.append("watch-error")
                        woke.set()
                        return
            except Exception as e:                  # API server blip: fall back to the resync
                if not done.is_set():
                    log.debug("watch %s failed: %s", path, e)

        threads = []
        for path, sel in self._watched():
            try:
                _, rv = self.client.list_with_version(path, sel)
            except KubeError as e:
                if e.status == 404:
                    continue
                raise
            t = threading.Thread(target=watch_one, args=(path, sel, rv), daemon=True,
                                 name="mxk8s-watch")
            t.start()
            threads.append(t)
        end = time.monotonic() + timeout
        result = None
        while result is None:
            if woke.is_set():
                result = why[0] if why else "watch"
            elif stop is not None and stop():
                result = "stop"
            elif end - time.monotonic() <= 0:
                result = "resync"
            else:
                woke.wait(min(end - time.monotonic(), 0.2))
        # end the other collections' long polls now instead of leaving their
        # threads (and API-server watch connections) open for up to `timeout`
        with lock:
            done.set()
            pending = list(cancels)
        for cancel in pending:
            cancel()
        for t in threads:
            t.join(timeout=2.0)
        self.wakeups.append(result)
        return result

    def next_wait(self, interval: float) -> float:
        """The wait before the next pass: ``interval``, or less when a held
        replace's backoff ends sooner (nothing else would wake the loop)."""
        now = self.clock()
        ends = [st[1] - now for st in self._replaces.values() if st[1] > now]
        return min([interval] + [max(0.05, e) for e in ends])

    def run(self, interval: float = 300.0, stop=None) -> None:
        """Level-triggered loop: reconcile, then sleep until something this
        controller owns (or its policy) changes, at most ``interval`` s or
        until the earliest replace backoff ends."""
        while stop is None or not stop():
            try:
                r = self.reconcile_once()
                if r.created or r.updated or r.deleted or r.pending or r.backoff:
                    log.info("reconciled: %s (created %d, updated %d, deleted %d, pending %d, "
                             "backing off %d)", r.state, len(r.created), len(r.updated),
                             len(r.deleted), len(r.pending), len(r.backoff))
            except Exception as e:   # API server blip: retry after the next wake-up
                log.error("reconcile failed: %s", e)
            try:
                self.wait_for_change(self.next_wait(interval), stop)
            except Exception as e:
                log.error("watch setup failed: %s", e)
                time.sleep(min(interval, 5.0))


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
