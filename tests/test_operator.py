"""GPUStackPolicy operator (ClusterPolicy-controller counterpart) against an
in-process fake API server: create from the policy, readiness in status,
drift repair, garbage collection on spec change, invalid specs rejected
without touching the operands."""
import copy
import threading
import time

import pytest
import yaml

from mxk8s import operator as op
from mxk8s.chart import render
from mxk8s.operator.fake_apiserver import FakeApiServer
from mxk8s.utils.kube import KubeClient

NS = "amd-gpu"
DS = f"/apis/apps/v1/namespaces/{NS}/daemonsets"
POL = op.POLICIES + "/default"


@pytest.fixture
def api():
    srv = FakeApiServer().start()
    yield srv
    srv.stop()


def _policy(api, spec=None, name="default"):
    api.put_object(f"{op.POLICIES}/{name}", {"apiVersion": op.GROUP_VERSION, "kind": op.KIND,
                                             "metadata": {"name": name}, "spec": spec or {}})


def _names(api, prefix):
    return sorted(p.rsplit("/", 1)[1] for p in api.objects if p.rsplit("/", 1)[0] == prefix)


def _ready(api, name, n=1):
    api.objects[f"{DS}/{name}"]["status"] = {"desiredNumberScheduled": n, "numberReady": n}


def test_creates_operands_and_reports_readiness(api):
    _policy(api)
    ctl = op.Controller(KubeClient(api.url), NS)
    r = ctl.reconcile_once()
    assert _names(api, DS) == ["amd-gpu-stack-device-plugin", "amd-gpu-stack-metrics-exporter",
                               "amd-gpu-stack-node-labeller", "amd-gpu-stack-node-validator"]
    assert f"/api/v1/namespaces/{NS}/services/amd-gpu-stack-metrics" in api.objects
    assert f"/apis/batch/v1/namespaces/{NS}/jobs/amd-gpu-stack-validator" in api.objects
    assert "/apis/rbac.authorization.k8s.io/v1/clusterroles/amd-gpu-stack-node-labeller" in api.objects
    ds = api.objects[f"{DS}/amd-gpu-stack-device-plugin"]
    assert ds["metadata"]["labels"][op.MANAGED_BY] == op.MANAGER
    assert ds["metadata"]["labels"][op.POLICY_LABEL] == "default"
    assert r.state == "notReady" and len(r.created) >= 8
    st = api.objects[POL]["status"]
    assert st["state"] == "notReady" and "device-plugin" in st["message"]
    # pods come up, the validator Job succeeds -> ready; nothing is re-applied
    for n in _names(api, DS):
        _ready(api, n)
    api.objects[f"/apis/batch/v1/namespaces/{NS}/jobs/amd-gpu-stack-validator"]["status"] = {"succeeded": 1}
    r = ctl.reconcile_once()
    assert r.state == "ready" and not (r.created or r.updated or r.deleted), r
    assert api.objects[POL]["status"]["state"] == "ready"
    assert all(o["ready"] for o in api.objects[POL]["status"]["operands"])
    assert api.objects[POL]["status"]["observedGeneration"] == 1


def test_repairs_drift_and_recreates_deleted(api):
    _policy(api)
    ctl = op.Controller(KubeClient(api.url), NS)
    ctl.reconcile_once()
    path = f"{DS}/amd-gpu-stack-device-plugin"
    live = api.objects[path]
    good = copy.deepcopy(live["spec"]["template"]["spec"]["containers"][0]["args"])
    live["spec"]["template"]["spec"]["containers"][0]["args"].append("--replicas=9")
    del api.objects[f"{DS}/amd-gpu-stack-node-labeller"]
    r = ctl.reconcile_once()
    assert "DaemonSet/amd-gpu-stack-device-plugin" in r.updated
    assert "DaemonSet/amd-gpu-stack-node-labeller" in r.created
    assert api.objects[path]["spec"]["template"]["spec"]["containers"][0]["args"] == good
    # server-side additions (defaults, status) are not drift
    api.objects[path]["spec"]["revisionHistoryLimit"] = 10
    api.objects[path]["status"] = {"numberReady": 1}
    assert not ctl.reconcile_once().updated


def test_spec_change_reconfigures_and_garbage_collects(api):
    _policy(api)
    ctl = op.Controller(KubeClient(api.url), NS)
    ctl.reconcile_once()
    api.objects[POL]["spec"] = {"exporter": {"enabled": False},
                                "devicePlugin": {"sharing": {"timeSlicing": {"replicas": 4}}}}
    api.objects[POL]["metadata"]["generation"] = 2
    r = ctl.reconcile_once()
    assert "DaemonSet/amd-gpu-stack-metrics-exporter" in r.deleted
    assert "Service/amd-gpu-stack-metrics" in r.deleted
    assert "amd-gpu-stack-metrics-exporter" not in _names(api, DS)
    args = api.objects[f"{DS}/amd-gpu-stack-device-plugin"]["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "--replicas=4" in args
    assert api.objects[POL]["status"]["observedGeneration"] == 2
    # objects it did not create are never collected
    api.put_object(f"{DS}/someone-elses", {"apiVersion": "apps/v1", "kind": "DaemonSet",
                                           "metadata": {"name": "someone-elses", "namespace": NS}})
    ctl.reconcile_once()
    assert f"{DS}/someone-elses" in api.objects


@pytest.mark.parametrize("spec,why", [({"driver": {"enabled": True}}, "driver.enabled"),
                                      ({"exporter": {"port": 70000}}, "exporter.port")])
def test_invalid_policy_is_reported_not_applied(api, spec, why):
    _policy(api)
    ctl = op.Controller(KubeClient(api.url), NS)
    ctl.reconcile_once()
    before = {p: copy.deepcopy(o) for p, o in api.objects.items() if p != POL}
    api.objects[POL]["spec"] = spec
    r = ctl.reconcile_once()
    assert r.state == "error" and why in r.message
    assert api.objects[POL]["status"]["state"] == "error"
    after = {p: o for p, o in api.objects.items() if p != POL}
    assert after == before            # operands untouched


def test_only_one_policy_is_reconciled(api):
    _policy(api, name="a-main")
    _policy(api, name="b-other")
    op.Controller(KubeClient(api.url), NS).reconcile_once()
    assert api.objects[op.POLICIES + "/b-other"]["status"]["state"] == "ignored"
    assert api.objects[op.POLICIES + "/a-main"]["status"]["state"] in ("ready", "notReady")


def test_chart_operator_mode_renders_crd_controller_and_policy():
    v = render.load_values(sets=["operator.enabled=true"])
    docs = render.manifests(render.render(v))
    kinds = [(d["kind"], d["metadata"]["name"]) for d in docs]
    assert ("DaemonSet", "amd-gpu-stack-device-plugin") not in kinds    # the operator owns them
    assert ("Deployment", "amd-gpu-stack-operator") in kinds
    crd = next(d for d in docs if d["kind"] == "CustomResourceDefinition")
    assert crd == op.crd()
    pol = next(d for d in docs if d["kind"] == op.KIND)
    assert pol["spec"]["devicePlugin"]["enabled"] is True and pol["spec"]["driver"]["enabled"] is False
    # the operator renders the same operands helm would have rendered
    want = render.manifests(render.render(render.load_values()))
    got = op.Controller(None, "amd-gpu").desired(pol["spec"])
    assert [(d["kind"], d["metadata"]["name"]) for d in got] == \
        [(d["kind"], d["metadata"]["name"]) for d in want]
    yaml.safe_dump(docs)


def test_is_subset():
    assert op.is_subset({"a": 1, "b": [{"c": "x"}]}, {"a": 1, "b": [{"c": "x", "d": 2}], "e": 3})
    assert not op.is_subset({"a": 1}, {"a": 2})
    assert not op.is_subset({"b": [1, 2]}, {"b": [1]})
    assert op.is_subset({"port": 9400}, {"port": "9400"})


def test_service_monitor_operand_created_and_collected(api):
    """exporter.serviceMonitor in the policy: the operator applies the
    ServiceMonitor (monitoring.coreos.com) and collects it when turned off."""
    sm = f"/apis/monitoring.coreos.com/v1/namespaces/{NS}/servicemonitors/amd-gpu-stack-metrics"
    _policy(api, {"exporter": {"serviceMonitor": {"enabled": True, "interval": "30s"}}})
    ctl = op.Controller(KubeClient(api.url), NS)
    r = ctl.reconcile_once()
    assert "ServiceMonitor/amd-gpu-stack-metrics" in r.created
    assert api.objects[sm]["spec"]["endpoints"][0]["interval"] == "30s"
    api.objects[POL]["spec"] = {}
    api.objects[POL]["metadata"]["generation"] = 2
    r = ctl.reconcile_once()
    assert "ServiceMonitor/amd-gpu-stack-metrics" in r.deleted and sm not in api.objects


def test_is_subset_quantities_and_named_lists():
    """server-side canonical quantities and defaulted /
    injected named list items are not drift; a real change still is."""
    assert op.is_subset({"cpu": "0.5", "memory": "1024Mi"}, {"cpu": "500m", "memory": "1Gi"})
    assert not op.is_subset({"cpu": "0.5"}, {"cpu": "50m"})
    want = {"env": [{"name": "A", "value": "1"}], "volumes": [{"name": "x"}, {"name": "y"}]}
    have = {"env": [{"name": "A", "value": "1"}],
            "volumes": [{"name": "y", "hostPath": {"path": "/y"}}, {"name": "x"},
                        {"name": "kube-api-access-7xk2p", "projected": {}}]}   # injected
    assert op.is_subset(want, have)
    assert not op.is_subset({"env": [{"name": "A", "value": "1"}]}, {"env": [{"name": "A", "value": "2"}]})
    assert not op.is_subset({"args": ["--a", "--b"]}, {"args": ["--b", "--a"]})   # order kept
    assert not op.is_subset({"enabled": True}, {"enabled": "True"})
    assert op.parse_quantity("1e3") == 1000 and op.parse_quantity("30s") is None


def test_is_subset_named_list_membership_and_order_are_drift():
    """an env var / volume / container the chart DROPPED is still
    on the live object -> drift (else the change is never applied); one the
    chart added is missing live -> drift; init containers run in order, so a
    re-ordering is drift; env order alone is not."""
    live = {"env": [{"name": "A", "value": "1"}, {"name": "OLD", "value": "x"}]}
    assert not op.is_subset({"env": [{"name": "A", "value": "1"}]}, live)
    assert not op.is_subset({"env": [{"name": "A", "value": "1"}, {"name": "NEW", "value": "y"},
                                     {"name": "OLD", "value": "x"}]}, live)
    assert op.is_subset({"env": [{"name": "OLD", "value": "x"}, {"name": "A", "value": "1"}]}, live)
    chain = [{"name": n, "image": "i"} for n in ("driver", "cdi", "vectoradd", "plugin")]
    spec = {"template": {"spec": {"initContainers": chain, "containers": [{"name": "main"}]}}}
    swapped = {"template": {"spec": {"initContainers": [chain[1], chain[0], *chain[2:]],
                                     "containers": [{"name": "main"}]}}}
    assert op.is_subset(spec, spec)
    assert not op.is_subset(spec, swapped)
    two = {"containers": [{"name": "a"}, {"name": "b"}]}
    assert not op.is_subset(two, {"containers": [{"name": "b"}, {"name": "a"}]})
    assert not op.is_subset({"containers": [{"name": "a"}]}, two)      # a container removed


def test_normalising_server_zero_writes_after_first_reconcile():
    srv = FakeApiServer(normalize=True).start()
    try:
        _policy(srv, {"devicePlugin": {"resources": {"requests": {"cpu": "0.05", "memory": "65536Ki"},
                                                     "limits": {"memory": "0.25Gi"}}}})
        # the fake server's "mutating webhook" injects INJECTED_BY_WEBHOOK
        ctl = op.Controller(KubeClient(srv.url), NS, injected=["INJECTED_BY_WEBHOOK"])
        r = ctl.reconcile_once()
        assert r.created
        live = srv.objects[f"{DS}/amd-gpu-stack-device-plugin"]["spec"]["template"]["spec"]
        c = live["containers"][0]
        assert c["resources"]["requests"] == {"cpu": "50m", "memory": "64Mi"}   # canonicalised
        assert live["volumes"][0]["name"] == "kube-api-access"                  # injected
        writes = {m: srv.count(m) for m in ("POST", "PUT", "DELETE")}
        for _ in range(3):
            r = ctl.reconcile_once()
            assert not (r.created or r.updated or r.deleted or r.pending), r
        assert {m: srv.count(m) for m in ("POST", "PUT", "DELETE")} == writes
    finally:
        srv.stop()


def test_owner_references_and_transition_times(api):
    _policy(api)
    uid = api.objects[POL]["metadata"]["uid"]
    ctl = op.Controller(KubeClient(api.url), NS)
    ctl.reconcile_once()
    for p, o in api.objects.items():
        if p == POL:
            continue
        refs = o["metadata"].get("ownerReferences")
        assert refs == [{"apiVersion": op.GROUP_VERSION, "kind": op.KIND, "name": "default",
                         "uid": uid, "controller": True, "blockOwnerDeletion": True}], p
    st = {o["name"]: o for o in api.objects[POL]["status"]["operands"]}
    t0 = st["amd-gpu-stack-device-plugin"]["lastTransitionTime"]
    assert st["amd-gpu-stack-device-plugin"]["ready"] is False and t0.endswith("Z")
    api.objects[POL]["status"]["operands"][0]["lastTransitionTime"] = "2020-01-01T00:00:00Z"
    ctl.reconcile_once()          # no transition: the time is kept
    kept = {o["name"]: o for o in api.objects[POL]["status"]["operands"]}
    first = api.objects[POL]["status"]["operands"][0]["name"]
    assert kept[first]["lastTransitionTime"] == "2020-01-01T00:00:00Z"
    _ready(api, "amd-gpu-stack-device-plugin")
    ctl.reconcile_once()
    now = {o["name"]: o for o in api.objects[POL]["status"]["operands"]}
    assert now["amd-gpu-stack-device-plugin"]["ready"] is True
    assert now["amd-gpu-stack-device-plugin"]["lastTransitionTime"] != "2020-01-01T00:00:00Z"


def test_job_recreate_uses_background_propagation_and_tolerates_lingering():
    """a plain DELETE of a Job orphans its pod and the Job lingers
    behind the orphan finalizer, so an immediate POST gets 409."""
    # a linger far beyond the test's run, released by the test itself: with
    # 0.6 s a loaded machine could let it pass before the pending assertion
    srv = FakeApiServer(job_orphan_linger=60.0).start()
    job = f"/apis/batch/v1/namespaces/{NS}/jobs/amd-gpu-stack-validator"
    try:
        _policy(srv)
        ctl = op.Controller(KubeClient(srv.url), NS, delete_wait_s=2.0)
        ctl.reconcile_once()
        uid0 = srv.objects[job]["metadata"]["uid"]
        srv.objects[job]["spec"]["template"]["spec"]["containers"][0]["args"].append("--x")
        r = ctl.reconcile_once()          # Background: gone at once, re-created this pass
        assert "Job/amd-gpu-stack-validator" in r.updated and not r.pending
        assert srv.objects[job]["metadata"]["uid"] != uid0
        # a Job stuck behind a finalizer (someone else's orphan delete): pending, no raise
        srv.handle("DELETE", job, None)
        assert "deletionTimestamp" in srv.objects[job]["metadata"]
        ctl.delete_wait_s = 0.1
        srv.objects[job]["spec"]["template"]["spec"]["containers"][0]["args"].append("--y")
        r = ctl.reconcile_once()
        assert r.pending == ["Job/amd-gpu-stack-validator"] and r.state == "notReady"
        srv.release_lingering()           # the garbage collector releases it
        r = ctl.reconcile_once()
        assert "Job/amd-gpu-stack-validator" in r.created and not r.pending
    finally:
        srv.stop()


def test_controller_wakes_on_watch_events_not_the_resync(api):
    ctl = op.Controller(KubeClient(api.url), NS)
    stop = threading.Event()
    t = threading.Thread(target=ctl.run, args=(60.0, stop.is_set), daemon=True)
    t.start()
    try:
        time.sleep(0.3)
        _policy(api)                       # a new policy: applied well before the 60 s resync
        end = time.monotonic() + 5
        while f"{DS}/amd-gpu-stack-device-plugin" not in api.objects and time.monotonic() < end:
            time.sleep(0.05)
        assert f"{DS}/amd-gpu-stack-device-plugin" in api.objects
        assert "watch:gpustackpolicies" in ctl.wakeups
        # drift on a managed DaemonSet (a PUT, so the server emits an event)
        path = f"{DS}/amd-gpu-stack-node-labeller"
        time.sleep(0.5)
        o = copy.deepcopy(api.objects[path])
        o["spec"]["template"]["spec"]["containers"][0]["args"].append("--bogus")
        api.handle("PUT", path, o)
        end = time.monotonic() + 5
        while "--bogus" in api.objects[path]["spec"]["template"]["spec"]["containers"][0]["args"] \
                and time.monotonic() < end:
            time.sleep(0.05)
        assert "--bogus" not in api.objects[path]["spec"]["template"]["spec"]["containers"][0]["args"]
        assert "watch:daemonsets" in ctl.wakeups and "resync" not in ctl.wakeups
    finally:
        stop.set()
        t.join(timeout=5)


def test_wait_for_change_leaves_no_watch_threads_behind(api):
    """each wakeup ends the OTHER collections' long polls too, so
    repeated wakeups (DaemonSet status churn) do not pile up threads and
    API-server watch connections for up to the resync interval."""
    ctl = op.Controller(KubeClient(api.url), NS)
    _policy(api)
    ctl.reconcile_once()
    path = f"{DS}/amd-gpu-stack-node-labeller"

    def live():
        return [t for t in threading.enumerate() if t.name == "mxk8s-watch" and t.is_alive()]

    for i in range(6):
        def poke():
            time.sleep(0.3)
            o = copy.deepcopy(api.objects[path])
            o.setdefault("status", {})["observedGeneration"] = i + 1
            api.handle("PUT", path, o)
        threading.Thread(target=poke, daemon=True).start()
        assert ctl.wait_for_change(60.0).startswith("watch:")
        assert live() == [], live()
    assert ctl.wait_for_change(0.5) == "resync" and live() == []


def test_mutating_policy_replace_loop_backs_off_and_names_drift(api, caplog):
    """A mutating admission policy (Kyverno-style) re-adds a container env var
    after every replace: the controller replaces once, then backs off
    (pending) instead of replacing on every pass, and logs which names
    drifted so the admin can pass --injected-name."""
    import logging
    _policy(api)
    now = [1000.0]                                   # injected clock: no timing flakiness
    ctl = op.Controller(KubeClient(api.url), NS, replace_backoff_s=0.3, clock=lambda: now[0])
    ctl.reconcile_once()
    path = f"{DS}/amd-gpu-stack-device-plugin"
    name = "DaemonSet/amd-gpu-stack-device-plugin"

    def mutate():
        c = api.objects[path]["spec"]["template"]["spec"]["containers"][0]
        c.setdefault("env", []).append({"name": "KYVERNO_INJECTED", "value": "1"})

    mutate()
    with caplog.at_level(logging.WARNING):
        r1 = ctl.reconcile_once()
    assert name in r1.updated
    assert any("KYVERNO_INJECTED" in rec.getMessage() for rec in caplog.records)
    mutate()                                   # the webhook mutates the replaced object again
    r2 = ctl.reconcile_once()
    assert name not in r2.updated and name in r2.backoff and not r2.pending
    assert "replace backing off" in r2.message and "re-creating" not in r2.message
    # nothing else would wake the loop when the backoff ends: run() waits at most that long
    assert 0.05 <= ctl.next_wait(300.0) <= 0.3
    now[0] += 0.35
    r3 = ctl.reconcile_once()                  # backoff expired: replaced again
    assert name in r3.updated
    mutate()
    now[0] += 0.35
    r4 = ctl.reconcile_once()                  # second backoff is twice as long (0.6 s)
    assert name in r4.backoff
    now[0] += 0.3
    assert name in ctl.reconcile_once().updated
    # a real policy change (new desired object) is not held by the old backoff
    mutate()
    assert name in ctl.reconcile_once().backoff
    _policy(api, {"devicePlugin": {"healthInterval": 7}})
    assert name in ctl.reconcile_once().updated
    assert ctl.next_wait(300.0) <= 0.3        # a fresh backoff: 1st step again
    # with the name allow-listed there is no drift at all
    ctl2 = op.Controller(KubeClient(api.url), NS, injected=["KYVERNO_"])
    assert name not in ctl2.reconcile_once().updated
