"""Node validator — the GPU Operator's ``operator-validator`` DaemonSet
counterpart (an operand of the chart the reference installs at
/root/reference/README.md:269-271 and watches come up at README.md:283-286;
SURVEY.md R26g).

NVIDIA's validator runs a chain of init containers (driver, toolkit, cuda,
plugin validation) on every node, writes ``/run/nvidia/validations/<step>-ready``
as each passes, and the other operands' init containers wait on those files.
Here, per node, with the MI355X stack's own checks:

  driver     amdgpu loaded, /dev/kfd present, every KFD GPU is gfx950 and has
             its render node (libmxnode topology)
  cdi        the CDI spec containerd resolves ``amd.com/gpu=<i>`` with exists
             and equals the one generated from the live render nodes
  vectoradd  HIP vectoradd, bit-exact, on every GPU (bin/mx-vector-add)
  plugin     the device plugin's socket answers as the kubelet would ask it:
             options, a ListAndWatch with every GPU, an Allocate carrying the
             CDI name and /dev/kfd + render-node DeviceSpecs

Markers: ``<state_dir>/validations/<step>-ready`` (JSON).  A marker is valid
only for the boot AND the driver instance it was written under: its
``fingerprint`` hashes the KFD topology generation and every GPU's (gpu_id,
render minor), so a driver reload or GPU reset voids every marker at once,
even before the validator notices.  ``--watch`` re-runs the chain whenever
the fingerprint changes (and retries failed steps), so the device plugin,
which serves only while ``driver-ready`` is valid, re-validates after a
driver reload without a pod restart.

    python -m mxk8s.validate.node --steps driver,cdi,vectoradd,plugin [--watch 30]
    python -m mxk8s.validate.node --wait driver          # init containers
"""
from __future__ import annotations

import argparse
import hashlib
import json
import logging
import os
import subprocess
import sys
import time
from typing import Callable, Optional

from ..native import node

log = logging.getLogger("mxk8s.validate.node")

STEPS = ("driver", "cdi", "vectoradd", "plugin")
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.environ.get("MXK8S_BIN", os.path.join(REPO, "bin"))


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _host(root: str, rel: str) -> str:
    return os.path.join(root or "/", rel.lstrip("/"))


def boot_id(root: str = "") -> str:
    return _read(_host(root, "/proc/sys/kernel/random/boot_id")) or "unknown"


def fingerprint(root: str = "") -> str:
    """Identity of the running driver instance: KFD topology generation plus
    every GPU's (gpu_id, render minor, BDF, partition).  Changes on a driver
    reload, a GPU reset that re-creates the topology, or a repartition."""
    gen = _read(_host(root, "/sys/class/kfd/kfd/topology/generation_id")) or "0"
    try:
        gpus = node.enumerate_gpus(root)
    except RuntimeError:
        gpus = []
    ident = ";".join(f"{g.gpu_id}:{g.render_minor}:{g.bdf}:{g.partition}" for g in gpus)
    return hashlib.sha1(f"gen={gen}|{ident}".encode()).hexdigest()[:16]


def validations_dir(state_dir: str) -> str:
    return os.path.join(state_dir, "validations")


def marker_path(state_dir: str, step: str) -> str:
    return os.path.join(validations_dir(state_dir), f"{step}-ready")


def write_marker(state_dir: str, step: str, root: str, detail: dict) -> None:
    os.makedirs(validations_dir(state_dir), exist_ok=True)
    doc = {"step": step, "ok": True, "boot_id": boot_id(root), "fingerprint": fingerprint(root),
           "unix_ms": int(time.time() * 1000), "detail": detail}
    p = marker_path(state_dir, step)
    with open(p + ".tmp", "w") as f:
        json.dump(doc, f)
    os.replace(p + ".tmp", p)


def remove_markers(state_dir: str, steps=STEPS) -> None:
    for s in steps:
        try:
            os.unlink(marker_path(state_dir, s))
        except FileNotFoundError:
            pass


def read_marker(state_dir: str, step: str) -> Optional[dict]:
    try:
        with open(marker_path(state_dir, step)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def marker_valid(state_dir: str, step: str, root: str = "",
                 fp: Optional[str] = None) -> bool:
    m = read_marker(state_dir, step)
    return bool(m and m.get("ok") and m.get("boot_id") == boot_id(root)
                and m.get("fingerprint") == (fp or fingerprint(root)))


def status(state_dir: str, root: str = "", steps=STEPS) -> dict:
    """{step: valid} for the exporter, doctor and the plugin."""
    fp = fingerprint(root)
    return {s: marker_valid(state_dir, s, root, fp) for s in steps}


def wait_for(state_dir: str, steps, root: str = "", timeout: float = 0.0, poll: float = 1.0,
             stop: Optional[Callable[[], bool]] = None) -> bool:
    """Block until every step's marker is valid (timeout <= 0: forever)."""
    end = time.monotonic() + timeout if timeout > 0 else None
    last_log = 0.0
    while True:
        st = status(state_dir, root, steps)
        if all(st.values()):
            return True
        if stop is not None and stop():
            return False
        now = time.monotonic()
        if end is not None and now >= end:
            return False
        if now - last_log >= 30:
            log.info("waiting for validation: %s", ", ".join(s for s, ok in st.items() if not ok))
            last_log = now
        time.sleep(poll)


# ---------------------------------------------------------------- checks
def check_driver(root: str = "") -> tuple[bool, dict]:
    facts: dict = {"amdgpu_module": os.path.isdir(_host(root, "/sys/module/amdgpu")),
                   "kfd": os.path.exists(_host(root, "/dev/kfd"))}
    try:
        gpus = node.enumerate_gpus(root)
    except RuntimeError as e:
        return False, {**facts, "error": str(e)}
    facts["gpus"] = len(gpus)
    facts["archs"] = sorted({g.arch for g in gpus})
    missing = [g.index for g in gpus if not os.path.exists(_host(root, g.render_path))]
    facts["missing_render_nodes"] = missing
    ok = (facts["amdgpu_module"] and facts["kfd"] and len(gpus) > 0 and not missing
          and facts["archs"] == ["gfx950"])
    return ok, facts


def check_cdi(root: str, spec_path: str, kind: str = "amd.com/gpu") -> tuple[bool, dict]:
    try:
        with open(spec_path) as f:
            have = json.load(f)
    except (OSError, ValueError) as e:
        return False, {"spec": spec_path, "error": f"unreadable: {e}"}
    want = node.cdi_spec(root, kind)
    ok = have == want
    return ok, {"spec": spec_path, "devices": len(want.get("devices", [])),
                **({} if ok else {"error": "stale: differs from the live render nodes"})}


def _run_vectoradd(index: int) -> tuple[bool, str]:
    cmd = [os.path.join(BIN, "mx-vector-add"), "--n", "50000", "--device", str(index)]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    except (OSError, subprocess.TimeoutExpired) as e:
        return False, str(e)
    res = [json.loads(l[7:]) for l in p.stdout.splitlines() if l.startswith("RESULT ")]
    return p.returncode == 0 and bool(res) and all(r.get("pass") for r in res), p.stdout[-300:]


def check_vectoradd(root: str = "",
                    run: Callable[[int], tuple[bool, str]] = _run_vectoradd) -> tuple[bool, dict]:
    try:
        gpus = node.enumerate_gpus(root)
    except RuntimeError as e:
        return False, {"error": str(e)}
    bad = {}
    for g in gpus:
        ok, out = run(g.index)
        if not ok:
            bad[g.index] = out
    return (not bad and bool(gpus)), {"gpus": len(gpus), "failed": bad}


def check_plugin(plugin_dir: str, socket_name: str, expect_gpus: int,
                 timeout: float = 10.0) -> tuple[bool, dict]:
    """Talk to the device plugin exactly as the kubelet does."""
    import grpc

    from ..deviceplugin import api
    sock = os.path.join(plugin_dir, socket_name)
    if not os.path.exists(sock):
        return False, {"socket": sock, "error": "not serving"}
    try:
        with grpc.insecure_channel("unix:" + sock) as ch:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            stub = api.Stub(ch, "DevicePlugin")
            opts = stub.GetDevicePluginOptions(api.Empty(), timeout=timeout)
            stream = stub.ListAndWatch(api.Empty(), timeout=timeout)
            devs = next(iter(stream)).devices
            stream.cancel()
            healthy = [d.ID for d in devs if d.health == api.HEALTHY]
            facts = {"socket": sock, "devices": len(devs), "healthy": len(healthy),
                     "preferred_allocation": opts.get_preferred_allocation_available}
            if not healthy:
                return False, {**facts, "error": "no healthy device advertised"}
            req = api.AllocateRequest()
            req.container_requests.add(devices_ids=[healthy[0]])
            c = stub.Allocate(req, timeout=timeout).container_responses[0]
            paths = [d.host_path for d in c.devices]
            facts["allocate"] = {"cdi": [d.name for d in c.cdi_devices], "devices": paths}
            ok = ("/dev/kfd" in paths or bool(c.cdi_devices)) and len(devs) >= expect_gpus
            return ok, facts
    except (grpc.RpcError, grpc.FutureTimeoutError, StopIteration) as e:
        return False, {"socket": sock, "error": f"{type(e).__name__}: {e}"}


class NodeValidator:
    def __init__(self, state_dir: str, root: str = "", steps=STEPS,
                 cdi_spec: str = "/etc/cdi/amd.com-gpu.json", cdi_kind: str = "amd.com/gpu",
                 plugin_dir: str = "/var/lib/kubelet/device-plugins",
                 plugin_socket: Optional[str] = None, step_timeout: float = 300.0,
                 poll: float = 1.0,
                 vectoradd: Callable[[int], tuple[bool, str]] = _run_vectoradd,
                 resource_name: str = "amd.com/gpu", partition_naming: str = "single",
                 rename_shared: bool = False, replicas: int = 1):
        unknown = [s for s in steps if s not in STEPS]
        if unknown:
            raise ValueError(f"unknown validation step(s): {unknown}")
        self.state_dir, self.root, self.steps = state_dir, root, list(steps)
        self.cdi_spec, self.cdi_kind = cdi_spec, cdi_kind
        self.plugin_dir, self.plugin_socket = plugin_dir, plugin_socket
        self.step_timeout, self.poll = step_timeout, poll
        self.vectoradd = vectoradd
        self.runs = 0
        self.resource_name, self.partition_naming = resource_name, partition_naming
        self.rename_shared, self.replicas = rename_shared, replicas

    def plugin_socket_for(self, gpus) -> str:
        """The socket the device plugin serves for the current GPU set: the
        explicit --plugin-socket, else resolved exactly as the plugin does
        (PluginConfig.effective_resource / socket_for), so a CPX/DPX node
        under partitionNaming=mixed is probed on amd-gpu-<mode>.sock."""
        if self.plugin_socket:
            return self.plugin_socket
        from ..deviceplugin.plugin import PluginConfig
        cfg = PluginConfig(resource_name=self.resource_name, plugin_dir=self.plugin_dir,
                           partition_naming=self.partition_naming, replicas=self.replicas,
                           rename_shared=self.rename_shared, register=False)
        return cfg.socket_for(cfg.effective_resource(gpus))

    def check(self, step: str) -> tuple[bool, dict]:
        if step == "driver":
            return check_driver(self.root)
        if step == "cdi":
            return check_cdi(self.root, self.cdi_spec, self.cdi_kind)
        if step == "vectoradd":
            return check_vectoradd(self.root, self.vectoradd)
        try:
            gpus = node.enumerate_gpus(self.root)
        except RuntimeError:
            gpus = []
        return check_plugin(self.plugin_dir, self.plugin_socket_for(gpus), max(1, len(gpus)))

    def run_chain(self, stop: Optional[Callable[[], bool]] = None) -> bool:
        """Run the steps in order; each is retried until it passes or its
        timeout ends the chain (the markers of later steps stay absent)."""
        self.runs += 1
        for step in self.steps:
            if marker_valid(self.state_dir, step, self.root):
                continue
            end = time.monotonic() + self.step_timeout
            while True:
                ok, facts = self.check(step)
                if ok:
                    write_marker(self.state_dir, step, self.root, facts)
                    print("RESULT " + json.dumps({"test": f"node-{step}", "pass": True, **facts}),
                          flush=True)
                    break
                if time.monotonic() >= end or (stop is not None and stop()):
                    print("RESULT " + json.dumps({"test": f"node-{step}", "pass": False, **facts}),
                          flush=True)
                    log.warning("validation %s failed: %s", step, facts.get("error", facts))
                    return False
                time.sleep(self.poll)
        return True

    def watch_once(self, last_fp: Optional[str]) -> str:
        """One watch pass: on a new driver instance drop every marker and
        re-validate; otherwise re-run only what is missing."""
        fp = fingerprint(self.root)
        if last_fp is not None and fp != last_fp:
            log.warning("driver instance changed (fingerprint %s -> %s): re-validating", last_fp, fp,
                        extra={"event": "revalidate"})
            remove_markers(self.state_dir, self.steps)
        if not all(status(self.state_dir, self.root, self.steps).values()):
            self.run_chain()
        return fp


def main(argv=None) -> int:
    from ..utils.logs import setup_logging
    p = argparse.ArgumentParser(description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--state-dir", default="/var/lib/mxk8s")
    p.add_argument("--sysfs-root", default="")
    p.add_argument("--steps", default=",".join(STEPS))
    p.add_argument("--wait", default=None, help="comma list: block until these markers are valid")
    p.add_argument("--timeout", type=float, default=0.0, help="--wait / per-step timeout (0 = forever)")
    p.add_argument("--watch", type=float, default=0.0, help="re-validate every N s (0 = run once)")
    p.add_argument("--cdi-spec", default="/etc/cdi/amd.com-gpu.json")
    p.add_argument("--cdi-kind", default="amd.com/gpu")
    p.add_argument("--plugin-dir", default="/var/lib/kubelet/device-plugins")
    p.add_argument("--plugin-socket", default=None,
                   help="default: the socket the plugin serves for the current GPU set")
    p.add_argument("--resource-name", default="amd.com/gpu")
    p.add_argument("--partition-naming", choices=["single", "mixed"], default="single")
    p.add_argument("--replicas", type=int, default=1)
    p.add_argument("--rename-shared", default="false")
    p.add_argument("--log-format", choices=["json", "text"], default="json")
    a = p.parse_args(argv)
    setup_logging(a.log_format)
    if a.wait:
        steps = [s for s in a.wait.split(",") if s]
        return 0 if wait_for(a.state_dir, steps, a.sysfs_root, a.timeout) else 1
    v = NodeValidator(a.state_dir, a.sysfs_root, [s for s in a.steps.split(",") if s],
                      a.cdi_spec, a.cdi_kind, a.plugin_dir, a.plugin_socket,
                      step_timeout=a.timeout if a.timeout > 0 else 300.0,
                      resource_name=a.resource_name, partition_naming=a.partition_naming,
                      replicas=a.replicas,
                      rename_shared=str(a.rename_shared).lower() in ("1", "true", "yes"))
    if a.watch <= 0:
        return 0 if v.run_chain() else 1
    fp = None
    while True:
        try:
            fp = v.watch_once(fp)
        except Exception:       # keep the DaemonSet alive; markers stay absent
            log.exception("validation pass failed")
        time.sleep(a.watch)


if __name__ == "__main__":
    sys.exit(main())
