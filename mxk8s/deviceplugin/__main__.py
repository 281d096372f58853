"""``python -m mxk8s.deviceplugin`` — the amd.com/gpu device plugin DaemonSet entry point."""
from __future__ import annotations

import argparse
import sys

from ..utils.logs import setup_logging
from .plugin import PluginConfig, run_forever


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "on")


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--resource-name", default="amd.com/gpu")
    p.add_argument("--plugin-dir", default="/var/lib/kubelet/device-plugins/")
    p.add_argument("--socket-name", default="amd-gpu.sock")
    p.add_argument("--sysfs-root", default="")
    p.add_argument("--health-interval", type=float, default=5.0)
    p.add_argument("--event-quarantine", type=float, default=60.0)
    p.add_argument("--cdi", type=_bool, default=True)
    p.add_argument("--device-specs", type=_bool, default=True)
    p.add_argument("--fault-file", default=None)
    p.add_argument("--no-smi-events", action="store_true")
    p.add_argument("--replicas", type=int, default=1,
                   help="time-slicing: advertise each GPU this many times")
    p.add_argument("--fail-requests-greater-than-one", type=_bool, default=False)
    p.add_argument("--rename-shared", type=_bool, default=False,
                   help="with --replicas>1 advertise <resource-name>.shared")
    p.add_argument("--ecc-quarantine", type=float, default=0.0,
                   help="seconds a GPU stays out after an uncorrectable-ECC increase "
                        "(0 = until reboot)")
    p.add_argument("--state-dir", default=None,
                   help="ECC baseline + health.json for the exporter (hostPath)")
    p.add_argument("--cdi-spec", default=None,
                   help="CDI spec file to keep in sync with the live render nodes")
    p.add_argument("--reconcile-interval", type=float, default=30.0,
                   help="seconds between GPU-set / CDI-spec reconciliations (0 = off)")
    p.add_argument("--partition-naming", choices=["single", "mixed"], default="single",
                   help="compute partitions as <resource> or <resource>-<mode>")
    p.add_argument("--require-validation", default="",
                   help="comma list of node-validator steps (e.g. driver) whose markers in "
                        "<state-dir>/validations must be valid before devices are served")
    p.add_argument("--log-format", choices=["json", "text"], default="json")
    a = p.parse_args(argv)
    setup_logging(a.log_format)
    cfg = PluginConfig(resource_name=a.resource_name, plugin_dir=a.plugin_dir,
                       socket_name=a.socket_name, sysfs_root=a.sysfs_root,
                       health_interval=a.health_interval, event_quarantine_s=a.event_quarantine,
                       use_cdi=a.cdi, use_device_specs=a.device_specs,
                       use_smi_events=not a.no_smi_events, replicas=a.replicas,
                       fail_requests_greater_than_one=a.fail_requests_greater_than_one,
                       rename_shared=a.rename_shared, ecc_quarantine_s=a.ecc_quarantine,
                       state_dir=a.state_dir, cdi_spec_path=a.cdi_spec,
                       reconcile_interval=a.reconcile_interval,
                       partition_naming=a.partition_naming,
                       require_validation=tuple(x for x in a.require_validation.split(",") if x))
    if a.fault_file:
        cfg.fault_file = a.fault_file
    run_forever(cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
