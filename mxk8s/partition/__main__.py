"""``python -m mxk8s.partition --node-name $NODE_NAME`` (DaemonSet entry point)."""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

from ..utils.kube import KubeClient
from ..utils.logs import setup_logging
from . import DEFAULT_PROFILES, PartitionManager, combined_busy, pod_resources_users, smi_users


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    p.add_argument("--interval", type=float, default=30.0, help="0 = run once")
    p.add_argument("--sysfs-root", default="")
    p.add_argument("--profiles", default=None,
                   help="JSON file {name: {compute: SPX..CPX, memory: NPS1|NPS2}}")
    p.add_argument("--pod-resources-socket", default="/var/lib/kubelet/pod-resources/kubelet.sock")
    p.add_argument("--settle-timeout", type=float, default=120.0)
    p.add_argument("--state-dir", default="/var/lib/mxk8s",
                   help="shared with the device plugin: drain handshake files")
    p.add_argument("--drain-timeout", type=float, default=30.0)
    p.add_argument("--server", default=None, help="API server URL (default: in-cluster)")
    p.add_argument("--token", default=None)
    p.add_argument("--log-format", choices=["json", "text"], default="json")
    a = p.parse_args(argv)
    setup_logging(a.log_format)
    log = logging.getLogger("mxk8s.partition")
    if not a.node_name:
        p.error("--node-name (or NODE_NAME) is required")
    profiles = DEFAULT_PROFILES
    if a.profiles:
        with open(a.profiles) as f:
            profiles = json.load(f)
    client = KubeClient(a.server, a.token) if a.server else KubeClient.in_cluster()
    mgr = PartitionManager(client, a.node_name, a.sysfs_root, profiles,
                           busy=combined_busy(lambda: pod_resources_users(a.pod_resources_socket),
                                              smi_users),
                           settle_timeout=a.settle_timeout, state_dir=a.state_dir,
                           drain_timeout=a.drain_timeout)
    while True:
        try:
            mgr.reconcile_once()
        except Exception as e:   # keep the DaemonSet alive; retry next interval
            log.error("partition reconcile failed: %s", e)
        if a.interval <= 0:
            return 0
        time.sleep(a.interval)


if __name__ == "__main__":
    sys.exit(main())
