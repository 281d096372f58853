"""``python -m mxk8s.labeller --node-name $NODE_NAME`` (DaemonSet entry point)."""
from __future__ import annotations

import argparse
import logging
import os
import sys
import time

from . import rocm_version, run_once
from ..native import node
from ..utils.kube import KubeClient
from ..utils.logs import setup_logging


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    p.add_argument("--interval", type=float, default=300.0, help="0 = run once")
    p.add_argument("--sysfs-root", default="")
    p.add_argument("--nfd-features-dir", default=None)
    p.add_argument("--server", default=None, help="API server URL (default: in-cluster)")
    p.add_argument("--token", default=None)
    p.add_argument("--log-format", choices=["json", "text"], default="json")
    a = p.parse_args(argv)
    setup_logging(a.log_format)
    log = logging.getLogger("mxk8s.labeller")
    if not a.node_name:
        p.error("--node-name (or NODE_NAME) is required")
    client = KubeClient(a.server, a.token) if a.server else KubeClient.in_cluster()
    driver = ""
    ok, _ = node.smi_open()
    if ok:
        driver = node.smi_driver_version()
    while True:
        try:
            gpus = node.enumerate_gpus(a.sysfs_root)
            patch = run_once(client, a.node_name, gpus, driver, rocm_version(), a.nfd_features_dir,
                             a.sysfs_root)
            log.info("node %s: %d GPU(s); patched %d label(s)", a.node_name, len(gpus), len(patch))
        except Exception as e:   # keep the DaemonSet alive; retry next interval
            log.error("labelling failed: %s", e)
            if a.interval <= 0:
                return 1
        if a.interval <= 0:
            return 0
        time.sleep(a.interval)


if __name__ == "__main__":
    sys.exit(main())
