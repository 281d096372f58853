"""``python -m mxk8s.operator`` (the operator Deployment's entry point)."""
from __future__ import annotations

import argparse
import logging
import sys
import time

from ..utils.kube import KubeClient
from ..utils.logs import setup_logging
from . import Controller


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--namespace", default="amd-gpu")
    p.add_argument("--release", default="amd-gpu-stack")
    p.add_argument("--interval", type=float, default=300.0,
                   help="resync period (s): between resyncs the controller sleeps on watches "
                        "of its policy and its DaemonSets / Jobs; 0 = reconcile once")
    p.add_argument("--server", default=None, help="API server URL (default: in-cluster)")
    p.add_argument("--token", default=None)
    p.add_argument("--log-format", choices=["json", "text"], default="json")
    p.add_argument("--injected-name", action="append", default=[],
                   help="name prefix of list items a mutating webhook adds to the operands "
                        "(not drift); repeatable")
    a = p.parse_args(argv)
    setup_logging(a.log_format)
    log = logging.getLogger("mxk8s.operator")
    client = KubeClient(a.server, a.token) if a.server else KubeClient.in_cluster()
    ctl = Controller(client, a.namespace, a.release, injected=a.injected_name)
    if a.interval <= 0:
        try:
            ctl.reconcile_once()
        except Exception as e:
            log.error("reconcile failed: %s", e)
            return 1
        return 0
    ctl.run(a.interval)
    return 0

if __name__ == "__main__":
    sys.exit(main())
