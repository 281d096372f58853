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
    p.add_argument("--interval", type=float, default=30.0, help="0 = reconcile once")
    p.add_argument("--server", default=None, help="API server URL (default: in-cluster)")
    p.add_argument("--token", default=None)
    p.add_argument("--log-format", choices=["json", "text"], default="json")
    a = p.parse_args(argv)
    setup_logging(a.log_format)
    log = logging.getLogger("mxk8s.operator")
    client = KubeClient(a.server, a.token) if a.server else KubeClient.in_cluster()
    ctl = Controller(client, a.namespace, a.release)
    while True:
        try:
            r = ctl.reconcile_once()
            if r.created or r.updated or r.deleted:
                log.info("reconciled: %s (created %d, updated %d, deleted %d)", r.state,
                         len(r.created), len(r.updated), len(r.deleted))
        except Exception as e:   # API server blip: retry next interval
            log.error("reconcile failed: %s", e)
        if a.interval <= 0:
            return 0
        time.sleep(a.interval)


if __name__ == "__main__":
    sys.exit(main())
