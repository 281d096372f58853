"""``python -m mxk8s.exporter --port 9400`` (DaemonSet entry point)."""
from __future__ import annotations

import argparse
import logging
import sys
import time

from ..utils.logs import setup_logging
from . import Exporter, ExporterConfig


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--port", type=int, default=9400)
    p.add_argument("--interval", type=float, default=5.0)
    p.add_argument("--pod-resources-socket", default=None)
    p.add_argument("--resource-name", default="amd.com/gpu",
                   help="device-plugin resource (its .shared rename is matched too)")
    p.add_argument("--health-state-file", default=None,
                   help="the device plugin's health.json (same verdicts as ListAndWatch)")
    p.add_argument("--sysfs-root", default="")
    p.add_argument("--state-dir", default=None,
                   help="node-validator markers (<state-dir>/validations): component 'validation'")
    p.add_argument("--once", action="store_true", help="print one sample and exit")
    p.add_argument("--log-format", choices=["json", "text"], default="json")
    a = p.parse_args(argv)
    setup_logging(a.log_format)
    ex = Exporter(ExporterConfig(port=a.port, interval=a.interval,
                                 pod_resources_socket=a.pod_resources_socket,
                                 resource_name=a.resource_name,
                                 health_state_file=a.health_state_file, sysfs_root=a.sysfs_root,
                                 state_dir=a.state_dir))
    if a.once:
        sys.stdout.write(ex.sample_once())
        return 0
    ex.start()
    logging.getLogger("mxk8s.exporter").info("serving /metrics on :%d", ex.port)
    while True:
        time.sleep(3600)


if __name__ == "__main__":
    sys.exit(main())
