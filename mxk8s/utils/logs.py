"""Structured logging for the node daemons (device plugin, labeller, exporter).

The reference's GPU triage step is ``kubectl logs`` on the device-plugin pod
(/root/reference/README.md:344).  With ``--log-format json`` (the chart
default) every record is one JSON object per line, so that triage is greppable
and machine-readable:

    {"ts": "2026-10-16T09:12:03.418Z", "level": "WARNING", "logger": "mxk8s.deviceplugin",
     "msg": "device 3 unhealthy", "device": "3", "event": "health_change",
     "reason": "uncorrectable ECC errors"}

Context fields are passed with ``extra={...}``; the keys below are lifted to
the top level of the object, anything else non-standard goes under "extra".
"""
from __future__ import annotations

import datetime
import json
import logging
import sys

FIELDS = ("device", "event", "reason", "bdf", "value", "resource", "component")
_STD = set(vars(logging.LogRecord("", 0, "", 0, "", (), None))) | {"message", "asctime"}


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        ts = datetime.datetime.fromtimestamp(record.created, tz=datetime.timezone.utc)
        out = {"ts": ts.strftime("%Y-%m-%dT%H:%M:%S.") + f"{int(record.msecs):03d}Z",
               "level": record.levelname, "logger": record.name, "msg": record.getMessage()}
        extra = {}
        for k, v in vars(record).items():
            if k in _STD or k.startswith("_"):
                continue
            if k in FIELDS:
                out[k] = v
            else:
                extra[k] = v
        if extra:
            out["extra"] = extra
        if record.exc_info:
            out["exc"] = self.formatException(record.exc_info)
        return json.dumps(out, default=str)


def setup_logging(fmt: str = "json", level: int = logging.INFO, stream=None) -> None:
    """Configure the root logger once: ``fmt`` is "json" or "text"."""
    h = logging.StreamHandler(stream or sys.stderr)
    if fmt == "json":
        h.setFormatter(JsonFormatter())
    elif fmt == "text":
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s %(message)s"))
    else:
        raise ValueError(f"log format must be json or text, got {fmt!r}")
    root = logging.getLogger()
    for old in list(root.handlers):
        root.removeHandler(old)
    root.addHandler(h)
    root.setLevel(level)
