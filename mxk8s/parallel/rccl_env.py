"""RCCL environment presets for one MI355X node (8 GPUs on xGMI).

The reference never runs a collective (it ends at a one-GPU smoke pod,
/root/reference/README.md:296-317); the GPU Operator it installs leaves NCCL
to its defaults.  Here the same knobs are one named profile, applied by the
trainer / bench before the process group (and the HIP runtime) starts, and
rendered by the chart into the validator Job and the example pods
(``rccl.profile`` / ``rccl.env`` in values.yaml), so a tuning run changes one
value instead of editing manifests.

Profiles:

  none       RCCL defaults.
  xgmi-node  single node, fully connected xGMI (7 links per GPU):
               NCCL_IB_DISABLE=1        no InfiniBand / RoCE probing inside one node
               HSA_NO_SCRATCH_RECLAIM=1 the runtime keeps kernel scratch allocated
                                        (RCCL kernels otherwise pay a re-allocation
                                        when a big compute kernel ran in between)
               TORCH_NCCL_HIGH_PRIORITY=1  the bucketed gradient reduce-scatter /
                                        all-gather streams run at high priority, so
                                        they are not starved by the backward GEMMs
                                        they overlap with

Channel counts (NCCL_MIN_NCHANNELS / NCCL_MAX_NCHANNELS), algorithm
(NCCL_ALGO) and protocol (NCCL_PROTO) stay with RCCL's topology-based choice
unless given explicitly in ``rccl.env``: ring collectives are bound per xGMI
link, and the right channel count depends on the message sizes of the
workload (``mx-allreduce-perf --scaling 1,2,4,8`` measures them).

Variables already present in the environment always win.
"""
from __future__ import annotations

import os
from typing import Mapping, MutableMapping, Optional

PROFILES: dict = {
    "none": {},
    "xgmi-node": {
        "NCCL_IB_DISABLE": "1",
        "HSA_NO_SCRATCH_RECLAIM": "1",
        "TORCH_NCCL_HIGH_PRIORITY": "1",
    },
}

# knobs the chart accepts in rccl.env (anything else is rejected at render time)
ALLOWED_PREFIXES = ("NCCL_", "RCCL_", "TORCH_NCCL_", "HSA_NO_SCRATCH_RECLAIM", "HSA_FORCE_FINE_GRAIN")


def resolve(profile: str = "xgmi-node", extra: Optional[Mapping[str, str]] = None) -> dict:
    if profile not in PROFILES:
        raise ValueError(f"unknown RCCL profile {profile!r} (have {sorted(PROFILES)})")
    env = dict(PROFILES[profile])
    for k, v in (extra or {}).items():
        if not k.startswith(ALLOWED_PREFIXES):
            raise ValueError(f"{k}: not an RCCL / NCCL variable")
        env[k] = str(v)
    return env


def apply(profile: str = "xgmi-node", extra: Optional[Mapping[str, str]] = None,
          environ: Optional[MutableMapping[str, str]] = None) -> dict:
    """Set the profile's variables that are not set yet; returns what the
    process runs with (for the result record).  Call before the first HIP call."""
    environ = os.environ if environ is None else environ
    out = {}
    for k, v in resolve(profile, extra).items():
        environ.setdefault(k, v)
        out[k] = environ[k]
    return out
