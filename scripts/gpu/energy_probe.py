#!/usr/bin/env python3
"""Live amd-smi energy accumulator probe (exporter's amd_gpu_energy_joules_total)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.native import node  # noqa: E402

ok, msg = node.smi_open()
print("smi_open", ok, msg, flush=True)
s1 = node.smi_sample(0)
time.sleep(1.0)
s2 = node.smi_sample(0)
print("energy_j", s1.energy_j, s2.energy_j, "power_w", s2.power_w, flush=True)
