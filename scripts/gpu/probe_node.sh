#!/usr/bin/env bash
# GPU-box probe: real sysfs capture, libmxnode on real hardware, amd-smi sample,
# rocprofv3 counter list and a kernel-trace profile of the GEMM bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/capture_node.sh /tmp/node_capture && cp /tmp/node_capture.tar.gz gpurun_out/ > gpurun_out/capture.log 2>&1
./bin/mx-gpu-enum --links > gpurun_out/gpu_enum.json 2> gpurun_out/gpu_enum.err; echo "enum rc=$?"
./bin/mx-cdi-gen > gpurun_out/cdi.json 2> gpurun_out/cdi.err; echo "cdi rc=$?"
timeout -k 5 60 rocminfo > gpurun_out/rocminfo.txt 2>&1; echo "rocminfo rc=$?"
timeout -k 5 60 python3 - > gpurun_out/smi_sample.json 2> gpurun_out/smi_sample.err <<'PY'
import json, dataclasses
from mxk8s.native import node
ok, err = node.smi_open()
out = {"open": ok, "err": err, "count": node.smi_count(), "driver": node.smi_driver_version()}
out["samples"] = [dataclasses.asdict(node.smi_sample(i)) for i in range(max(0, node.smi_count()))]
out["gpus"] = [g.to_dict() for g in node.enumerate_gpus()]
print(json.dumps(out, indent=1))
PY
echo "smi rc=$?"
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1; echo "rocprof -L rc=$?"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/gpurun_out/prof_gemm" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_gemm.log" 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
