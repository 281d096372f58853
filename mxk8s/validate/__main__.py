"""Validator Job entry point (``python -m mxk8s.validate``): BASELINE configs 2-5.

The reference's only validation is a pod that prints ``nvidia-smi`` output,
read after a fixed ``sleep 15`` (/root/reference/README.md:298-335); the NVIDIA
operator's own validator runs the CUDA ``vectorAdd`` sample [ext].  Here every
test launches real GPU work and prints machine-readable ``RESULT {json}``
lines; the process exits non-zero if any test fails.

  rocminfo   the pod sees exactly the allocated gfx950 agents
  vectoradd  HIP vectoradd, bit-exact (bin/mx-vector-add)           config 2
  gemm       CDNA4 bf16 MFMA GEMM TFLOPS vs rocBLAS (bin/mx-gemm-bench) config 3
  rccl       RCCL all-reduce sweep over xGMI (bin/mx-allreduce-perf)  config 4
  ddp        Llama-3-8B DDP synthetic training step (bench.py --mode ddp) config 5

  --profile  adds a rocprofv3 counter pass of the GEMM (separate processes,
             one counter group each): MFMA busy, LDS bank conflicts, clock,
             L2 hit rate as RESULT lines (mxk8s.validate.profile)
  --debug    runs every GPU step with AMD_SERIALIZE_KERNEL=3 and
             HIP_LAUNCH_BLOCKING=1, so a faulting kernel is reported at its
             own launch instead of at a later synchronisation
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.environ.get("MXK8S_BIN", os.path.join(REPO, "bin"))
DEBUG_ENV = {"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1"}
_extra_env: dict = {}


def emit(d: dict) -> None:
    print("RESULT " + json.dumps(d), flush=True)


def _run(cmd, timeout=None, env=None) -> tuple[int, str]:
    print("+ " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                       env={**os.environ, **_extra_env, **(env or {})})
    sys.stderr.write(p.stderr[-4000:])
    return p.returncode, p.stdout


def results_from(stdout: str) -> list[dict]:
    out = []
    for line in stdout.splitlines():
        if line.startswith("RESULT "):
            try:
                out.append(json.loads(line[7:]))
            except ValueError:
                pass
    return out


def test_rocminfo(gpus: int) -> bool:
    try:
        rc, out = _run(["rocminfo"], timeout=120)
    except FileNotFoundError:
        emit({"test": "rocminfo", "pass": False, "error": "rocminfo not found"})
        return False
    agents = re.findall(r"^\s+Name:\s+(gfx\w+)", out, re.M)
    ok = rc == 0 and len(agents) == gpus and all(a == "gfx950" for a in agents)
    emit({"test": "rocminfo", "pass": ok, "gpu_agents": agents, "expected": gpus})
    return ok


def test_vectoradd() -> bool:
    rc, out = _run([os.path.join(BIN, "mx-vector-add"), "--n", "50000"], timeout=300)
    rs = results_from(out)
    for r in rs:
        emit(r)
    return rc == 0 and bool(rs) and all(r.get("pass") for r in rs)


def test_gemm(sizes: str, gpus: int) -> bool:
    rc, out = _run([os.path.join(BIN, "mx-gemm-bench"), "--sizes", sizes, "--devices", "all"],
                   timeout=1800)
    rs = results_from(out)
    for r in rs:
        emit(r)
    if rs:
        by = {}
        for r in rs:
            if "tflops" in r:
                by.setdefault(r["M"], []).append(r["tflops"])
        emit({"test": "gemm_summary", "gpus": gpus,
              "aggregate_tflops": {str(k): round(sum(v), 1) for k, v in by.items()},
              "pass": rc == 0})
    return rc == 0 and bool(rs)


def test_gemm_profile(sizes: str, out_dir: str) -> bool:
    from . import profile
    try:
        summary = profile.profile_gemm(sizes.split(",")[0], out_dir, filt="gemm")
    except (RuntimeError, OSError, subprocess.TimeoutExpired) as e:
        emit({"test": "gemm_profile", "pass": False, "error": str(e)[-500:]})
        return False
    for k, v in summary.items():
        emit({"test": "gemm_profile", "kernel": k[:120], "pass": True, **v["derived"]})
    return bool(summary)


def test_rccl(gpus: int, minb: int, maxb: int, scaling: str, ops: str = "allreduce") -> bool:
    sc = scaling or str(gpus)
    rc, out = _run([os.path.join(BIN, "mx-allreduce-perf"), "-b", str(minb), "-e", str(maxb),
                    "-f", "2", "--scaling", sc, "--op", ops], timeout=3600)
    rs = results_from(out)
    for r in rs:
        if str(r.get("test", "")).endswith("_summary") or r.get("bytes") in (minb, maxb) \
                or not r.get("pass", True):
            emit(r)
    curves = {}
    for r in rs:
        t = str(r.get("test", ""))
        if t.endswith("_summary"):
            curves.setdefault(t[:-len("_summary")], {})[str(r["ngpus"])] = r["peak_busbw_GBps"]
    emit({"test": "rccl_summary", "peak_busbw_GBps_by_ngpus": curves.get("allreduce", {}),
          "peak_busbw_GBps_by_op": curves, "pass": rc == 0})
    return rc == 0 and bool(rs)


def test_ddp(gpus: int, seq_len: int, steps: int) -> bool:
    bench = os.path.join(REPO, "bench.py")
    cmd = [sys.executable, bench, "--mode", "ddp", "--steps", str(steps), "--warmup", "2",
           "--seq-len", str(seq_len)]
    if gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone",
               f"--nproc-per-node={gpus}", bench, "--mode", "ddp", "--gpus", str(gpus),
               "--steps", str(steps), "--warmup", "2", "--seq-len", str(seq_len)]
    rc, out = _run(cmd, timeout=7200)
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if lines:
        d = json.loads(lines[-1])
        d.update({"test": "ddp", "pass": rc == 0})
        emit(d)
    else:
        emit({"test": "ddp", "pass": False, "rc": rc})
    return rc == 0 and bool(lines)


def check_allocation(gpus: int, env=None) -> tuple[bool, list[str]]:
    """Compare the physical GPUs the device plugin handed this pod
    (AMD_GPU_DEVICE_IDS, de-duplicated from time-sliced replicas) with the
    requested count.  Outside a plugin-allocated pod the variable is unset and
    the check passes."""
    env = os.environ if env is None else env
    ids = [x for x in env.get("AMD_GPU_DEVICE_IDS", "").split(",") if x]
    if not ids:
        return True, []
    return len(ids) == gpus, ids


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--tests", default="rocminfo,vectoradd,gemm,rccl")
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--gemm-sizes", default="4096,8192,16384")
    p.add_argument("--rccl-min-bytes", type=int, default=8)
    p.add_argument("--rccl-max-bytes", type=int, default=1 << 33)
    p.add_argument("--rccl-scaling", default="")
    p.add_argument("--rccl-ops", default="allreduce",
                   help="comma list of allreduce,reducescatter,allgather,alltoall or 'all'")
    p.add_argument("--ddp", action="store_true")
    p.add_argument("--ddp-seq-len", type=int, default=2048)
    p.add_argument("--ddp-steps", type=int, default=10)
    p.add_argument("--profile", action="store_true", help="rocprofv3 counter pass of the GEMM")
    p.add_argument("--profile-dir", default=os.environ.get("MXK8S_PROFILE_DIR", "/tmp/mxk8s-pmc"))
    p.add_argument("--debug", action="store_true",
                   help="serialise kernels (AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1)")
    a = p.parse_args(argv)
    if a.debug:
        _extra_env.update(DEBUG_ENV)
    tests = [t for t in a.tests.split(",") if t]
    if a.ddp and "ddp" not in tests:
        tests.append("ddp")
    t0 = time.time()
    status = {}
    ok_alloc, got = check_allocation(a.gpus)
    if not ok_alloc:
        emit({"test": "allocation", "pass": False, "expected_gpus": a.gpus, "allocated": got,
              "message": f"the device plugin allocated {len(got)} physical GPU(s) {got} but "
                         f"--gpus is {a.gpus}: time-sliced replicas of one GPU were stacked "
                         f"into this pod; request exclusive amd.com/gpu or lower --gpus"})
        return 1
    for t in tests:
        if t == "rocminfo":
            status[t] = test_rocminfo(a.gpus)
        elif t == "vectoradd":
            status[t] = test_vectoradd()
        elif t == "gemm":
            status[t] = test_gemm(a.gemm_sizes, a.gpus)
            if a.profile:
                status["gemm_profile"] = test_gemm_profile(a.gemm_sizes, a.profile_dir)
        elif t == "rccl":
            status[t] = test_rccl(a.gpus, a.rccl_min_bytes, a.rccl_max_bytes, a.rccl_scaling,
                                  a.rccl_ops)
        elif t == "ddp":
            status[t] = test_ddp(a.gpus, a.ddp_seq_len, a.ddp_steps)
        else:
            print(f"unknown test {t}", file=sys.stderr)
            status[t] = False
    ok = all(status.values())
    emit({"test": "validator", "pass": ok, "results": status, "seconds": round(time.time() - t0, 1)})
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
