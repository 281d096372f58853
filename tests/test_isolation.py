"""BASELINE config 2's pass criterion (BASELINE.md:37: "pod sees exactly 1
gfx950 agent; vectoradd result exact"), checked on the smoke pod's logs by
``phase_validate`` and ``tests/e2e/run_e2e.sh``.  The reference only reads
``nvidia-smi`` output by eye (/root/reference/README.md:326-335)."""
import json
import subprocess
import sys

import pytest
import yaml

from mxk8s.bootstrap import manifests, phases
from mxk8s.validate import isolation


def _line(**kw):
    r = {"test": "vectoradd", "pass": True, "n": 50000, "mismatches": 0, "device": 0,
         "visible_gpus": 1, "expected_gpus": 1, "arch": "gfx950", "expected_arch": "gfx950",
         "bdfs": ["0000:05:00.0"], "expected_bdfs": ["0000:05:00.0"],
         "render_nodes": ["/dev/dri/renderD128"], "expected_render_nodes": ["/dev/dri/renderD128"]}
    r.update(kw)
    return "RESULT " + json.dumps(r)


GOOD = "        Name:                    gfx950\n" + _line() + "\n"


def test_good_log_passes():
    assert isolation.check_results(isolation.parse_results(GOOD.splitlines())) == []


@pytest.mark.parametrize("log,needle", [
    (_line(visible_gpus=8), "sees 8 GPU"),
    (_line(arch="gfx942"), "arch"),
    (_line(arch="gfx950:sramecc+:xnack-"), None),            # feature suffix ignored
    (_line(render_nodes=["/dev/dri/renderD128", "/dev/dri/renderD129"]), "render nodes"),
    (_line(bdfs=["0000:06:00.0"]), "PCI devices"),
    ('RESULT {"test":"rocminfo","pass":false}\n' + _line(), "rocminfo: pass=False"),
    ("no result here", "no RESULT line"),
    ('RESULT {"test":"other","pass":true}', "no vectoradd"),
    (_line(**{"pass": False}), "vectoradd: pass=False"),
])
def test_bad_logs_fail(log, needle):
    problems = isolation.check_results(isolation.parse_results(log.splitlines()))
    if needle is None:
        assert problems == []
    else:
        assert any(needle in p for p in problems), problems


def test_cli_exit_status():
    ok = subprocess.run([sys.executable, "-m", "mxk8s.validate.isolation", "--gpus", "1"],
                        input=GOOD, capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr
    bad = subprocess.run([sys.executable, "-m", "mxk8s.validate.isolation", "--gpus", "1"],
                         input=_line(visible_gpus=8), capture_output=True, text=True)
    assert bad.returncode == 1 and "sees 8 GPU" in bad.stderr


class _FakeKubectl(phases.Context):
    """Runs nothing; `kubectl logs pod/hip-vector-add` returns a canned log."""
    log: str = ""

    def run(self, cmd, check=True, capture=False, env=None):
        argv = list(cmd)
        self.actions.append(("run", argv))
        out = self.log if "logs" in argv and "pod/hip-vector-add" in argv else ""
        return subprocess.CompletedProcess(argv, 0, out, "")


def _ctx(log):
    c = _FakeKubectl(dry_run=False, out=lambda s: None)
    c.log = log
    return c


def test_phase_validate_accepts_isolated_pod():
    phases.phase_validate(_ctx(GOOD))


@pytest.mark.parametrize("log", [
    _line(visible_gpus=8),                                    # every render node injected
    _line(arch="gfx942"),
    _line(render_nodes=["/dev/dri/renderD129"]),              # the wrong minor
    'RESULT {"test":"vectoradd","pass":false}\n' + _line(),   # an earlier failure
])
def test_phase_validate_rejects(log):
    with pytest.raises(phases.PhaseError):
        phases.phase_validate(_ctx(log))


def test_smoke_manifest_asks_for_the_checks():
    pod = manifests.hip_vector_add()
    c = pod["spec"]["containers"][0]
    cmd = " ".join(c["command"])
    assert "--expect-gpus 1" in cmd and "--expect-arch gfx950" in cmd
    assert c["resources"]["limits"]["amd.com/gpu"] == 1
    with open(manifests.__file__.replace("mxk8s/bootstrap/manifests.py",
                                         "deploy/examples/hip-vector-add.yaml")) as f:
        assert yaml.safe_load(f) == pod


def test_e2e_script_checks_isolation():
    with open(phases.REPO + "/tests/e2e/run_e2e.sh") as f:
        s = f.read()
    assert "mxk8s.validate.isolation --gpus 1 --arch gfx950" in s
